// The ConvNet head as ONE launch in training: forward, loss and (speculatively) backward.
//
//   [BN2 finalize -> BN -> ReLU -> 2x2 max-pool -> flatten -> Linear]     (forward)
//   -> CrossEntropy(mean) on the logits + d(scale * loss)/dlogits          (loss)
//   -> Linear backward (dp2, dW_fc, db_fc) + the BN2 backward sums        (backward)
//
// Reference ops: /root/reference/origin_main.py:16-24,29-30 (BN2/ReLU/pool2, reshape,
// fc) and ddp_main.py:89,91 (CrossEntropyLoss on the logits, scaler.scale(loss).backward()).
// Replaces three launches of the step (head_fwd_kernel, ce_fwd_kernel,
// head_bwd_kernel in csrc/kernels/{convnet_fused,head}.hip) whenever the batch
// labels are known at forward time (the device loader pairs them with the
// images; ops/convnet_fused.py) -- the loss call and the head backward then
// find their results ready and launch nothing.
//
// Decomposition: one workgroup per BN2 channel c (C = 32).  A channel owns 49
// of the 1568 fc inputs, so it computes its BN / ReLU / pool slice and a K = 49
// split of the logits (MFMA 16x16x32: rows = images, cols = classes).  The
// partial logits are stored write-through (`sc1`) and every workgroup takes one
// agent-scope ticket (MI355X_MICROARCH.md "Valid forms" row 1: no release /
// acquire fence).  Without a backward the last arriver adds the bias, rounds the
// logits to the storage dtype and runs the loss (16 lanes per row, as head.hip
// ce_fwd_kernel: same formula, same rounding).  When an active GradScaler
// supplies the scale, the last ticket releases every workgroup, each of which
// sums the partials and runs the same loss itself (fixed order: identical
// d(scale*loss)/dlogits everywhere, no second hand-off) and does its channel's
// share of the fc backward on MFMA:
//   dp2[b, c*49 + j]   = sum_n dls[b, n] * W[n, c*49 + j]       (B x 49, K = N)
//   dW[n, c*49 + j]    = sum_b dls[b, n] * p2[b, c*49 + j]      (N x 49, K = B)
// plus the BN2 backward sums of channel c (complete: the channel is whole here).
// All 32 workgroups of the launch must be co-resident (they wait for the last
// arriver): 32 << 256 CUs, checked on the host (co_resident); every wait is
// bounded and sets the error word.
#include "comm/xgmi.h"
#include "convblock_impl.h"

namespace dpa {
namespace cnh {

using cb::BNParams;
using cb::IDX_RELU;
using cb::Pair2;

constexpr int NT = 256;    // 4 waves
constexpr int C = 32, H = 14, W = 14, HO = 7, WO = 7, PP = 49, K = C * PP;
constexpr int BMAX = 64;   // images (4 MFMA row tiles)
constexpr int NMAX = 16;   // classes (one MFMA column tile)
constexpr int KP = 64;     // 49 fc inputs per channel, padded to 2 MFMA k-steps

// state: int64[4] zero-initialised once: [0] {generation:32 | tickets:32} (the last
// ticket stores (generation + 1) << 32: re-arm and release), [1] unused, [2] error word
struct HeadStep {
  const int64_t* target;
  int64_t ignore_index;
  float smoothing;
  const float* scale;   // GradScaler scale (null: no scaler -> no speculative backward)
  float* part;          // [C][B][NMAX] partial logits (write-through)
  unsigned long long* state;
  float* loss;          // [2]: loss, loss * scale
  float* dlog;          // [B][N] (softmax - onehot) / count, f32
  void* dls;            // [B][N] dlog * scale, storage dtype (null without scaler)
  float* dlsf;          // [B][N] f32 scratch of the earlier two-hand-off protocol (unused; its
                        // presence still selects the speculative backward on the host)
  int do_bwd;
  void* dp2;            // [B][K] storage dtype
  float* dwfc;          // [N][K]
  float* dbfc;          // [N]
  float* dgamma;        // [C]
  float* dbeta;         // [C]
  float* bsum;          // [2C]: S1 | S2 (BN2 backward sums, this rank)
  long long timeout_ticks;
};

template <typename T>
__device__ __forceinline__ void st_wt(float* p, float v) {  // write-through 4-B store (global_store_dword sc1)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {     // L1-bypassing load (global_load_dword sc1)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int GL>
__device__ __forceinline__ float gmax(float v) {
#pragma unroll
  for (int o = GL / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
template <int GL>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
  for (int o = GL / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int BM>  // BM: images the tiles are sized for (32 or BM)
__global__ void __launch_bounds__(NT)
head_step_kernel(const T* __restrict__ y, BNParams bn, const float* __restrict__ wfc, const float* __restrict__ bfc,
                 T* __restrict__ logits, T* __restrict__ p_out, uint8_t* __restrict__ idx_out,
                 T* __restrict__ xh_out, int B, int N, HeadStep hs) {
  typedef MM<T> mm;
  typedef T E;  // operand tiles in the storage dtype (MM<T>::ld reads 8 of them)
  typedef typename Pair2<T>::type P;
  constexpr int ITB = (BM * PP + NT - 1) / NT;  // pooled outputs per lane
  __shared__ float sc_s[C], beta_s[C], mean_s[C], istd_s[C];
  __shared__ float part_s[NT];
  // MFMA operand tiles (row-major, k contiguous: every fragment is one 16-B read)
  __shared__ __attribute__((aligned(16))) E pcl[BM * KP];   // A fwd: p2 slice [b][j]
  // transposed tiles' rows padded by 16 B: their column-wise 2-byte writes (lanes along
  // the rows) then spread over the banks instead of hitting one bank pair
  constexpr int PCT_S = BM + 8, WDL_S = 32 + 8, DLT_S = BM + 8;
  __shared__ __attribute__((aligned(16))) E pct[KP * PCT_S];  // B dW: p2 slice as [j][b]
  __shared__ __attribute__((aligned(16))) E wcl[NMAX * KP];   // B fwd: W slice [n][j]
  __shared__ __attribute__((aligned(16))) E wdl[KP * WDL_S];  // B dp2: W slice [j][n] (k = n padded to 32)
  __shared__ __attribute__((aligned(16))) E dll[BM * 32];   // A dp2: dls [b][n]
  __shared__ __attribute__((aligned(16))) E dlt[NMAX * DLT_S]; // A dW: dls as [n][b]
  __shared__ float lg_s[BM * NMAX];                         // logits (rounded) / dls, f32
  __shared__ float dd_s[BM * NMAX];                         // (softmax - onehot) / count
  __shared__ int64_t tgt_s[BM];
  __shared__ float bias_s[NMAX];
  __shared__ E wdummy_s[2];
  __shared__ uint8_t ix_s[BM * PP];
  __shared__ float xh_s[BM * PP];
  __shared__ float red[2][NT / 64];
  __shared__ unsigned long long tk_s;
  __shared__ int cnt_s;

  const int tid = threadIdx.x, c = blockIdx.x;
  const int lane = tid & 63, wv = tid >> 6, r = lane & 15, q = lane >> 4;
  const int NPO = B * PP;  // pooled outputs of this channel

  DPA_STAMP(0);
  // 1. loads: this channel's pre-BN maps (two row pairs per pooled output) and W slice
  // Every load below is unconditional (clamped index, the value discarded where out of
  // range): a conditional load into a register array made hipcc branch around each load
  // and wait vmcnt(0) after it -- one memory round trip per load (head_step .s, ROCm 7.2).
  P top[ITB], bot[ITB];
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    const int e = min(tid + i * NT, NPO - 1);
    const int b = e / PP, j = e % PP, ho = j / WO, wo = j % WO;
    const P* src = reinterpret_cast<const P*>(y + (((size_t)b * C + c) * H + 2 * ho) * W + 2 * wo);
    top[i] = src[0];
    bot[i] = src[W / 2];
  }
  // the loss' inputs, loaded by every workgroup now (only the last arriver uses them, but
  // it cannot know it is last yet): no dependent global load on its serial path later
  const int64_t tgt_ld = hs.target[min(tid, B - 1)];
  const float bias_ld = bfc[min(tid, N - 1)];
  const int64_t tgt_r = tid < B ? tgt_ld : hs.ignore_index;
  const float bias_r = tid < N ? bias_ld : 0.f;
  const float scale_r = hs.scale != nullptr ? hs.scale[0] : 0.f;
  constexpr int WIT = (NMAX * PP + NT - 1) / NT;
  float wv_[WIT];
#pragma unroll
  for (int i = 0; i < WIT; ++i) {
    const int e = tid + i * NT;
    const int n = e / PP, j = e % PP;
    const float v = wfc[(size_t)min(n, N - 1) * K + c * PP + j];  // unconditional (see above)
    // a multiply, not a select: with a select (or a guarded use below) hipcc re-branches the
    // load by the condition and waits for it inside the branch
    wv_[i] = v * ((e < NMAX * PP && n < N) ? 1.f : 0.f);
  }
  DPA_STAMP(8);
  // zero the tiles' padding (rows past B, k past 49 / N)
  {  // 16-B LDS writes (every tile is 16-B aligned and a whole number of 16-B chunks)
    auto zero = [&](E* t, int n) {
      for (int e = tid; e < n * (int)sizeof(E) / 16; e += NT) reinterpret_cast<f32x4*>(t)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    static_assert((BM * KP) % 8 == 0 && (KP * PCT_S) % 8 == 0 && (BM * 32) % 8 == 0 && (KP * WDL_S) % 8 == 0 &&
                  (NMAX * DLT_S) % 8 == 0 && (NMAX * KP) % 8 == 0, "head tiles: whole 16-B chunks");
    zero(pcl, BM * KP);
    zero(pct, KP * PCT_S);
    zero(dll, BM * 32);
    zero(wdl, KP * WDL_S);
    zero(dlt, NMAX * DLT_S);
    zero(wcl, NMAX * KP);
  }
  DPA_STAMP(9);
  if (tid < BM) tgt_s[tid] = tgt_r;
  if (tid < NMAX) bias_s[tid] = bias_r;
  DPA_STAMP(10);
  cb::bn_finalize<C>(bn, sc_s, beta_s, mean_s, istd_s, part_s, c == 0);  // ends with a barrier
  DPA_STAMP(1);
  // W slice -> tiles
#pragma unroll
  for (int i = 0; i < WIT; ++i) {  // unconditional stores (lanes past the slice write a dummy word)
    const int e = tid + i * NT;
    const bool ok = e < NMAX * PP;
    const int ec = ok ? e : 0, n = ec / PP, j = ec % PP;
    const E wq = Cvt<T>::from_f(wv_[i]);
    *(ok ? &wcl[n * KP + j] : &wdummy_s[0]) = wq;
    *(ok ? &wdl[j * WDL_S + n] : &wdummy_s[1]) = wq;
  }
  // 2. BN -> ReLU -> 2x2 max of this channel; pooled value, argmax|relu index, xhat.
  //    LDS now; the global copies (read by later kernels) are written after the ticket,
  //    so the hand-off's vmcnt(0) drains only the partial-logit stores
  T pvr[ITB], xqr[ITB];
  uint8_t ixr[ITB];
  {
    const float sc = sc_s[c], bt = beta_s[c], mn = mean_s[c], is = istd_s[c];
#pragma unroll
    for (int i = 0; i < ITB; ++i) {
      const int e = tid + i * NT;
      if (e < NPO) {
        const int b = e / PP, j = e % PP;
        float best, xh;
        int bi;
        cb::bn_relu_max4x<T>(top[i], bot[i], sc, bt, mn, is, best, bi, xh);
        pvr[i] = Cvt<T>::from_f(best);
        ixr[i] = (uint8_t)(bi | (best > 0.f ? IDX_RELU : 0));
        xqr[i] = Cvt<T>::from_f(xh);
        pcl[b * KP + j] = pvr[i];
        pct[j * PCT_S + b] = pvr[i];
        ix_s[e] = ixr[i];
        xh_s[e] = Cvt<T>::to_f(xqr[i]);
      }
    }
  }
  auto store_pooled = [&]() {
#pragma unroll
    for (int i = 0; i < ITB; ++i) {
      const int e = tid + i * NT;
      if (e < NPO) {
        const size_t o = (size_t)(e / PP) * K + c * PP + e % PP;
        p_out[o] = pvr[i];
        idx_out[o] = ixr[i];
        xh_out[o] = xqr[i];
      }
    }
  };
  __syncthreads();
  DPA_STAMP(2);
  // 3. partial logits of this channel (K = 49 of 1568): wave w owns image rows 16w..16w+15
  const int MT = (B + 15) / 16;
  if (wv < MT) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KP / 32; ++s) {
      const typename mm::frag a = mm::ld(&pcl[(16 * wv + r) * KP + 32 * s + 8 * q]);
      const typename mm::frag bf = mm::ld(&wcl[r * KP + 32 * s + 8 * q]);
      acc = mm::mma(a, bf, acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = 16 * wv + 4 * q + i;
      if (b < B) st_wt<T>(&hs.part[((size_t)c * B + b) * NMAX + r], acc[i]);
    }
  }
  // publish (write-through stores drained by every wave, then ONE ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    tk_s = __hip_atomic_fetch_add(&hs.state[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  DPA_STAMP(3);
  const unsigned long long tk = tk_s;
  const uint32_t gen = (uint32_t)(tk >> 32);
  const bool last = (uint32_t)tk == (uint32_t)(C - 1);  // grid = C workgroups (not gridDim: a hidden-arg load)
  // The last ticket re-arms the word for the next launch ((gen + 1) << 32: stream order, no
  // workgroup of this launch takes a ticket after it) and that same store releases the
  // waiting workgroups: with the speculative backward EVERY workgroup then sums the C
  // partial logits and runs the loss itself (identical fixed-order arithmetic, so identical
  // results), instead of the last arriver computing it and publishing the loss gradient
  // behind a second flag -- one cross-workgroup hand-off on the serial path instead of two.
  if (last) {
    if (tid == 0)
      __hip_atomic_exchange(&hs.state[0], ((unsigned long long)(gen + 1u)) << 32, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
  } else if (hs.do_bwd) {
    // bounded wait for the last ticket: a timeout sets the error word and goes on
    if (tid == 0) {
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      while ((uint32_t)(__hip_atomic_load(&hs.state[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == gen) {
        __builtin_amdgcn_s_sleep(1);
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > hs.timeout_ticks) {
          __hip_atomic_store(&hs.state[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __syncthreads();
  } else {
    store_pooled();  // no backward: the last arriver alone computes the loss
    return;
  }
  // one writer of the launch-wide outputs (logits, loss, dlog, dls)
  const bool writer = hs.do_bwd ? c == 0 : true;
  DPA_STAMP(4);
  // 4. logits = sum of the C partials + bias, rounded to the storage dtype (every load sc1)
  constexpr int OIT = BM * NMAX / NT;
  T lgr[OIT];
#pragma unroll
  for (int k = 0; k < OIT; ++k) {
    const int o = tid + k * NT;
    const int b = o / NMAX, n = o % NMAX;
    if (b < B && n < N) {
      float v[C];
#pragma unroll
      for (int cc = 0; cc < C; ++cc) v[cc] = ld_wt(&hs.part[((size_t)cc * B + b) * NMAX + n]);
      float t = bias_s[n];
#pragma unroll
      for (int cc = 0; cc < C; ++cc) t += v[cc];
      lgr[k] = Cvt<T>::from_f(t);
      lg_s[o] = Cvt<T>::to_f(lgr[k]);
    }
  }
  if (tid == 0) cnt_s = 0;
  __syncthreads();
  // 5. cross entropy (mean over non-ignored rows), 16 lanes per row (ce_fwd_kernel's math)
  if (tid < B && tgt_s[tid] != hs.ignore_index) atomicAdd(&cnt_s, 1);
  __syncthreads();
  const float cnt = (float)cnt_s;
  const float inv = cnt > 0.f ? 1.f / cnt : 0.f;
  const float scv = scale_r;
  {
    const int gl = tid % 16, gr = tid / 16;
    float lsum = 0.f;
    for (int r0 = 0; r0 < B; r0 += NT / 16) {
      const int b = r0 + gr;
      const bool rv = b < B;
      const int64_t t = rv ? tgt_s[b] : hs.ignore_index;
      const float x = (rv && gl < N) ? lg_s[b * NMAX + gl] : -INFINITY;
      const float mx = gmax<16>(x);
      const float sx = gsum<16>(gl < N ? (rv ? x : 0.f) : 0.f);
      const float ex = (rv && gl < N) ? __expf(x - mx) : 0.f;
      const float se = gsum<16>(ex);
      const float lse = mx + __logf(se);
      const bool use = rv && t != hs.ignore_index;
      if (use && gl == 0) {
        const float xt = (t >= 0 && t < N) ? lg_s[b * NMAX + (int)t] : NAN;
        lsum += (1.f - hs.smoothing) * (lse - xt) + hs.smoothing * (lse - sx / (float)N);
      }
      if (rv) {
        float d = 0.f;
        if (use && gl < N) {
          const float sm = ex * (1.f / se);
          const float oh = (gl == t ? 1.f - hs.smoothing : 0.f) + hs.smoothing / (float)N;
          d = (sm - oh) * inv;
        }
        dd_s[b * NMAX + gl] = d;
      }
    }
    if (writer) {
      lsum = wave_sum(lsum);
      if (lane == 0) red[0][wv] = lsum;
    }
  }
  __syncthreads();
  DPA_STAMP(5);
  if (writer) {  // outputs nobody in this launch waits for
    if (tid == 0) {
      float tl = 0.f;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) tl += red[0][i];
      const float l = cnt > 0.f ? tl / cnt : NAN;
      hs.loss[0] = l;
      if (hs.scale != nullptr) hs.loss[1] = l * scv;
    }
#pragma unroll
    for (int k = 0; k < OIT; ++k) {
      const int o = tid + k * NT;
      const int b = o / NMAX, n = o % NMAX;
      if (b < B && n < N) {
        logits[(size_t)b * N + n] = lgr[k];
        const float d = dd_s[o];
        hs.dlog[(size_t)b * N + n] = d;
        if (hs.dls != nullptr) reinterpret_cast<T*>(hs.dls)[(size_t)b * N + n] = Cvt<T>::from_f(d * scv);
      }
    }
  }
  store_pooled();
  if (!hs.do_bwd) return;
  // the loss gradient the scaler seeds: d(scale * loss)/dlogits rounded to the storage dtype
  for (int o = tid; o < B * NMAX; o += NT) {
    const int n = o % NMAX;
    lg_s[o] = n < N ? Cvt<T>::to_f(Cvt<T>::from_f(dd_s[o] * scv)) : 0.f;
  }
  __syncthreads();
  DPA_STAMP(6);
  // 6. fc backward of channel c on MFMA
  for (int o = tid; o < B * NMAX; o += NT) {
    const int b = o / NMAX, n = o % NMAX;
    const E dq = Cvt<T>::from_f(n < N ? lg_s[o] : 0.f);
    dll[b * 32 + n] = dq;
    dlt[n * DLT_S + b] = dq;
  }
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  if (wv < MT) {  // dp2 rows 16w..16w+15, the 49 (-> 64) columns of this channel
    const typename mm::frag a = mm::ld(&dll[(16 * wv + r) * 32 + 8 * q]);
#pragma unroll
    for (int nt = 0; nt < KP / 16; ++nt) {
      const typename mm::frag bf = mm::ld(&wdl[(16 * nt + r) * WDL_S + 8 * q]);
      const f32x4 acc = mm::mma(a, bf, f32x4{0.f, 0.f, 0.f, 0.f});
      const int j = 16 * nt + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * wv + 4 * q + i;
        if (b < B && j < PP) {
          const T gt = Cvt<T>::from_f(acc[i]);
          reinterpret_cast<T*>(hs.dp2)[(size_t)b * K + c * PP + j] = gt;
          const int e = b * PP + j;
          if (ix_s[e] & IDX_RELU) {
            const float g = Cvt<T>::to_f(gt);
            s1 += g;
            s2 += g * xh_s[e];
          }
        }
      }
    }
  }
  {  // dW rows n (16), columns 16w..16w+15 of this channel, K = images
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < BM / 32; ++s) {
      const typename mm::frag a = mm::ld(&dlt[r * DLT_S + 32 * s + 8 * q]);
      const typename mm::frag bf = mm::ld(&pct[(16 * wv + r) * PCT_S + 32 * s + 8 * q]);
      acc = mm::mma(a, bf, acc);
    }
    const int j = 16 * wv + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * q + i;
      if (n < N && j < PP) hs.dwfc[(size_t)n * K + c * PP + j] = acc[i];
    }
  }
  if (c == 0) {  // fc bias gradient: 16 lanes per class (a serial loop over the batch in one
                 // lane made workgroup 0, and so the launch, ~1 us longer)
    static_assert(NT == 16 * NMAX, "dbfc: one 16-lane group per class");
    const int n = tid / 16, l = tid % 16;
    float a = 0.f;
    if (n < N)
      for (int b = l; b < B; b += 16) a += lg_s[b * NMAX + n];
    a = gsum<16>(a);
    if (n < N && l == 0) hs.dbfc[n] = a;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) { red[0][wv] = s1; red[1][wv] = s2; }
  __syncthreads();
  if (tid == 0) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) { t1 += red[0][i]; t2 += red[1][i]; }
    hs.dbeta[c] = t1;
    hs.dgamma[c] = t2;
    hs.bsum[c] = t1;
    hs.bsum[C + c] = t2;
  }
  DPA_STAMP(7);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
template <typename F>
static void with_t(DT dt, F&& f) {
  switch (dt) {
    case DT::F32: f(float{}); break;
    case DT::BF16: f(__hip_bfloat16{}); break;
    case DT::F16: f(__half{}); break;
  }
}

bool supported(int64_t B, int64_t N) { return B >= 1 && B <= BMAX && N >= 1 && N <= NMAX; }

// co-residency of the C = 32 workgroups (they wait for the last arriver)
bool resident(at::ScalarType st) {
  bool ok = true;
  with_t(dt_of(at::empty({0}, at::TensorOptions().dtype(st))), [&](auto tag) {
    typedef decltype(tag) T;
    ok = co_resident(reinterpret_cast<const void*>(&head_step_kernel<T, 32>), C, NT, 0) &&
         co_resident(reinterpret_cast<const void*>(&head_step_kernel<T, BMAX>), C, NT, 0);
  });
  return ok;
}

void head_step(at::Tensor y2, at::Tensor fslab2, at::Tensor fstats2, at::Tensor g2, at::Tensor b2, at::Tensor rm2,
               at::Tensor rv2, at::Tensor nbt2, double momentum, double eps, at::Tensor wfc, at::Tensor bfc,
               at::Tensor logits, at::Tensor p2, at::Tensor idx2, at::Tensor xh2, at::Tensor target,
               int64_t ignore_index, double smoothing, c10::optional<at::Tensor> scale, at::Tensor part,
               at::Tensor state, at::Tensor loss, at::Tensor dlog, c10::optional<at::Tensor> dls,
               c10::optional<at::Tensor> dlsf, c10::optional<at::Tensor> dp2, c10::optional<at::Tensor> dwfc,
               c10::optional<at::Tensor> dbfc, c10::optional<at::Tensor> dgamma2, c10::optional<at::Tensor> dbeta2,
               c10::optional<at::Tensor> bsum2, std::shared_ptr<xgmi::XgmiComm> xc, double timeout_s) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(wfc); DPA_CHECK_INPUT(logits); DPA_CHECK_INPUT(p2); DPA_CHECK_INPUT(target);
  const int B = (int)y2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(y2.size(1) == C && y2.size(2) == H && y2.size(3) == W && wfc.size(1) == K, "head_step: ConvNet shapes");
  TORCH_CHECK(supported(B, N), "head_step: B <= ", BMAX, " and N <= ", NMAX);
  TORCH_CHECK(logits.numel() == (int64_t)B * N && logits.scalar_type() == y2.scalar_type());
  TORCH_CHECK(p2.numel() == (int64_t)B * K && idx2.numel() == p2.numel() && xh2.numel() == p2.numel());
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == B);
  TORCH_CHECK(part.numel() >= (int64_t)C * B * NMAX && part.scalar_type() == at::kFloat);
  TORCH_CHECK(state.numel() >= 4 && state.scalar_type() == at::kLong && state.is_cuda());
  TORCH_CHECK(loss.numel() >= 2 && dlog.numel() == (int64_t)B * N && dlog.scalar_type() == at::kFloat);
  TORCH_CHECK(scale.has_value() == dls.has_value(), "head_step: scale and dls go together");
  const bool bwd = dlsf.has_value();
  if (bwd) {
    TORCH_CHECK(scale.has_value(), "head_step: the speculative backward needs the scaler's loss gradient");
    TORCH_CHECK(dp2.has_value() && dwfc.has_value() && dbfc.has_value() && dgamma2.has_value() &&
                dbeta2.has_value() && bsum2.has_value());
    TORCH_CHECK(dp2->numel() == p2.numel() && dwfc->numel() == wfc.numel() && dbfc->numel() == N &&
                bsum2->numel() == 2 * C && dlsf->numel() == (int64_t)B * N);
  }
  if (B == 0) return;
  BNParams bp;
  bp.fslab = fslab2.data_ptr<float>();
  bp.nrows = (int)(fslab2.numel() / cb::fslab_row(C));
  bp.fstats = fstats2.data_ptr<float>();
  bp.gamma = g2.data_ptr<float>();
  bp.beta = b2.data_ptr<float>();
  bp.rmean = rm2.data_ptr<float>();
  bp.rvar = rv2.data_ptr<float>();
  bp.nbt = nbt2.data_ptr<int64_t>();
  bp.momentum = (float)momentum;
  bp.eps = (float)eps;
  bp.train = 1;
  if (xc) bp.xs = xc->site(xgmi::kSiteFwd2);
  HeadStep hs;
  hs.target = target.data_ptr<int64_t>();
  hs.ignore_index = ignore_index;
  hs.smoothing = (float)smoothing;
  hs.scale = scale.has_value() ? scale->data_ptr<float>() : nullptr;
  hs.part = part.data_ptr<float>();
  hs.state = reinterpret_cast<unsigned long long*>(state.data_ptr<int64_t>());
  hs.loss = loss.data_ptr<float>();
  hs.dlog = dlog.data_ptr<float>();
  hs.dls = dls.has_value() ? dls->data_ptr() : nullptr;
  hs.dlsf = bwd ? dlsf->data_ptr<float>() : nullptr;
  hs.do_bwd = bwd ? 1 : 0;
  hs.dp2 = bwd ? dp2->data_ptr() : nullptr;
  hs.dwfc = bwd ? dwfc->data_ptr<float>() : nullptr;
  hs.dbfc = bwd ? dbfc->data_ptr<float>() : nullptr;
  hs.dgamma = bwd ? dgamma2->data_ptr<float>() : nullptr;
  hs.dbeta = bwd ? dbeta2->data_ptr<float>() : nullptr;
  hs.bsum = bwd ? bsum2->data_ptr<float>() : nullptr;
  hs.timeout_ticks = (long long)(timeout_s * 1e8);
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    if (bwd) TORCH_CHECK(dls->scalar_type() == y2.scalar_type() && dp2->scalar_type() == y2.scalar_type());
    // tiles sized for 32 images where the batch fits (fewer load / zeroing / MFMA iterations)
    auto kern = B <= 32 ? head_step_kernel<T, 32> : head_step_kernel<T, BMAX>;
    hipLaunchKernelGGL(kern, dim3(C), dim3(NT), 0, cur_stream(), dptr<T>(y2), bp,
                       wfc.data_ptr<float>(), bfc.data_ptr<float>(), dptr<T>(logits), dptr<T>(p2),
                       idx2.data_ptr<uint8_t>(), dptr<T>(xh2), B, N, hs);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace cnh

void register_convnet_head(pybind11::module& m) {
  auto s = m.def_submodule("convnet_head", "ConvNet head: forward + loss + backward in one launch");
  s.def("head_step", &cnh::head_step);
  s.def("supported", &cnh::supported);
  s.def("resident", &cnh::resident);
  DPA_DEF_STAMP_FNS(s);
  s.attr("C") = cnh::C;
  s.attr("NMAX") = cnh::NMAX;
}

}  // namespace dpa
