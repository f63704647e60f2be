// Fused "conv block" kernels for the ConvNet hot path:
//     Conv2d(CIN->COUT, 5x5, stride 1, pad 2) -> BatchNorm2d -> ReLU -> MaxPool2d(2,2)
// (reference: /root/reference/origin_main.py:12-23, ddp_main.py:16-27).
//
// Forward (train):  [conv_fwd: implicit-GEMM MFMA + bias + per-workgroup BN partial sums -> fslab]
//                   -> (SyncBN: one all-reduce of fslab, host side)
//                   -> [bn_relu_pool: reduce fslab, running-stat update,
//                       normalise, ReLU, 2x2 max-pool, argmax index]
// Backward:         [bwd_reduce: pool/ReLU routing + per-channel partial sum(dy), sum(dy*xhat) -> bslab]
//                   -> (SyncBN: one all-reduce of bslab)
//                   -> [bwd_elemt: BN input-grad at full resolution]
//                   -> [conv_wgrad: MFMA per image chunk -> wslab]
//                   -> [grad_reduce: wslab -> dW, db ; bslab -> dgamma, dbeta]
//                   -> [conv_fwd<DGRAD>: input grad = conv of dy with flipped W^T]
//
// Design notes (MI355X):
//  * Everything here is latency-bound (per-step GEMMs are 20-160 MFLOP): few
//    launches, one LDS round trip per operand, >= 64 workgroups per launch.
//  * No float atomics and no zero-fill launches: every cross-workgroup sum is
//    a per-workgroup partial row ("slab") reduced by its consumer kernel.
//    (Contended atomics — every workgroup adding into the same few hundred
//    addresses — serialise at the memory side; the first version of this file
//    spent 32 us per wgrad on them.)  Deterministic as a bonus.
//  * im2col never touches HBM: the input image (with halo) sits in LDS in
//    HWC order so that 8 K-consecutive elements (8 input channels of one tap)
//    are one 16-B ds_read; conv1 (CIN=1) gathers its 25 taps element-wise.
//  * wgrad keeps 5 kw-shifted copies of the input in LDS so that the B operand
//    (8 consecutive output columns of one tap) is again one aligned 16-B read.
//  * BN statistics are sums around a per-channel shift (the running mean,
//    identical on every rank) to avoid E[x^2]-E[x]^2 cancellation; partial
//    sums + counts make SyncBN ONE all-reduce with no device->host mask sync
//    (cf. torch/nn/modules/_functions.py:74-101).
#pragma once
#include "common.h"
#include "comm/xsite.h"

namespace dpa {
namespace cb {

constexpr int NTHR = 256;

// Final statistics buffer written by bn_relu_pool (read by the backward):
// [0,C) sum(y-shift) | [C,2C) sum((y-shift)^2) | [2C] count | [2C+1,3C+1) shift
__host__ __device__ constexpr int stats_len(int C) { return 3 * C + 1; }
// forward partial-sum row per conv workgroup: [sum(C) | sumsq(C) | count]
__host__ __device__ constexpr int fslab_row(int C) { return 2 * C + 1; }

template <int I> struct SH;
template <> struct SH<0> { static constexpr int CIN = 1, COUT = 16, H = 28, W = 28, SPLIT = 4, WROWS = 28; };
#ifndef DPA_FWD2_SPLIT
#define DPA_FWD2_SPLIT 2  // workgroups per image of the conv2 forward (experiment builds: -DDPA_FWD2_SPLIT=4)
#endif
template <> struct SH<1> { static constexpr int CIN = 16, COUT = 32, H = 14, W = 14, SPLIT = DPA_FWD2_SPLIT, WROWS = 14; };
constexpr int kBwdSplit = 8;  // batch split of bwd_reduce

// ---------------------------------------------------------------------------
// Staging helpers.  Every global->LDS staging loop is split into "issue every
// load into registers" then "convert + scatter into LDS", with compile-time
// trip counts so all of a thread's loads are in flight together: one L2
// round trip per staging phase instead of one per loop iteration (the loop
// form cost 20+ us per kernel in the first profile).
// ---------------------------------------------------------------------------
// f32 array of N elements (N % 4 == 0, 16-B aligned) -> sink(e, v) per element
template <int N, typename Sink>
__device__ __forceinline__ void stage_f32(const float* __restrict__ src, Sink&& sink) {
  static_assert(N % 4 == 0, "N must be a multiple of 4");
  constexpr int N4 = N / 4;
  constexpr int IT = (N4 + NTHR - 1) / NTHR;
  f32x4 v[IT];
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = threadIdx.x + i * NTHR;
    if (e < N4) v[i] = s4[e];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = threadIdx.x + i * NTHR;
    if (e < N4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) sink(4 * e + j, v[i][j]);
    }
  }
}

// [C][H][W] image of T (W even) -> sink(c, h, w, v_w, v_w+1) per element pair
template <typename T> struct Pair2 { typedef uint32_t type; };
template <> struct Pair2<float> { typedef uint64_t type; };
template <typename T, int C, int H, int W, typename Sink>
__device__ __forceinline__ void stage_chw(const T* __restrict__ src, Sink&& sink) {
  static_assert(W % 2 == 0, "W must be even");
  typedef typename Pair2<T>::type P;
  constexpr int NP = C * H * W / 2;
  constexpr int IT = (NP + NTHR - 1) / NTHR;
  P v[IT];
  const P* s2 = reinterpret_cast<const P*>(src);
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = threadIdx.x + i * NTHR;
    if (e < NP) v[i] = s2[e];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = threadIdx.x + i * NTHR;
    if (e < NP) {
      const int pe = 2 * e;
      const int c = pe / (H * W), rem = pe % (H * W);
      T a, b;
      __builtin_memcpy(&a, &v[i], sizeof(T));
      __builtin_memcpy(&b, reinterpret_cast<const char*>(&v[i]) + sizeof(T), sizeof(T));
      sink(c, rem / W, rem % W, a, b);
    }
  }
}

// ---------------------------------------------------------------------------
// BatchNorm finalize, shared by bn_relu_pool and the fused prologues of the
// next layer's kernel (ops/convnet_fused.py).  train: reduce the conv's
// per-workgroup partial sums (nrows x (2C+1), L2-resident), publish the final
// sums to fstats and update running stats on the leader workgroup; eval: use
// the running stats.  Leaves per-channel y*sc + sh coefficients in LDS.
// ---------------------------------------------------------------------------
struct BNParams {
  const float* fslab;
  int nrows;
  float* fstats;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float momentum;
  float eps;
  int train;
  xgmi::XSite xs;  // active: SyncBN sums exchanged in here (comm/xsite.h), fslab holds local rows
};

// Sum of src[r * RL + j] over rows r = g, g + G, ...: up to RSUM_U rows per
// lane are loaded in ONE batch (all loads in flight before the first add), so
// a slab of up to RSUM_U * G rows costs one L2 round trip instead of one per
// 4 rows (the partial-sum slabs are 64-256 rows: this was 3-5 serial trips).
constexpr int RSUM_U = 24;
template <typename F>
__device__ __forceinline__ float strided_rowsum(const float* __restrict__ src, int rows, int RL, int j, int g, int G,
                                                F&& after_issue) {
  // The first batch is peeled out of the loop (at a loop header hipcc waits vmcnt(0) for the
  // previous iteration's loads, which on entry also waited for every load the kernel had
  // issued before), and the loads are unconditional (clamped row, masked by a multiply: a
  // conditional load was branched around and its add waited right behind it) -- so the whole
  // batch is issued behind the kernel's earlier loads instead of a round trip after them.
  float acc = 0.f;
  auto batch = [&](int base, bool first) {
    float v[RSUM_U];
#pragma unroll
    for (int u = 0; u < RSUM_U; ++u) {
      const int rr = base + u * G;
      v[u] = src[(size_t)min(rr, rows - 1) * RL + j] * (rr < rows ? 1.f : 0.f);
    }
    if (first) after_issue();  // e.g. an atomic whose round trip then overlaps these loads
#pragma unroll
    for (int u = 0; u < RSUM_U; ++u) acc += v[u];
  };
  batch(g, true);
  for (int base = g + RSUM_U * G; base < rows; base += RSUM_U * G) batch(base, false);
  return acc;
}
__device__ __forceinline__ float strided_rowsum(const float* __restrict__ src, int rows, int RL, int j, int g, int G) {
  return strided_rowsum(src, rows, RL, j, g, G, [] {});
}

// part: >= NTHR floats of LDS; ends with __syncthreads().  Every caller runs NTHR-thread
// workgroups: the constant, not blockDim.x -- on gfx950 blockDim is a load from the hidden
// kernel arguments, and the s_waitcnt vmcnt(0) before its use waited for every load the
// kernel had issued so far (a whole memory round trip ahead of the slab loads, head .s).
template <int C>
__device__ __forceinline__ void bn_finalize(const BNParams& bp, float* sc_s, float* beta_s, float* mean_s,
                                            float* istd_s, float* part, int bid) {
  const int tid = threadIdx.x, nthr = NTHR;
  const bool leader = bid == 0;  // writes fstats / running stats (and pushes the SyncBN row)
  if (bp.train) {
    constexpr int RL = 2 * C + 1;
    const int G = nthr / RL;
    const int j = tid % RL, g = tid / RL;
    // per-channel parameters first: their loads overlap the slab reduction's
    float gam = 0.f, bet = 0.f, shf = 0.f, rm = 0.f, rv = 0.f;
    if (tid < C) {
      gam = bp.gamma[tid];
      bet = bp.beta[tid];
      shf = bp.fstats[2 * C + 1 + tid];
      if (leader) {
        rm = bp.rmean[tid];
        rv = bp.rvar[tid];
      }
    }
    const int64_t nb0 = leader ? bp.nbt[0] : 0;
    const bool xon = bp.xs.active();
    unsigned long long tk = 0;
    // the SyncBN ticket is taken right after the slab loads are issued: its round trip overlaps
    // theirs (taken before them, its returned value's wait held the loads back)
    auto ticket = [&] {
      if (xon && tid == 0) tk = xgmi::xsite_ticket(bp.xs, bid);
    };
    if (g < G) {
      part[tid] = strided_rowsum(bp.fslab, bp.nrows, RL, j, g, G, ticket);
    } else {
      ticket();
      part[tid] = 0.f;
    }
    DPA_STAMP(11);
    __syncthreads();
    DPA_STAMP(12);
    if (tid < RL) {
      float t = 0.f;
      for (int gg = 0; gg < G; ++gg) t += part[gg * RL + tid];
      part[tid] = t;  // only this thread reads slot tid (its gg = 0 term) before the write
    }
    __syncthreads();
    if (xon) xgmi::xsite_exchange(bp.xs, part, RL, tk, bid);  // local -> global sums (SyncBN)
    if (tid < C) {
      const float n = part[2 * C];
      const float m1 = part[tid] / n;
      const float mean = shf + m1;
      const float var = fmaxf(part[C + tid] / n - m1 * m1, 0.f);
      const float istd = rsqrtf(var + bp.eps);
      const float s = gam * istd;
      sc_s[tid] = s;
      beta_s[tid] = bet;
      mean_s[tid] = mean;
      istd_s[tid] = istd;
      if (leader) {
        bp.fstats[tid] = part[tid];
        bp.fstats[C + tid] = part[C + tid];
        if (tid == 0) bp.fstats[2 * C] = n;
        const int64_t nb = nb0 + 1;
        const float mom = bp.momentum >= 0.f ? bp.momentum : 1.f / (float)nb;
        bp.rmean[tid] = (1.f - mom) * rm + mom * mean;
        bp.rvar[tid] = (1.f - mom) * rv + mom * var * (n / fmaxf(n - 1.f, 1.f));
      }
    }
    __syncthreads();
    if (leader && tid == 0) bp.nbt[0] = nb0 + 1;
  } else {
    if (tid < C) {
      const float istd = rsqrtf(bp.rvar[tid] + bp.eps);
      const float s = bp.gamma[tid] * istd;
      sc_s[tid] = s;
      beta_s[tid] = bp.beta[tid];
      mean_s[tid] = bp.rmean[tid];
      istd_s[tid] = istd;
    }
    __syncthreads();
  }
}

// BN -> ReLU -> 2x2 max (first max wins, ATen's scan order) of one window given
// as two row pairs; also returns xhat = (y - mean) * invstd at the argmax.
// z = (y - mean) * (gamma * invstd) + beta: near the ReLU threshold this form
// keeps the rounding error at the scale of beta instead of gamma*mean*invstd.
template <typename T>
__device__ __forceinline__ void bn_relu_max4x(const typename Pair2<T>::type top, const typename Pair2<T>::type bot,
                                              float sc, float beta, float mean, float istd, float& best, int& bi,
                                              float& xh) {
  T v[4];
  __builtin_memcpy(&v[0], &top, 2 * sizeof(T));
  __builtin_memcpy(&v[2], &bot, 2 * sizeof(T));
  best = -1.f;
  bi = 0;
  float yb = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float yv = Cvt<T>::to_f(v[k]);
    const float z = fmaxf(rnd_t<T>((yv - mean) * sc + beta), 0.f);
    if (z > best) { best = z; bi = k; yb = yv; }
  }
  xh = (yb - mean) * istd;
}

// Pooled-index byte of the fused path: bits 0-1 argmax in the 2x2 window
// (dy * 2 + dx), bit 2 set when the ReLU passed the value (pooled output > 0).
constexpr int IDX_POS = 3, IDX_RELU = 4;

// Input of a conv that starts with the previous block's BN -> ReLU -> MaxPool.
template <typename T>
struct PoolIn {
  const T* y;          // previous conv output (pre-BN) [B][CIN][2H][2W]
  BNParams bn;         // its BatchNorm
  T* p_out;            // pooled output written for the backward (or null)
  uint8_t* idx_out;    // argmax index | relu bit, written for the backward
  T* xh_out;           // normalised value at the argmax (BN backward sums)
};

// ---------------------------------------------------------------------------
// Backward through [BN -> ReLU -> MaxPool2d(2,2)] fused into the staging of the
// next backward kernel: the conv-output gradient is produced on the fly as
//   dy = gi * (g - k1 - xhat * k2),  g = pooled grad at the window's argmax if
//   the ReLU passed it, else 0;  k1 = S1/n, k2 = S2/n, gi = gamma * invstd,
// with S1 = sum g, S2 = sum g * xhat over the (global) batch.
// ---------------------------------------------------------------------------
template <typename T>
struct BwdIn {
  const T* dp;            // pooled grad [B][C][H/2][W/2]
  const uint8_t* idx;     // argmax | relu bit
  const T* y;             // pre-BN conv output [B][C][H][W]
  const float* fstats;    // forward statistics (stats_len(C))
  const float* gsum;      // rows x [S1(C) | S2(C)], all-reduced under SyncBN
  int grows;
  const float* lsum;      // this rank's rows (dgamma / dbeta); may alias gsum
  int lrows;
  const float* gamma;
  float eps;
  float* dgamma;          // written by workgroup 0 when non-null
  float* dbeta;
  xgmi::XSite xs;         // active: gsum holds local rows, exchanged in here (comm/xsite.h)
  GradChk chk;            // producer-side non-finite check (common.h; not with xs active):
  int chk_coef = 0;       //   1: workgroup 0's dgamma / dbeta
  int chk_rows = 0;       //   1: the weight-gradient workgroups' partial rows (|v| <= chk_row_bound)
  float chk_row_bound = 0.f;
};

// Column sums of rows x RL floats (row-major) -> out[0..RL) in LDS, using the
// whole (NTHR-thread) workgroup; part: >= NTHR floats of LDS.  Ends with a barrier.
// (NTHR, not blockDim.x: see bn_finalize)
__device__ __forceinline__ void colsum_rows(const float* __restrict__ src, int rows, int RL, float* part,
                                            float* out) {
  const int tid = threadIdx.x, nthr = NTHR;
  const int G = nthr / RL;
  const int j = tid % RL, g = tid / RL;
  part[tid] = g < G ? strided_rowsum(src, rows, RL, j, g, G) : 0.f;
  __syncthreads();
  float t = 0.f;
  if (tid < RL)
    for (int gg = 0; gg < G; ++gg) t += part[gg * RL + tid];
  __syncthreads();
  if (tid < RL) out[tid] = t;
  __syncthreads();
}

// coef (LDS, 5C floats): [k1 | k2 | gi | mean | invstd]; part: >= blockDim.x
// floats of LDS, sums: >= 2C floats of LDS.  Workgroup `leader` also writes
// dgamma / dbeta from the local rows.  Ends with a barrier.
template <int C, typename T>
__device__ __forceinline__ void bn_bwd_coef(const BwdIn<T>& bi, float* coef, float* part, float* sums, int bid) {
  const int tid = threadIdx.x;
  const bool leader = bid == 0;
  float n = 0.f, f0 = 0.f, f1 = 0.f, shf = 0.f, gam = 0.f;
  if (tid < C) {  // issued before the reduction: latencies overlap
    n = bi.fstats[2 * C];
    f0 = bi.fstats[tid];
    f1 = bi.fstats[C + tid];
    shf = bi.fstats[2 * C + 1 + tid];
    gam = bi.gamma[tid];
  }
  const bool xon = bi.xs.active();
  unsigned long long tk = 0;
  if (xon && tid == 0) tk = xgmi::xsite_ticket(bi.xs, bid);  // latency hides behind the slab loads
  const bool cchk = leader && bi.dgamma != nullptr && bi.chk_coef && !xon;  // producer-side check (xon: above)
  colsum_rows(bi.gsum, bi.grows, 2 * C, part, sums);
  if (xon) {
    // dgamma / dbeta are this rank's (DDP averages them); the coefficients use the global sums
    if (leader && bi.dgamma != nullptr && tid < C) {
      bi.dgamma[tid] = sums[C + tid];
      bi.dbeta[tid] = sums[tid];
      if (bi.chk_coef) bi.chk.flag(GradChk::bad(sums[C + tid], bi.chk.bound) || GradChk::bad(sums[tid], bi.chk.bound));
    }
    xgmi::xsite_exchange(bi.xs, sums, 2 * C, tk, bid);
  }
  if (tid < C) {
    const float m1 = f0 / n;
    const float mean = shf + m1;
    const float istd = rsqrtf(fmaxf(f1 / n - m1 * m1, 0.f) + bi.eps);
    coef[tid] = sums[tid] / n;
    coef[C + tid] = sums[C + tid] / n;
    coef[2 * C + tid] = gam * istd;
    coef[3 * C + tid] = mean;
    coef[4 * C + tid] = istd;
    if (leader && bi.dgamma != nullptr && bi.lsum == bi.gsum && !xon) {
      bi.dgamma[tid] = sums[C + tid];
      bi.dbeta[tid] = sums[tid];
    }
  }
  __syncthreads();
  if (leader && bi.dgamma != nullptr && bi.lsum != bi.gsum && !xon) {
    colsum_rows(bi.lsum, bi.lrows, 2 * C, part, sums);
    if (tid < C) {
      bi.dgamma[tid] = sums[C + tid];
      bi.dbeta[tid] = sums[tid];
    }
  }
  if (cchk && tid < C)  // the values just written
    bi.chk.flag(GradChk::bad(sums[C + tid], bi.chk.bound) || GradChk::bad(sums[tid], bi.chk.bound));
}

// Produce dy[c][h][w] of image b for every 2x2 window.  Two phases so that the
// loads can be issued before the coefficient reduction (their latencies
// overlap): load(bi, b) ... bn_bwd_coef(...) ... emit(coef, sink) with
// sink(c, h, w, v00, v01, v10, v11), (h, w) = the window's top-left pixel.
// ROWS (even): the conv-output rows [r0, r0 + ROWS) of one image (pooled rows
// [r0/2, r0/2 + ROWS/2), clipped at the image); the sink gets chunk-relative rows.
template <typename T, int C, int H, int W, int NT_, int ROWS = H>
struct BnBwdStage {
  typedef typename Pair2<T>::type P;
  static_assert(ROWS % 2 == 0 && ROWS <= H, "BN-backward staging works on whole 2x2 pooling windows");
  static constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  static constexpr int CHO = ROWS / 2, CPP = CHO * WO, NWIN = C * CPP;  // windows of one chunk
  static constexpr int IT = (NWIN + NT_ - 1) / NT_;
  P top[IT], bot[IT];
  T g[IT];
  uint8_t ix[IT];
  int ho0 = 0;

  __device__ __forceinline__ void load(const BwdIn<T>& bi, int b, int r0 = 0) {
    ho0 = r0 / 2;
    const T* yb = bi.y + (size_t)b * C * H * W;
    const T* dpb = bi.dp + (size_t)b * C * PP;
    const uint8_t* ib = bi.idx + (size_t)b * C * PP;
    // unconditional loads (clamped window; emit() skips the out-of-range ones): guarded
    // loads were branched around and waited for group by group (conv2_bwd / wgrad1 .s,
    // scripts/asm_loads.py)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = min((int)threadIdx.x + i * NT_, NWIN - 1);
      const int c = e / CPP, pix = e % CPP, ho = min(ho0 + pix / WO, HO - 1), wo = pix % WO;
      const P* src = reinterpret_cast<const P*>(yb + ((size_t)c * H + 2 * ho) * W + 2 * wo);
      top[i] = src[0];
      bot[i] = src[W / 2];
      const int ew = c * PP + ho * WO + wo;
      g[i] = dpb[ew];
      ix[i] = ib[ew];
    }
  }

  template <typename Sink>
  __device__ __forceinline__ void emit(const float* coef, Sink&& sink) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = threadIdx.x + i * NT_;
      const int c = e / CPP, pix = e % CPP, hl = pix / WO, wo = pix % WO;
      if (e < NWIN && ho0 + hl < HO) {
        const int ho = hl;  // chunk-relative pooled row
        const float k1 = coef[c], k2 = coef[C + c], gi = coef[2 * C + c], mean = coef[3 * C + c],
                    istd = coef[4 * C + c];
        T v[4];
        __builtin_memcpy(&v[0], &top[i], 2 * sizeof(T));
        __builtin_memcpy(&v[2], &bot[i], 2 * sizeof(T));
        const int k = ix[i] & IDX_POS;
        const float gg = (ix[i] & IDX_RELU) ? Cvt<T>::to_f(g[i]) : 0.f;
        T o[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float xh = (Cvt<T>::to_f(v[qq]) - mean) * istd;
          o[qq] = Cvt<T>::from_f(gi * ((qq == k ? gg : 0.f) - k1 - xh * k2));
        }
        sink(c, 2 * ho, 2 * wo, o[0], o[1], o[2], o[3]);
      }
    }
  }
};

// As BnBwdStage (whole images), but a lane owns 8 CHANNELS of one 2x2 window
// (lanes along the windows: each load instruction still reads consecutive pairs of
// one row) and the sink receives the window's 4 pixels as 8-channel vectors: the
// data-grad kernel writes them as 16-B LDS stores into its [pixel][channel] image.
template <typename T, int C, int H, int W, int NT_>
struct BnBwdStage8 {
  typedef typename Pair2<T>::type P;
  static_assert(C % 8 == 0 && sizeof(T) == 2, "8-channel staging: 16-bit types, C % 8 == 0");
  static constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  static constexpr int NO = C / 8, NWIN = NO * PP;
  static constexpr int IT = (NWIN + NT_ - 1) / NT_;
  P top[IT][8], bot[IT][8];
  T g[IT][8];
  uint8_t ix[IT][8];

  __device__ __forceinline__ void load(const BwdIn<T>& bi, int b) {
    const T* yb = bi.y + (size_t)b * C * H * W;
    const T* dpb = bi.dp + (size_t)b * C * PP;
    const uint8_t* ib = bi.idx + (size_t)b * C * PP;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = min((int)threadIdx.x + i * NT_, NWIN - 1);  // clamped: unconditional loads
      const int o = e / PP, pix = e % PP, ho = pix / WO, wo = pix % WO;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * o + j;
        const P* src = reinterpret_cast<const P*>(yb + ((size_t)c * H + 2 * ho) * W + 2 * wo);
        top[i][j] = src[0];
        bot[i][j] = src[W / 2];
        g[i][j] = dpb[c * PP + pix];
        ix[i][j] = ib[c * PP + pix];
      }
    }
  }

  // sink(h, w, c0, q00, q01, q10, q11): the 4 pixels of window (h, w) (top-left),
  // channels c0 .. c0+7, each packed as uint4
  template <typename Sink>
  __device__ __forceinline__ void emit(const float* coef, Sink&& sink) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = (int)threadIdx.x + i * NT_;
      if (e < NWIN) {
        const int o = e / PP, pix = e % PP, ho = pix / WO, wo = pix % WO;
        unsigned q[4][4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = 8 * o + j;
          const float k1 = coef[c], k2 = coef[C + c], gi = coef[2 * C + c], mean = coef[3 * C + c],
                      istd = coef[4 * C + c];
          T v[4];
          __builtin_memcpy(&v[0], &top[i][j], 2 * sizeof(T));
          __builtin_memcpy(&v[2], &bot[i][j], 2 * sizeof(T));
          const int k = ix[i][j] & IDX_POS;
          const float gg = (ix[i][j] & IDX_RELU) ? Cvt<T>::to_f(g[i][j]) : 0.f;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const float xh = (Cvt<T>::to_f(v[qq]) - mean) * istd;
            const T o_ = Cvt<T>::from_f(gi * ((qq == k ? gg : 0.f) - k1 - xh * k2));
            const unsigned bits = __builtin_bit_cast(unsigned short, o_);
            if (j & 1) q[qq][j >> 1] |= bits << 16; else q[qq][j >> 1] = bits;
          }
        }
        sink(2 * ho, 2 * wo, 8 * o, make_uint4(q[0][0], q[0][1], q[0][2], q[0][3]),
             make_uint4(q[1][0], q[1][1], q[1][2], q[1][3]), make_uint4(q[2][0], q[2][1], q[2][2], q[2][3]),
             make_uint4(q[3][0], q[3][1], q[3][2], q[3][3]));
      }
    }
  }
};

// Epilogue of the data-grad kernel that produces a pooled grad: per-workgroup
// BN partial sums of the block below ([S1 | S2] per channel -> one slab row).
template <typename T>
struct BwdEpi {
  const uint8_t* idx;  // that block's pooled index (relu bit)
  const T* xh;         // that block's xhat at the argmax
  float* bslab;        // rows = workgroups, row = [S1(COUT) | S2(COUT)]
};

// ---------------------------------------------------------------------------
// Pre-packed low-precision weights of the 16->32 conv (ConvNet layer 2), in
// exactly the LDS tile layout conv5x5_kernel uses (rows padded to KPW, K
// padding zeroed): the forward tile [32][424] (k = tap*16 + ci) and the
// data-grad tile [16][808] (k = (24-tap)*32 + co, the flipped transpose).
// The layer-1 forward kernel writes them as a side job (its workgroups are
// idle for most of the chip anyway), so the layer-2 kernels stage their weight
// tile with straight 16-B copies instead of 12,800 converted, scattered
// element stores per workgroup (the VALU-heaviest part of their staging).
// ---------------------------------------------------------------------------
constexpr int W2F_ROWS = 32, W2F_PITCH = 424;   // ceil_to(25*16, 32) + 8
constexpr int W2D_ROWS = 16, W2D_PITCH = 808;   // ceil_to(25*32, 32) + 8
constexpr int W2F_LEN = W2F_ROWS * W2F_PITCH, W2D_LEN = W2D_ROWS * W2D_PITCH;
template <typename T>
struct WPack {
  const float* w2 = nullptr;  // [32][16][5][5] f32 master weights
  T* fwd = nullptr;           // [W2F_LEN]
  T* dgrad = nullptr;         // [W2D_LEN]
};
template <typename T>
__device__ __forceinline__ void pack_w2(const WPack<T>& pk) {
  const int total = W2F_LEN + W2D_LEN;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    if (e < W2F_LEN) {
      const int co = e / W2F_PITCH, k = e % W2F_PITCH;
      const float v = k < 400 ? pk.w2[(co * 16 + (k & 15)) * 25 + (k >> 4)] : 0.f;
      pk.fwd[e] = Cvt<T>::from_f(v);
    } else {
      const int e2 = e - W2F_LEN;
      const int ci = e2 / W2D_PITCH, k = e2 % W2D_PITCH;
      const float v = k < 800 ? pk.w2[((k & 31) * 16 + ci) * 25 + (24 - (k >> 5))] : 0.f;
      pk.dgrad[e2] = Cvt<T>::from_f(v);
    }
  }
}

// Batch gather fused into the first conv (PRO 3): the input image is read from
// the uint8 dataset resident in HBM through the epoch's sample order at the
// device step counter, converted (ToTensor: x * scale + shift, data/loader.py)
// and staged; split 0 of each image also writes it (and its label) to the
// batch buffers the rest of the step reads.  The launch's last-arriving
// workgroup advances the step counter (data.hip gather_kernel's protocol).
struct GatherIn {
  const uint8_t* imgs = nullptr;   // [N][npix]
  const int64_t* labels = nullptr; // [N]
  const int64_t* order = nullptr;  // epoch order
  long long order_len = 0;
  int* ctr = nullptr;              // [0] step, [1] arrivals (self-resetting)
  int64_t* lab_out = nullptr;      // [B]
  float scale = 1.f, shift = 0.f;
  int nimg = 0;                    // B (the launch has nimg * nsplit workgroups; not gridDim,
                                   // a hidden-argument load with its own wait on gfx950)
};

// ---------------------------------------------------------------------------
// Implicit-GEMM 5x5 convolution, one (image, m-range) per workgroup.
//   MODE 0: forward + bias + BN partial sums        (train)
//   MODE 1: forward + bias                          (eval)
//   MODE 2: data-grad: input = dy (CIN = COUT_orig), output = dx,
//           W_eff[co][ci][kh][kw] = W[ci][co][4-kh][4-kw], no bias
// GEMM view: rows = output pixels of one image, cols = output channels,
// K = 25*CIN ordered (kh, kw, ci) with ci fastest.
// ---------------------------------------------------------------------------
//   PRO 0: the input image is read from x;
//   PRO 3: (CIN 1) the input image is gathered from the dataset (gin, above) and
//          written to x by split 0;
//   PRO 1: the input is produced in the staging pass from the previous block's
//          pre-BN output (pin: BN finalize -> normalise -> ReLU -> 2x2 max-pool),
//          which also writes the pooled map + argmax|relu index + xhat at the
//          argmax for the backward (split 0);
//   PRO 2: (MODE 2) the input dy is produced from the pooled grad of the next
//          block (bin: backward through MaxPool -> ReLU -> BN, see BwdIn).
//   EPI 1: (MODE 2) the output is a pooled grad: also write this workgroup's
//          BN partial sums [S1 | S2] of the block below (epi).
//   WPK 0: stage the weight tile from the f32 master weights w;
//   WPK 1: w is ignored, the tile is copied from the pre-packed wpk (pack_w2);
//   WPK 2: as 0, and this launch also writes the layer-2 packs (pk).
// bid: this workgroup's index among the launch's workgroups of this role (blockIdx.x
// for a launch of its own; conv5x5_kernel / dgrad_wgrad_kernel below).
// DYN: the two big LDS tiles (image, weights) are carved from the launch's dynamic LDS
// instead of being static arrays, so a launch hosting several roles (convnet_fused.hip
// conv2_bwd_dyn_kernel) needs the LARGEST role's tiles, not their sum (conv5x5_dyn_bytes).
template <typename T, int CIN, int H, int W>
__host__ __device__ constexpr size_t conv5x5_img_bytes() {
  return ((sizeof(T) * (size_t)(H + 4) * (W + 4) * CIN) + 15) / 16 * 16;
}
template <typename T, int CIN, int COUT, int H, int W>
__host__ __device__ constexpr size_t conv5x5_dyn_bytes() {
  return conv5x5_img_bytes<T, CIN, H, W>() + sizeof(T) * (size_t)COUT * (ceil_to(25 * CIN, 32) + 8);
}
extern __shared__ __attribute__((aligned(16))) unsigned char dpa_dyn_lds[];

template <typename T, int CIN, int COUT, int H, int W, int MODE, int PRO = 0, int EPI = 0, int WPK = 0,
          bool DYN = false>
__device__ __forceinline__ void
conv5x5_body(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
             T* __restrict__ y, float* __restrict__ fslab, float* __restrict__ fstats,
             const float* __restrict__ shift, int nsplit, const PoolIn<T>& pin, const BwdIn<T>& bin,
             const BwdEpi<T>& epi, const T* __restrict__ wpk, const WPack<T>& pk, const int bid,
             const GatherIn& gin = GatherIn{}) {
  static_assert(CIN == 1 || CIN % 8 == 0, "CIN must be 1 or a multiple of 8");
  static_assert(COUT % 16 == 0, "COUT must be a multiple of 16");
  static_assert((H * W) % 4 == 0, "H*W must be a multiple of 4");
  static_assert(PRO != 2 || MODE == 2, "PRO 2 is a data-grad prologue");
  static_assert(PRO != 3 || (CIN == 1 && MODE != 2), "PRO 3 gathers single-channel input images");
  static_assert(EPI == 0 || MODE == 2, "EPI 1 is a data-grad epilogue");
  constexpr int NCH = CIN >= 8 ? CIN / 8 : 1;              // 16-B groups per pixel
#ifdef DPA_IMG_PAD8
  // 32-B pixels (CIN 16): pad rows to W + 8 so a row wrap shifts the pixel index by a
  // multiple of 8 (one 256-B bank row) and read unswizzled: the 16 lanes of a
  // ds_read_b128 group then hit 16 distinct 16-B slots (experiment build)
  constexpr bool PAD8 = NCH == 2;
#else
  constexpr bool PAD8 = false;
#endif
  constexpr int HP = H + 4, WPD = W + (PAD8 ? 8 : 4);
  constexpr int K = 25 * CIN;
  constexpr int KP = ceil_to(K, 32);
  constexpr int KS = KP / 32;
  constexpr int KPW = KP + 8;  // LDS row pitch of the weight tile (breaks bank aliasing)
  constexpr int NT = COUT / 16;
  constexpr int HW = H * W;
  constexpr int MT = (HW + 15) / 16;
  typedef MM<T> mm;

  static_assert(!DYN || !PAD8, "dynamic tiles: unpadded image rows (conv5x5_img_bytes)");
  T* img;
  T* wl;
  if constexpr (DYN) {
    img = reinterpret_cast<T*>(dpa_dyn_lds);
    wl = reinterpret_cast<T*>(dpa_dyn_lds + conv5x5_img_bytes<T, CIN, H, W>());
  } else {
    __shared__ __attribute__((aligned(16))) T img_s[HP * WPD * CIN];
    __shared__ __attribute__((aligned(16))) T wl_s[COUT * KPW];
    img = img_s;
    wl = wl_s;
  }
  // img is [padded pixel][CIN] with the 8-channel (16-B) groups of each pixel
  // XOR-swizzled by the pixel index: an A-fragment read takes 16 consecutive
  // pixels x one 16-B group; with a 32/64-B pixel pitch those 16 addresses would
  // share 8/4 bank groups (2/4-way conflicts), swizzled they hit 16 distinct ones
  // (conv2 dgrad: SQ_LDS_BANK_CONFLICT -54 %)
  constexpr int PPB = NCH <= 16 ? 16 / NCH : 1;            // pixels per 256-B bank row
  auto imo = [](int px, int c) -> int {
    if constexpr (NCH <= 1 || PAD8) {
      return px * CIN + c;
    } else {
      return px * CIN + ((((c >> 3) ^ ((px / PPB) & (NCH - 1)))) << 3) + (c & 7);
    }
  };
  __shared__ float lstat[(NTHR / 64) * 2 * COUT];

  const int tid = threadIdx.x;
  const int b = bid / nsplit;
  DPA_STAMP(0);
  const int sp = bid % nsplit;
  const T* xb = x + (size_t)b * CIN * HW;
  const int mt0 = (MT * sp) / nsplit, mt1 = (MT * (sp + 1)) / nsplit;
  // epilogue operands of this lane's channels (co = nt*16 + lane%16), loaded up front
  float pre_bias[NT], pre_shift[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int co = nt * 16 + (tid & 15);
    pre_bias[nt] = (MODE == 2) ? 0.f : bias[co];
    pre_shift[nt] = (MODE == 0) ? shift[co] : 0.f;
  }

  // --- stage weights (batched float4 reads in natural [co][ci][kh][kw] order,
  //     scattered LDS writes to wl[co][(kh*5+kw)*CIN + ci])
  const T zero = Cvt<T>::from_f(0.f);
  // WPK 1: the pre-packed tile goes global -> LDS directly (global_load_lds_dwordx4: no
  // VGPRs, so it can be issued with the prologue's first loads without register pressure);
  // with a BN prologue it is issued before the statistics reduction, whose loads and barrier
  // then cover its latency (the barrier's vmcnt(0) retires it; the tile is read only after
  // the compute barrier).  LDS destination = wave-uniform base + lane x 16 B: wl is a
  // contiguous run of 16-B chunks, chunk c at byte 16c.
  constexpr int WN16 = WPK == 1 ? COUT * KPW * (int)sizeof(T) / 16 : 1;
  constexpr int WIT = (WN16 + NTHR - 1) / NTHR;
  auto load_wpk = [&]() {
    if constexpr (WPK == 1) {
      static_assert((COUT * KPW * sizeof(T)) % 16 == 0, "packed weight tile must be whole 16-B chunks");
      static_assert(COUT * KPW == (MODE == 2 ? W2D_LEN : W2F_LEN), "pre-packed weights exist for layer 2 only");
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
      const uint4* src = reinterpret_cast<const uint4*>(wpk);
      uint4* dstl = reinterpret_cast<uint4*>(wl);
      const int wv0 = (tid >> 6) * 64, ln = tid & 63;
#pragma unroll
      for (int i = 0; i < WIT; ++i) {
        const int c0 = i * NTHR + wv0;  // this wave's first chunk (wave-uniform)
        if (c0 + ln < WN16)             // lanes past the tile are masked off: they write nothing
          __builtin_amdgcn_global_load_lds(src + c0 + ln, (lds_ptr_t)(dstl + c0), 16, 0, 0);
      }
    }
  };
  if constexpr (WPK == 1) {
    if constexpr (PRO == 0 || PRO == 3) load_wpk();
  } else {
    if constexpr (KP > K) {
      for (int e = tid; e < COUT * (KP - K); e += NTHR) wl[(e / (KP - K)) * KPW + K + e % (KP - K)] = zero;
    }
    // natural W index e = (o * WIN + i) * 25 + tap, WIN = in-channels of W
    // (= CIN here, = COUT for the data-grad where W is [CIN][COUT][5][5])
    constexpr int KO = 25 * (MODE == 2 ? COUT : CIN);
    stage_f32<COUT * K>(w, [&](int e, float v) {
      const int o = e / KO, rem = e % KO;      // o: out-ch of W
      const int i = rem / 25, tap = rem % 25;  // i: in-ch of W
      if (MODE == 2)  // W_eff[co=i][ci=o][tap'] with tap' = 24 - tap
        wl[i * KPW + (24 - tap) * CIN + o] = Cvt<T>::from_f(v);
      else
        wl[o * KPW + tap * CIN + i] = Cvt<T>::from_f(v);
    });
  }
  if constexpr (WPK == 2) pack_w2<T>(pk);
  DPA_STAMP(1);
  // --- stage the zero-padded image in HWC order: zero the halo pixels
  //     (whole 16-B groups when a pixel is, else element by element)
  if constexpr ((CIN * sizeof(T)) % 16 == 0) {
    constexpr int G = CIN * (int)sizeof(T) / 16;  // 16-B groups per pixel
    uint4* img4 = reinterpret_cast<uint4*>(img);
    for (int e = tid; e < HP * WPD * G; e += NTHR) {
      const int px = e / G, hp = px / WPD, wp = px % WPD;
      if (hp < 2 || hp >= H + 2 || wp < 2 || wp >= W + 2) img4[e] = make_uint4(0u, 0u, 0u, 0u);
    }
  } else {
    for (int e = tid; e < HP * WPD * CIN; e += NTHR) {
      const int hp = e / (WPD * CIN), rem = e % (WPD * CIN);
      const int wp = rem / CIN;
      if (hp < 2 || hp >= H + 2 || wp < 2 || wp >= W + 2) img[e] = zero;
    }
  }
  // EPI: this workgroup's output range of the pooled index / xhat of the block below
  constexpr int EPIX = EPI ? MT * 16 : 1;
  __shared__ uint8_t eidx[EPI ? COUT * EPIX : 1];
  __shared__ T exh[EPI ? COUT * EPIX : 1];
  // (the loads: issued after the BN prologue's barrier; the LDS stores: after
  //  the emit, so the round trip overlaps it)
  const int ep0 = mt0 * 16, enp = min(mt1 * 16, HW) - ep0;
  constexpr int EIT = EPI ? (COUT * EPIX + NTHR - 1) / NTHR : 1;
  uint8_t ei[EIT];
  T ex[EIT];
  auto load_epi = [&]() {
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < EIT; ++i) {
        const int e = tid + i * NTHR;
        const int ec = e < COUT * enp ? e : 0;  // clamped: the loads stay unconditional
        const int co = ec / enp, pp = ec % enp;
        const size_t o = ((size_t)b * COUT + co) * HW + ep0 + pp;
        ei[i] = epi.idx[o];
        ex[i] = epi.xh[o];
      }
    }
  };
  auto store_epi = [&]() {
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < EIT; ++i) {
        const int e = tid + i * NTHR;
        if (e < COUT * enp) {
          const int co = e / enp, pp = e % enp;
          eidx[co * EPIX + pp] = ei[i];
          exh[co * EPIX + pp] = ex[i];
        }
      }
    }
  };
  if constexpr (PRO != 2) {
    load_epi();
    store_epi();
  }
  DPA_STAMP(2);
  // PRO 1: this lane's pooled map / index / xhat outputs (for the backward) are stored AFTER
  // the compute barrier: __syncthreads() waits vmcnt(0), so issued before it they held the
  // whole workgroup until they retired; issued after it they overlap the MFMA loop (step
  // -0.4 us; the same deferral of conv1's gather stores measured no gain,
  // profiles/r4p_deferred_stores_ab.txt)
  constexpr int DQ = PRO != 1 ? 1
                     : (CIN % 8 == 0 && sizeof(T) == 2) ? 8 * ((CIN / 8 * HW + NTHR - 1) / NTHR)
                                                          : (CIN * HW + NTHR - 1) / NTHR;
  int dq_e[DQ];  // pooled-output element of entry d, -1: none
  T dq_p[DQ], dq_x[DQ];
  uint8_t dq_i[DQ];
#pragma unroll
  for (int d = 0; d < DQ; ++d) dq_e[d] = -1;
  if constexpr (PRO == 0) {
    stage_chw<T, CIN, H, W>(xb, [&](int ci, int h, int ww, T a, T bb) {
      img[imo((h + 2) * WPD + (ww + 2), ci)] = a;
      img[imo((h + 2) * WPD + (ww + 3), ci)] = bb;
    });
  } else if constexpr (PRO == 3) {
    // step counter -> sample -> 4 uint8 pixels per lane load
    static_assert(HW % 4 == 0 && W % 4 == 0, "4-pixel groups stay inside a row");
    constexpr int G4 = HW / 4, GIT = (G4 + NTHR - 1) / NTHR;
    const int step = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile int*>(gin.ctr));
    long long pos = (long long)step * gin.nimg + b;
    pos = pos < gin.order_len ? pos : gin.order_len - 1;  // never taken with a correct host-side batch count
    const int64_t src = gin.order[pos];
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(gin.imgs + src * HW);
    uint32_t v4[GIT];
#pragma unroll
    for (int i = 0; i < GIT; ++i)
      if (tid + i * NTHR < G4) v4[i] = s4[tid + i * NTHR];
    if (sp == 0 && tid == 0) gin.lab_out[b] = gin.labels[src];
    T* xo = const_cast<T*>(xb);
#pragma unroll
    for (int i = 0; i < GIT; ++i) {
      const int g = tid + i * NTHR;
      if (g < G4) {
        const int h = (4 * g) / W, ww = (4 * g) % W;
        T px[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          px[k] = Cvt<T>::from_f((float)((v4[i] >> (8 * k)) & 0xffu) * gin.scale + gin.shift);
          img[imo((h + 2) * WPD + (ww + k + 2), 0)] = px[k];
        }
        if (sp == 0) {  // the batch buffer (conv1's weight gradient and the user read it)
#pragma unroll
          for (int k = 0; k < 4; ++k) xo[4 * g + k] = px[k];
        }
      }
    }
    // advance the step counter once every workgroup has read it (relaxed: the next
    // launch reads it after this one completes)
    if (tid == 0) {
      const int arrived = __hip_atomic_fetch_add(&gin.ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (arrived == gin.nimg * nsplit - 1) {
        __hip_atomic_store(&gin.ctr[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&gin.ctr[0], step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if constexpr (PRO == 1) {
    __shared__ float sc_s[CIN], beta_s[CIN], mean_s[CIN], istd_s[CIN];
    __shared__ float part[NTHR];
    typedef typename Pair2<T>::type P;
    constexpr int NPO = CIN * HW;  // pooled outputs of one image = this conv's input
    const T* yb = pin.y + (size_t)b * CIN * 4 * HW;
    const bool wr = pin.p_out != nullptr;
    const int e_lo = NPO * sp / nsplit, e_hi = NPO * (sp + 1) / nsplit;
    if constexpr (CIN % 8 == 0 && sizeof(T) == 2) {
      // a lane owns 8 channels of one pooled pixel (lanes along the pixels: every load
      // instruction reads consecutive pairs of one row): ONE 16-B LDS write of the 8
      // pooled values instead of eight 2-B writes to the same bank group
      constexpr int NO = CIN / 8, NPI = NO * HW, IT8 = (NPI + NTHR - 1) / NTHR;
      P top[IT8][8], bot[IT8][8];
#pragma unroll
      for (int i = 0; i < IT8; ++i) {  // issued before the statistics reduction: the latencies overlap
        const int e8 = tid + i * NTHR;
        if (e8 < NPI) {
          const int o = e8 / HW, pix = e8 % HW, ho = pix / W, wo = pix % W;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const P* src =
                reinterpret_cast<const P*>(yb + ((size_t)(8 * o + j) * 2 * H + 2 * ho) * 2 * W + 2 * wo);
            top[i][j] = src[0];
            bot[i][j] = src[W];  // next input row (2W elements = W pairs)
          }
        }
      }
      load_wpk();
      bn_finalize<CIN>(pin.bn, sc_s, beta_s, mean_s, istd_s, part, bid);
      DPA_STAMP(3);
#pragma unroll
      for (int i = 0; i < IT8; ++i) {
        const int e8 = tid + i * NTHR;
        if (e8 < NPI) {
          const int o = e8 / HW, pix = e8 % HW, ho = pix / W, wo = pix % W;
          unsigned pk[4];  // the 8 pooled values packed in registers (no local array in memory)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int ci = 8 * o + j;
            float best, xh;
            int bi;
            bn_relu_max4x<T>(top[i][j], bot[i][j], sc_s[ci], beta_s[ci], mean_s[ci], istd_s[ci], best, bi, xh);
            const T pvj = Cvt<T>::from_f(best);
            const unsigned bits = __builtin_bit_cast(unsigned short, pvj);
            if (j & 1) pk[j >> 1] |= bits << 16; else pk[j >> 1] = bits;
            const int e = ci * HW + pix;  // (ci, pix) index of the pooled outputs
            const int d = i * 8 + j;
            dq_e[d] = wr && e >= e_lo && e < e_hi ? e : -1;
            dq_p[d] = pvj;
            dq_i[d] = (uint8_t)(bi | (best > 0.f ? IDX_RELU : 0));
            dq_x[d] = Cvt<T>::from_f(xh);
          }
          // imo keeps each 8-channel group of a pixel contiguous (the swizzle moves groups)
          *reinterpret_cast<uint4*>(&img[imo((ho + 2) * WPD + (wo + 2), 8 * o)]) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
      }
    } else {
      constexpr int IT = (NPO + NTHR - 1) / NTHR;
      P top[IT], bot[IT];
#pragma unroll
      for (int i = 0; i < IT; ++i) {  // issued before the statistics reduction: the latencies overlap
        const int e = tid + i * NTHR;
        if (e < NPO) {
          const int ci = e / HW, pix = e % HW, ho = pix / W, wo = pix % W;
          const P* src = reinterpret_cast<const P*>(yb + ((size_t)ci * 2 * H + 2 * ho) * 2 * W + 2 * wo);
          top[i] = src[0];
          bot[i] = src[W];  // next input row (2W elements = W pairs)
        }
      }
      load_wpk();
      bn_finalize<CIN>(pin.bn, sc_s, beta_s, mean_s, istd_s, part, bid);
      DPA_STAMP(3);
      // the pooled map / index / xhat outputs (for the backward) are written by all
      // nsplit workgroups of the image, each its share (was: split 0 alone)
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int e = tid + i * NTHR;
        if (e < NPO) {
          const int ci = e / HW, pix = e % HW, ho = pix / W, wo = pix % W;
          float best, xh;
          int bi;
          bn_relu_max4x<T>(top[i], bot[i], sc_s[ci], beta_s[ci], mean_s[ci], istd_s[ci], best, bi, xh);
          const T pv = Cvt<T>::from_f(best);
          img[imo((ho + 2) * WPD + (wo + 2), ci)] = pv;
          dq_e[i] = wr && e >= e_lo && e < e_hi ? e : -1;
          dq_p[i] = pv;
          dq_i[i] = (uint8_t)(bi | (best > 0.f ? IDX_RELU : 0));
          dq_x[i] = Cvt<T>::from_f(xh);
        }
      }
    }
  } else {
    __shared__ float coef[5 * CIN], sums[2 * CIN];
    __shared__ float part[NTHR];
    if constexpr (CIN % 8 == 0 && sizeof(T) == 2) {
      BnBwdStage8<T, CIN, H, W, NTHR> st;
      st.load(bin, b);
      DPA_STAMP(8);
      load_wpk();
      bn_bwd_coef<CIN, T>(bin, coef, part, sums, bid);
      load_epi();
      DPA_STAMP(3);
      st.emit(coef, [&](int h, int ww, int c0, uint4 q00, uint4 q01, uint4 q10, uint4 q11) {
        *reinterpret_cast<uint4*>(&img[imo((h + 2) * WPD + (ww + 2), c0)]) = q00;
        *reinterpret_cast<uint4*>(&img[imo((h + 2) * WPD + (ww + 3), c0)]) = q01;
        *reinterpret_cast<uint4*>(&img[imo((h + 3) * WPD + (ww + 2), c0)]) = q10;
        *reinterpret_cast<uint4*>(&img[imo((h + 3) * WPD + (ww + 3), c0)]) = q11;
      });
    } else {
      BnBwdStage<T, CIN, H, W, NTHR> st;
      st.load(bin, b);
      DPA_STAMP(8);
      load_wpk();
      bn_bwd_coef<CIN, T>(bin, coef, part, sums, bid);
      load_epi();
      DPA_STAMP(3);
      st.emit(coef, [&](int c, int h, int ww, T v00, T v01, T v10, T v11) {
        img[imo((h + 2) * WPD + (ww + 2), c)] = v00;
        img[imo((h + 2) * WPD + (ww + 3), c)] = v01;
        img[imo((h + 3) * WPD + (ww + 2), c)] = v10;
        img[imo((h + 3) * WPD + (ww + 3), c)] = v11;
      });
    }
    store_epi();
  }
  DPA_STAMP(4);
  __syncthreads();
  DPA_STAMP(5);
  if constexpr (PRO == 1) {  // the deferred pooled outputs (see dq_e)
    constexpr int NPO = CIN * HW;
#pragma unroll
    for (int d = 0; d < DQ; ++d)
      if (dq_e[d] >= 0) {
        const size_t o = (size_t)b * NPO + dq_e[d];
        pin.p_out[o] = dq_p[d];
        pin.idx_out[o] = dq_i[d];
        pin.xh_out[o] = dq_x[d];
      }
  }

  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, q = lane >> 4;

  float s1[NT], s2[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) s1[nt] = s2[nt] = 0.f;

  for (int mt = mt0 + wv; mt < mt1; mt += NTHR / 64) {
    const int m = mt * 16 + r;
    const int mm_ = m < HW ? m : HW - 1;
    const int oh = mm_ / W, ow = mm_ % W;
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      typename mm::frag a;
      if constexpr (CIN == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 32 * s + 8 * q + j;
          float v = 0.f;
          if (tap < 25) v = Cvt<T>::to_f(img[(oh + tap / 5) * WPD + ow + tap % 5]);
          a[j] = mm::cv(v);
        }
      } else {
        const int kb = 32 * s + 8 * q;
        int tap = kb / CIN;
        const int ci0 = kb % CIN;
        tap = tap < 25 ? tap : 24;  // K padding: weights are zero there
        a = mm::ld(&img[imo((oh + tap / 5) * WPD + ow + tap % 5, ci0)]);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const typename mm::frag bf = mm::ld(&wl[(nt * 16 + r) * KPW + 32 * s + 8 * q]);
        acc[nt] = mm::mma(a, bf, acc[nt]);
      }
    }
    // --- epilogue: D[row = 4q+i][col = r] -> pixel mt*16+4q+i, channel nt*16+r
    const int pix0 = mt * 16 + 4 * q;
    if (pix0 < HW) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int co = nt * 16 + r;
        const float bs = pre_bias[nt];
        T* dst = y + ((size_t)b * COUT + co) * HW + pix0;
        const float sh = pre_shift[nt];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[nt][i] + bs;
          dst[i] = Cvt<T>::from_f(v);
          if (MODE == 0) {
            const float d = rnd_t<T>(v) - sh;
            s1[nt] += d;
            s2[nt] += d * d;
          }
          if (EPI == 1) {
            const int le = co * EPIX + pix0 - mt0 * 16 + i;
            const float g = (eidx[le] & IDX_RELU) ? rnd_t<T>(v) : 0.f;
            s1[nt] += g;
            s2[nt] += g * Cvt<T>::to_f(exh[le]);
          }
        }
      }
    }
  }
  DPA_STAMP(6);
  if constexpr (MODE == 0 || EPI == 1) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      // lanes r, r+16, r+32, r+48 (VALU permlane swaps, no LDS round trip; every lane active)
      const float a1 = xor32_sum(xor16_sum(s1[nt])), a2 = xor32_sum(xor16_sum(s2[nt]));
      if (q == 0) {  // per-wave partials, summed below in a fixed order (deterministic)
        lstat[wv * 2 * COUT + nt * 16 + r] = a1;
        lstat[wv * 2 * COUT + COUT + nt * 16 + r] = a2;
      }
    }
    __syncthreads();
    float* row = (MODE == 0 ? fslab + (size_t)bid * fslab_row(COUT)
                            : epi.bslab + (size_t)bid * 2 * COUT);
    if (tid < 2 * COUT) {
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NTHR / 64; ++w2) t += lstat[w2 * 2 * COUT + tid];
      row[tid] = t;
    }
    if constexpr (MODE == 0) {
      if (tid == 0) {
        const int p0 = mt0 * 16, p1 = min(mt1 * 16, HW);
        row[2 * COUT] = (float)(p1 - p0);
      }
      if (bid == 0 && tid < COUT) fstats[2 * COUT + 1 + tid] = shift[tid];
    }
  }
  DPA_STAMP(7);
}

template <typename T, int CIN, int COUT, int H, int W, int MODE, int PRO = 0, int EPI = 0, int WPK = 0>
__global__ void __launch_bounds__(NTHR)
conv5x5_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
               T* __restrict__ y, float* __restrict__ fslab, float* __restrict__ fstats,
               const float* __restrict__ shift, int nsplit, PoolIn<T> pin = PoolIn<T>{},
               BwdIn<T> bin = BwdIn<T>{}, BwdEpi<T> epi = BwdEpi<T>{}, const T* __restrict__ wpk = nullptr,
               WPack<T> pk = WPack<T>{}, GatherIn gin = GatherIn{}) {
  conv5x5_body<T, CIN, COUT, H, W, MODE, PRO, EPI, WPK>(x, w, bias, y, fslab, fstats, shift, nsplit, pin, bin, epi,
                                                        wpk, pk, (int)blockIdx.x, gin);
}

// ---------------------------------------------------------------------------
// BN finalize + normalise + ReLU + 2x2/2 max-pool (+ argmax index, first max
// wins in (dy,dx) scan order as ATen's max_pool2d).  One thread per pooled
// output.  Each workgroup first reduces the conv's per-workgroup partial sums
// (nrows x (2C+1) floats, L2-resident); workgroup 0 publishes the final sums to
// fstats and updates the running stats (momentum<0 => cumulative average).
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bn_relu_pool_kernel(const T* __restrict__ y, const float* __restrict__ fslab, int nrows,
                    float* __restrict__ fstats, const float* __restrict__ gamma, const float* __restrict__ beta,
                    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
                    float momentum, float eps, int train, T* __restrict__ p, uint8_t* __restrict__ idx,
                    int total) {
  constexpr int HO = H / 2, WO = W / 2;
  constexpr int RL = 2 * C + 1;
  __shared__ float part[NTHR];
  __shared__ float sc_s[C], beta_s[C], mean_s[C];
  const int tid = threadIdx.x;
  if (train) {
    // column j of the slab summed over rows; NTHR/RL row-groups in parallel
    constexpr int G = NTHR / RL;  // >= 3 for C <= 32
    static_assert(G >= 1, "C too large");
    const int j = tid % RL, g = tid / RL;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (g < G) {
      int rr = g;
      for (; rr + 3 * G < nrows; rr += 4 * G) {
        a0 += fslab[(size_t)rr * RL + j];
        a1 += fslab[(size_t)(rr + G) * RL + j];
        a2 += fslab[(size_t)(rr + 2 * G) * RL + j];
        a3 += fslab[(size_t)(rr + 3 * G) * RL + j];
      }
      for (; rr < nrows; rr += G) a0 += fslab[(size_t)rr * RL + j];
    }
    part[tid] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (tid < RL) {
      float t = 0.f;
      for (int gg = 0; gg < G; ++gg) t += part[gg * RL + tid];
      part[tid] = t;  // each tid < RL only touches its own column's slots (gg*RL + tid)
    }
    __syncthreads();
    if (tid < C) {
      const float n = part[2 * C];
      const float m1 = part[tid] / n;
      const float shv = fstats[2 * C + 1 + tid];
      const float mean = shv + m1;
      const float var = fmaxf(part[C + tid] / n - m1 * m1, 0.f);
      const float invstd = rsqrtf(var + eps);
      const float s = gamma[tid] * invstd;
      sc_s[tid] = s;
      beta_s[tid] = beta[tid];
      mean_s[tid] = mean;
      if (blockIdx.x == 0) {
        fstats[tid] = part[tid];
        fstats[C + tid] = part[C + tid];
        if (tid == 0) fstats[2 * C] = n;
        const int64_t nb = nbt[0] + 1;
        const float mom = momentum >= 0.f ? momentum : 1.f / (float)nb;
        rmean[tid] = (1.f - mom) * rmean[tid] + mom * mean;
        rvar[tid] = (1.f - mom) * rvar[tid] + mom * var * (n / fmaxf(n - 1.f, 1.f));
      }
    }
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0) nbt[0] = nbt[0] + 1;
  } else {
    if (tid < C) {
      const float invstd = rsqrtf(rvar[tid] + eps);
      const float s = gamma[tid] * invstd;
      sc_s[tid] = s;
      beta_s[tid] = beta[tid];
      mean_s[tid] = rmean[tid];
    }
    __syncthreads();
  }
  const int e = blockIdx.x * NTHR + tid;
  if (e >= total) return;
  const int c = (e / (HO * WO)) % C;
  const float sc = sc_s[c], bt = beta_s[c], mn = mean_s[c];
  const int bc = e / (HO * WO), pix = e % (HO * WO);
  const int ho = pix / WO, wo = pix % WO;
  const T* src = y + (size_t)bc * H * W + (2 * ho) * W + 2 * wo;
  float best = -1.f;
  int bi = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = Cvt<T>::to_f(src[(k >> 1) * W + (k & 1)]);
    const float z = fmaxf(rnd_t<T>((v - mn) * sc + bt), 0.f);
    if (z > best) { best = z; bi = k; }
  }
  p[e] = Cvt<T>::from_f(best);
  idx[e] = (uint8_t)bi;
}

// mean / invstd of channel c from the final stats buffer.
template <int C>
__device__ __forceinline__ void stats_mean_invstd(const float* fstats, int c, float eps, float& mean,
                                                  float& invstd, float& n) {
  n = fstats[2 * C];
  const float m1 = fstats[c] / n;
  mean = fstats[2 * C + 1 + c] + m1;
  invstd = rsqrtf(fmaxf(fstats[C + c] / n - m1 * m1, 0.f) + eps);
}

// ---------------------------------------------------------------------------
// Backward part 1: route the pooled grad through max-pool (argmax) and ReLU
// (pooled output > 0), and reduce per channel into bslab[split][2C]:
//   [c]     sum dy          (-> grad of BN bias)
//   [C + c] sum dy * xhat   (-> grad of BN weight)
// grid = (C, kBwdSplit over the batch).
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bwd_reduce_kernel(const T* __restrict__ dp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                  const T* __restrict__ y, const float* __restrict__ fstats, float eps,
                  float* __restrict__ bslab, int B) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  __shared__ float red[2 * NTHR / 64];
  const int c = blockIdx.x;
  const int nsplit = gridDim.y;
  const int b0 = (B * blockIdx.y) / nsplit, b1 = (B * (blockIdx.y + 1)) / nsplit;
  float mean, invstd, n;
  stats_mean_invstd<C>(fstats, c, eps, mean, invstd, n);
  float a1 = 0.f, a2 = 0.f;
  const int cnt = (b1 - b0) * PP;
  for (int t = threadIdx.x; t < cnt; t += NTHR) {
    const int b = b0 + t / PP, pix = t % PP;
    const size_t e = ((size_t)b * C + c) * PP + pix;
    const float pv = Cvt<T>::to_f(p[e]);
    if (pv > 0.f) {
      const float g = Cvt<T>::to_f(dp[e]);
      const int k = idx[e];
      const int ho = pix / WO, wo = pix % WO;
      const float yv = Cvt<T>::to_f(
          y[((size_t)b * C + c) * H * W + (2 * ho + (k >> 1)) * W + 2 * wo + (k & 1)]);
      a1 += g;
      a2 += g * (yv - mean) * invstd;
    }
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { red[wv] = a1; red[NTHR / 64 + wv] = a2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t1 = 0.f, t2 = 0.f;
    for (int i = 0; i < NTHR / 64; ++i) { t1 += red[i]; t2 += red[NTHR / 64 + i]; }
    bslab[blockIdx.y * 2 * C + c] = t1;
    bslab[blockIdx.y * 2 * C + C + c] = t2;
  }
}

// ---------------------------------------------------------------------------
// Backward part 2: BN input gradient at full resolution, one thread per
// pooled element (its 2x2 window):
//   dx = gamma*invstd*(dy - S1/n - xhat*S2/n),  dy = routed pooled grad or 0
// S1, S2 = column sums of the (all-reduced) bslab.
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bwd_elemt_kernel(const T* __restrict__ dp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                 const T* __restrict__ y, const float* __restrict__ fstats,
                 const float* __restrict__ gslab, int nsplit, const float* __restrict__ gamma, float eps,
                 T* __restrict__ dx, int total) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  __shared__ float k_s[3 * C];
  __shared__ float m_s[2 * C];
  const int tid = threadIdx.x;
  if (tid < C) {
    float s1 = 0.f, s2 = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      s1 += gslab[s * 2 * C + tid];
      s2 += gslab[s * 2 * C + C + tid];
    }
    float mean, invstd, n;
    stats_mean_invstd<C>(fstats, tid, eps, mean, invstd, n);
    k_s[tid] = s1 / n;
    k_s[C + tid] = s2 / n;
    k_s[2 * C + tid] = gamma[tid] * invstd;
    m_s[tid] = mean;
    m_s[C + tid] = invstd;
  }
  __syncthreads();
  const int e = blockIdx.x * NTHR + tid;
  if (e >= total) return;
  const int bc = e / PP, pix = e % PP;
  const int c = bc % C;
  const float k1 = k_s[c], k2 = k_s[C + c], gi = k_s[2 * C + c];
  const float mean = m_s[c], invstd = m_s[C + c];
  const float pv = Cvt<T>::to_f(p[e]);
  const float g = pv > 0.f ? Cvt<T>::to_f(dp[e]) : 0.f;
  const int kk = idx[e];
  const int ho = pix / WO, wo = pix % WO;
  const size_t base = (size_t)bc * H * W + (2 * ho) * W + 2 * wo;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t o = base + (k >> 1) * W + (k & 1);
    const float xh = (Cvt<T>::to_f(y[o]) - mean) * invstd;
    const float dy = (k == kk) ? g : 0.f;
    dx[o] = Cvt<T>::from_f(gi * (dy - k1 - xh * k2));
  }
}

// ---------------------------------------------------------------------------
// Weight/bias gradient partials of the 5x5 conv.  One workgroup per
// (image, row-chunk); writes wslab[blk][COUT*N + COUT] (dW partial | db partial).
// GEMM: rows = COUT, cols = (ci, kh, kw) natural order, K = pixels of the chunk
// with the row padded to WP = ceil8(W) (dy is zero in the pad columns).
// LDS: dy[COUT][ROWS][WP] and 5 kw-shifted copies xs[kw][CIN][ROWS+4][WP] of
// the zero-padded input so both operands are aligned 16-B LDS reads.
// When there are fewer (m,n) tile pairs than waves, waves split K instead
// and combine through LDS.
// ---------------------------------------------------------------------------
// PRO 2: dy is produced on the fly from the pooled grad of the next block
// (bin: backward through MaxPool -> ReLU -> BN); needs ROWS == H.
// WT: the partial row is stored write-through (sc1) for an in-launch reduction
// (MI355X_MICROARCH.md "Valid forms" row 1; convnet_fused.hip wgrad1_reduce_kernel).
// Dynamic-LDS bytes of conv5x5_wgrad_body<..., DYN = true> (its dy rows, shifted input
// copies, padded input and staged partial row; the small arrays stay static).
template <typename T, int CIN, int COUT, int H, int W, int ROWS>
struct WgradLds {
  static constexpr int WP = ceil_to(W, 8), XR = ROWS + 4, WX = WP + 4, N = CIN * 25;
  static constexpr int DYS = ROWS * WP + 8, XCS = XR * WP + 8;
  static constexpr bool DIRECT = ROWS == H, CIF = CIN >= 16;
  static constexpr size_t DYL = sizeof(T) * (size_t)COUT * DYS;
  static constexpr size_t XS = sizeof(T) * (size_t)5 * CIN * XCS;
  static constexpr size_t XPAD = sizeof(T) * (size_t)(DIRECT ? 8 : CIN * XR * WX);
  static constexpr size_t BASE = DYL + XS + XPAD;
  static constexpr bool STAGE = CIF && BASE + sizeof(float) * (size_t)COUT * N <= 144 * 1024;
  static constexpr size_t o_xs = (DYL + 15) / 16 * 16, o_xpad = (o_xs + XS + 15) / 16 * 16,
                          o_wt = (o_xpad + XPAD + 15) / 16 * 16;
  static constexpr size_t bytes = o_wt + sizeof(float) * (STAGE ? (size_t)COUT * N : 4);
};

template <typename T, int CIN, int COUT, int H, int W, int ROWS, int PRO = 0, bool WT = false, bool CHK = false,
          bool DYN = false>
__device__ __forceinline__ void
conv5x5_wgrad_body(const T* __restrict__ x, const T* __restrict__ dy, float* __restrict__ wslab, int nsplit,
                   const BwdIn<T>& bin, const int bid) {
  auto put = [](float* p, float v) {
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
  };
  static_assert(PRO == 0 || (PRO == 2 && ROWS % 2 == 0), "PRO 2 works on whole 2x2 pooling windows");
  constexpr int WP = ceil_to(W, 8);
  static_assert((ROWS * WP) % 32 == 0, "ROWS*WP must be a multiple of 32");
  constexpr int KSTEPS = ROWS * WP / 32;
  constexpr int N = CIN * 25;
  constexpr int NTL = (N + 15) / 16;
  constexpr int MTL = COUT / 16;
  constexpr int PAIRS = MTL * NTL;
  constexpr int NW = NTHR / 64;
  constexpr int KSPLIT = PAIRS >= NW ? 1 : NW / PAIRS;  // waves per pair
  constexpr int XR = ROWS + 4;
  constexpr int ROWLEN = COUT * N + COUT;
  typedef MM<T> mm;
  // LDS pitches padded by 16 B so the MFMA operand reads spread over the banks:
  //  * dy rows (A operand: 16 lanes = 16 output channels) DYS apart;
  //  * input copies (B operand) XCS apart per (kw, ci); with CIN >= 16 the GEMM columns
  //    run ci-fastest (column n = tap*CIN + ci), so the 16 lanes of a fragment read 16
  //    channels of one tap: 16 distinct 4-bank windows.  (CIN = 1: 16 taps, <= 2-way.)
  constexpr int DYS = ROWS * WP + 8;
  constexpr int XCS = XR * WP + 8;
  constexpr bool CIF = CIN >= 16;  // ci-fastest column order
  constexpr int WX = WP + 4;  // padded input row (2 halo columns each side, room for the kw shift)
  // whole image per workgroup: the 5 shifted copies are written straight from
  // registers (no padded staging image, no LDS->LDS copy pass)
  constexpr bool DIRECT = (ROWS == H);
  __shared__ f32x4 kred[KSPLIT > 1 ? NW : 1][64];
  // the partial row in natural order, staged for whole-chunk stores where LDS allows
  using WL = WgradLds<T, CIN, COUT, H, W, ROWS>;
  constexpr bool STAGE = WL::STAGE;
  T* dyl;
  T* xs;
  T* xpad;
  float* wtile;
  if constexpr (DYN) {
    dyl = reinterpret_cast<T*>(dpa_dyn_lds);
    xs = reinterpret_cast<T*>(dpa_dyn_lds + WL::o_xs);
    xpad = reinterpret_cast<T*>(dpa_dyn_lds + WL::o_xpad);
    wtile = reinterpret_cast<float*>(dpa_dyn_lds + WL::o_wt);
  } else {
    __shared__ __attribute__((aligned(16))) T dyl_s[COUT * DYS];
    __shared__ __attribute__((aligned(16))) T xs_s[5 * CIN * XCS];
    __shared__ __attribute__((aligned(16))) T xpad_s[DIRECT ? 8 : CIN * XR * WX];
    __shared__ __attribute__((aligned(16))) float wtile_s[STAGE ? COUT * N : 4];
    dyl = dyl_s;
    xs = xs_s;
    xpad = xpad_s;
    wtile = wtile_s;
  }

  const int tid = threadIdx.x;
  const int b = bid / nsplit, sp = bid % nsplit;
  DPA_STAMP(0);
  // producer-side check of this workgroup's partial row (BwdIn::chk_row_slot0, common.h)
  const bool rchk = CHK && bin.chk_rows;  // (compiled only where a launch can ask for it)
  const int r0 = sp * ROWS;
  const T* xb = x + (size_t)b * CIN * H * W;
  // input rows r0-2 .. r0+ROWS+1 -> xpad interior; all loads issued before the
  // first LDS store (one memory round trip, not one per loop iteration)
  auto stage_xpad = [&]() {
    if constexpr (!DIRECT) {
      constexpr int XN = CIN * XR * W, XIT = (XN + NTHR - 1) / NTHR;
      T xv[XIT];
#pragma unroll
      for (int i = 0; i < XIT; ++i) {
        const int e = threadIdx.x + i * NTHR;
        const int ci = e / (XR * W), rem = e % (XR * W);
        const int rr = rem / W, cc = rem % W;
        const int ih = r0 + rr - 2;
        const bool ok = e < XN && ih >= 0 && ih < H;
        xv[i] = xb[ok ? (ci * H + ih) * W + cc : 0];
      }
#pragma unroll
      for (int i = 0; i < XIT; ++i) {
        const int e = threadIdx.x + i * NTHR;
        const int ci = e / (XR * W), rem = e % (XR * W);
        const int rr = rem / W, cc = rem % W;
        const int ih = r0 + rr - 2;
        if (e < XN && ih >= 0 && ih < H) xpad[(ci * XR + rr) * WX + cc + 2] = xv[i];
      }
    }
  };
  const T* dyb = dy + (size_t)b * COUT * H * W;
  const T zero = Cvt<T>::from_f(0.f);

  // dy chunk -> dyl[co][rr][0..WP) (pad columns zero)
  for (int e = tid; e < COUT * ROWS * (WP - W); e += NTHR) {
    const int cr = e / (WP - W), cc = W + e % (WP - W);
    dyl[(cr / ROWS) * DYS + (cr % ROWS) * WP + cc] = zero;
  }
  if (r0 + ROWS > H) {  // rows past the image (last chunk): zero
    for (int e = tid; e < COUT * ROWS * WP; e += NTHR)
      if (r0 + (e / WP) % ROWS >= H) dyl[(e / (ROWS * WP)) * DYS + e % (ROWS * WP)] = zero;
  }
  // xs[kw][ci][rr][c] = x[ci][r0 + rr - 2][c + kw - 2] (zero outside the image)
  auto scatter5 = [&](int ci, int rr, int w, T v) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
      const int c = w + 2 - kw;
      if (c >= 0 && c < WP) xs[(kw * CIN + ci) * XCS + rr * WP + c] = v;
    }
  };
  if constexpr (DIRECT) {
    constexpr int NZ = 5 * CIN * XCS * (int)sizeof(T) / 16;
    static_assert((5 * CIN * XCS * sizeof(T)) % 16 == 0, "xs must be a whole number of 16-B chunks");
    uint4* z = reinterpret_cast<uint4*>(xs);
    for (int e = tid; e < NZ; e += NTHR) z[e] = make_uint4(0u, 0u, 0u, 0u);
  } else {
    // input rows r0-2 .. r0+ROWS+1 -> xpad[ci][XR][WX], columns shifted by 2 (zero halo)
    for (int e = tid; e < CIN * XR * WX; e += NTHR) {
      const int cc = e % WX, rr = (e / WX) % XR;
      const int ih = r0 + rr - 2;
      if (cc < 2 || cc >= W + 2 || ih < 0 || ih >= H) xpad[e] = zero;
    }
  }
  if constexpr (PRO == 2) {
    __shared__ float coef[5 * COUT], sums[2 * COUT];
    __shared__ float part[NTHR];
    BnBwdStage<T, COUT, H, W, NTHR, ROWS> st;
    st.load(bin, b, r0);
    if constexpr (DIRECT) {
      __syncthreads();  // xs zero-fill before the scatter
      stage_chw<T, CIN, H, W>(xb, [&](int ci, int h, int ww, T a, T bb) {
        scatter5(ci, h + 2, ww, a);
        scatter5(ci, h + 2, ww + 1, bb);
      });
    } else {  // input rows r0-2 .. r0+ROWS+1 -> xpad (kw copies after the barrier below)
      stage_xpad();
    }
    bn_bwd_coef<COUT, T>(bin, coef, part, sums, bid);
    DPA_STAMP(3);
    st.emit(coef, [&](int co, int h, int ww, T v00, T v01, T v10, T v11) {
      dyl[co * DYS + h * WP + ww] = v00;
      dyl[co * DYS + h * WP + ww + 1] = v01;
      dyl[co * DYS + (h + 1) * WP + ww] = v10;
      dyl[co * DYS + (h + 1) * WP + ww + 1] = v11;
    });
  } else if constexpr (DIRECT) {  // both operands are full [C][H][W] images
    stage_chw<T, COUT, H, W>(dyb, [&](int co, int h, int ww, T a, T bb) {
      dyl[co * DYS + h * WP + ww] = a;
      dyl[co * DYS + h * WP + ww + 1] = bb;
    });
    __syncthreads();  // xs zero-fill before the scatter
    stage_chw<T, CIN, H, W>(xb, [&](int ci, int h, int ww, T a, T bb) {
      scatter5(ci, h + 2, ww, a);
      scatter5(ci, h + 2, ww + 1, bb);
    });
  } else {
    for (int e = tid; e < COUT * ROWS * W; e += NTHR) {
      const int co = e / (ROWS * W), rem = e % (ROWS * W);
      const int rr = rem / W, cc = rem % W;
      if (r0 + rr < H) dyl[co * DYS + rr * WP + cc] = dyb[(co * H + r0 + rr) * W + cc];
    }
    stage_xpad();
  }
  DPA_STAMP(4);
  __syncthreads();
  if constexpr (!DIRECT) {
    // 5 kw-shifted copies, LDS -> LDS: xs[kw][ci][rr][c] = xpad[ci][rr][c + kw]
    for (int e = tid; e < 5 * CIN * XR * (WP / 8); e += NTHR) {
      const int c8 = e % (WP / 8);
      const int rowid = e / (WP / 8);  // (kw, ci, rr)
      const int kw = rowid / (CIN * XR), cr = rowid % (CIN * XR);
      const T* srcp = &xpad[cr * WX + 8 * c8 + kw];
      T* dstp = &xs[(kw * CIN + cr / XR) * XCS + (cr % XR) * WP + 8 * c8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dstp[j] = srcp[j];
    }
    __syncthreads();
  }

  float* row_out = wslab + (size_t)bid * ROWLEN;
  DPA_STAMP(5);
  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  // bias grad partial: per output channel sum of dy over this chunk.  TPC lanes
  // per channel, each summing 16-B groups (fixed order), then a TPC-lane
  // butterfly: one pass for all channels (a wave-wide reduction per channel
  // cost ~2 us here)
  {
    constexpr int TPC = NTHR / COUT;
    static_assert(NTHR % COUT == 0 && TPC <= 64 && (TPC & (TPC - 1)) == 0, "bias-sum lane groups");
    constexpr int E = ROWS * WP;
    static_assert(E % 8 == 0, "dy rows are whole 16-B groups");
    const int co = tid / TPC, sub = tid % TPC;
    float a = 0.f;
    for (int i = sub * 8; i < E; i += TPC * 8) {
      const typename mm::frag v = mm::ld(&dyl[co * DYS + i]);
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) a += Cvt<T>::to_f(e[j]);
    }
    a = group_sum<TPC>(a);  // VALU lane moves (every lane active here)
    if (sub == 0) {
      put(&row_out[COUT * N + co], a);
      // the bias column is summed by the AMP step like the weight columns: same row bound
      if (rchk) bin.chk.flag(GradChk::bad(a, bin.chk_row_bound));
    }
  }
  DPA_STAMP(6);
  const int ks = KSPLIT > 1 ? wv % KSPLIT : 0;
  const int pstart = KSPLIT > 1 ? wv / KSPLIT : wv;
  const int pstep = KSPLIT > 1 ? NW / KSPLIT : NW;
  for (int pr = pstart; pr < PAIRS; pr += pstep) {
    const int mt = pr / NTL, nt = pr % NTL;
    int n = nt * 16 + r;
    n = n < N ? n : 0;
    const int ci = CIF ? n % CIN : n / 25, tap = CIF ? n / CIN : n % 25;
    const int kh = tap / 5, kw = tap % 5;
    const T* brow = &xs[(kw * CIN + ci) * XCS + kh * WP];
    const T* arow = &dyl[(mt * 16 + r) * DYS];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = ks; s < KSTEPS; s += KSPLIT) {
      const int P = 32 * s + 8 * q;  // pixel index within the chunk
      const int row = P / WP, col0 = P % WP;
      const typename mm::frag a = mm::ld(arow + P);
      const typename mm::frag bf = mm::ld(brow + row * WP + col0);
      acc = mm::mma(a, bf, acc);
    }
    if constexpr (KSPLIT > 1) {
      kred[wv][lane] = acc;
      __syncthreads();
      if (ks != 0) continue;
      for (int k2 = 1; k2 < KSPLIT; ++k2) acc += kred[wv + k2][lane];
    }
    // D[row = 4q+i][col = r]: dW[co = mt*16+4q+i][ci][kh][kw] (natural order in the row)
    const int col = nt * 16 + r;
    if (col < N) {
      const int nat = CIF ? (col % CIN) * 25 + col / CIN : col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (STAGE) wtile[(mt * 16 + 4 * q + i) * N + nat] = acc[i];
        else put(&row_out[(mt * 16 + 4 * q + i) * N + nat], acc[i]);
        if (rchk) bin.chk.flag(GradChk::bad(acc[i], bin.chk_row_bound));
      }
    }
  }
  if constexpr (STAGE) {
    // ci-fastest columns land 25 floats apart in the natural row: 64-lane stores to ~40
    // lines each.  Staged through LDS instead, the row leaves as whole 16-B chunks
    // (consecutive lanes, consecutive addresses).
    static_assert((COUT * N) % 4 == 0 && ROWLEN % 4 == 0, "wgrad rows: whole 16-B chunks");
    __syncthreads();
    if constexpr (WT) {  // 4-B write-through stores, consecutive lanes on consecutive words
      for (int e = tid; e < COUT * N; e += NTHR) put(&row_out[e], wtile[e]);
    } else {
      for (int e = tid; e < COUT * N / 4; e += NTHR)
        *reinterpret_cast<f32x4*>(&row_out[4 * e]) = *reinterpret_cast<const f32x4*>(&wtile[4 * e]);
    }
  }
  DPA_STAMP(7);
}

template <typename T, int CIN, int COUT, int H, int W, int ROWS, int PRO = 0>
__global__ void __launch_bounds__(NTHR)
conv5x5_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy, float* __restrict__ wslab,
                     int nsplit, BwdIn<T> bin = BwdIn<T>{}) {
  conv5x5_wgrad_body<T, CIN, COUT, H, W, ROWS, PRO>(x, dy, wslab, nsplit, bin, (int)blockIdx.x);
}

// ---------------------------------------------------------------------------
// Column sums of up to two slabs in one launch:
//   out1[i] = sum_r slab1[r*n1 + i]  (i < n1),  out2[j] = sum_r slab2[r*n2 + j]  (j < n2)
// A workgroup owns 16 columns; its 16 row-groups each sum every 16th row
// (independent loads in flight), then combine through LDS.
// ---------------------------------------------------------------------------
constexpr int SR_COLS = 16, SR_GROUPS = NTHR / SR_COLS;
__device__ __forceinline__ void slab_reduce_body(const float* __restrict__ slab1, int rows1, int n1,
                                                 float* __restrict__ out1, const float* __restrict__ slab2, int rows2,
                                                 int n2, float* __restrict__ out2, int bid,
                                                 GradChk chk = GradChk{}) {
  __shared__ float part[SR_GROUPS][SR_COLS + 1];
  const int nb1 = (n1 + SR_COLS - 1) / SR_COLS;
  const bool first = bid < nb1;
  const float* slab = first ? slab1 : slab2;
  const int rows = first ? rows1 : rows2;
  const int n = first ? n1 : n2;
  float* out = first ? out1 : out2;
  const int c0 = (first ? bid : bid - nb1) * SR_COLS;
  const int col = c0 + (threadIdx.x % SR_COLS), g = threadIdx.x / SR_COLS;
  part[g][threadIdx.x % SR_COLS] = slab_colsum<SR_GROUPS>(slab, rows, n, col, g);
  __syncthreads();
  if (threadIdx.x < SR_COLS && c0 + (int)threadIdx.x < n) {
    float t = 0.f;
#pragma unroll
    for (int gg = 0; gg < SR_GROUPS; ++gg) t += part[gg][threadIdx.x];
    out[c0 + threadIdx.x] = t;
    if (chk.word != nullptr) chk.flag(GradChk::bad(t, chk.bound));  // (producer-side check, common.h)
  }
}
static __global__ void __launch_bounds__(NTHR)
slab_reduce_kernel(const float* __restrict__ slab1, int rows1, int n1, float* __restrict__ out1,
                   const float* __restrict__ slab2, int rows2, int n2, float* __restrict__ out2) {
  slab_reduce_body(slab1, rows1, n1, out1, slab2, rows2, n2, out2, (int)blockIdx.x);
}

}  // namespace cb
}  // namespace dpa
