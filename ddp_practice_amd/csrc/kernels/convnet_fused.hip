// Whole-ConvNet fused kernels (ops/convnet_fused.py).  Layer boundaries are
// fused where the data dependence allows it:
//
//   forward   gather | conv1(+BN1 partial sums) | [BN1-ReLU-pool1 -> conv2 (+BN2 sums)]
//             | [BN2-ReLU-pool2 -> fc] -> logits
//   backward  [fc bwd + pool2/ReLU2 routing + BN2 reduce (+ BN2 input grad)]
//             | conv2 wgrad | conv2 dgrad | [pool1/ReLU1 routing + BN1 reduce (+ BN1 input grad)]
//             | conv1 wgrad | slab sums
//
// (reference model: /root/reference/origin_main.py:9-31.)  With SyncBN the BN
// input-grad steps run as separate launches after an all-reduce of the
// per-channel sums.  Everything stays deterministic (no float atomics).
#include "convblock_impl.h"

namespace dpa {
namespace cnf {

using cb::BNParams;
using cb::bn_finalize;
using cb::bn_relu_max4;
using cb::Pair2;
using cb::PoolIn;

constexpr int HT = 1024;       // head forward: one big workgroup per 16-row tile
constexpr int NTHR_HB = 256;   // head backward: one workgroup per BN2 channel
constexpr int NTHR_PB = 1024;  // pool1/BN1 backward: one workgroup per BN1 channel

// ---------------------------------------------------------------------------
// [BN2 finalize -> BN -> ReLU -> 2x2 max-pool -> flatten -> Linear] for 16
// batch rows per workgroup.  The pooled features of the 16 rows are staged in
// LDS as the MFMA A operand; fc weights (f32, row-major [N][K]) are read once
// per workgroup straight to registers.  NTL = ceil(N / 16) output tiles.
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W, int NTL>
__global__ void __launch_bounds__(HT)
head_fwd_kernel(const T* __restrict__ y, BNParams bn, const float* __restrict__ wfc,
                const float* __restrict__ bfc, T* __restrict__ logits, T* __restrict__ p_out,
                uint8_t* __restrict__ idx_out, int B, int N) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO, K = C * PP;
  constexpr int KPAD = ceil_to(K, 32) + 8;  // zero K-padding + 16 B row skew
  constexpr int KS = (K + 31) / 32;
  constexpr int NW = HT / 64;
  typedef MM<T> mm;
  typedef typename Pair2<T>::type P;
  __shared__ __attribute__((aligned(16))) T pimg[16 * KPAD];
  __shared__ float sc_s[C], sh_s[C];
  __shared__ float part[HT];
  __shared__ f32x4 red[NW][64];

  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * 16;
  const int rows = min(16, B - row0);
  bn_finalize<C>(bn, sc_s, sh_s, part, blockIdx.x == 0);

  // zero the K padding columns and the rows past the batch
  for (int e = tid; e < 16 * (KPAD - K); e += HT) pimg[(e / (KPAD - K)) * KPAD + K + e % (KPAD - K)] = Cvt<T>::from_f(0.f);
  // pooled features: 16 rows x K, 8 windows per thread in flight per batch
  constexpr int TOT = 16 * K;
  constexpr int U = 8;
  for (int base = 0; base < TOT; base += U * HT) {
    P top[U], bot[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * HT + tid;
      const int r = e / K, f = e % K;
      if (e < TOT && r < rows) {
        const int c = f / PP, pix = f % PP, ho = pix / WO, wo = pix % WO;
        const P* src = reinterpret_cast<const P*>(y + (((size_t)(row0 + r) * C + c) * H + 2 * ho) * W + 2 * wo);
        top[u] = src[0];
        bot[u] = src[W / 2];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * HT + tid;
      if (e >= TOT) continue;
      const int r = e / K, f = e % K;
      if (r < rows) {
        float best;
        int bi;
        bn_relu_max4<T>(top[u], bot[u], sc_s[f / PP], sh_s[f / PP], best, bi);
        const T pv = Cvt<T>::from_f(best);
        pimg[r * KPAD + f] = pv;
        if (p_out != nullptr) {
          p_out[(size_t)(row0 + r) * K + f] = pv;
          idx_out[(size_t)(row0 + r) * K + f] = (uint8_t)bi;
        }
      } else {
        pimg[r * KPAD + f] = Cvt<T>::from_f(0.f);
      }
    }
  }
  __syncthreads();

  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = wv; s < KS; s += NW) {
    const int k0 = 32 * s + 8 * q;
    const typename mm::frag a = mm::ld(&pimg[r * KPAD + k0]);
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int n = nt * 16 + r;
      typename mm::frag bf;
      if (n < N && k0 + 8 <= K) {
        const f32x4 lo = *reinterpret_cast<const f32x4*>(wfc + (size_t)n * K + k0);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(wfc + (size_t)n * K + k0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { bf[j] = mm::cv(lo[j]); bf[4 + j] = mm::cv(hi[j]); }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bf[j] = mm::cv((n < N && k0 + j < K) ? wfc[(size_t)n * K + k0 + j] : 0.f);
      }
      acc[nt] = mm::mma(a, bf, acc[nt]);
    }
  }
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    __syncthreads();
    red[wv][lane] = acc[nt];
    __syncthreads();
    if (wv == 0) {
      f32x4 t = red[0][lane];
#pragma unroll
      for (int i = 1; i < NW; ++i) t += red[i][lane];
      const int col = nt * 16 + r;
      if (col < N) {
        const float bb = bfc[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * q + i;
          if (row < rows) logits[(size_t)(row0 + row) * N + col] = Cvt<T>::from_f(t[i] + bb);
        }
      }
    }
  }
}

// mean / invstd / count of channel c from the final stats buffer.
template <int C>
__device__ __forceinline__ void mean_invstd(const float* fstats, int c, float eps, float& mean, float& invstd,
                                            float& n) {
  n = fstats[2 * C];
  const float m1 = fstats[c] / n;
  mean = fstats[2 * C + 1 + c] + m1;
  invstd = rsqrtf(fmaxf(fstats[C + c] / n - m1 * m1, 0.f) + eps);
}

// Per-channel BN backward over one pooled layer, one workgroup per channel.
// `gp(b, j)` returns the (un-routed) gradient of pooled output j of image b.
// Phase 1 routes it through ReLU (pooled value > 0) and the argmax and sums
// dy and dy*xhat; phase 2 (non-sync) writes the BN input gradient dx at full
// resolution, recomputing the routing.
template <typename T, int C, int H, int W, int THR, typename GP>
__device__ __forceinline__ void pool_bn_bwd_channel(GP&& gp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                                                    const T* __restrict__ y, const float* __restrict__ fstats,
                                                    const float* __restrict__ gamma, float eps, int B, int c,
                                                    float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                    float* __restrict__ bslab, T* __restrict__ dx, float* red) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  const int tid = threadIdx.x;
  float mean, invstd, n;
  mean_invstd<C>(fstats, c, eps, mean, invstd, n);
  float a1 = 0.f, a2 = 0.f;
  const int cnt = B * PP;
  for (int t = tid; t < cnt; t += THR) {
    const int b = t / PP, j = t % PP;
    const size_t e = ((size_t)b * C + c) * PP + j;
    if (Cvt<T>::to_f(p[e]) > 0.f) {
      const float g = gp(b, j);
      const int k = idx[e];
      const int ho = j / WO, wo = j % WO;
      const float yv = Cvt<T>::to_f(y[((size_t)b * C + c) * H * W + (2 * ho + (k >> 1)) * W + 2 * wo + (k & 1)]);
      a1 += g;
      a2 += g * (yv - mean) * invstd;
    }
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  const int lane = tid & 63, wv = tid >> 6;
  if (lane == 0) { red[wv] = a1; red[THR / 64 + wv] = a2; }
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  for (int i = 0; i < THR / 64; ++i) { s1 += red[i]; s2 += red[THR / 64 + i]; }
  if (tid == 0) {
    dbeta[c] = s1;
    dgamma[c] = s2;
    bslab[c] = s1;
    bslab[C + c] = s2;
  }
  if (dx == nullptr) return;
  const float k1 = s1 / n, k2 = s2 / n, gi = gamma[c] * invstd;
  for (int t = tid; t < cnt; t += THR) {
    const int b = t / PP, j = t % PP;
    const size_t e = ((size_t)b * C + c) * PP + j;
    const float g = Cvt<T>::to_f(p[e]) > 0.f ? gp(b, j) : 0.f;
    const int kk = idx[e];
    const int ho = j / WO, wo = j % WO;
    const size_t base = ((size_t)b * C + c) * H * W + (2 * ho) * W + 2 * wo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t o = base + (k >> 1) * W + (k & 1);
      const float xh = (Cvt<T>::to_f(y[o]) - mean) * invstd;
      dx[o] = Cvt<T>::from_f(gi * (((k == kk) ? g : 0.f) - k1 - xh * k2));
    }
  }
}

// ---------------------------------------------------------------------------
// fc backward + pool2/ReLU2 routing + BN2 reduce (+ BN2 input grad), one
// workgroup per BN2 channel c (its PP = 7*7 pooled features).
//   dW_fc[:, cPP..] = dlogits^T . p2[:, cPP..]     (complete: all batch rows)
//   dp2[b, cPP + j] = sum_n dlogits[b, n] W[n, cPP + j]
// dynamic LDS: dlogits [B][N] f32 + W columns [N][PP] f32 + p2 slice [B][PP] f32.
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR_HB)
head_bwd_kernel(const T* __restrict__ dlogits, const float* __restrict__ wfc, const T* __restrict__ p2,
                const uint8_t* __restrict__ idx2, const T* __restrict__ y2, const float* __restrict__ fstats2,
                const float* __restrict__ gamma2, float eps, int B, int N, float* __restrict__ dwfc,
                float* __restrict__ dbfc, float* __restrict__ dgamma, float* __restrict__ dbeta,
                float* __restrict__ bslab, T* __restrict__ dp2_out, T* __restrict__ dy2) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO, K = C * PP;
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  __shared__ float red[2 * NTHR_HB / 64];
  float* dl = hsm;               // [B][N]
  float* wc = dl + B * N;        // [N][PP]
  float* pc = wc + N * PP;       // [B][PP]
  const int tid = threadIdx.x, c = blockIdx.x, f0 = c * PP;
  for (int e = tid; e < B * N; e += NTHR_HB) dl[e] = Cvt<T>::to_f(dlogits[e]);
  for (int e = tid; e < N * PP; e += NTHR_HB) wc[e] = wfc[(size_t)(e / PP) * K + f0 + e % PP];
  for (int e = tid; e < B * PP; e += NTHR_HB) pc[e] = Cvt<T>::to_f(p2[(size_t)(e / PP) * K + f0 + e % PP]);
  __syncthreads();
  // fc weight grad for this channel's columns, fc bias grad on workgroup 0
  for (int e = tid; e < N * PP; e += NTHR_HB) {
    const int nn = e / PP, j = e % PP;
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += dl[b * N + nn] * pc[b * PP + j];
    dwfc[(size_t)nn * K + f0 + j] = a;
  }
  if (c == 0) {
    for (int nn = tid; nn < N; nn += NTHR_HB) {
      float a = 0.f;
      for (int b = 0; b < B; ++b) a += dl[b * N + nn];
      dbfc[nn] = a;
    }
  }
  auto gp = [&](int b, int j) {
    float a = 0.f;
    for (int nn = 0; nn < N; ++nn) a += dl[b * N + nn] * wc[nn * PP + j];
    return Cvt<T>::to_f(Cvt<T>::from_f(a));  // the pooled-map grad as stored in T (autocast semantics)
  };
  if (dp2_out != nullptr) {  // SyncBN path: materialise dp2 for the separate BN input-grad launch
    for (int e = tid; e < B * PP; e += NTHR_HB)
      dp2_out[(size_t)(e / PP) * K + f0 + e % PP] = Cvt<T>::from_f(gp(e / PP, e % PP));
  }
  pool_bn_bwd_channel<T, C, H, W, NTHR_HB>(gp, p2, idx2, y2, fstats2, gamma2, eps, B, c, dgamma, dbeta, bslab, dy2,
                                           red);
}

// pool1/ReLU1 routing + BN1 reduce (+ BN1 input grad), one workgroup per channel.
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR_PB)
pool_bn_bwd_kernel(const T* __restrict__ dp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                   const T* __restrict__ y, const float* __restrict__ fstats, const float* __restrict__ gamma,
                   float eps, int B, float* __restrict__ dgamma, float* __restrict__ dbeta,
                   float* __restrict__ bslab, T* __restrict__ dx) {
  constexpr int PP = (H / 2) * (W / 2);
  __shared__ float red[2 * NTHR_PB / 64];
  const int c = blockIdx.x;
  auto gp = [&](int b, int j) { return Cvt<T>::to_f(dp[((size_t)b * C + c) * PP + j]); };
  pool_bn_bwd_channel<T, C, H, W, NTHR_PB>(gp, p, idx, y, fstats, gamma, eps, B, c, dgamma, dbeta, bslab, dx, red);
}


// ===========================================================================
// Host side
// ===========================================================================
template <typename F>
static void with_t(DT dt, F&& f) {
  switch (dt) {
    case DT::F32: f(float{}); break;
    case DT::BF16: f(__hip_bfloat16{}); break;
    case DT::F16: f(__half{}); break;
  }
}

static BNParams bn_params(c10::optional<at::Tensor> fslab, at::Tensor fstats, at::Tensor gamma, at::Tensor beta,
                          at::Tensor rmean, at::Tensor rvar, at::Tensor nbt, double momentum, double eps, bool train,
                          int C) {
  TORCH_CHECK(!train || fslab.has_value(), "train mode needs the forward slab");
  BNParams bp;
  bp.fslab = fslab.has_value() ? fslab->data_ptr<float>() : nullptr;
  bp.nrows = fslab.has_value() ? (int)(fslab->numel() / cb::fslab_row(C)) : 0;
  bp.fstats = fstats.data_ptr<float>();
  bp.gamma = gamma.data_ptr<float>();
  bp.beta = beta.data_ptr<float>();
  bp.rmean = rmean.data_ptr<float>();
  bp.rvar = rvar.data_ptr<float>();
  bp.nbt = nbt.data_ptr<int64_t>();
  bp.momentum = (float)momentum;
  bp.eps = (float)eps;
  bp.train = (int)train;
  return bp;
}

// [BN1 -> ReLU -> pool1] -> conv2 (+ BN2 partial sums when training).
void conv2_fwd(at::Tensor y1, c10::optional<at::Tensor> fslab1, at::Tensor fstats1, at::Tensor g1, at::Tensor b1,
               at::Tensor rm1, at::Tensor rv1, at::Tensor nbt1, double momentum, double eps, bool train, at::Tensor w2,
               at::Tensor bias2, at::Tensor y2, c10::optional<at::Tensor> fslab2, at::Tensor fstats2, at::Tensor rm2,
               c10::optional<at::Tensor> p1_out, c10::optional<at::Tensor> idx1_out) {
  DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(w2); DPA_CHECK_INPUT(y2);
  const int B = (int)y1.size(0);
  TORCH_CHECK(y1.size(1) == 16 && y1.size(2) == 28 && y1.size(3) == 28 && w2.size(0) == 32 && w2.size(1) == 16,
              "fused conv2 expects the ConvNet shapes");
  TORCH_CHECK(y2.scalar_type() == y1.scalar_type());
  if (train) TORCH_CHECK(fslab2.has_value() && fslab2->numel() == (int64_t)B * 2 * cb::fslab_row(32));
  if (B == 0) return;
  const BNParams bp = bn_params(fslab1, fstats1, g1, b1, rm1, rv1, nbt1, momentum, eps, train, 16);
  constexpr int ns = 2;
  hipStream_t stream = cur_stream();
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    cb::PoolIn<T> pin{dptr<T>(y1), bp, p1_out.has_value() ? dptr<T>(*p1_out) : nullptr,
                      idx1_out.has_value() ? idx1_out->data_ptr<uint8_t>() : nullptr};
    if (train)
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 16, 32, 14, 14, 0, 1>), dim3(B * ns), dim3(cb::NTHR), 0, stream,
                         nullptr, w2.data_ptr<float>(), bias2.data_ptr<float>(), dptr<T>(y2),
                         fslab2->data_ptr<float>(), fstats2.data_ptr<float>(), rm2.data_ptr<float>(), ns, pin);
    else
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 16, 32, 14, 14, 1, 1>), dim3(B * ns), dim3(cb::NTHR), 0, stream,
                         nullptr, w2.data_ptr<float>(), bias2.data_ptr<float>(), dptr<T>(y2), nullptr, nullptr,
                         nullptr, ns, pin);
  });
  DPA_CHECK_LAUNCH();
}

// [BN2 -> ReLU -> pool2] -> flatten -> fc.
void head_fwd(at::Tensor y2, c10::optional<at::Tensor> fslab2, at::Tensor fstats2, at::Tensor g2, at::Tensor b2,
              at::Tensor rm2, at::Tensor rv2, at::Tensor nbt2, double momentum, double eps, bool train, at::Tensor wfc,
              at::Tensor bfc, at::Tensor logits, c10::optional<at::Tensor> p2_out, c10::optional<at::Tensor> idx2_out) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(wfc); DPA_CHECK_INPUT(logits);
  const int B = (int)y2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(y2.size(1) == 32 && y2.size(2) == 14 && y2.size(3) == 14 && wfc.size(1) == 32 * 49,
              "fused head expects the ConvNet shapes");
  TORCH_CHECK(N >= 1 && N <= 64, "fused head supports up to 64 classes");
  if (B == 0) return;
  const BNParams bp = bn_params(fslab2, fstats2, g2, b2, rm2, rv2, nbt2, momentum, eps, train, 32);
  const dim3 grid((B + 15) / 16);
  hipStream_t stream = cur_stream();
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    T* po = p2_out.has_value() ? dptr<T>(*p2_out) : nullptr;
    uint8_t* io = idx2_out.has_value() ? idx2_out->data_ptr<uint8_t>() : nullptr;
    auto go = [&](auto ntl) {
      hipLaunchKernelGGL((head_fwd_kernel<T, 32, 14, 14, decltype(ntl)::value>), grid, dim3(HT), 0, stream,
                         dptr<T>(y2), bp, wfc.data_ptr<float>(), bfc.data_ptr<float>(), dptr<T>(logits), po, io, B, N);
    };
    if (N <= 16) go(std::integral_constant<int, 1>{});
    else if (N <= 32) go(std::integral_constant<int, 2>{});
    else go(std::integral_constant<int, 4>{});
  });
  DPA_CHECK_LAUNCH();
}

// fc backward + pool2/ReLU2 routing + BN2 reduce (+ BN2 input grad when dy2 given).
void head_bwd(at::Tensor dlogits, at::Tensor wfc, at::Tensor p2, at::Tensor idx2, at::Tensor y2, at::Tensor fstats2,
              at::Tensor g2, double eps, at::Tensor dwfc, at::Tensor dbfc, at::Tensor dgamma2, at::Tensor dbeta2,
              at::Tensor bslab2, c10::optional<at::Tensor> dp2_out, c10::optional<at::Tensor> dy2) {
  DPA_CHECK_INPUT(dlogits); DPA_CHECK_INPUT(p2); DPA_CHECK_INPUT(y2);
  const int B = (int)y2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(dlogits.scalar_type() == y2.scalar_type() && p2.scalar_type() == y2.scalar_type());
  const size_t lds = sizeof(float) * ((size_t)B * N + (size_t)N * 49 + (size_t)B * 49);
  TORCH_CHECK(lds <= 64 * 1024, "fused head backward: batch too large for LDS (B*N)");
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((head_bwd_kernel<T, 32, 14, 14>), dim3(32), dim3(NTHR_HB), lds, cur_stream(),
                       dptr<T>(dlogits), wfc.data_ptr<float>(), dptr<T>(p2), idx2.data_ptr<uint8_t>(), dptr<T>(y2),
                       fstats2.data_ptr<float>(), g2.data_ptr<float>(), (float)eps, B, N, dwfc.data_ptr<float>(),
                       dbfc.data_ptr<float>(), dgamma2.data_ptr<float>(), dbeta2.data_ptr<float>(),
                       bslab2.data_ptr<float>(), dp2_out.has_value() ? dptr<T>(*dp2_out) : nullptr,
                       dy2.has_value() ? dptr<T>(*dy2) : nullptr);
  });
  DPA_CHECK_LAUNCH();
}

// pool1/ReLU1 routing + BN1 reduce (+ BN1 input grad when dy1 given).
void pool1_bwd(at::Tensor dp1, at::Tensor p1, at::Tensor idx1, at::Tensor y1, at::Tensor fstats1, at::Tensor g1,
               double eps, at::Tensor dgamma1, at::Tensor dbeta1, at::Tensor bslab1, c10::optional<at::Tensor> dy1) {
  DPA_CHECK_INPUT(dp1); DPA_CHECK_INPUT(p1); DPA_CHECK_INPUT(y1);
  const int B = (int)y1.size(0);
  TORCH_CHECK(y1.size(1) == 16 && y1.size(2) == 28 && y1.size(3) == 28);
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((pool_bn_bwd_kernel<T, 16, 28, 28>), dim3(16), dim3(NTHR_PB), 0, cur_stream(), dptr<T>(dp1),
                       dptr<T>(p1), idx1.data_ptr<uint8_t>(), dptr<T>(y1), fstats1.data_ptr<float>(),
                       g1.data_ptr<float>(), (float)eps, B, dgamma1.data_ptr<float>(), dbeta1.data_ptr<float>(),
                       bslab1.data_ptr<float>(), dy1.has_value() ? dptr<T>(*dy1) : nullptr);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace cnf

void register_convnet_fused(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("convnet", "whole-ConvNet fused kernels");
  s.def("conv2_fwd", &cnf::conv2_fwd);
  s.def("head_fwd", &cnf::head_fwd);
  s.def("head_bwd", &cnf::head_bwd);
  s.def("pool1_bwd", &cnf::pool1_bwd);
}

}  // namespace dpa
