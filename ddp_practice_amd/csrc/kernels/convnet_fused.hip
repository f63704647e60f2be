// Whole-ConvNet fused kernels (ops/convnet_fused.py).  Layer boundaries are
// fused where the data dependence allows it; every BatchNorm reduction is
// produced as per-workgroup partial sums in the epilogue of the kernel that
// computes its operand and reduced in the prologue of the kernel that needs
// the result, so no launch exists only to reduce or to apply a BatchNorm:
//
//   forward   gather | conv1 (+BN1 sums) | [BN1-ReLU-pool1 -> conv2 (+BN2 sums)]
//             | [BN2-ReLU-pool2 -> fc] -> logits                          (3 launches)
//   backward  [fc bwd -> dp2 (+BN2 sums: complete per channel)]
//             | [BN2/ReLU2/pool2 bwd -> conv2 dgrad -> dp1 (+BN1 partial sums)]
//             | [BN2/ReLU2/pool2 bwd -> conv2 wgrad]        (independent of dgrad)
//             | [BN1/ReLU1/pool1 bwd -> conv1 wgrad]
//             | weight-grad sums                                        (5 launches)
//
// (reference model: /root/reference/origin_main.py:9-31.)  With SyncBN the
// partial sums are all-reduced between the launches (host side).  Everything
// is deterministic (no float atomics).
#include <type_traits>

#include "convblock_impl.h"
#include "comm/xgmi.h"
#include "kernels/amp_step.h"

namespace dpa {
namespace cnf {

using cb::BNParams;
using cb::bn_finalize;
using cb::bn_relu_max4x;
using cb::BwdEpi;
using cb::BwdIn;
using cb::IDX_POS;
using cb::IDX_RELU;
using cb::Pair2;
using cb::PoolIn;

constexpr int HF = 256;        // head forward: one workgroup per image
constexpr int NTHR_HB = 256;   // head backward: one workgroup per BN2 channel

// ---------------------------------------------------------------------------
// [BN2 finalize -> BN -> ReLU -> 2x2 max-pool -> flatten -> Linear] for one
// image per workgroup (B workgroups: the whole chip works on the head instead
// of B/16 tiles).  The fc is a 1 x K x N GEMV per image: every thread owns K/HF
// pooled features, multiplies them against the fc rows and the N partial dot
// products are reduced across the workgroup.  The y2 loads are issued before
// the BN statistics reduction so the two latencies overlap.
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W, int NMAX>
__global__ void __launch_bounds__(HF)
head_fwd_kernel(const T* __restrict__ y, BNParams bn, const float* __restrict__ wfc, const float* __restrict__ bfc,
                T* __restrict__ logits, T* __restrict__ p_out, uint8_t* __restrict__ idx_out, T* __restrict__ xh_out,
                int N) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO, K = C * PP;
  constexpr int IT = (K + HF - 1) / HF;
  typedef typename Pair2<T>::type P;
  __shared__ float sc_s[C], beta_s[C], mean_s[C], istd_s[C];
  __shared__ float part[HF];
  __shared__ float red[HF / 64][NMAX];
  const int tid = threadIdx.x, b = blockIdx.x;
  const T* yb = y + (size_t)b * C * H * W;
  P top[IT], bot[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = tid + i * HF;
    if (k < K) {
      const int c = k / PP, pix = k % PP, ho = pix / WO, wo = pix % WO;
      const P* src = reinterpret_cast<const P*>(yb + ((size_t)c * H + 2 * ho) * W + 2 * wo);
      top[i] = src[0];
      bot[i] = src[W / 2];
    }
  }
  bn_finalize<C>(bn, sc_s, beta_s, mean_s, istd_s, part, b);
  float pf[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = tid + i * HF;
    pf[i] = 0.f;
    if (k < K) {
      const int c = k / PP;
      float best, xh;
      int bi;
      bn_relu_max4x<T>(top[i], bot[i], sc_s[c], beta_s[c], mean_s[c], istd_s[c], best, bi, xh);
      const T pv = Cvt<T>::from_f(best);
      pf[i] = Cvt<T>::to_f(pv);
      if (p_out != nullptr) {
        p_out[(size_t)b * K + k] = pv;
        idx_out[(size_t)b * K + k] = (uint8_t)(bi | (best > 0.f ? IDX_RELU : 0));
        xh_out[(size_t)b * K + k] = Cvt<T>::from_f(xh);
      }
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
  // fc rows in chunks of NC outputs: every load of a chunk is issued before
  // its first FMA (rows past N are clamped to N-1 and discarded)
  constexpr int NC = 8;
  for (int n0 = 0; n0 < N; n0 += NC) {  // uniform
    float wr[NC][IT];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int n = min(n0 + j, N - 1);
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int k = min(tid + i * HF, K - 1);
        wr[j][i] = wfc[(size_t)n * K + k];
      }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < IT; ++i) a += pf[i] * wr[j][i];  // pf = 0 past K
      a = wave_sum(a);
      if (lane == 0 && n0 + j < N) red[wv][n0 + j] = a;
    }
  }
  __syncthreads();
  if (tid < N) {
    float t = bfc[tid];
#pragma unroll
    for (int i = 0; i < HF / 64; ++i) t += red[i][tid];
    logits[(size_t)b * N + tid] = Cvt<T>::from_f(t);
  }
}

// ---------------------------------------------------------------------------
// fc backward + the BN2 backward sums, one workgroup per BN2 channel c (its
// PP = 7*7 pooled features; the sums are complete, no partial rows):
//   dp2[b, cPP + j]   = sum_n dlogits[b, n] W[n, cPP + j]          (stored in T)
//   dW_fc[n, cPP + j] = sum_b dlogits[b, n] p2[b, cPP + j]
//   S1[c] = sum g, S2[c] = sum g * xhat, g = dp2 where the ReLU passed it
// dynamic LDS: dlogits [B][N] + W columns [N][PP] + p2 slice [B][PP] (f32).
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR_HB)
head_bwd_kernel(const T* __restrict__ dlogits, const float* __restrict__ wfc, const T* __restrict__ p2,
                const uint8_t* __restrict__ idx2, const T* __restrict__ xh2, int B, int N, float* __restrict__ dwfc,
                float* __restrict__ dbfc, float* __restrict__ dgamma, float* __restrict__ dbeta,
                float* __restrict__ bsum, T* __restrict__ dp2) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO, K = C * PP;
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  __shared__ float red[2][NTHR_HB / 64];
  float* dl = hsm;               // [B][N]
  float* wc = dl + B * N;        // [N][PP]
  float* pc = wc + N * PP;       // [B][PP]
  const int tid = threadIdx.x, c = blockIdx.x, f0 = c * PP;
  for (int e = tid; e < B * N; e += NTHR_HB) dl[e] = Cvt<T>::to_f(dlogits[e]);
  for (int e = tid; e < N * PP; e += NTHR_HB) wc[e] = wfc[(size_t)(e / PP) * K + f0 + e % PP];
  for (int e = tid; e < B * PP; e += NTHR_HB) pc[e] = Cvt<T>::to_f(p2[(size_t)(e / PP) * K + f0 + e % PP]);
  __syncthreads();
  // pooled-map grad + BN2 sums
  float s1 = 0.f, s2 = 0.f;
  for (int e = tid; e < B * PP; e += NTHR_HB) {
    const int b = e / PP, j = e % PP;
    const size_t o = (size_t)b * K + f0 + j;
    const uint8_t ix = idx2[o];
    const float xh = Cvt<T>::to_f(xh2[o]);
    float a = 0.f;
    for (int nn = 0; nn < N; ++nn) a += dl[b * N + nn] * wc[nn * PP + j];
    const T gt = Cvt<T>::from_f(a);
    dp2[o] = gt;
    if (ix & IDX_RELU) {
      const float g = Cvt<T>::to_f(gt);
      s1 += g;
      s2 += g * xh;
    }
  }
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
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const int lane = tid & 63, wv = tid >> 6;
  if (lane == 0) { red[0][wv] = s1; red[1][wv] = s2; }
  __syncthreads();
  if (tid == 0) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int i = 0; i < NTHR_HB / 64; ++i) { t1 += red[0][i]; t2 += red[1][i]; }
    dbeta[c] = t1;
    dgamma[c] = t2;
    bsum[c] = t1;
    bsum[C + c] = t2;
  }
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

template <typename T>
static BwdIn<T> bwd_in(at::Tensor dp, at::Tensor idx, at::Tensor y, at::Tensor fstats, at::Tensor gsum,
                       c10::optional<at::Tensor> lsum, at::Tensor gamma, double eps, int C,
                       c10::optional<at::Tensor> dgamma, c10::optional<at::Tensor> dbeta) {
  TORCH_CHECK(gsum.numel() % (2 * C) == 0, "BN backward sums: rows of 2C floats expected");
  TORCH_CHECK(dp.scalar_type() == y.scalar_type() && idx.scalar_type() == at::kByte);
  TORCH_CHECK(fstats.numel() == cb::stats_len(C) && gamma.numel() == C);
  BwdIn<T> bi;
  bi.dp = dptr<T>(dp);
  bi.idx = idx.data_ptr<uint8_t>();
  bi.y = dptr<T>(y);
  bi.fstats = fstats.data_ptr<float>();
  bi.gsum = gsum.data_ptr<float>();
  bi.grows = (int)(gsum.numel() / (2 * C));
  at::Tensor ls = lsum.has_value() ? *lsum : gsum;
  TORCH_CHECK(ls.numel() % (2 * C) == 0);
  bi.lsum = ls.data_ptr<float>();
  bi.lrows = (int)(ls.numel() / (2 * C));
  bi.gamma = gamma.data_ptr<float>();
  bi.eps = (float)eps;
  bi.dgamma = dgamma.has_value() ? dgamma->data_ptr<float>() : nullptr;
  bi.dbeta = dbeta.has_value() ? dbeta->data_ptr<float>() : nullptr;
  return bi;
}

// xc (SyncBN over the xGMI engine, training only): the consumer kernel
// exchanges the BN sums itself (comm/xsite.h); the slab arguments then hold
// this rank's partial sums and no all-reduce runs between the launches.
typedef std::shared_ptr<xgmi::XgmiComm> XcPtr;
static xgmi::XSite site_of(const XcPtr& xc, int s) { return xc ? xc->site(s) : xgmi::XSite{}; }

// Workgroups per image of the conv2 forward.  bf16 / fp16: cb::SH<1>::SPLIT (2); fp32, whose
// 16x16x4 MFMA chain per output tile is 4x as long, runs 4 shorter workgroups per image: fp32
// step 0.0640 -> 0.0617 ms, while bf16 at 4 is 0.6 us slower (profiles/r6m_split_ab.txt).
// The consumers take the slab's row count from its size (nrows).
#ifndef DPA_FWD2_SPLIT_F32
#define DPA_FWD2_SPLIT_F32 4
#endif
int64_t fwd2_split(bool fp32) { return fp32 ? DPA_FWD2_SPLIT_F32 : cb::SH<1>::SPLIT; }

// [BN1 -> ReLU -> pool1] -> conv2 (+ BN2 partial sums when training).
void conv2_fwd(at::Tensor y1, c10::optional<at::Tensor> fslab1, at::Tensor fstats1, at::Tensor g1, at::Tensor b1,
               at::Tensor rm1, at::Tensor rv1, at::Tensor nbt1, double momentum, double eps, bool train, at::Tensor w2,
               at::Tensor bias2, at::Tensor y2, c10::optional<at::Tensor> fslab2, at::Tensor fstats2, at::Tensor rm2,
               c10::optional<at::Tensor> p1_out, c10::optional<at::Tensor> idx1_out,
               c10::optional<at::Tensor> xh1_out, at::Tensor wpk, XcPtr xc) {
  DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(w2); DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(wpk);
  TORCH_CHECK(wpk.numel() == cb::W2F_LEN && wpk.scalar_type() == y1.scalar_type(), "packed conv2 weights");
  const int B = (int)y1.size(0);
  TORCH_CHECK(y1.size(1) == 16 && y1.size(2) == 28 && y1.size(3) == 28 && w2.size(0) == 32 && w2.size(1) == 16,
              "fused conv2 expects the ConvNet shapes");
  TORCH_CHECK(y2.scalar_type() == y1.scalar_type());
  TORCH_CHECK(p1_out.has_value() == idx1_out.has_value() && p1_out.has_value() == xh1_out.has_value());
  if (p1_out.has_value())
    TORCH_CHECK(p1_out->numel() == (int64_t)B * 16 * 196 && idx1_out->numel() == p1_out->numel() &&
                xh1_out->numel() == p1_out->numel());
  const int ns = fwd2_split(y1.scalar_type() == at::kFloat);  // workgroups per image
  if (train) TORCH_CHECK(fslab2.has_value() && fslab2->numel() == (int64_t)B * ns * cb::fslab_row(32));
  if (B == 0) return;
  BNParams bp = bn_params(fslab1, fstats1, g1, b1, rm1, rv1, nbt1, momentum, eps, train, 16);
  if (train) {
    bp.xs = site_of(xc, xgmi::kSiteFwd1);
    xgmi::set_site_grid(bp.xs, B * ns, "conv2_fwd");  // the grid (ns workgroups per image)
  }
  hipStream_t stream = cur_stream();
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    PoolIn<T> pin{dptr<T>(y1), bp, p1_out.has_value() ? dptr<T>(*p1_out) : nullptr,
                  idx1_out.has_value() ? idx1_out->data_ptr<uint8_t>() : nullptr,
                  xh1_out.has_value() ? dptr<T>(*xh1_out) : nullptr};
    if (train)
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 16, 32, 14, 14, 0, 1, 0, 1>), dim3(B * ns), dim3(cb::NTHR), 0,
                         stream, nullptr, nullptr, bias2.data_ptr<float>(), dptr<T>(y2), fslab2->data_ptr<float>(),
                         fstats2.data_ptr<float>(), rm2.data_ptr<float>(), ns, pin, BwdIn<T>{}, BwdEpi<T>{},
                         dptr<T>(wpk), cb::WPack<T>{});
    else
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 16, 32, 14, 14, 1, 1, 0, 1>), dim3(B * ns), dim3(cb::NTHR), 0,
                         stream, nullptr, nullptr, bias2.data_ptr<float>(), dptr<T>(y2), nullptr, nullptr, nullptr,
                         ns, pin, BwdIn<T>{}, BwdEpi<T>{}, dptr<T>(wpk), cb::WPack<T>{});
  });
  DPA_CHECK_LAUNCH();
}

// [BN2 -> ReLU -> pool2] -> flatten -> fc.
void head_fwd(at::Tensor y2, c10::optional<at::Tensor> fslab2, at::Tensor fstats2, at::Tensor g2, at::Tensor b2,
              at::Tensor rm2, at::Tensor rv2, at::Tensor nbt2, double momentum, double eps, bool train, at::Tensor wfc,
              at::Tensor bfc, at::Tensor logits, c10::optional<at::Tensor> p2_out, c10::optional<at::Tensor> idx2_out,
              c10::optional<at::Tensor> xh2_out, XcPtr xc) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(wfc); DPA_CHECK_INPUT(logits);
  const int B = (int)y2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(y2.size(1) == 32 && y2.size(2) == 14 && y2.size(3) == 14 && wfc.size(1) == 32 * 49,
              "fused head expects the ConvNet shapes");
  TORCH_CHECK(N >= 1 && N <= 64, "fused head supports up to 64 classes");
  TORCH_CHECK(logits.numel() == (int64_t)B * N && logits.scalar_type() == y2.scalar_type());
  TORCH_CHECK(p2_out.has_value() == idx2_out.has_value() && p2_out.has_value() == xh2_out.has_value());
  if (p2_out.has_value())
    TORCH_CHECK(p2_out->numel() == (int64_t)B * 1568 && idx2_out->numel() == p2_out->numel() &&
                xh2_out->numel() == p2_out->numel());
  if (B == 0) return;
  BNParams bp = bn_params(fslab2, fstats2, g2, b2, rm2, rv2, nbt2, momentum, eps, train, 32);
  if (train) {
    bp.xs = site_of(xc, xgmi::kSiteFwd2);
    xgmi::set_site_grid(bp.xs, B, "head_fwd");  // one workgroup per image
    bp.xs.nblk = 0;                             // (the kernel reads the grid)
  }
  hipStream_t stream = cur_stream();
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    T* po = p2_out.has_value() ? dptr<T>(*p2_out) : nullptr;
    uint8_t* io = idx2_out.has_value() ? idx2_out->data_ptr<uint8_t>() : nullptr;
    T* xo = xh2_out.has_value() ? dptr<T>(*xh2_out) : nullptr;
    auto go = [&](auto nmax) {
      hipLaunchKernelGGL((head_fwd_kernel<T, 32, 14, 14, decltype(nmax)::value>), dim3(B), dim3(HF), 0, stream,
                         dptr<T>(y2), bp, wfc.data_ptr<float>(), bfc.data_ptr<float>(), dptr<T>(logits), po, io, xo,
                         N);
    };
    if (N <= 16) go(std::integral_constant<int, 16>{});
    else go(std::integral_constant<int, 64>{});
  });
  DPA_CHECK_LAUNCH();
}

size_t head_bwd_lds(int64_t B, int64_t N) { return sizeof(float) * (size_t)(B * N + N * 49 + B * 49); }

// fc backward + BN2 backward sums (local, complete per channel).
void head_bwd(at::Tensor dlogits, at::Tensor wfc, at::Tensor p2, at::Tensor idx2, at::Tensor xh2, at::Tensor dwfc,
              at::Tensor dbfc, at::Tensor dgamma2, at::Tensor dbeta2, at::Tensor bsum2, at::Tensor dp2) {
  DPA_CHECK_INPUT(dlogits); DPA_CHECK_INPUT(p2); DPA_CHECK_INPUT(dp2);
  const int B = (int)p2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(p2.numel() == (int64_t)B * 1568 && dp2.numel() == p2.numel() && xh2.numel() == p2.numel());
  TORCH_CHECK(dlogits.numel() == (int64_t)B * N);
  TORCH_CHECK(dlogits.scalar_type() == p2.scalar_type() && dp2.scalar_type() == p2.scalar_type());
  TORCH_CHECK(bsum2.numel() == 64 && dwfc.numel() == wfc.numel() && dbfc.numel() == N);
  const size_t lds = head_bwd_lds(B, N);
  TORCH_CHECK(lds <= 64 * 1024, "fused head backward: batch too large for LDS (B*N)");
  if (B == 0) return;
  with_t(dt_of(p2), [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((head_bwd_kernel<T, 32, 14, 14>), dim3(32), dim3(NTHR_HB), lds, cur_stream(),
                       dptr<T>(dlogits), wfc.data_ptr<float>(), dptr<T>(p2), idx2.data_ptr<uint8_t>(), dptr<T>(xh2), B,
                       N, dwfc.data_ptr<float>(), dbfc.data_ptr<float>(), dgamma2.data_ptr<float>(),
                       dbeta2.data_ptr<float>(), bsum2.data_ptr<float>(), dptr<T>(dp2));
  });
  DPA_CHECK_LAUNCH();
}

// Layer-1 conv (+BN1 sums when training) that also packs the layer-2 weights
// into their low-precision LDS tile layouts (cb::pack_w2).
void conv1_fwd_pack(at::Tensor x, at::Tensor w1, at::Tensor b1, at::Tensor y1, c10::optional<at::Tensor> fslab1,
                    c10::optional<at::Tensor> fstats1, c10::optional<at::Tensor> shift1, at::Tensor w2,
                    at::Tensor wpk_f, at::Tensor wpk_d) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w1); DPA_CHECK_INPUT(b1); DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(w2);
  DPA_CHECK_INPUT(wpk_f); DPA_CHECK_INPUT(wpk_d);
  const int B = (int)x.size(0);
  typedef cb::SH<0> S;
  TORCH_CHECK(x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28 && w1.numel() == 16 * 25 && b1.numel() == 16,
              "fused conv1 expects the ConvNet shapes");
  TORCH_CHECK(w2.numel() == 32 * 16 * 25 && w2.scalar_type() == at::kFloat && w1.scalar_type() == at::kFloat);
  TORCH_CHECK(y1.numel() == (int64_t)B * 16 * 784 && y1.scalar_type() == x.scalar_type());
  TORCH_CHECK(wpk_f.numel() == cb::W2F_LEN && wpk_d.numel() == cb::W2D_LEN &&
              wpk_f.scalar_type() == x.scalar_type() && wpk_d.scalar_type() == x.scalar_type());
  const bool st = fslab1.has_value();
  if (st)
    TORCH_CHECK(fslab1->numel() == (int64_t)B * S::SPLIT * cb::fslab_row(16) && fstats1->numel() == cb::stats_len(16) &&
                shift1->numel() == 16);
  if (B == 0) return;
  with_t(dt_of(x), [&](auto tag) {
    typedef decltype(tag) T;
    cb::WPack<T> pk{w2.data_ptr<float>(), dptr<T>(wpk_f), dptr<T>(wpk_d)};
    if (st)
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 1, 16, 28, 28, 0, 0, 0, 2>), dim3(B * S::SPLIT), dim3(cb::NTHR), 0,
                         cur_stream(), dptr<T>(x), w1.data_ptr<float>(), b1.data_ptr<float>(), dptr<T>(y1),
                         fslab1->data_ptr<float>(), fstats1->data_ptr<float>(), shift1->data_ptr<float>(), S::SPLIT,
                         PoolIn<T>{}, BwdIn<T>{}, BwdEpi<T>{}, nullptr, pk);
    else
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 1, 16, 28, 28, 1, 0, 0, 2>), dim3(B * S::SPLIT), dim3(cb::NTHR), 0,
                         cur_stream(), dptr<T>(x), w1.data_ptr<float>(), b1.data_ptr<float>(), dptr<T>(y1), nullptr,
                         nullptr, nullptr, S::SPLIT, PoolIn<T>{}, BwdIn<T>{}, BwdEpi<T>{}, nullptr, pk);
  });
  DPA_CHECK_LAUNCH();
}

// conv1_fwd_pack with the batch gather fused in (training; cb::GatherIn): x and lab_out
// are the loader's batch buffers, filled by this launch from the HBM-resident dataset
// at the device step counter, which the launch then advances (data.hip protocol).
void conv1_fwd_pack_gather(at::Tensor x, at::Tensor w1, at::Tensor b1, at::Tensor y1, at::Tensor fslab1,
                           at::Tensor fstats1, at::Tensor shift1, at::Tensor w2, at::Tensor wpk_f, at::Tensor wpk_d,
                           at::Tensor imgs, at::Tensor labels, at::Tensor order, at::Tensor ctr, at::Tensor lab_out,
                           double scale, double shift) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w1); DPA_CHECK_INPUT(b1); DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(w2);
  DPA_CHECK_INPUT(wpk_f); DPA_CHECK_INPUT(wpk_d); DPA_CHECK_INPUT(imgs); DPA_CHECK_INPUT(labels);
  DPA_CHECK_INPUT(order); DPA_CHECK_INPUT(ctr); DPA_CHECK_INPUT(lab_out);
  const int B = (int)x.size(0);
  typedef cb::SH<0> S;
  TORCH_CHECK(x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28 && w1.numel() == 16 * 25 && b1.numel() == 16,
              "fused conv1 expects the ConvNet shapes");
  TORCH_CHECK(imgs.scalar_type() == at::kByte && imgs.dim() == 3 && imgs.size(1) == 28 && imgs.size(2) == 28,
              "gather: uint8 [N][28][28] dataset");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == imgs.size(0));
  TORCH_CHECK(order.scalar_type() == at::kLong && ctr.scalar_type() == at::kInt && ctr.numel() >= 2);
  TORCH_CHECK(lab_out.scalar_type() == at::kLong && lab_out.numel() == B);
  TORCH_CHECK(w2.numel() == 32 * 16 * 25 && w2.scalar_type() == at::kFloat && w1.scalar_type() == at::kFloat);
  TORCH_CHECK(y1.numel() == (int64_t)B * 16 * 784 && y1.scalar_type() == x.scalar_type());
  TORCH_CHECK(wpk_f.numel() == cb::W2F_LEN && wpk_d.numel() == cb::W2D_LEN &&
              wpk_f.scalar_type() == x.scalar_type() && wpk_d.scalar_type() == x.scalar_type());
  TORCH_CHECK(fslab1.numel() == (int64_t)B * S::SPLIT * cb::fslab_row(16) && fstats1.numel() == cb::stats_len(16) &&
              shift1.numel() == 16);
  if (B == 0) return;
  cb::GatherIn gin;
  gin.imgs = imgs.data_ptr<uint8_t>();
  gin.labels = labels.data_ptr<int64_t>();
  gin.order = order.data_ptr<int64_t>();
  gin.order_len = order.numel();
  gin.ctr = ctr.data_ptr<int>();
  gin.lab_out = lab_out.data_ptr<int64_t>();
  gin.scale = (float)scale;
  gin.shift = (float)shift;
  gin.nimg = (int)B;
  with_t(dt_of(x), [&](auto tag) {
    typedef decltype(tag) T;
    cb::WPack<T> pk{w2.data_ptr<float>(), dptr<T>(wpk_f), dptr<T>(wpk_d)};
    hipLaunchKernelGGL((cb::conv5x5_kernel<T, 1, 16, 28, 28, 0, 3, 0, 2>), dim3(B * S::SPLIT), dim3(cb::NTHR), 0,
                       cur_stream(), dptr<T>(x), w1.data_ptr<float>(), b1.data_ptr<float>(), dptr<T>(y1),
                       fslab1.data_ptr<float>(), fstats1.data_ptr<float>(), shift1.data_ptr<float>(), S::SPLIT,
                       PoolIn<T>{}, BwdIn<T>{}, BwdEpi<T>{}, nullptr, pk, gin);
  });
  DPA_CHECK_LAUNCH();
}

// Workgroups per image of the conv2 data gradient: 2 for bf16 / fp16 (4: +2.5 us,
// profiles/r6m_split_ab.txt, r6ax_*), 4 for fp32, whose 16x16x4 MFMA chains are 4x as long
// (profiles/r6bf_fp32_dgrad_split_ab.txt).  Compile-time per dtype: the kernels take it as a
// constant (kDgradSplitT<T>), the host sizes follow from the tensor dtype (dgrad_split).
#ifndef DPA_DGRAD2_SPLIT
#define DPA_DGRAD2_SPLIT 2
#endif
#ifndef DPA_DGRAD2_SPLIT_F32
#define DPA_DGRAD2_SPLIT_F32 4
#endif
template <typename T>
constexpr int kDgradSplitT = std::is_same<T, float>::value ? DPA_DGRAD2_SPLIT_F32 : DPA_DGRAD2_SPLIT;
static int dgrad_split(bool fp32) { return fp32 ? DPA_DGRAD2_SPLIT_F32 : DPA_DGRAD2_SPLIT; }
int64_t dgrad2_rows(int64_t B, bool fp32) { return B * dgrad_split(fp32); }

// [pool2/ReLU2/BN2 backward] -> conv2 data grad -> dp1 (+ BN1 partial sums rows).
void conv2_dgrad(at::Tensor wpk_d, at::Tensor y2, at::Tensor dp2, at::Tensor idx2, at::Tensor fstats2,
                 at::Tensor gsum2, at::Tensor g2, double eps2, at::Tensor dp1, at::Tensor idx1, at::Tensor xh1,
                 at::Tensor bslab1, XcPtr xc) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(dp1); DPA_CHECK_INPUT(wpk_d);
  TORCH_CHECK(wpk_d.numel() == cb::W2D_LEN && wpk_d.scalar_type() == y2.scalar_type(),
              "packed conv2 data-grad weights");
  const int B = (int)y2.size(0);
  TORCH_CHECK(y2.size(1) == 32 && y2.size(2) == 14 && dp2.numel() == (int64_t)B * 32 * 49);
  TORCH_CHECK(dp1.numel() == (int64_t)B * 16 * 196 && idx1.numel() == dp1.numel() && xh1.numel() == dp1.numel());
  TORCH_CHECK(bslab1.numel() == dgrad2_rows(B, y2.scalar_type() == at::kFloat) * 32, "BN1 partial-sum slab size");
  if (B == 0) return;
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    constexpr int ds = kDgradSplitT<T>;
    BwdIn<T> bi = bwd_in<T>(dp2, idx2, y2, fstats2, gsum2, c10::nullopt, g2, eps2, 32, c10::nullopt, c10::nullopt);
    bi.xs = site_of(xc, xgmi::kSiteBwd2Dgrad);
    xgmi::set_site_grid(bi.xs, B * ds, "conv2_dgrad");
    BwdEpi<T> ep{idx1.data_ptr<uint8_t>(), dptr<T>(xh1), bslab1.data_ptr<float>()};
    hipLaunchKernelGGL((cb::conv5x5_kernel<T, 32, 16, 14, 14, 2, 2, 1, 1>), dim3(B * ds), dim3(cb::NTHR),
                       0, cur_stream(), nullptr, nullptr, nullptr, dptr<T>(dp1), nullptr, nullptr, nullptr,
                       ds, PoolIn<T>{}, bi, ep, dptr<T>(wpk_d), cb::WPack<T>{});
  });
  DPA_CHECK_LAUNCH();
}

// The backward through [BN2 -> ReLU2 -> pool2] feeds two independent products of
// layer 2: the data grad (-> dp1 + BN1 partial sums, kDgradSplitT<T> workgroups per
// image) and the weight-grad partials (WG2_ROWS-row chunks).  One launch hosts
// both roles -- workgroups [0, ndg) the data grad, [ndg, grid) the weight grad --
// so they overlap on the chip instead of running back to back (each alone fills
// only 64 / 128 of the 256 CUs at B = 32) and one kernel boundary disappears.
constexpr int WG2_ROWS_ = 4;
constexpr int WG1_ROWS_ = 4;
int64_t wgrad_bn_rows(int64_t layer, int64_t B);
// fc weight / bias gradient of the per-image head (csrc/kernels/convnet_head.hip): the head's
// one reduction over the batch, computed by extra workgroups of the conv2 backward launch
// (which needs none of it) instead of on the head's critical path:
//   dW[n][k] = sum_b dls[b][n] * p2[b][k],   db[n] = sum_b dls[b][n]
// dls = d(scale * loss)/dlogits and p2 = the pooled features, both in the storage dtype
// (autocast's operands); fp32 accumulation in batch order.
template <typename T>
struct FcW {
  const T* dls;  // [B][N]
  const T* p2;   // [B][K]
  float* dw;     // [N][K]
  float* db;     // [N]
  int B = 0, N = 0;
  GradChk chk;   // producer-side check (common.h)
};
constexpr int FC_K = 32 * 49;
constexpr int FC_COLS = cb::NTHR;  // columns per workgroup, one per lane
constexpr int FC_BMAX = 64, FC_NMAX = 16;
constexpr int FC_BLOCKS = (FC_K + FC_COLS - 1) / FC_COLS;

template <typename T>
__device__ __forceinline__ void fc_wgrad_body(const FcW<T>& f, int wg) {
  __shared__ __attribute__((aligned(16))) float dl_s[FC_BMAX][FC_NMAX];
  const int tid = threadIdx.x;
  const int col = wg * FC_COLS + tid, cc = min(col, FC_K - 1);
  const int B = f.B, N = f.N;
  const bool chk = f.chk.word != nullptr;  // producer-side check (common.h GradChk)
  // the dls table (B x N, zero-padded to 16 classes) through LDS, broadcast reads below
  for (int e = tid; e < FC_BMAX * FC_NMAX; e += cb::NTHR) {
    const int b = e / FC_NMAX, n = e % FC_NMAX;
    const float v = Cvt<T>::to_f(f.dls[min(b, B - 1) * N + min(n, N - 1)]);
    dl_s[b][n] = (b < B && n < N) ? v : 0.f;
  }
  float acc[FC_NMAX];
#pragma unroll
  for (int n = 0; n < FC_NMAX; ++n) acc[n] = 0.f;
  __syncthreads();
  for (int b0 = 0; b0 < B; b0 += 32) {  // 32 rows in flight per batch (one batch at B <= 32)
    float pv[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int b = b0 + u;
      pv[u] = Cvt<T>::to_f(f.p2[(size_t)min(b, B - 1) * FC_K + cc]) * (b < B ? 1.f : 0.f);
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const f32x4* row = reinterpret_cast<const f32x4*>(dl_s[min(b0 + u, FC_BMAX - 1)]);
#pragma unroll
      for (int q = 0; q < FC_NMAX / 4; ++q) {
        const f32x4 d = row[q];
        acc[4 * q + 0] += d[0] * pv[u];
        acc[4 * q + 1] += d[1] * pv[u];
        acc[4 * q + 2] += d[2] * pv[u];
        acc[4 * q + 3] += d[3] * pv[u];
      }
    }
  }
  bool bad = false;
  if (col < FC_K) {
#pragma unroll
    for (int n = 0; n < FC_NMAX; ++n)
      if (n < N) {
        f.dw[(size_t)n * FC_K + col] = acc[n];
        bad |= GradChk::bad(acc[n], f.chk.bound);
      }
  }
  if (wg == 0 && tid < N) {
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += dl_s[b][tid];
    f.db[tid] = a;
    bad |= GradChk::bad(a, f.chk.bound);
  }
  if (chk) f.chk.flag(bad);
}

template <typename T>
__global__ void __launch_bounds__(cb::NTHR) fc_wgrad_kernel(FcW<T> f) { fc_wgrad_body<T>(f, (int)blockIdx.x); }

template <typename T>
__global__ void __launch_bounds__(cb::NTHR)
conv2_bwd_kernel(const T* __restrict__ wpk_d, T* __restrict__ dp1, BwdIn<T> bi_d, BwdEpi<T> ep,
                 const T* __restrict__ p1, float* __restrict__ wslab2, BwdIn<T> bi_w, int ndg, int nwg, FcW<T> fw) {
  constexpr int nsw = (14 + WG2_ROWS_ - 1) / WG2_ROWS_;
  const int bid = (int)blockIdx.x;
  if (bid < ndg)
    cb::conv5x5_body<T, 32, 16, 14, 14, 2, 2, 1, 1>(nullptr, nullptr, nullptr, dp1, nullptr, nullptr, nullptr,
                                                    kDgradSplitT<T>, PoolIn<T>{}, bi_d, ep, wpk_d, cb::WPack<T>{}, bid);
  else if (bid < ndg + nwg)
    cb::conv5x5_wgrad_body<T, 16, 32, 14, 14, WG2_ROWS_, 2>(p1, nullptr, wslab2, nsw, bi_w, bid - ndg);
  else
    fc_wgrad_body<T>(fw, bid - ndg - nwg);
}

// fp32: the same three roles in ONE launch, with the big tiles of both conv roles in
// dynamic LDS (cb::conv5x5_body / conv5x5_wgrad_body DYN): each workgroup runs one role,
// so the launch needs the largest role's tiles (~114 KB) instead of the 173 KB sum of
// the static arrays, which does not fit a CU's 160 KB -- the reason fp32 ran the data
// gradient and the weight gradient as two launches, one after the other, each on at
// most half the CUs (profiles/r6g_cn_steady_fp32.txt: 16.7 + 15.2 us).
template <typename T>
__global__ void __launch_bounds__(cb::NTHR)
conv2_bwd_dyn_kernel(const T* __restrict__ wpk_d, T* __restrict__ dp1, BwdIn<T> bi_d, BwdEpi<T> ep,
                     const T* __restrict__ p1, float* __restrict__ wslab2, BwdIn<T> bi_w, int ndg, int nwg,
                     FcW<T> fw) {
  constexpr int nsw = (14 + WG2_ROWS_ - 1) / WG2_ROWS_;
  const int bid = (int)blockIdx.x;
  if (bid < ndg)
    cb::conv5x5_body<T, 32, 16, 14, 14, 2, 2, 1, 1, true>(nullptr, nullptr, nullptr, dp1, nullptr, nullptr, nullptr,
                                                          kDgradSplitT<T>, PoolIn<T>{}, bi_d, ep, wpk_d,
                                                          cb::WPack<T>{}, bid);
  else if (bid < ndg + nwg)
    cb::conv5x5_wgrad_body<T, 16, 32, 14, 14, WG2_ROWS_, 2, false, false, true>(p1, nullptr, wslab2, nsw, bi_w,
                                                                                bid - ndg);
  else
    fc_wgrad_body<T>(fw, bid - ndg - nwg);
}

template <typename T>
constexpr size_t conv2_bwd_dyn_bytes() {
  return std::max(cb::conv5x5_dyn_bytes<T, 32, 16, 14, 14>(), cb::WgradLds<T, 16, 32, 14, 14, WG2_ROWS_>::bytes);
}

// DPA_FP32_MERGED_BWD=0: the two fp32 launches below (A/B runs)
static bool fp32_merged_bwd() {
  static const bool on = [] {
    const char* e = std::getenv("DPA_FP32_MERGED_BWD");
    if (e != nullptr && std::atoi(e) == 0) return false;
    const size_t b = conv2_bwd_dyn_bytes<float>();
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv2_bwd_dyn_kernel<float>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)b) == hipSuccess;
  }();
  return on;
}

// bf16 / fp16: the merged launch with the conv tiles in dynamic LDS too -- the largest
// role's bytes per workgroup instead of the static arrays' sum: step 0.04859 -> 0.04823 ms
// over 5 same-box pairs (7 of 8 pairs faster; forced step unchanged,
// profiles/r6au_lp_dyn_bwd_ab.txt).  DPA_LP_DYN_BWD=0: the static-LDS kernel (A/B runs)
static bool lp_dyn_bwd() {
  static const bool on = [] {
    const char* e = std::getenv("DPA_LP_DYN_BWD");
    if (e != nullptr && std::atoi(e) == 0) return false;
    bool ok = true;
    for (const void* k : {reinterpret_cast<const void*>(&conv2_bwd_dyn_kernel<__hip_bfloat16>),
                          reinterpret_cast<const void*>(&conv2_bwd_dyn_kernel<__half>)})
      ok = ok && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)std::max(conv2_bwd_dyn_bytes<__hip_bfloat16>(),
                                                   conv2_bwd_dyn_bytes<__half>())) == hipSuccess;
    return ok;
  }();
  return on;
}

// fp32 without the merged launch: the conv2 weight-gradient role and the fc weight gradient
// in one launch (the data-gradient role's static LDS does not fit beside the weight gradient's)
template <typename T>
__global__ void __launch_bounds__(cb::NTHR)
conv2_wgrad_fc_kernel(const T* __restrict__ p1, float* __restrict__ wslab2, BwdIn<T> bi_w, int nwg, FcW<T> fw) {
  constexpr int nsw = (14 + WG2_ROWS_ - 1) / WG2_ROWS_;
  const int bid = (int)blockIdx.x;
  if (bid < nwg)
    cb::conv5x5_wgrad_body<T, 16, 32, 14, 14, WG2_ROWS_, 2>(p1, nullptr, wslab2, nsw, bi_w, bid);
  else
    fc_wgrad_body<T>(fw, bid - nwg);
}

template <typename T>
static FcW<T> fc_args(const c10::optional<at::Tensor>& dls, const c10::optional<at::Tensor>& p2,
                      const c10::optional<at::Tensor>& dw, const c10::optional<at::Tensor>& db, int B, at::ScalarType st) {
  FcW<T> f{};
  if (!dls.has_value()) return f;
  TORCH_CHECK(p2.has_value() && dw.has_value() && db.has_value(), "fc weight gradient: dls, p2, dw, db go together");
  DPA_CHECK_INPUT(*dls); DPA_CHECK_INPUT(*p2); DPA_CHECK_INPUT(*dw); DPA_CHECK_INPUT(*db);
  const int N = (int)(dls->numel() / std::max(B, 1));
  TORCH_CHECK(dls->numel() == (int64_t)B * N && N >= 1 && N <= FC_NMAX && B <= FC_BMAX, "fc weight gradient: dls [B][N <= 16]");
  TORCH_CHECK(dls->scalar_type() == st && p2->scalar_type() == st && p2->numel() == (int64_t)B * FC_K);
  TORCH_CHECK(dw->scalar_type() == at::kFloat && dw->numel() == (int64_t)N * FC_K && db->scalar_type() == at::kFloat &&
              db->numel() == N, "fc weight gradient: fp32 dw [N][1568], db [N]");
  f.dls = dptr<T>(*dls);
  f.p2 = dptr<T>(*p2);
  f.dw = dw->data_ptr<float>();
  f.db = db->data_ptr<float>();
  f.B = B;
  f.N = N;
  return f;
}

// fc weight / bias gradient as its own launch (fp32 / split-backward paths)
void fc_wgrad(at::Tensor dls, at::Tensor p2, at::Tensor dw, at::Tensor db) {
  const int B = (int)(p2.numel() / FC_K);
  if (B == 0) return;
  with_t(dt_of(p2), [&](auto tag) {
    typedef decltype(tag) T;
    FcW<T> f = fc_args<T>(dls, p2, dw, db, B, p2.scalar_type());
    hipLaunchKernelGGL(fc_wgrad_kernel<T>, dim3(FC_BLOCKS), dim3(cb::NTHR), 0, cur_stream(), f);
  });
  DPA_CHECK_LAUNCH();
}

// The producer-side gradient check's words (optim/sgd.py prechecked AMP step; common.h
// GradChk): int32[2], [0] cleared by the head launch and set by any producer lane that
// writes a bad value, [1] the step's scale (recorded by the head launch).
static GradChk grad_chk_of(const c10::optional<at::Tensor>& chk, const XcPtr& xc) {
  GradChk g;
  if (!chk.has_value()) return g;
  DPA_CHECK_INPUT(*chk);
  TORCH_CHECK(chk->scalar_type() == at::kInt && chk->numel() == 2, "gradient check: int32[2] words");
  g.word = chk->data_ptr<int>();
  g.bound = 3.402823466e38f / (float)(xc ? xc->world() : 1);
  return g;
}

// [pool2/ReLU2/BN2 backward] -> {conv2 data grad -> dp1 (+BN1 partial sums), conv2 weight-grad partials}
// (+ with fc_*: the fc weight / bias gradient of the per-image head in extra workgroups).
// gsum2: rows of BN2 backward sums ([S1 | S2] per row, summed here); lsum2: this rank's rows
// when gsum2 was all-reduced; dg2 / dbe2: BN2's dgamma / dbeta, written from this rank's sums.
void conv2_bwd(at::Tensor wpk_d, at::Tensor y2, at::Tensor dp2, at::Tensor idx2, at::Tensor fstats2,
               at::Tensor gsum2, at::Tensor g2, double eps2, at::Tensor dp1, at::Tensor idx1, at::Tensor xh1,
               at::Tensor bslab1, at::Tensor p1, at::Tensor wslab2, XcPtr xc, c10::optional<at::Tensor> lsum2,
               c10::optional<at::Tensor> dg2, c10::optional<at::Tensor> dbe2, c10::optional<at::Tensor> fc_dls,
               c10::optional<at::Tensor> fc_p2, c10::optional<at::Tensor> fc_dw, c10::optional<at::Tensor> fc_db,
               c10::optional<at::Tensor> chk) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(dp1); DPA_CHECK_INPUT(wpk_d); DPA_CHECK_INPUT(p1); DPA_CHECK_INPUT(wslab2);
  TORCH_CHECK(wpk_d.numel() == cb::W2D_LEN && wpk_d.scalar_type() == y2.scalar_type(),
              "packed conv2 data-grad weights");
  const int B = (int)y2.size(0);
  TORCH_CHECK(y2.size(1) == 32 && y2.size(2) == 14 && dp2.numel() == (int64_t)B * 32 * 49);
  TORCH_CHECK(dp1.numel() == (int64_t)B * 16 * 196 && idx1.numel() == dp1.numel() && xh1.numel() == dp1.numel());
  TORCH_CHECK(p1.numel() == dp1.numel() && p1.scalar_type() == y2.scalar_type());
  TORCH_CHECK(bslab1.numel() == dgrad2_rows(B, y2.scalar_type() == at::kFloat) * 32, "BN1 partial-sum slab size");
  TORCH_CHECK(dg2.has_value() == dbe2.has_value(), "conv2_bwd: dg2 and dbe2 go together");
  if (dg2.has_value()) TORCH_CHECK(dg2->numel() == 32 && dbe2->numel() == 32 && dg2->scalar_type() == at::kFloat);
  if (xc) TORCH_CHECK(!lsum2.has_value(), "fused SyncBN exchange: gsum2 must be this rank's rows (no lsum2)");
  const int ndg = B * dgrad_split(y2.scalar_type() == at::kFloat), nwg = (int)wgrad_bn_rows(2, B);
  TORCH_CHECK(wslab2.numel() == (int64_t)nwg * (32 * 400 + 32), "wgrad slab size");
  if (B == 0) return;
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    BwdIn<T> bd = bwd_in<T>(dp2, idx2, y2, fstats2, gsum2, lsum2, g2, eps2, 32, dg2, dbe2);
    BwdIn<T> bw = bd;
    bw.dgamma = bw.dbeta = nullptr;  // one writer: the data-gradient role's workgroup 0
    bd.xs = site_of(xc, xgmi::kSiteBwd2Dgrad);
    bw.xs = site_of(xc, xgmi::kSiteBwd2Wgrad);
    xgmi::set_site_grid(bd.xs, ndg, "conv2_bwd data gradient");  // each role's workgroups take
    xgmi::set_site_grid(bw.xs, nwg, "conv2_bwd weight gradient");  // tickets on their own site
    BwdEpi<T> ep{idx1.data_ptr<uint8_t>(), dptr<T>(xh1), bslab1.data_ptr<float>()};
    FcW<T> fw = fc_args<T>(fc_dls, fc_p2, fc_dw, fc_db, B, y2.scalar_type());
    const int nfc = fc_dls.has_value() ? FC_BLOCKS : 0;
    if (chk.has_value()) {  // every gradient this launch finishes: BN2's, the fc layer's
      TORCH_CHECK(nfc > 0 && dg2.has_value(), "gradient check: the launch with the fc role and BN2's gradients");
      bd.chk = fw.chk = grad_chk_of(chk, xc);
      bd.chk_coef = 1;
    }
    if constexpr (std::is_same<T, float>::value) {
      if (fp32_merged_bwd()) {  // one launch, the conv tiles in dynamic LDS (conv2_bwd_dyn_kernel)
        hipLaunchKernelGGL(conv2_bwd_dyn_kernel<T>, dim3(ndg + nwg + nfc), dim3(cb::NTHR), conv2_bwd_dyn_bytes<T>(),
                           cur_stream(), dptr<T>(wpk_d), dptr<T>(dp1), bd, ep, dptr<T>(p1), wslab2.data_ptr<float>(),
                           bw, ndg, nwg, fw);
        return;
      }
      // fp32 static tiles: the two roles' LDS (173 KB) exceed one CU's 160 KB -> separate launches
      // (the fc weight gradient: extra workgroups of the weight-gradient launch; its site's
      // tickets are the nwg conv workgroups', set above)
      bd.xs.nblk = 0;  // the data-gradient launch is its site's whole grid (ndg: checked above)
      hipLaunchKernelGGL((cb::conv5x5_kernel<T, 32, 16, 14, 14, 2, 2, 1, 1>), dim3(ndg), dim3(cb::NTHR), 0,
                         cur_stream(), nullptr, nullptr, nullptr, dptr<T>(dp1), nullptr, nullptr, nullptr,
                         kDgradSplitT<T>, PoolIn<T>{}, bd, ep, dptr<T>(wpk_d), cb::WPack<T>{});
      hipLaunchKernelGGL(conv2_wgrad_fc_kernel<T>, dim3(nwg + nfc), dim3(cb::NTHR), 0, cur_stream(), dptr<T>(p1),
                         wslab2.data_ptr<float>(), bw, nwg, fw);
    } else if (lp_dyn_bwd()) {  // the roles' tiles in dynamic LDS (the largest role's bytes)
      hipLaunchKernelGGL(conv2_bwd_dyn_kernel<T>, dim3(ndg + nwg + nfc), dim3(cb::NTHR), conv2_bwd_dyn_bytes<T>(),
                         cur_stream(), dptr<T>(wpk_d), dptr<T>(dp1), bd, ep, dptr<T>(p1), wslab2.data_ptr<float>(),
                         bw, ndg, nwg, fw);
    } else {
      hipLaunchKernelGGL(conv2_bwd_kernel<T>, dim3(ndg + nwg + nfc), dim3(cb::NTHR), 0, cur_stream(), dptr<T>(wpk_d),
                         dptr<T>(dp1), bd, ep, dptr<T>(p1), wslab2.data_ptr<float>(), bw, ndg, nwg, fw);
    }
  });
  DPA_CHECK_LAUNCH();
}

// [pool/ReLU/BN backward of the block whose conv is (CIN->COUT, HxW)] -> weight-grad partials.
// layer 2: x = p1 [B,16,14,14], (y, dp, idx) = layer-2 tensors; layer 1: x = images, layer-1 tensors.
// Weight-gradient row chunks (BN backward applied on the fly per chunk): more,
// shorter workgroups than one image each (B = 32 -> 32 workgroups for 256 CUs).
constexpr int WG1_ROWS = WG1_ROWS_;  // layer 1 (28 rows): 7 chunks per image
constexpr int WG2_ROWS = WG2_ROWS_;  // layer 2 (14 rows): 4 chunks per image (last one 2 rows)
int64_t wgrad_bn_rows(int64_t layer, int64_t B) {
  TORCH_CHECK(layer == 1 || layer == 2);
  return B * (layer == 1 ? (28 + WG1_ROWS - 1) / WG1_ROWS : (14 + WG2_ROWS - 1) / WG2_ROWS);
}

void conv_wgrad_bn(at::Tensor x, at::Tensor y, at::Tensor dp, at::Tensor idx, at::Tensor fstats, at::Tensor gsum,
                   c10::optional<at::Tensor> lsum, at::Tensor gamma, double eps, c10::optional<at::Tensor> dgamma,
                   c10::optional<at::Tensor> dbeta, at::Tensor wslab, XcPtr xc) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(y);
  const int B = (int)y.size(0);
  const int cin = (int)x.size(1), cout = (int)y.size(1), H = (int)y.size(2);
  TORCH_CHECK(x.scalar_type() == y.scalar_type());
  if (B == 0) return;
  with_t(dt_of(y), [&](auto tag) {
    typedef decltype(tag) T;
    BwdIn<T> bi = bwd_in<T>(dp, idx, y, fstats, gsum, lsum, gamma, eps, cout, dgamma, dbeta);
    if (xc) {
      TORCH_CHECK(!lsum.has_value(), "fused SyncBN exchange: gsum must be this rank's rows (no lsum)");
      bi.xs = site_of(xc, cout == 32 ? xgmi::kSiteBwd2Wgrad : xgmi::kSiteBwd1);
    }
    if (cin == 16 && cout == 32 && H == 14) {
      constexpr int ns = (14 + WG2_ROWS - 1) / WG2_ROWS;
      TORCH_CHECK(wslab.numel() == (int64_t)B * ns * (32 * 400 + 32), "wgrad slab size");
      hipLaunchKernelGGL((cb::conv5x5_wgrad_kernel<T, 16, 32, 14, 14, WG2_ROWS, 2>), dim3(B * ns), dim3(cb::NTHR),
                         0, cur_stream(), dptr<T>(x), nullptr, wslab.data_ptr<float>(), ns, bi);
    } else if (cin == 1 && cout == 16 && H == 28) {
      constexpr int ns = (28 + WG1_ROWS - 1) / WG1_ROWS;
      TORCH_CHECK(wslab.numel() == (int64_t)B * ns * (16 * 25 + 16), "wgrad slab size");
      hipLaunchKernelGGL((cb::conv5x5_wgrad_kernel<T, 1, 16, 28, 28, WG1_ROWS, 2>), dim3(B * ns), dim3(cb::NTHR),
                         0, cur_stream(), dptr<T>(x), nullptr, wslab.data_ptr<float>(), ns, bi);
    } else {
      TORCH_CHECK(false, "fused wgrad: shape not instantiated");
    }
  });
  DPA_CHECK_LAUNCH();
}


// ---------------------------------------------------------------------------
// The last backward launch: conv1 weight-grad partials AND every weight-grad
// column sum, so no separate reduction launch follows.
//   role A, workgroups [0, nwg1): BN1 bwd -> conv1 wgrad partial row (write-
//     through), then a two-level in-launch reduction: the last arriver of each
//     group of RG rows sums them into a group row; the last group sums the group
//     rows into [dW1 | db1] (tickets on self-resetting counters: graph-replayable).
//   role B, workgroups [nwg1, grid): column sums of the conv2 weight-grad slab
//     (written by the previous launch) into [dW2 | db2], RB_COLS columns each.
// Reference op: /root/reference/origin_main.py:13 (conv1 weight/bias grads),
// :19 (conv2's); replaces conv_wgrad_bn + slab_reduce (one launch and one
// kernel boundary less per step).
// ---------------------------------------------------------------------------
constexpr int RG = 16;        // role A: rows per group
constexpr int RB_COLS = 32;   // role B: columns per workgroup (8 row groups of 32 lanes)

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rows x n (row-major) -> out[n]: column sums in row order 0.. (deterministic)
__device__ __forceinline__ void colsum_sc1(const float* __restrict__ src, int rows, int n, float* __restrict__ out,
                                           bool wt) {
  for (int j = threadIdx.x; j < n; j += cb::NTHR) {
    float a = 0.f;
    int r = 0;
    for (; r + 7 < rows; r += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ld_sc1(src + (size_t)(r + k) * n + j);
#pragma unroll
      for (int k = 0; k < 8; ++k) a += v[k];
    }
    for (; r < rows; ++r) a += ld_sc1(src + (size_t)r * n + j);
    if (wt) __hip_atomic_store(out + j, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else out[j] = a;
  }
}

template <typename T>
__global__ void __launch_bounds__(cb::NTHR)
wgrad1_reduce_kernel(const T* __restrict__ x, float* __restrict__ wslab1, float* __restrict__ gslab1,
                     float* __restrict__ out1, BwdIn<T> bi, int nwg1, const float* __restrict__ wslab2, int rows2,
                     int n2, float* __restrict__ out2, int* __restrict__ cnt) {
  constexpr int N1 = 16 * 25 + 16;
  __shared__ int last_s;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= nwg1) {
    // role B: RB_COLS columns of the conv2 slab, 8 row groups of 32 lanes, fixed-order sums
    __shared__ float part[8][RB_COLS + 1];
    const int c0 = ((int)blockIdx.x - nwg1) * RB_COLS;
    const int col = c0 + (tid % RB_COLS), g = tid / RB_COLS;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (col < n2) {
      int r = g;
      for (; r + 3 * 8 < rows2; r += 4 * 8) {
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += wslab2[(size_t)(r + 8 * k) * n2 + col];
      }
      for (; r < rows2; r += 8) a[0] += wslab2[(size_t)r * n2 + col];
    }
    part[g][tid % RB_COLS] = (a[0] + a[1]) + (a[2] + a[3]);
    __syncthreads();
    if (tid < RB_COLS && c0 + tid < n2) {
      float t = 0.f;
#pragma unroll
      for (int gg = 0; gg < 8; ++gg) t += part[gg][tid];
      out2[c0 + tid] = t;
    }
    return;
  }
  // role A
  const int bid = blockIdx.x;
  constexpr int ns = (28 + WG1_ROWS_ - 1) / WG1_ROWS_;
  cb::conv5x5_wgrad_body<T, 1, 16, 28, 28, WG1_ROWS_, 2, true>(x, nullptr, wslab1, ns, bi, bid);
  const int ng = (nwg1 + RG - 1) / RG, g = bid / RG;
  const int grows = min(RG, nwg1 - g * RG);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's row has left the CU
  __syncthreads();
  if (tid == 0)
    last_s = __hip_atomic_fetch_add(&cnt[g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == grows - 1;
  __syncthreads();
  if (!last_s) return;
  colsum_sc1(wslab1 + (size_t)g * RG * N1, grows, N1, gslab1 + (size_t)g * N1, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(&cnt[g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm for the next launch
    last_s = __hip_atomic_fetch_add(&cnt[ng], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
  }
  __syncthreads();
  if (!last_s) return;
  colsum_sc1(gslab1, ng, N1, out1, false);
  if (tid == 0) __hip_atomic_store(&cnt[ng], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int64_t wgrad1_counters(int64_t B) { return (wgrad_bn_rows(1, B) + RG - 1) / RG + 1; }

// BN1 bwd -> conv1 wgrad, + the column sums of both weight-grad slabs:
// out1 = [dW1 | db1] (416 floats), out2 = [dW2 | db2] (12832 floats).
// cnt: int32[wgrad1_counters(B)], zeroed once (the kernel re-arms it).
void wgrad1_reduce(at::Tensor x, at::Tensor y1, at::Tensor dp1, at::Tensor idx1, at::Tensor fstats1, at::Tensor gsum,
                   c10::optional<at::Tensor> lsum, at::Tensor g1, double eps1, at::Tensor dg1, at::Tensor dbe1,
                   at::Tensor wslab1, at::Tensor gslab1, at::Tensor out1, at::Tensor wslab2, at::Tensor out2,
                   at::Tensor cnt, XcPtr xc) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(wslab1); DPA_CHECK_INPUT(wslab2); DPA_CHECK_INPUT(cnt);
  const int B = (int)y1.size(0);
  TORCH_CHECK(x.size(1) == 1 && y1.size(1) == 16 && y1.size(2) == 28 && x.scalar_type() == y1.scalar_type());
  const int nwg1 = (int)wgrad_bn_rows(1, B), ng = (nwg1 + RG - 1) / RG;
  constexpr int N1 = 16 * 25 + 16, N2 = 32 * 400 + 32;
  const int rows2 = (int)wgrad_bn_rows(2, B);
  TORCH_CHECK(wslab1.numel() == (int64_t)nwg1 * N1 && gslab1.numel() >= (int64_t)ng * N1 && out1.numel() == N1,
              "wgrad1_reduce: conv1 slab sizes");
  TORCH_CHECK(wslab2.numel() == (int64_t)rows2 * N2 && out2.numel() == N2, "wgrad1_reduce: conv2 slab sizes");
  TORCH_CHECK(cnt.scalar_type() == at::kInt && cnt.numel() >= ng + 1, "wgrad1_reduce: counters");
  if (B == 0) return;
  const int nred = (N2 + RB_COLS - 1) / RB_COLS;
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    BwdIn<T> bi = bwd_in<T>(dp1, idx1, y1, fstats1, gsum, lsum, g1, eps1, 16, dg1, dbe1);
    if (xc) {
      TORCH_CHECK(!lsum.has_value(), "fused SyncBN exchange: gsum must be this rank's rows (no lsum)");
      bi.xs = site_of(xc, xgmi::kSiteBwd1);
      xgmi::set_site_grid(bi.xs, nwg1, "wgrad1_reduce");  // the reduction workgroups take no tickets
    }
    hipLaunchKernelGGL(wgrad1_reduce_kernel<T>, dim3(nwg1 + nred), dim3(cb::NTHR), 0, cur_stream(), dptr<T>(x),
                       wslab1.data_ptr<float>(), gslab1.data_ptr<float>(), out1.data_ptr<float>(), bi, nwg1,
                       wslab2.data_ptr<float>(), rows2, N2, out2.data_ptr<float>(), cnt.data_ptr<int>());
  });
  DPA_CHECK_LAUNCH();
}

// BN1 bwd -> conv1 weight-grad partial rows (wslab1) AND, in extra workgroups, the
// column sums of the conv2 weight-grad slab into [dW2 | db2] (independent work that
// fills the CUs the 224 conv1 workgroups leave idle).  The conv1 slab's own column
// sums are left to the consumer: the fused AMP-SGD launch (optim.hip SlabSrc) or a
// slab_reduce launch.
template <typename T>
__global__ void __launch_bounds__(cb::NTHR)
wgrad1_slab2_kernel(const T* __restrict__ x, float* __restrict__ wslab1, BwdIn<T> bi, int nwg1,
                    const float* __restrict__ wslab2, int rows2, int n2, float* __restrict__ out2, GradChk rc) {
  constexpr int ns = (28 + WG1_ROWS_ - 1) / WG1_ROWS_;
  if ((int)blockIdx.x < nwg1)
    cb::conv5x5_wgrad_body<T, 1, 16, 28, 28, WG1_ROWS_, 2, false, true>(x, nullptr, wslab1, ns, bi, (int)blockIdx.x);
  else
    cb::slab_reduce_body(nullptr, 0, 0, nullptr, wslab2, rows2, n2, out2, (int)blockIdx.x - nwg1, rc);
}

void conv1_wgrad_slab2(at::Tensor x, at::Tensor y1, at::Tensor dp1, at::Tensor idx1, at::Tensor fstats1,
                       at::Tensor gsum, c10::optional<at::Tensor> lsum, at::Tensor g1, double eps1, at::Tensor dg1,
                       at::Tensor dbe1, at::Tensor wslab1, at::Tensor wslab2, at::Tensor out2, XcPtr xc,
                       c10::optional<at::Tensor> chk) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(wslab1); DPA_CHECK_INPUT(wslab2); DPA_CHECK_INPUT(out2);
  const int B = (int)y1.size(0);
  TORCH_CHECK(x.size(1) == 1 && y1.size(1) == 16 && y1.size(2) == 28 && x.scalar_type() == y1.scalar_type());
  const int nwg1 = (int)wgrad_bn_rows(1, B);
  constexpr int N1 = 16 * 25 + 16, N2 = 32 * 400 + 32;
  const int rows2 = (int)wgrad_bn_rows(2, B);
  TORCH_CHECK(wslab1.numel() == (int64_t)nwg1 * N1, "conv1_wgrad_slab2: conv1 slab size");
  TORCH_CHECK(wslab2.numel() == (int64_t)rows2 * N2 && out2.numel() == N2, "conv1_wgrad_slab2: conv2 slab sizes");
  if (B == 0) return;
  const int nred = (N2 + cb::SR_COLS - 1) / cb::SR_COLS;
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    BwdIn<T> bi = bwd_in<T>(dp1, idx1, y1, fstats1, gsum, lsum, g1, eps1, 16, dg1, dbe1);
    if (xc) {
      TORCH_CHECK(!lsum.has_value(), "fused SyncBN exchange: gsum must be this rank's rows (no lsum)");
      bi.xs = site_of(xc, xgmi::kSiteBwd1);
      xgmi::set_site_grid(bi.xs, nwg1, "conv1_wgrad_slab2");  // the reduction workgroups take no tickets
    }
    GradChk rc;
    if (chk.has_value()) {  // BN1's gradients, conv1's partial rows, conv2's column sums
      rc = bi.chk = grad_chk_of(chk, xc);
      bi.chk_coef = 1;
      bi.chk_rows = 1;
      bi.chk_row_bound = rc.bound / (float)nwg1;
    }
    hipLaunchKernelGGL(wgrad1_slab2_kernel<T>, dim3(nwg1 + nred), dim3(cb::NTHR), 0, cur_stream(), dptr<T>(x),
                       wslab1.data_ptr<float>(), bi, nwg1, wslab2.data_ptr<float>(), rows2, N2,
                       out2.data_ptr<float>(), rc);
  });
  DPA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// The ConvNet's optimizer step with the conv1 weight gradient inside it: ONE launch
// instead of [conv1 wgrad + conv2 column sums] and [fused AMP step] (optim/sgd.py
// defer_wgrad1: the backward leaves conv1's weight gradient to the optimizer, which
// computes it in its own launch -- the update still happens in scaler.step()).
//   workgroups [0, nw1): producers -- BN1 backward -> conv1 weight-gradient partial row,
//     stored write-through, then one arrival on w1cnt;
//   workgroups [nw1, grid): the fused AMP step (csrc/kernels/amp_step.h) with three
//     slab sources: BN1's [dbeta1 | dgamma1] from the conv2 backward's partial sums,
//     conv1's [dW1 | db1] (its owners wait for the producers' arrivals) and conv2's
//     [dW2 | db2] (written by the previous launch: summed at once).
// Producers come first in the grid, so the in-order dispatcher places all of them before
// any AMP workgroup: a waiting owner can never hold a slot a producer needs.
// Reference: /root/reference/ddp_main.py:91-93 (backward, scaler.step, update) and
// origin_main.py:13-14 (conv1 / BN1, whose gradients these are).
// ---------------------------------------------------------------------------
constexpr int CAS_U = 2;  // granules per lane of the AMP workgroups (keeps the AMP grid <= one per CU)

template <typename T, bool XG>
__global__ void __launch_bounds__(cb::NTHR)
convnet_amp_step_kernel(const T* __restrict__ x, float* __restrict__ wslab1, BwdIn<T> bi, int nw1,
                        int* __restrict__ w1cnt, opt::MTList L, float* __restrict__ scale, int* __restrict__ tracker,
                        float* __restrict__ found_inf, unsigned long long* __restrict__ sync, float lr, float momentum,
                        float dampening, float wd, int nesterov, int maximize, float growth, float backoff,
                        int interval, xgmi::XSite xg, int* __restrict__ err, long long barrier_ticks, opt::SlabSet ss,
                        int grid_amp) {
  const int bid = (int)blockIdx.x;
  DPA_STAMP(0);
  if (bid < nw1) {
    constexpr int ns = (28 + WG1_ROWS_ - 1) / WG1_ROWS_;
    cb::conv5x5_wgrad_body<T, 1, 16, 28, 28, WG1_ROWS_, 2, true>(x, nullptr, wslab1, ns, bi, bid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's row has left the CU
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(w1cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    DPA_STAMP(8);
    return;
  }
  opt::amp_sgd_body<CAS_U, XG>(L, scale, tracker, found_inf, sync, lr, momentum, dampening, wd, nesterov, maximize,
                               growth, backoff, interval, xg, err, barrier_ticks, ss, grid_amp, bid - nw1);
}

// Launch shape of convnet_amp_step at batch B: (producers, AMP workgroups).
static std::pair<int, int> cas_shape(int64_t B, int64_t n_params_granules) {
  const int nw1 = (int)wgrad_bn_rows(1, B);
  const int nreg = (int)std::max<int64_t>(1, (n_params_granules + opt::FUSED_THR * CAS_U - 1) / (opt::FUSED_THR * CAS_U));
  const int s0 = 1, s1 = (16 * 25 + 16 + 15) / 16, s2 = (32 * 400 + 32 + 63) / 64;
  return {nw1, nreg + s0 + s1 + s2};
}

// The AMP workgroups of the launch are co-resident (they meet at a grid barrier) and the
// producers of one XCD fit beside them once they are done.
bool convnet_amp_step_ok(int64_t B, int64_t n_params_granules, at::ScalarType st) {
  const auto sh = cas_shape(B, n_params_granules);
  bool ok = true;
  with_t(dt_of(at::empty({0}, at::TensorOptions().dtype(st))), [&](auto tag) {
    typedef decltype(tag) T;
    if constexpr (std::is_same<T, float>::value) {
      ok = false;  // fp32: no scaler in the reference path; the separate launches stay
    } else {
      ok = co_resident(reinterpret_cast<const void*>(&convnet_amp_step_kernel<T, false>), sh.second, cb::NTHR, 0) &&
           co_resident(reinterpret_cast<const void*>(&convnet_amp_step_kernel<T, true>), sh.second, cb::NTHR, 0) &&
           co_resident(reinterpret_cast<const void*>(&convnet_amp_step_kernel<T, false>), sh.first, cb::NTHR, 0);
    }
  });
  // with the xGMI engine both the conv1 BN site (sh.first workgroups) and the gradient
  // site (sh.second) ride this launch: each must fit its epoch words (comm/xgmi.h)
  return ok && xgmi::site_grid_fits(sh.first) && xgmi::site_grid_fits(sh.second);
}

// params / grads / bufs / first / lr ... sync / xc: as optim.amp_sgd_fused (one param group).
// conv1: x (batch images), y1, dp1, idx1, fstats1, gsum1 (BN1 backward sum rows; all-reduced
// under a host SyncBN), g1, eps1 -> wslab1 (partial rows), w1cnt (int32, zeroed once),
// out1 = [dW1 | db1]; bn1: the BN1 sum rows of this rank ([S1 | S2] per row) -> out0 =
// [dbeta1 | dgamma1]; conv2: wslab2 -> out2 = [dW2 | db2].
void convnet_amp_step(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> bufs,
                      double lr, double momentum, double dampening, double wd, bool nesterov, bool maximize,
                      std::vector<int64_t> first, at::Tensor scale, at::Tensor tracker, at::Tensor found_inf,
                      double growth, double backoff, int64_t interval, at::Tensor sync, XcPtr xc, at::Tensor x,
                      at::Tensor y1, at::Tensor dp1, at::Tensor idx1, at::Tensor fstats1, at::Tensor gsum1,
                      at::Tensor g1, double eps1, at::Tensor wslab1, at::Tensor w1cnt, at::Tensor out1, at::Tensor bn1,
                      at::Tensor out0, at::Tensor wslab2, at::Tensor out2) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(y1); DPA_CHECK_INPUT(wslab1); DPA_CHECK_INPUT(wslab2); DPA_CHECK_INPUT(w1cnt);
  const int B = (int)y1.size(0);
  TORCH_CHECK(x.size(1) == 1 && y1.size(1) == 16 && y1.size(2) == 28 && x.scalar_type() == y1.scalar_type());
  TORCH_CHECK(w1cnt.scalar_type() == at::kInt && w1cnt.numel() >= 1, "convnet_amp_step: w1cnt int32[1]");
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kLong && sync.is_contiguous(),
              "convnet_amp_step: sync must be a zero-initialised int64 device tensor");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && found_inf.scalar_type() == at::kFloat &&
              tracker.scalar_type() == at::kInt);
  constexpr int N1 = 16 * 25 + 16, N2 = 32 * 400 + 32;
  const int nw1 = (int)wgrad_bn_rows(1, B);
  TORCH_CHECK(wslab1.numel() == (int64_t)nw1 * N1 && out1.numel() == N1, "convnet_amp_step: conv1 slab sizes");
  TORCH_CHECK(wslab2.numel() == wgrad_bn_rows(2, B) * N2 && out2.numel() == N2, "convnet_amp_step: conv2 slab sizes");
  TORCH_CHECK(out0.numel() == 32 && bn1.numel() % 32 == 0, "convnet_amp_step: BN1 sum rows [rows][32] -> 32");
  if (B == 0) return;
  opt::MTList L = opt::fused_list(params, grads, bufs, first, momentum);
  opt::SlabSet ss;
  // the flush path's associations (bitwise the same gradients): BN1 sums as cb::colsum_rows
  // (2C = 32 columns, G = 8), the weight-gradient slabs as slab_reduce (G = 16)
  opt::add_slab(ss, L, bn1, out0, 8, 1, nullptr, 0);
  opt::add_slab(ss, L, wslab1, out1, 16, 1, w1cnt.data_ptr<int>(), nw1);
  opt::add_slab(ss, L, wslab2, out2, 16, 4, nullptr, 0);
  ss.rearm = w1cnt.data_ptr<int>();
  ss.blanes = 8;  // ~240 arriving workgroups: arrivals spread over 8 words
  TORCH_CHECK(sync.numel() >= 1 + 2 * ss.blanes * opt::kBarStride, "convnet_amp_step: sync must hold ",
              1 + 2 * ss.blanes * opt::kBarStride, " int64");
  const auto sh = cas_shape(B, L.chunk_off[L.n]);
  int nslab = 0;
  for (int s = 0; s < ss.ns; ++s) nslab += ss.s[s].nblk;
  const int nreg = (int)std::max<int64_t>(1, (L.chunk_off[L.n] + opt::FUSED_THR * CAS_U - 1) / (opt::FUSED_THR * CAS_U));
  const int grid_amp = nreg + nslab;
  TORCH_CHECK(grid_amp == sh.second && nw1 == sh.first, "convnet_amp_step: launch shape");
  constexpr double kBarrierSeconds = 10.0;
  with_t(dt_of(y1), [&](auto tag) {
    typedef decltype(tag) T;
    if constexpr (std::is_same<T, float>::value) {
      TORCH_CHECK(false, "convnet_amp_step: bf16 / fp16 only");
    } else {
      // producers: BN1 backward from the rows, no dgamma / dbeta (the BN1 slab source owns them)
      BwdIn<T> bi = bwd_in<T>(dp1, idx1, y1, fstats1, gsum1, c10::nullopt, g1, eps1, 16, c10::nullopt,
                              c10::nullopt);
      if (xc) {
        bi.xs = site_of(xc, xgmi::kSiteBwd1);
        xgmi::set_site_grid(bi.xs, nw1, "convnet_amp_step conv1 weight gradient");
      }
      xgmi::XSite xg;
      if (xc) {
        xg = xc->grad_site();
        TORCH_CHECK(L.chunk_off[L.n] * 4 <= xg.max_vals, "convnet_amp_step: too many elements for the xGMI engine");
        xgmi::set_site_grid(xg, grid_amp, "convnet_amp_step");
      }
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(nw1 + grid_amp), dim3(cb::NTHR), 0, cur_stream(), dptr<T>(x),
                           wslab1.data_ptr<float>(), bi, nw1, w1cnt.data_ptr<int>(), L, scale.data_ptr<float>(),
                           tracker.data_ptr<int>(), found_inf.data_ptr<float>(),
                           reinterpret_cast<unsigned long long*>(sync.data_ptr<int64_t>()), (float)lr,
                           (float)momentum, (float)dampening, (float)wd, (int)nesterov, (int)maximize, (float)growth,
                           (float)backoff, (int)interval, xg,
                           reinterpret_cast<int*>(sync.data_ptr<int64_t>() + sync.numel() - 1),
                           (long long)(kBarrierSeconds * 1e8), ss, grid_amp);
      };
      if (xc) go(convnet_amp_step_kernel<T, true>);
      else go(convnet_amp_step_kernel<T, false>);
    }
  });
  DPA_CHECK_LAUNCH();
}

// Whether every launch that exchanges SyncBN sums in-kernel (comm/xsite.h: all
// of its workgroups poll the peers' rows) is co-resident at batch B; if not,
// ops/convnet_fused.py all-reduces between the launches instead.
bool sites_resident(int64_t B, at::ScalarType st) {
  // every site launch must also fit its site's epoch words (comm/xgmi.h set_site_grid):
  // the conv1 weight gradient's 7 B workgroups pass kEpochWords at B >= 74
  bool ok = xgmi::site_grid_fits(wgrad_bn_rows(1, B)) && xgmi::site_grid_fits(wgrad_bn_rows(2, B)) &&
            xgmi::site_grid_fits(B * dgrad_split(st == at::kFloat)) &&
            xgmi::site_grid_fits(fwd2_split(st == at::kFloat) * B);
  auto chk = [&](const void* k, int64_t grid) { ok = ok && co_resident(k, (int)grid, cb::NTHR, 0); };
  with_t(dt_of(at::empty({0}, at::TensorOptions().dtype(st))), [&](auto tag) {
    typedef decltype(tag) T;
    chk(reinterpret_cast<const void*>(&cb::conv5x5_kernel<T, 16, 32, 14, 14, 0, 1, 0, 1>),
        B * fwd2_split(std::is_same<T, float>::value));
    ok = ok && co_resident(reinterpret_cast<const void*>(&head_fwd_kernel<T, 32, 14, 14, 16>), (int)B, HF, 0) &&
         co_resident(reinterpret_cast<const void*>(&head_fwd_kernel<T, 32, 14, 14, 64>), (int)B, HF, 0);
    chk(reinterpret_cast<const void*>(&cb::conv5x5_kernel<T, 32, 16, 14, 14, 2, 2, 1, 1>), B * kDgradSplitT<T>);
    if constexpr (!std::is_same<T, float>::value) {
      if (lp_dyn_bwd())
        ok = ok && co_resident(reinterpret_cast<const void*>(&conv2_bwd_dyn_kernel<T>),
                               (int)(B * kDgradSplitT<T> + wgrad_bn_rows(2, B) + FC_BLOCKS), cb::NTHR,
                               conv2_bwd_dyn_bytes<T>());
      else
        chk(reinterpret_cast<const void*>(&conv2_bwd_kernel<T>), B * kDgradSplitT<T> + wgrad_bn_rows(2, B) + FC_BLOCKS);
    } else if (fp32_merged_bwd())
      ok = ok && co_resident(reinterpret_cast<const void*>(&conv2_bwd_dyn_kernel<T>),
                             (int)(B * kDgradSplitT<T> + wgrad_bn_rows(2, B) + FC_BLOCKS), cb::NTHR,
                             conv2_bwd_dyn_bytes<T>());
    chk(reinterpret_cast<const void*>(&cb::conv5x5_wgrad_kernel<T, 16, 32, 14, 14, WG2_ROWS, 2>),
        wgrad_bn_rows(2, B));
    chk(reinterpret_cast<const void*>(&cb::conv5x5_wgrad_kernel<T, 1, 16, 28, 28, WG1_ROWS, 2>),
        wgrad_bn_rows(1, B));
    chk(reinterpret_cast<const void*>(&wgrad1_reduce_kernel<T>), wgrad_bn_rows(1, B));
    chk(reinterpret_cast<const void*>(&wgrad1_slab2_kernel<T>), wgrad_bn_rows(1, B));
  });
  return ok;
}

}  // namespace cnf

void register_convnet_fused(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("convnet", "whole-ConvNet fused kernels");
  s.def("conv2_fwd", &cnf::conv2_fwd);
  s.def("head_fwd", &cnf::head_fwd);
  s.def("head_bwd", &cnf::head_bwd);
  s.def("head_bwd_lds", &cnf::head_bwd_lds);
  s.def("dgrad2_rows", &cnf::dgrad2_rows, py::arg("B"), py::arg("fp32") = false);
  s.def("conv1_fwd_pack", &cnf::conv1_fwd_pack);
  s.def("conv1_fwd_pack_gather", &cnf::conv1_fwd_pack_gather);
#ifdef DPA_TIMING
  s.def("read_stamps", []() {
    auto out = at::empty({DPA_MAX_STAMP_BLOCKS, DPA_NSTAMPS}, at::TensorOptions().dtype(at::kLong));
    DPA_CHECK_HIP(hipDeviceSynchronize());
    DPA_CHECK_HIP(hipMemcpyFromSymbol(out.data_ptr(), HIP_SYMBOL(dpa_stamps), sizeof(unsigned long long) *
                                      DPA_MAX_STAMP_BLOCKS * DPA_NSTAMPS));
    return out;
  });
  s.def("clear_stamps", []() {
    DPA_CHECK_HIP(hipDeviceSynchronize());
    std::vector<unsigned long long> z(DPA_MAX_STAMP_BLOCKS * DPA_NSTAMPS, 0ull);
    DPA_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dpa_stamps), z.data(), z.size() * sizeof(unsigned long long)));
  });
#endif
  s.attr("W2F_LEN") = cb::W2F_LEN;
  s.attr("W2D_LEN") = cb::W2D_LEN;
  s.def("conv2_dgrad", &cnf::conv2_dgrad);
  s.def("conv2_bwd", &cnf::conv2_bwd);
  s.def("fc_wgrad", &cnf::fc_wgrad);
  s.def("conv_wgrad_bn", &cnf::conv_wgrad_bn);
  s.def("wgrad_bn_rows", &cnf::wgrad_bn_rows);
  s.def("sites_resident", &cnf::sites_resident);
  s.def("fwd2_split", &cnf::fwd2_split, py::arg("fp32"));
  s.def("wgrad1_reduce", &cnf::wgrad1_reduce);
  s.def("conv1_wgrad_slab2", &cnf::conv1_wgrad_slab2);
  s.def("convnet_amp_step", &cnf::convnet_amp_step);
  s.def("convnet_amp_step_ok", &cnf::convnet_amp_step_ok);
  s.def("wgrad1_counters", &cnf::wgrad1_counters);
}

}  // namespace dpa
