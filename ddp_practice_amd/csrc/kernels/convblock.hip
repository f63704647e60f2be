// Fused "conv block" kernels for the ConvNet hot path:
//     Conv2d(CIN->COUT, 5x5, stride 1, pad 2) -> BatchNorm2d -> ReLU -> MaxPool2d(2,2)
// (reference: /root/reference/origin_main.py:12-23, ddp_main.py:16-27).
//
// Forward (train):  [conv_fwd: implicit-GEMM MFMA + bias + BN partial stats]
//                   -> (optional SyncBN all-reduce of the 2C+1 stats, host side)
//                   -> [bn_relu_pool: finalize stats, running-stat update,
//                       normalise, ReLU, 2x2 max-pool, argmax index]
// Backward:         [bwd_reduce: pool/ReLU routing + per-channel sum(dy), sum(dy*xhat)]
//                   -> (optional SyncBN all-reduce of 2C sums)
//                   -> [bwd_elemt: BN input-grad at full resolution]
//                   -> [conv_wgrad: MFMA, split over images, f32 atomics into dW, db]
//                   -> [conv_fwd<DGRAD>: input grad = conv of dy with flipped W^T]
//
// Design notes (MI355X):
//  * Everything here is latency-bound (per-step GEMMs are 20-160 MFLOP), so the
//    goal is few launches, one LDS round trip per operand, and enough
//    workgroups (B x splits >= 64) to spread over XCDs.
//  * im2col never touches HBM: the input image (with halo) sits in LDS in
//    HWC order so that 8 K-consecutive elements (8 input channels of one tap)
//    are one 16-B ds_read; conv1 (CIN=1) gathers its 25 taps element-wise.
//  * wgrad keeps 5 kw-shifted copies of the input in LDS so that the B operand
//    (8 consecutive output columns of one tap) is again one aligned 16-B read.
//  * BN statistics are accumulated around a per-channel shift (the running
//    mean, identical on every rank) to avoid E[x^2]-E[x]^2 cancellation; the
//    sums are plain sums, so SyncBN needs one all-reduce of 2C+1 floats and
//    no device->host mask sync (cf. torch/nn/modules/_functions.py:74-101).
#include "common.h"

namespace dpa {
namespace cb {

constexpr int NTHR = 256;

// stats buffer layout (floats): [0,C) sum(y-shift) | [C,2C) sum((y-shift)^2) |
// [2C] count | [2C+1, 3C+1) shift copy.  First 2C+1 entries are all-reduced.
__host__ __device__ constexpr int stats_len(int C) { return 3 * C + 1; }

// ---------------------------------------------------------------------------
// Implicit-GEMM 5x5 convolution, one (image, m-range) per workgroup.
//   MODE 0: forward + bias + BN partial stats      (train)
//   MODE 1: forward + bias                         (eval / no BN stats)
//   MODE 2: data-grad: input = dy (CIN = COUT_orig), output = dx,
//           W_eff[co][ci][kh][kw] = W[ci][co][4-kh][4-kw], no bias
// GEMM view: rows = output pixels of one image, cols = output channels,
// K = 25*CIN ordered (kh, kw, ci) with ci fastest.
// ---------------------------------------------------------------------------
template <typename T, int CIN, int COUT, int H, int W, int MODE>
__global__ void __launch_bounds__(NTHR)
conv5x5_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
               T* __restrict__ y, float* __restrict__ stats, const float* __restrict__ shift,
               int nsplit) {
  static_assert(CIN == 1 || CIN % 8 == 0, "CIN must be 1 or a multiple of 8");
  static_assert(COUT % 16 == 0, "COUT must be a multiple of 16");
  static_assert((H * W) % 4 == 0, "H*W must be a multiple of 4");
  constexpr int HP = H + 4, WPD = W + 4;
  constexpr int K = 25 * CIN;
  constexpr int KP = ceil_to(K, 32);
  constexpr int KS = KP / 32;
  constexpr int KPW = KP + 8;  // LDS row pitch of the weight tile (breaks bank aliasing)
  constexpr int NT = COUT / 16;
  constexpr int HW = H * W;
  constexpr int MT = (HW + 15) / 16;
  typedef MM<T> mm;

  __shared__ __attribute__((aligned(16))) T img[HP * WPD * CIN];
  __shared__ __attribute__((aligned(16))) T wl[COUT * KPW];
  __shared__ float lstat[2 * COUT];

  const int tid = threadIdx.x;
  const int b = blockIdx.x / nsplit;
  const int sp = blockIdx.x % nsplit;
  const T* xb = x + (size_t)b * CIN * HW;

  // --- stage weights: wl[co][k], k = (kh*5+kw)*CIN + ci, zero for k >= K
  for (int e = tid; e < COUT * KP; e += NTHR) {
    const int co = e / KP, k = e % KP;
    float v = 0.f;
    if (k < K) {
      const int tap = k / CIN, ci = k % CIN;
      const int kh = tap / 5, kw = tap % 5;
      if (MODE == 2)
        v = w[((ci * COUT + co) * 5 + (4 - kh)) * 5 + (4 - kw)];
      else
        v = w[((co * CIN + ci) * 5 + kh) * 5 + kw];
    }
    wl[co * KPW + k] = Cvt<T>::from_f(v);
  }
  // --- stage the zero-padded image in HWC order
  for (int e = tid; e < HP * WPD * CIN; e += NTHR) img[e] = Cvt<T>::from_f(0.f);
  if (MODE == 0 && tid < 2 * COUT) lstat[tid] = 0.f;
  __syncthreads();
  for (int e = tid; e < CIN * HW; e += NTHR) {
    const int ci = e / HW, pix = e % HW;
    const int h = pix / W, ww = pix % W;
    img[((h + 2) * WPD + (ww + 2)) * CIN + ci] = xb[e];
  }
  __syncthreads();

  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int mt0 = (MT * sp) / nsplit, mt1 = (MT * (sp + 1)) / nsplit;

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
        a = mm::ld(&img[((oh + tap / 5) * WPD + ow + tap % 5) * CIN + ci0]);
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
        const float bs = (MODE == 2) ? 0.f : bias[co];
        T* dst = y + ((size_t)b * COUT + co) * HW + pix0;
        const float sh = (MODE == 0) ? shift[co] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[nt][i] + bs;
          dst[i] = Cvt<T>::from_f(v);
          if (MODE == 0) {
            const float d = rnd_t<T>(v) - sh;
            s1[nt] += d;
            s2[nt] += d * d;
          }
        }
      }
    }
  }
  if constexpr (MODE == 0) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float a1 = s1[nt], a2 = s2[nt];
      a1 += __shfl_xor(a1, 16, 64);
      a1 += __shfl_xor(a1, 32, 64);
      a2 += __shfl_xor(a2, 16, 64);
      a2 += __shfl_xor(a2, 32, 64);
      if (q == 0) {
        atomicAdd(&lstat[nt * 16 + r], a1);
        atomicAdd(&lstat[COUT + nt * 16 + r], a2);
      }
    }
    __syncthreads();
    if (tid < 2 * COUT) atomicAdd(&stats[tid], lstat[tid]);
    if (blockIdx.x == 0) {
      if (tid < COUT) stats[2 * COUT + 1 + tid] = shift[tid];
    }
    if (sp == 0 && tid == 0) atomicAdd(&stats[2 * COUT], (float)HW);
  }
}

// ---------------------------------------------------------------------------
// BN finalize + normalise + ReLU + 2x2/2 max-pool (+ argmax index, first max
// wins in (dy,dx) scan order as ATen's max_pool2d).  One thread per pooled
// output.  Block 0 updates running stats (momentum<0 => cumulative average).
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bn_relu_pool_kernel(const T* __restrict__ y, const float* __restrict__ stats,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
                    float momentum, float eps, int train, T* __restrict__ p,
                    uint8_t* __restrict__ idx, int total) {
  constexpr int HO = H / 2, WO = W / 2;
  const int e = blockIdx.x * NTHR + threadIdx.x;
  if (train && blockIdx.x == 0 && threadIdx.x < C) {
    const int c = threadIdx.x;
    const float n = stats[2 * C];
    const float m1 = stats[c] / n;
    const float mean = stats[2 * C + 1 + c] + m1;
    const float var = fmaxf(stats[C + c] / n - m1 * m1, 0.f);
    const int64_t nb = nbt[0] + 1;
    const float mom = momentum >= 0.f ? momentum : 1.f / (float)nb;
    rmean[c] = (1.f - mom) * rmean[c] + mom * mean;
    rvar[c] = (1.f - mom) * rvar[c] + mom * var * (n / fmaxf(n - 1.f, 1.f));
    if (c == 0) nbt[0] = nb;
  }
  if (e >= total) return;
  const int c = (e / (HO * WO)) % C;
  float mean, invstd;
  if (train) {
    const float n = stats[2 * C];
    const float m1 = stats[c] / n;
    mean = stats[2 * C + 1 + c] + m1;
    invstd = rsqrtf(fmaxf(stats[C + c] / n - m1 * m1, 0.f) + eps);
  } else {
    mean = rmean[c];
    invstd = rsqrtf(rvar[c] + eps);
  }
  const float sc = gamma[c] * invstd;
  const float sh = beta[c] - mean * sc;
  const int bc = e / (HO * WO), pix = e % (HO * WO);
  const int ho = pix / WO, wo = pix % WO;
  const T* src = y + (size_t)bc * H * W + (2 * ho) * W + 2 * wo;
  float best = -1.f;
  int bi = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = Cvt<T>::to_f(src[(k >> 1) * W + (k & 1)]);
    const float z = fmaxf(rnd_t<T>(v * sc + sh), 0.f);
    if (z > best) { best = z; bi = k; }
  }
  p[e] = Cvt<T>::from_f(best);
  idx[e] = (uint8_t)bi;
}

// mean / invstd of channel c from a (possibly all-reduced) stats buffer.
template <int C>
__device__ __forceinline__ void stats_mean_invstd(const float* stats, int c, float eps, float& mean,
                                                  float& invstd, float& n) {
  n = stats[2 * C];
  const float m1 = stats[c] / n;
  mean = stats[2 * C + 1 + c] + m1;
  invstd = rsqrtf(fmaxf(stats[C + c] / n - m1 * m1, 0.f) + eps);
}

// ---------------------------------------------------------------------------
// Backward part 1: route the pooled grad through max-pool (argmax) and ReLU
// (pooled output > 0), and reduce per channel
//   sums[c]     += sum dy          (= grad of BN bias)
//   sums[C + c] += sum dy * xhat   (= grad of BN weight)
// grid = (C, nsplit over the batch).
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bwd_reduce_kernel(const T* __restrict__ dp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                  const T* __restrict__ y, const float* __restrict__ stats, float eps,
                  float* __restrict__ sums, int B) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  __shared__ float red[2 * NTHR / 64];
  const int c = blockIdx.x;
  const int nsplit = gridDim.y;
  const int b0 = (B * blockIdx.y) / nsplit, b1 = (B * (blockIdx.y + 1)) / nsplit;
  float mean, invstd, n;
  stats_mean_invstd<C>(stats, c, eps, mean, invstd, n);
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
    atomicAdd(&sums[c], t1);
    atomicAdd(&sums[C + c], t2);
  }
}

// ---------------------------------------------------------------------------
// Backward part 2: BN input gradient at full resolution, one thread per
// pooled element (its 2x2 window):
//   dx = gamma*invstd*(dy - S1/n - xhat*S2/n),  dy = routed pooled grad or 0
// ---------------------------------------------------------------------------
template <typename T, int C, int H, int W>
__global__ void __launch_bounds__(NTHR)
bwd_elemt_kernel(const T* __restrict__ dp, const T* __restrict__ p, const uint8_t* __restrict__ idx,
                 const T* __restrict__ y, const float* __restrict__ stats,
                 const float* __restrict__ gsums, const float* __restrict__ gamma, float eps,
                 T* __restrict__ dx, int total) {
  constexpr int HO = H / 2, WO = W / 2, PP = HO * WO;
  const int e = blockIdx.x * NTHR + threadIdx.x;
  if (e >= total) return;
  const int bc = e / PP, pix = e % PP;
  const int c = bc % C;
  float mean, invstd, n;
  stats_mean_invstd<C>(stats, c, eps, mean, invstd, n);
  const float k1 = gsums[c] / n, k2 = gsums[C + c] / n;
  const float gi = gamma[c] * invstd;
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
// Weight/bias gradient of the 5x5 conv.  One workgroup per (image, row-chunk).
// GEMM: rows = COUT, cols = (ci, kh, kw) natural order, K = pixels of the chunk
// with the row padded to WP = ceil8(W) (dy is zero in the pad columns).
// LDS: dy[COUT][ROWS][WP] and 5 kw-shifted copies xs[kw][CIN][ROWS+4][WP] of
// the zero-padded input so both operands are aligned 16-B LDS reads.
// Partial sums go to dW/db with f32 atomics (buffers zeroed by the caller).
// ---------------------------------------------------------------------------
template <typename T, int CIN, int COUT, int H, int W, int ROWS>
__global__ void __launch_bounds__(NTHR)
conv5x5_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy, float* __restrict__ dw,
                     float* __restrict__ db, int nsplit) {
  constexpr int WP = ceil_to(W, 8);
  static_assert((ROWS * WP) % 32 == 0, "ROWS*WP must be a multiple of 32");
  constexpr int KSTEPS = ROWS * WP / 32;
  constexpr int N = CIN * 25;
  constexpr int NTL = (N + 15) / 16;
  constexpr int MTL = COUT / 16;
  constexpr int XR = ROWS + 4;
  typedef MM<T> mm;
  __shared__ __attribute__((aligned(16))) T dyl[COUT * ROWS * WP];
  __shared__ __attribute__((aligned(16))) T xs[5 * CIN * XR * WP];

  const int tid = threadIdx.x;
  const int b = blockIdx.x / nsplit, sp = blockIdx.x % nsplit;
  const int r0 = sp * ROWS;
  const T* xb = x + (size_t)b * CIN * H * W;
  const T* dyb = dy + (size_t)b * COUT * H * W;

  for (int e = tid; e < COUT * ROWS * WP; e += NTHR) {
    const int co = e / (ROWS * WP), rem = e % (ROWS * WP);
    const int rr = rem / WP, cc = rem % WP;
    const int row = r0 + rr;
    dyl[e] = (row < H && cc < W) ? dyb[(co * H + row) * W + cc] : Cvt<T>::from_f(0.f);
  }
  for (int e = tid; e < 5 * CIN * XR * WP; e += NTHR) {
    const int kw = e / (CIN * XR * WP);
    int rem = e % (CIN * XR * WP);
    const int ci = rem / (XR * WP);
    rem %= XR * WP;
    const int rr = rem / WP, cc = rem % WP;
    const int ih = r0 + rr - 2, iw = cc + kw - 2;
    xs[e] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xb[(ci * H + ih) * W + iw]
                                                     : Cvt<T>::from_f(0.f);
  }
  __syncthreads();

  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  // bias grad: per output channel sum of dy over this chunk
  for (int co = wv; co < COUT; co += NTHR / 64) {
    float a = 0.f;
    for (int i = lane; i < ROWS * WP; i += 64) a += Cvt<T>::to_f(dyl[co * ROWS * WP + i]);
    a = wave_sum(a);
    if (lane == 0) atomicAdd(&db[co], a);
  }
  for (int pr = wv; pr < MTL * NTL; pr += NTHR / 64) {
    const int mt = pr / NTL, nt = pr % NTL;
    int n = nt * 16 + r;
    const bool nvalid = n < N;
    n = nvalid ? n : 0;
    const int ci = n / 25, kh = (n % 25) / 5, kw = n % 5;
    const T* brow = &xs[((kw * CIN + ci) * XR + kh) * WP];
    const T* arow = &dyl[(mt * 16 + r) * ROWS * WP];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int P = 32 * s + 8 * q;  // pixel index within the chunk
      const int row = P / WP, col0 = P % WP;
      const typename mm::frag a = mm::ld(arow + P);
      const typename mm::frag bf = mm::ld(brow + row * WP + col0);
      acc = mm::mma(a, bf, acc);
    }
    // D[row = 4q+i][col = r]: dW[co = mt*16+4q+i][n]
    const int col = nt * 16 + r;
    if (col < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(&dw[(mt * 16 + 4 * q + i) * N + col], acc[i]);
    }
  }
}

// ===========================================================================
// Host side
// ===========================================================================
struct Shape {
  int cin, cout, h, w;
  bool operator==(const Shape& o) const {
    return cin == o.cin && cout == o.cout && h == o.h && w == o.w;
  }
};

// Compile-time instantiations (the ConvNet blocks).  Other shapes are routed
// to the generic layer kernels by the Python side.
static const Shape kShapes[] = {{1, 16, 28, 28}, {16, 32, 14, 14}};

// Call f(std::integral_constant<int, i>) for the instantiated shape index that
// matches (cin, cout, h, w); returns false if none does.
template <typename F>
static bool with_shape(const Shape& s, F&& f) {
  if (s == kShapes[0]) { f(std::integral_constant<int, 0>{}); return true; }
  if (s == kShapes[1]) { f(std::integral_constant<int, 1>{}); return true; }
  return false;
}
template <int I> struct SH;
template <> struct SH<0> { static constexpr int CIN = 1, COUT = 16, H = 28, W = 28, SPLIT = 4, WROWS = 7; };
template <> struct SH<1> { static constexpr int CIN = 16, COUT = 32, H = 14, W = 14, SPLIT = 2, WROWS = 14; };

template <typename F>
static void with_t(DT dt, F&& f) {
  switch (dt) {
    case DT::F32: f(float{}); break;
    case DT::BF16: f(__hip_bfloat16{}); break;
    case DT::F16: f(__half{}); break;
  }
}

bool supported(int cin, int cout, int h, int w) {
  return with_shape(Shape{cin, cout, h, w}, [](auto) {});
}

static Shape shape_of(const at::Tensor& x, const at::Tensor& w) {
  return Shape{(int)x.size(1), (int)w.size(0), (int)x.size(2), (int)x.size(3)};
}

// Forward conv (+bias) [+ BN partial stats into `stats` (zeroed, len 3C+1)].
void conv_fwd(at::Tensor x, at::Tensor w, at::Tensor bias, at::Tensor y, c10::optional<at::Tensor> stats,
              c10::optional<at::Tensor> shift) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(bias); DPA_CHECK_INPUT(y);
  TORCH_CHECK(w.scalar_type() == at::kFloat && bias.scalar_type() == at::kFloat);
  TORCH_CHECK(y.scalar_type() == x.scalar_type());
  const Shape s = shape_of(x, w);
  TORCH_CHECK(w.size(1) == s.cin && w.size(2) == 5 && w.size(3) == 5, "weight must be [COUT][CIN][5][5]");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == s.cout && y.size(2) == s.h && y.size(3) == s.w);
  const int B = (int)x.size(0);
  const bool st = stats.has_value();
  if (st) {
    DPA_CHECK_INPUT((*stats)); DPA_CHECK_INPUT((*shift));
    TORCH_CHECK(stats->numel() == stats_len(s.cout) && shift->numel() == s.cout);
  }
  if (B == 0) return;
  hipStream_t stream = cur_stream();
  const bool ok = with_shape(s, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    const dim3 grid(B * S::SPLIT), blk(NTHR);
    with_t(dt_of(x), [&](auto tag) {
      typedef decltype(tag) T;
      if (st)
        hipLaunchKernelGGL((conv5x5_kernel<T, S::CIN, S::COUT, S::H, S::W, 0>), grid, blk, 0, stream, dptr<T>(x),
                           w.data_ptr<float>(), bias.data_ptr<float>(), dptr<T>(y), stats->data_ptr<float>(),
                           shift->data_ptr<float>(), S::SPLIT);
      else
        hipLaunchKernelGGL((conv5x5_kernel<T, S::CIN, S::COUT, S::H, S::W, 1>), grid, blk, 0, stream, dptr<T>(x),
                           w.data_ptr<float>(), bias.data_ptr<float>(), dptr<T>(y), nullptr, nullptr, S::SPLIT);
    });
  });
  TORCH_CHECK(ok, "conv block shape not instantiated");
  DPA_CHECK_LAUNCH();
}

// Data gradient: dx[B][CIN][H][W] from dy[B][COUT][H][W] and w[COUT][CIN][5][5].
void conv_dgrad(at::Tensor dy, at::Tensor w, at::Tensor dx) {
  DPA_CHECK_INPUT(dy); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(dx);
  const int cout = (int)w.size(0), cin = (int)w.size(1);
  const int H = (int)dy.size(2), W = (int)dy.size(3);
  TORCH_CHECK(dy.size(1) == cout && dx.size(1) == cin && dx.scalar_type() == dy.scalar_type());
  const int B = (int)dy.size(0);
  const bool ok = (cin == 16 && cout == 32 && H == 14 && W == 14);
  TORCH_CHECK(ok, "dgrad shape not instantiated: ", cout, "->", cin, " ", H, "x", W);
  if (B == 0) return;
  constexpr int ns = 2;
  hipStream_t stream = cur_stream();
  with_t(dt_of(dy), [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((conv5x5_kernel<T, 32, 16, 14, 14, 2>), dim3(B * ns), dim3(NTHR), 0, stream, dptr<T>(dy),
                       w.data_ptr<float>(), nullptr, dptr<T>(dx), nullptr, nullptr, ns);
  });
  DPA_CHECK_LAUNCH();
}

// The per-channel kernels only depend on (C, H, W); find the instantiation.
template <typename F>
static bool with_chw(int C, int H, int W, F&& f) {
  if (C == 16 && H == 28 && W == 28) { f(std::integral_constant<int, 0>{}); return true; }
  if (C == 32 && H == 14 && W == 14) { f(std::integral_constant<int, 1>{}); return true; }
  return false;
}

void bn_relu_pool(at::Tensor y, at::Tensor stats, at::Tensor gamma, at::Tensor beta, at::Tensor rmean,
                  at::Tensor rvar, at::Tensor nbt, double momentum, double eps, bool train, at::Tensor p,
                  at::Tensor idx) {
  DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(p); DPA_CHECK_INPUT(idx);
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  TORCH_CHECK(idx.scalar_type() == at::kByte && p.scalar_type() == y.scalar_type());
  TORCH_CHECK(nbt.scalar_type() == at::kLong);
  const int total = B * C * (H / 2) * (W / 2);
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (total == 0) return;
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bn_relu_pool_kernel<T, S::COUT, S::H, S::W>), dim3((total + NTHR - 1) / NTHR), dim3(NTHR), 0,
                         stream, dptr<T>(y), stats.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                         rmean.data_ptr<float>(), rvar.data_ptr<float>(), nbt.data_ptr<int64_t>(), (float)momentum,
                         (float)eps, (int)train, dptr<T>(p), idx.data_ptr<uint8_t>(), total);
    });
  });
  TORCH_CHECK(ok, "bn_relu_pool shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void bwd_reduce(at::Tensor dp, at::Tensor p, at::Tensor idx, at::Tensor y, at::Tensor stats, double eps,
                at::Tensor sums) {
  DPA_CHECK_INPUT(dp); DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(sums);
  TORCH_CHECK(dp.scalar_type() == y.scalar_type() && p.scalar_type() == y.scalar_type());
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (B == 0) return;
    const int nsplit = B >= 8 ? 8 : B;
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bwd_reduce_kernel<T, S::COUT, S::H, S::W>), dim3(C, nsplit), dim3(NTHR), 0, stream,
                         dptr<T>(dp), dptr<T>(p), idx.data_ptr<uint8_t>(), dptr<T>(y), stats.data_ptr<float>(),
                         (float)eps, sums.data_ptr<float>(), B);
    });
  });
  TORCH_CHECK(ok, "bwd_reduce shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void bwd_elemt(at::Tensor dp, at::Tensor p, at::Tensor idx, at::Tensor y, at::Tensor stats, at::Tensor gsums,
               at::Tensor gamma, double eps, at::Tensor dx) {
  DPA_CHECK_INPUT(dp); DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(dx);
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  const int total = B * C * (H / 2) * (W / 2);
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (total == 0) return;
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bwd_elemt_kernel<T, S::COUT, S::H, S::W>), dim3((total + NTHR - 1) / NTHR), dim3(NTHR), 0,
                         stream, dptr<T>(dp), dptr<T>(p), idx.data_ptr<uint8_t>(), dptr<T>(y), stats.data_ptr<float>(),
                         gsums.data_ptr<float>(), gamma.data_ptr<float>(), (float)eps, dptr<T>(dx), total);
    });
  });
  TORCH_CHECK(ok, "bwd_elemt shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void conv_wgrad(at::Tensor x, at::Tensor dy, at::Tensor dw, at::Tensor db) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(dy); DPA_CHECK_INPUT(dw); DPA_CHECK_INPUT(db);
  TORCH_CHECK(dw.scalar_type() == at::kFloat && db.scalar_type() == at::kFloat);
  const int B = (int)x.size(0);
  const Shape s{(int)x.size(1), (int)dy.size(1), (int)x.size(2), (int)x.size(3)};
  hipStream_t stream = cur_stream();
  const bool ok = with_shape(s, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (B == 0) return;
    constexpr int ns = (S::H + S::WROWS - 1) / S::WROWS;
    with_t(dt_of(x), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((conv5x5_wgrad_kernel<T, S::CIN, S::COUT, S::H, S::W, S::WROWS>), dim3(B * ns), dim3(NTHR),
                         0, stream, dptr<T>(x), dptr<T>(dy), dw.data_ptr<float>(), db.data_ptr<float>(), ns);
    });
  });
  TORCH_CHECK(ok, "wgrad shape not instantiated");
  DPA_CHECK_LAUNCH();
}

}  // namespace cb

void register_convblock(pybind11::module& m) {
  auto s = m.def_submodule("convblock", "fused Conv5x5-BN-ReLU-MaxPool block kernels");
  s.def("supported", &cb::supported);
  s.def("stats_len", [](int C) { return cb::stats_len(C); });
  s.def("conv_fwd", &cb::conv_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"),
        pybind11::arg("y"), pybind11::arg("stats") = pybind11::none(), pybind11::arg("shift") = pybind11::none());
  s.def("conv_dgrad", &cb::conv_dgrad);
  s.def("conv_wgrad", &cb::conv_wgrad);
  s.def("bn_relu_pool", &cb::bn_relu_pool);
  s.def("bwd_reduce", &cb::bwd_reduce);
  s.def("bwd_elemt", &cb::bwd_elemt);
}

}  // namespace dpa
