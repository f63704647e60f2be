// Channels-last (NHWC) BatchNorm (+ residual add) (+ ReLU), max-pool 3x3/2 and
// global average pool for the ResNet-50 stress config (BASELINE.json config 5;
// SURVEY.md §7.3 step 8).  Activations are [M = N*H*W][C] rows with C
// contiguous, so one lane moves 16 B = 8 channels of one pixel per access and a
// wave covers whole cache lines.
//
//   forward (train)  stats:  per-channel sum(x - shift), sum((x - shift)^2) over
//                            the rows: per-workgroup partial rows, the LAST
//                            workgroup to finish (device-scope ticket) reduces them
//                            -> stats[2C+1] (+ shift copy); SyncBN all-reduces the
//                            first 2C+1 entries between the launches
//                    apply:  y = relu?((x - mean) * gamma*invstd + beta (+ res));
//                            workgroup 0 updates running stats (momentum, unbiased
//                            var) and saves mean / invstd for the backward
//   backward         stats:  dz = dy * [y > 0] (ReLU) ; sum(dz), sum(dz * xhat)
//                            -> the same ticket reduction; d(gamma), d(beta) from
//                            the local sums (torch SyncBN semantics); all-reduce
//                    elemt:  dx = gamma*invstd * (dz - S1/n - xhat * S2/n),
//                            d(res) = dz when the block had a residual input
// The per-channel statistics are sums around a shift (the running mean, equal
// on every rank) to avoid E[x^2] - E[x]^2 cancellation.  Deterministic: every
// reduction has a fixed order (no float atomics).
#include "common.h"

namespace dpa {
namespace bnh {

constexpr int THR = 256;
constexpr int MAXNV = 2;  // channel vectors per lane when C / VEC > THR (f32, C = 2048)

template <typename T> struct V16 { static constexpr int N = 16 / sizeof(T); };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* f) {
  const f32x4 raw = *reinterpret_cast<const f32x4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int j = 0; j < V16<T>::N; ++j) f[j] = Cvt<T>::to_f(e[j]);
}
template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* f) {
  f32x4 raw;
  T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
  for (int j = 0; j < V16<T>::N; ++j) e[j] = Cvt<T>::from_f(f[j]);
  *reinterpret_cast<f32x4*>(p) = raw;
}

// Lane geometry over a [rows][C] matrix: L = C/VEC vector columns; if L <= THR a
// pass covers RP = THR/L rows, lane -> (row offset, column); else one row per
// pass and each lane owns NV = L/THR columns.
struct Geo {
  int L, RP, roff, nv;
  bool active;
  __device__ Geo(int C, int vec) {
    L = C / vec;
    if (L <= THR) {
      RP = THR / L;
      roff = threadIdx.x / L;
      nv = 1;
      active = roff < RP;
    } else {
      RP = 1;
      roff = 0;
      nv = L / THR;
      active = true;
    }
  }
  __device__ int col(int k) const { return L <= THR ? (int)threadIdx.x % L : (int)threadIdx.x + k * THR; }
};

// Last-workgroup reduction of G partial rows of width W -> out[W] (fixed order).
__device__ __forceinline__ bool ticket_last(unsigned* ticket, int G) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its partial-row stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == (unsigned)G - 1);
    if (s_last) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm for the next launch
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return s_last != 0;
}

// (lo / hi non-null: also lo = out[0, W/2) and hi = out[W/2, W))
__device__ __forceinline__ void reduce_partials(const float* __restrict__ part, int G, int W, float* __restrict__ out,
                                                float* __restrict__ lo = nullptr, float* __restrict__ hi = nullptr) {
  for (int j = threadIdx.x; j < W; j += THR) {
    float acc = 0.f;
    int g = 0;
    for (; g + 8 <= G; g += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(g + u) * W + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; g < G; ++g) acc += part[(size_t)g * W + j];
    out[j] = acc;
    if (lo != nullptr) {
      if (j < W / 2) lo[j] = acc;
      else hi[j - W / 2] = acc;
    }
  }
}

// ----------------------------------------------------------------------------
// forward statistics: stats[0..C) = sum(x-shift), [C..2C) = sum((x-shift)^2),
// [2C] = rows, [2C+1 .. 3C+1) = shift (copied for the apply / backward)
template <typename T>
__global__ void __launch_bounds__(THR)
fwd_stats_kernel(const T* __restrict__ x, long long M, int C, const float* __restrict__ shift,
                 float* __restrict__ part, unsigned* __restrict__ ticket, float* __restrict__ stats) {
  constexpr int VEC = V16<T>::N;
  const Geo g(C, VEC);
  float s1[MAXNV][VEC], s2[MAXNV][VEC], sh[MAXNV][VEC];
  for (int k = 0; k < MAXNV; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) s1[k][j] = s2[k][j] = sh[k][j] = 0.f;
  const long long rows_per = (M + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  if (g.active) {
    for (int k = 0; k < g.nv; ++k)
#pragma unroll
      for (int j = 0; j < VEC; ++j) sh[k][j] = shift[g.col(k) * VEC + j];
    for (long long r = r0 + g.roff; r < r1; r += 2 * g.RP) {
      const bool two = r + g.RP < r1;  // two rows in flight per iteration
      for (int k = 0; k < g.nv; ++k) {
        const int c0 = g.col(k) * VEC;
        float a[VEC], b[VEC];
        load_vec<T>(x + r * C + c0, a);
        if (two) load_vec<T>(x + (r + g.RP) * C + c0, b);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float d = a[j] - sh[k][j];
          s1[k][j] += d;
          s2[k][j] += d * d;
          if (two) {
            const float e = b[j] - sh[k][j];
            s1[k][j] += e;
            s2[k][j] += e * e;
          }
        }
      }
    }
  }
  // combine the RP row-lanes of each column through LDS (fixed order)
  __shared__ float red[THR * 8];  // >= RP * VEC per column group, reused per k
  float* prow = part + (size_t)blockIdx.x * 2 * C;
  for (int k = 0; k < g.nv; ++k) {
    const int c0 = g.col(k) * VEC;
    for (int h = 0; h < 2; ++h) {
      __syncthreads();
      if (g.active)
#pragma unroll
        for (int j = 0; j < VEC; ++j) red[(g.roff * g.L + (g.L <= THR ? c0 / VEC : 0)) * VEC + j] =
            h == 0 ? s1[k][j] : s2[k][j];
      __syncthreads();
      if (g.L <= THR) {
        for (int cj = threadIdx.x; cj < C; cj += THR) {
          float t = 0.f;
          for (int rr = 0; rr < g.RP; ++rr) t += red[(rr * g.L + cj / VEC) * VEC + cj % VEC];
          prow[h * C + cj] = t;
        }
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) prow[h * C + c0 + j] = h == 0 ? s1[k][j] : s2[k][j];
      }
    }
    if (g.L <= THR) break;
  }
  if (ticket_last(ticket, gridDim.x)) {
    reduce_partials(part, gridDim.x, 2 * C, stats);
    if (threadIdx.x == 0) stats[2 * C] = (float)M;
    for (int c = threadIdx.x; c < C; c += THR) stats[2 * C + 1 + c] = shift[c];
  }
}

// y = act((x - mean) * gamma*invstd + beta (+ res)); block 0: running stats + save
template <typename T, bool RES, bool RELU>
__global__ void __launch_bounds__(THR)
apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, long long M, int C,
             const float* __restrict__ stats, const float* __restrict__ gamma, const float* __restrict__ beta,
             float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt, float momentum,
             float eps, int train, float* __restrict__ save) {
  constexpr int VEC = V16<T>::N;
  extern __shared__ float coef[];  // [C] scale, [C] shift-term
  for (int c = threadIdx.x; c < C; c += THR) {
    float mean, istd;
    if (train) {
      const float n = stats[2 * C];
      const float m1 = stats[c] / n;
      const float var = fmaxf(stats[C + c] / n - m1 * m1, 0.f);
      mean = stats[2 * C + 1 + c] + m1;
      istd = rsqrtf(var + eps);
      if (blockIdx.x == 0) {
        save[c] = mean;
        save[C + c] = istd;
        const int64_t nb = nbt[0] + 1;
        const float mom = momentum >= 0.f ? momentum : 1.f / (float)nb;
        rmean[c] = (1.f - mom) * rmean[c] + mom * mean;
        rvar[c] = (1.f - mom) * rvar[c] + mom * var * (n / fmaxf(n - 1.f, 1.f));
      }
    } else {
      mean = rmean[c];
      istd = rsqrtf(rvar[c] + eps);
    }
    const float s = gamma[c] * istd;
    coef[c] = s;
    coef[C + c] = beta[c] - mean * s;
  }
  __syncthreads();
  if (train && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] = nbt[0] + 1;
  const long long nvec = M * (C / VEC);
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const long long e = v * VEC;
    const int c0 = (int)(e % C);
    float a[VEC], r[VEC];
    load_vec<T>(x + e, a);
    if (RES) load_vec<T>(res + e, r);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float o = a[j] * coef[c0 + j] + coef[C + c0 + j];
      if (RES) o += r[j];
      if (RELU) o = fmaxf(o, 0.f);
      a[j] = o;
    }
    store_vec<T>(y + e, a);
  }
}

// backward statistics: S1 = sum dz, S2 = sum dz*xhat; dz = dy * [y > 0] if RELU.
// out[0..C) = S1, [C..2C) = S2; dgamma = S2, dbeta = S1 (local, f32).
template <typename T, bool RELU>
__global__ void __launch_bounds__(THR)
bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x, long long M, int C,
                 const float* __restrict__ save, float* __restrict__ part, unsigned* __restrict__ ticket,
                 float* __restrict__ out, float* __restrict__ dgamma, float* __restrict__ dbeta) {
  constexpr int VEC = V16<T>::N;
  const Geo g(C, VEC);
  float s1[MAXNV][VEC], s2[MAXNV][VEC], mu[MAXNV][VEC], is[MAXNV][VEC];
  for (int k = 0; k < MAXNV; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) s1[k][j] = s2[k][j] = mu[k][j] = is[k][j] = 0.f;
  const long long rows_per = (M + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  if (g.active) {
    for (int k = 0; k < g.nv; ++k)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        mu[k][j] = save[g.col(k) * VEC + j];
        is[k][j] = save[C + g.col(k) * VEC + j];
      }
    for (long long r = r0 + g.roff; r < r1; r += g.RP) {
      for (int k = 0; k < g.nv; ++k) {
        const long long o = r * C + g.col(k) * VEC;
        float d[VEC], xv[VEC], yv[VEC];
        load_vec<T>(dy + o, d);
        load_vec<T>(x + o, xv);
        if (RELU) load_vec<T>(y + o, yv);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float dz = (!RELU || yv[j] > 0.f) ? d[j] : 0.f;
          s1[k][j] += dz;
          s2[k][j] += dz * (xv[j] - mu[k][j]) * is[k][j];
        }
      }
    }
  }
  __shared__ float red[THR * 8];
  float* prow = part + (size_t)blockIdx.x * 2 * C;
  for (int k = 0; k < g.nv; ++k) {
    const int c0 = g.col(k) * VEC;
    for (int h = 0; h < 2; ++h) {
      __syncthreads();
      if (g.active)
#pragma unroll
        for (int j = 0; j < VEC; ++j) red[(g.roff * g.L + (g.L <= THR ? c0 / VEC : 0)) * VEC + j] =
            h == 0 ? s1[k][j] : s2[k][j];
      __syncthreads();
      if (g.L <= THR) {
        for (int cj = threadIdx.x; cj < C; cj += THR) {
          float t = 0.f;
          for (int rr = 0; rr < g.RP; ++rr) t += red[(rr * g.L + cj / VEC) * VEC + cj % VEC];
          prow[h * C + cj] = t;
        }
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) prow[h * C + c0 + j] = h == 0 ? s1[k][j] : s2[k][j];
      }
    }
    if (g.L <= THR) break;
  }
  if (ticket_last(ticket, gridDim.x)) {
    reduce_partials(part, gridDim.x, 2 * C, out, dbeta, dgamma);
  }
}

// dx = gamma*invstd*(dz - S1/n - xhat*S2/n); dres = dz
template <typename T, bool RELU, bool DRES>
__global__ void __launch_bounds__(THR)
bwd_elemt_kernel(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x, long long M, int C,
                 const float* __restrict__ save, const float* __restrict__ sums, const float* __restrict__ fstats,
                 const float* __restrict__ gamma, T* __restrict__ dx, T* __restrict__ dres) {
  constexpr int VEC = V16<T>::N;
  extern __shared__ float cf[];  // [C] gi, [C] k1, [C] k2, [C] mean, [C] istd
  const float n = fstats[2 * C];
  for (int c = threadIdx.x; c < C; c += THR) {
    const float istd = save[C + c];
    cf[c] = gamma[c] * istd;
    cf[C + c] = sums[c] / n;
    cf[2 * C + c] = sums[C + c] / n;
    cf[3 * C + c] = save[c];
    cf[4 * C + c] = istd;
  }
  __syncthreads();
  const long long nvec = M * (C / VEC);
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const long long e = v * VEC;
    const int c0 = (int)(e % C);
    float d[VEC], xv[VEC], yv[VEC], o[VEC];
    load_vec<T>(dy + e, d);
    load_vec<T>(x + e, xv);
    if (RELU) load_vec<T>(y + e, yv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int c = c0 + j;
      d[j] = (!RELU || yv[j] > 0.f) ? d[j] : 0.f;
      const float xh = (xv[j] - cf[3 * C + c]) * cf[4 * C + c];
      o[j] = cf[c] * (d[j] - cf[C + c] - xh * cf[2 * C + c]);
    }
    store_vec<T>(dx + e, o);
    if (DRES) store_vec<T>(dres + e, d);
  }
}

// ----------------------------------------------------------------------------
// MaxPool2d(3, 2, padding 1) NHWC: out + argmax tap (0..8, first max in kh, kw order)
template <typename T>
__global__ void __launch_bounds__(THR)
maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N, int H, int W,
                   int C, int OH, int OW) {
  constexpr int VEC = V16<T>::N;
  const long long nvec = (long long)N * OH * OW * (C / VEC);
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const int c0 = (int)(v % (C / VEC)) * VEC;
    long long p = v / (C / VEC);
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    float best[VEC];
    uint8_t bi[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float a[VEC];
        load_vec<T>(x + (((long long)n * H + ih) * W + iw) * C + c0, a);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          if (a[j] > best[j] || isnan(a[j])) { best[j] = a[j]; bi[j] = (uint8_t)(kh * 3 + kw); }
      }
    }
    const long long o = (((long long)n * OH + oh) * OW + ow) * C + c0;
    store_vec<T>(y + o, best);
#pragma unroll
    for (int j = 0; j < VEC; ++j) idx[o + j] = bi[j];
  }
}

// gather form: every input pixel sums the (<= 2x2) windows whose argmax it is
template <typename T>
__global__ void __launch_bounds__(THR)
maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx, int N, int H, int W,
                   int C, int OH, int OW) {
  constexpr int VEC = V16<T>::N;
  const long long nvec = (long long)N * H * W * (C / VEC);
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const int c0 = (int)(v % (C / VEC)) * VEC;
    long long p = v / (C / VEC);
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int n = (int)(p / H);
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    for (int kh = 0; kh < 3; ++kh) {
      const int t = h + 1 - kh;
      if (t < 0 || (t & 1)) continue;
      const int oh = t >> 1;
      if (oh >= OH) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int u = w + 1 - kw;
        if (u < 0 || (u & 1)) continue;
        const int ow = u >> 1;
        if (ow >= OW) continue;
        const long long o = (((long long)n * OH + oh) * OW + ow) * C + c0;
        float g[VEC];
        load_vec<T>(dy + o, g);
        const uint8_t want = (uint8_t)(kh * 3 + kw);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          if (idx[o + j] == want) acc[j] += g[j];
      }
    }
    store_vec<T>(dx + (((long long)n * H + h) * W + w) * C + c0, acc);
  }
}

// global average pool NHWC [N][HW][C] -> [N][C] (and its backward)
template <typename T>
__global__ void __launch_bounds__(THR)
avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int HW, int C) {
  constexpr int VEC = V16<T>::N;
  const long long nvec = (long long)N * (C / VEC);
  const float inv = 1.f / (float)HW;
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const int n = (int)(v / (C / VEC));
    const int c0 = (int)(v % (C / VEC)) * VEC;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    for (int p = 0; p < HW; ++p) {
      float a[VEC];
      load_vec<T>(x + ((long long)n * HW + p) * C + c0, a);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += a[j];
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] *= inv;
    store_vec<T>(y + (long long)n * C + c0, acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(THR)
avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  constexpr int VEC = V16<T>::N;
  const long long nvec = (long long)N * HW * (C / VEC);
  const float inv = 1.f / (float)HW;
  for (long long v = (long long)blockIdx.x * THR + threadIdx.x; v < nvec; v += (long long)gridDim.x * THR) {
    const int c0 = (int)(v % (C / VEC)) * VEC;
    const int n = (int)(v / ((long long)HW * (C / VEC)));
    float g[VEC];
    load_vec<T>(dy + (long long)n * C + c0, g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) g[j] *= inv;
    store_vec<T>(dx + v * VEC, g);
  }
}

// ----------------------------------------------------------------------------
template <typename F>
static void dispatch(const at::Tensor& t, F&& f) {
  switch (t.scalar_type()) {
    case at::kBFloat16: f(__hip_bfloat16{}); break;
    case at::kHalf: f(__half{}); break;
    case at::kFloat: f(float{}); break;
    default: TORCH_CHECK(false, "bn_nhwc: unsupported dtype ", t.scalar_type());
  }
}
template <typename T> T* dp(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

// rows x C with C fastest: an NCHW-shaped channels_last tensor, or a contiguous
// tensor whose last dimension is C ([M][C], [N][H][W][C])
static void check_rows(const at::Tensor& t, long long M, int C) {
  const bool cl = t.dim() == 4 && t.size(1) == C && t.is_contiguous(at::MemoryFormat::ChannelsLast);
  const bool rows = t.is_contiguous() && t.size(-1) == C;
  TORCH_CHECK(t.is_cuda() && (cl || rows) && t.numel() == M * C,
              "bn_nhwc: expected rows x C with C contiguous (channels_last NCHW, or [..][C])");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, "bn_nhwc: 16-B aligned tensors");
}

static int stats_grid(long long M, int C, int vec) {
  // enough workgroups to cover the chip, few enough that the last one's partial
  // reduction (G x 2C floats) stays small
  const long long work = M * (C / vec);
  long long g = (work + THR * 16 - 1) / (THR * 16);
  g = std::max<long long>(1, std::min<long long>(g, std::min<long long>(512, 262144 / (2 * C))));
  return (int)g;
}
static int elt_grid(long long nvec) {
  return (int)std::max<long long>(1, std::min<long long>((nvec + THR - 1) / THR, 4096));
}

// part: >= 512*2C floats; ticket: one zero-initialised uint32 (re-armed by the kernel)
void fwd_stats(at::Tensor x, int64_t C, at::Tensor shift, at::Tensor part, at::Tensor ticket, at::Tensor stats) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  TORCH_CHECK(stats.numel() >= 3 * C + 1 && shift.numel() == C && part.numel() >= 512 * 2 * C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    TORCH_CHECK(C % V16<T>::N == 0 && C / V16<T>::N <= THR * MAXNV && (C / V16<T>::N <= THR || (C / V16<T>::N) % THR == 0),
                "bn_nhwc: channel count");
    const int G = stats_grid(M, (int)C, V16<T>::N);
    hipLaunchKernelGGL(fwd_stats_kernel<T>, dim3(G), dim3(THR), 0, cur_stream(), dp<T>(x), M, (int)C,
                       shift.data_ptr<float>(), part.data_ptr<float>(),
                       reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), stats.data_ptr<float>());
  });
  DPA_CHECK_LAUNCH();
}

void apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, int64_t C, at::Tensor stats, at::Tensor gamma,
           at::Tensor beta, at::Tensor rmean, at::Tensor rvar, at::Tensor nbt, double momentum, double eps, bool train,
           bool relu, at::Tensor save) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(y, M, (int)C);
  if (res.has_value()) check_rows(*res, M, (int)C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const int grid = elt_grid(M * C / V16<T>::N);
    const size_t lds = 2 * C * sizeof(float);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(THR), lds, cur_stream(), dp<T>(x),
                         res.has_value() ? dp<T>(*res) : nullptr, dp<T>(y), M, (int)C, stats.data_ptr<float>(),
                         gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(),
                         rvar.data_ptr<float>(), nbt.data_ptr<int64_t>(), (float)momentum, (float)eps, (int)train,
                         save.data_ptr<float>());
    };
    if (res.has_value()) {
      if (relu) go(apply_kernel<T, true, true>); else go(apply_kernel<T, true, false>);
    } else {
      if (relu) go(apply_kernel<T, false, true>); else go(apply_kernel<T, false, false>);
    }
  });
  DPA_CHECK_LAUNCH();
}

void bwd_stats(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, int64_t C, at::Tensor save, at::Tensor part,
               at::Tensor ticket, at::Tensor out, at::Tensor dgamma, at::Tensor dbeta) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(dy, M, (int)C);
  if (y.has_value()) check_rows(*y, M, (int)C);
  TORCH_CHECK(out.numel() >= 2 * C && part.numel() >= 512 * 2 * C && save.numel() >= 2 * C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const int G = stats_grid(M, (int)C, V16<T>::N);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(G), dim3(THR), 0, cur_stream(), dp<T>(dy), y.has_value() ? dp<T>(*y) : nullptr,
                         dp<T>(x), M, (int)C, save.data_ptr<float>(), part.data_ptr<float>(),
                         reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), out.data_ptr<float>(),
                         dgamma.data_ptr<float>(), dbeta.data_ptr<float>());
    };
    if (y.has_value()) go(bwd_stats_kernel<T, true>); else go(bwd_stats_kernel<T, false>);
  });
  DPA_CHECK_LAUNCH();
}

void bwd_elemt(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, int64_t C, at::Tensor save, at::Tensor sums,
               at::Tensor fstats, at::Tensor gamma, at::Tensor dx, c10::optional<at::Tensor> dres) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(dy, M, (int)C);
  check_rows(dx, M, (int)C);
  if (y.has_value()) check_rows(*y, M, (int)C);
  if (dres.has_value()) check_rows(*dres, M, (int)C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const int grid = elt_grid(M * C / V16<T>::N);
    const size_t lds = 5 * C * sizeof(float);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(THR), lds, cur_stream(), dp<T>(dy),
                         y.has_value() ? dp<T>(*y) : nullptr, dp<T>(x), M, (int)C, save.data_ptr<float>(),
                         sums.data_ptr<float>(), fstats.data_ptr<float>(), gamma.data_ptr<float>(), dp<T>(dx),
                         dres.has_value() ? dp<T>(*dres) : nullptr);
    };
    const bool r = y.has_value(), d = dres.has_value();
    if (r && d) go(bwd_elemt_kernel<T, true, true>);
    else if (r) go(bwd_elemt_kernel<T, true, false>);
    else if (d) go(bwd_elemt_kernel<T, false, true>);
    else go(bwd_elemt_kernel<T, false, false>);
  });
  DPA_CHECK_LAUNCH();
}

void maxpool_fwd(at::Tensor x, at::Tensor y, at::Tensor idx) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4, "maxpool: NHWC tensors [N][H][W][C]");
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
  const int OH = (int)y.size(1), OW = (int)y.size(2);
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && y.size(3) == C && idx.numel() == y.numel());
  check_rows(x, (long long)N * H * W, C);
  check_rows(y, (long long)N * OH * OW, C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    TORCH_CHECK(C % V16<T>::N == 0);
    hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(elt_grid((long long)N * OH * OW * C / V16<T>::N)), dim3(THR), 0,
                       cur_stream(), dp<T>(x), dp<T>(y), idx.data_ptr<uint8_t>(), N, H, W, C, OH, OW);
  });
  DPA_CHECK_LAUNCH();
}

void maxpool_bwd(at::Tensor dy, at::Tensor idx, at::Tensor dx) {
  const int N = (int)dx.size(0), H = (int)dx.size(1), W = (int)dx.size(2), C = (int)dx.size(3);
  const int OH = (int)dy.size(1), OW = (int)dy.size(2);
  check_rows(dx, (long long)N * H * W, C);
  check_rows(dy, (long long)N * OH * OW, C);
  TORCH_CHECK(idx.numel() == dy.numel());
  dispatch(dx, [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(elt_grid((long long)N * H * W * C / V16<T>::N)), dim3(THR), 0,
                       cur_stream(), dp<T>(dy), idx.data_ptr<uint8_t>(), dp<T>(dx), N, H, W, C, OH, OW);
  });
  DPA_CHECK_LAUNCH();
}

void avgpool_fwd(at::Tensor x, at::Tensor y, int64_t HW) {
  const int C = (int)y.size(1), N = (int)y.size(0);
  check_rows(x, (long long)N * HW, C);
  check_rows(y, N, C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL(avgpool_fwd_kernel<T>, dim3(elt_grid((long long)N * C / V16<T>::N)), dim3(THR), 0,
                       cur_stream(), dp<T>(x), dp<T>(y), N, (int)HW, C);
  });
  DPA_CHECK_LAUNCH();
}

void avgpool_bwd(at::Tensor dy, at::Tensor dx, int64_t HW) {
  const int C = (int)dy.size(1), N = (int)dy.size(0);
  check_rows(dx, (long long)N * HW, C);
  check_rows(dy, N, C);
  dispatch(dx, [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(elt_grid((long long)N * HW * C / V16<T>::N)), dim3(THR), 0,
                       cur_stream(), dp<T>(dy), dp<T>(dx), N, (int)HW, C);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace bnh

void register_bn_nhwc(pybind11::module& m) {
  auto s = m.def_submodule("bn_nhwc", "channels-last BatchNorm(+add)(+ReLU), max-pool 3x3/2, global avg-pool");
  s.def("fwd_stats", &bnh::fwd_stats);
  s.def("apply", &bnh::apply);
  s.def("bwd_stats", &bnh::bwd_stats);
  s.def("bwd_elemt", &bnh::bwd_elemt);
  s.def("maxpool_fwd", &bnh::maxpool_fwd);
  s.def("maxpool_bwd", &bnh::maxpool_bwd);
  s.def("avgpool_fwd", &bnh::avgpool_fwd);
  s.def("avgpool_bwd", &bnh::avgpool_bwd);
  s.attr("MAX_PARTIAL_ROWS") = 512;
}

}  // namespace dpa
