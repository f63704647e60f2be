// Classifier head: Linear (MFMA small GEMM) and CrossEntropyLoss (fused
// log-softmax + NLL + analytic gradient), plus the eval accuracy counter.
// reference: /root/reference/origin_main.py:24,30,63 (fc, criterion),
//            ddp_main.py:104-107 (argmax == label accumulation).
#include <map>

#include "common.h"

namespace dpa {
namespace head {

constexpr int NTHR = 256;

// 8 K-consecutive elements of row `row` of a [rows][K] matrix of storage type
// S starting at k0, converted to MFMA element type of T; zero outside bounds.
template <typename T, typename S>
__device__ __forceinline__ typename MM<T>::frag load_row8(const S* base, int row, int rows, int k0, int K) {
  typename MM<T>::frag f;
  const bool rv = row < rows;
  const S* p = base + (size_t)(rv ? row : 0) * K;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    const float v = (rv && k < K) ? Cvt<S>::to_f(p[k]) : 0.f;
    f[j] = MM<T>::cv(v);
  }
  return f;
}
// 8 consecutive-row elements of column `col`: base[(k0+j)*ld + col]
template <typename T, typename S>
__device__ __forceinline__ typename MM<T>::frag load_col8(const S* base, int col, int cols, int k0, int K,
                                                          int ld) {
  typename MM<T>::frag f;
  const bool cv = col < cols;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    const float v = (cv && k < K) ? Cvt<S>::to_f(base[(size_t)k * ld + col]) : 0.f;
    f[j] = MM<T>::cv(v);
  }
  return f;
}

// Vector fast path: 8 elements of a row that is 16-B aligned when K % 8 == 0.
template <typename T, typename S>
__device__ __forceinline__ typename MM<T>::frag load_row8v(const S* base, int row, int rows, int k0, int K) {
  if (row < rows && k0 + 8 <= K && (K & 7) == 0) {
    const S* p = base + (size_t)row * K + k0;
    typename MM<T>::frag f;
    if constexpr (sizeof(S) == 4) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(p);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] = MM<T>::cv(lo[j]); f[4 + j] = MM<T>::cv(hi[j]); }
    } else {
      const u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned short bits = v[j];
        S sv;
        __builtin_memcpy(&sv, &bits, 2);
        f[j] = MM<T>::cv(Cvt<S>::to_f(sv));
      }
    }
    return f;
  }
  return load_row8<T, S>(base, row, rows, k0, K);
}

// out[M][N] = x[M][K] . w[N][K]^T + b ; one 16x16 tile per workgroup, K split
// over 16 waves (vector loads straight to registers: every element is read
// once, so no LDS staging), partials combined through LDS.
constexpr int LIN_THR = 1024;
template <typename T>
__global__ void __launch_bounds__(LIN_THR)
linear_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                  T* __restrict__ out, int M, int N, int K) {
  constexpr int NW = LIN_THR / 64;
  __shared__ f32x4 part[NW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int mt = blockIdx.x, nt = blockIdx.y;
  const int KS = (K + 31) / 32;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = wv; s < KS; s += NW) {
    const int k0 = 32 * s + 8 * q;
    const auto a = load_row8v<T, T>(x, mt * 16 + r, M, k0, K);
    const auto bf = load_row8v<T, float>(w, nt * 16 + r, N, k0, K);
    acc = MM<T>::mma(a, bf, acc);
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv == 0) {
    f32x4 t = part[0][lane];
#pragma unroll
    for (int i = 1; i < NW; ++i) t += part[i][lane];
    const int col = nt * 16 + r;
    if (col < N) {
      const float bb = b ? b[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = mt * 16 + 4 * q + i;
        if (row < M) out[(size_t)row * N + col] = Cvt<T>::from_f(t[i] + bb);
      }
    }
  }
}

// 8 elements base[(k0+j)*ld + col] / base[row*K + k0+j] as MFMA operands: clamped
// UNCONDITIONAL loads, the out-of-range values masked afterwards (a guarded load is
// branched around and waited for one by one, cdna_hip_programming.md §5 trap (c))
template <typename T, typename S>
__device__ __forceinline__ typename MM<T>::frag col8c(const S* base, int col, int cols, int k0, int K, int ld) {
  typename MM<T>::frag f;
  const int cc = col < cols ? col : cols - 1;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = Cvt<S>::to_f(base[(size_t)min(k0 + j, K - 1) * ld + cc]);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = MM<T>::cv(col < cols && k0 + j < K ? v[j] : 0.f);
  return f;
}
template <typename T, typename S>
__device__ __forceinline__ typename MM<T>::frag row8c(const S* base, int row, int rows, int k0, int K) {
  typename MM<T>::frag f;
  const S* p = base + (size_t)(row < rows ? row : rows - 1) * K;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = Cvt<S>::to_f(p[min(k0 + j, K - 1)]);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = MM<T>::cv(row < rows && k0 + j < K ? v[j] : 0.f);
  return f;
}

// dx[M][K] = dout[M][N] . w[N][K];  dw[N][K] = dout^T . x;  db[N] = sum_m dout.
// Grid (ceil(K/64), ydx + ceil(N/16)): wave wv of workgroup (j, y) owns the 16 columns
// [64j + 16wv, +16) of a 16-row tile -- of dx for y < ydx (row tile y, reduction over N),
// else of dw (row tile y - ydx, reduction over M; the column-0 workgroups also sum db).
// (One workgroup per 64 columns looping over every tile took 626 us on ResNet-50's fc,
// 128 x 1000 x 2048; this grid has ~2k workgroups there.)
template <typename T>
__global__ void __launch_bounds__(NTHR)
linear_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ x, const float* __restrict__ w,
                  T* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db, int M, int N, int K, int ydx) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int c0 = blockIdx.x * 64 + wv * 16;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int col = c0 + r;
  if ((int)blockIdx.y < ydx) {
    const int mt = blockIdx.y;
    const int NS = (N + 31) / 32;
    for (int s = 0; s < NS; ++s) {
      const int n0 = 32 * s + 8 * q;
      const auto a = row8c<T, T>(dout, mt * 16 + r, M, n0, N);
      const auto bf = col8c<T, float>(w, col, K, n0, N, K);
      acc = MM<T>::mma(a, bf, acc);
    }
    if (col < K) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = mt * 16 + 4 * q + i;
        if (row < M) dx[(size_t)row * K + col] = Cvt<T>::from_f(acc[i]);
      }
    }
    return;
  }
  const int nt = blockIdx.y - ydx;
  const int MS = (M + 31) / 32;
  for (int s = 0; s < MS; ++s) {
    const int m0 = 32 * s + 8 * q;
    const auto a = col8c<T, T>(dout, nt * 16 + r, N, m0, M, N);  // dout^T row n
    const auto bf = col8c<T, T>(x, col, K, m0, M, K);
    acc = MM<T>::mma(a, bf, acc);
  }
  if (col < K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = nt * 16 + 4 * q + i;
      if (row < N) dw[(size_t)row * K + col] = acc[i];
    }
  }
  if (db != nullptr && blockIdx.x == 0 && wv == 0) {  // db for this tile's 16 rows of w
    const int n = nt * 16 + r, nc = n < N ? n : N - 1;
    float t = 0.f;
    for (int m = q; m < M; m += 4) t += Cvt<T>::to_f(dout[(size_t)m * N + nc]);
    t += __shfl_xor(t, 16);
    t += __shfl_xor(t, 32);
    if (q == 0 && n < N) db[n] = t;
  }
}

// Cross-entropy (mean over non-ignored rows) of logits [B][N] (storage T,
// math f32).  Writes loss[0] and dlog[b][n] = (softmax - onehot)/count (f32).
// When `scale` is given (an active GradScaler) it also writes loss[1] =
// loss * scale and dls[b][n] = dlog * scale in T: the gradient of the scaled
// loss that the backward then returns without a launch (ops/head.py).
// One workgroup; a GL-lane group per row (GL = 16 for N <= 16), so 64 rows
// are processed per pass with group-local shuffles only.
template <int GL>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = GL / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
template <int GL>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = GL / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int CE_THR = 1024;

template <typename T, int GL>
__global__ void __launch_bounds__(CE_THR)
ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target, float* __restrict__ loss,
              float* __restrict__ dlog, int B, int N, int64_t ignore_index, float smoothing,
              const float* __restrict__ scale, T* __restrict__ dls) {
  constexpr int RPP = CE_THR / GL;  // rows per pass
  __shared__ float red[CE_THR / 64];
  __shared__ int cnt_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gl = tid % GL, gr = tid / GL;
  if (tid == 0) cnt_s = 0;
  __syncthreads();
  int c = 0;
  for (int b = tid; b < B; b += CE_THR) c += target[b] != ignore_index;
  if (c) atomicAdd(&cnt_s, c);  // integer: order-independent
  __syncthreads();
  const float cnt = (float)cnt_s;
  const float inv = cnt > 0.f ? 1.f / cnt : 0.f;
  const float sc = scale != nullptr ? scale[0] : 0.f;
  float lsum = 0.f;
  for (int r0 = 0; r0 < B; r0 += RPP) {
    const int b = r0 + gr;
    const bool rv = b < B;
    const T* row = logits + (size_t)(rv ? b : 0) * N;
    const int64_t t = rv ? target[b] : ignore_index;
    float mx = -INFINITY, sx = 0.f;
    for (int n = gl; n < N; n += GL) {
      const float v = Cvt<T>::to_f(row[n]);
      mx = fmaxf(mx, v);
      sx += v;
    }
    mx = group_max<GL>(mx);
    sx = group_sum<GL>(sx);
    float se = 0.f;
    for (int n = gl; n < N; n += GL) se += __expf(Cvt<T>::to_f(row[n]) - mx);
    se = group_sum<GL>(se);
    const float lse = mx + __logf(se);
    const bool use = rv && t != ignore_index;
    if (use && gl == 0) {
      const float xt = (t >= 0 && t < N) ? Cvt<T>::to_f(row[t]) : NAN;  // bad target -> NaN loss
      // (1-eps)*(lse - x_t) + eps*(lse - mean_n x_n)
      lsum += (1.f - smoothing) * (lse - xt) + smoothing * (lse - sx / (float)N);
    }
    if (rv) {
      const float rs = 1.f / se;
      for (int n = gl; n < N; n += GL) {
        float d = 0.f;
        if (use) {
          const float sm = __expf(Cvt<T>::to_f(row[n]) - mx) * rs;
          const float oh = (n == t ? 1.f - smoothing : 0.f) + smoothing / (float)N;
          d = (sm - oh) * inv;
        }
        dlog[(size_t)b * N + n] = d;
        if (dls != nullptr) dls[(size_t)b * N + n] = Cvt<T>::from_f(d * sc);
      }
    }
  }
  lsum = wave_sum(lsum);
  if (lane == 0) red[wv] = lsum;
  __syncthreads();
  if (tid == 0) {
    float tl = 0.f;
#pragma unroll
    for (int i = 0; i < CE_THR / 64; ++i) tl += red[i];
    const float l = cnt > 0.f ? tl / cnt : NAN;
    loss[0] = l;
    if (scale != nullptr) loss[1] = l * sc;
  }
}

// Many-row variant (B > 64): RT rows per workgroup, a GL = 64-lane group per row with
// the row held in registers (VPL values per lane: one read of the logits), grid-stride
// over row groups.  The per-workgroup loss partials are handed to the last-arriving
// workgroup write-through (MI355X_MICROARCH.md "Valid forms" row 1, as conv_igemm.hip's
// statistics tree), which sums them in workgroup order (deterministic) and writes the
// loss.  ws: [CE_MAXG] floats + one self-re-arming ticket word after them.
constexpr int CE_RT = 4, CE_RTHR = CE_RT * 64, CE_MAXG = 1024;

template <typename T, int VPL>
__global__ void __launch_bounds__(CE_RTHR)
ce_fwd_rows_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target, float* __restrict__ loss,
                   float* __restrict__ dlog, int B, int N, int64_t ignore_index, float smoothing,
                   const float* __restrict__ scale, T* __restrict__ dls, float* __restrict__ ws) {
  __shared__ float red[CE_RT];
  __shared__ int cnt_s, last_s;
  const int tid = threadIdx.x, gl = tid & 63, gr = tid >> 6;
  if (tid == 0) cnt_s = 0;
  __syncthreads();
  int c = 0;
  for (int b = tid; b < B; b += CE_RTHR) c += target[b] != ignore_index;
  if (c) atomicAdd(&cnt_s, c);  // integer: order-independent
  __syncthreads();
  const float cnt = (float)cnt_s;
  const float inv = cnt > 0.f ? 1.f / cnt : 0.f;
  const float sc = scale != nullptr ? scale[0] : 0.f;
  float lsum = 0.f;
  for (int r0 = blockIdx.x * CE_RT; r0 < B; r0 += gridDim.x * CE_RT) {
    const int b = r0 + gr;
    const bool rv = b < B;
    const T* row = logits + (size_t)(rv ? b : 0) * N;
    const int64_t t = rv ? target[b] : ignore_index;
    float v[VPL];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int n = gl + 64 * k;
      v[k] = (rv && n < N) ? Cvt<T>::to_f(row[n]) : -INFINITY;
    }
    float mx = -INFINITY, sx = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      mx = fmaxf(mx, v[k]);
      if (gl + 64 * k < N) sx += rv ? v[k] : 0.f;
    }
    mx = group_max<64>(mx);
    sx = group_sum<64>(sx);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      v[k] = (gl + 64 * k < N && rv) ? __expf(v[k] - mx) : 0.f;
      se += v[k];
    }
    se = group_sum<64>(se);
    const float lse = mx + __logf(se);
    const bool use = rv && t != ignore_index;
    if (use && gl == 0) {
      const float xt = (t >= 0 && t < N) ? Cvt<T>::to_f(row[t]) : NAN;  // bad target -> NaN loss
      lsum += (1.f - smoothing) * (lse - xt) + smoothing * (lse - sx / (float)N);
    }
    if (rv) {
      const float rs = 1.f / se;
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const int n = gl + 64 * k;
        if (n < N) {
          float d = 0.f;
          if (use) {
            const float oh = (n == t ? 1.f - smoothing : 0.f) + smoothing / (float)N;
            d = (v[k] * rs - oh) * inv;
          }
          dlog[(size_t)b * N + n] = d;
          if (dls != nullptr) dls[(size_t)b * N + n] = Cvt<T>::from_f(d * sc);
        }
      }
    }
  }
  lsum = wave_sum(lsum);
  if (gl == 0) red[gr] = lsum;
  __syncthreads();
  unsigned* ticket = reinterpret_cast<unsigned*>(ws + CE_MAXG);
  if (tid == 0) {
    float tl = 0.f;
#pragma unroll
    for (int i = 0; i < CE_RT; ++i) tl += red[i];
    __hip_atomic_store(ws + blockIdx.x, tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned k = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = k == gridDim.x - 1;
    if (last_s) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();
  if (!last_s || tid != 0) return;
  float tl = 0.f;
  for (int g = 0; g < (int)gridDim.x; ++g) tl += __hip_atomic_load(ws + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float l = cnt > 0.f ? tl / cnt : NAN;
  loss[0] = l;
  if (scale != nullptr) loss[1] = l * sc;
}

// dlogits (storage T) = dlog * grad[0]
template <typename T>
__global__ void ce_bwd_kernel(const float* __restrict__ dlog, const float* __restrict__ grad,
                              T* __restrict__ out, int n) {
  const int i = blockIdx.x * NTHR + threadIdx.x;
  if (i < n) out[i] = Cvt<T>::from_f(dlog[i] * grad[0]);
}

// counters[0] += B ; counters[1] += #(argmax(logits[b]) == target[b])
template <typename T>
__global__ void __launch_bounds__(NTHR)
accuracy_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                float* __restrict__ counters, int B, int N) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float correct = 0.f;
  for (int b = blockIdx.x * (NTHR / 64) + wv; b < B; b += gridDim.x * (NTHR / 64)) {
    const T* row = logits + (size_t)b * N;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int n = lane; n < N; n += 64) {
      const float v = Cvt<T>::to_f(row[n]);
      if (v > best || (v == best && n < bi)) { best = v; bi = n; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0 && bi == target[b]) correct += 1.f;
  }
  if (lane == 0 && correct != 0.f) atomicAdd(&counters[1], correct);
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&counters[0], (float)B);
}

void linear_fwd(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> b, at::Tensor out) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(out);
  TORCH_CHECK(w.scalar_type() == at::kFloat && out.scalar_type() == x.scalar_type());
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N);
  if (M == 0) return;
  const float* bp = b.has_value() ? b->data_ptr<float>() : nullptr;
  const dim3 grid((M + 15) / 16, (N + 15) / 16);
  DPA_DISPATCH_T(dt_of(x), {
    hipLaunchKernelGGL(linear_fwd_kernel<T>, grid, dim3(LIN_THR), 0, cur_stream(), dptr<T>(x),
                       w.data_ptr<float>(), bp, dptr<T>(out), M, N, K);
  });
  DPA_CHECK_LAUNCH();
}

void linear_bwd(at::Tensor dout, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> dx, at::Tensor dw,
                c10::optional<at::Tensor> db) {
  DPA_CHECK_INPUT(dout); DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(dw);
  TORCH_CHECK(dout.scalar_type() == x.scalar_type());
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  if (M == 0) { dw.zero_(); if (db) db->zero_(); return; }
  const int ydx = dx.has_value() ? (M + 15) / 16 : 0;
  const dim3 grid((K + 63) / 64, ydx + (N + 15) / 16);
  DPA_DISPATCH_T(dt_of(x), {
    hipLaunchKernelGGL(linear_bwd_kernel<T>, grid, dim3(NTHR), 0, cur_stream(), dptr<T>(dout), dptr<T>(x),
                       w.data_ptr<float>(), dx.has_value() ? dptr<T>(*dx) : nullptr, dw.data_ptr<float>(),
                       db.has_value() ? db->data_ptr<float>() : nullptr, M, N, K, ydx);
  });
  DPA_CHECK_LAUNCH();
}

void ce_fwd(at::Tensor logits, at::Tensor target, at::Tensor loss, at::Tensor dlog, int64_t ignore_index,
            double smoothing, c10::optional<at::Tensor> scale, c10::optional<at::Tensor> dls) {
  DPA_CHECK_INPUT(logits); DPA_CHECK_INPUT(target); DPA_CHECK_INPUT(loss); DPA_CHECK_INPUT(dlog);
  TORCH_CHECK(target.scalar_type() == at::kLong && dlog.scalar_type() == at::kFloat);
  const int B = (int)logits.size(0), N = (int)logits.size(1);
  TORCH_CHECK(scale.has_value() == dls.has_value());
  if (scale.has_value()) {
    TORCH_CHECK(loss.numel() >= 2 && scale->scalar_type() == at::kFloat && dls->numel() == logits.numel() &&
                dls->scalar_type() == logits.scalar_type());
  }
  if (B > 64 && N <= 64 * 16) {  // many rows: the multi-workgroup kernel (one read of each row)
    static auto* wss = new std::map<int, at::Tensor>();  // per device: partials + ticket, zeroed once (never freed)
    const int dev = logits.get_device();
    auto it = wss->find(dev);
    if (it == wss->end())
      it = wss->emplace(dev, at::zeros({CE_MAXG + 4}, logits.options().dtype(at::kFloat))).first;
    float* ws = it->second.data_ptr<float>();
    const int G = (int)std::min<int64_t>((B + CE_RT - 1) / CE_RT, CE_MAXG);
    DPA_DISPATCH_T(dt_of(logits), {
      auto go = [&](auto vpl) {
        hipLaunchKernelGGL((ce_fwd_rows_kernel<T, decltype(vpl)::value>), dim3(G), dim3(CE_RTHR), 0, cur_stream(),
                           dptr<T>(logits), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                           dlog.data_ptr<float>(), B, N, ignore_index, (float)smoothing,
                           scale.has_value() ? scale->data_ptr<float>() : nullptr,
                           dls.has_value() ? dptr<T>(*dls) : nullptr, ws);
      };
      if (N <= 256) go(std::integral_constant<int, 4>{});
      else go(std::integral_constant<int, 16>{});
    });
    DPA_CHECK_LAUNCH();
    return;
  }
  DPA_DISPATCH_T(dt_of(logits), {
    auto go = [&](auto gl) {
      hipLaunchKernelGGL((ce_fwd_kernel<T, decltype(gl)::value>), dim3(1), dim3(CE_THR), 0, cur_stream(),
                         dptr<T>(logits), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                         dlog.data_ptr<float>(), B, N, ignore_index, (float)smoothing,
                         scale.has_value() ? scale->data_ptr<float>() : nullptr,
                         dls.has_value() ? dptr<T>(*dls) : nullptr);
    };
    if (N <= 16) go(std::integral_constant<int, 16>{});
    else go(std::integral_constant<int, 64>{});
  });
  DPA_CHECK_LAUNCH();
}

void ce_bwd(at::Tensor dlog, at::Tensor grad, at::Tensor out) {
  DPA_CHECK_INPUT(dlog); DPA_CHECK_INPUT(grad); DPA_CHECK_INPUT(out);
  TORCH_CHECK(grad.scalar_type() == at::kFloat, "loss grad must be f32");
  const int n = (int)dlog.numel();
  if (n == 0) return;
  DPA_DISPATCH_T(dt_of(out), {
    hipLaunchKernelGGL(ce_bwd_kernel<T>, dim3((n + NTHR - 1) / NTHR), dim3(NTHR), 0, cur_stream(),
                       dlog.data_ptr<float>(), grad.data_ptr<float>(), dptr<T>(out), n);
  });
  DPA_CHECK_LAUNCH();
}

void accuracy(at::Tensor logits, at::Tensor target, at::Tensor counters) {
  DPA_CHECK_INPUT(logits); DPA_CHECK_INPUT(target); DPA_CHECK_INPUT(counters);
  const int B = (int)logits.size(0), N = (int)logits.size(1);
  if (B == 0) return;
  const int blocks = std::min(64, (B + 3) / 4);
  DPA_DISPATCH_T(dt_of(logits), {
    hipLaunchKernelGGL(accuracy_kernel<T>, dim3(blocks), dim3(NTHR), 0, cur_stream(), dptr<T>(logits),
                       target.data_ptr<int64_t>(), counters.data_ptr<float>(), B, N);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace head

void register_head(pybind11::module& m) {
  auto s = m.def_submodule("head", "Linear (MFMA) / CrossEntropy / accuracy kernels");
  s.def("linear_fwd", &head::linear_fwd);
  s.def("linear_bwd", &head::linear_bwd);
  s.def("ce_fwd", &head::ce_fwd, pybind11::arg("logits"), pybind11::arg("target"), pybind11::arg("loss"),
        pybind11::arg("dlog"), pybind11::arg("ignore_index"), pybind11::arg("smoothing"),
        pybind11::arg("scale") = pybind11::none(), pybind11::arg("dls") = pybind11::none());
  s.def("ce_bwd", &head::ce_bwd);
  s.def("accuracy", &head::accuracy);
}

}  // namespace dpa
