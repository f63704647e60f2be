// Channels-last (NHWC) BatchNorm (+ residual add) (+ ReLU), max-pool 3x3/2 and
// global average pool for the ResNet-50 stress config (BASELINE.json config 5;
// SURVEY.md §7.3 step 8).  Activations are [M = N*H*W][C] rows with C
// contiguous.
//
// Geometry (every BN kernel): the channels are cut into column chunks of
// CC = Lr*VEC <= 64 channels (8 lanes x 16 B bf16, 16 lanes fp32: 128 B of a row,
// blockIdx.y = chunk); a lane owns one 16-B channel vector of its chunk for the
// whole kernel (its per-channel coefficients live in registers) and walks rows
// with stride RP = 256/Lr, U = 4 rows in flight per lane.
//
//   forward (train)  stats:  per-channel sum(x - shift), sum((x - shift)^2);
//                            per-workgroup partial rows, combined by a
//                            two-level ticket tree (groups of 16 workgroups,
//                            then the groups) -> stats[2C+1] (+ shift copy);
//                            the final reducer of chunk 0 bumps
//                            num_batches_tracked.  SyncBN all-reduces the first
//                            2C+1 entries between the launches.
//                    apply:  y = relu?((x - mean) * gamma*invstd + beta (+ res));
//                            row-block 0 of each chunk updates running stats
//                            (momentum, unbiased var) and saves mean / invstd
//   backward         stats:  dz = dy * relu'(.) ; sum(dz), sum(dz * xhat) -> the
//                            same tree; d(gamma), d(beta) from the local sums
//                            (torch SyncBN semantics); all-reduce between
//                    elemt:  dx = gamma*invstd * (dz - S1/n - xhat * S2/n),
//                            d(res) = dz when the block had a residual input
// ReLU derivative: from the saved output y when a residual was added; without
// one it is recomputed from x with the forward's exact fma sequence
// (y > 0  <=>  fma(x, s, b) > 0), so y is neither kept nor re-read.
// The per-channel statistics are sums around a shift (the running mean, equal
// on every rank) to avoid E[x^2] - E[x]^2 cancellation.  Deterministic: every
// reduction has a fixed order (no float atomics).
#include "common.h"
#include "comm/xgmi.h"

namespace dpa {
namespace bnh {

constexpr int THR = 256;
constexpr int CC_MAX = 64;   // channels per column chunk, statistics kernels (128 B of a row)
constexpr int CC_ELT = 256;  // channels per column chunk, elementwise kernels (512 B of a row)
constexpr int G1 = 128;      // level-1 group size of the ticket tree (one level up to 128 row blocks)
constexpr int MAXGR = 1024;  // row blocks per chunk in the statistics kernels
constexpr int SHIFT_OFF = 4; // stats layout: [0,C) s1, [C,2C) s2, [2C] n, shift copy at 2C+SHIFT_OFF (16-B aligned)
#ifndef DPA_BN_U
#define DPA_BN_U 4
#endif
constexpr int U = DPA_BN_U;  // rows in flight per lane (A/B builds: -DDPA_BN_U=2|8)
constexpr int UF = 8;        // rows in flight per lane, forward statistics (one input)
constexpr int MAXTICKETS = 2048;

// Streaming (non-temporal) 16-B activation loads / stores in load_vec / store_vec (A/B builds:
// -DDPA_BN_NT_LOAD=0 / -DDPA_BN_NT_STORE=1).  Loads: ResNet-50 step 14.13 -> 13.93 ms; stores:
// no change (profiles/r6o_bn_nt_ab.txt).
#ifndef DPA_BN_NT_LOAD
#define DPA_BN_NT_LOAD 1
#endif
#ifndef DPA_BN_NT_STORE
#define DPA_BN_NT_STORE 0
#endif

template <typename T> struct V16 { static constexpr int N = 16 / sizeof(T); };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* f) {
#if DPA_BN_NT_LOAD
  const f32x4 raw = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
#else
  const f32x4 raw = *reinterpret_cast<const f32x4*>(p);
#endif
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
#if DPA_BN_NT_STORE
  __builtin_nontemporal_store(raw, reinterpret_cast<f32x4*>(p));
#else
  *reinterpret_cast<f32x4*>(p) = raw;
#endif
}

// VEC consecutive floats (VEC % 4 == 0, 16-B aligned) as 16-B loads
template <int VEC>
__device__ __forceinline__ void ldf(const float* __restrict__ p, float* d) {
#pragma unroll
  for (int k = 0; k < VEC / 4; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + 4 * k);
    d[4 * k] = v[0];
    d[4 * k + 1] = v[1];
    d[4 * k + 2] = v[2];
    d[4 * k + 3] = v[3];
  }
}
template <int VEC>
__device__ __forceinline__ void stf(float* __restrict__ p, const float* d) {
#pragma unroll
  for (int k = 0; k < VEC / 4; ++k) {
    f32x4 v = {d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
    *reinterpret_cast<f32x4*>(p + 4 * k) = v;
  }
}

// Column-chunk width: the largest cc' = cc / 2^k (>= vec) with C <= cc' (one chunk)
// or C % cc' == 0.  The kernels recover it as C / gridDim.y.
inline int chunk_width(int C, int vec, int cc) {
  while (cc > vec && !(C <= cc || C % cc == 0)) cc /= 2;
  return C <= cc ? C : cc;
}

// lane -> (row offset ro in [0, RP), channel c0 of its 16-B vector)
template <int VEC>
struct Chunk {
  int Lr, CC, RP, ro, c0;
  bool active;
  __device__ explicit Chunk(int C) {
    CC = C / (int)gridDim.y;  // chunk_width() on the host
    Lr = CC / VEC;
    RP = THR / Lr;
    ro = (int)threadIdx.x / Lr;
    active = ro < RP;
    c0 = (int)blockIdx.y * CC + ((int)threadIdx.x % Lr) * VEC;
  }
};

// rows [r0, r1) of this row block
__device__ __forceinline__ void row_range(long long M, long long& r0, long long& r1) {
  const long long per = (M + gridDim.x - 1) / gridDim.x;
  r0 = (long long)blockIdx.x * per;
  r1 = r0 + per < M ? r0 + per : M;
}

// Write-through hand-off (MI355X_MICROARCH.md "Valid forms", row 1): partial rows
// stored with agent-scope relaxed atomic stores (sc1, past the XCD's L2) and read
// back with agent-scope atomic loads, so the ticket needs no release / acquire
// fence -- an agent release writes back the whole L2 of the XCD, once per
// workgroup.  g_handoff_wt (bn_nhwc.set_handoff) = 0 restores the fenced form.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last-arriver election over `n` workgroups: fenced (wt = 0: agent-scope release /
// acquire around the ticket) or write-through (wt = 1: the rows were stored sc1).
__device__ __forceinline__ bool ticket_last(unsigned* ticket, int n, int* s_flag, int wt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its partial-row stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!wt) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == (unsigned)n - 1;
    *s_flag = last;
    if (last) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm for the next launch
      if (!wt) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  }
  __syncthreads();
  return *s_flag != 0;
}

// dst[t] = sum_{g < n} src[g*W + t], W % 4 == 0, fixed order.  Lanes load
// 16-B column vectors; the RG = THR/(W/4) row groups of the block each sum
// every RG-th row with up to 16 loads in flight per lane, then the RG partials
// are added in group order through LDS (scr: >= THR*4 floats).
__device__ __forceinline__ f32x4 ld4(const float* p, int wt) {
  if (!wt) return *reinterpret_cast<const f32x4*>(p);
  return f32x4{ld_wt(p), ld_wt(p + 1), ld_wt(p + 2), ld_wt(p + 3)};
}
__device__ __noinline__ void sum_rows(const float* __restrict__ src, int n, int W, float* __restrict__ dst,
                                      float* scr, int wt, int wt_dst) {
  const int W4 = W / 4;
  const int RG = W4 >= THR ? 1 : THR / W4;
  for (int base = 0; base < W4; base += THR) {
    const int col = base + (int)threadIdx.x % (W4 >= THR ? THR : W4);
    const int rg = W4 >= THR ? 0 : (int)threadIdx.x / W4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (rg < RG && col < W4) {
      for (int g0 = rg; g0 < n; g0 += 16 * RG) {
        f32x4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int g = g0 + u * RG;
          v[u] = ld4(src + (size_t)(g < n ? g : n - 1) * W + 4 * col, wt);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (g0 + u * RG < n) acc += v[u];
      }
    }
    __syncthreads();
    if (rg < RG && col < W4) *reinterpret_cast<f32x4*>(scr + 4 * ((size_t)rg * (W4 >= THR ? THR : W4) + (col - base))) = acc;
    __syncthreads();
    const int nc = W4 - base < THR ? W4 - base : THR;
    if ((int)threadIdx.x < nc) {
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < RG; ++r) t += *reinterpret_cast<const f32x4*>(scr + 4 * ((size_t)r * nc + threadIdx.x));
      float* d = dst + 4 * (base + threadIdx.x);
      if (wt_dst) {
        st_wt(d, t[0]); st_wt(d + 1, t[1]); st_wt(d + 2, t[2]); st_wt(d + 3, t[3]);
      } else {
        *reinterpret_cast<f32x4*>(d) = t;
      }
    }
  }
}

// Block partial -> part, then the two-level ticket tree of this chunk.  Returns
// true in the single workgroup per chunk that ends with the chunk's W totals in
// red[0, W).  part: [Gc*Gr + Gc*NG][W] floats; tickets: [Gc*NG + Gc].
// xs active (SyncBN): lane 0 of the chunk's finisher takes the site ticket into *tk before
// the last level's loads (its round trip overlaps them).
__device__ bool chunk_reduce(float* __restrict__ part, unsigned* __restrict__ tickets, int W, float* red,
                             float* scr, int* s_flag, int wt, const xgmi::XSite& xs, unsigned long long* tk) {
  const int Gr = gridDim.x, Gc = gridDim.y, y = blockIdx.y;
  const int NG = (Gr + G1 - 1) / G1;
  float* p1 = part + (size_t)y * Gr * W;
  float* p2 = part + (size_t)Gc * Gr * W + (size_t)y * NG * W;
  for (int t = threadIdx.x; t < W; t += THR) {
    if (wt) st_wt(p1 + (size_t)blockIdx.x * W + t, red[t]);
    else p1[(size_t)blockIdx.x * W + t] = red[t];
  }
  const int grp = blockIdx.x / G1;
  const int gsz = min(G1, Gr - grp * G1);
  if (!ticket_last(tickets + y * NG + grp, gsz, s_flag, wt)) return false;
  if (NG == 1) {
    if (xs.active() && threadIdx.x == 0) *tk = xgmi::xsite_ticket(xs, y);
    sum_rows(p1, gsz, W, red, scr, wt, 0);
    __syncthreads();
    return true;
  }
  sum_rows(p1 + (size_t)grp * G1 * W, gsz, W, p2 + (size_t)grp * W, scr, wt, wt);
  if (!ticket_last(tickets + Gc * NG + y, NG, s_flag, wt)) return false;
  if (xs.active() && threadIdx.x == 0) *tk = xgmi::xsite_ticket(xs, y);
  sum_rows(p2, NG, W, red, scr, wt, 0);
  __syncthreads();
  return true;
}
__device__ bool chunk_reduce(float* __restrict__ part, unsigned* __restrict__ tickets, int W, float* red,
                             float* scr, int* s_flag, int wt) {
  unsigned long long tk;
  return chunk_reduce(part, tickets, W, red, scr, s_flag, wt, xgmi::XSite{}, &tk);
}

// SyncBN inside a statistics finisher (chunk y of Gc, the site's nblk = Gc): red = [S1 | S2]
// of the chunk's CC channels (+ red[2 CC] = the row count in chunk 0 when `count`), local
// -> global in place (comm/xsite.h positioned form; row positions S1 at c, S2 at C + c,
// count at 2C).
__device__ __forceinline__ void chunk_exchange(const xgmi::XSite& xs, float* red, int CC, int C, bool count,
                                               unsigned long long tk) {
  const int y = blockIdx.y, cb = y * CC;
  const int n = 2 * CC + (count && y == 0 ? 1 : 0);
  xgmi::xsite_exchange_slice(xs, red, n, [&](int i) { return i < CC ? cb + i : i < 2 * CC ? C + cb + i - CC : 2 * C; },
                             tk, y, THR);
}

// Combine the RP row-lanes of the block: red[h*CC + c] = sum_ro acc_h (fixed order).
template <int VEC>
__device__ __forceinline__ void block_combine(const Chunk<VEC>& g, const float* s1, const float* s2, float* red,
                                              float* scratch) {
  const int cl = g.c0 - (int)blockIdx.y * g.CC;  // column within the chunk
  if (g.active)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      scratch[(size_t)g.ro * g.CC + cl + j] = s1[j];
      scratch[(size_t)(g.RP + g.ro) * g.CC + cl + j] = s2[j];
    }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * g.CC; t += THR) {
    const int h = t / g.CC, c = t % g.CC;
    float acc = 0.f;
    for (int rr = 0; rr < g.RP; ++rr) acc += scratch[(size_t)(h * g.RP + rr) * g.CC + c];
    red[t] = acc;
  }
  __syncthreads();
}

// ----------------------------------------------------------------------------
// forward statistics: stats[0..C) = sum(x-shift), [C..2C) = sum((x-shift)^2),
// [2C] = rows, [2C+4 .. 3C+4) = shift (copied for the apply / backward)
template <typename T>
__global__ void __launch_bounds__(THR)
fwd_stats_kernel(const T* __restrict__ x, long long M, int C, const float* __restrict__ shift,
                 float* __restrict__ part, unsigned* __restrict__ tickets, float* __restrict__ stats,
                 int64_t* __restrict__ nbt, int wt, xgmi::XSite xs) {
  constexpr int VEC = V16<T>::N;
  __shared__ float scratch[2 * THR * VEC];
  __shared__ float red[2 * CC_MAX + 1];
  __shared__ int s_flag;
  const Chunk<VEC> g(C);
  float s1[VEC], s2[VEC], sh[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) s1[j] = s2[j] = sh[j] = 0.f;
  long long r0, r1;
  row_range(M, r0, r1);
  if (g.active) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) sh[j] = shift[g.c0 + j];
    long long r = r0 + g.ro;
    for (; r + (UF - 1) * g.RP < r1; r += UF * g.RP) {
      float a[UF][VEC];
#pragma unroll
      for (int u = 0; u < UF; ++u) load_vec<T>(x + (r + u * g.RP) * C + g.c0, a[u]);
#pragma unroll
      for (int u = 0; u < UF; ++u)
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float d = a[u][j] - sh[j];
          s1[j] += d;
          s2[j] = fmaf(d, d, s2[j]);
        }
    }
    for (; r < r1; r += g.RP) {
      float a[VEC];
      load_vec<T>(x + r * C + g.c0, a);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = a[j] - sh[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
  block_combine<VEC>(g, s1, s2, red, scratch);
  unsigned long long tk = 0;
  if (!chunk_reduce(part, tickets, 2 * g.CC, red, scratch, &s_flag, wt, xs, &tk)) return;
  if (blockIdx.y == 0 && threadIdx.x == 0) red[2 * g.CC] = (float)M;
  if (xs.active()) chunk_exchange(xs, red, g.CC, C, true, tk);  // SyncBN: global sums and count
  const int cb = (int)blockIdx.y * g.CC;
  for (int t = threadIdx.x; t < g.CC; t += THR) {
    stats[cb + t] = red[t];
    stats[C + cb + t] = red[g.CC + t];
    stats[2 * C + SHIFT_OFF + cb + t] = shift[cb + t];
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    stats[2 * C] = red[2 * g.CC];
    if (nbt != nullptr) nbt[0] = nbt[0] + 1;
  }
}

// y = act((x - mean) * gamma*invstd + beta (+ res)) as fma(x, s, b) (+ res);
// row block 0 of each chunk: running stats + save
template <typename T, bool RES, bool RELU>
__global__ void __launch_bounds__(THR)
apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, long long M, int C,
             const float* __restrict__ stats, const float* __restrict__ gamma, const float* __restrict__ beta,
             float* __restrict__ rmean, float* __restrict__ rvar, const int64_t* __restrict__ nbt, float momentum,
             float eps, int train, float* __restrict__ save) {
  constexpr int VEC = V16<T>::N;
  const Chunk<VEC> g(C);
  if (!g.active) return;
  float s[VEC], b[VEC], mean[VEC], istd[VEC], ga[VEC], be[VEC];
  ldf<VEC>(gamma + g.c0, ga);
  ldf<VEC>(beta + g.c0, be);
  if (train) {
    float s1[VEC], s2[VEC], sh[VEC], var[VEC];
    ldf<VEC>(stats + g.c0, s1);
    ldf<VEC>(stats + C + g.c0, s2);
    ldf<VEC>(stats + 2 * C + SHIFT_OFF + g.c0, sh);
    const float n = stats[2 * C];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float m1 = s1[j] / n;
      var[j] = fmaxf(s2[j] / n - m1 * m1, 0.f);
      mean[j] = sh[j] + m1;
      istd[j] = rsqrtf(var[j] + eps);
    }
    if (blockIdx.x == 0 && g.ro == 0) {
      stf<VEC>(save + g.c0, mean);
      stf<VEC>(save + C + g.c0, istd);
      const float mom = momentum >= 0.f ? momentum : 1.f / (float)nbt[0];  // nbt bumped by the stats kernel
      float rm[VEC], rv[VEC];
      ldf<VEC>(rmean + g.c0, rm);
      ldf<VEC>(rvar + g.c0, rv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        rm[j] = (1.f - mom) * rm[j] + mom * mean[j];
        rv[j] = (1.f - mom) * rv[j] + mom * var[j] * (n / fmaxf(n - 1.f, 1.f));
      }
      stf<VEC>(rmean + g.c0, rm);
      stf<VEC>(rvar + g.c0, rv);
    }
  } else {
    float rv[VEC];
    ldf<VEC>(rmean + g.c0, mean);
    ldf<VEC>(rvar + g.c0, rv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) istd[j] = rsqrtf(rv[j] + eps);
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    s[j] = ga[j] * istd[j];
    b[j] = fmaf(-mean[j], s[j], be[j]);
  }
  long long r0, r1;
  row_range(M, r0, r1);
  auto row = [&](long long r, float* a, const float* rr) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float o = fmaf(a[j], s[j], b[j]);
      if (RES) o += rr[j];
      if (RELU) o = fmaxf(o, 0.f);
      a[j] = o;
    }
    store_vec<T>(y + r * C + g.c0, a);
  };
  long long r = r0 + g.ro;
  for (; r + (U - 1) * g.RP < r1; r += U * g.RP) {
    float a[U][VEC], q[U][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_vec<T>(x + (r + u * g.RP) * C + g.c0, a[u]);
      if (RES) load_vec<T>(res + (r + u * g.RP) * C + g.c0, q[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) row(r + u * g.RP, a[u], q[u]);
  }
  for (; r < r1; r += g.RP) {
    float a[VEC], q[VEC];
    load_vec<T>(x + r * C + g.c0, a);
    if (RES) load_vec<T>(res + r * C + g.c0, q);
    row(r, a, q);
  }
}

// A projection bottleneck's tail in one pass: y = relu(bn(x) + bn_r(res)) -- the
// downsample conv's BatchNorm applied while reading its raw output (apply_kernel would
// first write the normalised identity and read it back: one pass of 2 tensors less).
// Both BNs' coefficients, running stats and saves are handled as in apply_kernel.
struct BnCo {
  const float* stats;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  const int64_t* nbt;
  float momentum, eps;
  float* save;
};

template <int VEC>
__device__ __forceinline__ void bn_coef(const BnCo& p, int c0, int C, int train, bool leader, float* s, float* b) {
  float mean[VEC], istd[VEC], ga[VEC], be[VEC];
  ldf<VEC>(p.gamma + c0, ga);
  ldf<VEC>(p.beta + c0, be);
  if (train) {
    float s1[VEC], s2[VEC], sh[VEC], var[VEC];
    ldf<VEC>(p.stats + c0, s1);
    ldf<VEC>(p.stats + C + c0, s2);
    ldf<VEC>(p.stats + 2 * C + SHIFT_OFF + c0, sh);
    const float n = p.stats[2 * C];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float m1 = s1[j] / n;
      var[j] = fmaxf(s2[j] / n - m1 * m1, 0.f);
      mean[j] = sh[j] + m1;
      istd[j] = rsqrtf(var[j] + p.eps);
    }
    if (leader) {
      stf<VEC>(p.save + c0, mean);
      stf<VEC>(p.save + C + c0, istd);
      const float mom = p.momentum >= 0.f ? p.momentum : 1.f / (float)p.nbt[0];
      float rm[VEC], rv[VEC];
      ldf<VEC>(p.rmean + c0, rm);
      ldf<VEC>(p.rvar + c0, rv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        rm[j] = (1.f - mom) * rm[j] + mom * mean[j];
        rv[j] = (1.f - mom) * rv[j] + mom * var[j] * (n / fmaxf(n - 1.f, 1.f));
      }
      stf<VEC>(p.rmean + c0, rm);
      stf<VEC>(p.rvar + c0, rv);
    }
  } else {
    float rv[VEC];
    ldf<VEC>(p.rmean + c0, mean);
    ldf<VEC>(p.rvar + c0, rv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) istd[j] = rsqrtf(rv[j] + p.eps);
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    s[j] = ga[j] * istd[j];
    b[j] = fmaf(-mean[j], s[j], be[j]);
  }
}

template <typename T>
__global__ void __launch_bounds__(THR)
apply_resbn_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, long long M, int C,
                   BnCo m, BnCo r, int train) {
  constexpr int VEC = V16<T>::N;
  const Chunk<VEC> g(C);
  if (!g.active) return;
  float s[VEC], b[VEC], rs[VEC], rb[VEC];
  const bool leader = blockIdx.x == 0 && g.ro == 0;
  bn_coef<VEC>(m, g.c0, C, train, leader, s, b);
  bn_coef<VEC>(r, g.c0, C, train, leader, rs, rb);
  long long r0, r1;
  row_range(M, r0, r1);
  auto row = [&](long long rr, float* a, const float* q) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) a[j] = fmaxf(fmaf(a[j], s[j], b[j]) + fmaf(q[j], rs[j], rb[j]), 0.f);
    store_vec<T>(y + rr * C + g.c0, a);
  };
  long long rr = r0 + g.ro;
  for (; rr + (U - 1) * g.RP < r1; rr += U * g.RP) {
    float a[U][VEC], q[U][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_vec<T>(x + (rr + u * g.RP) * C + g.c0, a[u]);
      load_vec<T>(res + (rr + u * g.RP) * C + g.c0, q[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) row(rr + u * g.RP, a[u], q[u]);
  }
  for (; rr < r1; rr += g.RP) {
    float a[VEC], q[VEC];
    load_vec<T>(x + rr * C + g.c0, a);
    load_vec<T>(res + rr * C + g.c0, q);
    row(rr, a, q);
  }
}

// ReLU-derivative source of the backward kernels
enum { ACT_NONE = 0, ACT_Y = 1, ACT_RECOMPUTE = 2 };

template <int VEC, int ACT>
struct BwdLane {
  float mu[VEC], is[VEC], s[VEC], b[VEC];
  __device__ void init(int c0, int C, const float* save, const float* gamma, const float* beta) {
    ldf<VEC>(save + c0, mu);
    ldf<VEC>(save + C + c0, is);
    if (ACT == ACT_RECOMPUTE) {
      float ga[VEC], be[VEC];
      ldf<VEC>(gamma + c0, ga);
      ldf<VEC>(beta + c0, be);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        s[j] = ga[j] * is[j];
        b[j] = fmaf(-mu[j], s[j], be[j]);
      }
    }
  }
  // dz = dy * relu'(.)
  __device__ __forceinline__ float dz(int j, float d, float xv, float yv) const {
    if (ACT == ACT_Y) return yv > 0.f ? d : 0.f;
    if (ACT == ACT_RECOMPUTE) return fmaf(xv, s[j], b[j]) > 0.f ? d : 0.f;
    return d;
  }
};

// backward statistics: S1 = sum dz, S2 = sum dz*xhat.
// out[0..C) = S1, [C..2C) = S2; dbeta = S1, dgamma = S2 (local, f32).
template <typename T, int ACT>
__global__ void __launch_bounds__(THR)
bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x, long long M, int C,
                 const float* __restrict__ save, const float* __restrict__ gamma, const float* __restrict__ beta,
                 float* __restrict__ part, unsigned* __restrict__ tickets, float* __restrict__ out,
                 float* __restrict__ dgamma, float* __restrict__ dbeta, int wt, xgmi::XSite xs) {
  constexpr int VEC = V16<T>::N;
  __shared__ float scratch[2 * THR * VEC];
  __shared__ float red[2 * CC_MAX];
  __shared__ int s_flag;
  const Chunk<VEC> g(C);
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) s1[j] = s2[j] = 0.f;
  long long r0, r1;
  row_range(M, r0, r1);
  if (g.active) {
    BwdLane<VEC, ACT> L;
    L.init(g.c0, C, save, gamma, beta);
    auto acc = [&](const float* d, const float* xv, const float* yv) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float z = L.dz(j, d[j], xv[j], yv[j]);
        s1[j] += z;
        s2[j] = fmaf(z, (xv[j] - L.mu[j]) * L.is[j], s2[j]);
      }
    };
    long long r = r0 + g.ro;
    for (; r + (U - 1) * g.RP < r1; r += U * g.RP) {
      float d[U][VEC], xv[U][VEC], yv[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long o = (r + u * g.RP) * C + g.c0;
        load_vec<T>(dy + o, d[u]);
        load_vec<T>(x + o, xv[u]);
        if (ACT == ACT_Y) load_vec<T>(y + o, yv[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc(d[u], xv[u], yv[u]);
    }
    for (; r < r1; r += g.RP) {
      float d[VEC], xv[VEC], yv[VEC];
      const long long o = r * C + g.c0;
      load_vec<T>(dy + o, d);
      load_vec<T>(x + o, xv);
      if (ACT == ACT_Y) load_vec<T>(y + o, yv);
      acc(d, xv, yv);
    }
  }
  block_combine<VEC>(g, s1, s2, red, scratch);
  unsigned long long tk = 0;
  if (!chunk_reduce(part, tickets, 2 * g.CC, red, scratch, &s_flag, wt, xs, &tk)) return;
  const int cb = (int)blockIdx.y * g.CC;
  for (int t = threadIdx.x; t < g.CC; t += THR) {  // this rank's sums (DDP averages them)
    dbeta[cb + t] = red[t];
    dgamma[cb + t] = red[g.CC + t];
  }
  if (xs.active()) chunk_exchange(xs, red, g.CC, C, false, tk);  // SyncBN: out = the global sums
  for (int t = threadIdx.x; t < g.CC; t += THR) {
    out[cb + t] = red[t];
    out[C + cb + t] = red[g.CC + t];
  }
}

// dx = gamma*invstd*(dz - S1/n - xhat*S2/n); dres = dz
template <typename T, int ACT, bool DRES>
__global__ void __launch_bounds__(THR)
bwd_elemt_kernel(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x, long long M, int C,
                 const float* __restrict__ save, const float* __restrict__ sums, const float* __restrict__ fstats,
                 const float* __restrict__ gamma, const float* __restrict__ beta, T* __restrict__ dx,
                 T* __restrict__ dres) {
  constexpr int VEC = V16<T>::N;
  const Chunk<VEC> g(C);
  if (!g.active) return;
  BwdLane<VEC, ACT> L;
  L.init(g.c0, C, save, gamma, beta);
  float gi[VEC], k1[VEC], k2[VEC];
  const float n = fstats[2 * C];
  ldf<VEC>(gamma + g.c0, gi);
  ldf<VEC>(sums + g.c0, k1);
  ldf<VEC>(sums + C + g.c0, k2);
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    gi[j] *= L.is[j];
    k1[j] /= n;
    k2[j] /= n;
  }
  auto row = [&](long long o, const float* d, const float* xv, const float* yv) {
    float z[VEC], e[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      z[j] = L.dz(j, d[j], xv[j], yv[j]);
      const float xh = (xv[j] - L.mu[j]) * L.is[j];
      e[j] = gi[j] * (z[j] - k1[j] - xh * k2[j]);
    }
    store_vec<T>(dx + o, e);
    if (DRES) store_vec<T>(dres + o, z);
  };
  long long r0, r1;
  row_range(M, r0, r1);
  long long r = r0 + g.ro;
  for (; r + (U - 1) * g.RP < r1; r += U * g.RP) {
    float d[U][VEC], xv[U][VEC], yv[U][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = (r + u * g.RP) * C + g.c0;
      load_vec<T>(dy + o, d[u]);
      load_vec<T>(x + o, xv[u]);
      if (ACT == ACT_Y) load_vec<T>(y + o, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) row((r + u * g.RP) * C + g.c0, d[u], xv[u], yv[u]);
  }
  for (; r < r1; r += g.RP) {
    float d[VEC], xv[VEC], yv[VEC];
    const long long o = r * C + g.c0;
    load_vec<T>(dy + o, d);
    load_vec<T>(x + o, xv);
    if (ACT == ACT_Y) load_vec<T>(y + o, yv);
    row(o, d, xv, yv);
  }
}

// bwd_elemt_kernel<T, ACT_Y, true> of a projection block's last BN that also takes the
// downsample BN's backward sums from the dz it writes: rout = [S1 | S2] with S1 = sum dz,
// S2 = sum dz * (r - mean_r) * invstd_r (r: the downsample conv's output), rdbeta = S1,
// rdgamma = S2 -- the downsample BN's own statistics pass over dz and r disappears.
template <typename T>
__global__ void __launch_bounds__(THR)
bwd_elemt_rbn_kernel(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x, long long M, int C,
                     const float* __restrict__ save, const float* __restrict__ sums, const float* __restrict__ fstats,
                     const float* __restrict__ gamma, const float* __restrict__ beta, T* __restrict__ dx,
                     T* __restrict__ dres, const T* __restrict__ r, const float* __restrict__ rsave,
                     float* __restrict__ part, unsigned* __restrict__ tickets, float* __restrict__ rout,
                     float* __restrict__ rdgamma, float* __restrict__ rdbeta, int wt) {
  constexpr int VEC = V16<T>::N;
  __shared__ float scratch[2 * THR * VEC];
  __shared__ float red[2 * CC_ELT];
  __shared__ int s_flag;
  const Chunk<VEC> g(C);
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) s1[j] = s2[j] = 0.f;
  if (g.active) {
    BwdLane<VEC, ACT_Y> L;
    L.init(g.c0, C, save, gamma, beta);
    float gi[VEC], k1[VEC], k2[VEC], rmu[VEC], ris[VEC];
    const float n = fstats[2 * C];
    ldf<VEC>(gamma + g.c0, gi);
    ldf<VEC>(sums + g.c0, k1);
    ldf<VEC>(sums + C + g.c0, k2);
    ldf<VEC>(rsave + g.c0, rmu);
    ldf<VEC>(rsave + C + g.c0, ris);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      gi[j] *= L.is[j];
      k1[j] /= n;
      k2[j] /= n;
    }
    auto row = [&](long long o, const float* d, const float* xv, const float* yv, const float* rv) {
      float z[VEC], e[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        z[j] = L.dz(j, d[j], xv[j], yv[j]);
        const float xh = (xv[j] - L.mu[j]) * L.is[j];
        e[j] = gi[j] * (z[j] - k1[j] - xh * k2[j]);
      }
      store_vec<T>(dx + o, e);
      store_vec<T>(dres + o, z);
      // the downsample BN's sums of dz (dy masked: already a storage-exact value, so these
      // are the sums its own statistics pass over the stored dres would take)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        s1[j] += z[j];
        s2[j] = fmaf(z[j], (rv[j] - rmu[j]) * ris[j], s2[j]);
      }
    };
    long long r0, r1;
    row_range(M, r0, r1);
    long long rr = r0 + g.ro;
    for (; rr + (U - 1) * g.RP < r1; rr += U * g.RP) {
      float d[U][VEC], xv[U][VEC], yv[U][VEC], rv[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long o = (rr + u * g.RP) * C + g.c0;
        load_vec<T>(dy + o, d[u]);
        load_vec<T>(x + o, xv[u]);
        load_vec<T>(y + o, yv[u]);
        load_vec<T>(r + o, rv[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) row((rr + u * g.RP) * C + g.c0, d[u], xv[u], yv[u], rv[u]);
    }
    for (; rr < r1; rr += g.RP) {
      float d[VEC], xv[VEC], yv[VEC], rv[VEC];
      const long long o = rr * C + g.c0;
      load_vec<T>(dy + o, d);
      load_vec<T>(x + o, xv);
      load_vec<T>(y + o, yv);
      load_vec<T>(r + o, rv);
      row(o, d, xv, yv, rv);
    }
  }
  block_combine<VEC>(g, s1, s2, red, scratch);
  if (!chunk_reduce(part, tickets, 2 * g.CC, red, scratch, &s_flag, wt)) return;
  const int cb = (int)blockIdx.y * g.CC;
  for (int t = threadIdx.x; t < g.CC; t += THR) {
    rout[cb + t] = rdbeta[cb + t] = red[t];
    rout[C + cb + t] = rdgamma[cb + t] = red[g.CC + t];
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
        const unsigned want = (unsigned)(kh * 3 + kw);
        // the VEC argmax bytes of this vector as ONE load (o % VEC == 0: C % VEC == 0), not VEC
        // byte loads
        unsigned long long iv;
        if constexpr (VEC == 8) iv = *reinterpret_cast<const unsigned long long*>(idx + o);
        else iv = *reinterpret_cast<const unsigned*>(idx + o);  // fp32: 4 bytes (o % 4 == 0)
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          if (((iv >> (8 * j)) & 0xffull) == want) acc[j] += g[j];
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


// ----------------------------------------------------------------------------
struct Grid2 {
  int Gr, Gc;
};
// workgroup-count targets (tunable: bn_nhwc.set_grid_targets; scripts/bn_sweep.py).
// Statistics: fewer, longer workgroups win (the ticket tree's tail grows with the
// row-block count): 128 below 64 MB of input, 256 above (measured on ResNet-50
// shapes, profiles/r1_bn_sweep.txt).  0 = that rule.
static int g_stats_target = 0;
static int g_apply_target = 512;
static int g_elemt_target = 1024;
static int g_handoff_wt = 1;  // statistics ticket trees: write-through hand-off (1) or fenced (0)
void set_handoff(int64_t wt) { g_handoff_wt = wt ? 1 : 0; }
void set_grid_targets(int64_t stats, int64_t apply, int64_t elemt) {
  TORCH_CHECK(stats >= 0 && apply >= 1 && elemt >= 1);
  g_stats_target = (int)stats;
  g_apply_target = (int)apply;
  g_elemt_target = (int)elemt;
}
template <typename T>
static Grid2 chunk_grid(long long M, int C, int target, int cc = CC_MAX) {
  constexpr int VEC = V16<T>::N;
  TORCH_CHECK(C % VEC == 0, "bn_nhwc: channel count ", C, " must be a multiple of ", VEC);
  const int CCw = chunk_width(C, VEC, cc);
  const int Lr = CCw / VEC;
  const int RP = THR / Lr;
  const int Gc = C / CCw;
  const long long by_rows = std::max<long long>(1, (M + (long long)RP * U - 1) / ((long long)RP * U));
  const long long want = std::max<long long>(1, (target + Gc - 1) / Gc);
  return {(int)std::min<long long>(by_rows, want), Gc};
}
template <typename T>
static Grid2 stats_grid(long long M, int C) {
  const int target = g_stats_target > 0 ? g_stats_target : (M * C * (long long)sizeof(T) < (64ll << 20) ? 128 : 256);
  Grid2 g = chunk_grid<T>(M, C, target);
  g.Gr = std::min(g.Gr, MAXGR);
  return g;
}
static int elt_grid(long long nvec) {
  return (int)std::max<long long>(1, std::min<long long>((nvec + THR - 1) / THR, 4096));
}
static void check_workspace(const Grid2& g, int C, const at::Tensor& part, const at::Tensor& tickets) {
  const int NG = (g.Gr + G1 - 1) / G1;
  TORCH_CHECK(part.numel() >= (long long)2 * C * (g.Gr + NG), "bn_nhwc: partial-sum workspace too small");
  TORCH_CHECK(tickets.numel() >= g.Gc * (NG + 1) && tickets.scalar_type() == at::kInt, "bn_nhwc: ticket workspace");
}

// part: >= 2C*(MAXGR + MAXGR/G1) floats; tickets: >= MAXTICKETS zero-initialised int32 (re-armed by the kernels)
// SyncBN site (xc, the ResNet finishers' wide site): the statistics leave the launch global
static xgmi::XSite stats_site(const std::shared_ptr<xgmi::XgmiComm>& xc, int64_t C, int Gc) {
  if (!xc) return xgmi::XSite{};
  TORCH_CHECK(2 * C + 1 <= xgmi::kWideVals, "bn_nhwc: SyncBN site row holds 2C+1 <= ", xgmi::kWideVals);
  xgmi::XSite xs = xc->wide_site();
  xgmi::set_site_grid(xs, Gc, "bn_nhwc statistics");  // one finisher per channel chunk
  return xs;
}

void fwd_stats(at::Tensor x, int64_t C, at::Tensor shift, at::Tensor part, at::Tensor ticket, at::Tensor stats,
               c10::optional<at::Tensor> nbt, std::shared_ptr<xgmi::XgmiComm> xc) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  TORCH_CHECK(stats.numel() >= 3 * C + SHIFT_OFF && shift.numel() == C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const Grid2 g = stats_grid<T>(M, (int)C);
    check_workspace(g, (int)C, part, ticket);
    hipLaunchKernelGGL(fwd_stats_kernel<T>, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(x), M, (int)C,
                       shift.data_ptr<float>(), part.data_ptr<float>(),
                       reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), stats.data_ptr<float>(),
                       nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr, g_handoff_wt, stats_site(xc, C, g.Gc));
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
    const Grid2 g = chunk_grid<T>(M, (int)C, g_apply_target, CC_ELT);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(x),
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

// y = relu(bn(x) + bn_r(res)); both BNs' running stats / saves updated (train)
void apply_resbn(at::Tensor x, at::Tensor res, at::Tensor y, int64_t C, at::Tensor stats, at::Tensor gamma,
                 at::Tensor beta, at::Tensor rmean, at::Tensor rvar, at::Tensor nbt, double momentum, double eps,
                 at::Tensor save, at::Tensor rstats, at::Tensor rgamma, at::Tensor rbeta, at::Tensor rrmean,
                 at::Tensor rrvar, at::Tensor rnbt, double rmomentum, double reps, at::Tensor rsave, bool train) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(res, M, (int)C);
  check_rows(y, M, (int)C);
  TORCH_CHECK(x.scalar_type() == res.scalar_type() && x.scalar_type() == y.scalar_type(), "apply_resbn: one dtype");
  for (const at::Tensor* t : {&stats, &gamma, &beta, &rmean, &rvar, &save, &rstats, &rgamma, &rbeta, &rrmean, &rrvar,
                              &rsave})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "apply_resbn: fp32 contiguous BN tensors");
  TORCH_CHECK(save.numel() >= 2 * C && rsave.numel() >= 2 * C && gamma.numel() == C && rgamma.numel() == C,
              "apply_resbn: sizes");
  if (train)
    TORCH_CHECK(stats.numel() >= 3 * C + SHIFT_OFF && rstats.numel() >= 3 * C + SHIFT_OFF, "apply_resbn: stats");
  BnCo m{stats.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(),
         rvar.data_ptr<float>(), nbt.data_ptr<int64_t>(), (float)momentum, (float)eps, save.data_ptr<float>()};
  BnCo r{rstats.data_ptr<float>(), rgamma.data_ptr<float>(), rbeta.data_ptr<float>(), rrmean.data_ptr<float>(),
         rrvar.data_ptr<float>(), rnbt.data_ptr<int64_t>(), (float)rmomentum, (float)reps, rsave.data_ptr<float>()};
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const Grid2 g = chunk_grid<T>(M, (int)C, g_apply_target, CC_ELT);
    hipLaunchKernelGGL(apply_resbn_kernel<T>, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(x), dp<T>(res),
                       dp<T>(y), M, (int)C, m, r, (int)train);
  });
  DPA_CHECK_LAUNCH();
}

// act: 0 = no ReLU, 1 = ReLU derivative from y, 2 = recomputed from x (no residual)
void bwd_stats(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, int64_t C, int64_t act, at::Tensor save,
               at::Tensor gamma, at::Tensor beta, at::Tensor part, at::Tensor ticket, at::Tensor out,
               at::Tensor dgamma, at::Tensor dbeta, std::shared_ptr<xgmi::XgmiComm> xc) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(dy, M, (int)C);
  TORCH_CHECK(act >= 0 && act <= 2 && (act != ACT_Y || y.has_value()));
  if (act == ACT_Y) check_rows(*y, M, (int)C);
  TORCH_CHECK(out.numel() >= 2 * C && save.numel() >= 2 * C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const Grid2 g = stats_grid<T>(M, (int)C);
    check_workspace(g, (int)C, part, ticket);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(dy),
                         act == ACT_Y ? dp<T>(*y) : nullptr, dp<T>(x), M, (int)C, save.data_ptr<float>(),
                         gamma.data_ptr<float>(), beta.data_ptr<float>(), part.data_ptr<float>(),
                         reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), out.data_ptr<float>(),
                         dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), g_handoff_wt, stats_site(xc, C, g.Gc));
    };
    if (act == ACT_Y) go(bwd_stats_kernel<T, ACT_Y>);
    else if (act == ACT_RECOMPUTE) go(bwd_stats_kernel<T, ACT_RECOMPUTE>);
    else go(bwd_stats_kernel<T, ACT_NONE>);
  });
  DPA_CHECK_LAUNCH();
}

void bwd_elemt(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, int64_t C, int64_t act, at::Tensor save,
               at::Tensor sums, at::Tensor fstats, at::Tensor gamma, at::Tensor beta, at::Tensor dx,
               c10::optional<at::Tensor> dres) {
  const long long M = x.numel() / C;
  check_rows(x, M, (int)C);
  check_rows(dy, M, (int)C);
  check_rows(dx, M, (int)C);
  TORCH_CHECK(act >= 0 && act <= 2 && (act != ACT_Y || y.has_value()));
  if (act == ACT_Y) check_rows(*y, M, (int)C);
  if (dres.has_value()) check_rows(*dres, M, (int)C);
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    const Grid2 g = chunk_grid<T>(M, (int)C, g_elemt_target, CC_ELT);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(dy),
                         act == ACT_Y ? dp<T>(*y) : nullptr, dp<T>(x), M, (int)C, save.data_ptr<float>(),
                         sums.data_ptr<float>(), fstats.data_ptr<float>(), gamma.data_ptr<float>(),
                         beta.data_ptr<float>(), dp<T>(dx), dres.has_value() ? dp<T>(*dres) : nullptr);
    };
    const bool d = dres.has_value();
    if (act == ACT_Y) { if (d) go(bwd_elemt_kernel<T, ACT_Y, true>); else go(bwd_elemt_kernel<T, ACT_Y, false>); }
    else if (act == ACT_RECOMPUTE) { if (d) go(bwd_elemt_kernel<T, ACT_RECOMPUTE, true>); else go(bwd_elemt_kernel<T, ACT_RECOMPUTE, false>); }
    else { if (d) go(bwd_elemt_kernel<T, ACT_NONE, true>); else go(bwd_elemt_kernel<T, ACT_NONE, false>); }
  });
  DPA_CHECK_LAUNCH();
}

// bwd_elemt (act 1, with dres) + the downsample BN's backward sums of dres (see the kernel)
void bwd_elemt_rbn(at::Tensor dy, at::Tensor y, at::Tensor x, int64_t C, at::Tensor save, at::Tensor sums,
                   at::Tensor fstats, at::Tensor gamma, at::Tensor beta, at::Tensor dx, at::Tensor dres, at::Tensor r,
                   at::Tensor rsave, at::Tensor part, at::Tensor ticket, at::Tensor rout, at::Tensor rdgamma,
                   at::Tensor rdbeta) {
  const long long M = x.numel() / C;
  for (const at::Tensor* t : {&dy, &y, &x, &dx, &dres, &r}) check_rows(*t, M, (int)C);
  TORCH_CHECK(rsave.numel() >= 2 * C && rout.numel() >= 2 * C && rdgamma.numel() == C && rdbeta.numel() == C,
              "bwd_elemt_rbn: sizes");
  dispatch(x, [&](auto tag) {
    typedef decltype(tag) T;
    Grid2 g = chunk_grid<T>(M, (int)C, g_elemt_target, CC_ELT);
    g.Gr = std::min(g.Gr, MAXGR);
    check_workspace(g, (int)C, part, ticket);
    hipLaunchKernelGGL(bwd_elemt_rbn_kernel<T>, dim3(g.Gr, g.Gc), dim3(THR), 0, cur_stream(), dp<T>(dy), dp<T>(y),
                       dp<T>(x), M, (int)C, save.data_ptr<float>(), sums.data_ptr<float>(), fstats.data_ptr<float>(),
                       gamma.data_ptr<float>(), beta.data_ptr<float>(), dp<T>(dx), dp<T>(dres), dp<T>(r),
                       rsave.data_ptr<float>(), part.data_ptr<float>(),
                       reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), rout.data_ptr<float>(),
                       rdgamma.data_ptr<float>(), rdbeta.data_ptr<float>(), g_handoff_wt);
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
    TORCH_CHECK(C % V16<T>::N == 0, "maxpool_bwd: channels must be a multiple of ", V16<T>::N);
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
  s.def("fwd_stats", &bnh::fwd_stats, pybind11::arg("x"), pybind11::arg("C"), pybind11::arg("shift"),
        pybind11::arg("part"), pybind11::arg("ticket"), pybind11::arg("stats"), pybind11::arg("nbt"),
        pybind11::arg("xc") = pybind11::none());
  s.def("set_grid_targets", &bnh::set_grid_targets);
  s.def("set_handoff", &bnh::set_handoff);
  s.def("apply", &bnh::apply);
  s.def("apply_resbn", &bnh::apply_resbn);
  s.def("bwd_elemt_rbn", &bnh::bwd_elemt_rbn);
  s.def("bwd_stats", &bnh::bwd_stats, pybind11::arg("dy"), pybind11::arg("y"), pybind11::arg("x"), pybind11::arg("C"),
        pybind11::arg("act"), pybind11::arg("save"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("part"), pybind11::arg("ticket"), pybind11::arg("out"), pybind11::arg("dgamma"),
        pybind11::arg("dbeta"), pybind11::arg("xc") = pybind11::none());
  s.def("bwd_elemt", &bnh::bwd_elemt);
  s.def("maxpool_fwd", &bnh::maxpool_fwd);
  s.def("maxpool_bwd", &bnh::maxpool_bwd);
  s.def("avgpool_fwd", &bnh::avgpool_fwd);
  s.def("avgpool_bwd", &bnh::avgpool_bwd);
  s.attr("MAX_PARTIAL_ROWS") = bnh::MAXGR + bnh::MAXGR / bnh::G1;
  s.attr("MAX_TICKETS") = bnh::MAXTICKETS;
}

}  // namespace dpa
