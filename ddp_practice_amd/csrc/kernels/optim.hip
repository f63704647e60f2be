// Optimizer / AMP kernels (multi-tensor, one launch per <= MAXT tensors):
//   amp_unscale_check : g *= 1/scale in place; found_inf |= any(!isfinite(g))
//                       (== torch._amp_foreach_non_finite_check_and_unscale_,
//                        torch/amp/grad_scaler.py:235-286)
//   sgd_step          : SGD (momentum/dampening/nesterov/weight decay/maximize)
//                       predicated on found_inf read ON DEVICE, so GradScaler.step
//                       needs no found_inf.item() host sync (grad_scaler.py:356)
//   amp_update_scale  : == torch._amp_update_scale_ (grad_scaler.py:500-537)
//   flat_copy_scale   : multi-tensor gather into / scatter out of a flat bucket
//                       with an optional scale (DDP reducer pack/unpack)
// reference call sites: /root/reference/ddp_main.py:91-93 (scaler.scale/step/update),
// origin_main.py:87 (SGD lr=1e-4).
#include <cstdlib>
#include "common.h"
#include "comm/xgmi.h"

#include <vector>

namespace dpa {
namespace opt {

constexpr int NTHR = 256;
constexpr int MAXT = 36;
constexpr int CHUNK = 4096;

struct MTList {
  int n;
  unsigned long long first_bits;  // momentum: bit t set = tensor t's buffer is new (b = d)
  int64_t numel[MAXT];
  int64_t chunk_off[MAXT + 1];  // prefix sum of chunks
  float* p0[MAXT];
  float* p1[MAXT];
  float* p2[MAXT];
};

__device__ __forceinline__ int find_tensor(const MTList& L, int64_t c) {
  int t = 0;
  while (t + 1 < L.n && L.chunk_off[t + 1] <= c) ++t;
  return t;
}

__global__ void __launch_bounds__(NTHR)
unscale_check_kernel(MTList L, const float* __restrict__ scale, float* __restrict__ found_inf) {
  const float inv = 1.f / scale[0];
  const int64_t total = L.chunk_off[L.n];
  bool bad = false;
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(L, c);
    const int64_t base = (c - L.chunk_off[t]) * CHUNK;
    const int64_t end = min(base + (int64_t)CHUNK, L.numel[t]);
    float* g = L.p0[t];
    float v[CHUNK / NTHR];
#pragma unroll
    for (int k = 0; k < CHUNK / NTHR; ++k) {
      const int64_t i = base + k * NTHR + threadIdx.x;
      v[k] = i < end ? g[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < CHUNK / NTHR; ++k) {
      const int64_t i = base + k * NTHR + threadIdx.x;
      bad |= !isfinite(v[k]);
      if (i < end) g[i] = v[k] * inv;
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) found_inf[0] = 1.f;
}

// p0 = param, p1 = grad, p2 = momentum buffer (may be null)
__global__ void __launch_bounds__(NTHR)
sgd_kernel(MTList L, float lr, float momentum, float dampening, float wd, int nesterov, int maximize,
           const float* __restrict__ found_inf, const float* __restrict__ grad_scale) {
  if (found_inf != nullptr && found_inf[0] != 0.f) return;
  const float gs = grad_scale ? 1.f / grad_scale[0] : 1.f;
  const int64_t total = L.chunk_off[L.n];
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(L, c);
    const int64_t base = (c - L.chunk_off[t]) * CHUNK;
    const int64_t end = min(base + (int64_t)CHUNK, L.numel[t]);
    float* p = L.p0[t];
    const float* g = L.p1[t];
    float* buf = L.p2[t];
    const bool first = (L.first_bits >> t) & 1ull;
    float gv[CHUNK / NTHR], pv[CHUNK / NTHR], bv0[CHUNK / NTHR];
#pragma unroll
    for (int k = 0; k < CHUNK / NTHR; ++k) {
      const int64_t i = base + k * NTHR + threadIdx.x;
      const bool in = i < end;
      gv[k] = in ? g[i] : 0.f;
      pv[k] = in ? p[i] : 0.f;
      bv0[k] = (in && momentum != 0.f && !first) ? buf[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < CHUNK / NTHR; ++k) {
      const int64_t i = base + k * NTHR + threadIdx.x;
      if (i >= end) continue;
      float d = gv[k] * gs;
      if (maximize) d = -d;
      if (wd != 0.f) d += wd * pv[k];
      if (momentum != 0.f) {
        const float b = first ? d : momentum * bv0[k] + (1.f - dampening) * d;
        buf[i] = b;
        d = nesterov ? d + momentum * b : b;
      }
      p[i] = pv[k] - lr * d;
    }
  }
}

__global__ void update_scale_kernel(float* scale, int* tracker, float* found_inf, float growth,
                                    float backoff, int interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool inf = found_inf[0] != 0.f;
  found_inf[0] = 0.f;  // re-arm for the next step: unscale_check only ever sets it
  if (inf) {
    scale[0] = scale[0] * backoff;
    tracker[0] = 0;
  } else {
    const int succ = tracker[0] + 1;
    if (succ == interval) {
      const float ns = scale[0] * growth;
      if (isfinite(ns)) scale[0] = ns;
      tracker[0] = 0;
    } else {
      tracker[0] = succ;
    }
  }
}

// GradScaler.step + SGD + GradScaler.update in ONE launch over a small grid
// (the ConvNet: 29,034 floats -> 8 workgroups).  Every lane loads its grads,
// params (and momentum buffers) into registers, the workgroups agree on
// found_inf through ONE 64-bit device-scope atomic per generation
// ({arrivals, non-finite workgroups} in one word: no fence, no flag), and then
// each applies its own slice: unscaled grads written back (torch semantics),
// the update applied only if every grad is finite, scale / growth tracker
// updated and found_inf re-armed by workgroup 0.  p0 = param, p1 = grad,
// p2 = momentum buffer (or null).
//
// Grid barrier state `sync` (int64[3], zero-initialised, one per optimizer and
// grid size): [0] launch counter g, [1 + (g & 1)] this launch's word.  Block 0
// resets the other parity's word and bumps g after the barrier; the next launch
// is stream-ordered after this one, so it always finds its word at zero.  The
// grid (<= FUSED_MAX_BLOCKS of 256 lanes, one per CU at most) is co-resident.
constexpr int FUSED_THR = 256;
constexpr int FUSED_U = 4;                                  // float4 granules per lane
constexpr int FUSED_BLOCK_GRAN = FUSED_THR * FUSED_U;       // 4096 floats per workgroup
constexpr int FUSED_MAX_BLOCKS = 128;
constexpr int64_t FUSED_MAX = (int64_t)FUSED_MAX_BLOCKS * FUSED_BLOCK_GRAN * 4;
// (A one-workgroup variant of 1024 lanes x 8 granules for the ConvNet measured 10.9 us
// vs 8.6 us for 8 workgroups + grid barrier: one CU's bandwidth is the limit, not the
// barrier.  A grid of one still skips the barrier, below.)

// The flat index space is in float4 granules; tensor t owns ceil(numel/4)
// granules starting at chunk_off[t] (every pointer 16-B aligned, checked on the
// host), so a granule never straddles two tensors.  Tensor tables live in LDS
// (per-lane dynamic indexing of the by-value kernel argument is a chain of
// dependent scalar loads).
//
// XG (DDP over the xGMI engine, DistributedDataParallel.defer_grad_sync_to):
// the gradient all-reduce is fused in as well.  Each lane pushes its local
// gradient granules to every peer as {value, epoch} granules (the one-shot
// protocol of comm/xgmi_allreduce.hip, epoch from comm/xsite.h tickets), then
// sums the W ranks' values in rank order and divides by W before the inf check
// -- the reducer launched no collective for these buckets.  U = 1 granule per
// lane then (one poll round trip of W x 4 granules per lane, 4x the workgroups).
//
// SlabSrc (optional; with XG its columns are exchanged like granules): one gradient region [out, out + n) is still the
// per-workgroup partial rows of a producer (slab [rows][n], e.g. the ConvNet's conv1
// weight-gradient slab): nblk extra workgroups, appended after the granule grid, own
// it -- they sum its columns (16 columns x 16 row groups each, the association of the
// column-sum launch), check them, load the matching params / buffers, arrive at the
// grid barrier like the others and then apply the same update per element (unscaled
// gradient written to `out`).  The granule workgroups skip the region, and the separate
// column-sum launch disappears.
struct SlabSrc {
  const float* slab;
  float* out;
  int rows, n, nblk;
};
constexpr int SS_COLS = 16, SS_GROUPS = FUSED_THR / SS_COLS;

template <int U, bool XG, int THR = FUSED_THR>
__global__ void __launch_bounds__(THR)
amp_sgd_fused_kernel(MTList L, float* __restrict__ scale, int* __restrict__ tracker, float* __restrict__ found_inf,
                     unsigned long long* __restrict__ sync, float lr, float momentum, float dampening, float wd,
                     int nesterov, int maximize, float growth, float backoff, int interval,
                     xgmi::XSite xg, int* __restrict__ err, long long barrier_ticks, SlabSrc ss, int grid) {
  // grid == the launch's workgroup count, passed in: gridDim is a load from the hidden kernel
  // arguments on gfx950, and its wait at the top of the kernel came before the table loads
  constexpr int BG = THR * U;  // float4 granules per workgroup
  __shared__ int soff[MAXT + 1];
  __shared__ int snum[MAXT];
  __shared__ float* sp0[MAXT];
  __shared__ float* sp1[MAXT];
  __shared__ float* sp2[MAXT];
  __shared__ int s_bad;
  const int tid = threadIdx.x;
  const int n = L.n;
  {  // the table: every load issued before any LDS write (clamped index; a guarded load was
     // branched and waited for before the next group's loads were issued)
    const int ti = min(tid, MAXT - 1);
    const int64_t co = L.chunk_off[min(tid, MAXT)], nu = L.numel[ti];
    float* const a0 = L.p0[ti];
    float* const a1 = L.p1[ti];
    float* const a2 = L.p2[ti];
    if (tid <= n) soff[tid] = (int)co;
    if (tid < n) {
      snum[tid] = (int)nu;
      sp0[tid] = a0;
      sp1[tid] = a1;
      sp2[tid] = a2;
    }
  }
  __syncthreads();
  const int total = soff[n];
  // the barrier generation is only used by lane 0: issued after the table
  // barrier, its load stays in flight (no LDS round trip) with the gradients'
  unsigned long long gen = 0;
  if (tid == 0 && grid > 1)
    gen = __hip_atomic_fetch_add(&sync[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long tk = 0;
  if (XG && tid == 0) tk = xgmi::xsite_ticket(xg, (int)blockIdx.x);
  auto load4 = [](const float* p, int rem) {
    if (rem >= 4) return *reinterpret_cast<const f32x4*>(p);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < rem; ++j) v[j] = p[j];
    return v;
  };
  auto store4 = [](float* p, int rem, f32x4 v) {
    if (rem >= 4) { *reinterpret_cast<f32x4*>(p) = v; return; }
    for (int j = 0; j < rem; ++j) p[j] = v[j];
  };
  f32x4 gv[U], pv[U], bv[U];
  int tt[U];  // tensor of each granule (its offset is recomputed after the barrier)
  bool bad = false;
  const int nreg = grid - ss.nblk;  // granule workgroups; the rest own the slab region
  // slab workgroup lane (< SS_COLS): its column's sum, tensor and element, param / buffer
  float st_sum = 0.f, st_p = 0.f, st_b = 0.f;
  int st_t = -1, st_e = 0;
  if ((int)blockIdx.x >= nreg) {
    __shared__ float spart[SS_GROUPS][SS_COLS + 1];
    const int c0 = ((int)blockIdx.x - nreg) * SS_COLS;
    const int col = c0 + tid % SS_COLS, g = tid / SS_COLS;
    if (tid < SS_COLS && col < ss.n) {  // param / buffer loads in flight with the slab's
      const float* gp = ss.out + col;
      for (int i = 0; i < n; ++i)  // the tensor whose gradient holds this column (host-checked: one)
        if (gp >= sp1[i] && gp < sp1[i] + snum[i]) {
          st_t = i;
          st_e = (int)(gp - sp1[i]);
        }
      if (st_t >= 0) {
        st_p = sp0[st_t][st_e];
        if (momentum != 0.f && !((L.first_bits >> st_t) & 1ull)) st_b = sp2[st_t][st_e];
      }
    }
    spart[g][tid % SS_COLS] = slab_colsum<SS_GROUPS>(ss.slab, ss.rows, ss.n, col, g);  // = slab_reduce
    __syncthreads();
    if (tid < SS_COLS && col < ss.n) {
#pragma unroll
      for (int gg = 0; gg < SS_GROUPS; ++gg) st_sum += spart[gg][tid];
      bad = !isfinite(st_sum);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) tt[k] = -1;
  } else {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int gi = blockIdx.x * BG + k * THR + tid;
      tt[k] = -1;
      if (gi < total) {
        int lo = 0, hi = n - 1;  // tensor holding granule gi
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (soff[mid] <= gi) lo = mid; else hi = mid - 1;
        }
        const int o = (gi - soff[lo]) * 4, rem = snum[lo] - o;
        const float* gp = sp1[lo] + o;
        if (gp >= ss.out && gp < ss.out + ss.n) continue;  // the slab workgroups own it
        tt[k] = lo;
        gv[k] = load4(gp, rem);
        pv[k] = load4(sp0[lo] + o, rem);
        const bool use_buf = momentum != 0.f && !((L.first_bits >> lo) & 1ull);
        bv[k] = use_buf ? load4(sp2[lo] + o, rem) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  if constexpr (XG) {
    __shared__ uint32_t ep_x;
    if (tid == 0) ep_x = xgmi::xsite_epoch(xg, tk, (int)blockIdx.x);
    __syncthreads();
    const uint32_t ep = ep_x;
    const long long par = (long long)(ep & 1u) * xgmi::kMaxRanks * xg.slot_bytes;
    auto gran = [ep](float v) { return ((unsigned long long)ep << 32) | (unsigned long long)__float_as_uint(v); };
    typedef __attribute__((ext_vector_type(2))) unsigned long long u64x2;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (tt[k] < 0) continue;
      const long long fo = (long long)(blockIdx.x * BG + k * THR + tid) * 32;  // 4 granules of 8 B
      const u64x2 a = {gran(gv[k][0]), gran(gv[k][1])}, b = {gran(gv[k][2]), gran(gv[k][3])};
      for (int p = 0; p < xg.world; ++p) {
        if (p == xg.rank) continue;  // my own values stay in registers
        u64x2* dst = reinterpret_cast<u64x2*>(xg.base[p] + par + (long long)xg.rank * xg.slot_bytes + fo);
        dst[0] = a;
        dst[1] = b;
      }
    }
    const float invw = 1.f / (float)xg.world;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned polls = 0;
    bool fail = false;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (tt[k] < 0) continue;
      const long long fo = (long long)(blockIdx.x * BG + k * THR + tid) * 32;
      unsigned long long g[xgmi::kMaxRanks][4];
      const unsigned long long* src[xgmi::kMaxRanks];
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {  // every load issued before the first tag check
        src[p] = reinterpret_cast<const unsigned long long*>(xg.base[xg.rank] + par + (long long)p * xg.slot_bytes +
                                                             fo);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          g[p][j] = (p < xg.world && p != xg.rank)
                        ? __hip_atomic_load(src[p] + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                        : 0ull;
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {
        if (p >= xg.world) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x = p == xg.rank ? gv[k][j] : xgmi::xsite_wait(xg, src[p] + j, g[p][j], ep, t0, polls, fail);
          acc[j] = p == 0 ? x : acc[j] + x;
        }
      }
      gv[k] = acc * invw;
    }
    if (st_t >= 0) {
      // a slab column (this lane's element, summed above): the same exchange, one granule
      // at the element's position in the flat granule space -- the slab region needs no
      // separate column-sum launch at W > 1 either
      const long long fo = (long long)(soff[st_t] + st_e / 4) * 32 + (long long)(st_e % 4) * 8;
      const unsigned long long gm = gran(st_sum);
      for (int p = 0; p < xg.world; ++p) {
        if (p == xg.rank) continue;
        *reinterpret_cast<unsigned long long*>(xg.base[p] + par + (long long)xg.rank * xg.slot_bytes + fo) = gm;
      }
      unsigned long long g[xgmi::kMaxRanks];
      const unsigned long long* src[xgmi::kMaxRanks];
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {
        src[p] = reinterpret_cast<const unsigned long long*>(xg.base[xg.rank] + par + (long long)p * xg.slot_bytes +
                                                             fo);
        g[p] = (p < xg.world && p != xg.rank) ? __hip_atomic_load(src[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                              : 0ull;
      }
      float acc = 0.f;
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {
        if (p >= xg.world) continue;
        const float x = p == xg.rank ? st_sum : xgmi::xsite_wait(xg, src[p], g[p], ep, t0, polls, fail);
        acc = p == 0 ? x : acc + x;
      }
      st_sum = acc * invw;
      bad |= !isfinite(st_sum);
    }
    // a peer that never arrived (timeout / abort: error word set) leaves a partial sum:
    // take the skip path (no parameter / momentum / scale change) rather than apply it
    bad |= fail;
  }
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (tt[k] >= 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) bad |= !isfinite(gv[k][j]);
  // scale read before arriving: block 0 rewrites it once everyone has arrived, and a
  // workgroup that reads it late must not unscale with the next step's value
  const float inv = 1.f / scale[0];
  const bool block_bad = __syncthreads_or(bad);
  if (grid == 1) {  // uniform: one workgroup needs no grid barrier
    if (tid == 0) s_bad = block_bad;
  } else if (tid == 0) {
    unsigned long long* word = &sync[1 + (gen & 1)];
    const unsigned long long G = (unsigned long long)grid;
    __hip_atomic_fetch_add(word, 1ull | ((unsigned long long)block_bad << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long v;
    // bounded: the host sizes the grid to be co-resident (amp_sgd_fused), so every workgroup
    // arrives; should one never do, give up after barrier_ticks, flag it and skip the update
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool timed_out = false;
    while (((v = __hip_atomic_fetch_add(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & 0xffffffffull) <
           G) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > barrier_ticks) {
        timed_out = true;
        if (err != nullptr) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    s_bad = timed_out || (v >> 32) != 0;
    if (blockIdx.x == 0) {
      __hip_atomic_exchange(&sync[1 + ((gen + 1) & 1)], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&sync[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  const bool any_bad = s_bad;
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int t = tt[k];
    if (t < 0) continue;
    const int o = (blockIdx.x * BG + k * THR + tid - soff[t]) * 4, rem = snum[t] - o;
    const f32x4 g = gv[k] * inv;
    store4(sp1[t] + o, rem, g);
    if (any_bad) continue;
    f32x4 d = maximize ? -g : g;
    if (wd != 0.f) d += wd * pv[k];
    if (momentum != 0.f) {
      const bool first = (L.first_bits >> t) & 1ull;
      const f32x4 bb = first ? d : momentum * bv[k] + (1.f - dampening) * d;
      store4(sp2[t] + o, rem, bb);
      d = nesterov ? d + momentum * bb : bb;
    }
    store4(sp0[t] + o, rem, pv[k] - lr * d);
  }
  if (st_t >= 0) {  // a slab column: the same update, one element
    const float g = st_sum * inv;
    sp1[st_t][st_e] = g;
    if (!any_bad) {
      float d = maximize ? -g : g;
      if (wd != 0.f) d += wd * st_p;
      if (momentum != 0.f) {
        const bool first = (L.first_bits >> st_t) & 1ull;
        const float bb = first ? d : momentum * st_b + (1.f - dampening) * d;
        sp2[st_t][st_e] = bb;
        d = nesterov ? d + momentum * bb : bb;
      }
      sp0[st_t][st_e] = st_p - lr * d;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    // every workgroup read scale[0] before arriving, and block 0 passed the barrier
    found_inf[0] = 0.f;
    if (any_bad) {
      scale[0] = scale[0] * backoff;
      tracker[0] = 0;
    } else {
      const int succ = tracker[0] + 1;
      if (succ == interval) {
        const float ns = scale[0] * growth;
        if (isfinite(ns)) scale[0] = ns;
        tracker[0] = 0;
      } else {
        tracker[0] = succ;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Large-model fused AMP step (ResNet-50: 161 tensors, 25.6M floats): the same
// semantics as amp_sgd_fused_kernel -- unscale, global inf agreement, SGD, scale
// update -- in ONE launch of a co-resident grid, for any tensor count / size.
//   * the tensor table lives in device memory (built once per distinct set of
//     pointers by amp_sgd_table, captured into graphs by value) and is staged in LDS;
//   * phase A streams the grads once for the non-finite check (no write), the grid
//     agrees through one arrival word (the bounded barrier of the small kernel), and
//     phase B streams grads / params / buffers for the update -- the second grad
//     read mostly hits the 256 MB MALL for ResNet-50's 102 MB of grads;
//   * each workgroup owns one contiguous range of float4 granules, each lane walks it
//     with a monotone tensor cursor (no per-granule search).
// Table (int64): [0] n, [1] total granules, then off[n+1] | numel[n] | p0[n] | p1[n] |
// p2[n] | first[n]  (p0 param, p1 grad, p2 momentum buffer or 0).
constexpr int LARGE_THR = 256;
constexpr int LARGE_MAXT = 512;
constexpr int LARGE_UNROLL = 4;

__global__ void __launch_bounds__(64) amp_table_kernel(int64_t* __restrict__ table, int n, int s, int e,
                                                       MTList c, int64_t off_s, int64_t total) {
  // entries [s, e) of the table from a by-value chunk (graph-capturable, no host copy)
  const int k = threadIdx.x;
  int64_t* off = table + 2;
  int64_t* num = off + n + 1;
  int64_t* q0 = num + n;
  int64_t* q1 = q0 + n;
  int64_t* q2 = q1 + n;
  int64_t* fst = q2 + n;
  if (k == 0 && s == 0) { table[0] = n; table[1] = total; }
  if (k == 0 && e == n) off[n] = total;
  if (k < e - s) {
    const int t = s + k;
    off[t] = off_s + c.chunk_off[k];
    num[t] = c.numel[k];
    q0[t] = reinterpret_cast<int64_t>(c.p0[k]);
    q1[t] = reinterpret_cast<int64_t>(c.p1[k]);
    q2[t] = reinterpret_cast<int64_t>(c.p2[k]);
    fst[t] = (c.first_bits >> k) & 1ull;
  }
}

__global__ void __launch_bounds__(LARGE_THR)
amp_sgd_large_kernel(const int64_t* __restrict__ table, float* __restrict__ scale, int* __restrict__ tracker,
                     float* __restrict__ found_inf, unsigned long long* __restrict__ sync, float lr, float momentum,
                     float dampening, float wd, int nesterov, int maximize, float growth, float backoff, int interval,
                     int* __restrict__ err, long long barrier_ticks) {
  __shared__ long long soff[LARGE_MAXT + 1];
  __shared__ long long snum[LARGE_MAXT];
  __shared__ float* sp0[LARGE_MAXT];
  __shared__ float* sp1[LARGE_MAXT];
  __shared__ float* sp2[LARGE_MAXT];
  __shared__ unsigned char sfirst[LARGE_MAXT];
  __shared__ int s_bad;
  const int tid = threadIdx.x;
  const int n = (int)table[0];
  const long long total = table[1];
  const int64_t* off = table + 2;
  for (int t = tid; t <= n; t += LARGE_THR) soff[t] = off[t];
  for (int t = tid; t < n; t += LARGE_THR) {
    snum[t] = off[n + 1 + t];
    sp0[t] = reinterpret_cast<float*>(off[2 * n + 1 + t]);
    sp1[t] = reinterpret_cast<float*>(off[3 * n + 1 + t]);
    sp2[t] = reinterpret_cast<float*>(off[4 * n + 1 + t]);
    sfirst[t] = (unsigned char)off[5 * n + 1 + t];
  }
  unsigned long long gen = 0;
  if (tid == 0 && gridDim.x > 1)
    gen = __hip_atomic_fetch_add(&sync[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  // this workgroup's granule range, whole lanes-rows so every lane steps by LARGE_THR
  const long long per = ((total + gridDim.x - 1) / gridDim.x + LARGE_THR - 1) / LARGE_THR * LARGE_THR;
  const long long g0 = (long long)blockIdx.x * per, g1 = min(total, g0 + per);
  int t0 = 0;  // tensor holding g0 (binary search once per workgroup)
  if (g0 < total) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (soff[mid] <= g0) lo = mid; else hi = mid - 1;
    }
    t0 = lo;
  }
  auto load4 = [](const float* p, long long rem) {
    if (rem >= 4) return *reinterpret_cast<const f32x4*>(p);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < rem; ++j) v[j] = p[j];
    return v;
  };
  auto store4 = [](float* p, long long rem, f32x4 v) {
    if (rem >= 4) { *reinterpret_cast<f32x4*>(p) = v; return; }
    for (int j = 0; j < rem; ++j) p[j] = v[j];
  };
  // phase A: non-finite check over this range (LARGE_UNROLL granule loads in flight per lane)
  bool bad = false;
  {
    int t = t0;
    for (long long base = g0 + tid; base < g1; base += (long long)LARGE_THR * LARGE_UNROLL) {
      f32x4 v[LARGE_UNROLL];
#pragma unroll
      for (int u = 0; u < LARGE_UNROLL; ++u) {
        const long long gi = base + (long long)u * LARGE_THR;
        v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (gi < g1) {
          while (soff[t + 1] <= gi) ++t;
          const long long o = (gi - soff[t]) * 4;
          v[u] = load4(sp1[t] + o, snum[t] - o);
        }
      }
#pragma unroll
      for (int u = 0; u < LARGE_UNROLL; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) bad |= !isfinite(v[u][j]);
    }
  }
  const float inv = 1.f / scale[0];  // read before arriving (block 0 rewrites it after the barrier)
  const bool block_bad = __syncthreads_or(bad);
  if (gridDim.x == 1) {
    if (tid == 0) s_bad = block_bad;
  } else if (tid == 0) {
    unsigned long long* word = &sync[1 + (gen & 1)];
    const unsigned long long G = gridDim.x;
    __hip_atomic_fetch_add(word, 1ull | ((unsigned long long)block_bad << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long v;
    const long long ts = (long long)__builtin_amdgcn_s_memrealtime();
    bool timed_out = false;
    while (((v = __hip_atomic_fetch_add(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & 0xffffffffull) <
           G) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - ts > barrier_ticks) {
        timed_out = true;
        if (err != nullptr) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    s_bad = timed_out || (v >> 32) != 0;
    if (blockIdx.x == 0) {
      __hip_atomic_exchange(&sync[1 + ((gen + 1) & 1)], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&sync[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  const bool any_bad = s_bad;
  // phase B: unscaled grads written back (torch semantics); the update only if all finite
  {
    int t = t0;
    for (long long base = g0 + tid; base < g1; base += (long long)LARGE_THR * LARGE_UNROLL) {
      f32x4 gv[LARGE_UNROLL], pv[LARGE_UNROLL], bv[LARGE_UNROLL];
      int tt[LARGE_UNROLL];
#pragma unroll
      for (int u = 0; u < LARGE_UNROLL; ++u) {
        const long long gi = base + (long long)u * LARGE_THR;
        tt[u] = -1;
        if (gi < g1) {
          while (soff[t + 1] <= gi) ++t;
          tt[u] = t;
          const long long o = (gi - soff[t]) * 4, rem = snum[t] - o;
          gv[u] = load4(sp1[t] + o, rem);
          if (!any_bad) {
            pv[u] = load4(sp0[t] + o, rem);
            bv[u] = (momentum != 0.f && !sfirst[t]) ? load4(sp2[t] + o, rem) : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
#pragma unroll
      for (int u = 0; u < LARGE_UNROLL; ++u) {
        const int tu = tt[u];
        if (tu < 0) continue;
        const long long o = (base + (long long)u * LARGE_THR - soff[tu]) * 4, rem = snum[tu] - o;
        const f32x4 g = gv[u] * inv;
        store4(sp1[tu] + o, rem, g);
        if (any_bad) continue;
        f32x4 d = maximize ? -g : g;
        if (wd != 0.f) d += wd * pv[u];
        if (momentum != 0.f) {
          const f32x4 bb = sfirst[tu] ? d : momentum * bv[u] + (1.f - dampening) * d;
          store4(sp2[tu] + o, rem, bb);
          d = nesterov ? d + momentum * bb : bb;
        }
        store4(sp0[tu] + o, rem, pv[u] - lr * d);
      }
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    found_inf[0] = 0.f;
    if (any_bad) {
      scale[0] = scale[0] * backoff;
      tracker[0] = 0;
    } else {
      const int succ = tracker[0] + 1;
      if (succ == interval) {
        const float ns = scale[0] * growth;
        if (isfinite(ns)) scale[0] = ns;
        tracker[0] = 0;
      } else {
        tracker[0] = succ;
      }
    }
  }
}

// direction 0: flat[off_t + i] = src_t[i] * s ; direction 1: dst_t[i] = flat[off_t + i] * s
__global__ void __launch_bounds__(NTHR)
flat_copy_kernel(MTList L, float* __restrict__ flat, float s, int direction) {
  const int64_t total = L.chunk_off[L.n];
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const int t = find_tensor(L, c);
    const int64_t base = (c - L.chunk_off[t]) * CHUNK;
    const int64_t end = min(base + (int64_t)CHUNK, L.numel[t]);
    float* ext = L.p0[t];
    float* fl = flat + reinterpret_cast<int64_t>(L.p1[t]);  // p1 carries the element offset
    if (direction == 0)
      for (int64_t i = base + threadIdx.x; i < end; i += NTHR) fl[i] = ext[i] * s;
    else
      for (int64_t i = base + threadIdx.x; i < end; i += NTHR) ext[i] = fl[i] * s;
  }
}

// Build MTList batches of <= MAXT tensors.
template <typename F>
static void for_batches(size_t n, F&& f) {
  for (size_t s = 0; s < n; s += MAXT) f(s, std::min(n, s + MAXT));
}

static int grid_for(int64_t chunks) { return (int)std::max<int64_t>(1, std::min<int64_t>(chunks, 2048)); }

static void check_f32(const at::Tensor& t) {
  DPA_CHECK_INPUT(t);
  TORCH_CHECK(t.scalar_type() == at::kFloat, "optimizer tensors must be f32");
}

void unscale_check(std::vector<at::Tensor> grads, at::Tensor scale, at::Tensor found_inf) {
  check_f32(scale); check_f32(found_inf);
  for_batches(grads.size(), [&](size_t s, size_t e) {
    MTList L{};
    L.n = (int)(e - s);
    L.chunk_off[0] = 0;
    for (size_t i = s; i < e; ++i) {
      check_f32(grads[i]);
      const int k = (int)(i - s);
      L.numel[k] = grads[i].numel();
      L.p0[k] = grads[i].data_ptr<float>();
      L.chunk_off[k + 1] = L.chunk_off[k] + (L.numel[k] + CHUNK - 1) / CHUNK;
    }
    hipLaunchKernelGGL(unscale_check_kernel, dim3(grid_for(L.chunk_off[L.n])), dim3(NTHR), 0, cur_stream(), L,
                       scale.data_ptr<float>(), found_inf.data_ptr<float>());
    DPA_CHECK_LAUNCH();
  });
}

// first: per tensor, 1 = its momentum buffer is new (b = d, torch's first step); empty = none
static unsigned long long first_bits(const std::vector<int64_t>& first, size_t s, size_t e) {
  unsigned long long m = 0;
  for (size_t i = s; i < e && i < first.size(); ++i)
    if (first[i]) m |= 1ull << (i - s);
  return m;
}

void sgd_step(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> bufs,
              double lr, double momentum, double dampening, double wd, bool nesterov, bool maximize,
              std::vector<int64_t> first, c10::optional<at::Tensor> found_inf, c10::optional<at::Tensor> grad_scale) {
  TORCH_CHECK(params.size() == grads.size());
  TORCH_CHECK(bufs.empty() || bufs.size() == params.size());
  TORCH_CHECK(first.empty() || first.size() == params.size(), "sgd_step: one first flag per tensor");
  const float* fi = found_inf.has_value() ? found_inf->data_ptr<float>() : nullptr;
  const float* gsp = grad_scale.has_value() ? grad_scale->data_ptr<float>() : nullptr;
  for_batches(params.size(), [&](size_t s, size_t e) {
    MTList L{};
    L.n = (int)(e - s);
    L.first_bits = first_bits(first, s, e);
    L.chunk_off[0] = 0;
    for (size_t i = s; i < e; ++i) {
      check_f32(params[i]); check_f32(grads[i]);
      TORCH_CHECK(params[i].numel() == grads[i].numel());
      const int k = (int)(i - s);
      L.numel[k] = params[i].numel();
      L.p0[k] = params[i].data_ptr<float>();
      L.p1[k] = grads[i].data_ptr<float>();
      L.p2[k] = bufs.empty() ? nullptr : bufs[i].data_ptr<float>();
      L.chunk_off[k + 1] = L.chunk_off[k] + (L.numel[k] + CHUNK - 1) / CHUNK;
    }
    hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(L.chunk_off[L.n])), dim3(NTHR), 0, cur_stream(), L, (float)lr,
                       (float)momentum, (float)dampening, (float)wd, (int)nesterov, (int)maximize, fi, gsp);
    DPA_CHECK_LAUNCH();
  });
}

// elements the fused AMP-SGD kernel can exchange in one launch (U = 1 granule per lane)
int64_t amp_sgd_xg_max() { return (int64_t)FUSED_MAX_BLOCKS * FUSED_THR * 4; }

// The fused kernel's largest grid (FUSED_MAX_BLOCKS workgroups) is co-resident on this device.
bool amp_sgd_resident() {
  static const bool ok =
      co_resident(reinterpret_cast<const void*>(&amp_sgd_fused_kernel<1, false>), FUSED_MAX_BLOCKS, FUSED_THR) &&
      co_resident(reinterpret_cast<const void*>(&amp_sgd_fused_kernel<2, false>), FUSED_MAX_BLOCKS, FUSED_THR) &&
      co_resident(reinterpret_cast<const void*>(&amp_sgd_fused_kernel<FUSED_U, false>), FUSED_MAX_BLOCKS,
                  FUSED_THR) &&
      co_resident(reinterpret_cast<const void*>(&amp_sgd_fused_kernel<1, true>), FUSED_MAX_BLOCKS, FUSED_THR);
  return ok;
}

// sync: zero-initialised int64[4] device tensor: [0..2] grid-barrier state, [3] low
// word = error (3: a workgroup never reached the barrier within kBarrierSeconds)
constexpr double kBarrierSeconds = 10.0;

void amp_sgd_fused(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> bufs,
                   double lr, double momentum, double dampening, double wd, bool nesterov, bool maximize,
                   std::vector<int64_t> first, at::Tensor scale, at::Tensor tracker, at::Tensor found_inf,
                   double growth, double backoff, int64_t interval, at::Tensor sync,
                   std::shared_ptr<xgmi::XgmiComm> xc, c10::optional<at::Tensor> slab, c10::optional<at::Tensor> slab_out) {
  TORCH_CHECK(params.size() == grads.size() && params.size() <= (size_t)MAXT, "fused AMP-SGD: <= ", MAXT,
              " tensors");
  TORCH_CHECK(bufs.empty() || bufs.size() == params.size());
  TORCH_CHECK(first.empty() || first.size() == params.size(), "fused AMP-SGD: one first flag per tensor");
  check_f32(scale); check_f32(found_inf);
  TORCH_CHECK(tracker.scalar_type() == at::kInt);
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kLong && sync.numel() >= 4 && sync.is_contiguous(),
              "fused AMP-SGD: sync must be a zero-initialised int64[4] device tensor");
  TORCH_CHECK(amp_sgd_resident(), "fused AMP-SGD: grid not co-resident on this device (use the unfused step)");
  MTList L{};
  L.n = (int)params.size();
  L.first_bits = first_bits(first, 0, params.size());
  L.chunk_off[0] = 0;
  for (size_t i = 0; i < params.size(); ++i) {
    check_f32(params[i]); check_f32(grads[i]);
    TORCH_CHECK(params[i].numel() == grads[i].numel());
    L.numel[i] = params[i].numel();
    L.p0[i] = params[i].data_ptr<float>();
    L.p1[i] = grads[i].data_ptr<float>();
    L.p2[i] = bufs.empty() ? nullptr : bufs[i].data_ptr<float>();
    L.chunk_off[i + 1] = L.chunk_off[i] + (L.numel[i] + 3) / 4;  // float4-granule prefix for this kernel
    TORCH_CHECK(momentum == 0.0 || !bufs.empty(), "fused AMP-SGD: momentum needs buffers");
    auto al = [](const float* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    TORCH_CHECK(al(L.p0[i]) && al(L.p1[i]) && al(L.p2[i]), "fused AMP-SGD needs 16-byte aligned tensors");
  }
  TORCH_CHECK(L.chunk_off[L.n] * 4 <= FUSED_MAX, "fused AMP-SGD handles at most ", FUSED_MAX, " elements");
  SlabSrc ss{nullptr, nullptr, 0, 0, 0};
  TORCH_CHECK(slab.has_value() == slab_out.has_value(), "fused AMP-SGD: slab and slab_out go together");
  if (slab.has_value()) {
    check_f32(*slab); check_f32(*slab_out);
    const int64_t ncol = slab_out->numel();
    TORCH_CHECK(ncol > 0 && slab->numel() % ncol == 0, "fused AMP-SGD: slab must be [rows][slab_out.numel()]");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(slab_out->data_ptr()) & 15) == 0, "fused AMP-SGD: slab_out alignment");
    // the region must start and end on granule boundaries of the tensors that cover it
    const float* lo = slab_out->data_ptr<float>();
    const float* hi = lo + ncol;
    for (int i = 0; i < L.n; ++i) {
      const float* a = L.p1[i];
      const float* b = a + L.numel[i];
      if (b <= lo || a >= hi) continue;
      TORCH_CHECK(a >= lo && b <= hi && (L.numel[i] % 4 == 0 || b == hi),
                  "fused AMP-SGD: every gradient overlapping slab_out must lie inside it, in whole granules");
    }
    ss = SlabSrc{slab->data_ptr<float>(), slab_out->data_ptr<float>(), (int)(slab->numel() / ncol), (int)ncol,
                 (int)((ncol + SS_COLS - 1) / SS_COLS)};
  }
  auto launch = [&](auto kern, int bg, xgmi::XSite xg) {
    const int grid = (int)std::max<int64_t>(1, (L.chunk_off[L.n] + bg - 1) / bg) + ss.nblk;
    TORCH_CHECK(grid <= FUSED_MAX_BLOCKS, "fused AMP-SGD: grid exceeds the co-resident bound");
    if (xg.active()) xg.nblk = grid;  // every workgroup takes a ticket (no hidden-argument load)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(FUSED_THR), 0, cur_stream(), L, scale.data_ptr<float>(),
                       tracker.data_ptr<int>(), found_inf.data_ptr<float>(),
                       reinterpret_cast<unsigned long long*>(sync.data_ptr<int64_t>()), (float)lr, (float)momentum,
                       (float)dampening, (float)wd, (int)nesterov, (int)maximize, (float)growth, (float)backoff,
                       (int)interval, xg, reinterpret_cast<int*>(sync.data_ptr<int64_t>() + 3),
                       (long long)(kBarrierSeconds * 1e8), ss, grid);
  };
  if (xc) {
    const xgmi::XSite xg = xc->grad_site();
    TORCH_CHECK(L.chunk_off[L.n] * 4 <= std::min<int64_t>(xg.max_vals, amp_sgd_xg_max()),
                "fused AMP-SGD gradient exchange: too many elements for the xGMI engine");
    launch(amp_sgd_fused_kernel<1, true>, FUSED_THR, xg);
  } else {
    // Granules per lane: the smallest U whose grid fits FUSED_MAX_BLOCKS.  More workgroups
    // = more CUs pulling the grads/params through; the barrier's extra arrivals cost less
    // (ConvNet step: U=4 0.0868 ms, U=2 0.0850, U=1 0.0841).  DPA_SGD_U=1|2|4 forces one.
    static const int su = [] {
      const char* e = std::getenv("DPA_SGD_U");
      return e != nullptr ? std::atoi(e) : 0;
    }();
    const int64_t gran = L.chunk_off[L.n];
    if ((su == 0 || su == 1) && gran <= (int64_t)FUSED_MAX_BLOCKS * FUSED_THR)
      launch(amp_sgd_fused_kernel<1, false>, FUSED_THR, xgmi::XSite{});
    else if ((su == 0 || su == 2) && gran <= (int64_t)FUSED_MAX_BLOCKS * FUSED_THR * 2)
      launch(amp_sgd_fused_kernel<2, false>, FUSED_THR * 2, xgmi::XSite{});
    else
      launch(amp_sgd_fused_kernel<FUSED_U, false>, FUSED_BLOCK_GRAN, xgmi::XSite{});
  }
  DPA_CHECK_LAUNCH();
}

// Grid of the large fused step: 2 workgroups per CU when both fit at once, else 1.
static int large_grid() {
  static const int g = [] {
    int dev = 0, cus = 0;
    DPA_CHECK_HIP(hipGetDevice(&dev));
    DPA_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const void* k = reinterpret_cast<const void*>(&amp_sgd_large_kernel);
    for (int per = 2; per >= 1; --per)
      if (co_resident(k, cus * per, LARGE_THR)) return cus * per;
    return 0;
  }();
  return g;
}

bool amp_sgd_large_resident() { return large_grid() > 0; }

// Device table for amp_sgd_large: written by by-value upload launches (one per MAXT
// tensors), so building it is stream-ordered and graph-capturable.
at::Tensor amp_sgd_table(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> bufs,
                         std::vector<int64_t> first) {
  const size_t n = params.size();
  TORCH_CHECK(n >= 1 && n <= (size_t)LARGE_MAXT, "large fused AMP-SGD: 1..", LARGE_MAXT, " tensors");
  TORCH_CHECK(grads.size() == n && (bufs.empty() || bufs.size() == n) && (first.empty() || first.size() == n));
  auto al = [](const float* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  std::vector<int64_t> offs(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    check_f32(params[i]); check_f32(grads[i]);
    TORCH_CHECK(params[i].numel() == grads[i].numel());
    if (!bufs.empty()) { check_f32(bufs[i]); TORCH_CHECK(bufs[i].numel() == params[i].numel()); }
    TORCH_CHECK(al(params[i].data_ptr<float>()) && al(grads[i].data_ptr<float>()) &&
                    (bufs.empty() || al(bufs[i].data_ptr<float>())),
                "large fused AMP-SGD needs 16-byte aligned tensors");
    offs[i + 1] = offs[i] + (params[i].numel() + 3) / 4;
  }
  auto table = at::empty({(int64_t)(2 + (n + 1) + 5 * n)}, params[0].options().dtype(at::kLong));
  for_batches(n, [&](size_t s, size_t e) {
    MTList c{};
    c.n = (int)(e - s);
    c.first_bits = first_bits(first, s, e);
    for (size_t i = s; i < e; ++i) {
      const int k = (int)(i - s);
      c.numel[k] = params[i].numel();
      c.chunk_off[k] = offs[i] - offs[s];
      c.p0[k] = params[i].data_ptr<float>();
      c.p1[k] = grads[i].data_ptr<float>();
      c.p2[k] = bufs.empty() ? nullptr : bufs[i].data_ptr<float>();
    }
    hipLaunchKernelGGL(amp_table_kernel, dim3(1), dim3(64), 0, cur_stream(), table.data_ptr<int64_t>(), (int)n,
                       (int)s, (int)e, c, offs[s], offs[n]);
    DPA_CHECK_LAUNCH();
  });
  return table;
}

void amp_sgd_large(at::Tensor table, double lr, double momentum, double dampening, double wd, bool nesterov,
                   bool maximize, at::Tensor scale, at::Tensor tracker, at::Tensor found_inf, double growth,
                   double backoff, int64_t interval, at::Tensor sync) {
  check_f32(scale); check_f32(found_inf);
  TORCH_CHECK(tracker.scalar_type() == at::kInt);
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong, "large fused AMP-SGD: table from amp_sgd_table");
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kLong && sync.numel() >= 4 && sync.is_contiguous(),
              "large fused AMP-SGD: sync must be a zero-initialised int64[4] device tensor");
  const int grid = large_grid();
  TORCH_CHECK(grid > 0, "large fused AMP-SGD: grid not co-resident on this device (use the unfused step)");
  hipLaunchKernelGGL(amp_sgd_large_kernel, dim3(grid), dim3(LARGE_THR), 0, cur_stream(), table.data_ptr<int64_t>(),
                     scale.data_ptr<float>(), tracker.data_ptr<int>(), found_inf.data_ptr<float>(),
                     reinterpret_cast<unsigned long long*>(sync.data_ptr<int64_t>()), (float)lr, (float)momentum,
                     (float)dampening, (float)wd, (int)nesterov, (int)maximize, (float)growth, (float)backoff,
                     (int)interval, reinterpret_cast<int*>(sync.data_ptr<int64_t>() + 3),
                     (long long)(kBarrierSeconds * 1e8));
  DPA_CHECK_LAUNCH();
}

void update_scale(at::Tensor scale, at::Tensor tracker, at::Tensor found_inf, double growth, double backoff,
                  int64_t interval) {
  check_f32(scale); check_f32(found_inf);
  TORCH_CHECK(tracker.scalar_type() == at::kInt);
  hipLaunchKernelGGL(update_scale_kernel, dim3(1), dim3(64), 0, cur_stream(), scale.data_ptr<float>(),
                     tracker.data_ptr<int>(), found_inf.data_ptr<float>(), (float)growth, (float)backoff,
                     (int)interval);
  DPA_CHECK_LAUNCH();
}

// Copy tensors into (direction 0) / out of (direction 1) a flat f32 buffer at
// the given element offsets, multiplying by `s`.
void flat_copy(std::vector<at::Tensor> tensors, std::vector<int64_t> offsets, at::Tensor flat, double s,
               int64_t direction) {
  check_f32(flat);
  TORCH_CHECK(tensors.size() == offsets.size());
  for_batches(tensors.size(), [&](size_t b, size_t e) {
    MTList L{};
    L.n = (int)(e - b);
    L.chunk_off[0] = 0;
    for (size_t i = b; i < e; ++i) {
      check_f32(tensors[i]);
      TORCH_CHECK(offsets[i] + tensors[i].numel() <= flat.numel());
      const int k = (int)(i - b);
      L.numel[k] = tensors[i].numel();
      L.p0[k] = tensors[i].data_ptr<float>();
      L.p1[k] = reinterpret_cast<float*>(offsets[i]);
      L.chunk_off[k + 1] = L.chunk_off[k] + (L.numel[k] + CHUNK - 1) / CHUNK;
    }
    hipLaunchKernelGGL(flat_copy_kernel, dim3(grid_for(L.chunk_off[L.n])), dim3(NTHR), 0, cur_stream(), L,
                       flat.data_ptr<float>(), (float)s, (int)direction);
    DPA_CHECK_LAUNCH();
  });
}

}  // namespace opt

void register_optim(pybind11::module& m) {
  auto s = m.def_submodule("optim", "multi-tensor SGD / AMP GradScaler kernels");
  s.def("unscale_check", &opt::unscale_check);
  s.def("sgd_step", &opt::sgd_step, pybind11::arg("params"), pybind11::arg("grads"), pybind11::arg("bufs"),
        pybind11::arg("lr"), pybind11::arg("momentum"), pybind11::arg("dampening"), pybind11::arg("weight_decay"),
        pybind11::arg("nesterov"), pybind11::arg("maximize"), pybind11::arg("first") = std::vector<int64_t>{},
        pybind11::arg("found_inf") = pybind11::none(), pybind11::arg("grad_scale") = pybind11::none());
  s.def("update_scale", &opt::update_scale);
  s.def("amp_sgd_fused", &opt::amp_sgd_fused, pybind11::arg("params"), pybind11::arg("grads"), pybind11::arg("bufs"),
        pybind11::arg("lr"), pybind11::arg("momentum"), pybind11::arg("dampening"), pybind11::arg("wd"),
        pybind11::arg("nesterov"), pybind11::arg("maximize"), pybind11::arg("first"), pybind11::arg("scale"),
        pybind11::arg("tracker"), pybind11::arg("found_inf"), pybind11::arg("growth"), pybind11::arg("backoff"),
        pybind11::arg("interval"), pybind11::arg("sync"), pybind11::arg("xc"),
        pybind11::arg("slab") = pybind11::none(), pybind11::arg("slab_out") = pybind11::none());
  s.def("amp_sgd_xg_max", &opt::amp_sgd_xg_max);
  s.def("amp_sgd_resident", &opt::amp_sgd_resident);
  s.def("amp_sgd_table", &opt::amp_sgd_table, pybind11::arg("params"), pybind11::arg("grads"), pybind11::arg("bufs"),
        pybind11::arg("first") = std::vector<int64_t>{});
  s.def("amp_sgd_large", &opt::amp_sgd_large);
  s.def("amp_sgd_large_resident", &opt::amp_sgd_large_resident);
  s.attr("LARGE_MAXT") = opt::LARGE_MAXT;
  s.attr("FUSED_MAX") = opt::FUSED_MAX;
  s.attr("MAXT") = opt::MAXT;
  s.def("flat_copy", &opt::flat_copy);
}

}  // namespace dpa
