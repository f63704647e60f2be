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
#include "kernels/amp_step.h"

#include <vector>

namespace dpa {
namespace opt {

constexpr int NTHR = 256;
constexpr int CHUNK = 4096;

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
      float b = bv0[k];
      p[i] = sgd_rule(pv[k], gv[k] * gs, b, first, lr, momentum, dampening, wd, nesterov, maximize);
      if (momentum != 0.f) buf[i] = b;
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

// GradScaler.step + SGD + GradScaler.update in ONE launch over a small grid (the
// ConvNet: 29,034 floats), csrc/kernels/amp_step.h amp_sgd_body.  One optional slab
// source (ss.ns <= 1): the ConvNet's conv1 weight-gradient slab (optim/sgd.py defer_slab).
template <int U, bool XG, int THR = FUSED_THR>
__global__ void __launch_bounds__(THR)
amp_sgd_fused_kernel(MTList L, float* __restrict__ scale, int* __restrict__ tracker, float* __restrict__ found_inf,
                     unsigned long long* __restrict__ sync, float lr, float momentum, float dampening, float wd,
                     int nesterov, int maximize, float growth, float backoff, int interval,
                     xgmi::XSite xg, int* __restrict__ err, long long barrier_ticks, SlabSet ss, int grid,
                     const int* __restrict__ chk, int nchk) {
  // grid == the launch's workgroup count, passed in: gridDim is a load from the hidden kernel
  // arguments on gfx950, and its wait at the top of the kernel came before the table loads
  DPA_STAMP(0);
  amp_sgd_body<U, XG, THR>(L, scale, tracker, found_inf, sync, lr, momentum, dampening, wd, nesterov, maximize,
                           growth, backoff, interval, xg, err, barrier_ticks, ss, grid, (int)blockIdx.x, chk, nchk);
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
        f32x4 pn = pv[u], bb = bv[u];
        sgd_rule4(pn, g, bb, sfirst[tu], lr, momentum, dampening, wd, nesterov, maximize);
        if (momentum != 0.f) store4(sp2[tu] + o, rem, bb);
        store4(sp0[tu] + o, rem, pn);
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
                   std::vector<int64_t> first, c10::optional<at::Tensor> scale, c10::optional<at::Tensor> tracker,
                   c10::optional<at::Tensor> found_inf, double growth, double backoff, int64_t interval,
                   at::Tensor sync, std::shared_ptr<xgmi::XgmiComm> xc, c10::optional<at::Tensor> slab,
                   c10::optional<at::Tensor> slab_out, c10::optional<at::Tensor> prechk) {
  TORCH_CHECK(params.size() == grads.size() && params.size() <= (size_t)MAXT, "fused AMP-SGD: <= ", MAXT,
              " tensors");
  TORCH_CHECK(bufs.empty() || bufs.size() == params.size());
  TORCH_CHECK(first.empty() || first.size() == params.size(), "fused AMP-SGD: one first flag per tensor");
  // no scale: the plain SGD step (amp_step.h amp_sgd_body), tracker / found_inf unused
  const bool amp = scale.has_value();
  TORCH_CHECK(tracker.has_value() == amp && found_inf.has_value() == amp,
              "fused SGD: scale, tracker and found_inf go together");
  if (amp) {
    check_f32(*scale); check_f32(*found_inf);
    TORCH_CHECK(tracker->scalar_type() == at::kInt);
  }
  float* const sc = amp ? scale->data_ptr<float>() : nullptr;
  int* const tr = amp ? tracker->data_ptr<int>() : nullptr;
  float* const fi = amp ? found_inf->data_ptr<float>() : nullptr;
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kLong && sync.numel() >= 4 && sync.is_contiguous(),
              "fused AMP-SGD: sync must be a zero-initialised int64[4] device tensor");
  // prechk: the producer kernels' gradient-check words + the scale they used (common.h GradChk)
  const int* chk = nullptr;
  int nchk = 0;
  if (prechk.has_value()) {
    DPA_CHECK_INPUT(*prechk);
    TORCH_CHECK(amp && prechk->scalar_type() == at::kInt && prechk->numel() >= 2,
                "fused AMP-SGD: pre-checked gradients need the scaler and int32 words");
    chk = prechk->data_ptr<int>();
    nchk = (int)prechk->numel() - 1;
  }
  TORCH_CHECK(amp_sgd_resident(), "fused AMP-SGD: grid not co-resident on this device (use the unfused step)");
  MTList L = fused_list(params, grads, bufs, first, momentum);
  SlabSet ss;
  TORCH_CHECK(slab.has_value() == slab_out.has_value(), "fused AMP-SGD: slab and slab_out go together");
  if (slab.has_value()) add_slab(ss, L, *slab, *slab_out, 16, 1, nullptr, 0);
  auto launch = [&](auto kern, int bg, xgmi::XSite xg) {
    const int grid = (int)std::max<int64_t>(1, (L.chunk_off[L.n] + bg - 1) / bg) + (ss.ns ? ss.s[0].nblk : 0);
    TORCH_CHECK(grid <= FUSED_MAX_BLOCKS, "fused AMP-SGD: grid exceeds the co-resident bound");
    xgmi::set_site_grid(xg, grid, "fused AMP-SGD");  // every workgroup takes a ticket (no hidden-argument load)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(FUSED_THR), 0, cur_stream(), L, sc, tr, fi,
                       reinterpret_cast<unsigned long long*>(sync.data_ptr<int64_t>()), (float)lr, (float)momentum,
                       (float)dampening, (float)wd, (int)nesterov, (int)maximize, (float)growth, (float)backoff,
                       (int)interval, xg, reinterpret_cast<int*>(sync.data_ptr<int64_t>() + 3),
                       (long long)(kBarrierSeconds * 1e8), ss, grid, chk, nchk);
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
    cus = resident_cus(cus);
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
        pybind11::arg("slab") = pybind11::none(), pybind11::arg("slab_out") = pybind11::none(),
        pybind11::arg("prechk") = pybind11::none());
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
  DPA_DEF_STAMP_FNS(s);
}

}  // namespace dpa
