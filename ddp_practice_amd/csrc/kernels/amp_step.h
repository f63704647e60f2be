// The fused AMP optimizer step (GradScaler.step + SGD + GradScaler.update in ONE
// launch), shared by csrc/kernels/optim.hip (amp_sgd_fused: any small parameter set)
// and csrc/kernels/convnet_fused.hip (convnet_amp_step: the ConvNet's step with the
// conv1 weight gradient computed by producer workgroups of the same launch).
// Reference call sites: /root/reference/ddp_main.py:91-93 (scaler.scale/step/update),
// origin_main.py:87 (SGD lr=1e-4); torch semantics: torch/amp/grad_scaler.py:235-286,
// 348-357, 500-537 and torch/optim/sgd.py:471.
#pragma once
#include <vector>

#include "common.h"
#include "comm/xsite.h"

namespace dpa {
namespace opt {

constexpr int MAXT = 36;

struct MTList {
  int n;
  unsigned long long first_bits;  // momentum: bit t set = tensor t's buffer is new (b = d)
  int64_t numel[MAXT];
  int64_t chunk_off[MAXT + 1];  // prefix sum of chunks
  float* p0[MAXT];
  float* p1[MAXT];
  float* p2[MAXT];
};

// Every lane loads its grads, params (and momentum buffers) into registers, the
// workgroups agree on found_inf through ONE 64-bit device-scope atomic per generation
// ({arrivals, non-finite workgroups} in one word: no fence, no flag), and then each
// applies its own slice: unscaled grads written back (torch semantics), the update
// applied only if every grad is finite, scale / growth tracker updated and found_inf
// re-armed by workgroup 0.  p0 = param, p1 = grad, p2 = momentum buffer (or null).
//
// Grid barrier state `sync` (int64[3], zero-initialised, one per optimizer and grid
// size): [0] launch counter g, [1 + (g & 1)] this launch's word.  Block 0 resets the
// other parity's word and bumps g after the barrier; the next launch is stream-ordered
// after this one, so it always finds its word at zero.  The AMP workgroups (<=
// FUSED_MAX_BLOCKS of 256 lanes) are co-resident.
constexpr int FUSED_THR = 256;
constexpr int FUSED_U = 4;                                  // float4 granules per lane
constexpr int FUSED_BLOCK_GRAN = FUSED_THR * FUSED_U;       // 4096 floats per workgroup
constexpr int FUSED_MAX_BLOCKS = 128;
constexpr int64_t FUSED_MAX = (int64_t)FUSED_MAX_BLOCKS * FUSED_BLOCK_GRAN * 4;
// (A one-workgroup variant of 1024 lanes x 8 granules for the ConvNet measured 10.9 us
// vs 8.6 us for 8 workgroups + grid barrier: one CU's bandwidth is the limit, not the
// barrier.  A grid of one still skips the barrier, below.)

// The flat index space is in float4 granules; tensor t owns ceil(numel/4) granules
// starting at chunk_off[t] (every pointer 16-B aligned, checked on the host), so a
// granule never straddles two tensors.  Tensor tables live in LDS (per-lane dynamic
// indexing of the by-value kernel argument is a chain of dependent scalar loads).
//
// XG (DDP over the xGMI engine, DistributedDataParallel.defer_grad_sync_to): the
// gradient all-reduce is fused in as well.  Each lane pushes its local gradient
// granules to every peer as {value, epoch} granules (the one-shot protocol of
// comm/xgmi_allreduce.hip, epoch from comm/xsite.h tickets), then sums the W ranks'
// values in rank order and divides by W before the inf check -- the reducer launched
// no collective for these buckets.  U = 1 granule per lane then.
//
// Slab sources (optional, up to kMaxSlabs): a gradient region [out, out + n) that is
// still the per-workgroup partial rows of its producer (slab [rows][n]: e.g. the
// ConvNet's weight-gradient slabs).  nblk extra workgroups per source, appended after
// the granule workgroups, own it -- they sum its columns (`cols` columns x 256/cols row
// groups each), check them, load the matching params / buffers, take part in the
// gradient exchange (XG: one granule per element, at the element's position in the
// flat granule space), arrive at the grid barrier like the others and then apply the
// same update per element (unscaled gradient written to `out`).  The granule
// workgroups skip the regions, and the separate column-sum launches disappear.  A
// source with `wait` is produced IN THIS LAUNCH: its owners first wait (bounded) until
// the producers' arrival counter reaches wait_n and then read the rows with L2-coherent
// (sc1) loads; block 0 re-arms the counter after the barrier.
// Association: a column is summed over rows g, g + G, ... (g < G row groups of 256/G lanes)
// and the G partials are added in group order -- slab_reduce's (G = 16) and the BN
// backward-coefficient reduction's (cb::colsum_rows over 2C = 32 columns: G = 8), so a
// gradient summed here is bitwise the one the separate launches produce (the flush path).
struct SlabSrc {
  const float* slab = nullptr;
  float* out = nullptr;
  int rows = 0, n = 0, nblk = 0;
  int groups = 16;            // row groups G: 16 (16 columns per chunk) or 8 (32 columns)
  int chunks = 1;             // column chunks per workgroup: 1 or 4 (G = 16)
  const int* wait = nullptr;  // in-launch producers' arrival counter (nullptr: rows ready)
  int wait_n = 0;
};
constexpr int kMaxSlabs = 3;
struct SlabSet {
  SlabSrc s[kMaxSlabs];
  int ns = 0;
  int* rearm = nullptr;  // producer counter zeroed by block 0 after the barrier
  int blanes = 1;        // grid-barrier arrival words (> 1: kBarStride u64 apart, sync holds
                         // 1 + 2 * blanes * kBarStride words): arrivals of a few hundred
                         // workgroups on ONE word serialise (~10 ns each)
};
constexpr int kBarStride = 8;  // u64: 64 B

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// K column chunks of CC = 256/G columns at c0, c0 + CC, ...: this lane's column of each
// chunk (c0 + j*CC + tid % CC) summed over rows g, g + G, ... in that order, g = tid / CC.
// Every chunk's first 16 rows per lane are loaded before any add (one round trip for the
// ConvNet's <= 16 G-row slabs); clamped, masked.  SC1: L2-coherent loads (rows written by
// other workgroups of this launch).
template <int G, int K, bool SC1>
__device__ __forceinline__ void slab_colsum_k(const float* __restrict__ slab, int rows, int n, int c0, float* out) {
  constexpr int CC = 256 / G;
  const int g = threadIdx.x / CC, cl = threadIdx.x % CC;
  float v[K][16];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int cc = min(c0 + j * CC + cl, n - 1);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float* p = slab + (size_t)min(g + u * G, rows - 1) * n + cc;
      v[j][u] = SC1 ? ld_sc1(p) : *p;
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int cc = min(c0 + j * CC + cl, n - 1);
    float a = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) a += (g + u * G < rows) ? v[j][u] : 0.f;
    for (int r = g + 16 * G; r < rows; r += G) {  // slabs taller than 16 G rows
      const float* p = slab + (size_t)r * n + cc;
      a += SC1 ? ld_sc1(p) : *p;
    }
    out[j] = a;
  }
}

// bid: this workgroup's index among the launch's AMP workgroups; grid: their count.
template <int U, bool XG, int THR = FUSED_THR>
__device__ __forceinline__ void
amp_sgd_body(const MTList& L, float* __restrict__ scale, int* __restrict__ tracker, float* __restrict__ found_inf,
             unsigned long long* __restrict__ sync, float lr, float momentum, float dampening, float wd, int nesterov,
             int maximize, float growth, float backoff, int interval, const xgmi::XSite& xg, int* __restrict__ err,
             long long barrier_ticks, const SlabSet& ss, int grid, int bid, const int* __restrict__ chk = nullptr,
             int nchk = 0) {
  constexpr int BG = THR * U;  // float4 granules per workgroup
  __shared__ int soff[MAXT + 1];
  __shared__ int snum[MAXT];
  __shared__ float* sp0[MAXT];
  __shared__ float* sp1[MAXT];
  __shared__ float* sp2[MAXT];
  __shared__ int s_bad;
  __shared__ float spart[16 * 65];   // slab workgroups: G row groups x (columns + 1)
  const int tid = threadIdx.x;
  const int n = L.n;
  // scale == nullptr: the plain (unscaled fp32) SGD step -- no unscale, no non-finite
  // agreement, no grid barrier, no scale update: torch.optim.SGD's semantics, with the
  // slab sums and the DDP average (XG) still inside this launch.  A workgroup whose slab
  // producers or peers never arrived (error word set) skips its own update only.
  const bool amp = scale != nullptr;
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
  DPA_STAMP(9);
  const int total = soff[n];
  // the barrier generation is only used by lane 0: issued after the table
  // barrier, its load stays in flight (no LDS round trip) with the gradients'
  unsigned long long gen = 0;
  if (tid == 0 && grid > 1 && amp)
    gen = __hip_atomic_fetch_add(&sync[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long tk = 0;
  if (XG && tid == 0) tk = xgmi::xsite_ticket(xg, bid);
  // chk (pre-checked gradients, common.h GradChk): the producers' words -- every workgroup
  // reads all of them, so all agree on found_inf with no grid barrier -- and the scale of the
  // step (word nchk: block 0 may rewrite scale[0] while a late workgroup starts).  Valid for
  // a scale >= 1 only (the words describe the scaled values): else the barrier, as without
  bool cbad = false;
  float cscale = 1.f;
  if (chk != nullptr) {
    for (int i = tid; i < nchk; i += THR) cbad |= chk[i] != 0;
    cscale = __int_as_float(chk[nchk]);
  }
  const bool pre = chk != nullptr && cscale >= 1.f;  // uniform: every workgroup reads the same word
  // XG: a flagged rank pushes NaN in place of its values, so every peer's workgroup sees a
  // non-finite average of each element it owns and skips -- the ranks agree without a word
  // exchange (the producers' bound keeps a sum of W checked values finite)
  const bool poison = XG && pre && cbad;
  const float nanf_ = __int_as_float(0x7fc00000);
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
  auto in_slab = [&](const float* gp) {
#pragma unroll
    for (int s = 0; s < kMaxSlabs; ++s)
      if (s < ss.ns && gp >= ss.s[s].out && gp < ss.s[s].out + ss.s[s].n) return true;
    return false;
  };
  f32x4 gv[U], pv[U], bv[U];
  int tt[U];  // tensor of each granule (its offset is recomputed after the barrier)
  bool bad = false;
  int nslab = 0;
#pragma unroll
  for (int s = 0; s < kMaxSlabs; ++s) nslab += s < ss.ns ? ss.s[s].nblk : 0;
  const int nreg = grid - nslab;  // granule workgroups; the rest own the slab regions
  // slab workgroup lane (< cols): its column's sum, tensor and element, param / buffer
  float st_sum = 0.f, st_p = 0.f, st_b = 0.f;
  int st_t = -1, st_e = 0;
  bool wait_fail = false;  // lane 0 of a slab workgroup whose producers never all arrived
  if (bid >= nreg) {
    int si = 0, base = nreg;
#pragma unroll
    for (int s = 0; s + 1 < kMaxSlabs; ++s)
      if (si == s && s + 1 < ss.ns && bid >= base + ss.s[s].nblk) {
        base += ss.s[s].nblk;
        si = s + 1;
      }
    const SlabSrc S = ss.s[si];
    const int G = S.groups, CC = THR / G, K = S.chunks, cols = CC * K;
    const int c0 = (bid - base) * cols;
    const int col = c0 + tid;  // the column this lane owns (tid < cols)
    if (tid < cols && col < S.n) {  // param / buffer loads in flight with the slab's
      const float* gp = S.out + col;
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
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const bool sc1 = S.wait != nullptr;
    if (sc1) {
      // rows produced in this launch: wait (bounded) for every producer's arrival
      if (tid == 0) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(S.wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S.wait_n) {
          __builtin_amdgcn_s_sleep(1);
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > barrier_ticks) {
            if (err != nullptr) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            wait_fail = true;  // the rows are incomplete: the step must be skipped
            break;
          }
        }
      }
      __syncthreads();
      DPA_STAMP(10);
    }
    if (G == 8)
      slab_colsum_k<8, 1, false>(S.slab, S.rows, S.n, c0, v);
    else if (K == 4)
      slab_colsum_k<16, 4, false>(S.slab, S.rows, S.n, c0, v);
    else if (sc1)
      slab_colsum_k<16, 1, true>(S.slab, S.rows, S.n, c0, v);
    else
      slab_colsum_k<16, 1, false>(S.slab, S.rows, S.n, c0, v);
    const int g = tid / CC, cl = tid % CC;
    for (int j = 0; j < K; ++j) spart[g * (cols + 1) + j * CC + cl] = v[j];
    __syncthreads();
    if (tid < cols && col < S.n) {
      for (int gg = 0; gg < G; ++gg) st_sum += spart[gg * (cols + 1) + tid];
      bad = amp && !isfinite(st_sum);
    }
    bad |= wait_fail;
#pragma unroll
    for (int k = 0; k < U; ++k) tt[k] = -1;
  } else {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int gi = bid * BG + k * THR + tid;
      tt[k] = -1;
      if (gi < total) {
        int lo = 0, hi = n - 1;  // tensor holding granule gi
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (soff[mid] <= gi) lo = mid; else hi = mid - 1;
        }
        const int o = (gi - soff[lo]) * 4, rem = snum[lo] - o;
        const float* gp = sp1[lo] + o;
        if (in_slab(gp)) continue;  // the slab workgroups own it
        tt[k] = lo;
        gv[k] = load4(gp, rem);
        pv[k] = load4(sp0[lo] + o, rem);
        const bool use_buf = momentum != 0.f && !((L.first_bits >> lo) & 1ull);
        bv[k] = use_buf ? load4(sp2[lo] + o, rem) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  DPA_STAMP(11);
  if constexpr (XG && !xgmi::kXsNoop) {
    __shared__ uint32_t ep_x;
    if (tid == 0) ep_x = xgmi::xsite_epoch(xg, tk, bid);
#ifdef DPA_XG_LDSBAR
    // LDS-only broadcast of the epoch: the gradient / parameter loads above stay in flight
    // while the epoch words are stored and the peers' granules are polled
    DPA_XS_BARRIER();
#else
    __syncthreads();
#endif
    const uint32_t ep = ep_x;
    xgmi::xsite_advance(xg, ep, bid, THR);
    const long long par = (long long)(ep & 1u) * xgmi::kMaxRanks * xg.slot_bytes;
    auto gran = [ep](float v) { return ((unsigned long long)ep << 32) | (unsigned long long)__float_as_uint(v); };
    typedef __attribute__((ext_vector_type(2))) unsigned long long u64x2;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (tt[k] < 0) continue;
      const long long fo = (long long)(bid * BG + k * THR + tid) * 32;  // 4 granules of 8 B
      const f32x4 pv_ = poison ? f32x4{nanf_, nanf_, nanf_, nanf_} : gv[k];
      const u64x2 a = {gran(pv_[0]), gran(pv_[1])}, b = {gran(pv_[2]), gran(pv_[3])};
      for (int p = 0; p < xg.world; ++p) {
        if (p == xg.rank) continue;  // my own values stay in registers
        unsigned long long* dst =
            reinterpret_cast<unsigned long long*>(xg.base[p] + par + (long long)xg.rank * xg.slot_bytes + fo);
        xgmi::xgmi_put2(dst, a[0], a[1]);
        xgmi::xgmi_put2(dst + 2, b[0], b[1]);
      }
    }
    const float invw = 1.f / (float)xg.world;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned polls = 0;
    bool fail = false;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (tt[k] < 0) continue;
      const long long fo = (long long)(bid * BG + k * THR + tid) * 32;
      unsigned long long g[xgmi::kMaxRanks][4];
      const unsigned long long* src[xgmi::kMaxRanks];
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {  // every load issued before the first tag check
        src[p] = reinterpret_cast<const unsigned long long*>(xg.mine + par + (long long)p * xg.slot_bytes +
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
      // at the element's position in the flat granule space -- the slab regions need no
      // separate column-sum launch at W > 1 either
      const long long fo = (long long)(soff[st_t] + st_e / 4) * 32 + (long long)(st_e % 4) * 8;
      const unsigned long long gm = gran(poison ? nanf_ : st_sum);
      for (int p = 0; p < xg.world; ++p) {
        if (p == xg.rank) continue;
        xgmi::xgmi_put(reinterpret_cast<unsigned long long*>(xg.base[p] + par + (long long)xg.rank * xg.slot_bytes + fo),
                       gm);
      }
      unsigned long long g[xgmi::kMaxRanks];
      const unsigned long long* src[xgmi::kMaxRanks];
#pragma unroll
      for (int p = 0; p < xgmi::kMaxRanks; ++p) {
        src[p] = reinterpret_cast<const unsigned long long*>(xg.mine + par + (long long)p * xg.slot_bytes +
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
      bad |= amp && !isfinite(st_sum);
    }
    // a peer that never arrived (timeout / abort: error word set) leaves a partial sum:
    // take the skip path (no parameter / momentum / scale change) rather than apply it
    bad |= fail;
  }
  if (amp)
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (tt[k] >= 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) bad |= !isfinite(gv[k][j]);
  // scale read before arriving: block 0 rewrites it once everyone has arrived, and a
  // workgroup that reads it late must not unscale with the next step's value
  const float inv = pre ? 1.f / cscale : amp ? 1.f / scale[0] : 1.f;
  // pre-checked: this rank's word (XG: and the peers' NaN in the averages, with `bad`)
  const bool block_bad = __syncthreads_or(pre ? (cbad || (XG && bad)) : bad);
  if (grid == 1 || !amp || pre) {  // uniform: one workgroup, the plain step or pre-checked gradients need no grid barrier
    if (tid == 0) s_bad = block_bad;
  } else if (tid == 0) {
    // arrival words of this launch's parity: one (blanes == 1) or blanes, kBarStride apart
    const int nl = ss.blanes, st = nl > 1 ? kBarStride : 1;
    unsigned long long* words = &sync[1 + (int)(gen & 1) * nl * st];
    const unsigned long long Gn = (unsigned long long)grid;
    __hip_atomic_fetch_add(words + (bid % nl) * st, 1ull | ((unsigned long long)block_bad << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // bounded: the host sizes the grid to be co-resident, so every workgroup arrives;
    // should one never do, give up after barrier_ticks, flag it and skip the update.
    // Polled with atomic loads (a polling read-modify-write competes with the arrivals)
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool timed_out = false, any = false;
    for (;;) {
      unsigned long long cnt = 0;
      any = false;
      for (int l = 0; l < nl; ++l) {
        const unsigned long long v = __hip_atomic_load(words + l * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cnt += v & 0xffffffffull;
        any |= (v >> 32) != 0;
      }
      if (cnt >= Gn) break;
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > barrier_ticks) {
        timed_out = true;
        if (err != nullptr) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    s_bad = timed_out || any;
    if (bid == 0) {
      unsigned long long* other = &sync[1 + (int)((gen + 1) & 1) * nl * st];
      for (int l = 0; l < nl; ++l)
        __hip_atomic_store(other + l * st, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&sync[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // every slab owner waiting on the in-launch producers passed its wait before arriving
      if (ss.rearm != nullptr) __hip_atomic_store(ss.rearm, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  DPA_STAMP(12);
  const bool any_bad = s_bad;
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int t = tt[k];
    if (t < 0) continue;
    const int o = (bid * BG + k * THR + tid - soff[t]) * 4, rem = snum[t] - o;
    const f32x4 g = gv[k] * inv;
    if (amp || XG) store4(sp1[t] + o, rem, g);  // plain step: the gradient is unchanged
    if (any_bad) continue;
    f32x4 pn = pv[k], bb = bv[k];
    sgd_rule4(pn, g, bb, (L.first_bits >> t) & 1ull, lr, momentum, dampening, wd, nesterov, maximize);
    if (momentum != 0.f) store4(sp2[t] + o, rem, bb);
    store4(sp0[t] + o, rem, pn);
  }
  if (st_t >= 0) {  // a slab column: the same update, one element
    const float g = st_sum * inv;
    sp1[st_t][st_e] = g;
    if (!any_bad) {
      float bb = st_b;
      sp0[st_t][st_e] = sgd_rule(st_p, g, bb, (L.first_bits >> st_t) & 1ull, lr, momentum, dampening, wd, nesterov,
                                 maximize);
      if (momentum != 0.f) sp2[st_t][st_e] = bb;
    }
  }
  DPA_STAMP(13);
  if (amp && bid == 0 && tid == 0) {
    // every workgroup read scale[0] before arriving, and block 0 passed the barrier.
    // Without the barrier (pre-checked / XG) a peer that never arrived skips only the
    // workgroups that timed out; block 0 also backs off when the engine's error word is set
    // (any workgroup's timeout, or an earlier failure).  The ranks' parameters may then
    // differ: an engine error is fatal -- the watchdog aborts the job and cli.check_health
    // refuses to checkpoint (tests/test_aux_cpu.py, utils/watchdog.py).
    bool eng_bad = false;
    if constexpr (XG)
      eng_bad = xg.err != nullptr && __hip_atomic_load(xg.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    found_inf[0] = 0.f;
    if (any_bad || eng_bad) {
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
// Host helpers (amp_sgd_fused, convnet_amp_step)
// ---------------------------------------------------------------------------
// tensor table in float4 granules (every tensor 16-B aligned, momentum needs buffers)
inline MTList fused_list(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
                         const std::vector<at::Tensor>& bufs, const std::vector<int64_t>& first, double momentum) {
  TORCH_CHECK(params.size() == grads.size() && params.size() <= (size_t)MAXT, "fused AMP-SGD: <= ", MAXT,
              " tensors");
  TORCH_CHECK(bufs.empty() || bufs.size() == params.size());
  TORCH_CHECK(first.empty() || first.size() == params.size(), "fused AMP-SGD: one first flag per tensor");
  TORCH_CHECK(momentum == 0.0 || !bufs.empty(), "fused AMP-SGD: momentum needs buffers");
  MTList L{};
  L.n = (int)params.size();
  L.first_bits = 0;
  for (size_t i = 0; i < first.size(); ++i)
    if (first[i]) L.first_bits |= 1ull << i;
  L.chunk_off[0] = 0;
  auto f32 = [](const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat, "optimizer tensors must be f32");
  };
  for (size_t i = 0; i < params.size(); ++i) {
    f32(params[i]); f32(grads[i]);
    TORCH_CHECK(params[i].numel() == grads[i].numel());
    L.numel[i] = params[i].numel();
    L.p0[i] = params[i].data_ptr<float>();
    L.p1[i] = grads[i].data_ptr<float>();
    L.p2[i] = bufs.empty() ? nullptr : bufs[i].data_ptr<float>();
    L.chunk_off[i + 1] = L.chunk_off[i] + (L.numel[i] + 3) / 4;  // float4-granule prefix for this kernel
    auto al = [](const float* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    TORCH_CHECK(al(L.p0[i]) && al(L.p1[i]) && al(L.p2[i]), "fused AMP-SGD needs 16-byte aligned tensors");
  }
  TORCH_CHECK(L.chunk_off[L.n] * 4 <= FUSED_MAX, "fused AMP-SGD handles at most ", FUSED_MAX, " elements");
  return L;
}

// one slab source: slab [rows][out.numel()] -> the gradient region `out`, which must start
// and end on granule boundaries of the tensors that cover it
inline void add_slab(SlabSet& ss, const MTList& L, const at::Tensor& slab, const at::Tensor& out, int groups,
                     int chunks, const int* wait, int wait_n) {
  TORCH_CHECK(ss.ns < kMaxSlabs, "fused AMP-SGD: at most ", kMaxSlabs, " slab sources");
  TORCH_CHECK((groups == 16 && (chunks == 1 || chunks == 4)) || (groups == 8 && chunks == 1),
              "fused AMP-SGD: slab layouts G = 16 x 1 | 4 chunks, G = 8 x 1 chunk");
  TORCH_CHECK(wait == nullptr || (groups == 16 && chunks == 1), "fused AMP-SGD: an in-launch slab is G = 16 x 1");
  const int cols = 256 / groups * chunks;
  TORCH_CHECK(slab.is_cuda() && slab.is_contiguous() && slab.scalar_type() == at::kFloat && out.is_cuda() &&
                  out.is_contiguous() && out.scalar_type() == at::kFloat, "fused AMP-SGD: f32 slab / out");
  const int64_t ncol = out.numel();
  TORCH_CHECK(ncol > 0 && slab.numel() % ncol == 0, "fused AMP-SGD: slab must be [rows][out.numel()]");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0, "fused AMP-SGD: slab_out alignment");
  const float* lo = out.data_ptr<float>();
  const float* hi = lo + ncol;
  for (int i = 0; i < L.n; ++i) {
    const float* a = L.p1[i];
    const float* b = a + L.numel[i];
    if (b <= lo || a >= hi) continue;
    TORCH_CHECK(a >= lo && b <= hi && (L.numel[i] % 4 == 0 || b == hi),
                "fused AMP-SGD: every gradient overlapping slab_out must lie inside it, in whole granules");
  }
  for (int s = 0; s < ss.ns; ++s)
    TORCH_CHECK(hi <= ss.s[s].out || lo >= ss.s[s].out + ss.s[s].n, "fused AMP-SGD: slab regions overlap");
  SlabSrc& S = ss.s[ss.ns++];
  S.slab = slab.data_ptr<float>();
  S.out = out.data_ptr<float>();
  S.rows = (int)(slab.numel() / ncol);
  S.n = (int)ncol;
  S.groups = groups;
  S.chunks = chunks;
  S.nblk = (int)((ncol + cols - 1) / cols);
  S.wait = wait;
  S.wait_n = wait_n;
}

}  // namespace opt
}  // namespace dpa
