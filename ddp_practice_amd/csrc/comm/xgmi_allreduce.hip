// One-shot all-reduce over xGMI: peer-mapped (IPC) uncached workspaces, one
// kernel per collective, no host involvement.
//
// Why: every ConvNet collective is latency-bound (SyncBN partial-sum slabs of a
// few KB, the 116 KB DDP bucket), and there are five of
// them in the critical path of each step.  The 8 MI355X of a node are fully
// connected (7 point-to-point xGMI links per GPU), so the fastest small
// all-reduce is a single "push to every peer, wait, sum locally" kernel: each
// rank writes its chunk straight into every peer's workspace over its own link
// (all 7 links busy at once), raises a per-block flag there, and sums the W
// slots of its own workspace once every peer's flag for that block has arrived.
// This replaces the fork/join + RCCL kernel of the same collective
// (ProcessGroupNCCL in the reference: /root/reference/ddp_main.py:73, and the
// all-reduces inside DDP / SyncBatchNorm, SURVEY.md §2.2 U-PG / U-RED / U-SBN).
//
// Protocol (per block b of the grid, 2048 elements per block; blocks are
// independent, no grid sync):
//   ep  = ctr[b] + 1      ctr[b]: this rank's count of collectives that had a  (ordinary device memory)
//                         block b (equal on every rank: every rank issues the
//                         same sequence of collectives, stream-ordered)
//   par = ep & 1          double-buffered slots
//   1. each lane turns its 8 elements into 8-byte granules {fp32 value, ep} and
//      stores them into slot[par][me] of EVERY rank (incl. me) over xGMI
//   2. each lane polls its granules in slot[par][p] for p = 0..W-1 until their
//      tag is ep (bounded: timeout/abort -> host-visible error word), and
//      reduces them in rank order (bit-identical results on every rank)
//   3. ctr[b] = ep
// A granule is written by one naturally aligned 8-byte store, so value and tag
// arrive together: no flag, no release/acquire fence, one xGMI hop of latency
// (MI355X_MICROARCH.md "handoff-1to1" vs "handoff-flag").  Reuse safety: a rank
// writes parity par of epoch ep+2 only after reading every peer's ep+1
// granules, which each peer wrote after its kernel for ep had completed.
//
// Workspaces are hipExtMallocWithFlags(hipDeviceMallocUncached): no XCD L2
// holds a stale line of them; polls are sc0 sc1 (L1-bypassing) loads.
// Everything is enqueue-only (one kernel launch), so a collective can be
// captured into a hipGraph and replayed: the epoch lives in device memory.
#include <c10/hip/HIPGuard.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "comm/xgmi.h"

#include <future>
#include <sstream>
#include <thread>
#include "common.h"

namespace dpa {
namespace xgmi {

constexpr int kThreads = 256;
constexpr int kPerThread = 8;                        // elements per lane
constexpr int kChunkElems = kThreads * kPerThread;   // 2048 elements per block
constexpr int kTwoShotMaxBlocks = 256;               // two-shot grid cap (one per CU)

typedef __attribute__((ext_vector_type(2))) unsigned long long u64x2;

struct Args {
  Peers peers;
  const void* in;
  void* out;
  long long n;              // elements
  long long slot_bytes;     // per-rank slot (granules) in the workspace
  uint32_t* ctr;            // this rank's per-block epoch counters
  int rank, world;
  int* err;                 // host-mapped: 0 ok, 1 timeout, 2 aborted
  const int* abort_flag;    // host-mapped: non-zero -> stop waiting
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ unsigned long long granule(float v, uint32_t ep) {
  return ((unsigned long long)ep << 32) | (unsigned long long)__float_as_uint(v);
}

// op: 0 sum, 1 avg, 2 max, 3 min
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void oneshot_kernel(Args a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  DPA_STAMP(0);
  char* mine = a.peers.base[a.rank];
  uint32_t* ctr = a.ctr + b;
  const uint32_t ep = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const long long par_off = (long long)(ep & 1) * kMaxRanks * a.slot_bytes;
  const long long e0 = (long long)b * kChunkElems + (long long)tid * kPerThread;
  const int ne = (int)max(0LL, min((long long)kPerThread, a.n - e0));

  // 1. my elements -> {value, epoch} granules in slot[parity][me] of every other rank
  float v[kPerThread];
  const T* in = static_cast<const T*>(a.in) + e0;
  if (ne == kPerThread) {
    if constexpr (sizeof(T) == 4) {
      const f32x4 x0 = reinterpret_cast<const f32x4*>(in)[0], x1 = reinterpret_cast<const f32x4*>(in)[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = x0[j]; v[4 + j] = x1[j]; }
    } else {
      const f32x4 raw = *reinterpret_cast<const f32x4*>(in);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) v[j] = Cvt<T>::to_f(e[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) v[j] = j < ne ? Cvt<T>::to_f(in[j]) : 0.f;
  }
  for (int p = 0; p < a.world; ++p) {
    if (p == a.rank) continue;  // my own values stay in registers (v)
    unsigned long long* dst =
        reinterpret_cast<unsigned long long*>(a.peers.base[p] + par_off + (long long)a.rank * a.slot_bytes) + e0;
    if (ne == kPerThread) {
#pragma unroll
      for (int j = 0; j < kPerThread; j += 2) xgmi_put2(dst + j, granule(v[j], ep), granule(v[j + 1], ep));
    } else {
      for (int j = 0; j < ne; ++j) xgmi_put(dst + j, granule(v[j], ep));
    }
  }

  DPA_STAMP(1);
  // 2. every rank's granules for my elements, in rank order (identical result on
  //    every rank); each granule carries its own epoch tag: no flag, no fence.
  //    The loads of PB ranks x 8 elements are all issued before the first tag
  //    check (one memory round trip per batch, not one per granule); only a
  //    granule that has not arrived yet is re-polled.
  constexpr int PB = 4;
  float acc[kPerThread];
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) acc[j] = 0.f;
  bool fail = false;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  unsigned polls = 0;
  for (int p0 = 0; p0 < a.world && !fail; p0 += PB) {
    unsigned long long g[PB][kPerThread];
    const unsigned long long* src[PB];
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int p = p0 + q < a.world ? p0 + q : p0;  // out-of-range batch slots re-read rank p0 (ignored)
      src[q] = reinterpret_cast<const unsigned long long*>(mine + par_off + (long long)p * a.slot_bytes) + e0;
#pragma unroll
      for (int j = 0; j < kPerThread; ++j)  // slots hold whole chunks: j >= ne stays inside the slot
        g[q][j] = __hip_atomic_load(src[q] + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      if (p0 + q >= a.world || fail) continue;
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        if (j >= ne || fail) continue;
        if (p0 + q == a.rank) g[q][j] = granule(v[j], ep);  // own contribution: not written, not polled
        while ((g[q][j] >> 32) != ep) {
          __builtin_amdgcn_s_sleep(1);
          g[q][j] = __hip_atomic_load(src[q] + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((++polls & 255u) == 0) {
            const int why = give_up(a.err, a.abort_flag, t0, a.timeout_ticks);
            if (why) {
              if (why > 0) __hip_atomic_store(a.err, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              fail = true;
              break;
            }
          }
        }
        if (fail) continue;
        const float x = __uint_as_float((uint32_t)g[q][j]);
        if (p0 + q == 0) acc[j] = x;
        else if (OP == 2) acc[j] = fmaxf(acc[j], x);
        else if (OP == 3) acc[j] = fminf(acc[j], x);
        else acc[j] += x;
      }
    }
  }
  DPA_STAMP(2);
  if (!fail) {
    T* out = static_cast<T*>(a.out) + e0;
    const float s = OP == 1 ? 1.f / (float)a.world : 1.f;
    if (ne == kPerThread && sizeof(T) == 2) {
      f32x4 raw;
      T* r = reinterpret_cast<T*>(&raw);
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) r[j] = Cvt<T>::from_f(acc[j] * s);
      *reinterpret_cast<f32x4*>(out) = raw;
    } else if (ne == kPerThread) {
      reinterpret_cast<f32x4*>(out)[0] = f32x4{acc[0] * s, acc[1] * s, acc[2] * s, acc[3] * s};
      reinterpret_cast<f32x4*>(out)[1] = f32x4{acc[4] * s, acc[5] * s, acc[6] * s, acc[7] * s};
    } else {
      for (int j = 0; j < ne; ++j) out[j] = Cvt<T>::from_f(acc[j] * s);
    }
  }
  // 3. this block's epoch is done (after every lane read the counter)
  __syncthreads();
  if (tid == 0 && !fail) __hip_atomic_store(ctr, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DPA_STAMP(3);
}

// ---------------------------------------------------------------------------
// Two-shot all-reduce for large messages (DDP buckets of MBs): reduce-scatter then
// all-gather, both as direct peer writes over the 7 xGMI links.
//
// A one-shot pushes the whole message to every peer: (W-1) * S bytes out per rank
// (W = 8, 25 MiB bucket: 175 MiB per rank).  Here rank r owns shard r of the
// message (S/W elements): every rank pushes each peer only that peer's shard
// (reduce-scatter, (W-1)/W * S), the owner sums the W contributions in rank order,
// then pushes its reduced shard to every peer (all-gather, (W-1)/W * S again) --
// 2 (W-1)/W * S per rank, spread over all W-1 links at once (a ring moves the same
// bytes over one link per direction).  SURVEY.md §2.6 item 2.
//
// Same transport as the one-shot: {value, epoch} 8-byte granules (value and tag
// land together: no flag, no fence), bounded waits, per-block epochs kept in device
// memory (graph-replayable), parity double-buffering.  Block b handles chunk b
// (kChunkElems elements) of EVERY shard, so a block's reduce-scatter output is its
// own all-gather input.  The reduced shard is rounded to the storage dtype before
// it is pushed, so every rank's result is bit-identical.  The region and the epoch
// counters are its own (a one-shot and a two-shot never share bytes: a peer may
// still be reading one collective's granules while this rank starts the next).
//   region layout, per parity: [RS: W src slots x shard] [AG: the whole message]
struct TSArgs {
  Peers peers;              // every rank's two-shot region
  const void* in;
  void* out;
  long long n;              // elements
  long long shard;          // elements per shard (multiple of kChunkElems)
  long long stride;         // region slot stride in granules (the largest shard): block b
                            // touches the same bytes whatever the message size, so its
                            // per-block epoch alone tells its granules apart
  long long par_bytes;      // bytes of one parity of the region
  uint32_t* ctr;            // per-block epoch counters
  int rank, world;
  int* err;
  const int* abort_flag;
  long long timeout_ticks;
};

__device__ __forceinline__ bool ts_wait(const TSArgs& a, const unsigned long long* src, unsigned long long& g,
                                        uint32_t ep, long long t0, unsigned& polls) {
  while ((uint32_t)(g >> 32) != ep) {
    __builtin_amdgcn_s_sleep(1);
    g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((++polls & 255u) == 0) {
      const int why = give_up(a.err, a.abort_flag, t0, a.timeout_ticks);
      if (why) {
        if (why > 0) __hip_atomic_store(a.err, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
  }
  return true;
}

template <typename T>
__device__ __forceinline__ void ts_load8(const T* p, long long e0, long long n, float (&v)[kPerThread]) {
  const int ne = (int)max(0LL, min((long long)kPerThread, n - e0));
  if (ne == kPerThread) {
    if constexpr (sizeof(T) == 4) {
      const f32x4 x0 = reinterpret_cast<const f32x4*>(p + e0)[0], x1 = reinterpret_cast<const f32x4*>(p + e0)[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = x0[j]; v[4 + j] = x1[j]; }
    } else {
      const f32x4 raw = *reinterpret_cast<const f32x4*>(p + e0);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) v[j] = Cvt<T>::to_f(e[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) v[j] = j < ne ? Cvt<T>::to_f(p[e0 + j]) : 0.f;
  }
}

template <typename T>
__device__ __forceinline__ void ts_store8(T* p, long long e0, long long n, const float (&v)[kPerThread]) {
  const int ne = (int)max(0LL, min((long long)kPerThread, n - e0));
  if (ne == kPerThread) {
    if constexpr (sizeof(T) == 2) {
      f32x4 raw;
      T* r = reinterpret_cast<T*>(&raw);
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) r[j] = Cvt<T>::from_f(v[j]);
      *reinterpret_cast<f32x4*>(p + e0) = raw;
    } else {
      reinterpret_cast<f32x4*>(p + e0)[0] = f32x4{v[0], v[1], v[2], v[3]};
      reinterpret_cast<f32x4*>(p + e0)[1] = f32x4{v[4], v[5], v[6], v[7]};
    }
  } else {
    for (int j = 0; j < ne; ++j) p[e0 + j] = Cvt<T>::from_f(v[j]);
  }
}

__device__ __forceinline__ void push8(unsigned long long* dst, const float (&v)[kPerThread], uint32_t ep) {
#pragma unroll
  for (int j = 0; j < kPerThread; j += 2) xgmi_put2(dst + j, granule(v[j], ep), granule(v[j + 1], ep));
}

// op: 0 sum, 1 avg, 2 max, 3 min.  A FIXED grid of G blocks (every call): block b
// owns chunks b, b+G, b+2G, ... of every shard.  Every block bumps its epoch once per
// call, so all blocks' epochs equal the call count and a chunk's slot is always
// written by the same block index on every rank; G is small enough that the grids of
// all ranks can be resident together even when ranks share a GPU (tests), and a block
// never waits on a block of its own rank.
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void twoshot_kernel(TSArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x, G = gridDim.x;
  uint32_t* ctr = a.ctr + b;
  const uint32_t ep = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const long long par = (long long)(ep & 1u) * a.par_bytes;
  const long long nch = a.shard / kChunkElems;                                      // chunks per shard
  const long long rs_bytes = (long long)a.world * a.stride * 8;                     // RS part of a parity
  const T* in = static_cast<const T*>(a.in);
  T* out = static_cast<T*>(a.out);
  char* mybase = a.peers.base[a.rank] + par;
  // 1. reduce-scatter push: peer p gets my chunk c of its shard p, into its RS slot [me]
  for (long long c = b; c < nch; c += G) {
    const long long c0 = c * kChunkElems + (long long)tid * kPerThread;  // offset inside a shard
    for (int i = 1; i < a.world; ++i) {
      const int p = (a.rank + i) % a.world;  // staggered: the ranks start on different links
      float v[kPerThread];
      ts_load8<T>(in, (long long)p * a.shard + c0, a.n, v);
      push8(reinterpret_cast<unsigned long long*>(a.peers.base[p] + par + ((long long)a.rank * a.stride + c0) * 8),
            v, ep);
    }
  }
  bool ok = true;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  unsigned polls = 0;
  const float s = OP == 1 ? 1.f / (float)a.world : 1.f;
  // 2. my shard's chunks: the W contributions in rank order (identical on every rank),
  //    rounded to the storage dtype once, then pushed to every peer's AG part
  for (long long c = b; c < nch && ok; c += G) {
    const long long c0 = c * kChunkElems + (long long)tid * kPerThread;
    const long long mine_off = (long long)a.rank * a.shard + c0;
    float acc[kPerThread];
    for (int p = 0; p < a.world; ++p) {
      float v[kPerThread];
      if (p == a.rank) {
        ts_load8<T>(in, mine_off, a.n, v);
      } else {
        const unsigned long long* src =
            reinterpret_cast<const unsigned long long*>(mybase + ((long long)p * a.stride + c0) * 8);
        unsigned long long g[kPerThread];
#pragma unroll
        for (int j = 0; j < kPerThread; ++j)
          g[j] = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int j = 0; j < kPerThread; ++j) {
          if (ok) ok = ts_wait(a, src + j, g[j], ep, t0, polls);
          v[j] = __uint_as_float((uint32_t)g[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        if (p == 0) acc[j] = v[j];
        else if (OP == 2) acc[j] = fmaxf(acc[j], v[j]);
        else if (OP == 3) acc[j] = fminf(acc[j], v[j]);
        else acc[j] += v[j];
      }
    }
    if (!ok) break;
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) acc[j] = Cvt<T>::to_f(Cvt<T>::from_f(acc[j] * s));
    for (int i = 1; i < a.world; ++i) {
      const int p = (a.rank + i) % a.world;
      push8(reinterpret_cast<unsigned long long*>(a.peers.base[p] + par + rs_bytes +
                                                  ((long long)a.rank * a.stride + c0) * 8),
            acc, ep);
    }
    ts_store8<T>(out, mine_off, a.n, acc);
  }
  // 3. every other shard's chunks from my AG part
  for (long long c = b; c < nch && ok; c += G) {
    const long long c0 = c * kChunkElems + (long long)tid * kPerThread;
    for (int i = 1; i < a.world && ok; ++i) {
      const int q = (a.rank + a.world - i) % a.world;
      const unsigned long long* src =
          reinterpret_cast<const unsigned long long*>(mybase + rs_bytes + ((long long)q * a.stride + c0) * 8);
      unsigned long long g[kPerThread];
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) g[j] = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      float v[kPerThread];
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        if (ok) ok = ts_wait(a, src + j, g[j], ep, t0, polls);
        v[j] = __uint_as_float((uint32_t)g[j]);
      }
      if (ok) ts_store8<T>(out, (long long)q * a.shard + c0, a.n, v);
    }
  }
  __syncthreads();
  if (tid == 0 && ok) __hip_atomic_store(ctr, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

XgmiComm::XgmiComm(int rank, int world, int device, long long slot_bytes, double timeout_s, long long ts_bytes)
    : rank_(rank), world_(world), device_(device) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "xgmi: 1..", kMaxRanks, " ranks");
  TORCH_CHECK(rank >= 0 && rank < world);
  // max_bytes is counted as fp32 elements; every element travels as an 8-B granule
  max_elems_ = ((std::max(slot_bytes, 4LL) / 4 + kChunkElems - 1) / kChunkElems) * kChunkElems;
  max_blocks_ = (int)(max_elems_ / kChunkElems);
  slot_bytes_ = max_elems_ * 8;
  // the epoch counters are only ever touched by this rank, kernel after kernel
  // on one stream: ordinary device memory (stream order makes each kernel's
  // store visible to the next), read at L2 latency instead of an uncached trip
  ctr_off_ = 0;
  site_off_ = 2LL * kMaxRanks * slot_bytes_;  // then kSites fused-site regions (comm/xsite.h)
  grad_off_ = site_off_ + kSites * kSiteBytes;  // then the gradient-exchange slots [2][kMaxRanks]
  // then the two-shot region: 2 parities x ([W shards of RS slots] + [the whole message]),
  // i.e. 2 x 2 x the message as granules; shards are whole chunks
  ts_off_ = grad_off_ + 2LL * kMaxRanks * slot_bytes_;
  if (ts_bytes > 0) {
    const long long ts_elems = std::max(ts_bytes, 4LL) / 4;
    ts_shard_max_ = ((ts_elems + world_ - 1) / world_ + kChunkElems - 1) / kChunkElems * kChunkElems;
    ts_max_elems_ = ts_elems;
    ts_par_bytes_ = 2LL * world_ * ts_shard_max_ * 8;
    ts_blocks_ = kTwoShotMaxBlocks;
    ts_grid_ = (int)std::min<long long>(kTwoShotMaxBlocks, ts_shard_max_ / kChunkElems);
  }
  wide_off_ = ((ts_off_ + 2 * ts_par_bytes_ + 4095) / 4096) * 4096;  // then the wide site: [2][kMaxRanks] rows
  ws_bytes_ = ((wide_off_ + 2LL * kMaxRanks * kWideVals * 8 + 4095) / 4096) * 4096;
  timeout_ticks_ = (long long)(timeout_s * 1e8);
  c10::hip::HIPGuard guard(device_);
  void* p = nullptr;
  DPA_CHECK_HIP(hipExtMallocWithFlags(&p, ws_bytes_, hipDeviceMallocUncached));
  DPA_CHECK_HIP(hipMemset(p, 0, ws_bytes_));
  DPA_CHECK_HIP(hipDeviceSynchronize());
  local_ = static_cast<char*>(p);
  void* c = nullptr;
  DPA_CHECK_HIP(hipMalloc(&c, (size_t)max_blocks_ * sizeof(uint32_t)));
  DPA_CHECK_HIP(hipMemset(c, 0, (size_t)max_blocks_ * sizeof(uint32_t)));
  DPA_CHECK_HIP(hipDeviceSynchronize());
  ctr_ = static_cast<uint32_t*>(c);
  if (ts_blocks_ > 0) {
    void* c2 = nullptr;
    DPA_CHECK_HIP(hipMalloc(&c2, (size_t)ts_blocks_ * sizeof(uint32_t)));
    DPA_CHECK_HIP(hipMemset(c2, 0, (size_t)ts_blocks_ * sizeof(uint32_t)));
    DPA_CHECK_HIP(hipDeviceSynchronize());
    ts_ctr_ = static_cast<uint32_t*>(c2);
  }
  void* tk = nullptr;
  DPA_CHECK_HIP(hipMalloc(&tk, kSites * kEpochWords * sizeof(unsigned long long)));
  DPA_CHECK_HIP(hipMemset(tk, 0, kSites * kEpochWords * sizeof(unsigned long long)));
  DPA_CHECK_HIP(hipDeviceSynchronize());
  ticks_ = static_cast<unsigned long long*>(tk);
  for (int i = 0; i < kMaxRanks; ++i) peers_.base[i] = nullptr;
  peers_.base[rank_] = local_;
  void* h = nullptr;
  DPA_CHECK_HIP(hipHostMalloc(&h, 2 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  host_words_ = static_cast<int*>(h);
  host_words_[0] = host_words_[1] = 0;
  void* d = nullptr;
  DPA_CHECK_HIP(hipHostGetDevicePointer(&d, h, 0));
  dev_words_ = static_cast<int*>(d);
}

XgmiComm::~XgmiComm() { close(); }

void XgmiComm::close() {
  if (local_ == nullptr) return;
  c10::hip::HIPGuard guard(device_);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < world_; ++p)
    if (p != rank_ && peers_.base[p] != nullptr) (void)hipIpcCloseMemHandle(peers_.base[p]);
  (void)hipFree(local_);
  if (ctr_ != nullptr) (void)hipFree(ctr_);
  ctr_ = nullptr;
  if (ts_ctr_ != nullptr) (void)hipFree(ts_ctr_);
  ts_ctr_ = nullptr;
  if (ticks_ != nullptr) (void)hipFree(ticks_);
  ticks_ = nullptr;
  if (host_words_ != nullptr) (void)hipHostFree(host_words_);
  local_ = nullptr;
  host_words_ = dev_words_ = nullptr;
  opened_ = false;
}

pybind11::bytes XgmiComm::handle() const {
  TORCH_CHECK(local_ != nullptr, "xgmi: closed");
  hipIpcMemHandle_t h;
  DPA_CHECK_HIP(hipIpcGetMemHandle(&h, local_));
  return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiComm::open(std::vector<std::string> handles) {
  TORCH_CHECK((int)handles.size() == world_, "xgmi: need one handle per rank");
  c10::hip::HIPGuard guard(device_);
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    TORCH_CHECK(handles[p].size() == sizeof(hipIpcMemHandle_t), "xgmi: bad handle size");
    hipIpcMemHandle_t h;
    memcpy(&h, handles[p].data(), sizeof(h));
    void* ptr = nullptr;
    DPA_CHECK_HIP(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
    peers_.base[p] = static_cast<char*>(ptr);
  }
  opened_ = true;
}

bool XgmiComm::supports(const at::Tensor& t) const {
  const auto st = t.scalar_type();
  return opened_ && t.is_cuda() && t.get_device() == device_ && t.is_contiguous() &&
         (st == at::kFloat || st == at::kBFloat16 || st == at::kHalf) && t.numel() > 0 &&
         (long long)t.numel() <= max_elems_ && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

void XgmiComm::all_reduce(const at::Tensor& in, const at::Tensor& out, RedOp op, hipStream_t stream) {
  TORCH_CHECK(supports(in) && supports(out) && in.numel() == out.numel() &&
                  in.scalar_type() == out.scalar_type(),
              "xgmi all_reduce: unsupported tensor (device/dtype/size/alignment)");
  TORCH_CHECK(op != RedOp::PROD, "xgmi all_reduce: prod is not supported");
  ar_calls_.fetch_add(1, std::memory_order_relaxed);
  ar_last_bytes_.store((long long)in.nbytes(), std::memory_order_relaxed);
  Args a;
  a.peers = peers_;
  a.in = in.data_ptr();
  a.out = out.data_ptr();
  a.n = in.numel();
  a.slot_bytes = slot_bytes_;
  a.ctr = ctr_;
  a.rank = rank_;
  a.world = world_;
  a.err = dev_words_;
  a.abort_flag = dev_words_ + 1;
  a.timeout_ticks = timeout_ticks_;
  const int grid = (int)((a.n + kChunkElems - 1) / kChunkElems);
  hipStream_t s = stream ? stream : cur_stream();
  const int o = op == RedOp::SUM ? 0 : op == RedOp::AVG ? 1 : op == RedOp::MAX ? 2 : 3;
  auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, s, a); };
#define DPA_XG(T)                                \
  switch (o) {                                   \
    case 0: launch(oneshot_kernel<T, 0>); break; \
    case 1: launch(oneshot_kernel<T, 1>); break; \
    case 2: launch(oneshot_kernel<T, 2>); break; \
    default: launch(oneshot_kernel<T, 3>); break; \
  }
  switch (in.scalar_type()) {
    case at::kFloat: DPA_XG(float); break;
    case at::kBFloat16: DPA_XG(__hip_bfloat16); break;
    default: DPA_XG(__half); break;
  }
#undef DPA_XG
  DPA_CHECK_LAUNCH();
}

void XgmiComm::set_twoshot_blocks(int g) {
  TORCH_CHECK(g >= 1 && g <= kTwoShotMaxBlocks, "two-shot grid: 1..", kTwoShotMaxBlocks);
  TORCH_CHECK(ts_blocks_ > 0, "no two-shot region");
  // every block's epoch must stay equal: only while no two-shot has run yet
  TORCH_CHECK(!ts_used_, "set_twoshot_blocks: the two-shot engine has already run");
  ts_grid_ = (int)std::min<long long>(g, ts_shard_max_ / kChunkElems);
}

bool XgmiComm::supports_twoshot(const at::Tensor& t) const {
  const auto st = t.scalar_type();
  return opened_ && ts_blocks_ > 0 && t.is_cuda() && t.get_device() == device_ && t.is_contiguous() &&
         (st == at::kFloat || st == at::kBFloat16 || st == at::kHalf) && t.numel() > 0 &&
         (long long)t.numel() <= ts_max_elems_ && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

void XgmiComm::all_reduce_twoshot(const at::Tensor& in, const at::Tensor& out, RedOp op, hipStream_t stream) {
  TORCH_CHECK(supports_twoshot(in) && supports_twoshot(out) && in.numel() == out.numel() &&
                  in.scalar_type() == out.scalar_type(),
              "xgmi two-shot all_reduce: unsupported tensor (device/dtype/size/alignment)");
  TORCH_CHECK(op != RedOp::PROD, "xgmi all_reduce: prod is not supported");
  ts_calls_.fetch_add(1, std::memory_order_relaxed);
  ar_last_bytes_.store((long long)in.nbytes(), std::memory_order_relaxed);
  TSArgs a;
  for (int p = 0; p < kMaxRanks; ++p) a.peers.base[p] = peers_.base[p] ? peers_.base[p] + ts_off_ : nullptr;
  a.in = in.data_ptr();
  a.out = out.data_ptr();
  a.n = in.numel();
  // shard: whole chunks, every element inside [0, W * shard)
  a.shard = ((a.n + world_ - 1) / world_ + kChunkElems - 1) / kChunkElems * kChunkElems;
  a.stride = ts_shard_max_;
  ts_used_ = true;
  a.par_bytes = ts_par_bytes_;
  a.ctr = ts_ctr_;
  a.rank = rank_;
  a.world = world_;
  a.err = dev_words_;
  a.abort_flag = dev_words_ + 1;
  a.timeout_ticks = timeout_ticks_;
  const int grid = ts_grid_;  // fixed for the engine's lifetime (see twoshot_kernel)
  hipStream_t s = stream ? stream : cur_stream();
  const int o = op == RedOp::SUM ? 0 : op == RedOp::AVG ? 1 : op == RedOp::MAX ? 2 : 3;
  auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, s, a); };
#define DPA_TS(T)                                \
  switch (o) {                                   \
    case 0: launch(twoshot_kernel<T, 0>); break; \
    case 1: launch(twoshot_kernel<T, 1>); break; \
    case 2: launch(twoshot_kernel<T, 2>); break; \
    default: launch(twoshot_kernel<T, 3>); break; \
  }
  switch (in.scalar_type()) {
    case at::kFloat: DPA_TS(float); break;
    case at::kBFloat16: DPA_TS(__hip_bfloat16); break;
    default: DPA_TS(__half); break;
  }
#undef DPA_TS
  DPA_CHECK_LAUNCH();
}

XSite XgmiComm::site(int s) const {
  TORCH_CHECK(opened_ && local_ != nullptr, "xgmi: site of a closed or unopened communicator");
  TORCH_CHECK(s >= 0 && s < kSites, "xgmi: site id out of range");
  site_calls_[s].fetch_add(1, std::memory_order_relaxed);  // (a handle per attached launch)
  XSite x;
  for (int p = 0; p < world_; ++p) x.base[p] = peers_.base[p] + site_off_ + (long long)s * kSiteBytes;
  x.mine = x.base[rank_];
  x.tick = ticks_ + (long long)s * kEpochWords;
  x.rank = rank_;
  x.world = world_;
  x.err = dev_words_;
  x.abort_flag = dev_words_ + 1;
  x.timeout_ticks = timeout_ticks_;
  return x;
}

XSite XgmiComm::grad_site() const {
  XSite x = site(kSiteGrad);
  for (int p = 0; p < world_; ++p) x.base[p] = peers_.base[p] + grad_off_;
  x.mine = x.base[rank_];
  x.slot_bytes = slot_bytes_;
  x.max_vals = max_elems_;
  return x;
}

XSite XgmiComm::wide_site() const {
  XSite x = site(kSiteWide);
  for (int p = 0; p < world_; ++p) x.base[p] = peers_.base[p] + wide_off_;
  x.mine = x.base[rank_];
  x.slot_bytes = (long long)kWideVals * 8;
  x.max_vals = kWideVals;
  return x;
}

// Test entry for the positioned exchange: finisher b of nblk owns the row positions
// [b*n/nblk, (b+1)*n/nblk), stored to out from the exchanged slice (the statistics
// finishers of conv_igemm.hip / bn_nhwc.hip in isolation: sizes up to 2*2048+1).
__global__ void __launch_bounds__(256) wide_probe_kernel(XSite xs, const float* __restrict__ in,
                                                         float* __restrict__ out, int n) {
  __shared__ float vals[kWideVals];
  const int b = (int)blockIdx.x, nb = (int)gridDim.x;
  const int lo = (int)((long long)n * b / nb), hi = (int)((long long)n * (b + 1) / nb);
  unsigned long long tk = 0;
  if (threadIdx.x == 0) tk = xsite_ticket(xs, b);
  for (int i = threadIdx.x; i < hi - lo; i += 256) vals[i] = in[lo + i];
  __syncthreads();
  xsite_exchange_slice(xs, vals, hi - lo, [&](int i) { return lo + i; }, tk, b, 256);
  for (int i = threadIdx.x; i < hi - lo; i += 256) out[lo + i] = vals[i];
}

void XgmiComm::wide_probe(const at::Tensor& in, const at::Tensor& out, int nblk) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kFloat && in.is_contiguous() && in.numel() <= kWideVals &&
                  in.numel() >= 1,
              "wide_probe: 1..", kWideVals, " contiguous f32 values");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() == in.numel(), "wide_probe: out like in");
  TORCH_CHECK(nblk >= 1 && nblk <= in.numel(), "wide_probe: 1..n finishers");
  XSite xs = wide_site();
  set_site_grid(xs, nblk, "wide_probe");
  hipLaunchKernelGGL(wide_probe_kernel, dim3(nblk), dim3(256), 0, cur_stream(), xs, in.data_ptr<float>(),
                     out.data_ptr<float>(), (int)in.numel());
  DPA_CHECK_LAUNCH();
}

// Test entry for the in-kernel exchange (comm/xsite.h): `grid` workgroups each
// exchange the same n (<= kSiteVals) floats through site s and write the
// rank-ordered global sums to out[block][n] -- the protocol every fused SyncBN
// consumer runs in its prologue, isolated (numerics, epochs, parity reuse,
// bounded waits).
__global__ void __launch_bounds__(256) site_probe_kernel(XSite xs, const float* __restrict__ in,
                                                         float* __restrict__ out, int n) {
  __shared__ float vals[kSiteVals];
  unsigned long long tk = 0;
  if (threadIdx.x == 0) tk = xsite_ticket(xs, (int)blockIdx.x);
  if ((int)threadIdx.x < n) vals[threadIdx.x] = in[threadIdx.x];
  __syncthreads();
  xsite_exchange(xs, vals, n, tk, (int)blockIdx.x);
  if ((int)threadIdx.x < n) out[(long long)blockIdx.x * n + threadIdx.x] = vals[threadIdx.x];
}

void XgmiComm::site_probe(int s, const at::Tensor& in, const at::Tensor& out, int grid) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kFloat && in.is_contiguous() && in.numel() <= kSiteVals,
              "site_probe: <= ", kSiteVals, " contiguous f32 values");
  TORCH_CHECK(out.numel() == (int64_t)grid * in.numel() && out.scalar_type() == at::kFloat && grid >= 1);
  TORCH_CHECK(s >= 0 && s < kSiteGrad, "site_probe: SyncBN site id");
  XSite xs = site(s);
  set_site_grid(xs, grid, "site_probe");
  xs.nblk = 0;  // the whole grid
  hipLaunchKernelGGL(site_probe_kernel, dim3(grid), dim3(256), 0, cur_stream(), xs, in.data_ptr<float>(),
                     out.data_ptr<float>(), (int)in.numel());
  DPA_CHECK_LAUNCH();
}

int XgmiComm::error() const { return host_words_ ? __atomic_load_n(&host_words_[0], __ATOMIC_ACQUIRE) : 0; }

std::string XgmiComm::error_string() const {
  const int e = error();
  return e == 0 ? std::string() : e == 1 ? std::string("xgmi all-reduce: a peer never arrived (timeout)")
                                         : std::string("xgmi all-reduce: aborted");
}

void XgmiComm::abort() {
  if (host_words_) __atomic_store_n(&host_words_[1], 1, __ATOMIC_RELEASE);
}

std::string XgmiComm::debug_state(double wait_s) const {
  std::ostringstream o;
  o << "xgmi rank " << rank_ << "/" << world_;
  if (host_words_ == nullptr || local_ == nullptr) {
    o << ": closed";
    return o.str();
  }
  o << ": err=" << __atomic_load_n(&host_words_[0], __ATOMIC_ACQUIRE)
    << " abort=" << __atomic_load_n(&host_words_[1], __ATOMIC_ACQUIRE);
  // host side first (needs no device work): equal counts on every rank mean the ranks issued
  // the same sequence, so a stall is co-residency / scheduling, not a diverged protocol
  o << "; host issued: oneshot " << ar_calls_.load() << " twoshot " << ts_calls_.load() << " (last "
    << ar_last_bytes_.load() << " B), site handles";
  for (int s = 0; s < kSites; ++s) o << (s ? "," : " ") << site_calls_[s].load();
  // regions: the SyncBN sites 0..4, the wide site, the gradient site, the one-shot slots
  struct Reg {
    const char* name;
    int site;            // epoch words (-1: per-block counters)
    long long off, slot;
  };
  std::vector<Reg> regs;
  static const char* names[] = {"fwd1", "fwd2", "bwd2d", "bwd2w", "bwd1"};
  for (int s = 0; s < kSiteWide; ++s) regs.push_back({names[s], s, site_off_ + (long long)s * kSiteBytes, kSiteSlotBytes});
  regs.push_back({"wide", kSiteWide, wide_off_, (long long)kWideVals * 8});
  regs.push_back({"grad", kSiteGrad, grad_off_, slot_bytes_});
  regs.push_back({"oneshot", -1, 0, slot_bytes_});
  const int nr = (int)regs.size();
  struct Snap {
    std::vector<unsigned long long> ticks, tags;
    std::vector<uint32_t> ctr, tctr;
  };
  auto snap = std::make_shared<Snap>();
  snap->ticks.assign((size_t)kSites * kEpochWords, 0);
  snap->tags.assign((size_t)nr * 2 * world_, 0);
  snap->ctr.assign(4, 0);
  snap->tctr.assign(4, 0);
  const int dev = device_, world = world_, maxb = max_blocks_, tsb = ts_blocks_;
  const unsigned long long* ticks = ticks_;
  const uint32_t *ctr = ctr_, *tctr = ts_ctr_;
  const char* local = local_;
  std::vector<long long> goff;
  for (const auto& r : regs)
    for (int par = 0; par < 2; ++par)
      for (int p = 0; p < world; ++p) goff.push_back(r.off + (long long)par * kMaxRanks * r.slot + (long long)p * r.slot);
  auto done = std::make_shared<std::promise<bool>>();
  auto fut = done->get_future();
  std::thread([=]() {
    bool ok = hipSetDevice(dev) == hipSuccess;
    hipStream_t st = nullptr;
    ok = ok && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
    if (ok) {
      ok = hipMemcpyAsync(snap->ticks.data(), ticks, snap->ticks.size() * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
      for (size_t i = 0; ok && i < goff.size(); ++i)
        ok = hipMemcpyAsync(&snap->tags[i], local + goff[i], 8, hipMemcpyDeviceToHost, st) == hipSuccess;
      if (ok) ok = hipMemcpyAsync(snap->ctr.data(), ctr, 4 * std::min(4, maxb), hipMemcpyDeviceToHost, st) == hipSuccess;
      if (ok && tctr != nullptr)
        ok = hipMemcpyAsync(snap->tctr.data(), tctr, 4 * std::min(4, tsb), hipMemcpyDeviceToHost, st) == hipSuccess;
      ok = ok && hipStreamSynchronize(st) == hipSuccess;
    }
    done->set_value(ok);
  }).detach();
  if (fut.wait_for(std::chrono::duration<double>(wait_s)) != std::future_status::ready) {
    o << "; device snapshot timed out after " << wait_s << " s";
    return o.str();
  }
  if (!fut.get()) {
    o << "; device snapshot failed";
    return o.str();
  }
  size_t g = 0;
  for (const auto& r : regs) {
    unsigned long long lo = ~0ull, hi = 0;
    if (r.site >= 0)
      for (int w = 0; w < kEpochWords; ++w) {
        const unsigned long long v = snap->ticks[(size_t)r.site * kEpochWords + w];
        lo = std::min(lo, v);
        hi = std::max(hi, v);
      }
    std::ostringstream t;
    bool any = hi > 0;
    for (int par = 0; par < 2; ++par) {
      t << (par ? " | " : "");
      for (int p = 0; p < world; ++p, ++g) {
        const uint32_t tag = (uint32_t)(snap->tags[g] >> 32);
        any = any || tag != 0;
        t << (p ? "," : "") << (p == rank_ ? "*" : "") << tag;
      }
    }
    if (!any) continue;  // a site this run never used
    o << "; " << r.name;
    if (r.site >= 0) o << " ep=" << (lo == hi ? std::to_string(hi) : std::to_string(lo) + ".." + std::to_string(hi));
    o << " peers[par0|par1]=" << t.str();
  }
  o << "; oneshot blk ep=" << snap->ctr[0] << "," << snap->ctr[1];
  if (tctr != nullptr) o << "; twoshot blk ep=" << snap->tctr[0] << "," << snap->tctr[1];
  return o.str();
}

}  // namespace xgmi

// The engine as the reducer's Collective (csrc/ddp/reducer.cpp): async
// all-reduces on a side stream fenced by events, like the RCCL communicator.
// Used when every all-reduce of a run fits the engine (multi-process runs on
// one GPU in the test tier, where RCCL refuses duplicate devices).
class XgmiCollective : public Collective {
 public:
  explicit XgmiCollective(std::shared_ptr<xgmi::XgmiComm> x)
      : x_(std::move(x)), stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, x_->device())) {
    for (int i = 0; i < kSlots; ++i) DPA_CHECK_HIP(hipEventCreateWithFlags(&slot_[i], hipEventDisableTiming));
    for (int i = 0; i < kRing; ++i) {
      DPA_CHECK_HIP(hipEventCreateWithFlags(&fork_[i], hipEventDisableTiming));
      DPA_CHECK_HIP(hipEventCreateWithFlags(&join_[i], hipEventDisableTiming));
    }
  }
  ~XgmiCollective() override {
    for (auto& e : slot_) if (e) (void)hipEventDestroy(e);
    for (auto& e : fork_) if (e) (void)hipEventDestroy(e);
    for (auto& e : join_) if (e) (void)hipEventDestroy(e);
  }
  int rank() const override { return x_->rank(); }
  int world() const override { return x_->world(); }
  void all_reduce_async(at::Tensor t, RedOp op, int slot) override {
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    const int i = next_++ % kRing;
    DPA_CHECK_HIP(hipEventRecord(fork_[i], cur_stream()));
    DPA_CHECK_HIP(hipStreamWaitEvent(stream_.stream(), fork_[i], 0));
    chunked(t, t, op);
    DPA_CHECK_HIP(hipEventRecord(slot_[slot], stream_.stream()));
  }
  void wait(int slot, hipStream_t stream) override {
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    DPA_CHECK_HIP(hipStreamWaitEvent(stream ? stream : cur_stream(), slot_[slot], 0));
  }
  // stream-synchronous form: on the same side stream as the async ones, so all
  // collectives of this rank run in issue order
  void all_reduce(const at::Tensor& in, const at::Tensor& out, RedOp op) {
    hipStream_t cur = cur_stream();
    const int i = next_++ % kRing;
    DPA_CHECK_HIP(hipEventRecord(fork_[i], cur));
    DPA_CHECK_HIP(hipStreamWaitEvent(stream_.stream(), fork_[i], 0));
    chunked(in, out, op);
    DPA_CHECK_HIP(hipEventRecord(join_[i], stream_.stream()));
    DPA_CHECK_HIP(hipStreamWaitEvent(cur, join_[i], 0));
  }
  std::string async_error() override { return x_->error_string(); }
  void abort_now() override { x_->abort(); }
  std::string debug_state() override { return x_->debug_state(2.0); }

 private:
  // Tensors larger than the workspace slot (ResNet-50 DDP buckets) go as back-to-back
  // one-shot launches over slot-sized views; max_elems() is a multiple of kChunkElems,
  // so every view keeps the 16-B alignment of the base pointer.
  void chunked(const at::Tensor& in, const at::Tensor& out, RedOp op) {
    const int64_t n = in.numel(), m = x_->max_elems();
    if (n <= m) {
      x_->all_reduce(in, out, op, stream_.stream());
      return;
    }
    if (x_->supports_twoshot(in) && x_->supports_twoshot(out)) {
      x_->all_reduce_twoshot(in, out, op, stream_.stream());
      return;
    }
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && out.numel() == n,
                "xgmi all_reduce: chunked path needs contiguous same-size tensors");
    const auto fi = in.view(-1), fo = out.view(-1);
    for (int64_t o = 0; o < n; o += m) {
      const int64_t k = std::min(m, n - o);
      x_->all_reduce(fi.narrow(0, o, k), fo.narrow(0, o, k), op, stream_.stream());
    }
  }

  static constexpr int kSlots = 256, kRing = 64;
  std::shared_ptr<xgmi::XgmiComm> x_;
  c10::hip::HIPStream stream_;
  hipEvent_t slot_[kSlots] = {};
  hipEvent_t fork_[kRing] = {};
  hipEvent_t join_[kRing] = {};
  int next_ = 0;
};

void register_xgmi(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("xgmi", "one-shot all-reduce over xGMI peer-mapped workspaces");
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
  py::class_<xgmi::XgmiComm, std::shared_ptr<xgmi::XgmiComm>>(s, "XgmiComm")
      .def(py::init<int, int, int, long long, double, long long>(), py::arg("rank"), py::arg("world"),
           py::arg("device"), py::arg("max_bytes") = 1 << 20, py::arg("timeout_s") = 600.0,
           py::arg("twoshot_max_bytes") = 0)
      .def("handle", &xgmi::XgmiComm::handle)
      .def("open", &xgmi::XgmiComm::open)
      .def("supports", &xgmi::XgmiComm::supports)
      .def("all_reduce",
           [](xgmi::XgmiComm& c, at::Tensor t, const std::string& op, c10::optional<at::Tensor> out) {
             at::Tensor dst = out.has_value() ? *out : t;
             c.all_reduce(t, dst, parse_op(op), nullptr);
             return dst;
           },
           py::arg("t"), py::arg("op") = "sum", py::arg("out") = py::none())
      .def("wide_probe", &xgmi::XgmiComm::wide_probe, py::arg("inp"), py::arg("out"), py::arg("nblk"))
      .def("debug_state", &xgmi::XgmiComm::debug_state, py::arg("wait_s") = 2.0)
      .def("site_probe", &xgmi::XgmiComm::site_probe, py::arg("site"), py::arg("inp"), py::arg("out"),
           py::arg("grid") = 1)
      .def("all_reduce_twoshot",
           [](xgmi::XgmiComm& c, at::Tensor t, const std::string& op, c10::optional<at::Tensor> out) {
             at::Tensor dst = out.has_value() ? *out : t;
             c.all_reduce_twoshot(t, dst, parse_op(op), nullptr);
             return dst;
           },
           py::arg("t"), py::arg("op") = "sum", py::arg("out") = py::none())
      .def("supports_twoshot", &xgmi::XgmiComm::supports_twoshot)
      .def("set_twoshot_blocks", &xgmi::XgmiComm::set_twoshot_blocks)
      .def_property_readonly("twoshot_max_bytes", &xgmi::XgmiComm::twoshot_max_bytes)
      .def("error", &xgmi::XgmiComm::error)
      .def("error_string", &xgmi::XgmiComm::error_string)
      .def("abort", &xgmi::XgmiComm::abort)
      .def("set_timeout", &xgmi::XgmiComm::set_timeout)
      .def("close", &xgmi::XgmiComm::close)
      .def_property_readonly("max_bytes", &xgmi::XgmiComm::max_bytes)
      .def_property_readonly("workspace_bytes", &xgmi::XgmiComm::workspace_bytes)
      .def_property_readonly("rank", &xgmi::XgmiComm::rank)
      .def_property_readonly("world_size", &xgmi::XgmiComm::world);
  // registered after comm.Collective (bind.cpp registers comm first)
  py::class_<XgmiCollective, Collective, std::shared_ptr<XgmiCollective>>(s, "XgmiCollective")
      .def(py::init<std::shared_ptr<xgmi::XgmiComm>>())
      .def("all_reduce",
           [](XgmiCollective& c, at::Tensor t, const std::string& op, c10::optional<at::Tensor> out) {
             at::Tensor dst = out.has_value() ? *out : t;
             c.all_reduce(t, dst, parse_op(op));
             return dst;
           },
           py::arg("t"), py::arg("op") = "sum", py::arg("out") = py::none());
}

}  // namespace dpa
