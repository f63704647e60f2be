// In-kernel SyncBN exchange over xGMI ("fused site"): the all-reduce of a
// BatchNorm's per-channel sums runs inside the kernel that consumes them,
// instead of as a collective kernel of its own between producer and consumer.
//
// Why: at W > 1 every SyncBN all-reduce (2C+1 floats forward,
// 2C backward; /root/reference/ddp_main.py:120 convert_sync_batchnorm) is a
// launch in the critical path that moves a few hundred bytes.  The consumer
// kernel already reduces the producer's per-workgroup partial-sum slab to one
// row of local sums in its prologue (cb::bn_finalize / cb::bn_bwd_coef); with
// a site attached it then
//   1. (workgroup 0 only) stores that row as {fp32 value, epoch} granules into
//      slot[parity][me] of this site's region in EVERY peer's workspace,
//   2. (every workgroup) polls the W rows of its own region and sums them in
//      rank order -- bit-identical global sums on every rank and workgroup.
// The granule protocol is the one-shot all-reduce's (comm/xgmi_allreduce.hip):
// value and tag land in one 8-byte store, no flag, no fence.
//
// Epoch without host involvement (graph-replayable, any grid size <= kEpochWords): every
// site keeps one epoch word per workgroup index in this rank's memory.  Workgroup b of a
// launch reads word b (no atomic read-modify-write, no contention: its round trip hides
// behind the caller's slab loads), uses epoch = word + 1, and writes that epoch to words
// b, b + nblk, b + 2 nblk, ... -- so every word advances by exactly one per launch whatever
// the launch's workgroup count, all workgroups of a launch see the same epoch (launches of
// a site are stream-ordered; kernel boundaries make the words visible across XCDs), and
// every rank issues the same sequence of launches.  (Round 3 took tickets from shared
// words with device-scope atomics: same-address atomics of up to 224 workgroups serialized,
// and the last ticket of each word re-armed it with a second atomic.)
// Reuse safety as for the one-shot kernel: a rank writes parity p of epoch e+2
// only after its launch e+1 read every peer's e+1 row, which each peer wrote
// after its own launch e had completed.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

// The exchange's two workgroup barriers order LDS only (the epoch broadcast, the summed
// row): an LDS-only barrier (s_waitcnt lgkmcnt(0) + s_barrier) instead of __syncthreads(),
// whose vmcnt(0) made every wave wait for ALL its outstanding global operations -- the
// epoch-word stores and peer pushes just issued, and whatever loads the caller had in
// flight -- at every exchange, with nothing to wait for at W = 1.  Nothing after an
// exchange reads those stores inside the launch (the epoch words are read by the next
// launch, the pushes by the peers' polls).  DPA_XS_FULLBAR (experiment builds): the
// __syncthreads() form, for the A/B.
#ifdef DPA_XS_FULLBAR
#define DPA_XS_BARRIER() __syncthreads()
#elif defined(DPA_XS_NO_BAR)
#define DPA_XS_BARRIER() do {} while (0)
#else
#define DPA_XS_BARRIER()                          \
  do {                                            \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_s_barrier();                 \
  } while (0)
#endif

namespace dpa {
namespace xgmi {

constexpr int kMaxRanks = 8;
constexpr int kEpochWords = 512;  // epoch words per site: the largest site grid (7 x 64 images: conv1 weight gradient)
constexpr int kSites = 8;                                             // sites per communicator
constexpr int kSiteVals = 128;                                        // floats per rank row (>= 2C+1)
constexpr long long kSiteSlotBytes = kSiteVals * 8LL;                 // granules
constexpr long long kSiteBytes = 2LL * kMaxRanks * kSiteSlotBytes;   // both parities

// site ids (ops/convnet_fused.py): one per consumer launch of a step
enum : int { kSiteFwd1 = 0, kSiteFwd2 = 1, kSiteBwd2Dgrad = 2, kSiteBwd2Wgrad = 3, kSiteBwd1 = 4 };
// the statistics finishers of the ResNet kernels (conv_igemm.hip stat trees, bn_nhwc.hip
// fwd / bwd statistics): every SyncBN exchange of the network on ONE site, launch after
// launch on the compute stream, rows of up to kWideVals floats (2C+1, C <= 2048)
constexpr int kSiteWide = 5;
constexpr int kWideVals = 4224;
// the DDP gradient exchange inside the fused AMP-SGD kernel (XgmiComm::grad_site):
// its own epoch word, slots of the engine's full message size
constexpr int kSiteGrad = kSites - 1;

struct XSite {
  char* base[kMaxRanks] = {};            // this site's region in every rank's workspace (peer-mapped)
  char* mine = nullptr;                  // base[rank]: polled without a rank-indexed kernel-argument load
  unsigned long long* tick = nullptr;    // this rank's kEpochWords epoch words of the site;
                                         // nullptr: site inactive
  int rank = 0, world = 1;
  int* err = nullptr;                    // host-mapped: 1 timeout, 2 aborted
  const int* abort_flag = nullptr;
  long long timeout_ticks = 0;           // s_memrealtime ticks (100 MHz)
  long long slot_bytes = kSiteSlotBytes; // one rank's row of granules; a parity holds kMaxRanks rows
  long long max_vals = kSiteVals;        // floats per row
  int nblk = 0;                          // workgroups of a launch taking tickets (0: the whole grid;
                                         // set when one launch hosts several roles, each with its site)
  __host__ __device__ bool active() const { return tick != nullptr; }
};

// Every remote granule push of the engine (one-shot, two-shot, sites, the AMP-SGD gradient
// exchange) goes through these.  8-byte granules are the unit of atomicity (value and epoch
// tag together).  A single granule (sites, positioned rows, slab columns) is a system-scope
// relaxed atomic store: its visibility to the peer's system-scope polls is explicit in the
// memory model and costs nothing over a plain 8-B store (same instruction, sc0 sc1 bits).
// A granule PAIR (the bandwidth paths) is one naturally aligned 16-B vector store into the
// peer's hipDeviceMallocUncached workspace: as two 8-B system-scope atomic stores the
// two-shot all-reduce of 8 MiB took 96 vs 62 us with 2 ranks and 1040 vs 651 us with 8
// (profiles/r6c_push_store_ab.txt), twice the store instructions and half-width writes over
// the links.  DPA_PUSH_ATOMIC2 (experiment builds) selects the atomic pair for the A/B.
__device__ __forceinline__ void xgmi_put(unsigned long long* dst, unsigned long long g) {
  __hip_atomic_store(dst, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void xgmi_put2(unsigned long long* dst, unsigned long long a, unsigned long long b) {
#ifdef DPA_PUSH_ATOMIC2
  __hip_atomic_store(dst, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(dst + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  typedef __attribute__((ext_vector_type(2))) unsigned long long v2;
  *reinterpret_cast<v2*>(dst) = v2{a, b};
#endif
}

// Lane 0 of every workgroup, once per launch, as early as possible (the returned word is
// only needed by xsite_exchange: its round trip hides behind the caller's slab loads).
// bid: the workgroup's index among the launch's workgroups on this site.
// DPA_XS_NOOP (experiment builds, world-1 A/Bs only): ticket, exchange and advance compiled
// out -- the floor of what the exchanges cost a forced (W > 1-shaped) step on one GPU.
// Finer world-1 bisection switches (experiment builds): DPA_XS_NO_TICKET (no ticket load),
// DPA_XS_NO_ADVANCE (no epoch-word stores), DPA_XS_NO_BAR (no barriers in the exchange),
// DPA_XS_NO_XG (the AMP step's gradient average only).
#if defined(DPA_XS_NOOP) || defined(DPA_XS_NO_XG)
constexpr bool kXsNoop = true;
#else
constexpr bool kXsNoop = false;
#endif
__device__ __forceinline__ unsigned long long xsite_ticket(const XSite& xs, int bid) {
#if defined(DPA_XS_NOOP) || defined(DPA_XS_NO_TICKET)
  (void)xs;
  (void)bid;
  return 0ull;
#endif
  // (a plain load, plain epoch stores and advancing the words after the exchange measured no
  // faster on the forced step: profiles/r5o_xsite_mode_ab.txt, r5s_xsite_plain_ab.txt)
  return __hip_atomic_load(xs.tick + (bid < kEpochWords ? bid : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#if defined(DPA_TIMING) && defined(DPA_STAMP)
#define DPA_XS_STAMP(i) DPA_STAMP(i)
#else
#define DPA_XS_STAMP(i) do {} while (0)
#endif

// The launch's epoch from the word xsite_ticket read.
__device__ __forceinline__ uint32_t xsite_epoch(const XSite& xs, unsigned long long tk, int bid) {
  (void)xs;
  (void)bid;
  return (uint32_t)tk + 1u;
}

// Every thread of workgroup bid (nthr threads), after the epoch is known: advance this
// workgroup's residue class of epoch words (b, b + nblk, ...) to ep.  A grid larger than
// kEpochWords cannot keep its workgroups' epochs equal: flagged as an error (the exchange
// then gives up), and the host checks grids against it.
__device__ __forceinline__ void xsite_advance(const XSite& xs, uint32_t ep, int bid, int nthr) {
#ifdef DPA_XS_NO_ADVANCE
  return;
#endif
  const int nblk = xs.nblk > 0 ? xs.nblk : (int)(gridDim.x * gridDim.y * gridDim.z);
  const int tid = threadIdx.x;
  if (nblk > kEpochWords) {
    if (tid == 0) __hip_atomic_store(xs.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  for (int w = bid + tid * nblk; w < kEpochWords; w += nthr * nblk)
    __hip_atomic_store(xs.tick + w, (unsigned long long)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Checked every 256 polls of a bounded wait: 2 = aborted (watchdog), 1 = this wait timed
// out, -1 = an earlier exchange of this rank already failed (its error word is set):
// give up at once -- this rank's epochs no longer match its peers', so every later
// wait would only run into its own timeout; the poisoned engine then costs
// microseconds per exchange until the error is reported (host error word, watchdog).
__device__ __forceinline__ int give_up(const int* err, const int* abort_flag, long long t0, long long timeout_ticks) {
  if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return 2;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return -1;
  if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) return 1;
  return 0;
}

// Spin until granule *src carries epoch ep (bounded: abort flag / timeout ->
// error word, fail = true).  g: the granule already loaded.
__device__ __forceinline__ float xsite_wait(const XSite& xs, const unsigned long long* src, unsigned long long g,
                                            uint32_t ep, long long t0, unsigned& polls, bool& fail) {
  while (!fail && (uint32_t)(g >> 32) != ep) {
    __builtin_amdgcn_s_sleep(1);
    g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((++polls & 255u) == 0) {
      const int why = give_up(xs.err, xs.abort_flag, t0, xs.timeout_ticks);
      if (why) {
        if (why > 0) __hip_atomic_store(xs.err, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        fail = true;
      }
    }
  }
  return fail ? 0.f : __uint_as_float((uint32_t)g);
}

// vals: n (<= kSiteVals, <= blockDim.x) floats of LDS holding this rank's local
// row; replaced by the rank-ordered sum over all ranks.  tk: lane 0's ticket.
// bid: the workgroup's index in its role (the role's workgroup 0 pushes).  Called by
// every thread of the workgroup; ends with an LDS-only barrier.
__device__ __forceinline__ void xsite_exchange(const XSite& xs, float* vals, int n, unsigned long long tk,
                                               int bid, int nthr = 256 /* <= the workgroup size */) {
#ifdef DPA_XS_NOOP
  return;
#endif
  __shared__ uint32_t ep_s;
  const int tid = threadIdx.x;
  const bool pusher = bid == 0;
  if (tid == 0) ep_s = xsite_epoch(xs, tk, bid);
  DPA_XS_BARRIER();
  DPA_XS_STAMP(13);
  const uint32_t ep = ep_s;
  if (tid < n) {
    const long long par = (long long)(ep & 1u) * kMaxRanks * xs.slot_bytes;
    const float mine = vals[tid];
    const unsigned long long gm = ((unsigned long long)ep << 32) | (unsigned long long)__float_as_uint(mine);
    // peers unrolled with a predicate: the kernel-argument loads of base[p] carry static
    // offsets (issued together, not a rank-indexed dependent chain in a loop)
    if (pusher) {
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p)
        if (p < xs.world && p != xs.rank)
          xgmi_put(reinterpret_cast<unsigned long long*>(xs.base[p] + par + (long long)xs.rank * xs.slot_bytes +
                                                         (long long)tid * 8),
                   gm);
    }
    // every peer's granule loaded before the first tag check (one round trip)
    unsigned long long g[kMaxRanks];
    const unsigned long long* src[kMaxRanks];
#pragma unroll
    for (int p = 0; p < kMaxRanks; ++p) {
      src[p] = reinterpret_cast<const unsigned long long*>(xs.mine + par + (long long)p * xs.slot_bytes +
                                                           (long long)tid * 8);
      g[p] = (p < xs.world && p != xs.rank) ? __hip_atomic_load(src[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                            : gm;
    }
    float acc = 0.f;
    bool fail = false;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned polls = 0;
#pragma unroll
    for (int p = 0; p < kMaxRanks; ++p) {
      if (p >= xs.world) continue;
      const float x = xsite_wait(xs, src[p], g[p], ep, t0, polls, fail);
      acc = p == 0 ? x : acc + x;
    }
    vals[tid] = acc;  // only this lane reads or writes slot tid in here
  }
  DPA_XS_STAMP(14);
  // the epoch words last: read only by the site's next launch, so their stores drain behind
  // the LDS-only barrier and the caller's work instead of ahead of the polls' first wait
  // (an s_waitcnt vmcnt(0) there also retired every store issued before it)
  xsite_advance(xs, ep, bid, nthr);
  DPA_XS_BARRIER();
  DPA_XS_STAMP(15);
}

// ---------------------------------------------------------------------------
// Positioned form, for launches whose row is split over several finisher workgroups
// (the last arriver of each channel slice of a statistics tree): each lane exchanges the
// values it owns at their row positions.  Lane 0 of every finisher takes one ticket
// (xsite_ticket with XSite.nblk = the launch's finisher count) and the launch's epoch
// (xsite_epoch); a lane pushes all its positions first (xsite_push_at), then pulls them
// (xsite_pull_at: every peer's granule, summed in rank order).  Same granules, parities
// and reuse argument as above: positions are disjoint between a launch's finishers.
__device__ __forceinline__ void xsite_push_at(const XSite& xs, uint32_t ep, int pos, float mine) {
  const long long off = (long long)(ep & 1u) * kMaxRanks * xs.slot_bytes + (long long)xs.rank * xs.slot_bytes +
                        (long long)pos * 8;
  const unsigned long long gm = ((unsigned long long)ep << 32) | (unsigned long long)__float_as_uint(mine);
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p)
    if (p < xs.world && p != xs.rank) xgmi_put(reinterpret_cast<unsigned long long*>(xs.base[p] + off), gm);
}

__device__ __forceinline__ float xsite_pull_at(const XSite& xs, uint32_t ep, int pos, float mine, long long t0,
                                               unsigned& polls, bool& fail) {
  const long long off = (long long)(ep & 1u) * kMaxRanks * xs.slot_bytes + (long long)pos * 8;
  unsigned long long g[kMaxRanks];
  const unsigned long long* src[kMaxRanks];
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {  // every peer's granule in flight before the first check
    src[p] = reinterpret_cast<const unsigned long long*>(xs.mine + off + (long long)p * xs.slot_bytes);
    g[p] = (p < xs.world && p != xs.rank) ? __hip_atomic_load(src[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                          : (((unsigned long long)ep << 32) | __float_as_uint(mine));
  }
  float acc = 0.f;
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {
    if (p >= xs.world) continue;
    const float x = xsite_wait(xs, src[p], g[p], ep, t0, polls, fail);
    acc = p == 0 ? x : acc + x;
  }
  return acc;
}

// A finisher's slice in LDS: vals[i] (i < n) sits at row position pos(i); replaced by the
// rank-ordered global sums.  tk: lane 0's ticket; bid: the finisher's index (< nblk);
// nthr: the workgroup size.  Called by every thread; ends with a barrier.
template <typename PosF>
__device__ __forceinline__ void xsite_exchange_slice(const XSite& xs, float* vals, int n, PosF pos,
                                                     unsigned long long tk, int bid, int nthr) {
#ifdef DPA_XS_NOOP
  return;
#endif
  __shared__ uint32_t ep_s;
  const int tid = threadIdx.x;
  if (tid == 0) ep_s = xsite_epoch(xs, tk, bid);
  DPA_XS_BARRIER();
  const uint32_t ep = ep_s;
  for (int i = tid; i < n; i += nthr) xsite_push_at(xs, ep, pos(i), vals[i]);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  unsigned polls = 0;
  bool fail = false;
  for (int i = tid; i < n; i += nthr) vals[i] = xsite_pull_at(xs, ep, pos(i), vals[i], t0, polls, fail);
  xsite_advance(xs, ep, bid, nthr);  // last, as in xsite_exchange
  DPA_XS_BARRIER();
}

}  // namespace xgmi
}  // namespace dpa
