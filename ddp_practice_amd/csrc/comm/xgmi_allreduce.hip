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
// Protocol (per block b of the grid; blocks are independent, no grid sync):
//   ep  = ctr[b] + 1                      ctr[b]: this rank's count of collectives
//                                          that had a block b (same on every rank:
//                                          every rank issues the same sequence)
//   par = ep & 1                           double-buffered slots/flags
//   1. store my chunk b into slot[par][me] of EVERY rank (incl. me)
//   2. system-scope release; flag[par][me][b] = ep on every rank
//   3. poll my flags[par][p][b] == ep for all p (bounded: timeout/abort -> error word)
//   4. system-scope acquire; out[chunk b] = op over p = 0..W-1 of slot[par][p]
//      (same order on every rank -> bit-identical results everywhere)
//   5. ctr[b] = ep
// Reuse safety: a rank writes slot parity par of epoch ep+2 only after it saw
// every peer's flag for ep+1, which each peer raised after finishing ep.
//
// Workspaces are hipExtMallocWithFlags(hipDeviceMallocUncached): neither side
// caches them in its XCD L2, so the only ordering needed is the system-scope
// release/acquire pair around the flag.  Everything is enqueue-only (a kernel
// launch), so a collective can be captured into a hipGraph and replayed: the
// epoch lives in device memory and advances on replay.
#include <c10/hip/HIPGuard.h>

#include <atomic>
#include <cstring>

#include "comm/xgmi.h"
#include "common.h"

namespace dpa {
namespace xgmi {

constexpr int kThreads = 256;
constexpr int kVecBytes = 16;                         // one 16-B store per lane per rank
constexpr int kChunkBytes = kThreads * kVecBytes * 2;  // 8 KB of payload per block

struct Args {
  Peers peers;
  const char* in;
  char* out;
  long long nbytes;         // payload bytes (multiple of the element size)
  long long slot_bytes;     // per-rank slot size in the workspace
  long long flags_off;      // byte offset of the flag array in every workspace
  long long ctr_off;        // byte offset of this rank's epoch counters
  int rank, world, max_blocks;
  int* err;                 // host-mapped: 0 ok, 1 timeout, 2 aborted
  const int* abort_flag;    // host-mapped: non-zero -> stop waiting
  long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ uint32_t* flag_ptr(char* ws, const Args& a, int par, int src, int b) {
  return reinterpret_cast<uint32_t*>(ws + a.flags_off) + ((size_t)(par * kMaxRanks + src) * a.max_blocks + b);
}

template <typename T>
__device__ __forceinline__ float to_f(T v) { return Cvt<T>::to_f(v); }

// op: 0 sum, 1 avg, 2 max, 3 min
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void oneshot_kernel(Args a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = a.peers.base[a.rank];
  uint32_t* ctr = reinterpret_cast<uint32_t*>(mine + a.ctr_off) + b;
  __shared__ uint32_t s_ep;
  __shared__ int s_fail;
  if (tid == 0) {
    s_ep = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_fail = 0;
  }
  __syncthreads();
  const uint32_t ep = s_ep;
  const int par = ep & 1;
  const long long c0 = (long long)b * kChunkBytes;
  const long long cb = min((long long)kChunkBytes, a.nbytes - c0);
  const long long slot0 = (long long)par * kMaxRanks * a.slot_bytes;

  // 1. push my chunk into slot[par][me] of every rank
  f32x4 v[2];
  int have[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const long long o = (long long)(k * kThreads + tid) * kVecBytes;
    have[k] = o < cb;
    if (cb - o >= kVecBytes) {
      v[k] = *reinterpret_cast<const f32x4*>(a.in + c0 + o);
    } else if (have[k]) {  // ragged tail: never read past the tensor
      v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint16_t* src = reinterpret_cast<const uint16_t*>(a.in + c0 + o);
      uint16_t* d = reinterpret_cast<uint16_t*>(&v[k]);
      for (int j = 0; j < (int)((cb - o) >> 1); ++j) d[j] = src[j];
    }
  }
  for (int p = 0; p < a.world; ++p) {
    char* dst = a.peers.base[p] + slot0 + (long long)a.rank * a.slot_bytes + c0;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (have[k]) *reinterpret_cast<f32x4*>(dst + (long long)(k * kThreads + tid) * kVecBytes) = v[k];
  }
  // 2. release (every storing lane), then one lane per destination raises the flag
  __threadfence_system();
  __syncthreads();
  if (tid < a.world) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag_ptr(a.peers.base[tid], a, par, a.rank, b), ep, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every rank's chunk b: one lane of wave 0 per source rank, bounded;
  //    wave 0 then acquires (invalidates this CU's caches) before the barrier
  if (tid < 64) {
    if (tid < a.world) {
      const uint32_t* f = flag_ptr(mine, a, par, tid, b);
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      unsigned polls = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != ep) {
        __builtin_amdgcn_s_sleep(1);
        if ((++polls & 1023u) == 0) {
          int why = 0;
          if (__hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) why = 2;
          else if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) why = 1;
          if (why) {
            __hip_atomic_store(a.err, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_fail = 1;
            break;
          }
        }
      }
    }
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (s_fail) return;  // fatal: the host sees the error word; epochs are no longer consistent

  // 4. reduce the W slots in rank order (identical on every rank)
  constexpr int E = kVecBytes / sizeof(T);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (!have[k]) continue;
    const long long o = c0 + (long long)(k * kThreads + tid) * kVecBytes;
    const int ne = (int)min((long long)E, (cb - (long long)(k * kThreads + tid) * kVecBytes) / (long long)sizeof(T));
    float acc[E];
    for (int p = 0; p < a.world; ++p) {
      const f32x4 raw = *reinterpret_cast<const f32x4*>(mine + slot0 + (long long)p * a.slot_bytes + o);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float x = to_f<T>(e[j]);
        if (p == 0) acc[j] = x;
        else if (OP == 2) acc[j] = fmaxf(acc[j], x);
        else if (OP == 3) acc[j] = fminf(acc[j], x);
        else acc[j] += x;
      }
    }
    T* dst = reinterpret_cast<T*>(a.out + o);
    if (ne == E) {
      f32x4 res;
      T* r = reinterpret_cast<T*>(&res);
#pragma unroll
      for (int j = 0; j < E; ++j) r[j] = Cvt<T>::from_f(OP == 1 ? acc[j] / (float)a.world : acc[j]);
      *reinterpret_cast<f32x4*>(dst) = res;
    } else {
      for (int j = 0; j < ne; ++j) dst[j] = Cvt<T>::from_f(OP == 1 ? acc[j] / (float)a.world : acc[j]);
    }
  }
  // 5. this block's epoch is done
  __syncthreads();
  if (tid == 0) __hip_atomic_store(ctr, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

XgmiComm::XgmiComm(int rank, int world, int device, long long slot_bytes, double timeout_s)
    : rank_(rank), world_(world), device_(device) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "xgmi: 1..", kMaxRanks, " ranks");
  TORCH_CHECK(rank >= 0 && rank < world);
  slot_bytes_ = ((std::max(slot_bytes, 1LL) + kChunkBytes - 1) / kChunkBytes) * kChunkBytes;
  max_blocks_ = (int)(slot_bytes_ / kChunkBytes);
  flags_off_ = 2LL * kMaxRanks * slot_bytes_;
  ctr_off_ = flags_off_ + 2LL * kMaxRanks * max_blocks_ * 4;
  ws_bytes_ = ((ctr_off_ + (long long)max_blocks_ * 4 + 4095) / 4096) * 4096;
  timeout_ticks_ = (long long)(timeout_s * 1e8);
  c10::hip::HIPGuard guard(device_);
  void* p = nullptr;
  DPA_CHECK_HIP(hipExtMallocWithFlags(&p, ws_bytes_, hipDeviceMallocUncached));
  DPA_CHECK_HIP(hipMemset(p, 0, ws_bytes_));
  DPA_CHECK_HIP(hipDeviceSynchronize());
  local_ = static_cast<char*>(p);
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
         (st == at::kFloat || st == at::kBFloat16 || st == at::kHalf) && t.nbytes() > 0 &&
         (long long)t.nbytes() <= slot_bytes_ && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

void XgmiComm::all_reduce(const at::Tensor& in, const at::Tensor& out, RedOp op, hipStream_t stream) {
  TORCH_CHECK(supports(in) && supports(out) && in.nbytes() == out.nbytes() &&
                  in.scalar_type() == out.scalar_type(),
              "xgmi all_reduce: unsupported tensor (device/dtype/size/alignment)");
  TORCH_CHECK(op != RedOp::PROD, "xgmi all_reduce: prod is not supported");
  Args a;
  a.peers = peers_;
  a.in = static_cast<const char*>(in.data_ptr());
  a.out = static_cast<char*>(out.data_ptr());
  a.nbytes = (long long)in.nbytes();
  a.slot_bytes = slot_bytes_;
  a.flags_off = flags_off_;
  a.ctr_off = ctr_off_;
  a.rank = rank_;
  a.world = world_;
  a.max_blocks = max_blocks_;
  a.err = dev_words_;
  a.abort_flag = dev_words_ + 1;
  a.timeout_ticks = timeout_ticks_;
  const int grid = (int)((a.nbytes + kChunkBytes - 1) / kChunkBytes);
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

int XgmiComm::error() const { return host_words_ ? __atomic_load_n(&host_words_[0], __ATOMIC_ACQUIRE) : 0; }

std::string XgmiComm::error_string() const {
  const int e = error();
  return e == 0 ? std::string() : e == 1 ? std::string("xgmi all-reduce: a peer never arrived (timeout)")
                                         : std::string("xgmi all-reduce: aborted");
}

void XgmiComm::abort() {
  if (host_words_) __atomic_store_n(&host_words_[1], 1, __ATOMIC_RELEASE);
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
    for (int i = 0; i < kRing; ++i) DPA_CHECK_HIP(hipEventCreateWithFlags(&fork_[i], hipEventDisableTiming));
  }
  ~XgmiCollective() override {
    for (auto& e : slot_) if (e) (void)hipEventDestroy(e);
    for (auto& e : fork_) if (e) (void)hipEventDestroy(e);
  }
  int rank() const override { return x_->rank(); }
  int world() const override { return x_->world(); }
  void all_reduce_async(at::Tensor t, RedOp op, int slot) override {
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    const int i = next_++ % kRing;
    DPA_CHECK_HIP(hipEventRecord(fork_[i], cur_stream()));
    DPA_CHECK_HIP(hipStreamWaitEvent(stream_.stream(), fork_[i], 0));
    x_->all_reduce(t, t, op, stream_.stream());
    DPA_CHECK_HIP(hipEventRecord(slot_[slot], stream_.stream()));
  }
  void wait(int slot, hipStream_t stream) override {
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    DPA_CHECK_HIP(hipStreamWaitEvent(stream ? stream : cur_stream(), slot_[slot], 0));
  }
  std::string async_error() override { return x_->error_string(); }
  void abort_now() override { x_->abort(); }

 private:
  static constexpr int kSlots = 256, kRing = 64;
  std::shared_ptr<xgmi::XgmiComm> x_;
  c10::hip::HIPStream stream_;
  hipEvent_t slot_[kSlots] = {};
  hipEvent_t fork_[kRing] = {};
  int next_ = 0;
};

void register_xgmi(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("xgmi", "one-shot all-reduce over xGMI peer-mapped workspaces");
  py::class_<xgmi::XgmiComm, std::shared_ptr<xgmi::XgmiComm>>(s, "XgmiComm")
      .def(py::init<int, int, int, long long, double>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("max_bytes") = 1 << 20, py::arg("timeout_s") = 600.0)
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
      .def(py::init<std::shared_ptr<xgmi::XgmiComm>>());
}

}  // namespace dpa
