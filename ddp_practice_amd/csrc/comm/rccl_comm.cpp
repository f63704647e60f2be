// RCCL communicator: one per process (one process per GPU), collectives on a
// dedicated high-priority HIP stream, fenced to the caller's compute stream by
// events.  Every call is hipGraph-capturable (event record/wait + RCCL kernel
// launches only; no host sync except barrier()).
//
// Replaces the reference's implicit ProcessGroupNCCL usage
// (/root/reference/ddp_main.py:73 init_process_group("nccl"), :108-109
// dist.reduce, and the collectives inside DDP / SyncBatchNorm).  The unique id
// is exchanged through the torch TCPStore created by init_process_group(env://)
// (Python side: ddp_practice_amd/parallel/comm.py).
//
// On MI355X the 8 GPUs of a node are fully connected by xGMI (7 links per GPU);
// RCCL picks ring/tree/direct algorithms per size.  The SyncBN/ConvNet
// messages are a few hundred bytes to 116 KB (latency-bound); ResNet-50 buckets
// are tens of MB (link-bandwidth-bound) — see parallel/ddp.py for bucket sizing.
#include <rccl/rccl.h>
#include <c10/hip/HIPGuard.h>

#include <atomic>
#include <chrono>
#include <thread>

#include "comm/collective.h"
#include "comm/xgmi.h"
#include "common.h"

namespace dpa {

RedOp parse_op(const std::string& op) {
  if (op == "sum") return RedOp::SUM;
  if (op == "prod") return RedOp::PROD;
  if (op == "max") return RedOp::MAX;
  if (op == "min") return RedOp::MIN;
  if (op == "avg") return RedOp::AVG;
  TORCH_CHECK(false, "unknown reduce op ", op);
  return RedOp::SUM;
}

namespace comm {

#define DPA_NCCL(cmd)                                                                         \
  do {                                                                                        \
    ncclResult_t _r = (cmd);                                                                  \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error ", ncclGetErrorString(_r), " (", (int)_r,      \
                ") at ", __FILE__, ":", __LINE__, " ", ncclGetLastError(nullptr));            \
  } while (0)

static ncclDataType_t nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
  return ncclFloat32;
}

static ncclRedOp_t nccl_op(RedOp op) {
  switch (op) {
    case RedOp::SUM: return ncclSum;
    case RedOp::PROD: return ncclProd;
    case RedOp::MAX: return ncclMax;
    case RedOp::MIN: return ncclMin;
    case RedOp::AVG: return ncclAvg;
  }
  return ncclSum;
}

class RcclComm : public Collective {
 public:
  static pybind11::bytes unique_id() {
    ncclUniqueId id;
    DPA_NCCL(ncclGetUniqueId(&id));
    return pybind11::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  }

  static std::string version() {
    int v = 0;
    ncclGetVersion(&v);
    return std::to_string(v);
  }

  RcclComm(const std::string& uid, int rank, int world, int device)
      : rank_(rank), world_(world), device_(device),
        stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, device)) {
    TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "bad RCCL unique id size ", uid.size());
    ncclUniqueId id;
    memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    c10::hip::HIPGuard guard(device);
    {
      pybind11::gil_scoped_release nogil;  // init rendezvous blocks until every rank arrives
      ncclComm_t c = nullptr;
      DPA_NCCL(ncclCommInitRank(&c, world, id, rank));
      comm_ = c;
    }
    for (int i = 0; i < kRing; ++i) {
      DPA_CHECK_HIP(hipEventCreateWithFlags(&fork_[i], hipEventDisableTiming));
      DPA_CHECK_HIP(hipEventCreateWithFlags(&join_[i], hipEventDisableTiming));
    }
    for (int i = 0; i < kSlots; ++i) DPA_CHECK_HIP(hipEventCreateWithFlags(&slot_[i], hipEventDisableTiming));
  }

  ~RcclComm() override { destroy(); }

  void destroy() {
    ncclComm_t c = comm_.exchange(nullptr);
    if (c != nullptr) {
      hipStreamSynchronize(stream_.stream());
      ncclCommDestroy(c);
    }
    for (int i = 0; i < kRing; ++i) {
      if (fork_[i]) hipEventDestroy(fork_[i]);
      if (join_[i]) hipEventDestroy(join_[i]);
      fork_[i] = join_[i] = nullptr;
    }
    for (int i = 0; i < kSlots; ++i) {
      if (slot_[i]) hipEventDestroy(slot_[i]);
      slot_[i] = nullptr;
    }
  }

  // Abort outstanding work (failure handling / watchdog path).
  void abort() {
    if (auto x = xgmi_) x->abort();
    ncclComm_t c = comm_.exchange(nullptr);
    if (c != nullptr) ncclCommAbort(c);
  }
  void abort_now() override { abort(); }
  std::string debug_state() override {
    auto x = xgmi_;
    return x ? x->debug_state(2.0) : std::string();
  }

  std::string async_error() override {
    if (auto x = xgmi_; x && x->error() != 0) return x->error_string();
    ncclComm_t c = comm_.load();
    if (c == nullptr) return "destroyed";
    ncclResult_t st = ncclSuccess;
    ncclCommGetAsyncError(c, &st);
    return st == ncclSuccess ? std::string() : std::string(ncclGetErrorString(st));
  }

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  int device() const { return device_; }
  uintptr_t stream_handle() const { return reinterpret_cast<uintptr_t>(stream_.stream()); }

  // ---------------------------------------------------------------- sync-style
  at::Tensor all_reduce(at::Tensor t, const std::string& op, c10::optional<at::Tensor> out) {
    check(t);
    at::Tensor dst = out.has_value() ? *out : t;
    if (out.has_value()) {
      check(dst);
      TORCH_CHECK(dst.numel() == t.numel() && dst.scalar_type() == t.scalar_type());
    }
    const RedOp rop = parse_op(op);
    // on the comm stream like every collective: one total order per rank = issue order
    fenced([&](hipStream_t s) {
      if (const int r = route(t, dst, rop); r == 1)
        xgmi_->all_reduce(t, dst, rop, s);
      else if (r == 2)
        xgmi_->all_reduce_twoshot(t, dst, rop, s);
      else
        DPA_NCCL(ncclAllReduce(t.data_ptr(), dst.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(rop),
                               comm_.load(), s));
    });
    return dst;
  }

  void all_gather(at::Tensor out, at::Tensor in) {
    check(in); check(out);
    TORCH_CHECK(out.numel() == in.numel() * world_ && out.scalar_type() == in.scalar_type());
    fenced([&](hipStream_t s) {
      DPA_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in), comm_.load(), s));
    });
  }

  void reduce_scatter(at::Tensor out, at::Tensor in, const std::string& op) {
    check(in); check(out);
    TORCH_CHECK(in.numel() == out.numel() * world_ && out.scalar_type() == in.scalar_type());
    fenced([&](hipStream_t s) {
      DPA_NCCL(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(in),
                                 nccl_op(parse_op(op)), comm_.load(), s));
    });
  }

  void broadcast(at::Tensor t, int root) {
    check(t);
    fenced([&](hipStream_t s) {
      DPA_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_.load(), s));
    });
  }

  void reduce(at::Tensor t, int root, const std::string& op) {
    check(t);
    fenced([&](hipStream_t s) {
      DPA_NCCL(ncclReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(parse_op(op)), root,
                          comm_.load(), s));
    });
  }

  // out/in: [world * chunk] laid out by destination / source rank.
  void all_to_all(at::Tensor out, at::Tensor in) {
    check(in); check(out);
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % world_ == 0);
    const size_t chunk = in.numel() / world_;
    const size_t esz = in.element_size();
    fenced([&](hipStream_t s) {
      DPA_NCCL(ncclGroupStart());
      for (int r = 0; r < world_; ++r) {
        DPA_NCCL(ncclSend(static_cast<char*>(in.data_ptr()) + r * chunk * esz, chunk, nccl_dtype(in), r, comm_.load(), s));
        DPA_NCCL(ncclRecv(static_cast<char*>(out.data_ptr()) + r * chunk * esz, chunk, nccl_dtype(in), r, comm_.load(), s));
      }
      DPA_NCCL(ncclGroupEnd());
    });
  }

  // Host-blocking barrier: a 1-element all-reduce, then wait for the comm stream.
  void barrier() {
    if (!barrier_buf_.defined())
      barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
    all_reduce(barrier_buf_, "sum", c10::nullopt);
    pybind11::gil_scoped_release nogil;
    DPA_CHECK_HIP(hipStreamSynchronize(stream_.stream()));
  }

  // ------------------------------------------------------------------- async
  void all_reduce_async(at::Tensor t, RedOp op, int slot) override {
    check(t);
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    hipStream_t cur = cur_stream();
    const int i = next_++ % kRing;
    DPA_CHECK_HIP(hipEventRecord(fork_[i], cur));
    DPA_CHECK_HIP(hipStreamWaitEvent(stream_.stream(), fork_[i], 0));
    if (const int r = route(t, t, op); r == 1)
      xgmi_->all_reduce(t, t, op, stream_.stream());
    else if (r == 2)
      xgmi_->all_reduce_twoshot(t, t, op, stream_.stream());
    else
      DPA_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_.load(),
                             stream_.stream()));
    DPA_CHECK_HIP(hipEventRecord(slot_[slot], stream_.stream()));
  }

  // Route all-reduces of at most `max_bytes` to the one-shot xGMI engine and the ones
  // above it, up to `twoshot_max_bytes`, to its two-shot (reduce-scatter + all-gather);
  // RCCL above that (max_bytes <= 0: detach).  Every rank must attach the same way.
  void attach_xgmi(std::shared_ptr<xgmi::XgmiComm> x, long long max_bytes, long long twoshot_max_bytes) {
    if (x) {
      TORCH_CHECK(x->device() == device_ && x->world() == world_ && x->rank() == rank_,
                  "xgmi engine does not match this communicator");
    }
    xgmi_ = max_bytes > 0 ? std::move(x) : nullptr;
    xgmi_max_ = xgmi_ ? std::min(max_bytes, xgmi_->max_bytes()) : 0;
    ts_max_ = xgmi_ ? std::min(twoshot_max_bytes, xgmi_->twoshot_max_bytes()) : 0;
  }
  long long xgmi_max_bytes() const { return xgmi_ ? xgmi_max_ : 0; }
  long long twoshot_max_bytes() const { return xgmi_ ? ts_max_ : 0; }

  void wait(int slot, hipStream_t stream) override {
    TORCH_CHECK(slot >= 0 && slot < kSlots, "slot out of range");
    DPA_CHECK_HIP(hipStreamWaitEvent(stream ? stream : cur_stream(), slot_[slot], 0));
  }

 private:
  // 0: RCCL, 1: xGMI one-shot, 2: xGMI two-shot.  A pure function of (size, dtype,
  // alignment, op): identical on every rank for the same collective.
  int route(const at::Tensor& in, const at::Tensor& out, RedOp op) const {
    if (!xgmi_ || op == RedOp::PROD) return 0;
    const long long nb = (long long)in.nbytes();
    if (nb <= xgmi_max_ && xgmi_->supports(in) && xgmi_->supports(out)) return 1;
    if (nb <= ts_max_ && xgmi_->supports_twoshot(in) && xgmi_->supports_twoshot(out)) return 2;
    return 0;
  }

  static constexpr int kRing = 64;
  static constexpr int kSlots = 256;

  void check(const at::Tensor& t) const {
    TORCH_CHECK(comm_.load() != nullptr, "communicator destroyed or aborted");
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL tensors must be contiguous device tensors");
    TORCH_CHECK(t.get_device() == device_, "tensor on device ", t.get_device(), ", communicator on ", device_);
  }

  template <typename F>
  void fenced(F&& f) {
    hipStream_t cur = cur_stream();
    const int i = next_++ % kRing;
    DPA_CHECK_HIP(hipEventRecord(fork_[i], cur));
    DPA_CHECK_HIP(hipStreamWaitEvent(stream_.stream(), fork_[i], 0));
    f(stream_.stream());
    DPA_CHECK_HIP(hipEventRecord(join_[i], stream_.stream()));
    DPA_CHECK_HIP(hipStreamWaitEvent(cur, join_[i], 0));
  }

  std::atomic<ncclComm_t> comm_{nullptr};
  int rank_, world_, device_;
  c10::hip::HIPStream stream_;
  hipEvent_t fork_[kRing] = {};
  hipEvent_t join_[kRing] = {};
  hipEvent_t slot_[kSlots] = {};
  int next_ = 0;
  at::Tensor barrier_buf_;
  std::shared_ptr<xgmi::XgmiComm> xgmi_;
  long long xgmi_max_ = 0, ts_max_ = 0;
};

// Python-implemented collective (torch.distributed / gloo on CPU; tests).
class PyCollective : public Collective {
 public:
  explicit PyCollective(pybind11::object obj) : obj_(std::move(obj)) {
    pybind11::gil_scoped_acquire g;
    rank_ = obj_.attr("rank").cast<int>();
    world_ = obj_.attr("world_size").cast<int>();
  }
  ~PyCollective() override {
    pybind11::gil_scoped_acquire g;
    obj_ = pybind11::object();
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void all_reduce_async(at::Tensor t, RedOp op, int) override {
    pybind11::gil_scoped_acquire g;
    const char* names[] = {"sum", "prod", "max", "min", "avg"};
    obj_.attr("all_reduce_")(t, names[(int)op]);
  }
  void wait(int, hipStream_t) override {}

 private:
  pybind11::object obj_;
  int rank_ = 0, world_ = 1;
};

}  // namespace comm

void register_comm(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("comm", "RCCL communicator");
  py::class_<Collective, std::shared_ptr<Collective>>(s, "Collective")
      .def_property_readonly("rank", &Collective::rank)
      .def_property_readonly("world_size", &Collective::world);
  py::class_<comm::RcclComm, Collective, std::shared_ptr<comm::RcclComm>>(s, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::arg("uid"), py::arg("rank"), py::arg("world"),
           py::arg("device"))
      .def_static("unique_id", &comm::RcclComm::unique_id)
      .def_static("version", &comm::RcclComm::version)
      .def_property_readonly("device", &comm::RcclComm::device)
      .def_property_readonly("stream_handle", &comm::RcclComm::stream_handle)
      .def("all_reduce", &comm::RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum",
           py::arg("out") = py::none())
      .def("all_gather", &comm::RcclComm::all_gather)
      .def("reduce_scatter", &comm::RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum")
      .def("broadcast", &comm::RcclComm::broadcast)
      .def("reduce", &comm::RcclComm::reduce, py::arg("t"), py::arg("root"), py::arg("op") = "sum")
      .def("all_to_all", &comm::RcclComm::all_to_all)
      .def("barrier", &comm::RcclComm::barrier)
      .def("all_reduce_async", [](comm::RcclComm& c, at::Tensor t, const std::string& op, int slot) {
        c.all_reduce_async(t, parse_op(op), slot);
      })
      .def("wait", [](comm::RcclComm& c, int slot) { c.wait(slot, nullptr); })
      .def("attach_xgmi", &comm::RcclComm::attach_xgmi, py::arg("engine"), py::arg("max_bytes"),
           py::arg("twoshot_max_bytes") = 0)
      .def_property_readonly("xgmi_max_bytes", &comm::RcclComm::xgmi_max_bytes)
      .def_property_readonly("twoshot_max_bytes", &comm::RcclComm::twoshot_max_bytes)
      .def("async_error", &comm::RcclComm::async_error)
      .def("abort", &comm::RcclComm::abort)
      .def("destroy", &comm::RcclComm::destroy);
  py::class_<comm::PyCollective, Collective, std::shared_ptr<comm::PyCollective>>(s, "PyCollective")
      .def(py::init<py::object>());
}

}  // namespace dpa
