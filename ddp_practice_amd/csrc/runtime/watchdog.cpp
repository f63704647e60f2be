// Collective / step watchdog and roctx tracing.
//
// The reference has no failure detection of its own: it relies on
// ProcessGroupNCCL's watchdog thread (10 min default timeout,
// torch/distributed/constants.py:21) and on the launcher tearing the group
// down (mp.spawn join, torchrun's agent with TORCH_NCCL_ASYNC_ERROR_HANDLING=1;
// SURVEY.md §5).  This framework owns its communicator, so it owns the
// watchdog too:
//
//   * tick(): records a HIP event on the caller's current stream after the work
//     of one step (collectives included).  A background thread polls the oldest
//     outstanding event; if it has not completed ``timeout`` seconds after it
//     was recorded, the device made no progress (typically a peer that never
//     entered a collective) -> report, ncclCommAbort (unblocks the spinning RCCL
//     kernels so the GPU is left usable) and _Exit(code) so the launcher tears
//     the other ranks down.
//   * heartbeat(): host-only progress (CPU/gloo ranks, host loops): no
//     heartbeat for ``timeout`` seconds while armed -> same failure path.
//   * the communicator's asynchronous error state is polled too.
//
// Ticks issued while the stream is being captured are ignored (a captured
// event record would be a graph node, not a progress marker).
#include <hip/hip_runtime.h>
#include <c10/hip/HIPStream.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>

#include "comm/collective.h"
#include "common.h"

namespace dpa {
namespace rt {

using Clock = std::chrono::steady_clock;

class Watchdog {
 public:
  Watchdog(double timeout_s, std::shared_ptr<Collective> comm, int exit_code, std::string tag, double poll_s)
      : timeout_(timeout_s), poll_(poll_s), comm_(std::move(comm)), exit_code_(exit_code), tag_(std::move(tag)) {
    TORCH_CHECK(timeout_s > 0 && poll_s > 0, "watchdog timeout and poll interval must be positive");
    last_beat_ = Clock::now();
    thread_ = std::thread([this] { loop(); });
  }

  ~Watchdog() { stop(); }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stopping_) return;
      stopping_ = true;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
    for (auto& p : pending_) hipEventDestroy(p.first);
    pending_.clear();
    for (auto e : free_) hipEventDestroy(e);
    free_.clear();
  }

  // Device progress marker on the current stream.
  void tick() {
    hipStream_t s = cur_stream();
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DPA_CHECK_HIP(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) return;
    std::lock_guard<std::mutex> g(mu_);
    if (pending_.size() >= kMaxPending) return;  // the oldest marker still bounds the wait
    hipEvent_t e;
    if (!free_.empty()) {
      e = free_.back();
      free_.pop_back();
    } else {
      DPA_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    DPA_CHECK_HIP(hipEventRecord(e, s));
    pending_.emplace_back(e, Clock::now());
    ++ticks_;
  }

  // Host progress marker; the first call arms host-side monitoring.
  void heartbeat() {
    std::lock_guard<std::mutex> g(mu_);
    last_beat_ = Clock::now();
    host_armed_ = true;
  }

  void disarm() {
    std::lock_guard<std::mutex> g(mu_);
    host_armed_ = false;
  }

  // What the rank last reported doing (host side, e.g. "epoch 0: step 112 queued"): named
  // in the report, so a stall record says which step the stuck device work belongs to.
  void note(std::string what) {
    std::lock_guard<std::mutex> g(mu_);
    note_ = std::move(what);
  }

  int64_t ticks() const { return ticks_.load(); }
  int64_t outstanding() {
    std::lock_guard<std::mutex> g(mu_);
    return (int64_t)pending_.size();
  }
  bool fired() const { return fired_.load(); }

  // Testing hook: run the failure path without exiting.
  void set_exit(bool do_exit) { do_exit_ = do_exit; }
  std::string reason() {
    std::lock_guard<std::mutex> g(mu_);
    return reason_;
  }

 private:
  static constexpr size_t kMaxPending = 4096;

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stopping_) {
      cv_.wait_for(lk, std::chrono::duration<double>(poll_));
      if (stopping_ || fired_) break;
      const auto now = Clock::now();
      // retire completed device markers (in order: one stream)
      while (!pending_.empty()) {
        hipError_t q = hipEventQuery(pending_.front().first);
        if (q == hipErrorNotReady) break;
        if (q != hipSuccess) {
          (void)hipGetLastError();
          fire(lk, std::string("device error while polling progress: ") + hipGetErrorString(q));
          return;
        }
        free_.push_back(pending_.front().first);
        pending_.pop_front();
      }
      if (!pending_.empty()) {
        const double age = std::chrono::duration<double>(now - pending_.front().second).count();
        if (age > timeout_) {
          fire(lk, "no device progress for " + std::to_string(age) + " s (" + std::to_string(pending_.size()) +
                       " step(s) outstanding; a peer rank is probably not entering a collective)");
          return;
        }
      }
      if (host_armed_) {
        const double idle = std::chrono::duration<double>(now - last_beat_).count();
        if (idle > timeout_) {
          fire(lk, "no host heartbeat for " + std::to_string(idle) + " s");
          return;
        }
      }
      if (comm_) {
        std::string err = comm_->async_error();
        if (!err.empty() && err != "destroyed") {
          fire(lk, "communicator asynchronous error: " + err);
          return;
        }
      }
    }
  }

  void fire(std::unique_lock<std::mutex>& lk, const std::string& why) {
    fired_ = true;
    reason_ = why;
    const int rank = comm_ ? comm_->rank() : -1;
    lk.unlock();
    std::fprintf(stderr, "[dpa watchdog] rank %d (%s): %s; timeout %.1f s -> aborting the communicator\n", rank,
                 tag_.c_str(), why.c_str(), timeout_);
    std::fflush(stderr);
    if (comm_) comm_->abort_now();
    // after the abort (spinning exchanges give up, the device drains): where the in-kernel
    // exchanges stood, and what the host last queued -- one line the supervisor records
    const std::string st = comm_ ? comm_->debug_state() : std::string();
    std::string last;
    {
      std::lock_guard<std::mutex> g(mu_);
      last = note_;
    }
    std::fprintf(stderr, "[dpa watchdog] rank %d (%s): %s; last: %s%s%s\n", rank, tag_.c_str(), why.c_str(),
                 last.empty() ? "(no step noted)" : last.c_str(), st.empty() ? "" : "; ", st.c_str());
    std::fflush(stderr);
    if (do_exit_) std::_Exit(exit_code_);
    lk.lock();
  }

  const double timeout_, poll_;
  std::shared_ptr<Collective> comm_;
  const int exit_code_;
  const std::string tag_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread thread_;
  std::deque<std::pair<hipEvent_t, Clock::time_point>> pending_;
  std::vector<hipEvent_t> free_;
  Clock::time_point last_beat_;
  bool host_armed_ = false;
  bool stopping_ = false;
  std::atomic<bool> fired_{false};
  std::atomic<bool> do_exit_{true};
  std::atomic<int64_t> ticks_{0};
  std::string reason_;
  std::string note_;
};

}  // namespace rt

void register_runtime(pybind11::module& m) {
  namespace py = pybind11;
  using rt::Watchdog;
  auto s = m.def_submodule("runtime", "watchdog + roctx tracing");
  py::class_<Watchdog, std::shared_ptr<Watchdog>>(s, "Watchdog")
      .def(py::init<double, std::shared_ptr<dpa::Collective>, int, std::string, double>(), py::arg("timeout"),
           py::arg("comm") = nullptr, py::arg("exit_code") = 124, py::arg("tag") = "", py::arg("poll") = 0.5)
      .def("tick", &Watchdog::tick)
      .def("heartbeat", &Watchdog::heartbeat)
      .def("disarm", &Watchdog::disarm)
      .def("stop", &Watchdog::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_exit", &Watchdog::set_exit)
      .def_property_readonly("ticks", &Watchdog::ticks)
      .def_property_readonly("outstanding", &Watchdog::outstanding)
      .def("note", &Watchdog::note)
      .def_property_readonly("fired", &Watchdog::fired)
      .def_property_readonly("reason", &Watchdog::reason);
  // roctx ranges: visible in rocprofv3 --marker-trace timelines
  s.def("range_push", [](const std::string& name) { return roctxRangePushA(name.c_str()); });
  s.def("range_pop", []() { return roctxRangePop(); });
  s.def("mark", [](const std::string& name) { roctxMarkA(name.c_str()); });
  // Upload an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) to the device on
  // the current stream without running it: the first replay of a captured step otherwise pays
  // the upload inside the timed / training loop (runtime/graph.py CapturedStep.capture)
  s.def("graph_upload", [](uintptr_t exec) {
    TORCH_CHECK(exec != 0, "graph_upload: no instantiated graph");
    DPA_CHECK_HIP(hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), c10::hip::getCurrentHIPStream().stream()));
  });
}

}  // namespace dpa
