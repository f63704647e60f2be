// DDP gradient reducer: buckets, autograd post-hooks, in-order async
// all-reduce overlapped with the rest of backward.
//
// Semantics of torch's C++ Reducer (torch/csrc/distributed/c10d/reducer.cpp,
// driven from torch/nn/parallel/distributed.py:1199-1248,1521-1617) re-designed
// for one process per MI355X:
//  * Buckets are flat f32/bf16/f16 device buffers; the bucket plan (reverse
//    parameter order, first bucket small, then a cap) is computed in Python and
//    re-planned after the first iteration in actual grad-ready order.
//  * A post-hook on each parameter's AccumulateGrad node marks it ready.  When
//    a bucket's last gradient arrives it is packed with ONE multi-tensor kernel
//    (grad * 1/W into the bucket) and its all-reduce is launched on the
//    communicator's stream; buckets launch strictly in index order so every
//    rank issues identical collective sequences.
//  * Zero-copy buckets: when a bucket's gradients already tile one contiguous
//    buffer (the fused ConvNet op writes all its parameter gradients into one
//    output), that buffer is all-reduced in place with AVG: no pack kernel.
//  * After the last bucket launches, the compute stream is fenced on all of
//    them and every param.grad becomes a view of its bucket (the
//    gradient_as_bucket_view=True layout: no copy-back kernel).
//  * Everything is enqueue-only (kernels, events, RCCL), so a whole DDP step
//    can be captured into a hipGraph.
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <cstdlib>
#include <mutex>

#include "comm/collective.h"
#include "common.h"

#include <c10/hip/HIPGuard.h>
#include <algorithm>

namespace dpa {
namespace ddp {

using torch::autograd::variable_list;

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
          std::shared_ptr<Collective> comm, bool find_unused)
      : params_(std::move(params)), comm_(std::move(comm)), find_unused_(find_unused) {
    TORCH_CHECK(comm_ != nullptr);
    if (const char* e = std::getenv("DPA_REDUCER_JOIN_EACH")) join_each_ = e[0] == '1';
    if (const char* e = std::getenv("DPA_REDUCER_ZERO_COPY")) zero_copy_ = e[0] != '0';
    ready_.assign(params_.size(), 0);
    set_buckets(buckets);
  }

  // (Re)bind the post-hooks to the parameters' AccumulateGrad nodes.
  //
  // An AccumulateGrad node records the stream that was current when it was
  // created, and the autograd engine syncs that "leaf stream" with the caller's
  // stream at the end of every backward.  Nodes created on the legacy default
  // stream therefore poison a hipGraph capture (an event record on the null
  // stream while another stream captures).  So the nodes are (re)created lazily
  // on the stream of the forward that will produce the backward — first
  // training forward, and again at the forward of a graph capture — after
  // dropping this reducer's strong references to the old ones.
  void refresh_hooks_locked() {
    std::weak_ptr<Reducer> self = shared_from_this();
    accs_.clear();
    for (size_t i = 0; i < params_.size(); ++i) {
      auto& p = params_[i];
      TORCH_CHECK(p.requires_grad(), "DDP parameter ", i, " does not require grad");
      auto acc = torch::autograd::impl::grad_accumulator(p);
      TORCH_CHECK(acc != nullptr, "parameter ", i, " has no grad accumulator (not a leaf?)");
      bool hooked = false;
      for (auto& w : hooked_)
        if (auto n = w.lock(); n && n.get() == acc.get()) hooked = true;
      if (!hooked) {
        acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
            [self, i](const variable_list& outputs, const variable_list&) {
              if (auto r = self.lock()) r->mark_ready(i);
              return outputs;
            }));
        hooked_.push_back(acc);
      }
      accs_.push_back(std::move(acc));
    }
    // forget expired nodes
    hooked_.erase(std::remove_if(hooked_.begin(), hooked_.end(), [](auto& w) { return w.expired(); }),
                  hooked_.end());
    hooks_ready_ = true;
  }

  void set_buckets(const std::vector<std::vector<int64_t>>& buckets) {
    std::lock_guard<std::mutex> g(mu_);
    buckets_.clear();
    param_bucket_.assign(params_.size(), -1);
    param_offset_.assign(params_.size(), 0);
    for (size_t b = 0; b < buckets.size(); ++b) {
      Bucket bk;
      int64_t off = 0;
      at::ScalarType dt = at::kFloat;
      for (size_t j = 0; j < buckets[b].size(); ++j) {
        const int64_t i = buckets[b][j];
        TORCH_CHECK(i >= 0 && i < (int64_t)params_.size(), "bad param index in bucket");
        TORCH_CHECK(param_bucket_[i] < 0, "param ", i, " in two buckets");
        if (j == 0) dt = params_[i].scalar_type();
        TORCH_CHECK(params_[i].scalar_type() == dt, "bucket mixes dtypes");
        param_bucket_[i] = (int)b;
        param_offset_[i] = off;
        bk.params.push_back(i);
        bk.offsets.push_back(off);
        // 16-byte aligned views: the grads stay valid float4 operands for the
        // vectorised optimizer kernels (the pad elements stay zero)
        const int64_t al = std::max<int64_t>(1, 16 / (int64_t)params_[i].element_size());
        off += (params_[i].numel() + al - 1) / al * al;
      }
      bk.flat = at::zeros({off}, params_[buckets[b].empty() ? 0 : buckets[b][0]].options().requires_grad(false));
      buckets_.push_back(std::move(bk));
    }
    for (size_t i = 0; i < params_.size(); ++i)
      TORCH_CHECK(param_bucket_[i] >= 0, "param ", i, " not assigned to a bucket");
    reset_locked();
  }

  // Called by DDP.forward (train mode, grad enabled) before the graph is built.
  void prepare_for_backward(bool sync) {
    std::lock_guard<std::mutex> g(mu_);
    if (expect_ && !finalized_ && any_ready_)
      TORCH_CHECK(false,
                  "DDP: the previous iteration's reduction did not finish (some parameters received no "
                  "gradient). Use find_unused_parameters=True if parameters can be unused.");
    reset_locked();
    sync_ = sync;
    expect_ = true;
    // all reducer work (pack, collective fork/join) goes to the forward's stream,
    // which is the stream the backward kernels run on (the capture stream when
    // capturing), whatever stream the AccumulateGrad hooks happen to run under
    on_cuda_ = !params_.empty() && params_[0].is_cuda();
    if (on_cuda_) {
      device_ = params_[0].get_device();
      work_stream_ = cur_stream();
    }
    bool capturing = false;
    if (on_cuda_) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      DPA_CHECK_HIP(hipStreamIsCapturing(work_stream_, &st));
      capturing = st == hipStreamCaptureStatusActive;
    }
    if (!hooks_ready_ || capturing) refresh_hooks_locked();
  }

  void mark_ready(size_t i) {
    std::lock_guard<std::mutex> g(mu_);
    if (!expect_ || !sync_) return;  // no_sync() or backward outside a DDP forward
    if (ready_[i]) return;           // reentrant backward hits the same hook twice: ignore
    if (!any_ready_) {
      any_ready_ = true;
      if (find_unused_) {
        // params that never get a grad must still be reduced: finalize at the end
        // of this backward (engine final callback)
        std::weak_ptr<Reducer> self = shared_from_this();
        torch::autograd::Engine::get_default_engine().queue_callback([self]() {
          if (auto r = self.lock()) r->finalize();
        });
      }
    }
    ready_[i] = 1;
    ++n_ready_;
    if (record_order_) order_.push_back((int64_t)i);
    Bucket& bk = buckets_[param_bucket_[i]];
    bk.pending -= 1;
    launch_ready_locked();
    // every parameter reported: finalize right here, on the backward's stream
    if (!find_unused_ && n_ready_ == params_.size()) finalize_locked();
  }

  void finalize() {
    std::lock_guard<std::mutex> g(mu_);
    finalize_locked();
  }

  void finalize_locked() {
    if (!expect_ || finalized_) return;
    c10::optional<c10::hip::HIPStreamGuard> guard;
    bind_stream(guard);
    if (find_unused_) {
      for (size_t i = 0; i < params_.size(); ++i) {
        if (!ready_[i]) {
          ready_[i] = 1;
          Bucket& bk = buckets_[param_bucket_[i]];
          bk.unused.push_back(i);
          bk.pending -= 1;
        }
      }
      launch_ready_locked();
    }
    for (auto& bk : buckets_)
      TORCH_CHECK(bk.launched, "DDP: bucket not reduced at end of backward (unused parameters? set "
                               "find_unused_parameters=True)");
    // join on the stream the buckets were launched from (the backward's stream,
    // i.e. the capture stream under hipGraph capture) — not whatever stream is
    // current on the thread that runs the engine's final callback
    if (defer_)
      deferred_ = true;  // the buckets hold this rank's gradients until flush_deferred() / a fused consumer
    else
      for (size_t b = 0; b < buckets_.size(); ++b) comm_->wait((int)b, on_cuda_ ? work_stream_ : nullptr);
    // grads become views of the all-reduced buckets (in-place buckets: they already are);
    // gradient_as_bucket_view=False: the averaged values are copied back into the gradient
    // tensors autograd produced (their identity and storage are kept, torch's default layout)
    for (auto& bk : buckets_) {
      if (bk.inplace) continue;
      for (size_t j = 0; j < bk.params.size(); ++j) {
        auto& p = params_[bk.params[j]];
        at::Tensor view = bk.flat.narrow(0, bk.offsets[j], p.numel()).view(p.sizes());
        if (grad_as_view_) {
          p.mutable_grad() = view;
        } else if (p.grad().defined() && p.grad().sizes() == p.sizes()) {
          p.mutable_grad().copy_(view);
        } else {
          p.mutable_grad() = view.clone();  // an unused parameter: the reduced (zero) gradient
        }
      }
    }
    finalized_ = true;
    record_order_ = false;
  }

  // Deferred gradient averaging (DistributedDataParallel.defer_grad_sync_to):
  // buckets are not all-reduced at the end of backward; the gradient consumer
  // either averages them itself (the fused AMP-SGD kernel over the xGMI engine:
  // consume_deferred()) or calls flush_deferred(), which runs the bucket
  // all-reduces now, on the caller's stream, and joins them.
  void set_defer(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(!(defer_ && !on && deferred_), "DDP: gradients still pending a deferred all-reduce");
    defer_ = on;
    if (!on) require_inplace_ = false;  // only the deferred slab sink needs in-place buckets
  }
  bool deferred_pending() const { return deferred_; }
  void set_grad_as_view(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(on || !defer_, "DDP: gradient_as_bucket_view=False with deferred gradient averaging");
    grad_as_view_ = on;
  }
  void set_require_inplace(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    require_inplace_ = on;
  }
  void consume_deferred() {
    std::lock_guard<std::mutex> g(mu_);
    deferred_ = false;
  }
  void flush_deferred() {
    std::lock_guard<std::mutex> g(mu_);
    if (!deferred_) return;
    for (size_t b = 0; b < buckets_.size(); ++b)
      comm_->all_reduce_async(buckets_[b].red, RedOp::AVG, (int)b);
    for (size_t b = 0; b < buckets_.size(); ++b) comm_->wait((int)b, nullptr);
    deferred_ = false;
  }

  std::vector<int64_t> ready_order() const { return order_; }
  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  std::vector<at::Tensor> bucket_tensors() const {
    std::vector<at::Tensor> v;
    for (auto& b : buckets_) v.push_back(b.flat);
    return v;
  }
  std::vector<std::vector<int64_t>> bucket_indices() const {
    std::vector<std::vector<int64_t>> v;
    for (auto& b : buckets_) v.push_back(b.params);
    return v;
  }
  void set_record_order(bool on) {
    record_order_ = on;
    if (on) order_.clear();
  }

 private:
  struct Bucket {
    std::vector<int64_t> params, offsets;
    std::vector<int64_t> unused;
    at::Tensor flat;
    at::Tensor red;  // what the all-reduce covers: the in-place gradient region or flat
    int64_t pending = 0;
    bool launched = false;
    bool inplace = false;  // reduced where the grads live (no pack)
  };

  // Zero-copy bucket: when every gradient of the bucket is a contiguous view and
  // together they tile one contiguous region of one storage exactly (the fused
  // ConvNet op hands autograd views of ONE gradient buffer), that region is
  // all-reduced in place with AVG -- no pack kernel, no 1/W pass, grads stay put.
  bool tiled_region_locked(const Bucket& bk, at::Tensor& region) {
    if (!bk.unused.empty() || bk.params.empty()) return false;
    std::vector<std::pair<int64_t, int64_t>> spans;
    const at::Tensor g0 = params_[bk.params[0]].grad();
    if (!g0.defined() || !g0.is_cuda() || g0.scalar_type() != bk.flat.scalar_type()) return false;
    for (int64_t i : bk.params) {
      const at::Tensor g = params_[i].grad();
      if (!g.defined() || !g.is_contiguous() || g.scalar_type() != g0.scalar_type() ||
          !g.storage().is_alias_of(g0.storage()) || g.numel() != params_[i].numel())
        return false;
      spans.emplace_back(g.storage_offset(), g.numel());
    }
    std::sort(spans.begin(), spans.end());
    for (size_t k = 1; k < spans.size(); ++k)
      if (spans[k].first != spans[k - 1].first + spans[k - 1].second) return false;
    const int64_t lo = spans.front().first, n = spans.back().first + spans.back().second - lo;
    region = at::empty({0}, g0.options()).set_(g0.storage(), lo, {n}, {1});
    return true;
  }

  void reset_locked() {
    std::fill(ready_.begin(), ready_.end(), 0);
    for (auto& bk : buckets_) {
      bk.pending = (int64_t)bk.params.size();
      bk.launched = false;
      bk.inplace = false;
      bk.unused.clear();
    }
    next_launch_ = 0;
    n_ready_ = 0;
    any_ready_ = false;
    finalized_ = false;
    expect_ = false;
  }

  // launch every complete bucket whose predecessors have launched
  void bind_stream(c10::optional<c10::hip::HIPStreamGuard>& g) {
    if (on_cuda_ && work_stream_ != nullptr)
      g.emplace(c10::hip::getStreamFromExternal(work_stream_, (c10::DeviceIndex)device_));
  }

  void launch_ready_locked() {
    c10::optional<c10::hip::HIPStreamGuard> guard;
    bind_stream(guard);
    while (next_launch_ < buckets_.size() && buckets_[next_launch_].pending == 0) {
      Bucket& bk = buckets_[next_launch_];
      at::Tensor region;
      if (zero_copy_ && tiled_region_locked(bk, region)) {
        bk.red = region;
        if (!defer_) {
          comm_->all_reduce_async(region, RedOp::AVG, (int)next_launch_);
          if (join_each_) comm_->wait((int)next_launch_, nullptr);
        }
        bk.inplace = bk.launched = true;
        ++next_launch_;
        continue;
      }
      bk.inplace = false;
      // a gradient still held as a producer's partial rows (a deferred slab, summed inside
      // the fused optimizer launch) has no values yet: only the in-place bucket is valid then
      TORCH_CHECK(!require_inplace_, "DDP: the deferred weight-gradient slab needs the zero-copy bucket "
                                     "(every gradient of a bucket a view of one buffer, tiling it)");
      std::vector<at::Tensor> srcs;
      std::vector<int64_t> offs;
      const double inv_w = defer_ ? 1.0 : 1.0 / (double)comm_->world();  // deferred: averaged by the consumer
      for (size_t j = 0; j < bk.params.size(); ++j) {
        const int64_t i = bk.params[j];
        at::Tensor gr = params_[i].grad();
        const bool unused = std::find(bk.unused.begin(), bk.unused.end(), i) != bk.unused.end();
        if (unused || !gr.defined()) {
          bk.flat.narrow(0, bk.offsets[j], params_[i].numel()).zero_();
          continue;
        }
        TORCH_CHECK(gr.numel() == params_[i].numel());
        srcs.push_back(gr.is_contiguous() ? gr.view({-1}) : gr.contiguous().view({-1}));
        offs.push_back(bk.offsets[j]);
      }
      if (!srcs.empty()) {
        if (bk.flat.is_cuda() && bk.flat.scalar_type() == at::kFloat) {
          opt::flat_copy(srcs, offs, bk.flat, inv_w, 0);
        } else {
          for (size_t k = 0; k < srcs.size(); ++k)
            bk.flat.narrow(0, offs[k], srcs[k].numel()).copy_(srcs[k]).mul_(inv_w);
        }
      }
      bk.red = bk.flat;
      if (!defer_) {
        comm_->all_reduce_async(bk.flat, RedOp::SUM, (int)next_launch_);
        if (join_each_) comm_->wait((int)next_launch_, nullptr);
      }
      bk.launched = true;
      ++next_launch_;
    }
  }

  std::vector<at::Tensor> params_;
  std::vector<std::shared_ptr<torch::autograd::Node>> accs_;
  std::shared_ptr<Collective> comm_;
  bool find_unused_;
  std::vector<Bucket> buckets_;
  std::vector<int> param_bucket_;
  std::vector<int64_t> param_offset_;
  std::vector<char> ready_;
  size_t next_launch_ = 0;
  size_t n_ready_ = 0;
  bool any_ready_ = false, finalized_ = false, expect_ = false, sync_ = true;
  bool record_order_ = true;
  hipStream_t work_stream_ = nullptr;
  int device_ = 0;
  bool on_cuda_ = false;
  bool hooks_ready_ = false;
  std::vector<std::weak_ptr<torch::autograd::Node>> hooked_;
  bool defer_ = false, deferred_ = false;  // see set_defer
  bool require_inplace_ = false;           // see set_require_inplace (DDP.set_slab_sink)
  bool join_each_ = false;  // join every bucket immediately (no overlap)
  bool grad_as_view_ = true;  // param.grad = views of the buckets (gradient_as_bucket_view)
  bool zero_copy_ = true;   // reduce tiled gradient regions in place (DPA_REDUCER_ZERO_COPY=0: always pack)
  std::vector<int64_t> order_;
  std::mutex mu_;
};

}  // namespace ddp

void register_reducer(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("ddp", "DDP gradient reducer");
  py::class_<ddp::Reducer, std::shared_ptr<ddp::Reducer>>(s, "Reducer")
      .def(py::init([](std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
                       std::shared_ptr<Collective> comm, bool find_unused) {
             return std::make_shared<ddp::Reducer>(std::move(params), std::move(buckets), std::move(comm),
                                                   find_unused);
           }),
           py::arg("params"), py::arg("buckets"), py::arg("comm"), py::arg("find_unused") = false)
      .def("prepare_for_backward", &ddp::Reducer::prepare_for_backward, py::arg("sync") = true)
      .def("finalize", &ddp::Reducer::finalize)
      .def("set_buckets", &ddp::Reducer::set_buckets)
      .def("ready_order", &ddp::Reducer::ready_order)
      .def("num_buckets", &ddp::Reducer::num_buckets)
      .def("bucket_tensors", &ddp::Reducer::bucket_tensors)
      .def("bucket_indices", &ddp::Reducer::bucket_indices)
      .def("set_record_order", &ddp::Reducer::set_record_order)
      .def("set_defer", &ddp::Reducer::set_defer)
      .def("deferred_pending", &ddp::Reducer::deferred_pending)
      .def("set_require_inplace", &ddp::Reducer::set_require_inplace)
      .def("set_grad_as_view", &ddp::Reducer::set_grad_as_view)
      .def("consume_deferred", &ddp::Reducer::consume_deferred)
      .def("flush_deferred", &ddp::Reducer::flush_deferred);
}

}  // namespace dpa
