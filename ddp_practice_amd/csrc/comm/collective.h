// Collective interface shared by the RCCL communicator and the DDP reducer.
#pragma once

#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include <memory>
#include <string>

namespace dpa {

enum class RedOp : int { SUM = 0, PROD = 1, MAX = 2, MIN = 3, AVG = 4 };

RedOp parse_op(const std::string& op);

// Minimal asynchronous collective surface the reducer needs.  "async" work is
// ordered after everything already enqueued on the caller's current stream;
// wait(slot) orders the caller's current stream after that work.
struct Collective {
  virtual ~Collective() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual void all_reduce_async(at::Tensor t, RedOp op, int slot) = 0;
  // stream == nullptr: the caller's current stream
  virtual void wait(int slot, hipStream_t stream) = 0;
  // failure handling (watchdog thread): may be called concurrently with other calls
  virtual std::string async_error() { return std::string(); }
  virtual void abort_now() {}
  // one line describing where the communicator's in-kernel exchanges stand (watchdog report,
  // after abort_now): empty when there is nothing device-side to show
  virtual std::string debug_state() { return std::string(); }
};

// Flat multi-tensor copy (csrc/kernels/optim.hip): direction 0 = pack into flat.
namespace opt {
void flat_copy(std::vector<at::Tensor> tensors, std::vector<int64_t> offsets, at::Tensor flat, double s,
               int64_t direction);
}

}  // namespace dpa
