// Single Python module for every native component of ddp_practice_amd.
// Each translation unit exposes a register_* function; nothing here but glue.
#include <torch/extension.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>

namespace dpa {
void register_selftest(pybind11::module& m);
void register_convblock(pybind11::module& m);
void register_head(pybind11::module& m);
void register_optim(pybind11::module& m);
void register_data(pybind11::module& m);
void register_comm(pybind11::module& m);
void register_xgmi(pybind11::module& m);
void register_reducer(pybind11::module& m);
void register_convnet_fused(pybind11::module& m);
void register_convnet_head(pybind11::module& m);
void register_runtime(pybind11::module& m);
void register_bn_nhwc(pybind11::module& m);
void register_conv_igemm(pybind11::module& m);
}

// sha1 of the sources this library was built from (build.py generates it; _ext.py compares
// it with the tree on import so a stale binary cannot pass for the current kernels)
extern "C" const char dpa_source_digest[];

// Opt-in (DPA_NATIVE_BACKTRACE=1) host-side SIGSEGV handler printing the native
// stack: diagnostics for crashes inside the HIP runtime / RCCL / torch.
static void dpa_segv_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\n[ddp_practice_amd] native backtrace:\n";
  ssize_t w = write(2, msg, sizeof(msg) - 1);
  (void)w;
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

PYBIND11_MODULE(_C, m) {
  if (const char* e = std::getenv("DPA_NATIVE_BACKTRACE"); e && e[0] == '1') {
    signal(SIGSEGV, dpa_segv_handler);
    signal(SIGABRT, dpa_segv_handler);
  }
  m.doc() = "ddp_practice_amd native extension (gfx950 HIP kernels, RCCL communicator, DDP reducer)";
  m.attr("source_digest") = pybind11::str(dpa_source_digest);
  dpa::register_selftest(m);
  dpa::register_convblock(m);
  dpa::register_head(m);
  dpa::register_optim(m);
  dpa::register_data(m);
  dpa::register_comm(m);
  dpa::register_xgmi(m);
  dpa::register_reducer(m);
  dpa::register_convnet_fused(m);
  dpa::register_convnet_head(m);
  dpa::register_runtime(m);
  dpa::register_bn_nhwc(m);
  dpa::register_conv_igemm(m);
}
