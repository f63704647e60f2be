// Single Python module for every native component of ddp_practice_amd.
// Each translation unit exposes a register_* function; nothing here but glue.
#include <torch/extension.h>

namespace dpa {
void register_selftest(pybind11::module& m);
void register_convblock(pybind11::module& m);
void register_head(pybind11::module& m);
void register_optim(pybind11::module& m);
void register_data(pybind11::module& m);
void register_comm(pybind11::module& m);
void register_reducer(pybind11::module& m);
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "ddp_practice_amd native extension (gfx950 HIP kernels, RCCL communicator, DDP reducer)";
  dpa::register_selftest(m);
  dpa::register_convblock(m);
  dpa::register_head(m);
  dpa::register_optim(m);
  dpa::register_data(m);
  dpa::register_comm(m);
  dpa::register_reducer(m);
}
