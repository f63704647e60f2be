// Host side of the fused conv-block kernels (device code: convblock_impl.h).
#include "convblock_impl.h"

namespace dpa {
namespace cb {

// ===========================================================================
// Host side
// ===========================================================================
struct Shape {
  int cin, cout, h, w;
  bool operator==(const Shape& o) const {
    return cin == o.cin && cout == o.cout && h == o.h && w == o.w;
  }
};

// Compile-time instantiations (the ConvNet blocks).
static const Shape kShapes[] = {{1, 16, 28, 28}, {16, 32, 14, 14}};

template <typename F>
static bool with_shape(const Shape& s, F&& f) {
  if (s == kShapes[0]) { f(std::integral_constant<int, 0>{}); return true; }
  if (s == kShapes[1]) { f(std::integral_constant<int, 1>{}); return true; }
  return false;
}
// The per-channel kernels only depend on (C, H, W).
template <typename F>
static bool with_chw(int C, int H, int W, F&& f) {
  if (C == 16 && H == 28 && W == 28) { f(std::integral_constant<int, 0>{}); return true; }
  if (C == 32 && H == 14 && W == 14) { f(std::integral_constant<int, 1>{}); return true; }
  return false;
}

template <typename F>
static void with_t(DT dt, F&& f) {
  switch (dt) {
    case DT::F32: f(float{}); break;
    case DT::BF16: f(__hip_bfloat16{}); break;
    case DT::F16: f(__half{}); break;
  }
}

bool supported(int cin, int cout, int h, int w) {
  return with_shape(Shape{cin, cout, h, w}, [](auto) {});
}

// number of conv-forward workgroups (= rows of the forward stats slab)
int64_t fwd_rows(int cin, int cout, int h, int w, int64_t B) {
  int64_t r = -1;
  with_shape(Shape{cin, cout, h, w}, [&](auto I) { r = B * SH<decltype(I)::value>::SPLIT; });
  TORCH_CHECK(r >= 0, "conv block shape not instantiated");
  return r;
}
// number of wgrad workgroups (= rows of the wgrad slab)
int64_t wgrad_rows(int cin, int cout, int h, int w, int64_t B) {
  int64_t r = -1;
  with_shape(Shape{cin, cout, h, w}, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    r = B * ((S::H + S::WROWS - 1) / S::WROWS);
  });
  TORCH_CHECK(r >= 0, "conv block shape not instantiated");
  return r;
}
int64_t bwd_split(int64_t B) { return B >= kBwdSplit ? kBwdSplit : std::max<int64_t>(B, 1); }

// Forward conv (+bias) [+ BN partial sums into fslab, shift copy into fstats].
void conv_fwd(at::Tensor x, at::Tensor w, at::Tensor bias, at::Tensor y, c10::optional<at::Tensor> fslab,
              c10::optional<at::Tensor> fstats, c10::optional<at::Tensor> shift) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(bias); DPA_CHECK_INPUT(y);
  TORCH_CHECK(w.scalar_type() == at::kFloat && bias.scalar_type() == at::kFloat);
  TORCH_CHECK(y.scalar_type() == x.scalar_type());
  const Shape s{(int)x.size(1), (int)w.size(0), (int)x.size(2), (int)x.size(3)};
  TORCH_CHECK(w.size(1) == s.cin && w.size(2) == 5 && w.size(3) == 5, "weight must be [COUT][CIN][5][5]");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == s.cout && y.size(2) == s.h && y.size(3) == s.w);
  const int B = (int)x.size(0);
  const bool st = fslab.has_value();
  if (st) {
    DPA_CHECK_INPUT((*fslab)); DPA_CHECK_INPUT((*fstats)); DPA_CHECK_INPUT((*shift));
    TORCH_CHECK(fstats->numel() == stats_len(s.cout) && shift->numel() == s.cout);
    TORCH_CHECK(fslab->numel() == fwd_rows(s.cin, s.cout, s.h, s.w, B) * fslab_row(s.cout), "fslab size");
  }
  if (B == 0) return;
  hipStream_t stream = cur_stream();
  const bool ok = with_shape(s, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    const dim3 grid(B * S::SPLIT), blk(NTHR);
    with_t(dt_of(x), [&](auto tag) {
      typedef decltype(tag) T;
      if (st)
        hipLaunchKernelGGL((conv5x5_kernel<T, S::CIN, S::COUT, S::H, S::W, 0>), grid, blk, 0, stream, dptr<T>(x),
                           w.data_ptr<float>(), bias.data_ptr<float>(), dptr<T>(y), fslab->data_ptr<float>(),
                           fstats->data_ptr<float>(), shift->data_ptr<float>(), S::SPLIT);
      else
        hipLaunchKernelGGL((conv5x5_kernel<T, S::CIN, S::COUT, S::H, S::W, 1>), grid, blk, 0, stream, dptr<T>(x),
                           w.data_ptr<float>(), bias.data_ptr<float>(), dptr<T>(y), nullptr, nullptr, nullptr,
                           S::SPLIT);
    });
  });
  TORCH_CHECK(ok, "conv block shape not instantiated");
  DPA_CHECK_LAUNCH();
}

// Data gradient: dx[B][CIN][H][W] from dy[B][COUT][H][W] and w[COUT][CIN][5][5].
void conv_dgrad(at::Tensor dy, at::Tensor w, at::Tensor dx) {
  DPA_CHECK_INPUT(dy); DPA_CHECK_INPUT(w); DPA_CHECK_INPUT(dx);
  const int cout = (int)w.size(0), cin = (int)w.size(1);
  const int H = (int)dy.size(2), W = (int)dy.size(3);
  TORCH_CHECK(dy.size(1) == cout && dx.size(1) == cin && dx.scalar_type() == dy.scalar_type());
  const int B = (int)dy.size(0);
  TORCH_CHECK(cin == 16 && cout == 32 && H == 14 && W == 14, "dgrad shape not instantiated: ", cout, "->", cin, " ",
              H, "x", W);
  if (B == 0) return;
  constexpr int ns = 2;
  hipStream_t stream = cur_stream();
  with_t(dt_of(dy), [&](auto tag) {
    typedef decltype(tag) T;
    hipLaunchKernelGGL((conv5x5_kernel<T, 32, 16, 14, 14, 2>), dim3(B * ns), dim3(NTHR), 0, stream, dptr<T>(dy),
                       w.data_ptr<float>(), nullptr, dptr<T>(dx), nullptr, nullptr, nullptr, ns);
  });
  DPA_CHECK_LAUNCH();
}

void bn_relu_pool(at::Tensor y, c10::optional<at::Tensor> fslab, at::Tensor fstats, at::Tensor gamma, at::Tensor beta,
                  at::Tensor rmean, at::Tensor rvar, at::Tensor nbt, double momentum, double eps, bool train,
                  at::Tensor p, at::Tensor idx) {
  DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(p); DPA_CHECK_INPUT(idx);
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  TORCH_CHECK(idx.scalar_type() == at::kByte && p.scalar_type() == y.scalar_type());
  TORCH_CHECK(nbt.scalar_type() == at::kLong);
  TORCH_CHECK(!train || fslab.has_value(), "train mode needs the forward slab");
  const int total = B * C * (H / 2) * (W / 2);
  const int nrows = fslab.has_value() ? (int)(fslab->numel() / fslab_row(C)) : 0;
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (total == 0) return;
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bn_relu_pool_kernel<T, S::COUT, S::H, S::W>), dim3((total + NTHR - 1) / NTHR), dim3(NTHR),
                         0, stream, dptr<T>(y), fslab.has_value() ? fslab->data_ptr<float>() : nullptr, nrows,
                         fstats.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                         rmean.data_ptr<float>(), rvar.data_ptr<float>(), nbt.data_ptr<int64_t>(), (float)momentum,
                         (float)eps, (int)train, dptr<T>(p), idx.data_ptr<uint8_t>(), total);
    });
  });
  TORCH_CHECK(ok, "bn_relu_pool shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void bwd_reduce(at::Tensor dp, at::Tensor p, at::Tensor idx, at::Tensor y, at::Tensor fstats, double eps,
                at::Tensor bslab) {
  DPA_CHECK_INPUT(dp); DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(bslab);
  TORCH_CHECK(dp.scalar_type() == y.scalar_type() && p.scalar_type() == y.scalar_type());
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  const int nsplit = (int)bwd_split(B);
  TORCH_CHECK(bslab.numel() == (int64_t)nsplit * 2 * C, "bslab size");
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (B == 0) { bslab.zero_(); return; }
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bwd_reduce_kernel<T, S::COUT, S::H, S::W>), dim3(C, nsplit), dim3(NTHR), 0, stream,
                         dptr<T>(dp), dptr<T>(p), idx.data_ptr<uint8_t>(), dptr<T>(y), fstats.data_ptr<float>(),
                         (float)eps, bslab.data_ptr<float>(), B);
    });
  });
  TORCH_CHECK(ok, "bwd_reduce shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void bwd_elemt(at::Tensor dp, at::Tensor p, at::Tensor idx, at::Tensor y, at::Tensor fstats, at::Tensor gslab,
               at::Tensor gamma, double eps, at::Tensor dx) {
  DPA_CHECK_INPUT(dp); DPA_CHECK_INPUT(y); DPA_CHECK_INPUT(dx); DPA_CHECK_INPUT(gslab);
  const int B = (int)y.size(0), C = (int)y.size(1), H = (int)y.size(2), W = (int)y.size(3);
  const int total = B * C * (H / 2) * (W / 2);
  const int nsplit = (int)(gslab.numel() / (2 * C));
  hipStream_t stream = cur_stream();
  const bool ok = with_chw(C, H, W, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (total == 0) return;
    with_t(dt_of(y), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((bwd_elemt_kernel<T, S::COUT, S::H, S::W>), dim3((total + NTHR - 1) / NTHR), dim3(NTHR), 0,
                         stream, dptr<T>(dp), dptr<T>(p), idx.data_ptr<uint8_t>(), dptr<T>(y), fstats.data_ptr<float>(),
                         gslab.data_ptr<float>(), nsplit, gamma.data_ptr<float>(), (float)eps, dptr<T>(dx), total);
    });
  });
  TORCH_CHECK(ok, "bwd_elemt shape not instantiated");
  DPA_CHECK_LAUNCH();
}

void conv_wgrad(at::Tensor x, at::Tensor dy, at::Tensor wslab) {
  DPA_CHECK_INPUT(x); DPA_CHECK_INPUT(dy); DPA_CHECK_INPUT(wslab);
  TORCH_CHECK(wslab.scalar_type() == at::kFloat);
  const int B = (int)x.size(0);
  const Shape s{(int)x.size(1), (int)dy.size(1), (int)x.size(2), (int)x.size(3)};
  TORCH_CHECK(wslab.numel() == wgrad_rows(s.cin, s.cout, s.h, s.w, B) * (s.cout * s.cin * 25 + s.cout),
              "wslab size");
  hipStream_t stream = cur_stream();
  const bool ok = with_shape(s, [&](auto I) {
    typedef SH<decltype(I)::value> S;
    if (B == 0) return;
    constexpr int ns = (S::H + S::WROWS - 1) / S::WROWS;
    with_t(dt_of(x), [&](auto tag) {
      typedef decltype(tag) T;
      hipLaunchKernelGGL((conv5x5_wgrad_kernel<T, S::CIN, S::COUT, S::H, S::W, S::WROWS>), dim3(B * ns), dim3(NTHR),
                         0, stream, dptr<T>(x), dptr<T>(dy), wslab.data_ptr<float>(), ns);
    });
  });
  TORCH_CHECK(ok, "wgrad shape not instantiated");
  DPA_CHECK_LAUNCH();
}

// out1 = column sums of slab1 [rows1][n1]; out2 = column sums of slab2 [rows2][n2]
void slab_reduce(at::Tensor slab1, int64_t n1, at::Tensor out1, c10::optional<at::Tensor> slab2, int64_t n2,
                 c10::optional<at::Tensor> out2) {
  DPA_CHECK_INPUT(slab1); DPA_CHECK_INPUT(out1);
  TORCH_CHECK(slab1.numel() % n1 == 0 && out1.numel() == n1);
  const int rows1 = (int)(slab1.numel() / n1);
  int rows2 = 0;
  if (slab2.has_value()) {
    DPA_CHECK_INPUT((*slab2)); DPA_CHECK_INPUT((*out2));
    TORCH_CHECK(slab2->numel() % n2 == 0 && out2->numel() == n2);
    rows2 = (int)(slab2->numel() / n2);
  } else {
    n2 = 0;
  }
  const int64_t nblk = (n1 + SR_COLS - 1) / SR_COLS + (n2 + SR_COLS - 1) / SR_COLS;
  if (nblk == 0) return;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(nblk), dim3(NTHR), 0, cur_stream(),
                     slab1.data_ptr<float>(), rows1, (int)n1, out1.data_ptr<float>(),
                     slab2.has_value() ? slab2->data_ptr<float>() : nullptr, rows2, (int)n2,
                     out2.has_value() ? out2->data_ptr<float>() : nullptr);
  DPA_CHECK_LAUNCH();
}

}  // namespace cb

void register_convblock(pybind11::module& m) {
  namespace py = pybind11;
  auto s = m.def_submodule("convblock", "fused Conv5x5-BN-ReLU-MaxPool block kernels");
  s.def("supported", &cb::supported);
  s.def("stats_len", [](int C) { return cb::stats_len(C); });
  s.def("fslab_row", [](int C) { return cb::fslab_row(C); });
  s.def("fwd_rows", &cb::fwd_rows);
  s.def("wgrad_rows", &cb::wgrad_rows);
  s.def("bwd_split", &cb::bwd_split);
  s.def("conv_fwd", &cb::conv_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"),
        py::arg("fslab") = py::none(), py::arg("fstats") = py::none(), py::arg("shift") = py::none());
  s.def("conv_dgrad", &cb::conv_dgrad);
  s.def("conv_wgrad", &cb::conv_wgrad);
  s.def("bn_relu_pool", &cb::bn_relu_pool);
  s.def("bwd_reduce", &cb::bwd_reduce);
  s.def("bwd_elemt", &cb::bwd_elemt);
  s.def("slab_reduce", &cb::slab_reduce, py::arg("slab1"), py::arg("n1"), py::arg("out1"),
        py::arg("slab2") = py::none(), py::arg("n2") = 0, py::arg("out2") = py::none());
}

}  // namespace dpa
