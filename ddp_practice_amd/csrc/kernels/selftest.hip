// MFMA fragment-map self test: D[16x16] = A[16x32] * B[32x16] on one wave with
// v_mfma_f32_16x16x32_bf16 and, for f32 inputs, 8 chained v_mfma_f32_16x16x4_f32.
// Used by tests/test_kernels_gpu.py to pin the lane maps common.h documents.
#include "common.h"

namespace dpa {

__global__ void __launch_bounds__(64) mfma_selftest_kernel(const float* __restrict__ A,
                                                           const float* __restrict__ B,
                                                           float* __restrict__ Dbf,
                                                           float* __restrict__ Df32) {
  const int l = threadIdx.x;
  const int r = l & 15, q = l >> 4;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[r * 32 + 8 * q + j];
    b[j] = (__bf16)B[(8 * q + j) * 16 + r];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    acc2 = mfma_f32_16x16x4(A[r * 32 + 4 * ks + q], B[(4 * ks + q) * 16 + r], acc2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Dbf[(4 * q + i) * 16 + r] = acc[i];
    Df32[(4 * q + i) * 16 + r] = acc2[i];
  }
}

std::vector<at::Tensor> mfma_selftest(at::Tensor A, at::Tensor B) {
  DPA_CHECK_INPUT(A);
  DPA_CHECK_INPUT(B);
  TORCH_CHECK(A.scalar_type() == at::kFloat && A.numel() == 16 * 32 && B.numel() == 32 * 16);
  auto Dbf = at::empty({16, 16}, A.options());
  auto Df = at::empty({16, 16}, A.options());
  hipLaunchKernelGGL(mfma_selftest_kernel, dim3(1), dim3(64), 0, cur_stream(), A.data_ptr<float>(),
                     B.data_ptr<float>(), Dbf.data_ptr<float>(), Df.data_ptr<float>());
  DPA_CHECK_LAUNCH();
  return {Dbf, Df};
}

void register_selftest(pybind11::module& m) {
  m.def("mfma_selftest", &mfma_selftest, "16x16x32 bf16 and 16x16x4 f32 MFMA lane-map test");
}

}  // namespace dpa
