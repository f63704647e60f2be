// MFMA fragment-map self test: D[16x16] = A[16x32] * B[32x16] on one wave with
// v_mfma_f32_16x16x32_bf16 and, for f32 inputs, 8 chained v_mfma_f32_16x16x4_f32.
// Used by tests/test_kernels_gpu.py to pin the lane maps common.h documents.
#include "common.h"

#include <chrono>

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

__global__ void noop_kernel(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}

// Launch-floor microbenchmark: n dependent no-op launches on the current
// stream, either eagerly or captured once into a hipGraph and replayed `reps`
// times.  Returns microseconds per kernel (host wall clock, stream-synced).
double launch_floor(at::Tensor buf, int64_t n, int64_t reps, bool graph, int64_t blocks) {
  hipStream_t s = cur_stream();
  float* p = buf.data_ptr<float>();
  DPA_CHECK_HIP(hipStreamSynchronize(s));
  if (!graph) {
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int64_t r = 0; r < reps; ++r)
      for (int64_t i = 0; i < n; ++i) hipLaunchKernelGGL(noop_kernel, dim3(blocks), dim3(64), 0, s, p);
    DPA_CHECK_HIP(hipStreamSynchronize(s));
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / (double)(n * reps);
  }
  hipStream_t cs;
  DPA_CHECK_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  DPA_CHECK_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  for (int64_t i = 0; i < n; ++i) hipLaunchKernelGGL(noop_kernel, dim3(blocks), dim3(64), 0, cs, p);
  DPA_CHECK_HIP(hipStreamEndCapture(cs, &g));
  DPA_CHECK_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  DPA_CHECK_HIP(hipGraphLaunch(ge, cs));
  DPA_CHECK_HIP(hipStreamSynchronize(cs));
  auto t0 = std::chrono::high_resolution_clock::now();
  for (int64_t r = 0; r < reps; ++r) DPA_CHECK_HIP(hipGraphLaunch(ge, cs));
  DPA_CHECK_HIP(hipStreamSynchronize(cs));
  auto t1 = std::chrono::high_resolution_clock::now();
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  hipStreamDestroy(cs);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / (double)(n * reps);
}

// Workgroup start probe: per workgroup [start s_memrealtime, XCC id, end], so the
// dispatch order / per-XCD start offsets of a launch can be measured.  `spin`
// (100 MHz ticks) keeps every workgroup alive for a while (one wave per workgroup).
__global__ void __launch_bounds__(64) xcd_probe_kernel(long long* out, long long spin) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  // HW_REG_XCC_ID (hwreg 20), bits [3:0]
  const int xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
  long long t = t0;
  while (t - t0 < spin) t = (long long)__builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = t0;
    out[3 * blockIdx.x + 1] = xcc;
    out[3 * blockIdx.x + 2] = t;
  }
}

void xcd_probe(at::Tensor out, int64_t blocks, int64_t spin) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.numel() >= 3 * blocks, "xcd_probe: out");
  hipLaunchKernelGGL(xcd_probe_kernel, dim3((unsigned)blocks), dim3(64), 0, cur_stream(),
                     reinterpret_cast<long long*>(out.data_ptr<int64_t>()), (long long)spin);
  DPA_CHECK_LAUNCH();
}

void register_selftest(pybind11::module& m) {
  m.def("xcd_probe", &xcd_probe, "per-workgroup start time / XCC id of one launch");
  m.def("launch_floor", &launch_floor, "us per dependent no-op kernel (eager or hipGraph)");
  m.def("mfma_selftest", &mfma_selftest, "16x16x32 bf16 and 16x16x4 f32 MFMA lane-map test");
}

}  // namespace dpa
