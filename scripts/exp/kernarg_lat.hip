// Kernel-argument load latency on MI355X: each workgroup records s_memrealtime as its first
// instruction and again once its first kernel argument (a pointer) has arrived, plus the
// launch-to-launch gap; eager launches and a captured hipGraph.  Run with and without
// HIP_FORCE_DEV_KERNARG=1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned long long* out, const float* a, float* b) {
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  unsigned long long* o = out;  // first kernarg use
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "s"(o));
  if (threadIdx.x == 0) {
    o[blockIdx.x * 2] = t0;
    o[blockIdx.x * 2 + 1] = t1;
  }
  if (threadIdx.x == 1 && a[blockIdx.x] < -1e30f) b[blockIdx.x] = 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static void report(const char* what, std::vector<unsigned long long>& h, int grid) {
  std::vector<double> st(grid), ka(grid);
  unsigned long long t0 = ~0ull;
  for (int i = 0; i < grid; ++i) t0 = std::min(t0, h[2 * i]);
  for (int i = 0; i < grid; ++i) { st[i] = (h[2 * i] - t0) / 100.0; ka[i] = (h[2 * i + 1] - h[2 * i]) / 100.0; }
  std::sort(st.begin(), st.end());
  std::sort(ka.begin(), ka.end());
  printf("%-8s grid %3d start q:", what, grid);
  for (int k = 0; k <= 4; ++k) printf(" %5.2f", st[(size_t)k * (grid - 1) / 4]);
  printf(" | kernarg latency q:");
  for (int k = 0; k <= 4; ++k) printf(" %5.2f", ka[(size_t)k * (grid - 1) / 4]);
  printf(" us\n");
}

int main() {
  const char* e = getenv("HIP_FORCE_DEV_KERNARG");
  printf("HIP_FORCE_DEV_KERNARG=%s\n", e ? e : "(unset)");
  unsigned long long* d;
  float *a, *b;
  CK(hipMalloc(&d, sizeof(unsigned long long) * 2 * 1024));
  CK(hipMalloc(&a, 4 * 1024));
  CK(hipMalloc(&b, 4 * 1024));
  CK(hipMemset(a, 0, 4 * 1024));
  std::vector<unsigned long long> h(2 * 1024);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int grid : {64, 224}) {
    for (int rep = 0; rep < 4; ++rep) hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, s, d, a, b);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
    report("eager", h, grid);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, s, d, a, b);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
    report("graph", h, grid);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
