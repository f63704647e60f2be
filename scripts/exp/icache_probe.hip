// Instruction-fetch cost on MI355X: each workgroup stamps s_memrealtime first, runs N KB of
// straight-line code (cold in the instruction cache after a different kernel ran), stamps
// again.  Printed: quantiles of (t1 - t0) and of the workgroups' t1 offsets, per code size,
// for a grid of 64 and 224 workgroups.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define REP(n) ".rept " #n "\n s_nop 0\n .endr\n"

template <int KB>
__global__ void __launch_bounds__(256) body(unsigned long long* out) {
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  if constexpr (KB == 8) asm volatile(REP(2048) ::: "v0");
  if constexpr (KB == 32) asm volatile(REP(8192) ::: "v0");
  if constexpr (KB == 64) asm volatile(REP(16384) ::: "v0");
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = t0;
    out[blockIdx.x * 2 + 1] = t1;
  }
}
__global__ void other(float* p) { p[threadIdx.x] += 1.f; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int KB>
int run(int grid, unsigned long long* d, float* f, std::vector<unsigned long long>& h) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(other, dim3(1), dim3(64), 0, 0, f);
    hipLaunchKernelGGL(body<KB>, dim3(grid), dim3(256), 0, 0, d);
  }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  std::vector<double> dur(grid), end(grid);
  unsigned long long t0 = ~0ull;
  for (int i = 0; i < grid; ++i) t0 = std::min(t0, h[2 * i]);
  for (int i = 0; i < grid; ++i) { dur[i] = (h[2 * i + 1] - h[2 * i]) / 100.0; end[i] = (h[2 * i + 1] - t0) / 100.0; }
  std::sort(dur.begin(), dur.end());
  std::sort(end.begin(), end.end());
  printf("code %2d KB grid %3d  body time q:", KB, grid);
  for (int k = 0; k <= 4; ++k) printf(" %5.2f", dur[(size_t)k * (grid - 1) / 4]);
  printf("  | body end q:");
  for (int k = 0; k <= 4; ++k) printf(" %5.2f", end[(size_t)k * (grid - 1) / 4]);
  printf(" us\n");
  return 0;
}

int main() {
  unsigned long long* d;
  float* f;
  CK(hipMalloc(&d, sizeof(unsigned long long) * 2 * 1024));
  CK(hipMalloc(&f, 4096));
  std::vector<unsigned long long> h(2 * 1024);
  for (int grid : {64, 224}) {
    if (run<0>(grid, d, f, h) || run<8>(grid, d, f, h) || run<32>(grid, d, f, h) || run<64>(grid, d, f, h)) return 1;
  }
  return 0;
}
