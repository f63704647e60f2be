// Workgroup dispatch skew on MI355X: each workgroup records s_memrealtime (100 MHz) as its
// first instruction; printed: start offsets (us) by block index and sorted quantiles, for
// grids of 32-224 workgroups of 256 lanes with 0 / 40 / 64 KB of LDS, after a preceding
// launch of the same kernel (the steady-state case of a step of back-to-back kernels).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int LDS_KB>
__global__ void __launch_bounds__(256) probe(unsigned long long* out, int spin) {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  __shared__ float lds[LDS_KB > 0 ? LDS_KB * 256 : 1];
  if (LDS_KB > 0) lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  // a little work so the grid is not instantly done
  float a = LDS_KB > 0 ? lds[(threadIdx.x + 1) & 255] : 0.f;
  for (int i = 0; i < spin; ++i) a = a * 0.999f + 1.f;
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = t;
    out[blockIdx.x * 2 + 1] = (unsigned long long)__float_as_uint(a);
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LDS_KB>
int run(int grid, unsigned long long* d, std::vector<unsigned long long>& h) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe<LDS_KB>, dim3(grid), dim3(256), 0, 0, d, 2000);
    hipLaunchKernelGGL(probe<LDS_KB>, dim3(grid), dim3(256), 0, 0, d, 2000);
  }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  std::vector<double> st(grid);
  unsigned long long t0 = ~0ull;
  for (int i = 0; i < grid; ++i) t0 = std::min(t0, h[2 * i]);
  for (int i = 0; i < grid; ++i) st[i] = (h[2 * i] - t0) / 100.0;
  std::vector<double> srt = st;
  std::sort(srt.begin(), srt.end());
  printf("lds %2d KB grid %3d  by index:", LDS_KB, grid);
  for (int k = 0; k <= 8; ++k) printf(" %5.2f", st[(size_t)k * (grid - 1) / 8]);
  printf("  | first 8:");
  for (int k = 0; k < 8 && k < grid; ++k) printf(" %5.2f", st[k]);
  printf("  | sorted q:");
  for (int k = 0; k <= 8; ++k) printf(" %5.2f", srt[(size_t)k * (grid - 1) / 8]);
  printf("\n");
  return 0;
}

int main() {
  unsigned long long* d;
  CK(hipMalloc(&d, sizeof(unsigned long long) * 2 * 4096));
  std::vector<unsigned long long> h(2 * 4096);
  for (int grid : {32, 64, 199, 224, 512}) {
    if (run<0>(grid, d, h)) return 1;
    if (run<40>(grid, d, h)) return 1;
    if (run<64>(grid, d, h)) return 1;
  }
  CK(hipFree(d));
  return 0;
}
