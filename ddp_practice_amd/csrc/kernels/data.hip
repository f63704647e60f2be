// Device-resident data pipeline: the whole uint8 image set lives in HBM (MNIST
// train is 47 MB; 288 GB per GPU makes this free), and one kernel per step
// gathers the batch through the epoch's DistributedSampler index list and
// converts to the compute dtype (ToTensor semantics: x/255, no normalisation;
// reference: /root/reference/ddp_main.py:127-142, 86-87).
//
// The batch position is read from a DEVICE step counter that the kernel
// advances itself (last-arriving workgroup), so a captured hipGraph of N
// training steps replays with zero host work per step.
#include "common.h"

namespace dpa {
namespace data {

constexpr int NTHR = 256;

// ctr[0] = step within the epoch, ctr[1] = arrival counter (self-resetting).
template <typename T>
__global__ void __launch_bounds__(NTHR)
gather_kernel(const uint8_t* __restrict__ imgs, const int64_t* __restrict__ labels,
              const int64_t* __restrict__ order, int64_t order_len, int* __restrict__ ctr,
              int64_t fixed_step, T* __restrict__ out, int64_t* __restrict__ lab_out, int B, int npix,
              float scale, float shift) {
  __shared__ int step_sh;
  if (threadIdx.x == 0) step_sh = fixed_step >= 0 ? (int)fixed_step : ctr[0];
  __syncthreads();
  const int64_t base = (int64_t)step_sh * B;
  // one workgroup per image (grid-stride)
  for (int i = blockIdx.x; i < B; i += gridDim.x) {
    int64_t pos = base + i;
    if (pos >= order_len) pos = order_len - 1;  // never reached with a correct host-side batch count
    const int64_t src = order[pos];
    const uint8_t* s = imgs + src * npix;
    T* d = out + (int64_t)i * npix;
    if ((npix & 3) == 0) {
      const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s);
      for (int j = threadIdx.x; j < npix / 4; j += NTHR) {
        const uint32_t v = s4[j];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          d[4 * j + k] = Cvt<T>::from_f((float)((v >> (8 * k)) & 0xff) * scale + shift);
      }
    } else {
      for (int j = threadIdx.x; j < npix; j += NTHR) d[j] = Cvt<T>::from_f((float)s[j] * scale + shift);
    }
    if (threadIdx.x == 0) lab_out[i] = labels[src];
  }
  if (fixed_step < 0) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const int arrived = atomicAdd(&ctr[1], 1);
      if (arrived == (int)gridDim.x - 1) {
        ctr[1] = 0;
        ctr[0] = step_sh + 1;
        __threadfence();
      }
    }
  }
}

// ----------------------------------------------------------------------------
// Synthetic MNIST-shaped set generated in HBM (data/mnist.py ``synthetic(device=)``):
// image i = clip(variant[label_i, shift_i] * amp_i + 0.25 * N(0,1), 0, 1) as uint8,
// the per-pixel normal from a counter-based generator (splitmix64 of
// seed * 2^40 + i * npix + p, Box-Muller), so the set never exists on the host
// (no 0.5 s of host RNG and no 47 MB upload at start-up) and the host reference
// (mnist._noise_np) computes the same formula.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(NTHR)
synth_kernel(const float* __restrict__ variants, const int64_t* __restrict__ labels,
             const int64_t* __restrict__ which, const float* __restrict__ amp, int nvar, unsigned long long seed,
             int64_t n, int npix, uint8_t* __restrict__ out) {
  const int64_t total = n * npix;
  for (int64_t e = (int64_t)blockIdx.x * NTHR + threadIdx.x; e < total; e += (int64_t)gridDim.x * NTHR) {
    const int64_t i = e / npix;
    const int p = (int)(e - i * npix);
    const float base = variants[(labels[i] * nvar + which[i]) * npix + p] * amp[i];
    const unsigned long long z = splitmix64((seed << 40) + (unsigned long long)e);
    const float u1 = (float)((z >> 40) + 1ull) * (1.0f / 16777216.0f);  // (0, 1]
    const float u2 = (float)((z >> 16) & 0xFFFFFFull) * (1.0f / 16777216.0f);
    const float g = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795864f * u2);
    const float v = fminf(fmaxf(base + 0.25f * g, 0.0f), 1.0f) * 255.0f + 0.5f;
    out[e] = (uint8_t)v;
  }
}

void synth(at::Tensor variants, at::Tensor labels, at::Tensor which, at::Tensor amp, int64_t nvar, int64_t seed,
           at::Tensor out) {
  DPA_CHECK_INPUT(variants); DPA_CHECK_INPUT(labels); DPA_CHECK_INPUT(which); DPA_CHECK_INPUT(amp);
  DPA_CHECK_INPUT(out);
  TORCH_CHECK(variants.scalar_type() == at::kFloat && amp.scalar_type() == at::kFloat);
  TORCH_CHECK(labels.scalar_type() == at::kLong && which.scalar_type() == at::kLong && out.scalar_type() == at::kByte);
  const int64_t n = out.size(0);
  const int npix = (int)(out.numel() / std::max<int64_t>(n, 1));
  TORCH_CHECK(labels.numel() == n && which.numel() == n && amp.numel() == n && nvar > 0);
  TORCH_CHECK(variants.numel() % (nvar * npix) == 0, "variants must be [classes, nvar, npix]");
  const int64_t nclass = variants.numel() / (nvar * npix);
  (void)nclass;  // labels < classes and which < nvar are the host's contract (data/mnist.py)
  if (n == 0) return;
  const int64_t total = n * npix;
  const int grid = (int)std::min<int64_t>((total + NTHR - 1) / NTHR, 8192);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(NTHR), 0, cur_stream(), variants.data_ptr<float>(),
                     labels.data_ptr<int64_t>(), which.data_ptr<int64_t>(), amp.data_ptr<float>(), (int)nvar,
                     (unsigned long long)seed, n, npix, out.data_ptr<uint8_t>());
  DPA_CHECK_LAUNCH();
}

// step < 0 => use and advance the device counter `ctr` (int32[2]).
void gather(at::Tensor imgs, at::Tensor labels, at::Tensor order, at::Tensor ctr, int64_t step, at::Tensor out,
            at::Tensor lab_out, double scale, double shift) {
  DPA_CHECK_INPUT(imgs); DPA_CHECK_INPUT(labels); DPA_CHECK_INPUT(order); DPA_CHECK_INPUT(ctr);
  DPA_CHECK_INPUT(out); DPA_CHECK_INPUT(lab_out);
  TORCH_CHECK(imgs.scalar_type() == at::kByte && labels.scalar_type() == at::kLong);
  TORCH_CHECK(order.scalar_type() == at::kLong && ctr.scalar_type() == at::kInt && ctr.numel() >= 2);
  const int B = (int)out.size(0);
  const int npix = (int)(imgs.numel() / imgs.size(0));
  TORCH_CHECK(out.numel() == (int64_t)B * npix && lab_out.numel() == B);
  if (B == 0) return;
  const int grid = std::min(B, 1024);
  DPA_DISPATCH_T(dt_of(out), {
    hipLaunchKernelGGL(gather_kernel<T>, dim3(grid), dim3(NTHR), 0, cur_stream(), imgs.data_ptr<uint8_t>(),
                       labels.data_ptr<int64_t>(), order.data_ptr<int64_t>(), order.numel(), ctr.data_ptr<int>(),
                       step, dptr<T>(out), lab_out.data_ptr<int64_t>(), B, npix, (float)scale, (float)shift);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace data

void register_data(pybind11::module& m) {
  auto s = m.def_submodule("data", "device-resident dataset gather");
  s.def("gather", &data::gather);
  s.def("synth", &data::synth);
}

}  // namespace dpa
