// Shared helpers for the gfx950 (MI355X, CDNA4) kernels of ddp_practice_amd.
//
// Conventions used by every kernel file:
//  * wave = 64 lanes; block sizes are multiples of 64.
//  * MFMA fragments follow the gfx950 maps documented in
//    /opt/skills/guides/cdna_hip_programming.md §3:
//      16x16x32 (bf16/f16): lane l holds A[l&15][8*(l>>4)+j], B[8*(l>>4)+j][l&15],
//                           C/D: col = l&15, row = 4*(l>>4)+r (r = 0..3)
//      16x16x4  (f32)     : lane l holds A[l&15][l>>4],      B[l>>4][l&15]
//  * every launch goes to the caller's current HIP stream (graph-capturable:
//    no allocation, no host sync inside a launch function).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>
#include <cstdlib>

namespace dpa {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// Non-finite check of AMP gradients by the kernels that produce them (the ConvNet's
// pre-checked optimizer step, optim/sgd.py): the step's head launch clears word[0] (and
// records the scale in word[1]); a producer lane that writes a (scaled) value that is
// non-finite -- or, for partial rows summed later, could overflow the sum (|v| > bound =
// FLT_MAX / rows) -- sets word[0].  The fused AMP step reads the word and agrees on found_inf
// without a grid barrier.  Scaled and unscaled finiteness agree while the scale is >= 1
// (unscaling only shrinks); the step takes the barrier for a smaller scale.  At W > 1 the
// bound is FLT_MAX / W (the step's average of W checked values cannot overflow) and a
// flagged rank pushes NaN to its peers in the step's gradient exchange, so every rank skips.
struct GradChk {
  int* word = nullptr;  // nullptr: no check
  float bound = 3.402823466e38f;  // |final value| limit (FLT_MAX / world)
  __device__ __forceinline__ static bool bad(float v, float bound) {
    return !(fabsf(v) <= bound);  // NaN / inf / beyond the bound
  }
  __device__ __forceinline__ void flag(bool b) const {
    if (b) *word = 1;  // (every writer stores the same value; ordered by the kernel boundary)
  }
};

#define DPA_CHECK_HIP(expr)                                                          \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ",       \
                __FILE__, ":", __LINE__);                                            \
  } while (0)

#define DPA_CHECK_LAUNCH() DPA_CHECK_HIP(hipGetLastError())

// Phase timestamps for kernel tuning (experiment builds with -DDPA_TIMING only):
// DPA_STAMP(i) records s_memrealtime (100 MHz) of wave 0 of every workgroup in
// dpa_stamps[block][i]; read back with runtime.read_stamps().
#ifdef DPA_TIMING
#define DPA_MAX_STAMP_BLOCKS 512
#define DPA_NSTAMPS 16
// one copy per translation unit (-fno-gpu-rdc): read back from the TU that owns the kernels
static __device__ unsigned long long dpa_stamps[DPA_MAX_STAMP_BLOCKS * DPA_NSTAMPS];
// The clock is read first (volatile asm, its own wait): with the builtin, the compiler put the
// scalar load of the stamp array's address in front of it, and the read queued behind that
// load's miss -- workgroup starts looked 2-4 us late (scripts/exp/dispatch_skew.hip: real
// dispatch skew <= 0.4 us).
#define DPA_STAMP(i)                                                                                     \
  do {                                                                                                   \
    unsigned long long dpa_t_;                                                                           \
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(dpa_t_));                             \
    if (threadIdx.x == 0 && blockIdx.x < DPA_MAX_STAMP_BLOCKS)                                           \
      dpa_stamps[blockIdx.x * DPA_NSTAMPS + (i)] = dpa_t_;                                               \
  } while (0)
// read_stamps() / clear_stamps() of the calling translation unit's stamp array
#define DPA_DEF_STAMP_FNS(s)                                                                          \
  do {                                                                                                \
    (s).def("read_stamps", []() {                                                                     \
      auto out = at::empty({DPA_MAX_STAMP_BLOCKS, DPA_NSTAMPS}, at::TensorOptions().dtype(at::kLong)); \
      DPA_CHECK_HIP(hipDeviceSynchronize());                                                          \
      DPA_CHECK_HIP(hipMemcpyFromSymbol(out.data_ptr(), HIP_SYMBOL(dpa_stamps),                       \
                                        sizeof(unsigned long long) * DPA_MAX_STAMP_BLOCKS * DPA_NSTAMPS)); \
      return out;                                                                                     \
    });                                                                                               \
    (s).def("clear_stamps", []() {                                                                    \
      DPA_CHECK_HIP(hipDeviceSynchronize());                                                          \
      std::vector<unsigned long long> z(DPA_MAX_STAMP_BLOCKS * DPA_NSTAMPS, 0ull);                    \
      DPA_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dpa_stamps), z.data(),                               \
                                      z.size() * sizeof(unsigned long long)));                         \
    });                                                                                               \
  } while (0)
#else
#define DPA_STAMP(i) do {} while (0)
#define DPA_DEF_STAMP_FNS(s) do {} while (0)
#endif

#define DPA_CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP device tensor")
#define DPA_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define DPA_CHECK_INPUT(t) \
  do {                     \
    DPA_CHECK_DEV(t);      \
    DPA_CHECK_CONTIG(t);   \
  } while (0)

// Storage dtype tags for activations: fp32, bf16, fp16.
enum class DT : int { F32 = 0, BF16 = 1, F16 = 2 };

inline DT dt_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DT::F32;
    case at::kBFloat16: return DT::BF16;
    case at::kHalf: return DT::F16;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return DT::F32;
}

// ---- scalar conversions (device) -------------------------------------------
template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float x) { return x; }
  __device__ __forceinline__ static float from_f(float x) { return x; }
};
template <> struct Cvt<__hip_bfloat16> {
  __device__ __forceinline__ static float to_f(__hip_bfloat16 x) { return __bfloat162float(x); }
  __device__ __forceinline__ static __hip_bfloat16 from_f(float x) { return __float2bfloat16(x); }
};
template <> struct Cvt<__half> {
  __device__ __forceinline__ static float to_f(__half x) { return __half2float(x); }
  __device__ __forceinline__ static __half from_f(float x) { return __float2half(x); }
};

template <typename T> __device__ __forceinline__ float ld_f(const T* p) { return Cvt<T>::to_f(*p); }
template <typename T> __device__ __forceinline__ void st_f(T* p, float v) { *p = Cvt<T>::from_f(v); }

// ---- wave reductions ----------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// LDS-only workgroup barrier: __syncthreads() is a workgroup fence whose s_waitcnt vmcnt(0)
// makes every wave wait for ALL its outstanding global memory operations (stores included)
// before the barrier.  Where the barrier only orders LDS accesses, wait for LDS alone.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Lane-group sums without an LDS round trip.  __shfl_xor compiles to ds_bpermute_b32, each
// step an LDS round trip waited with lgkmcnt(0): the ConvNet head's ten 64-lane reductions
// were 60 serialized round trips (~3.5 us, head_row_kernel ISA).  Here: DPP lane moves inside
// 16-lane rows (quad butterflies, half-row and row mirrors) and gfx950's v_permlane16_swap /
// v_permlane32_swap across rows -- all VALU.  group_sum<G>: every lane gets the sum over its
// aligned group of G lanes, in a fixed association (deterministic, the same in every lane of
// the group).  Needs all lanes of the group active (a DPP read of an inactive lane sees a
// stale register).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// v[l] + v[l ^ 16] (low row first) in every lane
__device__ __forceinline__ float xor16_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
// v[l] + v[l ^ 32] (low half first) in every lane
__device__ __forceinline__ float xor32_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "lane group of 2..64");
  v += dpp_mov<0xB1>(v);                       // quad_perm [1,0,3,2]: pairs
  if constexpr (G >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: quads
  if constexpr (G >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: the other quad of the 8
  if constexpr (G >= 16) v += dpp_mov<0x140>(v); // row_mirror: the other 8 of the row
  if constexpr (G >= 32) v = xor16_sum(v);
  if constexpr (G >= 64) v = xor32_sum(v);
  return v;
}
__device__ __forceinline__ float wave_sum_dpp(float v) { return group_sum<64>(v); }
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of one float; `red` must hold >= blockDim/64 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---- MFMA wrappers -------------------------------------------------------------
// Low-precision element type -> 8-element MFMA operand vector.
template <typename T> struct Mfma16;
template <> struct Mfma16<__hip_bfloat16> {
  typedef bf16x8 frag;
  __device__ __forceinline__ static f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma16<__half> {
  typedef f16x8 frag;
  __device__ __forceinline__ static f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ f32x4 mfma_f32_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(8))) float f32x8;

// Storage-type traits for the "16 x 16 x (8 per lane-group)" MFMA step used by
// every GEMM-shaped kernel here.  Each lane supplies 8 K-consecutive operand
// elements (lane group q = lane>>4 owns logical k = 8q..8q+7 of a 32-deep step):
//   bf16/f16 : one v_mfma_f32_16x16x32_{bf16,f16}
//   f32      : eight v_mfma_f32_16x16x4_f32 (exact fp32); sub-step s pairs the
//              s-th element of every lane group, i.e. logical k = 8q+s, which is
//              a consistent permutation of K for A and B, so the sum is the same.
template <typename T> struct MM;
template <> struct MM<float> {
  typedef f32x8 frag;
  typedef float elem;
  __device__ __forceinline__ static f32x4 mma(const frag& a, const frag& b, f32x4 c) {
#pragma unroll
    for (int s = 0; s < 8; ++s) c = mfma_f32_16x16x4(a[s], b[s], c);
    return c;
  }
  __device__ __forceinline__ static frag ld(const float* p) {  // 16-B aligned
    f32x4 lo = *reinterpret_cast<const f32x4*>(p);
    f32x4 hi = *reinterpret_cast<const f32x4*>(p + 4);
    frag f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
  __device__ __forceinline__ static elem cv(float x) { return x; }
  __device__ __forceinline__ static float rnd(float x) { return x; }
};
template <> struct MM<__hip_bfloat16> {
  typedef bf16x8 frag;
  typedef __bf16 elem;
  __device__ __forceinline__ static f32x4 mma(const frag& a, const frag& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static frag ld(const __hip_bfloat16* p) {
    return *reinterpret_cast<const frag*>(p);
  }
  __device__ __forceinline__ static elem cv(float x) { return (__bf16)x; }
  __device__ __forceinline__ static float rnd(float x) { return (float)(__bf16)x; }
};
template <> struct MM<__half> {
  typedef f16x8 frag;
  typedef _Float16 elem;
  __device__ __forceinline__ static f32x4 mma(const frag& a, const frag& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static frag ld(const __half* p) {
    return *reinterpret_cast<const frag*>(p);
  }
  __device__ __forceinline__ static elem cv(float x) { return (_Float16)x; }
  __device__ __forceinline__ static float rnd(float x) { return (float)(_Float16)x; }
};

// Round a float through storage type T (what a stored-then-reloaded value is).
template <typename T> __device__ __forceinline__ float rnd_t(float x) { return MM<T>::rnd(x); }

// Dispatch a templated lambda over the activation storage dtype.
#define DPA_DISPATCH_T(dt, ...)                                  \
  do {                                                           \
    switch (dt) {                                                \
      case ::dpa::DT::F32: { typedef float T; __VA_ARGS__; break; }          \
      case ::dpa::DT::BF16: { typedef __hip_bfloat16 T; __VA_ARGS__; break; } \
      case ::dpa::DT::F16: { typedef __half T; __VA_ARGS__; break; }         \
    }                                                            \
  } while (0)

template <typename T> inline T* dptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}

constexpr int ceil_to(int x, int m) { return (x + m - 1) / m * m; }

// torch.optim.SGD's update with ATen's foreach rounding, spelled out: d = g + wd*p (one fma),
// buf = buf*momentum (rounded) + (1-dampening)*d (one fma), d = d + momentum*buf (nesterov,
// one fma), p = p - lr*d (one fma).  Every SGD kernel of the package (optim.hip,
// amp_step.h) goes through it, so the fused, multi-tensor and slab-column updates round alike
// and train bit-identically (left to -ffp-contract, the same source line was contracted
// differently in different kernels, and the 1-ulp differences grew over a few steps).
__device__ __forceinline__ float sgd_rule(float p, float g, float& buf, bool first, float lr, float momentum,
                                          float dampening, float wd, int nesterov, int maximize) {
  float d = maximize ? -g : g;
  if (wd != 0.f) d = __builtin_fmaf(wd, p, d);
  if (momentum != 0.f) {
    const float mb = momentum * buf;  // its own rounding (ATen: a separate _foreach_mul_)
    buf = first ? d : __builtin_fmaf(1.f - dampening, d, mb);
    d = nesterov ? __builtin_fmaf(momentum, buf, d) : buf;
  }
  return __builtin_fmaf(-lr, d, p);
}
// four lanes of a granule: p, buf updated in place
__device__ __forceinline__ void sgd_rule4(f32x4& p, f32x4 g, f32x4& buf, bool first, float lr, float momentum,
                                          float dampening, float wd, int nesterov, int maximize) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float b = buf[j];
    p[j] = sgd_rule(p[j], g[j], b, first, lr, momentum, dampening, wd, nesterov, maximize);
    buf[j] = b;
  }
}

// Can every workgroup of a `grid` x `threads` launch of `kernel` (dynamic LDS
// `lds`) be resident on the current device at once?  Launches whose
// workgroups wait on each other (grid barriers, in-kernel exchanges polled by
// every workgroup) must pass this before they are taken.  The occupancy API
// can over-report by one workgroup per CU for SGPR-heavy kernels
// (MI355X_MICROARCH.md "Residency and cooperative launch"), so one is taken
// off whenever it reports more than one.
// The CUs this process's workgroups may use: the device's, or fewer for a rank confined to a
// CU range (runtime/device.shared_cu_mask: HSA_CU_MASK, DPA_RESIDENT_CUS).
inline int resident_cus(int device_cus) {
  static const int cap = [] {
    const char* e = std::getenv("DPA_RESIDENT_CUS");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  return cap > 0 && cap < device_cus ? cap : device_cus;
}

inline bool co_resident(const void* kernel, int grid, int threads, size_t lds = 0) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  cus = resident_cus(cus);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess) return false;
  const int eff = per_cu > 1 ? per_cu - 1 : per_cu;
  return (long long)grid <= (long long)eff * cus;
}

// Column `col` of a [rows][n] slab summed over rows g, g + G, g + 2G, ... in that order.
// Up to 16 rows per lane are loaded in ONE batch (clamped addresses, every load in flight
// before the first add; the surplus is dropped by a select on registers), so a lane
// costs one memory round trip for the ConvNet's 224- and 128-row slabs.  Shared by the
// column-sum launch and the fused AMP-SGD SlabSrc workgroups (csrc/kernels/optim.hip):
// both produce bitwise the same sums.
template <int G>
__device__ __forceinline__ float slab_colsum(const float* __restrict__ slab, int rows, int n, int col, int g) {
  if (rows <= 0 || n <= 0) return 0.f;
  const int cc = col < n ? col : n - 1;
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = slab[(size_t)min(g + j * G, rows - 1) * n + cc];
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) a += (g + j * G < rows) ? v[j] : 0.f;
  for (int r = g + 16 * G; r < rows; r += G) a += slab[(size_t)r * n + cc];
  return col < n ? a : 0.f;
}

}  // namespace dpa
