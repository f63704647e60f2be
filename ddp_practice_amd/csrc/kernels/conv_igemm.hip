// NHWC implicit-GEMM convolution on MFMA for the ResNet-50 stress config
// (BASELINE.json config 5; the reference has no ResNet, its conv semantics are
// torch's: /root/reference/ddp_main.py:83-93 trains the ConvNet with nn.Conv2d).
//
//   y[p][k] = sum_{r,s,c} x[n][oh*st+r-pad][ow*st+s-pad][c] * w[k][r][s][c]
//   (p = (n, oh, ow): GEMM M = N*OH*OW pixels, N = Cout, K = R*S*C)
//
// with the BatchNorm statistics of the (storage-rounded) output produced in the
// epilogue -- per channel sum(y - shift), sum((y - shift)^2) around the running
// mean, the layout ops/bn_nhwc.py's kernels consume -- so a BN after a conv
// needs no separate statistics pass over the activation.
//
// Geometry (MI355X, 64-wide waves, 160 KB LDS):
//   * workgroup = 4 waves, tile 128 pixels x BN (64|128) channels, K-step 64
//     (one filter tap (r,s) x 64 input channels: C % 64 == 0);
//   * operands staged global -> registers -> LDS (double-buffered, one barrier
//     per K-step), 16-B chunks, rows of 64 bf16 with the chunk index XOR-swizzled
//     by (row & 7): the MFMA fragment reads (ds_read_b128) are at most 2-way;
//   * MFMA orientation: A = weights (rows = output channels), B = pixels, so a
//     lane's accumulator holds 4 CONSECUTIVE channels of one pixel
//     (C/D map: row = 4*(lane>>4) + j, col = lane & 15): the BN sums reduce over
//     lanes only, and the rounded tile is staged through LDS so it leaves as
//     whole-row 16-B stores;
//   * XCD-aware workgroup order (the channel tiles of one pixel tile share an L2);
//   * the pixel tile's im2col addresses (n, ih0, iw0) are computed once per
//     workgroup; padding / ragged M are zero-filled in the loader.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.h"
#include "comm/xgmi.h"

namespace dpa {
namespace igemm {

constexpr int THR = 256;
constexpr int BM = 128;  // pixels per workgroup
constexpr int BK = 64;   // reduction elements per K-step
constexpr int SHIFT_OFF = 4;  // stats layout of bn_nhwc.hip: [2C] = rows, shift at [2C+4 ...)

struct Geom {
  int N, H, W, C, OH, OW, K, R, S, stride, pad;
  long long M;  // N*OH*OW
  int accumulate = 0;  // conv_fwd: y += conv(x, w) (a residual gradient already in y)
  long long cls_rows = 0;  // MODE_S2T: pixel tiles per output parity class
  const void* aux = nullptr;  // conv_fwd epilogue: y[n][oh][ow] += aux[n][oh/2][ow/2] at even (oh, ow)
};

// Loader modes of the implicit-GEMM kernels:
//   MODE_GEN  one filter tap x 64 input channels per K-step (C % 64 == 0);
//   MODE_STEM the 7x7 / stride-2 stem on a 4-channel (3 + one zero) NHWC image: K is
//             the flattened (r, s, c) space padded to 8 x 8 x 4 = 256 (4 K-steps), a
//             16-B chunk is two horizontally adjacent taps x 4 channels (two 8-B loads);
//             the packed filter is [K][8][8][4] with zeros in the padding;
//   MODE_S2T  the data gradient of a 3x3 / stride-2 / pad-1 conv (a transposed conv):
//             dx is split by output parity (py, px) into four stride-1 sub-convolutions
//             of dy with 1, 2, 2 and 4 of the taps -- no zero-inserted dy, no wasted MFMA
//             -- each written with stride 2 into dx; filter = the flipped transpose.
constexpr int MODE_GEN = 0, MODE_STEM = 1, MODE_S2T = 2;
typedef __attribute__((ext_vector_type(2))) float f32x2;

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// Statistics tree (all in the conv launch, deterministic: fixed-order sums):
// every workgroup writes its [2][BN] partial row for its channel tile; the last
// arriver of each group of G1 pixel tiles (ticket) sums the group's rows into a
// level-2 row; the last level-2 arriver sums those and writes the final stats.
// Tickets are re-armed by their last arriver (graph replays need no reset).
constexpr int G1 = 32;

struct StatArgs {
  float* part;        // [nct][rows][2*BN] level 1, then [nct][NG][2*BN] level 2
  unsigned* tickets;  // [nct][NG] + [nct], zero-initialised
  float* stats;       // [3K+4]
  const float* shift; // running mean (the sums are taken around it)
  int64_t* nbt;       // num_batches_tracked (bumped once) or null
  int defer;          // 1: level-1 rows only (plain stores, no ticket), stat_tree_kernel follows
  // backward statistics of the BatchNorm whose output gradient this conv produces
  // (conv_glds_kernel BS > 0): stats = out [S1 | S2], plus dbeta = S1, dgamma = S2
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  int bwd = 0;
  // SyncBN: the finishers of the deferred tree (stat_sum1_kernel / stat_tree_kernel) exchange
  // their slices through this site (comm/xsite.h positioned form) -- the statistics leave
  // the launch already global, no all-reduce launch follows.  dgamma / dbeta stay local.
  xgmi::XSite xs;
};

// BS (conv_glds_kernel): the output is the gradient dy of a BatchNorm's output; the epilogue
// also takes that BN's backward sums S1 = sum dz, S2 = sum dz * xhat (dz = dy * relu'),
// as the separate bn_nhwc bwd_stats pass would (csrc/kernels/bn_nhwc.hip):
//   BS_Y:   ReLU mask from the BN's output y (a residual was added); the gradient is
//           accumulated onto the tapped residual gradient (Geom.accumulate)
//   BS_REC: ReLU mask recomputed from x (fma(x, gamma*invstd, beta - mean*gamma*invstd) > 0)
constexpr int BS_NONE = 0, BS_Y = 1, BS_REC = 2;
template <typename T>
struct BwdStatArgs {
  const T* x = nullptr;         // the BN's input (this conv's gradient layout [M][K])
  const T* y = nullptr;         // BS_Y: the BN's output
  const float* save = nullptr;  // mean[K], invstd[K] of the forward
  const float* gamma = nullptr;
  const float* beta = nullptr;
};

// Hand-off without fences (MI355X_MICROARCH.md "valid forms"): partial rows are
// written with agent-scope relaxed atomic stores (write-through past the XCD's L2),
// every wave drains its stores, one relaxed ticket per workgroup; the last arriver
// reads the rows with agent-scope atomic loads.  No release fence: that would write
// back the whole L2 (the conv output is dirty in it) once per workgroup.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool last_arriver(unsigned* ticket, unsigned n, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == n - 1;
    *s_flag = last;
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();
  return *s_flag != 0;
}

// dst[0, W) = sum over rows g < n of src[g*W + .] in row order (W = 2*BN <= 256 floats;
// src read with write-through loads; dst written write-through when `wt`): lane owns a
// column, THR/W row groups, combined in group order via scr
template <int W>
__device__ __forceinline__ void sum_rows(const float* __restrict__ src, int n, float* __restrict__ dst, float* scr,
                                         bool wt) {
  constexpr int RG = THR / W;
  const int col = threadIdx.x % W, rg = threadIdx.x / W;
  float acc = 0.f;
  for (int g0 = rg; g0 < n; g0 += 8 * RG) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int gg = g0 + u * RG;
      v[u] = ld_wt(src + (long long)(gg < n ? gg : 0) * W + col);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (g0 + u * RG < n) acc += v[u];
  }
  scr[rg * W + col] = acc;
  __syncthreads();
  if ((int)threadIdx.x < W) {
    float t = 0.f;
    for (int r = 0; r < RG; ++r) t += scr[r * W + threadIdx.x];
    if (wt) st_wt(dst + threadIdx.x, t); else dst[threadIdx.x] = t;
  }
  __syncthreads();
}

// slab: [gridDim(pixel tiles)][2][K] partial statistics (null: none)
template <typename T, int BN, int MODE = MODE_GEN>
__global__ void __launch_bounds__(THR)
conv_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y, StatArgs sa, Geom g) {
  using MMT = MM<T>;
  typedef typename MMT::frag frag;
  constexpr int CT = BN / 32;         // 16-channel tiles per wave (2 channel-waves)
  constexpr int PT = 4;               // 16-pixel tiles per wave (64 pixels)
  constexpr int BLD = BN / 32;        // B (weight) 16-B chunks per thread per K-step
  __shared__ __attribute__((aligned(16))) T lds[2][(BM + BN) * BK];
  __shared__ __attribute__((aligned(16))) float red[4][2][BN];
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave & 1, wc = wave >> 1;  // pixel half, channel half
  const int nct = g.K / BN;
  // XCD-aware tile order: the hardware deals workgroup i to XCD i % 8; remap so that
  // consecutive logical tiles -- the nct channel tiles of one pixel tile, which read the
  // same activation rows -- run on one XCD and share its L2 (bijective for any grid)
  const unsigned nwg = gridDim.x, hw = blockIdx.x;
  const unsigned q8 = nwg / 8, r8 = nwg % 8, xcd = hw % 8, slot = hw / 8;
  const unsigned lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const long long bm_all = lid / nct;
  const int bn = (int)(lid % nct);
  int cls = 0;  // MODE_S2T: output parity class (py, px)
  long long bm = bm_all;
  if constexpr (MODE == MODE_S2T) {
    cls = (int)(bm_all / g.cls_rows);
    bm = bm_all - (long long)cls * g.cls_rows;
  }
  const int py = cls >> 1, px = cls & 1;
  const int nsx = px ? 2 : 1;  // MODE_S2T: column taps of this class
  const long long p0 = bm * BM;
  const int k0 = bn * BN;
  const int cpt = MODE == MODE_STEM ? 1 : g.C / BK;
  const int KT = MODE == MODE_STEM ? 4 : (MODE == MODE_S2T ? (py ? 2 : 1) * nsx : g.R * g.S) * cpt;
  // loader geometry: chunk cc of rows rr + 32 i
  const int cc = tid & 7, rr = tid >> 3;
  long long xb[4];
  int ih0[4], iw0[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long p = p0 + rr + 32 * i;
    if (p < g.M) {
      const int ow = (int)(p % g.OW);
      const long long t = p / g.OW;
      const int oh = (int)(t % g.OH);
      const int n = (int)(t / g.OH);
      xb[i] = (long long)n * g.H * g.W * g.C;
      ih0[i] = MODE == MODE_S2T ? oh : oh * g.stride - g.pad;
      iw0[i] = MODE == MODE_S2T ? ow : ow * g.stride - g.pad;
    } else {
      xb[i] = -1;
      ih0[i] = iw0[i] = 0;
    }
  }
  const long long wrow = MODE == MODE_STEM ? 256 : (long long)g.R * g.S * g.C;
  f32x4 rx[4], rw[BLD];
  auto gload = [&](int kt) {
    long long woff;  // this K-step's offset inside a filter row
    if constexpr (MODE == MODE_STEM) {
      const int r = 2 * kt + (cc >> 2), s = (cc & 3) * 2;  // taps (r, s) and (r, s + 1)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ih = ih0[i] + r, iw = iw0[i] + s;
        const bool rok = xb[i] >= 0 && r < 7 && (unsigned)ih < (unsigned)g.H;
        const T* px_ = x + xb[i] + ((long long)ih * g.W + iw) * 4;
        f32x2 lo = {0.f, 0.f}, hi = {0.f, 0.f};
        if (rok && (unsigned)iw < (unsigned)g.W) lo = *reinterpret_cast<const f32x2*>(px_);
        if (rok && s + 1 < 7 && (unsigned)(iw + 1) < (unsigned)g.W) hi = *reinterpret_cast<const f32x2*>(px_ + 4);
        rx[i] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      }
      woff = (long long)kt * BK + cc * 8;
    } else if constexpr (MODE == MODE_S2T) {
      const int t = kt / cpt, c0 = (kt - t * cpt) * BK + cc * 8;
      const int ri = t / nsx, si = t - ri * nsx;
      const int r = py ? (ri ? 2 : 0) : 1, s = px ? (si ? 2 : 0) : 1;  // forward-filter tap
      const int dh = (py && !ri) ? 1 : 0, dw = (px && !si) ? 1 : 0;    // dy row / col offset
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ih = ih0[i] + dh, iw = iw0[i] + dw;
        const bool ok = xb[i] >= 0 && ih < g.H && iw < g.W;
        rx[i] = ok ? *reinterpret_cast<const f32x4*>(x + xb[i] + ((long long)ih * g.W + iw) * g.C + c0)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      woff = (long long)(8 - (r * 3 + s)) * g.C + c0;  // flipped filter: tap 8 - (3r + s)
    } else {
      const int rs = kt / cpt, c0 = (kt - rs * cpt) * BK + cc * 8;
      const int r = rs / g.S, s = rs - r * g.S;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ih = ih0[i] + r, iw = iw0[i] + s;
        const bool ok = xb[i] >= 0 && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        rx[i] = ok ? *reinterpret_cast<const f32x4*>(x + xb[i] + ((long long)ih * g.W + iw) * g.C + c0)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      woff = (long long)kt * BK + cc * 8;
    }
#pragma unroll
    for (int i = 0; i < BLD; ++i)
      rw[i] = *reinterpret_cast<const f32x4*>(w + (long long)(k0 + rr + 32 * i) * wrow + woff);
  };
  auto lstore = [&](int buf) {
    T* A = lds[buf];           // weights: rows [0, BN)
    T* B = lds[buf] + BN * BK;  // pixels:  rows [0, BM)
#pragma unroll
    for (int i = 0; i < BLD; ++i) *reinterpret_cast<f32x4*>(A + swz(rr + 32 * i, cc)) = rw[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(B + swz(rr + 32 * i, cc)) = rx[i];
  };
  f32x4 acc[CT][PT];
#pragma unroll
  for (int a = 0; a < CT; ++a)
#pragma unroll
    for (int b = 0; b < PT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the statistics' shift (running mean) for this lane's epilogue chunk, loaded with tile 0:
  // loaded after the K loop it cost every workgroup a dependent global-load latency
  float shp[8];
  if (sa.part != nullptr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) shp[j] = sa.shift[k0 + (tid % (BN / 8)) * 8 + j];
  }
  gload(0);
  lstore(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) gload(kt + 1);
    const T* A = lds[buf];
    const T* B = lds[buf] + BN * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag fa[CT], fb[PT];
#pragma unroll
      for (int a = 0; a < CT; ++a)
        fa[a] = *reinterpret_cast<const frag*>(A + swz(wc * (BN / 2) + a * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int b = 0; b < PT; ++b)
        fb[b] = *reinterpret_cast<const frag*>(B + swz(wp * 64 + b * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int a = 0; a < CT; ++a)
#pragma unroll
        for (int b = 0; b < PT; ++b) acc[a][b] = MMT::mma(fa[a], fb[b], acc[a][b]);
    }
    if (kt + 1 < KT) lstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds channels k0 + wc*BN/2 + 16a + 4fq + j of pixel p0 + wp*64 + 16b + fr.
  // The rounded tile goes through LDS ([pixel][channel], rows padded by 16 B: the
  // 8-byte writes of a 16-pixel column are conflict-free) and leaves as whole 16-B
  // chunks, consecutive lanes along a pixel's channels (full rows per store).
  constexpr int RS = BN + 8;  // LDS row stride (elements)
  T* tile = lds[0];
#pragma unroll
  for (int a = 0; a < CT; ++a) {
    const int cl = wc * (BN / 2) + a * 16 + 4 * fq;
#pragma unroll
    for (int b = 0; b < PT; ++b) {
      const int pl = wp * 64 + b * 16 + fr;
      T v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = Cvt<T>::from_f(acc[a][b][j]);
      *reinterpret_cast<u16x4*>(tile + pl * RS + cl) = *reinterpret_cast<const u16x4*>(v);
    }
  }
  __syncthreads();
  // With statistics, each lane first sums its fixed 8-channel chunk over its rows of
  // the tile (the rounded values, around the running mean) and the workgroup's partial
  // row goes out (write-through) and is ticketed BEFORE the output stores are issued:
  // the ticket's store drain then never waits for the output tile.
  constexpr int CPR = BN / 8;        // 16-B chunks per pixel row
  constexpr int RPI = THR / CPR;     // pixel rows per pass
  const bool stats = sa.part != nullptr;
  const int ch = tid % CPR;
  // output stores: whole 16-B chunks, consecutive lanes along a pixel's channels
  const T* aux = reinterpret_cast<const T*>(g.aux);
  auto store_tile = [&]() {
#pragma unroll
    for (int it = 0; it < BM / RPI; ++it) {
      const int pl = it * RPI + tid / CPR;
      const long long p = p0 + pl;
      if (p < g.M) {
        long long op = p;  // output pixel
        int oh = 0, ow = 0, n = 0;
        if (MODE == MODE_S2T || aux != nullptr) {
          ow = (int)(p % g.OW);
          const long long t = p / g.OW;
          oh = (int)(t % g.OH);
          n = (int)(t / g.OH);
        }
        if constexpr (MODE == MODE_S2T) op = ((long long)n * (2 * g.OH) + 2 * oh + py) * (2 * g.OW) + 2 * ow + px;
        f32x4* dst = reinterpret_cast<f32x4*>(y + op * g.K + k0 + ch * 8);
        f32x4 raw = *reinterpret_cast<const f32x4*>(tile + pl * RS + ch * 8);
        const bool add_aux = aux != nullptr && !(oh & 1) && !(ow & 1);
        if (g.accumulate || add_aux) {  // y (+)= tile (+ aux), summed in fp32, rounded once
          f32x4 old = {0.f, 0.f, 0.f, 0.f}, ax = {0.f, 0.f, 0.f, 0.f};
          if (g.accumulate) old = *dst;
          if (add_aux)
            ax = *reinterpret_cast<const f32x4*>(
                aux + (((long long)n * (g.OH >> 1) + (oh >> 1)) * (g.OW >> 1) + (ow >> 1)) * g.K + k0 + ch * 8);
          const T* a = reinterpret_cast<const T*>(&old);
          const T* e = reinterpret_cast<const T*>(&ax);
          T* b = reinterpret_cast<T*>(&raw);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            b[j] = Cvt<T>::from_f(Cvt<T>::to_f(a[j]) + Cvt<T>::to_f(e[j]) + Cvt<T>::to_f(b[j]));
        }
        *dst = raw;
      }
    }
  };
  // Without statistics, or with the tree deferred to stat_tree_kernel, the stores leave
  // first and drain while the sums are taken from the tile still in LDS (the barrier
  // after the sums is LDS-only: __syncthreads() would wait for the stores); with the
  // in-launch tree they follow the ticket, whose vmcnt(0) must not wait for the tile.
  const bool stores_first = !stats || sa.defer;
  if (stores_first) store_tile();
  bool last1 = false;
  long long rows = 0;
  int NG = 0, grp = 0, gsz = 0;
  if (stats) {
    float s1[8], s2[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] = s2[j] = 0.f;
      sh[j] = shp[j];
    }
    // unconditional reads of clamped rows (a per-row guard was a branch + wait per row)
    const int plast = (int)min((long long)BM, g.M - p0) - 1;
    f32x4 raw[BM / RPI];
#pragma unroll
    for (int it = 0; it < BM / RPI; ++it)
      raw[it] = *reinterpret_cast<const f32x4*>(tile + min(it * RPI + tid / CPR, plast) * RS + ch * 8);
#pragma unroll
    for (int it = 0; it < BM / RPI; ++it) {
      const float m = it * RPI + tid / CPR <= plast ? 1.f : 0.f;
      const T* e = reinterpret_cast<const T*>(&raw[it]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (Cvt<T>::to_f(e[j]) - sh[j]) * m;
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
    // lanes of one wave sharing the chunk: xor over the row bits of the lane index
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += __shfl_xor(s1[j], o);
        s2[j] += __shfl_xor(s2[j], o);
      }
    if (lane < CPR)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[wave][0][ch * 8 + j] = s1[j];
        red[wave][1][ch * 8 + j] = s2[j];
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    rows = (g.M + BM - 1) / BM;
    NG = (int)((rows + G1 - 1) / G1);
    float* lvl1 = sa.part + (long long)bn * rows * (2 * BN);
    if (sa.defer) {  // plain stores; the tree runs in stat_tree_kernel after this launch
      for (int t = tid; t < 2 * BN; t += THR) {
        const int q = t / BN, c = t % BN;
        lvl1[bm * (2 * BN) + t] = red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c];
      }
    } else {
      for (int t = tid; t < 2 * BN; t += THR) {
        const int q = t / BN, c = t % BN;
        st_wt(lvl1 + bm * (2 * BN) + t, red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c]);
      }
      grp = (int)(bm / G1);
      gsz = (int)min((long long)G1, rows - (long long)grp * G1);
      last1 = last_arriver(sa.tickets + bn * NG + grp, (unsigned)gsz, &s_flag);
    }
  }
  if (!stores_first) store_tile();
  if (!last1) return;
  __syncthreads();  // every lane is done with the tile: its LDS becomes the tree's scratch
  float* scr = reinterpret_cast<float*>(lds[1]);
  float* lvl1 = sa.part + (long long)bn * rows * (2 * BN);
  float* lvl2 = sa.part + (long long)nct * rows * (2 * BN) + (long long)bn * NG * (2 * BN);
  sum_rows<2 * BN>(lvl1 + (long long)grp * G1 * (2 * BN), gsz, lvl2 + (long long)grp * (2 * BN), scr, true);
  if (!last_arriver(sa.tickets + nct * NG + bn, (unsigned)NG, &s_flag)) return;
  float* tot = &red[0][0][0];
  sum_rows<2 * BN>(lvl2, NG, tot, scr, false);
  for (int t = tid; t < BN; t += THR) {
    sa.stats[k0 + t] = tot[t];
    sa.stats[g.K + k0 + t] = tot[BN + t];
    sa.stats[2 * g.K + SHIFT_OFF + k0 + t] = sa.shift[k0 + t];
  }
  if (bn == 0 && tid == 0) {
    sa.stats[2 * g.K] = (float)g.M;
    if (sa.nbt != nullptr) sa.nbt[0] = sa.nbt[0] + 1;
  }
}

// ---------------------------------------------------------------------------
// Implicit-GEMM convolution with both operands staged by LDS-DMA (MODE_GEN: any R x S,
// stride, padding; C % 64 == 0).  Written first for the 1x1 convs, a plain GEMM over the
// NHWC rows (y[p][k] = sum_c x[row(p)][c] * w[k][c]; M = pixels, N = Cout, K = C) -- the
// forward of 36 of ResNet-50's 53 convs and, with the transposed filter, their data
// gradients; a K-step is one filter tap x 64 channels, a padding tap reads a zero page.
// The general kernel above is LDS-bound on these shapes: a 64 x 64
// wave tile reads 32 FLOP per LDS byte and its register-staged ds_write_b128 stores
// cost ~13 LDS cycles per KiB, so the MFMAs idle behind the LDS (2x slower than
// hipBLASLt on the deep layers, profiles/r2_conv_igemm_fwd_vs_library_bs128.txt).
// This one:
//   * BP x BN tile (256 or 128 pixels x 128 or 64 channels), 4 waves as 2 x 2, wave tile
//     BP/2 x BN/2 (128 x 64: 43 FLOP per LDS byte);
//   * operands go global -> LDS with global_load_lds_dwordx4 (no VGPRs, no ds_write):
//     one wave-instruction fills 8 rows of 128 B, lane l its row l/8 at slot l%8; the
//     XOR swizzle of the LDS image (chunk ^ row&7, the same image the general kernel
//     writes) goes on the per-lane SOURCE address, since the LDS side is lane-linear;
//   * two LDS buffers, ONE barrier per K-step: wait the landed tile (vmcnt(0)) +
//     barrier, issue tile t+1 into the other buffer, MFMA on tile t; every LDS byte
//     lives in one __shared__ array (a second __shared__ object can make hipcc wait
//     vmcnt(0) before each K-step's first LDS read, cdna_hip_programming.md §5);
//   * the epilogue of the general kernel: rounded tile staged through LDS, the next
//     BN's statistics tree, whole-row stores, accumulate / aux for the fused gradients.
template <typename T, int BP, int BN, int NS = 2, int NW = 4>
struct G1x1Lds {
  static constexpr int STAGE = (BP + BN) * BK;            // elements per buffer
  static constexpr int RS = BN + 8;                       // epilogue tile row stride
  static constexpr int TILE = BP * RS * (int)sizeof(T);   // epilogue tile bytes
  static constexpr int RED = TILE;                        // float red[4][2][BN]
  static constexpr int FLAG = RED + NW * 2 * BN * 4;      // int s_flag
  static constexpr int SCR = FLAG + 16;                   // float scr[THR]
  static constexpr int EPI = SCR + 64 * NW * 4;
  static constexpr int MAIN = NS * STAGE * (int)sizeof(T);
  static constexpr int SHIFT = MAIN > EPI ? MAIN : EPI;  // float shift[BN] (statistics only)
  static constexpr int BWC = SHIFT + BN * 4;              // float mean|invstd|gamma|beta [4][BN] (BS)
  static constexpr int BYTES = BWC + 4 * BN * 4;
};

// one global_load_lds_dwordx4: 16 B per lane from `src` (per lane) to dst + 16 * lane (dst
// wave-uniform).  A non-template device function: called directly inside the kernel
// template, hipcc's host pass fails to instantiate it and emits no launch stub (undefined
// __device_stub__ at load time).
typedef __attribute__((address_space(3))) void* lds_vptr;
__device__ __forceinline__ void glds16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_vptr)dst, 16, 0, 0);
}

// 16 zero bytes: the LDS-DMA source of padding taps and out-of-range rows (a DMA cannot
// zero-fill; its per-lane source address can point here instead)
__device__ __attribute__((aligned(16))) unsigned char g_zero16[16] = {0};

// NS = 3 | 4 (DPA_GLDS_STAGES): three or four LDS buffers, NS - 1 tiles in flight across every barrier --
// the wait is a counted vmcnt (this wave's DMAs of the newest tile stay outstanding) and the
// barrier a raw s_barrier (__syncthreads() would add vmcnt(0)); one workgroup per CU (96 or 128 KB).
//
// NWP x NWC waves (pixels x channels; default 2 x 2 = 256 threads): the wide tiles run 8
// waves -- 256 x 128 (4 x 2) or 256 x 256 (2 x 4, wave tile 128 x 64) -- so each LDS-DMA byte
// feeds 1.33x / 2x the MFMAs of the 128 x 128 tile (its per-K-step cost is the DMA issue:
// profiles/r5b_stage_ab.txt, two or three tiles in flight gained nothing), and the second
// wave on every SIMD hides the first's fragment-read waits.  The wide variants always defer
// the statistics tree (stat_sum1_kernel / stat_tree_kernel).
template <typename T, int BP, int BN, int BS = BS_NONE, bool KXK = false, int NS = 2, int NWP = 2, int NWC = 2>
__global__ void __launch_bounds__(64 * NWP * NWC)
conv_glds_kernel(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y, StatArgs sa, Geom g,
               BwdStatArgs<T> bs) {
  using MMT = MM<T>;
  constexpr int NW = NWP * NWC, NT = 64 * NW;  // waves, threads
  using L = G1x1Lds<T, BP, BN, NS, NW>;
  static_assert(NS == 2 || ((NS == 3 || NS == 4) && BS == BS_NONE), "3-4 stages: forward / plain data gradients only");
  static_assert(NW == 4 || BS == BS_NONE || BP == 128, "wide pixel tiles: forward / plain data gradients only");
  typedef typename MMT::frag frag;
  constexpr int CT = BN / (16 * NWC);  // 16-channel tiles per wave
  constexpr int PT = BP / (16 * NWP);  // 16-pixel tiles per wave
  constexpr int AR = BP / (8 * NW);    // pixel rows per lane per K-step (8 rows per wave-instruction)
  constexpr int WR = BN / (8 * NW);    // filter rows per lane per K-step
  static_assert(CT >= 1 && PT >= 1 && AR >= 1 && WR >= 1 && AR * 8 * NW == BP && WR * 8 * NW == BN, "tile / waves");
  // the in-launch statistics tree (sum_rows) is written for 256 threads and 2 BN <= 256
  constexpr bool kInTree = NT == THR && 2 * BN <= THR;
  __shared__ __attribute__((aligned(16))) unsigned char smem[L::BYTES];
  T* const lds = reinterpret_cast<T*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave % NWP, wc = wave / NWP;
  const int nct = g.K / BN;
  // XCD-aware order (as conv_fwd_kernel): the channel tiles of one pixel tile share an L2
  const unsigned nwg = gridDim.x, hw = blockIdx.x;
  const unsigned q8 = nwg / 8, r8 = nwg % 8, xcd = hw % 8, slot = hw / 8;
  const unsigned lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const long long bm = lid / nct;
  const int bn = (int)(lid % nct);
  const long long p0 = bm * BP;
  const int k0 = bn * BN;
  // this lane's source rows: wave-instruction i covers rows (NW i + wave) * 8 .. + 7, the lane
  // row (lane >> 3) of them, logical chunk (lane & 7) ^ (row & 7) (row & 7 == lane >> 3).
  // KXK: a K-step is one filter tap (r, s) x 64 input channels (C % 64 == 0): the pixel's
  // input row is (n, oh*st - pad + r, ow*st - pad + s) and a padding tap reads the zero
  // page; else (1x1, pad 0) the K-steps walk the pixel's own input row (no bounds checks,
  // no per-step tap arithmetic: the general form costs the 1x1 shapes 5-12 %).
  const int lr = lane >> 3, chunk = (lane & 7) ^ lr;
  unsigned xo[AR], wo[WR];  // element offsets of the pixel rows / (n, ih0, iw0), filter rows (< 2^31)
  int ih0[AR], iw0[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    long long p = p0 + (i * NW + wave) * 8 + lr;
    p = p < g.M ? p : g.M - 1;  // ragged tail: a valid row, its output is not stored
    if constexpr (KXK) {
      const int ow = (int)(p % g.OW);
      const long long t = p / g.OW;
      const int oh = (int)(t % g.OH);
      const int n = (int)(t / g.OH);
      ih0[i] = oh * g.stride - g.pad;
      iw0[i] = ow * g.stride - g.pad;
      xo[i] = (unsigned)((((long long)n * g.H + ih0[i]) * g.W + iw0[i]) * g.C + chunk * 8);
    } else {
      long long r = p;
      if (g.stride != 1) {
        const int ow = (int)(p % g.OW);
        const long long t = p / g.OW;
        const int oh = (int)(t % g.OH);
        const int n = (int)(t / g.OH);
        r = ((long long)n * g.H + (long long)oh * g.stride) * g.W + (long long)ow * g.stride;
      }
      xo[i] = (unsigned)(r * g.C + chunk * 8);
      ih0[i] = iw0[i] = 0;
    }
  }
  const int wrow = KXK ? g.R * g.S * g.C : g.C;
#pragma unroll
  for (int i = 0; i < WR; ++i) wo[i] = (unsigned)((k0 + (i * NW + wave) * 8 + lr) * wrow + chunk * 8);
  const int cpt = g.C / BK;
  const int KT = KXK ? g.R * g.S * cpt : cpt;
  auto issue = [&](int kt, int buf) {
    T* base = lds + buf * L::STAGE;
#pragma unroll
    for (int i = 0; i < WR; ++i)
      glds16(w + wo[i] + kt * BK, base + (i * NW + wave) * 8 * BK);
    if constexpr (KXK) {
      const int rs = kt / cpt, c0 = (kt - rs * cpt) * BK;  // wave-uniform
      const int r = rs / g.S, s = rs - r * g.S;
      const int xk = (r * g.W + s) * g.C + c0;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bool ok = (unsigned)(ih0[i] + r) < (unsigned)g.H && (unsigned)(iw0[i] + s) < (unsigned)g.W;
        glds16(ok ? (const void*)(x + (int)xo[i] + xk) : (const void*)g_zero16,
               base + (BN + (i * NW + wave) * 8) * BK);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AR; ++i) glds16(x + xo[i] + kt * BK, base + (BN + (i * NW + wave) * 8) * BK);
    }
  };
  f32x4 acc[CT][PT];
#pragma unroll
  for (int a = 0; a < CT; ++a)
#pragma unroll
    for (int b = 0; b < PT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // the statistics' shift (running mean) rides with tile 0 into LDS: loaded after the K loop
  // it cost every workgroup a dependent global-load latency in its epilogue
  if (BS == BS_NONE && sa.part != nullptr && wave == 0 && lane < BN / 4)
    glds16(sa.shift + k0 + lane * 4, reinterpret_cast<float*>(smem + L::SHIFT));
  // BS: the BN's per-channel constants ride with tile 0 too (wave w: array w), and this
  // lane's epilogue chunks of x (and y, and the accumulated-onto gradient) are loaded into
  // registers now -- they land with tile 0 instead of stalling the epilogue
  constexpr int CPR = BN / 8;     // 16-B chunks per pixel row (epilogue)
  constexpr int RPI = NT / CPR;   // pixel rows per pass
  constexpr int NIT = BS != BS_NONE ? BP / RPI : 1;
  const int ch = tid % CPR;
  f32x4 bxr[NIT], byr[NIT], bor[NIT];
  if constexpr (BS != BS_NONE) {
    if (lane < BN / 4 && (BS == BS_REC ? wave < 4 : wave < 2)) {
      const float* src = wave == 0 ? bs.save + k0 : wave == 1 ? bs.save + g.K + k0 : wave == 2 ? bs.gamma + k0
                                                                                                : bs.beta + k0;
      glds16(src + lane * 4, reinterpret_cast<float*>(smem + L::BWC) + wave * BN);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const long long pp = min(p0 + it * RPI + tid / CPR, g.M - 1);
      const long long o = pp * g.K + k0 + ch * 8;
      bxr[it] = *reinterpret_cast<const f32x4*>(bs.x + o);
      if constexpr (BS == BS_Y) {
        byr[it] = *reinterpret_cast<const f32x4*>(bs.y + o);
        bor[it] = *reinterpret_cast<const f32x4*>(y + o);  // the tapped residual gradient
      }
    }
  }
  issue(0, 0);
  if (NS >= 3 && KT > 1) issue(1, 1);
  if (NS == 4 && KT > 2) issue(2, 2);
  int buf = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (NS == 2) {
      buf = kt & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of tile kt has landed
      __syncthreads();  // ... every wave's, and tile kt-1 (the other buffer) is no longer read
      if (kt + 1 < KT) issue(kt + 1, buf ^ 1);
    } else {
      // tile kt landed (the WR + AR DMAs per younger tile of this wave -- up to NS - 2 of
      // them -- may still be in flight); the barrier orders every wave's DMAs of tile kt
      // before any read, and every wave's reads of buffer (kt-1)%NS (tile kt-1, done: its
      // MFMAs have issued) before its refill with tile kt+NS-1
      if (NS == 4 && kt + 2 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (WR + AR)) : "memory");
      else if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WR + AR) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + NS - 1 < KT) issue(kt + NS - 1, buf == 0 ? NS - 1 : buf - 1);
    }
    const T* A = lds + buf * L::STAGE;  // filter rows [0, BN)
    const T* B = A + BN * BK;           // pixel rows [0, BP)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag fa[CT], fb[PT];
#pragma unroll
      for (int a = 0; a < CT; ++a)
        fa[a] = *reinterpret_cast<const frag*>(A + swz(wc * (BN / NWC) + a * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int b = 0; b < PT; ++b)
        fb[b] = *reinterpret_cast<const frag*>(B + swz(wp * (BP / NWP) + b * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int a = 0; a < CT; ++a)
#pragma unroll
        for (int b = 0; b < PT; ++b) acc[a][b] = MMT::mma(fa[a], fb[b], acc[a][b]);
    }
    if constexpr (NS >= 3) buf = buf == NS - 1 ? 0 : buf + 1;
  }
  __syncthreads();  // the last tile is read: the buffers become the epilogue's tile
  // ---- epilogue (conv_fwd_kernel's, for a BP-pixel tile) ----
  constexpr int RS = L::RS;
  T* tile = lds;
  float(*red)[2][BN] = reinterpret_cast<float(*)[2][BN]>(smem + L::RED);
  auto wave_sum = [&](int t) {  // column t of [2][BN] summed over the waves, in wave order
    const int q = t / BN, c = t % BN;
    float v = red[0][q][c];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][q][c];
    return v;
  };
  int* s_flag = reinterpret_cast<int*>(smem + L::FLAG);
  float* scr = reinterpret_cast<float*>(smem + L::SCR);
  const float* shl = reinterpret_cast<const float*>(smem + L::SHIFT);
#pragma unroll
  for (int a = 0; a < CT; ++a) {
    const int cl = wc * (BN / NWC) + a * 16 + 4 * fq;
#pragma unroll
    for (int b = 0; b < PT; ++b) {
      const int pl = wp * (BP / NWP) + b * 16 + fr;
      T v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = Cvt<T>::from_f(acc[a][b][j]);
      *reinterpret_cast<u16x4*>(tile + pl * RS + cl) = *reinterpret_cast<const u16x4*>(v);
    }
  }
  __syncthreads();
  const bool stats = BS == BS_NONE && sa.part != nullptr;
  // BS: this lane's 8 channels' BN constants, and its running sums of dz, dz * xhat
  float bmu[8], bis[8], bsc[8], bsh[8], bs1[8], bs2[8];
  if constexpr (BS != BS_NONE) {
    const float* bwc = reinterpret_cast<const float*>(smem + L::BWC);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = bwc[ch * 8 + j];
      bis[j] = bwc[BN + ch * 8 + j];
      if (BS == BS_REC) {
        bsc[j] = bwc[2 * BN + ch * 8 + j] * bis[j];
        bsh[j] = fmaf(-bmu[j], bsc[j], bwc[3 * BN + ch * 8 + j]);
      }
      bs1[j] = bs2[j] = 0.f;
    }
  }
  // output stores: whole 16-B chunks, consecutive lanes along a pixel's channels
  const T* aux = reinterpret_cast<const T*>(g.aux);
  auto store_tile = [&]() {
#pragma unroll
    for (int it = 0; it < BP / RPI; ++it) {
      const int pl = it * RPI + tid / CPR;
      const long long p = p0 + pl;
      if (p < g.M) {
        f32x4* dst = reinterpret_cast<f32x4*>(y + p * g.K + k0 + ch * 8);
        f32x4 raw = *reinterpret_cast<const f32x4*>(tile + pl * RS + ch * 8);
        int oh = 0, ow = 0, n = 0;
        if (aux != nullptr) {
          ow = (int)(p % g.OW);
          const long long t = p / g.OW;
          oh = (int)(t % g.OH);
          n = (int)(t / g.OH);
        }
        const bool add_aux = aux != nullptr && !(oh & 1) && !(ow & 1);
        if (g.accumulate || add_aux) {
          f32x4 old = {0.f, 0.f, 0.f, 0.f}, ax = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BS == BS_Y) old = bor[it];  // prefetched with tile 0
          else if (g.accumulate) old = *dst;
          if (add_aux)
            ax = *reinterpret_cast<const f32x4*>(
                aux + (((long long)n * (g.OH >> 1) + (oh >> 1)) * (g.OW >> 1) + (ow >> 1)) * g.K + k0 + ch * 8);
          const T* a = reinterpret_cast<const T*>(&old);
          const T* e = reinterpret_cast<const T*>(&ax);
          T* b = reinterpret_cast<T*>(&raw);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            b[j] = Cvt<T>::from_f(Cvt<T>::to_f(a[j]) + Cvt<T>::to_f(e[j]) + Cvt<T>::to_f(b[j]));
        }
        *dst = raw;
        if constexpr (BS != BS_NONE) {  // the BN backward sums of the stored (rounded) gradient
          const T* d = reinterpret_cast<const T*>(&raw);
          const T* xv = reinterpret_cast<const T*>(&bxr[it]);
          const T* yv = reinterpret_cast<const T*>(&byr[it]);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xf = Cvt<T>::to_f(xv[j]);
            const bool on = BS == BS_Y ? Cvt<T>::to_f(yv[j]) > 0.f : fmaf(xf, bsc[j], bsh[j]) > 0.f;
            const float z = on ? Cvt<T>::to_f(d[j]) : 0.f;
            bs1[j] += z;
            bs2[j] = fmaf(z, (xf - bmu[j]) * bis[j], bs2[j]);
          }
        }
      }
    }
  };
  // Without statistics, or with the tree deferred to stat_tree_kernel, the stores leave
  // first and drain while the sums are taken from the tile still in LDS; with the
  // in-launch tree they follow the ticket (its vmcnt(0) must not wait for the tile).
  const bool stores_first = !stats || sa.defer || !kInTree;
  if (stores_first) store_tile();
  if constexpr (BS != BS_NONE) {  // -> level-1 row of this pixel tile (stat_tree_kernel follows)
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bs1[j] += __shfl_xor(bs1[j], o);
        bs2[j] += __shfl_xor(bs2[j], o);
      }
    if (lane < CPR)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[wave][0][ch * 8 + j] = bs1[j];
        red[wave][1][ch * 8 + j] = bs2[j];
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const long long nrows = (g.M + BP - 1) / BP;
    float* lvl1 = sa.part + (long long)bn * nrows * (2 * BN);
    for (int t = tid; t < 2 * BN; t += NT) lvl1[bm * (2 * BN) + t] = wave_sum(t);
    return;
  }
  bool last1 = false;
  long long rows = 0;
  int NG = 0, grp = 0, gsz = 0;
  if (stats) {
    float s1[8], s2[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] = s2[j] = 0.f;
      sh[j] = shl[ch * 8 + j];
    }
    // unconditional reads of clamped rows (a per-row guard was a branch + wait per row)
    const int plast = (int)min((long long)BP, g.M - p0) - 1;
    f32x4 raw[BP / RPI];
#pragma unroll
    for (int it = 0; it < BP / RPI; ++it)
      raw[it] = *reinterpret_cast<const f32x4*>(tile + min(it * RPI + tid / CPR, plast) * RS + ch * 8);
#pragma unroll
    for (int it = 0; it < BP / RPI; ++it) {
      const float m = it * RPI + tid / CPR <= plast ? 1.f : 0.f;
      const T* e = reinterpret_cast<const T*>(&raw[it]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (Cvt<T>::to_f(e[j]) - sh[j]) * m;
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += __shfl_xor(s1[j], o);
        s2[j] += __shfl_xor(s2[j], o);
      }
    if (lane < CPR)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[wave][0][ch * 8 + j] = s1[j];
        red[wave][1][ch * 8 + j] = s2[j];
      }
    // LDS-only barrier: __syncthreads() is a workgroup fence whose vmcnt(0) would wait
    // here for the whole output tile's stores to drain (~30 us on a 56x56 x 256 conv)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    rows = (g.M + BP - 1) / BP;
    NG = (int)((rows + G1 - 1) / G1);
    float* lvl1 = sa.part + (long long)bn * rows * (2 * BN);
    if (sa.defer || !kInTree) {  // plain stores; the tree runs in stat_tree_kernel after this launch
      for (int t = tid; t < 2 * BN; t += NT) lvl1[bm * (2 * BN) + t] = wave_sum(t);
    } else {
      for (int t = tid; t < 2 * BN; t += NT) st_wt(lvl1 + bm * (2 * BN) + t, wave_sum(t));
      grp = (int)(bm / G1);
      gsz = (int)min((long long)G1, rows - (long long)grp * G1);
      last1 = last_arriver(sa.tickets + bn * NG + grp, (unsigned)gsz, s_flag);
    }
  }
  if (!stores_first) store_tile();
  if (!last1) return;
  if constexpr (kInTree) {  // (wide tiles always defer: last1 is false there)
    __syncthreads();
    float* lvl1 = sa.part + (long long)bn * rows * (2 * BN);
    float* lvl2 = sa.part + (long long)nct * rows * (2 * BN) + (long long)bn * NG * (2 * BN);
    sum_rows<2 * BN>(lvl1 + (long long)grp * G1 * (2 * BN), gsz, lvl2 + (long long)grp * (2 * BN), scr, true);
    if (!last_arriver(sa.tickets + nct * NG + bn, (unsigned)NG, s_flag)) return;
    float* tot = &red[0][0][0];
    sum_rows<2 * BN>(lvl2, NG, tot, scr, false);
    for (int t = tid; t < BN; t += NT) {
      sa.stats[k0 + t] = tot[t];
      sa.stats[g.K + k0 + t] = tot[BN + t];
      sa.stats[2 * g.K + SHIFT_OFF + k0 + t] = sa.shift[k0 + t];
    }
    if (bn == 0 && tid == 0) {
      sa.stats[2 * g.K] = (float)g.M;
      if (sa.nbt != nullptr) sa.nbt[0] = sa.nbt[0] + 1;
    }
  }
}

// The statistics tree of a conv launch with StatArgs.defer: the conv's workgroups stored
// their level-1 partial rows with plain stores and exited (no write-through drain, no
// ticket round trip per workgroup: on a many-round grid that serial hand-off cost each
// workgroup ~3 us, ~30 us per large conv); this launch runs the same two levels --
// workgroup (bn, grp) sums its group of G1 rows into a level-2 row, the last of a
// channel tile's NG arrivals sums those into the final statistics.  Same association
// as the in-launch tree: the result is bitwise the same.
// One-level variant for grids of <= S1_MAXROWS pixel tiles (every ResNet-50 conv but the
// 56x56 ones): a
// workgroup of 1024 lanes owns S1_COLS of the 2*BN level-1 columns of one channel tile as
// 16 row groups x 64 columns, each group with every row it sums in flight (16 loads),
// combined in group order through LDS -- one dependent round trip instead of the two
// levels' three (rows, ticket, level-2 rows).  Fixed order: deterministic.
constexpr int S1_THR = 1024, S1_COLS = 64, S1_RG = S1_THR / S1_COLS, S1_MAXROWS = 1024;
// NL: loads per lane, all in flight (16: up to 256 rows; 64: up to S1_MAXROWS)
template <int BN, int NL>
__global__ void __launch_bounds__(S1_THR) stat_sum1_kernel(StatArgs sa, long long M, int BM_, int K) {
  __shared__ float part[S1_RG][S1_COLS];
  __shared__ uint32_t ep_s;
  const int nct = K / BN, bn = blockIdx.x, c0 = blockIdx.y * S1_COLS;
  const int rows = (int)((M + BM_ - 1) / BM_);
  const int col = threadIdx.x % S1_COLS, rg = threadIdx.x / S1_COLS;
  // SyncBN: every workgroup of this launch finishes 64 columns; its ticket's round trip
  // overlaps the row loads
  const bool xon = sa.xs.active();
  const int xbid = (int)(blockIdx.x + blockIdx.y * gridDim.x);
  unsigned long long tk = 0;
  if (xon && threadIdx.x == 0) tk = xgmi::xsite_ticket(sa.xs, xbid);
  const float* lvl1 = sa.part + (long long)bn * rows * (2 * BN) + c0 + col;
  float v[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const int r = rg + u * S1_RG;
    v[u] = lvl1[(long long)(r < rows ? r : 0) * (2 * BN)];
  }
  float a = 0.f;
#pragma unroll
  for (int u = 0; u < NL; ++u)
    if (rg + u * S1_RG < rows) a += v[u];
  part[rg][col] = a;
  if (xon && threadIdx.x == 0) ep_s = xgmi::xsite_epoch(sa.xs, tk, xbid);
  __syncthreads();
  if (xon) xgmi::xsite_advance(sa.xs, ep_s, xbid, S1_THR);
  if (threadIdx.x >= S1_COLS) return;
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < S1_RG; ++g) t += part[g][threadIdx.x];
  const int cc = c0 + threadIdx.x;  // column of [S1 | S2] (or [sum | sumsq])
  const int h = cc / BN, k = bn * BN + cc % BN;
  const bool cnt = !sa.bwd && bn == 0 && cc == 0;  // the lane that writes the row count
  float tg = t, mg = (float)M;
  if (xon) {  // local -> global (rank-ordered sums; the count too)
    const uint32_t ep = ep_s;
    xgmi::xsite_push_at(sa.xs, ep, h * K + k, t);
    if (cnt) xgmi::xsite_push_at(sa.xs, ep, 2 * K, mg);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned polls = 0;
    bool fail = false;
    tg = xgmi::xsite_pull_at(sa.xs, ep, h * K + k, t, t0, polls, fail);
    if (cnt) mg = xgmi::xsite_pull_at(sa.xs, ep, 2 * K, mg, t0, polls, fail);
  }
  if (sa.bwd) {  // dbeta / dgamma: this rank's sums (DDP averages them); out: global
    if (h == 0) {
      sa.dbeta[k] = t;
      sa.stats[k] = tg;
    } else {
      sa.dgamma[k] = t;
      sa.stats[K + k] = tg;
    }
    return;
  }
  sa.stats[h * K + k] = tg;
  if (h == 0) sa.stats[2 * K + SHIFT_OFF + k] = sa.shift[k];
  if (cnt) {
    sa.stats[2 * K] = mg;
    if (sa.nbt != nullptr) sa.nbt[0] = sa.nbt[0] + 1;
  }
  (void)nct;
}

template <int BN>
__global__ void __launch_bounds__(THR) stat_tree_kernel(StatArgs sa, long long M, int BM_, int K) {
  __shared__ float scr[THR];
  __shared__ float tot[2 * BN + 1];  // + the row count (SyncBN exchange)
  __shared__ int s_flag;
  const int nct = K / BN;
  const long long rows = (M + BM_ - 1) / BM_;
  const int NG = (int)((rows + G1 - 1) / G1);
  const int bn = (int)(blockIdx.x / NG), grp = (int)(blockIdx.x % NG);
  const int gsz = (int)min((long long)G1, rows - (long long)grp * G1);
  const int k0 = bn * BN, tid = threadIdx.x;
  float* lvl1 = sa.part + (long long)bn * rows * (2 * BN);
  float* lvl2 = sa.part + (long long)nct * rows * (2 * BN) + (long long)bn * NG * (2 * BN);
  sum_rows<2 * BN>(lvl1 + (long long)grp * G1 * (2 * BN), gsz, lvl2 + (long long)grp * (2 * BN), scr, true);
  if (!last_arriver(sa.tickets + nct * NG + bn, (unsigned)NG, &s_flag)) return;
  // SyncBN: the nct finishers exchange their slices (ticket round trip behind the level-2 loads)
  const bool xon = sa.xs.active();
  unsigned long long tk = 0;
  if (xon && tid == 0) tk = xgmi::xsite_ticket(sa.xs, bn);
  sum_rows<2 * BN>(lvl2, NG, tot, scr, false);
  if (sa.bwd) {  // BN backward sums: out = [S1 | S2], dbeta = S1, dgamma = S2 (bn_nhwc layout)
    for (int t = tid; t < BN; t += THR) {
      sa.dbeta[k0 + t] = tot[t];  // this rank's (DDP averages them)
      sa.dgamma[k0 + t] = tot[BN + t];
    }
    if (xon) xgmi::xsite_exchange_slice(sa.xs, tot, 2 * BN, [&](int i) { return i < BN ? k0 + i : K + k0 + i - BN; },
                                        tk, bn, THR);
    for (int t = tid; t < BN; t += THR) {
      sa.stats[k0 + t] = tot[t];
      sa.stats[K + k0 + t] = tot[BN + t];
    }
    return;
  }
  __shared__ float cnt[1];
  if (tid == 0) cnt[0] = (float)M;
  if (xon) {
    // the row count rides with finisher 0's slice (position 2K)
    const int n = 2 * BN + (bn == 0 ? 1 : 0);
    if (bn == 0 && tid == 0) tot[2 * BN] = cnt[0];
    xgmi::xsite_exchange_slice(sa.xs, tot, n, [&](int i) { return i < BN ? k0 + i : i < 2 * BN ? K + k0 + i - BN : 2 * K; },
                               tk, bn, THR);
    if (bn == 0 && tid == 0) cnt[0] = tot[2 * BN];
  }
  for (int t = tid; t < BN; t += THR) {
    sa.stats[k0 + t] = tot[t];
    sa.stats[K + k0 + t] = tot[BN + t];
    sa.stats[2 * K + SHIFT_OFF + k0 + t] = sa.shift[k0 + t];
  }
  if (bn == 0 && tid == 0) {
    sa.stats[2 * K] = cnt[0];
    if (sa.nbt != nullptr) sa.nbt[0] = sa.nbt[0] + 1;
  }
}

// ---------------------------------------------------------------------------
// Weight gradient:  dW[k][r][s][c] = sum_p dy[p][k] * x[n][oh*st+r-pad][ow*st+s-pad][c]
// GEMM M = Cout, N = R*S*C, reduction over the pixels p -- both operands are stored
// pixel-major, so they are staged in LDS as [64 pixels][cols] rows and read TRANSPOSED
// into the MFMA operands with ds_read_b64_tr_b16 (each 16-lane group: 4 pixel rows x
// 16 columns; two reads make a lane's 8 consecutive pixels).  Row chunks are XOR-
// swizzled by 2*f(row), f(row) = (row&3) | ((row>>1)&4): the 8 rows one 32-lane half
// reads map to 8 distinct chunk pairs (conflict-free with 16 chunks per row).
// Split over the pixels: S partial fp32 tiles -> wgrad_reduce_kernel, which also
// writes the fp32 OIHW gradient directly (no separate layout/cast pass).
typedef __attribute__((ext_vector_type(4))) short v4s;

// With 8 chunks per row (128-B rows: 64-channel tiles) one 32-lane half reads rows
// {0..3, 8..11} (+4, +32kk), the even ones in one bank half: their 4 chunk pairs must
// differ, so the XOR there is 2*f8(row), f8 = bit 1 | bit 3 of the row (was 2*(row&3):
// rows r and r+8 shared a pair, 2-way -- 1.6 conflict cycles per LDS instruction in the
// 64-wide wgrad kernels, profiles/r3s2l_resnet50_pmc_pass1.txt).
template <int CH>
__device__ __forceinline__ int wswz_xor(int row) {
  if constexpr (CH >= 16) return 2 * ((row & 3) | ((row >> 1) & 4));
  return 2 * (((row >> 1) & 1) | ((row >> 2) & 2));
}

template <int CH>  // 16-B chunks per LDS row
__device__ __forceinline__ int wswz(int row, int chunk) {
  return row * CH * 8 + ((chunk ^ wswz_xor<CH>(row)) << 3);
}

template <typename T, int BM, int BN, int MODE = MODE_GEN>
__global__ void __launch_bounds__(THR)
conv_wgrad_kernel(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ slab, Geom g, int splits,
                  long long pps) {
  typedef typename MM<T>::frag frag;
  constexpr int BP = 64;                 // pixels per K-step
  constexpr int CHA = BM / 8, CHB = BN / 8;
  constexpr int LA = BP * CHA / THR, LB = BP * CHB / THR;  // 16-B loads per thread
  constexpr int MT = BM / 32, NT = BN / 32;
  __shared__ __attribute__((aligned(16))) T lds[2][BP * (BM + BN)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int RSC = MODE == MODE_STEM ? 256 : g.R * g.S * g.C;  // stem: [8][8][4] padded columns
  const int tm = g.K / BM, tn = RSC / BN, tiles = tm * tn;
  const unsigned nwg = gridDim.x, hw = blockIdx.x;
  const unsigned q8 = nwg / 8, r8 = nwg % 8, xcd = hw % 8, slot = hw / 8;
  const unsigned lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int sp = (int)(lid / tiles), tile = (int)(lid % tiles);
  const int k0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int rs = n0 / g.C, c0 = n0 - rs * g.C, fr_ = rs / g.S, fs_ = rs - fr_ * g.S;
  const long long pa = sp * pps, pb = min(g.M, pa + pps);
  const int steps = (int)((pb - pa + BP - 1) / BP);
  f32x4 ra[LA], rb[LB];
  auto gload = [&](int t) {
    const long long pbase = pa + (long long)t * BP;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int e = i * THR + tid, row = e / CHA, cc = e % CHA;
      const long long p = pbase + row;
      ra[i] = p < pb ? *reinterpret_cast<const f32x4*>(dy + p * g.K + k0 + cc * 8) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int e = i * THR + tid, row = e / CHB, cc = e % CHB;
      const long long p = pbase + row;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < pb) {
        const unsigned pu = (unsigned)p, q = pu / (unsigned)g.OW;  // M < 2^31 (host check)
        const int ow = (int)(pu - q * (unsigned)g.OW);
        const unsigned n = q / (unsigned)g.OH;
        const int oh = (int)(q - n * (unsigned)g.OH);
        if constexpr (MODE == MODE_STEM) {
          // column n0 + 8cc: taps (r, s), (r, s + 1) of the [8][8][4] padded filter space
          const int col = n0 + cc * 8, r = col >> 5, s = (col >> 2) & 7;
          const int ih = oh * g.stride + r - g.pad, iw = ow * g.stride + s - g.pad;
          const bool rok = r < 7 && (unsigned)ih < (unsigned)g.H;
          const T* px_ = x + (((long long)n * g.H + ih) * g.W + iw) * 4;
          f32x2 lo = {0.f, 0.f}, hi = {0.f, 0.f};
          if (rok && (unsigned)iw < (unsigned)g.W) lo = *reinterpret_cast<const f32x2*>(px_);
          if (rok && s + 1 < 7 && (unsigned)(iw + 1) < (unsigned)g.W) hi = *reinterpret_cast<const f32x2*>(px_ + 4);
          v = f32x4{lo[0], lo[1], hi[0], hi[1]};
        } else {
          const int ih = oh * g.stride + fr_ - g.pad, iw = ow * g.stride + fs_ - g.pad;
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            v = *reinterpret_cast<const f32x4*>(x + (((long long)n * g.H + ih) * g.W + iw) * g.C + c0 + cc * 8);
        }
      }
      rb[i] = v;
    }
  };
  auto lstore = [&](int buf) {
    T* A = lds[buf];
    T* B = lds[buf] + BP * BM;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int e = i * THR + tid;
      *reinterpret_cast<f32x4*>(A + wswz<CHA>(e / CHA, e % CHA)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int e = i * THR + tid;
      *reinterpret_cast<f32x4*>(B + wswz<CHB>(e / CHB, e % CHB)) = rb[i];
    }
  };
  // transposed fragment: 8 consecutive pixel rows (32kk + 8g .. +7) of column cb + (lane & 15)
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pq = gi & 3;
  auto trfrag = [&](const T* base, int kk, int cb, auto chtag) -> frag {
    constexpr int CH = decltype(chtag)::value;
    const int row = 32 * kk + 8 * grp + q, col = cb + 4 * pq;
    const T* a0 = base + wswz<CH>(row, col >> 3) + (col & 7);
    const T* a1 = base + wswz<CH>(row + 4, col >> 3) + (col & 7);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a1);
    typedef __attribute__((ext_vector_type(8))) short v8s;
    const v8s v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag, v);
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (steps > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int t = 0; t < steps; ++t) {
    const int buf = t & 1;
    if (t + 1 < steps) gload(t + 1);
    const T* A = lds[buf];
    const T* B = lds[buf] + BP * BM;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag fa[MT], fb[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
        fa[a] = trfrag(A, kk, wm * (BM / 2) + a * 16, std::integral_constant<int, CHA>{});
#pragma unroll
      for (int b = 0; b < NT; ++b)
        fb[b] = trfrag(B, kk, wn * (BN / 2) + b * 16, std::integral_constant<int, CHB>{});
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = MM<T>::mma(fa[a], fb[b], acc[a][b]);
    }
    if (t + 1 < steps) lstore(buf ^ 1);
    __syncthreads();
  }
  // partial tile: C[m = k][n = (r,s,c)]; lane: col n = lane & 15, rows 4*(lane>>4) + j
  float* out = slab + (long long)sp * g.K * RSC;
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = k0 + wm * (BM / 2) + a * 16 + 4 * grp + j, n = n0 + wn * (BN / 2) + b * 16 + gi;
        out[(long long)m * RSC + n] = acc[a][b][j];
      }
}

// The same weight gradient with both operand tiles staged global -> LDS by LDS-DMA
// (MODE_GEN): no VGPR staging and no ds_write_b128 pass (the register-staged loop pays
// ~13 LDS cycles per KiB written).  A wave-instruction fills 64/CH whole rows of the
// [64 pixels][CH chunks] image, lane l row l / CH at slot l % CH; the wswz swizzle goes on
// the per-lane source address (logical chunk = slot ^ xor(row)); padding taps and pixels
// past the split's end read a 16-B zero page instead of being zero-filled by the loader.
// One barrier per 64-pixel step: wait the landed step (vmcnt(0)) + barrier, issue step
// t+1 into the other buffer, MFMA on step t (as conv_glds_kernel).

// NWM x NWN waves (default 2 x 2; 2 x 4 = 8 waves, DPA_WGRAD_WAVES=8: the second wave on
// every SIMD hides the other's transposed-read waits, as the forward's 8-wave tiles do).
// FIX (DPA_WGRAD_FIXUP_MAXSP, opt-in): the split-K reduction in this launch -- partial
// tiles stored write-through, one ticket per output tile, and the tile's last arriver sums
// the splits in split order and writes the fp32 OIHW gradient (no wgrad_reduce launch).
template <typename T, int BM, int BN, int NWM = 2, int NWN = 2, bool FIX = false>
__global__ void __launch_bounds__(64 * NWM * NWN)
conv_wgrad_glds_kernel(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ slab, Geom g,
                       int splits, long long pps, float* __restrict__ grad, unsigned* __restrict__ tickets) {
  typedef typename MM<T>::frag frag;
  constexpr int BP = 64;
  constexpr int CHA = BM / 8, CHB = BN / 8;
  constexpr int NW = NWM * NWN;
  constexpr int IA = CHA / NW, IB = CHB / NW;  // wave-instructions per wave per step
  constexpr int MT = BM / (16 * NWM), NT = BN / (16 * NWN);
  static_assert(IA >= 1 && IB >= 1 && IA * NW == CHA && IB * NW == CHB && MT >= 1 && NT >= 1, "tile / waves");
  constexpr int STAGE = BP * (BM + BN);
  __shared__ __attribute__((aligned(16))) T lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % NWM, wn = wave / NWM;
  const int RSC = g.R * g.S * g.C;
  const int tm = g.K / BM, tn = RSC / BN, tiles = tm * tn;
  const unsigned nwg = gridDim.x, hw = blockIdx.x;
  const unsigned q8 = nwg / 8, r8 = nwg % 8, xcd = hw % 8, slot = hw / 8;
  const unsigned lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int sp = (int)(lid / tiles), tile = (int)(lid % tiles);
  const int k0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int rs = n0 / g.C, c0 = n0 - rs * g.C, fr_ = rs / g.S, fs_ = rs - fr_ * g.S;
  const long long pa = sp * pps, pb = min(g.M, pa + pps);
  const int steps = (int)((pb - pa + BP - 1) / BP);
  const bool plain = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;  // x rows = pixels
  // this lane's rows and source chunks (row = (i*4 + wave) * (64/CH) + lane / CH)
  const int ra = lane / CHA, rb = lane / CHB;
  auto issue = [&](int t, int buf) {
    T* A = lds + buf * STAGE;
    T* B = A + BP * BM;
    const long long pbase = pa + (long long)t * BP;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int row = (i * NW + wave) * (64 / CHA) + ra;
      const int ck = (lane % CHA) ^ wswz_xor<CHA>(row);
      const long long p = pbase + row;
      const void* src = p < pb ? (const void*)(dy + p * g.K + k0 + ck * 8) : (const void*)g_zero16;
      glds16(src, A + (i * NW + wave) * (64 / CHA) * BM);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int row = (i * NW + wave) * (64 / CHB) + rb;
      const int ck = (lane % CHB) ^ wswz_xor<CHB>(row);
      const long long p = pbase + row;
      const void* src = g_zero16;
      if (p < pb) {
        if (plain) {
          src = x + p * g.C + c0 + ck * 8;
        } else {
          const unsigned pu = (unsigned)p, q = pu / (unsigned)g.OW;  // M < 2^31 (host check)
          const int ow = (int)(pu - q * (unsigned)g.OW);
          const unsigned n = q / (unsigned)g.OH;
          const int oh = (int)(q - n * (unsigned)g.OH);
          const int ih = oh * g.stride + fr_ - g.pad, iw = ow * g.stride + fs_ - g.pad;
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            src = x + (((long long)n * g.H + ih) * g.W + iw) * g.C + c0 + ck * 8;
        }
      }
      glds16(src, B + (i * NW + wave) * (64 / CHB) * BN);
    }
  };
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pq = gi & 3;
  auto trfrag = [&](const T* base, int kk, int cb, auto chtag) -> frag {
    constexpr int CH = decltype(chtag)::value;
    const int row = 32 * kk + 8 * grp + q, col = cb + 4 * pq;
    const T* a0 = base + wswz<CH>(row, col >> 3) + (col & 7);
    const T* a1 = base + wswz<CH>(row + 4, col >> 3) + (col & 7);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a1);
    typedef __attribute__((ext_vector_type(8))) short v8s;
    const v8s v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag, v);
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (steps > 0) issue(0, 0);
  for (int t = 0; t < steps; ++t) {
    const int buf = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < steps) issue(t + 1, buf ^ 1);
    const T* A = lds + buf * STAGE;
    const T* B = A + BP * BM;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag fa[MT], fb[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
        fa[a] = trfrag(A, kk, wm * (BM / NWM) + a * 16, std::integral_constant<int, CHA>{});
#pragma unroll
      for (int b = 0; b < NT; ++b)
        fb[b] = trfrag(B, kk, wn * (BN / NWN) + b * 16, std::integral_constant<int, CHB>{});
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = MM<T>::mma(fa[a], fb[b], acc[a][b]);
    }
  }
  float* out = slab + (long long)sp * g.K * RSC;
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = k0 + wm * (BM / NWM) + a * 16 + 4 * grp + j, n = n0 + wn * (BN / NWN) + b * 16 + gi;
        if constexpr (FIX) st_wt(out + (long long)m * RSC + n, acc[a][b][j]);
        else out[(long long)m * RSC + n] = acc[a][b][j];
      }
  if constexpr (FIX) {
    __shared__ int s_flag;
    // (last_arriver: this wave's write-through stores drained, one ticket per workgroup)
    if (!last_arriver(tickets + tile, (unsigned)splits, &s_flag)) return;
    // the tile's splits in split order, 8 loads in flight per lane; consecutive lanes take
    // consecutive columns (channels of one tap: unit-stride OIHW writes on a 1x1 conv)
    const long long plane = (long long)g.K * RSC;
    const int st = g.R * g.S;
    for (int e = tid; e < BM * BN; e += 64 * NW) {
      const int r = e / BN, cn = e - r * BN;
      const long long off = (long long)(k0 + r) * RSC + n0 + cn;
      float t = 0.f;
      int s0 = 0;
      for (; s0 + 8 <= splits; s0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld_wt(slab + (s0 + u) * plane + off);
#pragma unroll
        for (int u = 0; u < 8; ++u) t += v[u];
      }
      for (; s0 < splits; ++s0) t += ld_wt(slab + s0 * plane + off);
      const int n = n0 + cn, c = n % g.C, rs = n / g.C;  // (r*S + s)*C + c
      grad[((long long)(k0 + r) * g.C + c) * st + rs] = t;
    }
  }
}

constexpr int WR_QC = 16;  // float4 columns per wgrad_reduce_kernel workgroup

// grad[k][c][r][s] (fp32 OIHW) = sum over splits of slab[sp][k][(r*S + s)*C + c]:
// a workgroup owns 64 consecutive slab columns as 16 float4 quads x 16 split groups
// (every 4th split, fixed order, 4 loads in flight), combined through LDS in group
// order, written in the OIHW order of a [K][Cd][Rd][Sd] gradient (Cd <= C, Rd <= R,
// Sd <= S: the stem's padded columns are dropped here).
__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ grad, int splits, int K, int C, int R, int S,
                    int Cd, int Rd, int Sd) {
  // 16 float4 columns x 16 split groups per workgroup (was 64 x 4: a grid of ~150
  // workgroups whose lanes each waited ~6 dependent rounds of 4 loads)
  constexpr int QC = WR_QC, SG = 256 / WR_QC;
  __shared__ f32x4 part[SG][QC];
  const long long RSC = (long long)R * S * C, total = (long long)K * RSC;
  const int qd = threadIdx.x % QC, rg = threadIdx.x / QC;
  const long long col = (blockIdx.x * (long long)QC + qd) * 4;  // total % 4 == 0 (C % 64 == 0)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (col < total) {
    int sp = rg;
    for (; sp + 3 * SG < splits; sp += 4 * SG) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(slab + (long long)sp * total + col);
      const f32x4 b = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + SG) * total + col);
      const f32x4 c = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + 2 * SG) * total + col);
      const f32x4 d = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + 3 * SG) * total + col);
      acc += a;
      acc += b;
      acc += c;
      acc += d;
    }
    for (; sp < splits; sp += SG) acc += *reinterpret_cast<const f32x4*>(slab + (long long)sp * total + col);
  }
  part[rg][qd] = acc;
  __syncthreads();
  if (rg == 0 && col < total) {
    f32x4 t = part[0][qd];
#pragma unroll
    for (int gg = 1; gg < SG; ++gg) t += part[gg][qd];
    const int k = (int)(col / RSC);
    const long long n = col - (long long)k * RSC;  // (r*S + s)*C + c, c % 4 == 0
    const int c = (int)(n % C), rs = (int)(n / C), r = rs / S, s = rs - r * S;
    if (r < Rd && s < Sd) {
      float* o = grad + (((long long)k * Cd + c) * Rd + r) * Sd + s;
      const int st = Rd * Sd;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < Cd) o[j * st] = t[j];
    }
  }
}

// The same reduction for a whole backward pass's weight gradients in ONE launch
// (ops/conv_igemm.WgradBatch): every conv left its split partials in a slab of its own, and
// at the end of the backward one grid covers all of them -- instead of one small, tail-bound
// launch per conv (53 launches, ~9 us each on ResNet-50: profiles/r5a_rn_steady.txt).  The
// entries ride in the kernel arguments by value (graph-capturable, no table upload); a
// workgroup finds its entry by its block index (prefix blk0).  Same per-block association
// as wgrad_reduce_kernel: bitwise the same gradients.
constexpr int WB_MAX = 48;
struct WBEntry {
  const float* slab;
  float* grad;
  int splits, K, C, R, S, Cd, Rd, Sd;
  long long blk0;  // first block of this entry
};
struct WBList {
  int n;
  WBEntry e[WB_MAX];
};

__global__ void __launch_bounds__(256) wgrad_reduce_batch_kernel(WBList L) {
  constexpr int QC = WR_QC, SG = 256 / WR_QC;
  __shared__ f32x4 part[SG][QC];
  const long long b = blockIdx.x;
  int lo = 0, hi = L.n - 1;  // the entry holding block b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.e[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const WBEntry& E = L.e[lo];
  const float* __restrict__ slab = E.slab;
  const int splits = E.splits, C = E.C, S = E.S, Cd = E.Cd, Rd = E.Rd, Sd = E.Sd;
  const long long RSC = (long long)E.R * S * C, total = (long long)E.K * RSC;
  const int qd = threadIdx.x % QC, rg = threadIdx.x / QC;
  const long long col = ((b - E.blk0) * QC + qd) * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (col < total) {
    int sp = rg;
    for (; sp + 3 * SG < splits; sp += 4 * SG) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(slab + (long long)sp * total + col);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + SG) * total + col);
      const f32x4 v2 = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + 2 * SG) * total + col);
      const f32x4 v3 = *reinterpret_cast<const f32x4*>(slab + (long long)(sp + 3 * SG) * total + col);
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; sp < splits; sp += SG) acc += *reinterpret_cast<const f32x4*>(slab + (long long)sp * total + col);
  }
  part[rg][qd] = acc;
  __syncthreads();
  if (rg == 0 && col < total) {
    f32x4 t = part[0][qd];
#pragma unroll
    for (int gg = 1; gg < SG; ++gg) t += part[gg][qd];
    const int k = (int)(col / RSC);
    const long long n = col - (long long)k * RSC;
    const int c = (int)(n % C), rs = (int)(n / C), r = rs / S, s_ = rs - r * S;
    if (r < Rd && s_ < Sd) {
      float* o = E.grad + (((long long)k * Cd + c) * Rd + r) * Sd + s_;
      const int st = Rd * Sd;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < Cd) o[j * st] = t[j];
    }
  }
}

// ---------------------------------------------------------------------------
// Per-step weight packing for every implicit-GEMM conv of a network in ONE launch:
// fp32 OIHW master weights -> the compute-dtype forward filter wf[k][r][s][c] (the
// channels_last layout the kernels read) and, where a data gradient runs on the
// kernel, the flipped transposed filter wd[c][R-1-r][S-1-s][k] (for a 1x1 conv: the
// plain transpose).  64 x 64 (k, c) tiles of one tap through LDS: both writes are
// whole 128-B rows.  Table (int64, 8 per conv): src, wf, wd (0: none), K, C, R*S,
// first tile (prefix over the convs), unused.
template <typename T>
__global__ void __launch_bounds__(256)
pack_weights_kernel(const int64_t* __restrict__ table, int n) {
  __shared__ float tile[64][65];
  const long long t = blockIdx.x;
  int lo = 0, hi = n - 1;  // the conv holding tile t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[8 * mid + 6] <= t) lo = mid; else hi = mid - 1;
  }
  const int64_t* d = table + 8 * lo;
  const float* src = reinterpret_cast<const float*>(d[0]);
  T* wf = reinterpret_cast<T*>(d[1]);
  T* wd = reinterpret_cast<T*>(d[2]);
  const int K = (int)d[3], C = (int)d[4], RS = (int)d[5];
  const long long lt = t - d[6];
  const int rs = (int)(lt % RS);
  const long long kc = lt / RS;
  const int ct = C / 64, k0 = (int)(kc / ct) * 64, c0 = (int)(kc % ct) * 64;
  const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = src[((long long)(k0 + rg * 16 + i) * C + c0 + cl) * RS + rs];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int kl = rg * 16 + i;
    wf[((long long)(k0 + kl) * RS + rs) * C + c0 + cl] = Cvt<T>::from_f(v[i]);
    tile[kl][cl] = v[i];
  }
  if (wd == nullptr) return;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = rg * 16 + i;  // lanes along k
    wd[((long long)(c0 + c) * RS + (RS - 1 - rs)) * K + k0 + cl] = Cvt<T>::from_f(tile[cl][c]);
  }
}

// Stem operands in one launch: the [N][3][H][W] image (fp32 or the compute dtype)
// -> the 4-channel NHWC image [N][H][W][4] (one 8-B store per pixel, 4th channel 0),
// and, in the trailing workgroups, the fp32 [K][3][7][7] filter -> [K][8][8][4] in the
// compute dtype with zeros in the padding (the MODE_STEM K space).
template <typename T, typename S>
__global__ void __launch_bounds__(256)
stem_pack_kernel(const S* __restrict__ x, T* __restrict__ x4, long long npix, int HW, const float* __restrict__ w,
                 T* __restrict__ w4, int K, long long xblocks) {
  if ((long long)blockIdx.x < xblocks) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    const long long n = p / HW, hw = p - n * HW;
    const S* src = x + n * 3 * HW + hw;
    T v[4] = {Cvt<T>::from_f(Cvt<S>::to_f(src[0])), Cvt<T>::from_f(Cvt<S>::to_f(src[HW])),
              Cvt<T>::from_f(Cvt<S>::to_f(src[2 * HW])), Cvt<T>::from_f(0.f)};
    *reinterpret_cast<u16x4*>(x4 + p * 4) = *reinterpret_cast<const u16x4*>(v);
    return;
  }
  const int e = (int)((long long)blockIdx.x - xblocks) * 256 + threadIdx.x;
  if (e >= K * 256) return;
  const int k = e >> 8, rem = e & 255, r = rem >> 5, s = (rem >> 2) & 7, c = rem & 3;
  w4[e] = Cvt<T>::from_f(r < 7 && s < 7 && c < 3 ? w[((k * 3 + c) * 7 + r) * 7 + s] : 0.f);
}

// x: [N, 3, H, W] contiguous (fp32 / bf16 / f16); w: fp32 [K, 3, 7, 7]; x4: [N, 4, H, W]
// channels_last, w4: [K, 4, 8, 8] channels_last, both in the compute dtype.
void stem_pack(at::Tensor x, at::Tensor w, at::Tensor x4, at::Tensor w4) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 && x.size(1) == 3, "stem_pack: x [N, 3, H, W]");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.size(1) == 3 && w.size(2) == 7 &&
                  w.size(3) == 7, "stem_pack: fp32 [K, 3, 7, 7] filter");
  TORCH_CHECK(x4.is_contiguous(at::MemoryFormat::ChannelsLast) && x4.size(0) == x.size(0) && x4.size(1) == 4 &&
                  x4.size(2) == x.size(2) && x4.size(3) == x.size(3), "stem_pack: x4 [N, 4, H, W] channels_last");
  TORCH_CHECK(w4.is_contiguous(at::MemoryFormat::ChannelsLast) && w4.size(0) == w.size(0) && w4.size(1) == 4 &&
                  w4.size(2) == 8 && w4.size(3) == 8 && w4.scalar_type() == x4.scalar_type(), "stem_pack: w4");
  TORCH_CHECK(x4.scalar_type() == at::kBFloat16 || x4.scalar_type() == at::kHalf, "stem_pack: bf16 / f16");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == x4.scalar_type(), "stem_pack: x dtype");
  const long long HW = x.size(2) * x.size(3), npix = x.size(0) * HW;
  const int K = (int)w.size(0);
  const long long xblocks = (npix + 255) / 256, wblocks = ((long long)K * 256 + 255) / 256;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    T* x4p = reinterpret_cast<T*>(x4.data_ptr());
    T* w4p = reinterpret_cast<T*>(w4.data_ptr());
    if (x.scalar_type() == at::kFloat)
      hipLaunchKernelGGL((stem_pack_kernel<T, float>), dim3((unsigned)(xblocks + wblocks)), dim3(256), 0,
                         cur_stream(), x.data_ptr<float>(), x4p, npix, (int)HW, w.data_ptr<float>(), w4p, K, xblocks);
    else
      hipLaunchKernelGGL((stem_pack_kernel<T, T>), dim3((unsigned)(xblocks + wblocks)), dim3(256), 0, cur_stream(),
                         reinterpret_cast<const T*>(x.data_ptr()), x4p, npix, (int)HW, w.data_ptr<float>(), w4p, K,
                         xblocks);
  };
  if (x4.scalar_type() == at::kBFloat16) launch(__hip_bfloat16{}); else launch(__half{});
  DPA_CHECK_LAUNCH();
}

void pack_weights(at::Tensor table, int64_t n, int64_t tiles, int64_t dtype_code) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.numel() >= 8 * n, "pack_weights: table");
  if (tiles <= 0) return;
  if (dtype_code == 0)
    hipLaunchKernelGGL(pack_weights_kernel<__hip_bfloat16>, dim3((unsigned)tiles), dim3(256), 0, cur_stream(),
                       table.data_ptr<int64_t>(), (int)n);
  else
    hipLaunchKernelGGL(pack_weights_kernel<__half>, dim3((unsigned)tiles), dim3(256), 0, cur_stream(),
                       table.data_ptr<int64_t>(), (int)n);
  DPA_CHECK_LAUNCH();
}

static Geom geom(const at::Tensor& x, const at::Tensor& w, int stride, int pad) {
  // x: [N, C, H, W] channels_last; w: [K, C, R, S] channels_last (= [K][R][S][C] in memory)
  Geom g;
  g.N = (int)x.size(0); g.C = (int)x.size(1); g.H = (int)x.size(2); g.W = (int)x.size(3);
  g.K = (int)w.size(0); g.R = (int)w.size(2); g.S = (int)w.size(3);
  g.stride = stride; g.pad = pad;
  g.OH = (g.H + 2 * pad - g.R) / stride + 1;
  g.OW = (g.W + 2 * pad - g.S) / stride + 1;
  g.M = (long long)g.N * g.OH * g.OW;
  return g;
}

bool supported(int64_t C, int64_t K) { return C % BK == 0 && K % 64 == 0; }

static int tile_n(int64_t K) { return K % 128 == 0 ? 128 : 64; }

// 1x1 convs on conv_glds_kernel (DPA_G1X1=0: the general kernel, A/B runs; g1x1_config
// switches both at run time for tests and sweeps)
static int g_g1x1_on = -1, g_g1x1_bp = -1;
static long long g_g1x1_min256 = -1;

static void g1x1_init() {
  if (g_g1x1_on >= 0) return;
  const char* e = std::getenv("DPA_G1X1");
  g_g1x1_on = (e == nullptr || e[0] != '0') ? 1 : 0;
  const char* b = std::getenv("DPA_G1X1_BP");
  g_g1x1_bp = b != nullptr ? std::atoi(b) : 0;
  const char* m = std::getenv("DPA_G1X1_MIN256");
  g_g1x1_min256 = m != nullptr ? std::atoll(m) : (1LL << 40);  // 256-pixel tiles measured slower: off
}

static bool g1x1_enabled() {
  g1x1_init();
  return g_g1x1_on != 0;
}

// LDS buffers of conv_glds_kernel (forward / plain data gradients): 2 (default) or 3
// (DPA_GLDS_STAGES=3; glds_config(stages) at run time)
static int g_glds_stages = -1;
static int glds_stages() {
  if (g_glds_stages < 0) {
    const char* e = std::getenv("DPA_GLDS_STAGES");
    g_glds_stages = e != nullptr && (std::atoi(e) == 3 || std::atoi(e) == 4) ? std::atoi(e) : 2;
  }
  return g_glds_stages;
}
int64_t glds_config(int64_t stages) {
  glds_stages();
  const int64_t prev = g_glds_stages;
  if (stages >= 2 && stages <= 4) g_glds_stages = (int)stages;
  return prev;
}

// 128-channel tiles of conv_glds_kernel narrowed to 64 when the grid would have fewer than
// this many workgroups (DPA_G1X1_BN64_BELOW; 0 = never; bn64_config at run time)
static long long g_bn64_below = -1;
static long long bn64_below() {
  if (g_bn64_below < 0) {
    const char* e = std::getenv("DPA_G1X1_BN64_BELOW");
    g_bn64_below = e != nullptr ? std::atoll(e) : 0LL;
  }
  return g_bn64_below;
}
int64_t bn64_config(int64_t below) {
  bn64_below();
  const int64_t prev = g_bn64_below;
  if (below >= 0) g_bn64_below = below;
  return prev;
}

// KxK convs (any stride / padding) on the glds kernel too (DPA_G3X3=0: 1x1 only, A/B runs)
static int g_g3x3_on = -1;
static bool g3x3_enabled() {
  if (g_g3x3_on < 0) {
    const char* e = std::getenv("DPA_G3X3");
    g_g3x3_on = (e == nullptr || e[0] != '0') ? 1 : 0;
  }
  return g_g3x3_on != 0;
}
int64_t g3x3_config(int64_t on) {
  g3x3_enabled();
  const int64_t prev = g_g3x3_on;
  if (on >= 0) g_g3x3_on = on ? 1 : 0;
  return prev;
}

// Measured and not kept (profiles/r5j_wide_ns_ab.txt): the 8-wave 128 x 128 tile with three or
// four LDS stages (two / three tiles in flight, one workgroup per CU) -- no faster even where
// the grid is one workgroup per CU anyway (512 -> 512 3x3 at 7x7: 56.1 vs 57.9 / 58.1 us),
// 23 % slower over the network: the K-loop does not wait on DMA latency (PMC,
// profiles/r5i_conv_pmc.txt: MFMA busy 27-32 %, waits at the barrier / LDS-read counters).
// Wide 8-wave tiles of conv_glds_kernel for the forward / plain data-gradient convs
// (DPA_WIDE; wide_config at run time): 0 off, 1 auto (see wide_pick), 2 force 256 x 128,
// 3 force 256 x 256, 4 force 128 x 128 on 8 waves.  Shapes a forced tile does not fit keep
// the 4-wave kernel.
static int g_wide = -1;
static int wide_mode() {
  if (g_wide < 0) {
    const char* e = std::getenv("DPA_WIDE");
    g_wide = e != nullptr ? std::atoi(e) : 1;
  }
  return g_wide;
}
int64_t wide_config(int64_t m) {
  wide_mode();
  const int64_t prev = g_wide;
  if (m >= 0) g_wide = (int)m;
  return prev;
}
// -> 0 (the 4-wave 128 x 128 / x 64 tiles), 1 (256 x 128), 2 (256 x 256), 3 (128 x 128, 8 waves).
// Auto (profiles/r5c_wide_ab.txt, every ResNet-50 forward shape): 8 waves on the 128 x 128
// tile wherever Cout % 128 == 0 (the second wave on each SIMD hides the other's fragment-read
// waits: network forward convs 2459 -> 2380 us); 256 x 256 where the reduction is deep
// (C R S >= 1024) and the grid still fills the chip (>= 196 workgroups: 40.5 vs 42.9-44.3 us
// on 1024 -> 512 at 14x14).  bs: BN backward sums in the epilogue (128-pixel tiles only).
static int wide_pick(long long M, int64_t K, int64_t CRS, bool bs) {
  const int m = wide_mode();
  const long long r256 = (M + 255) / 256;
  const bool ok2 = !bs && K % 256 == 0 && r256 <= S1_MAXROWS;  // the deferred tree: one level at BN = 256
  const bool ok1 = K % 128 == 0;
  if (m == 2) return ok1 && !bs ? 1 : 0;
  if (m == 3) return ok2 ? 2 : 0;
  if (m == 4) return ok1 ? 3 : 0;
  if (m != 1) return 0;
  if (ok2 && CRS >= 1024 && r256 * (K / 256) >= 196) return 2;
  return ok1 ? 3 : 0;
}

// pixel tile of conv_glds_kernel: 256 when the grid still has >= min256 workgroups (default
// 2 per CU: the 96 KB of LDS leave one 256-pixel workgroup per CU), else 128 (64 KB: two
// per CU); DPA_G1X1_BP=128|256 forces one.
static int g1x1_bp(long long M, int64_t K) {
  g1x1_init();
  if (g_g1x1_bp == 128 || g_g1x1_bp == 256) return g_g1x1_bp;
  const long long t256 = (M + 255) / 256 * (K / tile_n(K));
  return t256 >= g_g1x1_min256 ? 256 : 128;
}

// deferred statistics tree (StatArgs.defer + stat_tree_kernel) for grids of more than
// g_defer_min workgroups (several rounds per CU: the in-launch hand-off is then paid
// serially by every round); DPA_STAT_DEFER_MIN overrides, 0 = always, -1 = never
static long long g_defer_min = -2;
static bool defer_stats(long long blocks) {
  if (g_defer_min == -2) {
    const char* e = std::getenv("DPA_STAT_DEFER_MIN");
    g_defer_min = e != nullptr ? std::atoll(e) : 0LL;  // always: measured 14.73 vs 14.77-14.84 ms (1024)
  }
  return g_defer_min >= 0 && blocks > g_defer_min;
}
int64_t stat_defer_config(int64_t min_blocks) {
  defer_stats(0);
  const int64_t prev = g_defer_min;
  if (min_blocks >= -1) g_defer_min = min_blocks;
  return prev;
}

static void launch_stat_tree(StatArgs sa, long long M, int bm, int K, int BN) {
  const long long rows = (M + bm - 1) / bm, NG = (rows + G1 - 1) / G1;
  if (rows <= S1_MAXROWS) {  // one level: every row in flight at once, no ticket
    const dim3 gr((unsigned)(K / BN), (unsigned)(2 * BN / S1_COLS)), th(S1_THR);
    xgmi::set_site_grid(sa.xs, (long long)gr.x * gr.y, "stat_sum1");  // SyncBN finishers: every workgroup
    if (rows <= 16 * S1_RG) {
      if (BN == 256) hipLaunchKernelGGL((stat_sum1_kernel<256, 16>), gr, th, 0, cur_stream(), sa, M, bm, K);
      else if (BN == 128) hipLaunchKernelGGL((stat_sum1_kernel<128, 16>), gr, th, 0, cur_stream(), sa, M, bm, K);
      else hipLaunchKernelGGL((stat_sum1_kernel<64, 16>), gr, th, 0, cur_stream(), sa, M, bm, K);
    } else {
      if (BN == 256) hipLaunchKernelGGL((stat_sum1_kernel<256, S1_MAXROWS / S1_RG>), gr, th, 0, cur_stream(), sa, M, bm, K);
      else if (BN == 128) hipLaunchKernelGGL((stat_sum1_kernel<128, S1_MAXROWS / S1_RG>), gr, th, 0, cur_stream(), sa, M, bm, K);
      else hipLaunchKernelGGL((stat_sum1_kernel<64, S1_MAXROWS / S1_RG>), gr, th, 0, cur_stream(), sa, M, bm, K);
    }
    DPA_CHECK_LAUNCH();
    return;
  }
  TORCH_CHECK(BN <= 128, "stat_tree: 256-channel tiles need <= ", S1_MAXROWS, " pixel tiles");
  const dim3 gr((unsigned)(NG * (K / BN))), th(THR);
  xgmi::set_site_grid(sa.xs, K / BN, "stat_tree");  // SyncBN finishers: the last arriver of each channel tile
  if (BN == 128) hipLaunchKernelGGL(stat_tree_kernel<128>, gr, th, 0, cur_stream(), sa, M, bm, K);
  else hipLaunchKernelGGL(stat_tree_kernel<64>, gr, th, 0, cur_stream(), sa, M, bm, K);
  DPA_CHECK_LAUNCH();
}

// (on, bp, min256) -> previous; a negative argument leaves that setting alone
std::vector<int64_t> g1x1_config(int64_t on, int64_t bp, int64_t min256) {
  g1x1_init();
  std::vector<int64_t> prev{g_g1x1_on, g_g1x1_bp, g_g1x1_min256};
  if (on >= 0) g_g1x1_on = on ? 1 : 0;
  if (bp >= 0) g_g1x1_bp = (int)bp;
  if (min256 >= 0) g_g1x1_min256 = min256;
  return prev;
}

// statistics workspace: level-1 + level-2 partial rows (floats) and tickets (int32)
int64_t stat_part_len(int64_t M, int64_t K) {
  const int64_t rows = (M + BM - 1) / BM, ng = (rows + G1 - 1) / G1;
  return 2 * K * (rows + ng);
}
int64_t stat_tickets_len(int64_t M, int64_t K) {
  const int64_t rows = (M + BM - 1) / BM, ng = (rows + G1 - 1) / G1;
  return (K / 64) * (ng + 1);  // 64-channel tiles at most (conv_glds_kernel may narrow 128 -> 64)
}

// y: [N, K, OH, OW] channels_last (preallocated).  With `stats` (fp32 [3K+4], the
// bn_nhwc layout), also part / tickets (stat_part_len / stat_tickets_len; tickets
// zero-initialised once), shift (running mean) and nbt: the fused BN statistics.
//
// mode MODE_STEM: x = the stem_pack image [N, 4, H, W], w = [K, 4, 8, 8] (stride 2, pad 3,
// a 7x7 filter); mode MODE_S2T: x = dy [N, Cf, OHf, OWf] of a 3x3 / stride-2 / pad-1 conv,
// w = its flipped transposed filter [Cin, Cf, 3, 3], y = dx [N, Cin, 2 OHf, 2 OWf].
// aux (MODE_GEN, channels_last [N, K, OH/2, OW/2]): added at the even output pixels --
// a stride-2 1x1 conv's data gradient folded into this one's output.
//
// bn_x (1x1, stride 1, on conv_glds_kernel): y is the output gradient of a training BatchNorm
// whose input was bn_x; the epilogue also produces that BN's backward sums (bn_nhwc
// bwd_stats: bn_out = [S1 | S2], bn_dbeta = S1, bn_dgamma = S2) -- bn_y given: the ReLU
// mask comes from the BN's output (and y accumulates onto the tapped residual gradient,
// accumulate = true); else it is recomputed from bn_x with bn_gamma / bn_beta.  bn_save =
// the forward's [mean | invstd]; part / tickets = the statistics workspace.
void conv_fwd(at::Tensor x, at::Tensor w, at::Tensor y, int64_t stride, int64_t pad, c10::optional<at::Tensor> part,
              c10::optional<at::Tensor> tickets, c10::optional<at::Tensor> stats, c10::optional<at::Tensor> shift,
              c10::optional<at::Tensor> nbt, bool accumulate, int64_t mode, c10::optional<at::Tensor> aux,
              c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_y, c10::optional<at::Tensor> bn_save,
              c10::optional<at::Tensor> bn_gamma, c10::optional<at::Tensor> bn_beta,
              c10::optional<at::Tensor> bn_out, c10::optional<at::Tensor> bn_dgamma,
              c10::optional<at::Tensor> bn_dbeta, std::shared_ptr<xgmi::XgmiComm> xc) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && y.is_cuda(), "conv_fwd: device tensors");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && x.scalar_type() == y.scalar_type(), "conv_fwd: one dtype");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "conv_fwd: bf16 / f16");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd: channels_last x / w / y");
  Geom g = geom(x, w, (int)stride, (int)pad);
  g.accumulate = accumulate ? 1 : 0;
  TORCH_CHECK(mode == MODE_GEN || mode == MODE_STEM || mode == MODE_S2T, "conv_fwd: mode");
  if (mode == MODE_STEM) {
    TORCH_CHECK(g.C == 4 && w.size(1) == 4 && g.R == 8 && g.S == 8 && stride == 2 && pad == 3 && g.K % 64 == 0,
                "conv_fwd: stem needs the stem_pack operands (x [N,4,H,W], w [K,4,8,8]), stride 2, pad 3");
    g.R = g.S = 7;
    g.OH = (g.H + 2 * g.pad - 7) / 2 + 1;
    g.OW = (g.W + 2 * g.pad - 7) / 2 + 1;
    g.M = (long long)g.N * g.OH * g.OW;
  } else {
    TORCH_CHECK(w.size(1) == g.C && supported(g.C, g.K), "conv_fwd: needs C % 64 == 0 and Cout % 64 == 0");
  }
  if (mode == MODE_S2T) {
    TORCH_CHECK(g.R == 3 && g.S == 3 && stride == 2 && pad == 1, "conv_fwd: the S2T mode is a 3x3/s2/p1 dgrad");
    g.OH = g.H;
    g.OW = g.W;
    g.M = (long long)g.N * g.OH * g.OW;
    g.cls_rows = (g.M + BM - 1) / BM;
    TORCH_CHECK(y.size(0) == g.N && y.size(1) == g.K && y.size(2) == 2 * g.OH && y.size(3) == 2 * g.OW,
                "conv_fwd: S2T dx must be [N, Cin, 2 OHf, 2 OWf]");
    TORCH_CHECK(!stats.has_value() && !aux.has_value(), "conv_fwd: S2T has no statistics / aux");
  } else {
    TORCH_CHECK(y.size(0) == g.N && y.size(1) == g.K && y.size(2) == g.OH && y.size(3) == g.OW, "conv_fwd: y shape");
  }
  if (aux.has_value()) {
    TORCH_CHECK(mode == MODE_GEN && g.OH % 2 == 0 && g.OW % 2 == 0 && aux->scalar_type() == y.scalar_type() &&
                    aux->is_contiguous(at::MemoryFormat::ChannelsLast) && aux->size(0) == g.N &&
                    aux->size(1) == g.K && aux->size(2) == g.OH / 2 && aux->size(3) == g.OW / 2,
                "conv_fwd: aux must be [N, K, OH/2, OW/2] channels_last in y's dtype");
    g.aux = aux->data_ptr();
  }
  const bool st = stats.has_value();
  const bool bwdst = bn_x.has_value();
  TORCH_CHECK(!(st && accumulate), "conv_fwd: statistics of an accumulated output are not supported");
  if (bwdst) {
    TORCH_CHECK(mode == MODE_GEN && g.stride == 1 && g1x1_enabled() && x.numel() < (1LL << 31) &&
                    w.numel() < (1LL << 31) && ((g.R == 1 && g.S == 1 && g.pad == 0) || g3x3_enabled()),
                "conv_fwd: BN backward sums need the LDS-DMA kernel (stride 1)");
    TORCH_CHECK(bn_y.has_value() || !accumulate, "conv_fwd: recomputed-mask BN sums on an accumulated output");
    TORCH_CHECK(!st && !aux.has_value() && part.has_value() && tickets.has_value(),
                "conv_fwd: BN backward sums take part / tickets and no forward statistics / aux");
    TORCH_CHECK(accumulate == bn_y.has_value(), "conv_fwd: bn_y (ReLU after a residual) goes with accumulate");
    TORCH_CHECK(bn_save.has_value() && bn_out.has_value() && bn_dgamma.has_value() && bn_dbeta.has_value() &&
                    (bn_y.has_value() || (bn_gamma.has_value() && bn_beta.has_value())),
                "conv_fwd: BN backward sums need save / out / dgamma / dbeta (+ gamma / beta to recompute)");
    auto rows_like_y = [&](const at::Tensor& t) {
      return t.scalar_type() == y.scalar_type() && t.is_contiguous(at::MemoryFormat::ChannelsLast) &&
             t.sizes() == y.sizes();
    };
    TORCH_CHECK(rows_like_y(*bn_x) && (!bn_y.has_value() || rows_like_y(*bn_y)), "conv_fwd: bn_x / bn_y like y");
    for (const at::Tensor* t : {&*bn_save, &*bn_out})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() >= 2 * g.K, "conv_fwd: bn f32");
    for (const at::Tensor* t : {&*bn_dgamma, &*bn_dbeta})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == g.K, "conv_fwd: bn dgamma / dbeta");
    if (!bn_y.has_value())
      TORCH_CHECK(bn_gamma->scalar_type() == at::kFloat && bn_gamma->numel() == g.K && bn_beta->numel() == g.K,
                  "conv_fwd: bn gamma / beta");
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->numel() >= stat_part_len(g.M, g.K) &&
                    tickets->scalar_type() == at::kInt && tickets->numel() >= stat_tickets_len(g.M, g.K),
                "conv_fwd: statistics workspace");
  }
  TORCH_CHECK(st == shift.has_value() && (bwdst || (st == part.has_value() && st == tickets.has_value())),
              "conv_fwd: part, tickets, stats and shift go together");
  StatArgs sa{nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  if (st) {
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->numel() >= stat_part_len(g.M, g.K), "conv_fwd: part size");
    TORCH_CHECK(tickets->scalar_type() == at::kInt && tickets->numel() >= stat_tickets_len(g.M, g.K),
                "conv_fwd: tickets size");
    TORCH_CHECK(stats->scalar_type() == at::kFloat && stats->numel() >= 3 * g.K + 4, "conv_fwd: stats size");
    TORCH_CHECK(shift->scalar_type() == at::kFloat && shift->numel() == g.K, "conv_fwd: shift size");
    sa.part = part->data_ptr<float>();
    sa.tickets = reinterpret_cast<unsigned*>(tickets->data_ptr<int>());
    sa.stats = stats->data_ptr<float>();
    sa.shift = shift->data_ptr<float>();
    sa.nbt = nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr;
  }
  // SyncBN inside the statistics finishers: they run in the deferred tree launch
  if (xc) {
    TORCH_CHECK(st || bwdst, "conv_fwd: xc (SyncBN site) goes with statistics");
    TORCH_CHECK(2 * g.K + 1 <= xgmi::kWideVals, "conv_fwd: SyncBN site row holds 2K+1 <= ", xgmi::kWideVals);
    sa.xs = xc->wide_site();
  }
  const int BN0 = tile_n(g.K);
  if (mode == MODE_GEN && g1x1_enabled() && x.numel() < (1LL << 31) && w.numel() < (1LL << 31) &&
      (g3x3_enabled() || (g.R == 1 && g.S == 1 && g.pad == 0))) {
    // the glds-staged implicit-GEMM kernel (pixel tile 256 or 128, see g1x1_bp; 64-channel
    // tiles when 128-channel ones leave the grid below g_bn64_below workgroups)
    const int wide = wide_pick(g.M, g.K, (int64_t)g.C * g.R * g.S, bwdst);
    int BP = (bwdst || !(g.R == 1 && g.S == 1 && g.pad == 0)) ? 128 : g1x1_bp(g.M, g.K);
    int BN = BN0 == 128 && BP == 128 && (g.M + 127) / 128 * (g.K / 128) < bn64_below() ? 64 : BN0;
    if (wide == 1 || wide == 2) BP = 256;
    if (wide == 1 || wide == 3) BN = 128;
    if (wide == 2) BN = 256;
    if (wide == 3) BP = 128;
    const long long blocks = (g.M + BP - 1) / BP * (g.K / BN);
    TORCH_CHECK(blocks < (1LL << 31), "conv_fwd: grid too large");
    sa.defer = st && (defer_stats(blocks) || xc || wide) ? 1 : 0;
    if (bwdst) {  // the BN backward sums: level-1 rows in the conv, the tree after it
      sa.part = part->data_ptr<float>();
      sa.tickets = reinterpret_cast<unsigned*>(tickets->data_ptr<int>());
      sa.stats = bn_out->data_ptr<float>();
      sa.dgamma = bn_dgamma->data_ptr<float>();
      sa.dbeta = bn_dbeta->data_ptr<float>();
      sa.bwd = 1;
      sa.defer = 1;
    }
    auto launch = [&](auto tag) {
      using T = decltype(tag);
      const T* xp = reinterpret_cast<const T*>(x.data_ptr());
      const T* wp = reinterpret_cast<const T*>(w.data_ptr());
      T* yp = reinterpret_cast<T*>(y.data_ptr());
      const dim3 gr((unsigned)blocks), th(THR);
      BwdStatArgs<T> bs;
      if (bwdst) {
        bs.x = reinterpret_cast<const T*>(bn_x->data_ptr());
        bs.y = bn_y.has_value() ? reinterpret_cast<const T*>(bn_y->data_ptr()) : nullptr;
        bs.save = bn_save->data_ptr<float>();
        bs.gamma = bn_gamma.has_value() ? bn_gamma->data_ptr<float>() : nullptr;
        bs.beta = bn_beta.has_value() ? bn_beta->data_ptr<float>() : nullptr;
        const dim3 t8(512);
        if (!(g.R == 1 && g.S == 1 && g.pad == 0)) {  // KxK data gradient (recomputed ReLU mask)
          TORCH_CHECK(!bn_y.has_value(), "conv_fwd: KxK BN sums take the recomputed mask");
          if (wide == 3) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_REC, true, 2, 2, 4>), gr, t8, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_REC, true>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_REC, true>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        } else if (bn_y.has_value()) {
          // BS_Y stays on 4 waves unless forced (DPA_WIDE=4): its epilogue prefetches three
          // operand rows, and 8 waves measured +218 us over the network's 12 launches
          // (profiles/r5d_resnet50_steady_wide.txt)
          if (wide == 3 && wide_mode() == 4) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_Y, false, 2, 2, 4>), gr, t8, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_Y>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_Y>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        } else {
          if (wide == 3) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_REC, false, 2, 2, 4>), gr, t8, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_REC>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
          else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_REC>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        }
        return;
      }
      const bool kxk = !(g.R == 1 && g.S == 1 && g.pad == 0);
      if (wide) {  // 8 waves
        if (wide == 1 && kxk) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 128, BS_NONE, true, 2, 4, 2>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (wide == 1) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 128, BS_NONE, false, 2, 4, 2>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (wide == 2 && kxk) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 256, BS_NONE, true, 2, 2, 4>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (wide == 2) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 256, BS_NONE, false, 2, 2, 4>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (kxk) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, true, 2, 2, 4>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, false, 2, 2, 4>), gr, dim3(512), 0, cur_stream(), xp, wp, yp, sa, g, bs);
        return;
      }
      if (glds_stages() == 3 && BP == 128) {  // three LDS buffers (one workgroup per CU)
        if (kxk && BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, true, 3>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (kxk) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_NONE, true, 3>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, false, 3>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_NONE, false, 3>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        return;
      }
      if (glds_stages() == 4 && BP == 128) {  // four LDS buffers (three tiles in flight)
        if (kxk && BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, true, 4>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (kxk) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_NONE, true, 4>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, false, 4>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_NONE, false, 4>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        return;
      }
      if (kxk) {  // KxK: tap-walking loader (128-pixel tiles)
        if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128, BS_NONE, true>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64, BS_NONE, true>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
        return;
      }
      if (BP == 256 && BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 128>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
      else if (BP == 256) hipLaunchKernelGGL((conv_glds_kernel<T, 256, 64>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
      else if (BN == 128) hipLaunchKernelGGL((conv_glds_kernel<T, 128, 128>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
      else hipLaunchKernelGGL((conv_glds_kernel<T, 128, 64>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g, bs);
    };
    if (x.scalar_type() == at::kBFloat16) launch(__hip_bfloat16{}); else launch(__half{});
    DPA_CHECK_LAUNCH();
    if (sa.defer) launch_stat_tree(sa, g.M, BP, (int)g.K, BN);
    return;
  }
  TORCH_CHECK(!bwdst, "conv_fwd: BN backward sums need the 1x1 kernel");
  const int BN = BN0;
  const long long rows = (g.M + BM - 1) / BM;
  const long long blocks = rows * (g.K / BN) * (mode == MODE_S2T ? 4 : 1);
  TORCH_CHECK(blocks < (1LL << 31), "conv_fwd: grid too large");
  sa.defer = st && (defer_stats(blocks) || xc) ? 1 : 0;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    const T* xp = reinterpret_cast<const T*>(x.data_ptr());
    const T* wp = reinterpret_cast<const T*>(w.data_ptr());
    T* yp = reinterpret_cast<T*>(y.data_ptr());
    const dim3 gr((unsigned)blocks), th(THR);
    if (mode == MODE_STEM) {
      if (BN == 128) hipLaunchKernelGGL((conv_fwd_kernel<T, 128, MODE_STEM>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
      else hipLaunchKernelGGL((conv_fwd_kernel<T, 64, MODE_STEM>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
    } else if (mode == MODE_S2T) {
      if (BN == 128) hipLaunchKernelGGL((conv_fwd_kernel<T, 128, MODE_S2T>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
      else hipLaunchKernelGGL((conv_fwd_kernel<T, 64, MODE_S2T>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
    } else {
      if (BN == 128) hipLaunchKernelGGL((conv_fwd_kernel<T, 128>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
      else hipLaunchKernelGGL((conv_fwd_kernel<T, 64>), gr, th, 0, cur_stream(), xp, wp, yp, sa, g);
    }
  };
  if (x.scalar_type() == at::kBFloat16) launch(__hip_bfloat16{}); else launch(__half{});
  DPA_CHECK_LAUNCH();
  if (sa.defer) launch_stat_tree(sa, g.M, BM, (int)g.K, BN);
}

// weight gradients on conv_wgrad_glds_kernel: DPA_WGRAD_GLDS = 1 (default) the 1x1 convs,
// 2 every MODE_GEN conv, 0 none (the register-staged kernel); wgrad_config sets it at run time
static int g_wgrad_glds = -1;
static int wgrad_glds() {
  if (g_wgrad_glds < 0) {
    const char* e = std::getenv("DPA_WGRAD_GLDS");
    // 2 (every MODE_GEN conv, 3x3 included, with 8-wave workgroups): network wgrad 2600 vs
    // 2668 us (1x1 only) vs 2760 (4 waves): profiles/r5d_wgrad_ab.txt
    g_wgrad_glds = e == nullptr ? 2 : std::atoi(e);
  }
  return g_wgrad_glds;
}
int64_t wgrad_config(int64_t glds) {
  wgrad_glds();
  const int64_t prev = g_wgrad_glds;
  if (glds >= 0) g_wgrad_glds = (int)glds;
  return prev;
}
// waves per workgroup of conv_wgrad_glds_kernel: 8 (default) or 4 (DPA_WGRAD_WAVES; wgrad_waves_config)
static int g_wgrad_waves = -1;
static int wgrad_waves() {
  if (g_wgrad_waves < 0) {
    const char* e = std::getenv("DPA_WGRAD_WAVES");
    g_wgrad_waves = e != nullptr && std::atoi(e) == 4 ? 4 : 8;  // 8: network wgrad 2668 vs 2760 us
  }
  return g_wgrad_waves;
}
int64_t wgrad_waves_config(int64_t w) {
  wgrad_waves();
  const int64_t prev = g_wgrad_waves;
  if (w == 4 || w == 8) g_wgrad_waves = (int)w;
  return prev;
}

// wgrad tile shapes: BM | Cout, BN | C (a column tile stays inside one filter tap)
static int wtile(int64_t v) { return v % 128 == 0 ? 128 : 64; }

// In-launch split-K reduction (conv_wgrad_glds_kernel FIX) for convs of at most
// DPA_WGRAD_FIXUP_MAXSP splits (default 0: off; wgrad_fixup_config sets it).  Measured
// slower on ResNet-50 at every bound -- 13.77 ms off, 14.02 at 8 splits, 14.74 at 32, 17.69
// for every conv (profiles/r6v_wgrad_fixup_ab.txt): the partial tiles' write-through stores
// and each tile's serial last-arriver sum cost more than the separate, fully parallel launch.  Tickets: one
// zeroed device array per device, re-armed by every tile's last arriver; allocated outside
// any capture (a first use inside one takes the reduce launch instead).
static long long g_fix_maxsp = -1;
static long long fix_maxsp() {
  if (g_fix_maxsp < 0) {
    const char* e = std::getenv("DPA_WGRAD_FIXUP_MAXSP");
    g_fix_maxsp = e != nullptr ? std::atoll(e) : 0LL;
  }
  return g_fix_maxsp;
}
int64_t wgrad_fixup_config(int64_t maxsp) {
  const int64_t prev = fix_maxsp();
  if (maxsp >= 0) g_fix_maxsp = maxsp;
  return prev;
}
constexpr int kFixTickets = 4096;
static unsigned* fix_tickets(long long tiles) {
  static unsigned* per_dev[64] = {};
  if (tiles > kFixTickets) return nullptr;
  int dev = 0;
  DPA_CHECK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return nullptr;
  if (per_dev[dev] == nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    DPA_CHECK_HIP(hipStreamIsCapturing(cur_stream(), &st));
    if (st != hipStreamCaptureStatusNone) return nullptr;
    unsigned* p = nullptr;
    DPA_CHECK_HIP(hipMalloc(&p, kFixTickets * sizeof(unsigned)));
    DPA_CHECK_HIP(hipMemset(p, 0, kFixTickets * sizeof(unsigned)));
    DPA_CHECK_HIP(hipDeviceSynchronize());
    per_dev[dev] = p;
  }
  return per_dev[dev];
}

int64_t wgrad_splits(int64_t M, int64_t K, int64_t C, int64_t R, int64_t S) {
  // ~2 workgroups per CU, each at least 16 K-steps of 64 pixels, and the fp32
  // partials at most ~48 MB (written and re-read once: ~12 us at HBM rate)
  const int64_t tiles = (K / wtile(K)) * (R * S * C / wtile(C));
  static const int64_t target = [] {
    const char* e = std::getenv("DPA_WGRAD_BLOCKS");
    return e != nullptr ? std::atoll(e) : 512LL;  // ResNet-50 sweep: 384 15.01, 512 14.50, 768 14.59, 1024 14.67 ms
  }();
  static const int64_t minpix = [] {  // round 6 re-sweep: 1024 13.81, 512 13.73, 384 13.74, 256 13.72 ms
    const char* e = std::getenv("DPA_WGRAD_MINPIX");    // (profiles/r6bb_rn_wgrad_minpix.txt)
    return e != nullptr ? std::atoll(e) : 512LL;
  }();
  int64_t sp = std::max<int64_t>(1, target / tiles);
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, M / minpix));
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, (12LL << 20) / (K * R * S * C)));
  return sp;
}

// dy: [N, K, OH, OW] channels_last; x: [N, C, H, W] channels_last; grad: fp32 [K, C, R, S]
// contiguous (written, not accumulated); slab: fp32 >= splits * K * R*S*C.
// mode MODE_STEM: x = the stem_pack image [N, 4, H, W], grad [K, 3, 7, 7] (stride 2, pad 3).
std::vector<int64_t> conv_wgrad(at::Tensor dy, at::Tensor x, at::Tensor grad, int64_t stride, int64_t pad,
                                at::Tensor slab, int64_t mode, bool reduce) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && grad.is_cuda() && slab.is_cuda(), "conv_wgrad: device tensors");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "conv_wgrad: bf16 / f16 activations");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_wgrad: channels_last dy / x");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.is_contiguous() && grad.dim() == 4, "conv_wgrad: fp32 grad");
  const bool stem = mode == MODE_STEM;
  TORCH_CHECK(mode == MODE_GEN || stem, "conv_wgrad: mode");
  Geom g = geom(x, grad, (int)stride, (int)pad);
  int Cd = g.C, Rd = g.R, Sd = g.S;  // gradient dims (the stem's padded K space drops to these)
  if (stem) {
    TORCH_CHECK(x.size(1) == 4 && grad.size(1) == 3 && g.R == 7 && g.S == 7 && stride == 2 && pad == 3 &&
                    g.K % 64 == 0, "conv_wgrad: stem needs the stem_pack image and a [K, 3, 7, 7] gradient");
    g.C = 4;
    Cd = 3;
  } else {
    TORCH_CHECK(grad.size(1) == g.C && supported(g.C, g.K), "conv_wgrad: needs C % 64 == 0 and Cout % 64 == 0");
  }
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.K && dy.size(2) == g.OH && dy.size(3) == g.OW, "conv_wgrad: dy");
  TORCH_CHECK(g.M < (1LL << 31), "conv_wgrad: too many pixels");
  const int SR = stem ? 8 : g.R, SS = stem ? 8 : g.S;  // slab column space [SR][SS][C]
  const int64_t sp = wgrad_splits(g.M, g.K, g.C, SR, SS);
  const int64_t RSC = (int64_t)SR * SS * g.C;
  TORCH_CHECK(slab.scalar_type() == at::kFloat && slab.numel() >= sp * g.K * RSC, "conv_wgrad: slab too small");
  const long long pps = ((g.M + sp - 1) / sp + 63) / 64 * 64;
  const int BM = wtile(g.K), BN = wtile(g.C);
  const long long blocks = sp * (g.K / BM) * (RSC / BN);
  // in-launch split-K reduction: 8-wave LDS-DMA kernels, reduced gradients wanted
  const bool glds = !stem && ((g.R == 1 && g.S == 1 && wgrad_glds() >= 1) || wgrad_glds() == 2);
  unsigned* tk = nullptr;
  const bool fixed = reduce && glds && wgrad_waves() == 8 && sp <= fix_maxsp() &&
                     (tk = fix_tickets((g.K / BM) * (RSC / BN))) != nullptr;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    const T* dp = reinterpret_cast<const T*>(dy.data_ptr());
    const T* xp = reinterpret_cast<const T*>(x.data_ptr());
    float* sl = slab.data_ptr<float>();
    const dim3 gr((unsigned)blocks), th(THR);
    // 1x1 (mode 1, default) or every MODE_GEN conv (mode 2): on 3x3 it measured ~5 % slower
    if (!stem && ((g.R == 1 && g.S == 1 && wgrad_glds() >= 1) || wgrad_glds() == 2)) {
      float* gp = grad.data_ptr<float>();
      if (wgrad_waves() == 8) {
        const dim3 t8(512);
        if (fixed) {
          if (BM == 128 && BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 128, 2, 4, true>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, tk);
          else if (BM == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 64, 4, 2, true>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, tk);
          else if (BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 128, 2, 4, true>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, tk);
          else hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 64, 2, 4, true>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, tk);
          return;
        }
        if (BM == 128 && BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 128, 2, 4>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
        else if (BM == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 64, 4, 2>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
        else if (BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 128, 2, 4>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
        else hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 64, 2, 4>), gr, t8, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
        return;
      }
      if (BM == 128 && BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 128>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
      else if (BM == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 128, 64>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
      else if (BN == 128) hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 128>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
      else hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, 64, 64>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps, gp, nullptr);
      return;
    }
    if (stem && BM == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 64, MODE_STEM>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
    else if (stem) hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 64, MODE_STEM>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
    else if (BM == 128 && BN == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 128>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
    else if (BM == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 64>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
    else if (BN == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 128>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
    else hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 64>), gr, th, 0, cur_stream(), dp, xp, sl, g, (int)sp, pps);
  };
  if (x.scalar_type() == at::kBFloat16) launch(__hip_bfloat16{}); else launch(__half{});
  DPA_CHECK_LAUNCH();
  // reduce = false: the slab stays for wgrad_reduce_batch (the geometry below is its entry)
  std::vector<int64_t> geo{sp, g.K, g.C, SR, SS, Cd, Rd, Sd};
  if (!reduce || fixed) return geo;
  const long long total = (long long)g.K * RSC;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((total + 4 * WR_QC - 1) / (4 * WR_QC))), dim3(256), 0,
                     cur_stream(),
                     slab.data_ptr<float>(), grad.data_ptr<float>(), (int)sp, g.K, g.C, SR, SS, Cd, Rd, Sd);
  DPA_CHECK_LAUNCH();
  return geo;
}

// One launch reducing every (slab, grad) pair of a backward pass (conv_wgrad with reduce =
// false; geo = the geometry it returned), WB_MAX entries per launch.
void wgrad_reduce_batch(std::vector<at::Tensor> slabs, std::vector<at::Tensor> grads,
                        std::vector<std::vector<int64_t>> geos) {
  TORCH_CHECK(slabs.size() == grads.size() && slabs.size() == geos.size(), "wgrad_reduce_batch: one geometry per pair");
  for (size_t s0 = 0; s0 < slabs.size(); s0 += WB_MAX) {
    WBList L{};
    long long blk = 0;
    const size_t e = std::min(slabs.size(), s0 + (size_t)WB_MAX);
    for (size_t i = s0; i < e; ++i) {
      const auto& q = geos[i];
      TORCH_CHECK(q.size() == 8, "wgrad_reduce_batch: geometry {splits, K, C, R, S, Cd, Rd, Sd}");
      const long long total = q[1] * q[3] * q[4] * q[2];
      TORCH_CHECK(slabs[i].is_cuda() && slabs[i].scalar_type() == at::kFloat && slabs[i].numel() >= q[0] * total,
                  "wgrad_reduce_batch: slab");
      TORCH_CHECK(grads[i].is_cuda() && grads[i].scalar_type() == at::kFloat && grads[i].is_contiguous() &&
                      grads[i].numel() == q[1] * q[5] * q[6] * q[7], "wgrad_reduce_batch: fp32 OIHW grad");
      WBEntry& E = L.e[i - s0];
      E.slab = slabs[i].data_ptr<float>();
      E.grad = grads[i].data_ptr<float>();
      E.splits = (int)q[0]; E.K = (int)q[1]; E.C = (int)q[2]; E.R = (int)q[3]; E.S = (int)q[4];
      E.Cd = (int)q[5]; E.Rd = (int)q[6]; E.Sd = (int)q[7];
      E.blk0 = blk;
      blk += (total + 4 * WR_QC - 1) / (4 * WR_QC);
    }
    L.n = (int)(e - s0);
    if (blk == 0) continue;
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((unsigned)blk), dim3(256), 0, cur_stream(), L);
    DPA_CHECK_LAUNCH();
  }
}

}  // namespace igemm

void register_conv_igemm(pybind11::module& m) {
  auto s = m.def_submodule("conv_igemm", "NHWC implicit-GEMM convolution on MFMA (+ fused BN statistics)");
  s.def("conv_fwd", &igemm::conv_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("part") = pybind11::none(),
        pybind11::arg("tickets") = pybind11::none(), pybind11::arg("stats") = pybind11::none(),
        pybind11::arg("shift") = pybind11::none(), pybind11::arg("nbt") = pybind11::none(),
        pybind11::arg("accumulate") = false, pybind11::arg("mode") = 0, pybind11::arg("aux") = pybind11::none(),
        pybind11::arg("bn_x") = pybind11::none(), pybind11::arg("bn_y") = pybind11::none(),
        pybind11::arg("bn_save") = pybind11::none(), pybind11::arg("bn_gamma") = pybind11::none(),
        pybind11::arg("bn_beta") = pybind11::none(), pybind11::arg("bn_out") = pybind11::none(),
        pybind11::arg("bn_dgamma") = pybind11::none(), pybind11::arg("bn_dbeta") = pybind11::none(),
        pybind11::arg("xc") = pybind11::none());
  s.def("supported", &igemm::supported);
  s.def("stat_part_len", &igemm::stat_part_len);
  s.def("stat_tickets_len", &igemm::stat_tickets_len);
  s.def("conv_wgrad", &igemm::conv_wgrad, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("grad"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("slab"), pybind11::arg("mode") = 0,
        pybind11::arg("reduce") = true);
  s.def("wgrad_reduce_batch", &igemm::wgrad_reduce_batch);
  s.def("wgrad_waves_config", &igemm::wgrad_waves_config, pybind11::arg("waves") = -1);
  s.def("stem_pack", &igemm::stem_pack);
  s.attr("MODE_STEM") = igemm::MODE_STEM;
  s.attr("MODE_S2T") = igemm::MODE_S2T;
  s.def("pack_weights", &igemm::pack_weights);
  s.def("wgrad_splits", &igemm::wgrad_splits);
  s.def("wgrad_fixup_config", &igemm::wgrad_fixup_config, pybind11::arg("maxsp") = -1);
  s.def("wgrad_config", &igemm::wgrad_config, pybind11::arg("glds") = -1);
  s.def("g3x3_config", &igemm::g3x3_config, pybind11::arg("on") = -1);
  s.def("glds_config", &igemm::glds_config, pybind11::arg("stages") = -1);
  s.def("wide_config", &igemm::wide_config, pybind11::arg("mode") = -1);
  s.def("bn64_config", &igemm::bn64_config, pybind11::arg("below") = -1);
  s.def("stat_defer_config", &igemm::stat_defer_config, pybind11::arg("min_blocks") = -2);
  s.def("g1x1_config", &igemm::g1x1_config, pybind11::arg("on") = -1, pybind11::arg("bp") = -1,
        pybind11::arg("min256") = -1);
}

}  // namespace dpa
