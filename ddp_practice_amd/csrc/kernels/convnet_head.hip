// The ConvNet head as ONE launch in training: forward, loss and (speculatively) backward.
//
//   [BN2 finalize -> BN -> ReLU -> 2x2 max-pool -> flatten -> Linear]     (forward)
//   -> CrossEntropy(mean) on the logits + d(scale * loss)/dlogits          (loss)
//   -> Linear input gradient dp2 + the BN2 backward sums of this image     (backward)
//
// Reference ops: /root/reference/origin_main.py:16-24,29-30 (BN2/ReLU/pool2, reshape,
// fc) and ddp_main.py:89,91 (CrossEntropyLoss on the logits, scaler.scale(loss).backward()).
// Replaces three launches of the step (head_fwd_kernel, ce_fwd_kernel,
// head_bwd_kernel in csrc/kernels/{convnet_fused,head}.hip) whenever the batch
// labels are known at forward time (the device loader pairs them with the
// images; ops/convnet_fused.py) -- the loss call and the head backward then
// find their results ready and launch nothing.
//
// Decomposition: ONE WORKGROUP PER IMAGE, and no workgroup waits for another.
// An image's row of the head is independent of every other row except for
// three batch reductions, each moved off the critical path:
//   * the loss mean: every workgroup adds its row loss to ONE 64-bit word with a
//     single atomic, as an integer (fixed point, 2^-24), together with an arrival
//     count; the workgroup whose add completes the count holds the exact total in
//     the value its atomic returned (integer addition is associative: the result
//     does not depend on the arrival order) and writes the loss.  No partial
//     store, no fence, no wait, no second hand-off;
//   * the fc weight / bias gradient (a K = batch reduction): computed by extra
//     workgroups of the next launch (conv2_bwd, csrc/kernels/convnet_fused.hip
//     fc_wgrad_body), which overlap the conv2 backward;
//   * the BN2 backward sums: one row of per-channel [S1 | S2] per image, reduced
//     by the consumer kernel's prologue (cb::bn_bwd_coef, like every other slab).
// The mean's row count (non-ignored targets) comes from one ballot over the
// batch's labels, so d(loss)/dlogits of a row is complete inside its workgroup.
// Round 3's channel-per-workgroup head (32 workgroups, partial logits handed to a
// last arriver and back: two cross-workgroup round trips on every workgroup's
// path) took 15.5 us of the 57.7 us step (profiles/r3_head_granule_vs_ticket_ab.txt).
#include <cstdlib>

#include "comm/xgmi.h"
#include "convblock_impl.h"

namespace dpa {
namespace cnh {

using cb::BNParams;
using cb::IDX_RELU;
using cb::Pair2;

// workgroup size (template parameter NT of head_row_kernel): 256 lanes, or 1024 with
// DPA_HEAD_NT=1024 (16 waves, 4 per SIMD).  Same-box A/B with the DPP lane sums: 0.0520 /
// 0.0519 vs 0.0519 / 0.0523 ms per step (profiles/r4n_head_dpp_nt_ab.txt): the BN-pool / GEMV
// phase was the ds_bpermute chain, not lane count
constexpr int NT_MAX = 1024;
constexpr int C = 32, H = 14, W = 14, HO = 7, WO = 7, PP = 49, K = C * PP;
constexpr int BMAX = 64;   // images (one ballot counts the batch's rows)
constexpr int NMAX = 16;   // classes

// loss word (state[0], zero-initialised once; the completing workgroup re-arms it):
// [63:57] arrivals | [56:50] rows whose loss is out of range | [49:0] sum over the
// counted rows of round((row loss + 1) * 2^24) (the +1 keeps rounding-negative rows,
// -1e-7 when one logit dominates, representable)
constexpr int kArrShift = 57, kBadShift = 50;
constexpr unsigned long long kSumMask = (1ull << kBadShift) - 1ull;
constexpr double kFix = 16777216.0;   // 2^24
constexpr float kRowMax = 1048575.f;  // 2^20 - 1: 64 rows of (loss + 1) * 2^24 fit in 50 bits

struct HeadRow {
  const int64_t* target;
  int64_t ignore_index;
  float smoothing;
  const float* scale;   // GradScaler scale (always valid; has_scale = 0: unused)
  int has_scale;
  unsigned long long* state;  // [0] loss word
  float* loss;          // [2]: loss, loss * scale
  float* dlog;          // [B][N] (softmax - onehot) / count, f32
  void* dls;            // [B][N] dlog * scale, storage dtype (null without scaler)
  void* dp2;            // [B][K] storage dtype (null: forward + loss only)
  float* bsum;          // [B][2C] BN2 backward sums of each image (S1 | S2)
  int* chk;             // producer-side gradient check words (common.h GradChk) or null:
                        // cleared here, [1] = this step's scale
};

// lds_barrier (common.h): the global stores (pooled outputs, dp2) and the loss atomic are not waited


// NM: classes the register tiles are sized for (>= N); NT: workgroup size (256 | 1024)
template <typename T, int NM, int NT>
__global__ void __launch_bounds__(NT)
head_row_kernel(const T* __restrict__ y, BNParams bn, const float* __restrict__ wfc, const float* __restrict__ bfc,
                T* __restrict__ logits, T* __restrict__ p_out, uint8_t* __restrict__ idx_out,
                T* __restrict__ xh_out, int B, int N, HeadRow hr) {
  typedef typename Pair2<T>::type P;
  constexpr int IT = (K + NT - 1) / NT;  // pooled features per lane (7 | 2)
  constexpr int NW = NT / 64;
  constexpr int CL = NT / C;             // lanes per channel in the BN2 backward sums (8 | 32)
  __shared__ float sc_s[C], beta_s[C], mean_s[C], istd_s[C];
  __shared__ float part_s[NT];
  __shared__ float red[NW][NM];
  __shared__ float lgs[NM];
  __shared__ float gs[2][IT * NT];  // per pooled feature: g, g * xhat (BN2 backward sums)

  const int tid = threadIdx.x, b = blockIdx.x;
  const int lane = tid & 63, wv = tid >> 6;

  DPA_STAMP(0);
  // 1. every load of the kernel up front.  Unconditional (clamped index, discarded by a
  //    multiply): a conditional load into a register array is branched around and waited
  //    for one by one (head_step .s, ROCm 7.2).
  const T* yb = y + (size_t)b * C * H * W;
  P top[IT], bot[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = min(tid + i * NT, K - 1);
    const int c = k / PP, j = k % PP, ho = j / WO, wo = j % WO;
    const P* src = reinterpret_cast<const P*>(yb + ((size_t)c * H + 2 * ho) * W + 2 * wo);
    top[i] = src[0];
    bot[i] = src[W / 2];
  }
  float wq[NM][IT];  // fc weights of this lane's features, every class
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    const float* wr = wfc + (size_t)min(n, N - 1) * K;
#pragma unroll
    for (int i = 0; i < IT; ++i) wq[n][i] = wr[min(tid + i * NT, K - 1)];
  }
  float bias[NM];
#pragma unroll
  for (int n = 0; n < NM; ++n) bias[n] = bfc[min(n, N - 1)];
  const int64_t tgt_lane = hr.target[min(lane, B - 1)];  // the batch's labels, one per lane
  const int64_t tgt = hr.target[b];
  const float scv = hr.scale[0];
  DPA_STAMP(1);
  cb::bn_finalize<C>(bn, sc_s, beta_s, mean_s, istd_s, part_s, b);  // ends with a barrier
  DPA_STAMP(2);
  if (hr.chk != nullptr && b == 0 && tid == 0) {  // the step's gradient-check words (GradChk)
    hr.chk[0] = 0;
    hr.chk[1] = __float_as_int(scv);
  }
  // 2. BN -> ReLU -> 2x2 max of this image; pooled value, argmax|relu index, xhat
  float pf[IT], xf[IT];
  uint8_t ixr[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = tid + i * NT;
    const int c = min(k, K - 1) / PP;
    float best, xh;
    int bi;
    cb::bn_relu_max4x<T>(top[i], bot[i], sc_s[c], beta_s[c], mean_s[c], istd_s[c], best, bi, xh);
    const T pv = Cvt<T>::from_f(best);
    const T xq = Cvt<T>::from_f(xh);
    ixr[i] = (uint8_t)(bi | (best > 0.f ? IDX_RELU : 0));
    pf[i] = k < K ? Cvt<T>::to_f(pv) : 0.f;
    xf[i] = Cvt<T>::to_f(xq);
    if (k < K) {
      const size_t o = (size_t)b * K + k;
      p_out[o] = pv;
      idx_out[o] = ixr[i];
      xh_out[o] = xq;
    }
  }
  // fc weights in the compute dtype (autocast casts the fp32 master weight)
#pragma unroll
  for (int n = 0; n < NM; ++n)
#pragma unroll
    for (int i = 0; i < IT; ++i) wq[n][i] = n < N ? rnd_t<T>(wq[n][i]) : 0.f;
  // 3. logits = p . W^T + bias: lane-partial dot products, reduced over the wave
  //    (butterfly) and over the 4 waves (LDS, fixed order)
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) a += pf[i] * wq[n][i];
    a = wave_sum_dpp(a);  // every lane active here (full-wave DPP)
    if (lane == 0) red[wv][n] = a;
  }
  lds_barrier();
  if (NW > 4) {  // 16 wave partials: one lane per class adds them (fixed order), then broadcast
    if (tid < NM) {
      float t = 0.f;
#pragma unroll
      for (int n = 0; n < NM; ++n) t = tid == n ? bias[n] : t;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w][tid];
      lgs[tid] = t;
    }
    lds_barrier();
  }
  DPA_STAMP(3);
  // 4. cross entropy of this row, computed by every lane (identical arithmetic): the
  //    same formula and rounding as head.hip ce_fwd_kernel
  float lg[NM];
  float mx = -INFINITY, sx = 0.f, xt = 0.f;
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    float t;
    if (NW > 4) {
      t = lgs[n];
    } else {
      t = bias[n];
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w][n];
    }
    lg[n] = rnd_t<T>(t);
    if (n < N) {
      mx = fmaxf(mx, lg[n]);
      sx += lg[n];
      xt = (n == tgt) ? lg[n] : xt;
    }
  }
  float ex[NM], se = 0.f;
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    ex[n] = n < N ? __expf(lg[n] - mx) : 0.f;
    se += ex[n];
  }
  const float lse = mx + __logf(se);
  const unsigned long long counted =
      __ballot(lane < B && tgt_lane != hr.ignore_index);  // the batch's rows in the mean
  const float cnt = (float)__popcll(counted);
  const float inv = cnt > 0.f ? 1.f / cnt : 0.f;
  const bool use = tgt != hr.ignore_index;
  if (!(tgt >= 0 && tgt < N)) xt = NAN;  // an out-of-range target: NaN loss (torch raises)
  const float row_loss = use ? (1.f - hr.smoothing) * (lse - xt) + hr.smoothing * (lse - sx / (float)N) : 0.f;
  float ds[NM];  // d(scale * loss)/dlogits of this row, rounded to the storage dtype
  float my_lg = 0.f, my_d = 0.f;  // lane n < N: class n's logit and gradient (selected, no branch)
  const float rse = 1.f / se, sm0 = hr.smoothing / (float)N;
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    float d = 0.f;
    if (use && n < N) {
      const float sm = ex[n] * rse;
      const float oh = (n == tgt ? 1.f - hr.smoothing : 0.f) + sm0;
      d = (sm - oh) * inv;
    }
    ds[n] = rnd_t<T>(d * scv);
    my_lg = tid == n ? lg[n] : my_lg;
    my_d = tid == n ? d : my_d;
  }
  if (tid < N) {  // one lane per class writes the row's outputs (one branch, not one per class)
    const size_t o = (size_t)b * N + tid;
    logits[o] = Cvt<T>::from_f(my_lg);
    hr.dlog[o] = my_d;
    if (hr.dls != nullptr) reinterpret_cast<T*>(hr.dls)[o] = Cvt<T>::from_f(my_d * scv);
  }
  if (hr.dp2 != nullptr) {
    DPA_STAMP(4);
    // 6. backward of this row: dp2 = dls . W (the same weight registers), and the BN2
    //    backward sums of each channel over this image's pooled positions
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int k = tid + i * NT;
      float a = 0.f;
#pragma unroll
      for (int n = 0; n < NM; ++n) a += ds[n] * wq[n][i];
      const T gt = Cvt<T>::from_f(a);
      if (k < K) reinterpret_cast<T*>(hr.dp2)[(size_t)b * K + k] = gt;
      const float g = (ixr[i] & IDX_RELU) ? Cvt<T>::to_f(gt) : 0.f;
      gs[0][k] = g;
      gs[1][k] = g * xf[i];
    }
    lds_barrier();
    {  // channel c = tid / CL: CL lanes sum its 49 positions in a fixed order
      const int c = tid / CL, j = tid % CL;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int f = j; f < PP; f += CL) {
        s1 += gs[0][c * PP + f];
        s2 += gs[1][c * PP + f];
      }
      s1 = group_sum<CL>(s1);  // every lane active (DPP)
      s2 = group_sum<CL>(s2);
      if (j == 0) {
        hr.bsum[(size_t)b * 2 * C + c] = s1;
        hr.bsum[(size_t)b * 2 * C + C + c] = s2;
      }
    }
    DPA_STAMP(5);
  }
  // 7. the loss mean (last: nothing in this workgroup waits for the atomic's return but
  //    the workgroup that completes the batch): one atomic per workgroup (see the loss word above)
  if (tid == 0) {
    const bool ok = !use || (row_loss > -1.f && row_loss < kRowMax);
    const unsigned long long inc =
        (1ull << kArrShift) +
        (ok ? (use ? (unsigned long long)(((double)row_loss + 1.0) * kFix + 0.5) : 0ull) : (1ull << kBadShift));
    const unsigned long long old =
        __hip_atomic_fetch_add(hr.state, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)(old >> kArrShift) == B - 1) {  // this add completed the batch: old + inc is the total
      const unsigned long long tot = old + inc;
      const int bad = (int)((tot >> kBadShift) & 127ull);
      const double sum = (double)(tot & kSumMask) / kFix - (double)cnt;
      const float l = (cnt > 0.f && bad == 0) ? (float)(sum / (double)cnt) : NAN;
      hr.loss[0] = l;
      if (hr.has_scale) hr.loss[1] = l * scv;
      __hip_atomic_store(hr.state, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
template <typename F>
static void with_t(DT dt, F&& f) {
  switch (dt) {
    case DT::F32: f(float{}); break;
    case DT::BF16: f(__hip_bfloat16{}); break;
    case DT::F16: f(__half{}); break;
  }
}

bool supported(int64_t B, int64_t N) { return B >= 1 && B <= BMAX && N >= 1 && N <= NMAX; }

// no workgroup of the launch waits for another (SyncBN's in-kernel exchange aside, whose
// B workgroups are far below one per CU); kept for the host-side dispatch check
bool resident(at::ScalarType st) {
  bool ok = true;
  with_t(dt_of(at::empty({0}, at::TensorOptions().dtype(st))), [&](auto tag) {
    typedef decltype(tag) T;
    ok = co_resident(reinterpret_cast<const void*>(&head_row_kernel<T, 10, NT_MAX>), BMAX, NT_MAX, 0) &&
         co_resident(reinterpret_cast<const void*>(&head_row_kernel<T, NMAX, 256>), BMAX, 256, 0);
  });
  return ok;
}

// Forward + loss (+ with dp2 / bsum: the row backward, the GradScaler's scale seeding it).
// state: int64[>= 1] zeroed once (the kernel re-arms its loss word).
void head_step(at::Tensor y2, at::Tensor fslab2, at::Tensor fstats2, at::Tensor g2, at::Tensor b2, at::Tensor rm2,
               at::Tensor rv2, at::Tensor nbt2, double momentum, double eps, at::Tensor wfc, at::Tensor bfc,
               at::Tensor logits, at::Tensor p2, at::Tensor idx2, at::Tensor xh2, at::Tensor target,
               int64_t ignore_index, double smoothing, c10::optional<at::Tensor> scale, at::Tensor state,
               at::Tensor loss, at::Tensor dlog, c10::optional<at::Tensor> dls, c10::optional<at::Tensor> dp2,
               c10::optional<at::Tensor> bsum_rows, std::shared_ptr<xgmi::XgmiComm> xc,
               c10::optional<at::Tensor> chk) {
  DPA_CHECK_INPUT(y2); DPA_CHECK_INPUT(wfc); DPA_CHECK_INPUT(logits); DPA_CHECK_INPUT(p2); DPA_CHECK_INPUT(target);
  DPA_CHECK_INPUT(bfc); DPA_CHECK_INPUT(idx2); DPA_CHECK_INPUT(xh2); DPA_CHECK_INPUT(dlog);
  const int B = (int)y2.size(0), N = (int)wfc.size(0);
  TORCH_CHECK(y2.size(1) == C && y2.size(2) == H && y2.size(3) == W && wfc.size(1) == K, "head_step: ConvNet shapes");
  TORCH_CHECK(supported(B, N), "head_step: B <= ", BMAX, " and N <= ", NMAX);
  TORCH_CHECK(bfc.numel() == N && wfc.scalar_type() == at::kFloat && bfc.scalar_type() == at::kFloat);
  TORCH_CHECK(logits.numel() == (int64_t)B * N && logits.scalar_type() == y2.scalar_type());
  TORCH_CHECK(p2.numel() == (int64_t)B * K && idx2.numel() == p2.numel() && xh2.numel() == p2.numel());
  TORCH_CHECK(p2.scalar_type() == y2.scalar_type() && xh2.scalar_type() == y2.scalar_type() &&
              idx2.scalar_type() == at::kByte);
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == B);
  TORCH_CHECK(state.numel() >= 1 && state.scalar_type() == at::kLong && state.is_cuda());
  TORCH_CHECK(loss.numel() >= 2 && loss.scalar_type() == at::kFloat && loss.is_cuda());
  TORCH_CHECK(dlog.numel() == (int64_t)B * N && dlog.scalar_type() == at::kFloat);
  TORCH_CHECK(scale.has_value() == dls.has_value(), "head_step: scale and dls go together");
  const bool bwd = dp2.has_value();
  TORCH_CHECK(bwd == bsum_rows.has_value(), "head_step: dp2 and bsum_rows go together");
  if (scale.has_value()) {
    DPA_CHECK_INPUT(*scale); DPA_CHECK_INPUT(*dls);
    TORCH_CHECK(scale->numel() >= 1 && scale->scalar_type() == at::kFloat);
    TORCH_CHECK(dls->numel() == (int64_t)B * N && dls->scalar_type() == y2.scalar_type());
  }
  if (bwd) {
    TORCH_CHECK(scale.has_value(), "head_step: the speculative backward needs the scaler's loss gradient");
    DPA_CHECK_INPUT(*dp2); DPA_CHECK_INPUT(*bsum_rows);
    TORCH_CHECK(dp2->numel() == p2.numel() && dp2->scalar_type() == y2.scalar_type());
    TORCH_CHECK(bsum_rows->numel() == (int64_t)B * 2 * C && bsum_rows->scalar_type() == at::kFloat);
  }
  if (B == 0) return;
  BNParams bp;
  bp.fslab = fslab2.data_ptr<float>();
  bp.nrows = (int)(fslab2.numel() / cb::fslab_row(C));
  bp.fstats = fstats2.data_ptr<float>();
  bp.gamma = g2.data_ptr<float>();
  bp.beta = b2.data_ptr<float>();
  bp.rmean = rm2.data_ptr<float>();
  bp.rvar = rv2.data_ptr<float>();
  bp.nbt = nbt2.data_ptr<int64_t>();
  bp.momentum = (float)momentum;
  bp.eps = (float)eps;
  bp.train = 1;
  if (xc) {
    bp.xs = xc->site(xgmi::kSiteFwd2);
    xgmi::set_site_grid(bp.xs, B, "convnet head");  // the grid (spares the kernel a hidden-argument load)
  }
  HeadRow hr;
  hr.target = target.data_ptr<int64_t>();
  hr.ignore_index = ignore_index;
  hr.smoothing = (float)smoothing;
  hr.scale = scale.has_value() ? scale->data_ptr<float>() : loss.data_ptr<float>();  // unread without a scaler
  hr.has_scale = scale.has_value() ? 1 : 0;
  hr.chk = nullptr;
  if (chk.has_value()) {
    DPA_CHECK_INPUT(*chk);
    TORCH_CHECK(chk->scalar_type() == at::kInt && chk->numel() == 2 && scale.has_value(),
                "head_step: gradient-check words need the scaler's scale and int32[2]");
    hr.chk = chk->data_ptr<int>();
  }
  hr.state = reinterpret_cast<unsigned long long*>(state.data_ptr<int64_t>());
  hr.loss = loss.data_ptr<float>();
  hr.dlog = dlog.data_ptr<float>();
  hr.dls = dls.has_value() ? dls->data_ptr() : nullptr;
  hr.dp2 = bwd ? dp2->data_ptr() : nullptr;
  hr.bsum = bwd ? bsum_rows->data_ptr<float>() : nullptr;
  with_t(dt_of(y2), [&](auto tag) {
    typedef decltype(tag) T;
    static const int nt = [] {
      const char* e = std::getenv("DPA_HEAD_NT");
      return e != nullptr && std::atoi(e) == NT_MAX ? NT_MAX : 256;
    }();
    // 16-class tiles stay at 256 lanes (at 1024 the 128-VGPR budget spills them)
    const int ntl = N <= 10 ? nt : 256;
    auto kern = N > 10 ? head_row_kernel<T, NMAX, 256>
                       : (nt == 256 ? head_row_kernel<T, 10, 256> : head_row_kernel<T, 10, NT_MAX>);
    hipLaunchKernelGGL(kern, dim3(B), dim3(ntl), 0, cur_stream(), dptr<T>(y2), bp, wfc.data_ptr<float>(),
                       bfc.data_ptr<float>(), dptr<T>(logits), dptr<T>(p2), idx2.data_ptr<uint8_t>(), dptr<T>(xh2), B,
                       N, hr);
  });
  DPA_CHECK_LAUNCH();
}

}  // namespace cnh

void register_convnet_head(pybind11::module& m) {
  auto s = m.def_submodule("convnet_head", "ConvNet head: forward + loss + backward in one launch");
  s.def("head_step", &cnh::head_step);
  s.def("supported", &cnh::supported);
  s.def("resident", &cnh::resident);
  DPA_DEF_STAMP_FNS(s);
  s.attr("C") = cnh::C;
  s.attr("NMAX") = cnh::NMAX;
}

}  // namespace dpa
