// BatchNorm2d (training mode) forward/backward with fused ReLU and residual add, NHWC bf16.
//
// Replaces `nn.BatchNorm2d` (reference src/*/net.py:21,25,37,92), `F.relu` and
// `out += self.shortcut(x)` (net.py:41-44, 108). Semantics follow torch's training-mode
// batch norm: batch statistics over N*H*W with biased variance for normalisation,
// unbiased variance for running_var, running = (1-momentum)*running + momentum*batch,
// num_batches_tracked += 1. Under autocast the conv output is bf16, BN computes in fp32
// and emits bf16, ReLU's backward masks with its own (bf16) output.
//
// Statistics: the forward sums (sum x, sum x^2) are produced by the conv epilogues into
// fixed-point slots (common.h); here they are finalised. Backward sums (sum dz, sum dz*xhat)
// are reduced per workgroup through LDS and then added into the same kind of slots.
#include "common.h"
#include "kernels.h"
#include "tile_common.h"
#include "bn_coef.h"

namespace dtc {

static inline int ceil_div_i(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Finalize layout: a 256-thread workgroup owns FIN_CH = 32 channels; thread t reads word (t >> 5) & 3
// (statistic, hi / lo: common.h) of channel c0 + (t & 31) in half t >> 7 of the slots (8 loads, all
// issued before any use), re-zeroes them, sums them as integers, and the two halves are combined in LDS.
// Few registers and no scratch: measured on MI355X, a finalize holding all 64 slot values per thread
// spilled to scratch (44-284 B/lane) and cost 10-16 us per launch instead of ~2.
constexpr int FIN_CH = 32, FIN_GROUPS = 8, FIN_PER = DTC_STAT_SLOTS / 2;

__device__ __forceinline__ bool fin_sum_slots(int64_t* __restrict__ base, int C, double& s, double& q,
                                              int64_t (*red)[FIN_CH]) {
  const int t = threadIdx.x, cl = t & (FIN_CH - 1), g = t >> 5, wd = g & 3, half = g >> 2;
  const int c = blockIdx.x * FIN_CH + cl;
  const int64_t flag = base[0];
  if (c < C) {
    int64_t v[FIN_PER];
#pragma unroll
    for (int j = 0; j < FIN_PER; ++j) v[j] = base[stat_word(half * FIN_PER + j, wd >> 1, wd & 1, C) + c];
    int64_t a = 0;
#pragma unroll
    for (int j = 0; j < FIN_PER; ++j) a += v[j];
#pragma unroll
    for (int j = 0; j < FIN_PER; ++j) base[stat_word(half * FIN_PER + j, wd >> 1, wd & 1, C) + c] = 0;
    red[g][cl] = a;
  }
  __syncthreads();  // (the header's flag is left as it is: the slots' owner zeroes the header)
  if (t >= FIN_CH || c >= C) return false;
  s = stat_total(red[0][cl] + red[4][cl], red[1][cl] + red[5][cl], flag);
  q = stat_total(red[2][cl] + red[6][cl], red[3][cl] + red[7][cl], flag);
  return true;
}

__global__ void __launch_bounds__(256) bn_fwd_finalize_kernel(
    int64_t* __restrict__ stats, int C, double count, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt, float momentum, float eps,
    float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ int64_t red[FIN_GROUPS][FIN_CH];
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  double s, q;
  if (!fin_sum_slots(stats, C, s, q, red)) return;
  const int c = blockIdx.x * FIN_CH + threadIdx.x;
  const double mu = s / count;
  double var = q / count - mu * mu;
  if (var < 0.0) var = 0.0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)mu;
  invstd[c] = is;
  if (rmean) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
  const float a = gamma[c] * is;
  scale[c] = a;
  shift[c] = beta[c] - (float)mu * a;
}

int bn_fwd_finalize(int64_t* stats, int C, int64_t count, const float* gamma, const float* beta, float* running_mean,
                    float* running_var, int64_t* num_batches, float momentum, float eps, float* mean, float* invstd,
                    float* scale, float* shift, hipStream_t st) {
  DTC_CHECK_ARG(stats && gamma && beta && mean && invstd && scale && shift && C > 0 && count > 0,
                "bn_fwd_finalize: bad args");
  DTC_KLAUNCH(bn_fwd_finalize_kernel, dim3(ceil_div_i(C, FIN_CH)), dim3(256), 0, st, stats, C, (double)count,
                     gamma, beta, running_mean, running_var, num_batches, momentum, eps, mean, invstd, scale, shift);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void bn_eval_coef_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                    float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ scale,
                                    float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = 1.f / sqrtf(rv[c] + eps);
  mean[c] = rm[c];
  invstd[c] = is;
  const float a = gamma[c] * is;
  scale[c] = a;
  shift[c] = beta[c] - rm[c] * a;
}

int bn_eval_coef(int C, const float* gamma, const float* beta, const float* running_mean, const float* running_var,
                 float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st) {
  DTC_CHECK_ARG(gamma && beta && running_mean && running_var && mean && invstd && scale && shift && C > 0,
                "bn_eval_coef: bad args");
  DTC_KLAUNCH(bn_eval_coef_kernel, dim3(ceil_div_i(C, 256)), dim3(256), 0, st, C, gamma, beta, running_mean,
                     running_var, eps, mean, invstd, scale, shift);
  DTC_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ forward apply
enum { APPLY_PLAIN = 0, APPLY_RELU = 1, APPLY_ADD_RELU = 2, APPLY_DUAL_RELU = 3 };

template <int MODE, typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, const T* __restrict__ x2,
                                                      const float* __restrict__ scale2,
                                                      const float* __restrict__ shift2, T* __restrict__ y,
                                                      int64_t nvec, int cvec) {
  typedef Elt<T> E;
  for (int64_t v = blockIdx.x * (int64_t)256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cvec) * 8;
    float a[8], o[8];
    E::unpack(E::ld(x + v * 8), a);
    const f32x4 s0 = *(const f32x4*)(scale + c0), s1 = *(const f32x4*)(scale + c0 + 4);
    const f32x4 h0 = *(const f32x4*)(shift + c0), h1 = *(const f32x4*)(shift + c0 + 4);
    const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = a[k] * sc[k] + sh[k];
    if constexpr (MODE == APPLY_ADD_RELU) {
      float r[8];
      E::unpack(E::ld(x2 + v * 8), r);
      // torch rounds the BN output to bf16 before `out += shortcut(x)` (autocast; identity in fp32)
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = E::round(o[k]) + r[k];
    }
    if constexpr (MODE == APPLY_DUAL_RELU) {
      float r[8];
      E::unpack(E::ld(x2 + v * 8), r);
      const f32x4 t0 = *(const f32x4*)(scale2 + c0), t1 = *(const f32x4*)(scale2 + c0 + 4);
      const f32x4 u0 = *(const f32x4*)(shift2 + c0), u1 = *(const f32x4*)(shift2 + c0 + 4);
      const float sc2[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
      const float sh2[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      // torch rounds each BN output to bf16 before the residual add (autocast; identity in fp32)
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = E::round(o[k]) + E::round(r[k] * sc2[k] + sh2[k]);
    }
    if constexpr (MODE != APPLY_PLAIN) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaxf(o[k], 0.f);
    }
    E::st(y + v * 8, E::pack(o));
  }
}

template <int MODE, typename T>
static int launch_apply(const T* x, const float* s, const float* h, const T* x2, const float* s2, const float* h2,
                        T* y, int64_t M, int C, hipStream_t st) {
  DTC_CHECK_ARG(x && s && h && y && C % 8 == 0 && M > 0, "bn_apply: bad args (C=%d)", C);
  const int64_t nvec = M * C / 8;
  const int blocks = (int)std::min<int64_t>(4096, (nvec + 255) / 256);
  DTC_KLAUNCH((bn_apply_kernel<MODE, T>), dim3(blocks), dim3(256), 0, st, x, s, h, x2, s2, h2, y, nvec, C / 8);
  DTC_LAUNCH_CHECK();
  return 0;
}

#define DTC_BN_APPLY_DEFS(T)                                                                                      \
  int bn_apply(const T* x, const float* s, const float* h, T* y, int64_t M, int C, hipStream_t st) {             \
    return launch_apply<APPLY_PLAIN, T>(x, s, h, nullptr, nullptr, nullptr, y, M, C, st);                         \
  }                                                                                                               \
  int bn_apply_relu(const T* x, const float* s, const float* h, T* y, int64_t M, int C, hipStream_t st) {        \
    return launch_apply<APPLY_RELU, T>(x, s, h, nullptr, nullptr, nullptr, y, M, C, st);                          \
  }                                                                                                               \
  int bn_apply_add_relu(const T* x, const float* s, const float* h, const T* res, T* y, int64_t M, int C,       \
                        hipStream_t st) {                                                                         \
    DTC_CHECK_ARG(res != nullptr, "bn_apply_add_relu: residual required");                                       \
    return launch_apply<APPLY_ADD_RELU, T>(x, s, h, res, nullptr, nullptr, y, M, C, st);                          \
  }                                                                                                               \
  int bn_apply_dual_relu(const T* x, const float* s, const float* h, const T* x2, const float* s2, const float* h2, \
                         T* y, int64_t M, int C, hipStream_t st) {                                               \
    DTC_CHECK_ARG(x2 && s2 && h2, "bn_apply_dual_relu: second branch required");                                 \
    return launch_apply<APPLY_DUAL_RELU, T>(x, s, h, x2, s2, h2, y, M, C, st);                                    \
  }
DTC_BN_APPLY_DEFS(u16)
DTC_BN_APPLY_DEFS(float)
#undef DTC_BN_APPLY_DEFS

// ------------------------------------------------------------------ fused finalize + apply (forward)
// The consumer computes the BN coefficients itself: workgroup (pixel block, 64-channel group)
// sums the DTC_STAT_SLOTS fixed-point slots of its 64 channels (32 KB, L2-resident: every workgroup of
// the launch reads the same lines; exact integer sums), then normalises its pixels. The first pixel
// block of each channel group also writes the saved mean / invstd and the running statistics
// (and num_batches_tracked once). Removes the separate finalize launch and its kernel boundary;
// the slots are zeroed by a memset node at the start of the executor's forward.
constexpr int FA_GROUP = 64;  // channels per workgroup
constexpr int FA_UNROLL = 4;  // pixel rows in flight per thread

// mask (optional): the ReLU mask of y, one bit per element (byte o/8 of element offset o, bit k =
// channel c0 + k): the backward reads it instead of y (0.125 B instead of 2 B per element).
template <int MODE, typename T>
__global__ void __launch_bounds__(256) bn_fin_apply_kernel(const T* __restrict__ x, const BnFwdArgs a1,
                                                          const T* __restrict__ x2, const BnFwdArgs a2,
                                                          T* __restrict__ y, int64_t M, int C, int rows,
                                                          uint8_t* __restrict__ mask, u64* ts) {
  typedef Elt<T> E;
  __shared__ int64_t part[256];
  __shared__ float coef[4][64];  // scale1, shift1, scale2, shift2
  stamp_start(ts);
  const int cg = blockIdx.y * FA_GROUP;
  const int t = threadIdx.x, q8 = (t & 7) * 8, pr = t >> 3;
  const int64_t m0 = (int64_t)blockIdx.x * rows, m1 = std::min<int64_t>(M, m0 + rows);
  typename E::V xa[FA_UNROLL], xr[FA_UNROLL];
  auto load = [&](int64_t mb) {  // branch-free: rows past the block's end load a valid row (unused)
#pragma unroll
    for (int u = 0; u < FA_UNROLL; ++u) {
      const int64_t o = std::min<int64_t>(mb + 32 * u, M - 1) * C + cg + q8;
      xa[u] = E::ld(x + o);
      if constexpr (MODE != APPLY_RELU) xr[u] = E::ld(x2 + o);
    }
  };
  // the first trip's loads are issued before the coefficient fold, so their latency overlaps it (the
  // small layers' launches are one trip per thread)
  SlotFold f1, f2;
  fold_issue_fwd(a1, C, cg, f1);
  if constexpr (MODE == APPLY_DUAL_RELU) fold_issue_fwd(a2, C, cg, f2);
  load(m0 + pr);
  fa_fwd_coef_from(a1, f1, C, cg, part, coef[0], coef[1]);
  if constexpr (MODE == APPLY_DUAL_RELU) fa_fwd_coef_from(a2, f2, C, cg, part, coef[2], coef[3]);
  float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = coef[0][q8 + k];
    sh[k] = coef[1][q8 + k];
    if constexpr (MODE == APPLY_DUAL_RELU) {
      sc2[k] = coef[2][q8 + k];
      sh2[k] = coef[3][q8 + k];
    }
  }
  // FA_UNROLL rows per thread per trip: every load of the trip is issued before the first
  // dependent use (memory-level parallelism); elementwise, so results are unchanged
  for (int64_t mb = m0 + pr; mb < m1; mb += 32 * FA_UNROLL) {
    if (mb != m0 + pr) load(mb);
#pragma unroll
    for (int u = 0; u < FA_UNROLL; ++u) {
      const int64_t m = mb + 32 * u;
      if (m >= m1) break;
      const int64_t o = m * C + cg + q8;
      float a[8], r[8], v[8];
      E::unpack(xa[u], a);
      if constexpr (MODE != APPLY_RELU) E::unpack(xr[u], r);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] = a[k] * sc[k] + sh[k];
        // torch rounds each BN output to bf16 before the residual add (autocast)
        if constexpr (MODE == APPLY_ADD_RELU) v[k] = E::round(v[k]) + r[k];
        if constexpr (MODE == APPLY_DUAL_RELU) v[k] = E::round(v[k]) + E::round(r[k] * sc2[k] + sh2[k]);
        v[k] = fmaxf(v[k], 0.f);
      }
      const typename E::V pk = E::pack(v);
      E::st(y + o, pk);
      if (mask != nullptr) mask[o >> 3] = (uint8_t)E::mask8(pk);
    }
  }
  stamp_end(ts);
}

static void fa_grid(int64_t M, int C, int& nblk, int& rows) {
  const int groups = C / FA_GROUP;
  nblk = std::max(1, option_get(OPT_BN_FA_BLOCKS) / groups);  // workgroups per launch (default 1024)
  rows = (int)((M + nblk - 1) / nblk);
  // at least FA_UNROLL rows per thread: each workgroup's prologue folds 32 KB of statistic slots, which
  // dominated the small (layer3/4) launches at one row per thread
  rows = std::max(32 * FA_UNROLL, (rows + 31) / 32 * 32);
  nblk = (int)((M + rows - 1) / rows);
}

template <typename T>
static int fin_apply(int mode, const T* x, const BnFwdArgs& a1, const T* x2, const BnFwdArgs* a2, T* y, int64_t M,
                     int C, hipStream_t st, uint8_t* mask, u64* ts) {
  DTC_CHECK_ARG(x && y && a1.stats && a1.gamma && a1.beta && a1.mean && a1.invstd && C % FA_GROUP == 0 && M > 0,
                "bn_fin_apply: bad args (C=%d)", C);
  int nblk, rows;
  fa_grid(M, C, nblk, rows);
  const dim3 grid(nblk, C / FA_GROUP);
  const BnFwdArgs none{};
  switch (mode) {
    case APPLY_RELU:
      DTC_KLAUNCH((bn_fin_apply_kernel<APPLY_RELU, T>), grid, dim3(256), 0, st, x, a1, x2, none, y, M, C, rows, mask, ts);
      break;
    case APPLY_ADD_RELU:
      DTC_CHECK_ARG(x2 != nullptr, "bn_fin_apply: residual required");
      DTC_KLAUNCH((bn_fin_apply_kernel<APPLY_ADD_RELU, T>), grid, dim3(256), 0, st, x, a1, x2, none, y, M, C, rows, mask, ts);
      break;
    default:
      DTC_CHECK_ARG(x2 && a2 && a2->stats, "bn_fin_apply: second branch required");
      DTC_KLAUNCH((bn_fin_apply_kernel<APPLY_DUAL_RELU, T>), grid, dim3(256), 0, st, x, a1, x2, *a2, y, M, C, rows, mask, ts);
      break;
  }
  DTC_LAUNCH_CHECK();
  return 0;
}

int bn_fin_apply(int mode, const u16* x, const BnFwdArgs& a1, const u16* x2, const BnFwdArgs* a2, u16* y, int64_t M,
                 int C, hipStream_t st, uint8_t* mask, u64* ts) {
  return fin_apply<u16>(mode, x, a1, x2, a2, y, M, C, st, mask, ts);
}
int bn_fin_apply(int mode, const float* x, const BnFwdArgs& a1, const float* x2, const BnFwdArgs* a2, float* y,
                 int64_t M, int C, hipStream_t st) {
  return fin_apply<float>(mode, x, a1, x2, a2, y, M, C, st, nullptr, nullptr);
}

// ------------------------------------------------------------------ fused finalize + apply (backward)
// dx = A*dz + B*x + Cc with the coefficients computed per workgroup from the statistic slots of
// sum(dz), sum(dz*xhat); the first pixel block writes dgamma / dbeta (x gscale).
// MB: dz is formed here from the raw gradient (`dz` = dy) and the forward's ReLU mask bits
// (dz = dy * [y > 0]; exact), and optionally stored to dzo (may alias dy: each element is read and
// written by the same lane) for a consumer that needs it (the identity shortcut's residual).
template <bool DUAL, bool MB, typename T>
__global__ void __launch_bounds__(256) bn_bwd_fin_apply_kernel(const T* __restrict__ dz, const T* __restrict__ x1,
                                                              const BnBwdArgs a1, T* __restrict__ dx1,
                                                              const T* __restrict__ x2, const BnBwdArgs a2,
                                                              T* __restrict__ dx2, int64_t M, int C, int rows,
                                                              const uint8_t* __restrict__ mbits, T* dzo, u64* ts) {
  typedef Elt<T> E;
  __shared__ int64_t part[256];
  __shared__ float coef[6][64];
  stamp_start(ts);
  const int cg = blockIdx.y * FA_GROUP;
  const int t = threadIdx.x, q8 = (t & 7) * 8, pr = t >> 3;
  const int64_t m0 = (int64_t)blockIdx.x * rows, m1 = std::min<int64_t>(M, m0 + rows);
  typename E::V vd[FA_UNROLL], va[FA_UNROLL], vb[FA_UNROLL];
  uint32_t mk[FA_UNROLL];
  auto load = [&](int64_t mb) {  // branch-free (see bn_fin_apply_kernel)
#pragma unroll
    for (int u = 0; u < FA_UNROLL; ++u) {
      const int64_t o = std::min<int64_t>(mb + 32 * u, M - 1) * C + cg + q8;
      vd[u] = E::ld(dz + o);
      va[u] = E::ld(x1 + o);
      if constexpr (DUAL) vb[u] = E::ld(x2 + o);
      if constexpr (MB) mk[u] = mbits[o >> 3];
    }
  };
  SlotFold f1, f2;
  fold_issue_bwd(a1, C, cg, f1);
  if constexpr (DUAL) fold_issue_bwd(a2, C, cg, f2);
  load(m0 + pr);  // in flight during the coefficient fold (see bn_fin_apply_kernel)
  fa_bwd_coef_from(a1, f1, C, cg, part, coef[0], coef[1], coef[2]);
  if constexpr (DUAL) fa_bwd_coef_from(a2, f2, C, cg, part, coef[3], coef[4], coef[5]);
  float A1[8], B1[8], C1[8], A2[8], B2[8], C2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A1[k] = coef[0][q8 + k]; B1[k] = coef[1][q8 + k]; C1[k] = coef[2][q8 + k];
    if constexpr (DUAL) {
      A2[k] = coef[3][q8 + k]; B2[k] = coef[4][q8 + k]; C2[k] = coef[5][q8 + k];
    }
  }
  for (int64_t mb = m0 + pr; mb < m1; mb += 32 * FA_UNROLL) {  // loads of a trip first (see bn_fin_apply)
    if (mb != m0 + pr) load(mb);
#pragma unroll
    for (int u = 0; u < FA_UNROLL; ++u) {
      const int64_t m = mb + 32 * u;
      if (m >= m1) break;
      const int64_t o = m * C + cg + q8;
      float d[8], a[8], v[8];
      E::unpack(vd[u], d);
      if constexpr (MB) {
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = (mk[u] >> k) & 1u ? d[k] : 0.f;
        if (dzo != nullptr) E::st(dzo + o, E::pack(d));  // exact: masking is exact
      }
      E::unpack(va[u], a);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = A1[k] * d[k] + B1[k] * a[k] + C1[k];
      E::st(dx1 + o, E::pack(v));
      if constexpr (DUAL) {
        E::unpack(vb[u], a);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = A2[k] * d[k] + B2[k] * a[k] + C2[k];
        E::st(dx2 + o, E::pack(v));
      }
    }
  }
  stamp_end(ts);
}

template <typename T>
static int bwd_fin_apply(const T* dz, const T* x1, const BnBwdArgs& a1, T* dx1, const T* x2, const BnBwdArgs* a2,
                         T* dx2, int64_t M, int C, hipStream_t st, const uint8_t* mbits = nullptr, T* dzo = nullptr,
                         u64* ts = nullptr) {
  DTC_CHECK_ARG(dz && x1 && dx1 && a1.acc && a1.gamma && a1.mean && a1.invstd && C % FA_GROUP == 0 && M > 0,
                "bn_bwd_fin_apply: bad args (C=%d)", C);
  DTC_CHECK_ARG(mbits || !dzo, "bn_bwd_fin_apply: a dz output needs the mask bits");
  int nblk, rows;
  fa_grid(M, C, nblk, rows);
  const dim3 grid(nblk, C / FA_GROUP);
  const BnBwdArgs none{};
  if (x2) DTC_CHECK_ARG(a2 && a2->acc && dx2, "bn_bwd_fin_apply: dual branch args");
#define DTC_BFA(D_, M_) \
  DTC_KLAUNCH((bn_bwd_fin_apply_kernel<D_, M_, T>), grid, dim3(256), 0, st, dz, x1, a1, dx1, x2, D_ ? *a2 : none, \
                     dx2, M, C, rows, mbits, dzo, ts)
  if (x2 && mbits) DTC_BFA(true, true);
  else if (x2) DTC_BFA(true, false);
  else if (mbits) DTC_BFA(false, true);
  else DTC_BFA(false, false);
#undef DTC_BFA
  DTC_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_fin_apply_mask(const u16* dy, const uint8_t* mbits, u16* dzo, const u16* x1, const BnBwdArgs& a1, u16* dx1,
                          const u16* x2, const BnBwdArgs* a2, u16* dx2, int64_t M, int C, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(mbits != nullptr, "bn_bwd_fin_apply_mask: mask bits required");
  return bwd_fin_apply<u16>(dy, x1, a1, dx1, x2, a2, dx2, M, C, st, mbits, dzo, ts);
}

int bn_bwd_fin_apply(const u16* dz, const u16* x1, const BnBwdArgs& a1, u16* dx1, const u16* x2, const BnBwdArgs* a2,
                     u16* dx2, int64_t M, int C, hipStream_t st) {
  return bwd_fin_apply<u16>(dz, x1, a1, dx1, x2, a2, dx2, M, C, st);
}
int bn_bwd_fin_apply(const float* dz, const float* x1, const BnBwdArgs& a1, float* dx1, const float* x2,
                     const BnBwdArgs* a2, float* dx2, int64_t M, int C, hipStream_t st) {
  return bwd_fin_apply<float>(dz, x1, a1, dx1, x2, a2, dx2, M, C, st);
}

// ------------------------------------------------------------------ one-pass backward, channel groups
// Small BN tensors (M <= 4096 pixels, 2048 with the projection's second BN: layer4 at batch 256, layers 3-4 at the per-rank batches
// of BASELINE config 3) are launch-latency bound: the reduce + apply pair costs two kernel boundaries for a
// few MB. Here ONE launch does both without any cross-workgroup step: workgroup g owns channels 8g..8g+7 of
// EVERY pixel (grid = C / 8), holds its slice of (dy, mask bits, x [, x2]) in registers (CG_NP pixels per
// thread), reduces sum(dz) and sum(dz * xhat) over the whole batch inside the workgroup (fixed order: lane
// butterflies, then the waves in order, in fp64), computes the coefficients as fa_bwd_coef_from does and
// writes dx (and dz / dx2) from the registers: 6.125 B per element read / written once, one launch.
constexpr int CG_THREADS = 512;
template <bool DUAL>
constexpr int cg_np() { return DUAL ? 4 : 8; }  // pixels per thread (the dual form holds a third tensor)

template <bool DUAL>
__global__ void __launch_bounds__(CG_THREADS) bn_bwd_cg_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ mbits,
                                                            u16* dzo, const u16* __restrict__ x1, const BnBwdArgs a1,
                                                            u16* __restrict__ dx1, const u16* __restrict__ x2,
                                                            const BnBwdArgs a2, u16* __restrict__ dx2, int M, int C,
                                                            u64* ts) {
  __shared__ float wred[CG_THREADS / 64][24];
  __shared__ float coef[6][8];
  stamp_start(ts);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c0 = blockIdx.x * 8;
  constexpr int CG_NP = cg_np<DUAL>();
  uint4 vd[CG_NP], va[CG_NP], vb[CG_NP];
  uint32_t mk[CG_NP];
#pragma unroll
  for (int u = 0; u < CG_NP; ++u) {  // branch-free loads (clamped): all in flight together
    const int m = min(t + u * CG_THREADS, M - 1);
    const size_t o = (size_t)m * C + c0;
    vd[u] = *(const uint4*)(dy + o);
    va[u] = *(const uint4*)(x1 + o);
    if constexpr (DUAL) vb[u] = *(const uint4*)(x2 + o);
    mk[u] = mbits[o >> 3];
  }
  // the 8 channels' mean / invstd (both BNs) in LDS: broadcast reads, no 32 registers held across the loads
  __shared__ float mi[4][8];
  if (t < 32) {
    const int k = t & 7, w = t >> 3;
    const float* src = w == 0 ? a1.mean : w == 1 ? a1.invstd : w == 2 ? (DUAL ? a2.mean : a1.mean) : (DUAL ? a2.invstd : a1.invstd);
    mi[w][k] = src[c0 + k];
  }
  __syncthreads();
  float sd[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sd[k] = s1[k] = s2[k] = 0.f;
#pragma unroll
  for (int u = 0; u < CG_NP; ++u) {
    const bool ok = t + u * CG_THREADS < M;
    float d[8], a[8], b[8];
    unpack8(vd[u], d);
    unpack8(va[u], a);
    if constexpr (DUAL) unpack8(vb[u], b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d[k] = ok && ((mk[u] >> k) & 1u) ? d[k] : 0.f;
      sd[k] += d[k];
      s1[k] += d[k] * ((a[k] - mi[0][k]) * mi[1][k]);
      if constexpr (DUAL) s2[k] += d[k] * ((b[k] - mi[2][k]) * mi[3][k]);
    }
    vd[u] = pack8(d);  // dz (exact: masking is exact)
  }
  // fixed-order workgroup reduction: lane butterfly, then the waves in order (fp64)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float a = wave_sum(sd[k]), b = wave_sum(s1[k]);
    const float e = DUAL ? wave_sum(s2[k]) : 0.f;
    if (lane == 0) {
      wred[wave][k] = a;
      wred[wave][8 + k] = b;
      wred[wave][16 + k] = e;
    }
  }
  __syncthreads();
  if (t < 8) {
    double d = 0.0, x = 0.0, y = 0.0;
#pragma unroll
    for (int w = 0; w < CG_THREADS / 64; ++w) {
      d += wred[w][t];
      x += wred[w][8 + t];
      y += wred[w][16 + t];
    }
    const int c = c0 + t;
    const double cnt = (double)a1.count;
    {
      const double is = mi[1][t], a = (double)a1.gamma[c] * is, b = -a * is * x / cnt;
      coef[0][t] = (float)a;
      coef[1][t] = (float)b;
      coef[2][t] = (float)(-a * d / cnt - b * (double)mi[0][t]);
      if (a1.dgamma) a1.dgamma[c] = (float)(x * a1.gscale);
      if (a1.dbeta) a1.dbeta[c] = (float)(d * a1.gscale);
    }
    if constexpr (DUAL) {
      const double is = mi[3][t], a = (double)a2.gamma[c] * is, b = -a * is * y / cnt;
      coef[3][t] = (float)a;
      coef[4][t] = (float)b;
      coef[5][t] = (float)(-a * d / cnt - b * (double)mi[2][t]);
      if (a2.dgamma) a2.dgamma[c] = (float)(y * a2.gscale);
      if (a2.dbeta) a2.dbeta[c] = (float)(d * a2.gscale);
    }
  }
  __syncthreads();
  float A1[8], B1[8], C1[8], A2[8], B2[8], C2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A1[k] = coef[0][k]; B1[k] = coef[1][k]; C1[k] = coef[2][k];
    if constexpr (DUAL) {
      A2[k] = coef[3][k]; B2[k] = coef[4][k]; C2[k] = coef[5][k];
    }
  }
#pragma unroll
  for (int u = 0; u < CG_NP; ++u) {
    const int m = t + u * CG_THREADS;
    if (m >= M) break;
    const size_t o = (size_t)m * C + c0;
    float d[8], a[8], v[8];
    unpack8(vd[u], d);
    if (dzo != nullptr) *(uint4*)(dzo + o) = vd[u];
    unpack8(va[u], a);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = A1[k] * d[k] + B1[k] * a[k] + C1[k];
    *(uint4*)(dx1 + o) = pack8(v);
    if constexpr (DUAL) {
      unpack8(vb[u], a);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = A2[k] * d[k] + B2[k] * a[k] + C2[k];
      *(uint4*)(dx2 + o) = pack8(v);
    }
  }
  stamp_end(ts);
}

bool bn_bwd_cg_ok(int64_t M, int C, bool dual) {
  return M >= 1 && M <= (int64_t)CG_THREADS * (dual ? cg_np<true>() : cg_np<false>()) && C % 8 == 0 && C >= 8;
}

int bn_bwd_cg(const u16* dy, const uint8_t* mbits, u16* dzo, const u16* x1, const BnBwdArgs& a1, u16* dx1,
              const u16* x2, const BnBwdArgs* a2, u16* dx2, int64_t M, int C, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(dy && mbits && x1 && dx1 && a1.gamma && a1.mean && a1.invstd && M >= 1,
                "bn_bwd_cg: bad args (M=%lld C=%d)", (long long)M, C);
  DTC_CHECK_ARG(bn_bwd_cg_ok(M, C, x2 != nullptr), "bn_bwd_cg: M=%lld too large", (long long)M);
  DTC_CHECK_ARG(!x2 || (a2 && a2->gamma && a2->mean && a2->invstd && dx2), "bn_bwd_cg: dual branch args");
  const BnBwdArgs none{};
  if (x2)
    DTC_KLAUNCH(bn_bwd_cg_kernel<true>, dim3(C / 8), dim3(CG_THREADS), 0, st, dy, mbits, dzo, x1, a1, dx1, x2,
                       *a2, dx2, (int)M, C, ts);
  else
    DTC_KLAUNCH(bn_bwd_cg_kernel<false>, dim3(C / 8), dim3(CG_THREADS), 0, st, dy, mbits, dzo, x1, a1, dx1,
                       nullptr, none, nullptr, (int)M, C, ts);
  DTC_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ backward
// MASK: dz = dy * [ym > 0], stored. MB: dz = dy * mask bit (the forward's ReLU mask), not stored
// (bn_bwd_fin_apply_mask forms it again from the same bits): 4.125 B per element instead of 8.
template <bool MASK, bool DUAL, typename T, bool MB = false, int RU = 4>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const T* __restrict__ dy, const T* __restrict__ ym, const T* __restrict__ x1,
    const float* __restrict__ mean1, const float* __restrict__ invstd1, int64_t* __restrict__ acc1,
    const T* __restrict__ x2, const float* __restrict__ mean2, const float* __restrict__ invstd2,
    int64_t* __restrict__ acc2, T* __restrict__ dz, int64_t M, int C, int rows_per_block,
    const uint8_t* __restrict__ mbits = nullptr, u64* ts = nullptr) {
  typedef Elt<T> E;
  __shared__ float red[256 * 24];
  stamp_start(ts);
  const int tpr = C >> 3, rpp = 256 / tpr;
  const int t = threadIdx.x, g = t % tpr, rr = t / tpr;
  const int c0 = g * 8;
  float m1[8], i1[8], m2[8], i2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    m1[k] = mean1[c0 + k];
    i1[k] = invstd1[c0 + k];
    if constexpr (DUAL) {
      m2[k] = mean2[c0 + k];
      i2[k] = invstd2[c0 + k];
    }
  }
  float sd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t m_begin = (int64_t)blockIdx.x * rows_per_block;
  const int64_t m_end = std::min<int64_t>(M, m_begin + rows_per_block);
  // one row of this thread: the loaded operands -> the running sums (same order as a plain loop)
  auto accumulate = [&](int64_t o, const typename E::V& vd, uint32_t mk, const typename E::V& vy,
                        const typename E::V& va, const typename E::V& vb) {
    float d[8], a[8];
    E::unpack(vd, d);
    if constexpr (MB) {
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = (mk >> k) & 1u ? d[k] : 0.f;
    }
    if constexpr (MASK) {
      float yv[8];
      E::unpack(vy, yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
      E::st(dz + o, E::pack(d));  // exact: masking is exact
    }
    E::unpack(va, a);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sd[k] += d[k];
      s1[k] += d[k] * ((a[k] - m1[k]) * i1[k]);
    }
    if constexpr (DUAL) {
      float b[8];
      E::unpack(vb, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) s2[k] += d[k] * ((b[k] - m2[k]) * i2[k]);
    }
  };
  // RU rows per thread per round, all their loads issued before the first row's math: RU x the bytes in
  // flight of a load-use loop (RU = 1: it waited on every row, ~33 B per thread in flight -- the layer1
  // reductions ran at 3.6-4.2 TB/s against ~5.8 for the apply kernels, which already batch 4 rows)
  typename E::V vd[RU], vy[RU], va[RU], vb[RU];
  uint32_t mk[RU];
  int64_t m = m_begin + rr;
  for (; m + (RU - 1) * rpp < m_end; m += RU * rpp) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t o = (m + u * rpp) * C + c0;
      vd[u] = E::ld(dy + o);
      mk[u] = MB ? (uint32_t)mbits[o >> 3] : 0u;
      if constexpr (MASK) vy[u] = E::ld(ym + o);
      va[u] = E::ld(x1 + o);
      if constexpr (DUAL) vb[u] = E::ld(x2 + o);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) accumulate((m + u * rpp) * C + c0, vd[u], mk[u], vy[u], va[u], vb[u]);
  }
  for (; m < m_end; m += rpp) {
    const int64_t o = m * C + c0;
    vd[0] = E::ld(dy + o);
    mk[0] = MB ? (uint32_t)mbits[o >> 3] : 0u;
    if constexpr (MASK) vy[0] = E::ld(ym + o);
    va[0] = E::ld(x1 + o);
    if constexpr (DUAL) vb[0] = E::ld(x2 + o);
    accumulate(o, vd[0], mk[0], vy[0], va[0], vb[0]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[t * 24 + k] = sd[k];
    red[t * 24 + 8 + k] = s1[k];
    red[t * 24 + 16 + k] = s2[k];
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    const int gg = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f, e = 0.f;
    for (int r2 = 0; r2 < rpp; ++r2) {
      const float* q = red + (r2 * tpr + gg) * 24;
      a += q[k];
      b += q[8 + k];
      e += q[16 + k];
    }
    stat_add(acc1, C, c, a, b);
    if constexpr (DUAL) stat_add(acc2, C, c, a, e);
  }
  stamp_end(ts);
}

template <typename T>
static int bwd_reduce(const T* dy, const T* ymask, const T* x1, const float* mean1, const float* invstd1, int64_t* acc1,
                      const T* x2, const float* mean2, const float* invstd2, int64_t* acc2, T* dz, int64_t M, int C,
                      hipStream_t st) {
  DTC_CHECK_ARG(dy && x1 && mean1 && invstd1 && acc1 && C % 8 == 0 && C <= 2048 && M > 0, "bn_bwd_reduce: bad args");
  DTC_CHECK_ARG(!ymask || dz, "bn_bwd_reduce: masked reduce needs a dz output");
  const int tpr = C / 8, rpp = 256 / tpr;
  // 256..1024 workgroups of >= 16K elements where the tensor allows, each a whole number of passes
  int64_t rpb = std::max<int64_t>({(int64_t)rpp, (M + 1023) / 1024,
                                   std::min<int64_t>((16384 + C - 1) / C, (M + 255) / 256)});
  rpb = ((rpb + rpp - 1) / rpp) * rpp;
  const int blocks = ceil_div_i(M, rpb);
  const bool dual = x2 != nullptr;
  if (dual) DTC_CHECK_ARG(mean2 && invstd2 && acc2, "bn_bwd_reduce: dual branch args");
  const bool ru1 = option_get(OPT_BN_RED_UNROLL) <= 1;  // as the mask-bit path: 1 = the load-use loop
#define DTC_BR(MK_, D_)                                                                                          \
  if (ru1) DTC_KLAUNCH((bn_bwd_reduce_kernel<MK_, D_, T, false, 1>), dim3(blocks), dim3(256), 0, st, dy,  \
                              ymask, x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, dz, M, C, (int)rpb,     \
                              (const uint8_t*)nullptr, (u64*)nullptr);                                          \
  else DTC_KLAUNCH((bn_bwd_reduce_kernel<MK_, D_, T, false, 4>), dim3(blocks), dim3(256), 0, st, dy,      \
                          ymask, x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, dz, M, C, (int)rpb,         \
                          (const uint8_t*)nullptr, (u64*)nullptr)
  if (ymask && dual) { DTC_BR(true, true); }
  else if (ymask) { DTC_BR(true, false); }
  else if (dual) { DTC_BR(false, true); }
  else { DTC_BR(false, false); }
#undef DTC_BR
  DTC_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_reduce_mask(const u16* dy, const uint8_t* mbits, const u16* x1, const float* mean1, const float* invstd1,
                       int64_t* acc1, const u16* x2, const float* mean2, const float* invstd2, int64_t* acc2, int64_t M,
                       int C, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(dy && mbits && x1 && mean1 && invstd1 && acc1 && C % 8 == 0 && C <= 2048 && M > 0,
                "bn_bwd_reduce_mask: bad args");
  const int tpr = C / 8, rpp = 256 / tpr;
  // >= bn_red_elems elements per workgroup where that still leaves >= bn_red_blocks workgroups
  const int64_t elems = std::max(1024, option_get(OPT_BN_RED_ELEMS));
  const int64_t minblk = std::max(1, option_get(OPT_BN_RED_BLOCKS));
  int64_t rpb = std::max<int64_t>({(int64_t)rpp, (M + 1023) / 1024,
                                   std::min<int64_t>((elems + C - 1) / C, (M + minblk - 1) / minblk)});
  rpb = ((rpb + rpp - 1) / rpp) * rpp;
  const int blocks = ceil_div_i(M, rpb);
  if (x2) DTC_CHECK_ARG(mean2 && invstd2 && acc2, "bn_bwd_reduce_mask: dual branch args");
  const int ru = option_get(OPT_BN_RED_UNROLL);
#define DTC_BRM(D_, R_)                                                                                            \
  DTC_KLAUNCH((bn_bwd_reduce_kernel<false, D_, u16, true, R_>), dim3(blocks), dim3(256), 0, st, dy, nullptr, \
                     x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, nullptr, M, C, (int)rpb, mbits, ts)
  if (x2) {
    if (ru <= 1) DTC_BRM(true, 1);
    else if (ru == 2) DTC_BRM(true, 2);
    else DTC_BRM(true, 4);
  } else {
    if (ru <= 1) DTC_BRM(false, 1);
    else if (ru == 2) DTC_BRM(false, 2);
    else DTC_BRM(false, 4);
  }
#undef DTC_BRM
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void __launch_bounds__(256) bn_mask_apply_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ mbits,
                                                            u16* __restrict__ dz, int64_t nvec) {
  for (int64_t v = blockIdx.x * (int64_t)256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    float d[8];
    unpack8(*(const uint4*)(dy + v * 8), d);
    const uint32_t mk = mbits[v];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = (mk >> k) & 1u ? d[k] : 0.f;
    *(uint4*)(dz + v * 8) = pack8(d);
  }
}

int bn_mask_apply(const u16* dy, const uint8_t* mbits, u16* dz, int64_t M, int C, hipStream_t st) {
  DTC_CHECK_ARG(dy && mbits && dz && C % 8 == 0 && M > 0, "bn_mask_apply: bad args");
  const int64_t nvec = M * C / 8;
  DTC_KLAUNCH(bn_mask_apply_kernel, dim3((unsigned)std::min<int64_t>(4096, (nvec + 255) / 256)), dim3(256), 0, st,
                     dy, mbits, dz, nvec);
  DTC_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_reduce(const u16* dy, const u16* ymask, const u16* x1, const float* mean1, const float* invstd1,
                  int64_t* acc1, const u16* x2, const float* mean2, const float* invstd2, int64_t* acc2, u16* dz,
                  int64_t M, int C, hipStream_t st) {
  return bwd_reduce<u16>(dy, ymask, x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, dz, M, C, st);
}
int bn_bwd_reduce(const float* dy, const float* ymask, const float* x1, const float* mean1, const float* invstd1,
                  int64_t* acc1, const float* x2, const float* mean2, const float* invstd2, int64_t* acc2, float* dz,
                  int64_t M, int C, hipStream_t st) {
  return bwd_reduce<float>(dy, ymask, x1, mean1, invstd1, acc1, x2, mean2, invstd2, acc2, dz, M, C, st);
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(
    int64_t* __restrict__ acc, int C, double count, const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, float gscale, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ coef) {
  __shared__ int64_t red[FIN_GROUPS][FIN_CH];
  double sd, sx;
  if (!fin_sum_slots(acc, C, sd, sx, red)) return;
  const int c = blockIdx.x * FIN_CH + threadIdx.x;
  if (dgamma) dgamma[c] = (float)(sx * gscale);
  if (dbeta) dbeta[c] = (float)(sd * gscale);
  const double is = invstd[c];
  const double A = (double)gamma[c] * is;
  const double B = -A * is * sx / count;
  const double Cc = -A * sd / count - B * (double)mean[c];
  coef[c] = (float)A;
  coef[C + c] = (float)B;
  coef[2 * C + c] = (float)Cc;
}

int bn_bwd_finalize(int64_t* acc, int C, int64_t count, const float* gamma, const float* mean, const float* invstd,
                    float gscale, float* dgamma, float* dbeta, float* coef, hipStream_t st) {
  DTC_CHECK_ARG(acc && gamma && mean && invstd && coef && C > 0 && count > 0, "bn_bwd_finalize: bad args");
  DTC_KLAUNCH(bn_bwd_finalize_kernel, dim3(ceil_div_i(C, FIN_CH)), dim3(256), 0, st, acc, C, (double)count, gamma,
                     mean, invstd, gscale, dgamma, dbeta, coef);
  DTC_LAUNCH_CHECK();
  return 0;
}

template <bool DUAL, typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dz, const T* __restrict__ x1,
                                                          const float* __restrict__ coef1, T* __restrict__ dx1,
                                                          const T* __restrict__ x2, const float* __restrict__ coef2,
                                                          T* __restrict__ dx2, int64_t nvec, int C) {
  typedef Elt<T> E;
  const int cvec = C >> 3;
  for (int64_t v = blockIdx.x * (int64_t)256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cvec) * 8;
    float d[8], a[8], o[8];
    E::unpack(E::ld(dz + v * 8), d);
    E::unpack(E::ld(x1 + v * 8), a);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = coef1[c0 + k] * d[k] + coef1[C + c0 + k] * a[k] + coef1[2 * C + c0 + k];
    E::st(dx1 + v * 8, E::pack(o));
    if constexpr (DUAL) {
      E::unpack(E::ld(x2 + v * 8), a);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = coef2[c0 + k] * d[k] + coef2[C + c0 + k] * a[k] + coef2[2 * C + c0 + k];
      E::st(dx2 + v * 8, E::pack(o));
    }
  }
}

template <typename T>
static int bwd_apply(const T* dz, const T* x1, const float* coef1, T* dx1, const T* x2, const float* coef2, T* dx2,
                     int64_t M, int C, hipStream_t st) {
  DTC_CHECK_ARG(dz && x1 && coef1 && dx1 && C % 8 == 0 && M > 0, "bn_bwd_apply: bad args");
  const int64_t nvec = M * C / 8;
  const int blocks = (int)std::min<int64_t>(4096, (nvec + 255) / 256);
  if (x2) {
    DTC_CHECK_ARG(coef2 && dx2, "bn_bwd_apply: dual branch args");
    DTC_KLAUNCH((bn_bwd_apply_kernel<true, T>), dim3(blocks), dim3(256), 0, st, dz, x1, coef1, dx1, x2, coef2, dx2,
                       nvec, C);
  } else {
    DTC_KLAUNCH((bn_bwd_apply_kernel<false, T>), dim3(blocks), dim3(256), 0, st, dz, x1, coef1, dx1, x2, coef2,
                       dx2, nvec, C);
  }
  DTC_LAUNCH_CHECK();
  return 0;
}

int bn_bwd_apply(const u16* dz, const u16* x1, const float* coef1, u16* dx1, const u16* x2, const float* coef2,
                 u16* dx2, int64_t M, int C, hipStream_t st) {
  return bwd_apply<u16>(dz, x1, coef1, dx1, x2, coef2, dx2, M, C, st);
}
int bn_bwd_apply(const float* dz, const float* x1, const float* coef1, float* dx1, const float* x2, const float* coef2,
                 float* dx2, int64_t M, int C, hipStream_t st) {
  return bwd_apply<float>(dz, x1, coef1, dx1, x2, coef2, dx2, M, C, st);
}

// ---------------------------------------------------------------- SyncBN slot compaction
// Folds the slots into slot 0 (exact integer sums; lo carried into hi, so slot 0's lo word stays below 2^44
// and a SUM over ranks cannot overflow it) and zeroes the others: the collective then carries the header
// and slot 0 (DTC_STAT_HDR + 4 C words, contiguous) instead of every slot.
__global__ void bn_fold_slots_kernel(int64_t* __restrict__ st, int C) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;  // (statistic, channel)
  if (j >= 2 * C) return;
  const int stat = j / C, c = j - stat * C;
  int64_t hi = 0, lo = 0;
  for (int k = 0; k < DTC_STAT_SLOTS; ++k) {
    hi += st[stat_word(k, stat, 0, C) + c];
    lo += st[stat_word(k, stat, 1, C) + c];
  }
  st[stat_word(0, stat, 0, C) + c] = hi + (lo >> 44);
  st[stat_word(0, stat, 1, C) + c] = lo & ((1ll << 44) - 1);
  for (int k = 1; k < DTC_STAT_SLOTS; ++k) {
    st[stat_word(k, stat, 0, C) + c] = 0;
    st[stat_word(k, stat, 1, C) + c] = 0;
  }
}

int bn_fold_slots(int64_t* slots, int C, hipStream_t st) {
  DTC_CHECK_ARG(slots && C > 0, "bn_fold_slots: bad args");
  DTC_KLAUNCH(bn_fold_slots_kernel, dim3((2 * C + 255) / 256), dim3(256), 0, st, slots, C);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
