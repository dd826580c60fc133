// BN coefficient helpers shared by the BN kernels (bn.hip) and the kernels that fuse a BN step into
// their prologue (stem.hip): the fold of a BN's DTC_STAT_SLOTS fixed-point partial-sum slots (common.h) and the
// backward coefficients computed from it.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dtc {

// LDS-only workgroup barrier for the coefficient folds: __syncthreads() also waits for every
// outstanding global load (vmcnt(0) before the s_barrier), which would serialise the data loads a
// kernel issues above its fold behind the fold; this waits for LDS (and scalar) traffic only. Global
// values read after it are ordered by the compiler's own per-use vmcnt waits.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// A fold's global loads, issued by the caller AHEAD of its own data loads: vmcnt counts loads in
// issue order, so fold loads issued after the data would make the fold wait for the data too. Loads
// on both sides are branch-free (clamped addresses): a load inside a divergent region is waited for
// at the region's end, which would drain every load issued before it.
struct SlotFold {
  int64_t w[DTC_STAT_SLOTS];  // this thread's word (statistic, hi / lo) of its channel in every slot
  int64_t flag = 0;           // the accumulator's non-finite flag (common.h)
  float g = 0.f, h = 0.f, mu = 0.f;  // t < 64: gamma and invstd / beta, mean
};

// thread t: channel cg + t%64, word t/64 (0 / 1: first statistic hi / lo, 2 / 3: second) of every slot
// (needs 256 threads)
__device__ __forceinline__ void fold_issue(const int64_t* __restrict__ st, int C, int cg, SlotFold& f) {
  const int t = threadIdx.x, cl = t & 63, wd = t >> 6;
#pragma unroll
  for (int k = 0; k < DTC_STAT_SLOTS; ++k) f.w[k] = st[stat_word(k, wd >> 1, wd & 1, C) + cg + cl];
  f.flag = st[0];
}

// exact integer sums over the slots (any order gives the same bits), then thread t < 64 forms its
// channel's two totals; part: 256 words of LDS
__device__ __forceinline__ void fold_sums(const SlotFold& f, int64_t* part, double& s, double& q) {
  const int t = threadIdx.x;
  int64_t a = 0;
#pragma unroll
  for (int k = 0; k < DTC_STAT_SLOTS; ++k) a += f.w[k];
  part[t] = a;
  lds_barrier();
  s = q = 0.0;
  if (t < 64) {
    s = stat_total(part[t], part[64 + t], f.flag);
    q = stat_total(part[128 + t], part[192 + t], f.flag);
  }
}

__device__ __forceinline__ void fa_slot_sums(const int64_t* __restrict__ st, int C, int cg, int64_t* part, double& s,
                                             double& q) {
  SlotFold f;
  fold_issue(st, C, cg, f);
  fold_sums(f, part, s, q);
}

// backward: dx = A*dz + B*x + Cc with the coefficients computed per workgroup from the slots of
// sum(dz), sum(dz*xhat); the first pixel block writes dgamma / dbeta (x gscale).
__device__ __forceinline__ void fold_issue_bwd(const BnBwdArgs& A, int C, int cg, SlotFold& f) {
  fold_issue(A.acc, C, cg, f);
  const int c = cg + (threadIdx.x & 63);  // every thread loads (no branch: see fold_issue's note)
  f.g = A.gamma[c];
  f.h = A.invstd[c];
  f.mu = A.mean[c];
}

__device__ __forceinline__ void fa_bwd_coef_from(const BnBwdArgs& A, const SlotFold& f, int C, int cg, int64_t* part,
                                                 float* ca, float* cb, float* cc) {
  double sd, sx;
  fold_sums(f, part, sd, sx);
  const int t = threadIdx.x;
  if (t < 64) {
    const int c = cg + t;
    const double cnt = (double)A.count;
    const double is = f.h;
    const double a = (double)f.g * is;
    const double b = -a * is * sx / cnt;
    ca[t] = (float)a;
    cb[t] = (float)b;
    cc[t] = (float)(-a * sd / cnt - b * (double)f.mu);
    if (blockIdx.x == 0) {
      if (A.dgamma) A.dgamma[c] = (float)(sx * A.gscale);
      if (A.dbeta) A.dbeta[c] = (float)(sd * A.gscale);
    }
  }
  lds_barrier();
}

__device__ __forceinline__ void fa_bwd_coef(const BnBwdArgs& A, int C, int cg, int64_t* part, float* ca, float* cb,
                                            float* cc) {
  SlotFold f;
  fold_issue_bwd(A, C, cg, f);
  fa_bwd_coef_from(A, f, C, cg, part, ca, cb, cc);
}

// forward: scale / shift from the slots of sum(x), sum(x^2); the first pixel block writes the saved
// mean / invstd and the running statistics (and num_batches_tracked once)
__device__ __forceinline__ void fold_issue_fwd(const BnFwdArgs& A, int C, int cg, SlotFold& f) {
  fold_issue(A.stats, C, cg, f);
  const int c = cg + (threadIdx.x & 63);
  f.g = A.gamma[c];
  f.h = A.beta[c];
}

__device__ __forceinline__ void fa_fwd_coef_from(const BnFwdArgs& A, const SlotFold& f, int C, int cg, int64_t* part,
                                                 float* sc, float* sh) {
  double s, q;
  fold_sums(f, part, s, q);
  const int t = threadIdx.x;
  if (t < 64) {
    const int c = cg + t;
    const double cnt = (double)A.count;
    const double mu = s / cnt;
    double var = q / cnt - mu * mu;
    if (var < 0.0) var = 0.0;
    const float is = (float)(1.0 / sqrt(var + (double)A.eps));
    const float a = f.g * is;
    sc[t] = a;
    sh[t] = f.h - (float)mu * a;
    if (blockIdx.x == 0) {
      A.mean[c] = (float)mu;
      A.invstd[c] = is;
      if (A.rmean) {
        const double unbiased = cnt > 1.0 ? var * cnt / (cnt - 1.0) : var;
        A.rmean[c] = (float)((1.0 - A.momentum) * A.rmean[c] + A.momentum * mu);
        A.rvar[c] = (float)((1.0 - A.momentum) * A.rvar[c] + A.momentum * unbiased);
      }
      if (t == 0 && blockIdx.y == 0 && A.nbt) *A.nbt += 1;
    }
  }
  lds_barrier();
}

__device__ __forceinline__ void fa_fwd_coef(const BnFwdArgs& A, int C, int cg, int64_t* part, float* sc, float* sh) {
  SlotFold f;
  fold_issue_fwd(A, C, cg, f);
  fa_fwd_coef_from(A, f, C, cg, part, sc, sh);
}

}  // namespace dtc
