// BN coefficient helpers shared by the BN kernels (bn.hip) and the kernels that fuse a BN step into
// their prologue (stem.hip): the fixed-order fold of a BN's DTC_STAT_SLOTS fp64 partial-sum slots and the
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
  double a[DTC_STAT_SLOTS / 4], b[DTC_STAT_SLOTS / 4];  // this thread's 8 slots of (sum, second sum)
  float g = 0.f, h = 0.f, mu = 0.f;                    // t < 64: gamma and invstd / beta, mean
};

// thread t: channel cg + t%64, slots 8*(t/64) .. +7 (needs 256 threads)
__device__ __forceinline__ void fold_issue(const double* __restrict__ st, int C, int cg, SlotFold& f) {
  const int t = threadIdx.x, cl = t & 63, g = t >> 6;
#pragma unroll
  for (int j = 0; j < DTC_STAT_SLOTS / 4; ++j) {
    const size_t k = (size_t)(g * (DTC_STAT_SLOTS / 4) + j);
    f.a[j] = st[k * 2 * C + cg + cl];
    f.b[j] = st[k * 2 * C + C + cg + cl];
  }
}

// fixed-order fold: each group of 64 threads adds its 8 slots, then thread t < 64 adds the 4 groups
__device__ __forceinline__ void fold_sums(const SlotFold& f, double* part, double& s, double& q) {
  const int t = threadIdx.x, cl = t & 63, g = t >> 6;
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int j = 0; j < DTC_STAT_SLOTS / 4; ++j) {
    a += f.a[j];
    b += f.b[j];
  }
  part[(g * 2 + 0) * 64 + cl] = a;
  part[(g * 2 + 1) * 64 + cl] = b;
  lds_barrier();
  s = q = 0.0;
  if (t < 64) {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      s += part[(gg * 2 + 0) * 64 + t];
      q += part[(gg * 2 + 1) * 64 + t];
    }
  }
}

__device__ __forceinline__ void fa_slot_sums(const double* __restrict__ st, int C, int cg, double* part, double& s,
                                             double& q) {
  SlotFold f;
  fold_issue(st, C, cg, f);
  fold_sums(f, part, s, q);
}

// backward: dx = A*dz + B*x + Cc with the coefficients computed per workgroup from the fp64 slots of
// sum(dz), sum(dz*xhat); the first pixel block writes dgamma / dbeta (x gscale).
__device__ __forceinline__ void fold_issue_bwd(const BnBwdArgs& A, int C, int cg, SlotFold& f) {
  fold_issue(A.acc, C, cg, f);
  const int c = cg + (threadIdx.x & 63);  // every thread loads (no branch: see fold_issue's note)
  f.g = A.gamma[c];
  f.h = A.invstd[c];
  f.mu = A.mean[c];
}

__device__ __forceinline__ void fa_bwd_coef_from(const BnBwdArgs& A, const SlotFold& f, int C, int cg, double* part,
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

__device__ __forceinline__ void fa_bwd_coef(const BnBwdArgs& A, int C, int cg, double* part, float* ca, float* cb,
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

__device__ __forceinline__ void fa_fwd_coef_from(const BnFwdArgs& A, const SlotFold& f, int C, int cg, double* part,
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

__device__ __forceinline__ void fa_fwd_coef(const BnFwdArgs& A, int C, int cg, double* part, float* sc, float* sh) {
  SlotFold f;
  fold_issue_fwd(A, C, cg, f);
  fa_fwd_coef_from(A, f, C, cg, part, sc, sh);
}

}  // namespace dtc
