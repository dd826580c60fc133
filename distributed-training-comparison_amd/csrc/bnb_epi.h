// Fused BatchNorm-backward prologue for the data-gradient epilogues (conv_c64.hip, conv_halo.hip,
// igemm.hip incl. splitk_reduce).
//
// In the executor's backward every data gradient a conv produces is the gradient dy of a post-ReLU
// BN output, y = relu(bn(x) [+ shortcut]) (reference src/*/net.py:41-44, 108). The unfused path
// stores dy and then runs bn_bwd_reduce (bn.hip): read dy, y and x, store dz = dy * [y > 0], add
// sum(dz) and sum(dz * xhat) into fp64 slots. Here the dgrad epilogue does that work on the value
// it already holds: it rounds dy to bf16 (the unfused store), masks it with y, stores dz in place of
// dy and accumulates the two per-channel sums (a second BN sharing dz for a projection block's
// shortcut branch). Per element this saves the dy store + reload and dz reload of the separate
// kernel; the sums take the route of the forward statistics (per lane, DPP row of 16 pixels, LDS
// across waves, one fp64 atomic per channel per workgroup into slot blockIdx & 31).
#pragma once
#include "common.h"

namespace dtc {

struct BnbArgs {
  const u16* ym = nullptr;  // post-ReLU activation y (mask source); null (and mb null): plain dgrad epilogue
  // the forward's ReLU mask bits of y instead (option bnb_mask; bit e & 7 of byte e >> 3 for element e):
  // 1/16 of ym's bytes
  const uint8_t* mb = nullptr;
  const u16* x1 = nullptr;  // input of the (first) BN: the conv output it normalised
  const float* mean1 = nullptr;
  const float* invstd1 = nullptr;
  double* acc1 = nullptr;  // [SLOTS][2][C]: sum dz, sum dz * xhat
  const u16* x2 = nullptr;  // second BN sharing dz (projection shortcut) or null
  const float* mean2 = nullptr;
  const float* invstd2 = nullptr;
  double* acc2 = nullptr;
};

__host__ __device__ __forceinline__ bool bnb_on(const BnbArgs& a) { return a.ym != nullptr || a.mb != nullptr; }

// The 4 ReLU-mask bits of the elements o .. o + 3 (o % 4 == 0) as y-like values (1.0 = kept, 0 = masked).
__device__ __forceinline__ uint2 bnb_bits_as_y(const uint8_t* mb, size_t o) {
  const uint32_t nib = (uint32_t)(mb[o >> 3] >> (o & 4)) & 15u;
  // bf16 1.0 = 0x3F80 in the lanes whose bit is set
  return uint2{((nib & 1u) ? 0x3F80u : 0u) | ((nib & 2u) ? 0x3F800000u : 0u),
               ((nib & 4u) ? 0x3F80u : 0u) | ((nib & 8u) ? 0x3F800000u : 0u)};
}

// Per-lane state for 4 consecutive channels (one MFMA output row group of a fragment column).
struct Bnb4 {
  float m1[4], i1[4], m2[4], i2[4];
  float s[4], q1[4], q2[4];
};

__device__ __forceinline__ void bnb4_init(const BnbArgs& a, int c, bool dual, Bnb4& b) {
  const f32x4 m = *(const f32x4*)(a.mean1 + c), i = *(const f32x4*)(a.invstd1 + c);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    b.m1[t] = m[t];
    b.i1[t] = i[t];
    b.s[t] = b.q1[t] = b.q2[t] = 0.f;
    b.m2[t] = b.i2[t] = 0.f;
  }
  if (dual) {
    const f32x4 m2 = *(const f32x4*)(a.mean2 + c), i2 = *(const f32x4*)(a.invstd2 + c);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      b.m2[t] = m2[t];
      b.i2[t] = i2[t];
    }
  }
}

// v: the 4 values the epilogue would store, rounded to bf16 here and masked: they become dz.
// y / x / x2: the 4 bf16 values of the mask source and the BN inputs at the same (pixel, channels).
__device__ __forceinline__ void bnb4_vals(uint2 y, uint2 x, uint2 x2, bool valid, bool dual, float v[4], Bnb4& b) {
  const float yv[4] = {bf_lo(y.x), bf_hi(y.x), bf_lo(y.y), bf_hi(y.y)};
  const float xv[4] = {bf_lo(x.x), bf_hi(x.x), bf_lo(x.y), bf_hi(x.y)};
  const float xw[4] = {bf_lo(x2.x), bf_hi(x2.x), bf_lo(x2.y), bf_hi(x2.y)};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    v[t] = yv[t] > 0.f ? round_bf(v[t]) : 0.f;  // exact: masking a bf16 value
    const float d = valid ? v[t] : 0.f;
    b.s[t] += d;
    b.q1[t] += d * ((xv[t] - b.m1[t]) * b.i1[t]);
    if (dual) b.q2[t] += d * ((xw[t] - b.m2[t]) * b.i2[t]);
  }
}

// The same with the operands loaded from global memory at element offset `o` (pixel, first channel).
__device__ __forceinline__ void bnb4_apply(const BnbArgs& a, size_t o, bool valid, bool dual, float v[4], Bnb4& b) {
  uint2 y{0u, 0u}, x{0u, 0u}, x2{0u, 0u};
  if (valid) {
    y = a.mb ? bnb_bits_as_y(a.mb, o) : *(const uint2*)(a.ym + o);
    x = *(const uint2*)(a.x1 + o);
    if (dual) x2 = *(const uint2*)(a.x2 + o);
  }
  bnb4_vals(y, x, x2, valid, dual, v, b);
}

// Sum over the 16 pixel lanes of each DPP row (every lane of a row holds the same 4 channels).
__device__ __forceinline__ void bnb4_rowsum(Bnb4& b, bool dual) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    b.s[t] = row16_sum(b.s[t]);
    b.q1[t] = row16_sum(b.q1[t]);
    if (dual) b.q2[t] = row16_sum(b.q2[t]);
  }
}

// Final per-channel add of a workgroup's channel totals into the fp64 slots.
__device__ __forceinline__ void bnb_commit(const BnbArgs& a, int C, int c, float s, float q1, float q2, bool dual) {
  const size_t slot = (size_t)(blockIdx.x & (DTC_STAT_SLOTS - 1)) * 2 * C;
  unsafeAtomicAdd(a.acc1 + slot + c, (double)s);
  unsafeAtomicAdd(a.acc1 + slot + C + c, (double)q1);
  if (dual) {
    unsafeAtomicAdd(a.acc2 + slot + c, (double)s);
    unsafeAtomicAdd(a.acc2 + slot + C + c, (double)q2);
  }
}

}  // namespace dtc
