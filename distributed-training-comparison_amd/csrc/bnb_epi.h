// BatchNorm-backward arguments of a data gradient (conv_dgrad's `bnb`, dtc_conv2d_dgrad_bn): in the
// executor's backward every data gradient a conv produces is the gradient dy of a post-ReLU BN output,
// y = relu(bn(x) [+ shortcut]) (reference src/*/net.py:41-44, 108); with these arguments the conv is followed
// by that BN's backward reduction (bn_bwd_reduce / _mask, bn.hip: sum(dz), sum(dz * xhat) into fp64 slots).
// (Rounds 3-4 also accumulated the sums in the dgrad epilogues -- options bnb_fuse / bnb_mask -- which
// measured slower than the separate pass in-step and were removed in round 5: DESIGN.md.)
#pragma once
#include "common.h"

namespace dtc {

struct BnbArgs {
  const u16* ym = nullptr;  // post-ReLU activation y (mask source); null (and mb null): plain dgrad epilogue
  // the forward's ReLU mask bits of y instead (bit e & 7 of byte e >> 3 for element e): 1/16 of ym's bytes
  const uint8_t* mb = nullptr;
  const u16* x1 = nullptr;  // input of the (first) BN: the conv output it normalised
  const float* mean1 = nullptr;
  const float* invstd1 = nullptr;
  int64_t* acc1 = nullptr;  // [SLOTS][2][C]: sum dz, sum dz * xhat
  const u16* x2 = nullptr;  // second BN sharing dz (projection shortcut) or null
  const float* mean2 = nullptr;
  const float* invstd2 = nullptr;
  int64_t* acc2 = nullptr;
};

__host__ __device__ __forceinline__ bool bnb_on(const BnbArgs& a) { return a.ym != nullptr || a.mb != nullptr; }

}  // namespace dtc
