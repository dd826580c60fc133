// Internal host-side launcher declarations (C++). The public C ABI is include/dtc.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <algorithm>
#include "common.h"
#include "bnb_epi.h"

namespace dtc {

// ------------------------------------------------------------------ tuning options (atomic ints)
// X(ID, name, default): the live options only. Variants that measured negative or neutral were
// deleted with their code paths (round 4; their numbers are in DESIGN.md).
#define DTC_OPTION_LIST(X)                                                                                   \
  X(XCD_REMAP, xcd_remap, 1)            /* igemm: tiles sharing operands on one XCD */                       \
  X(DGRAD_CLASSES, dgrad_classes, 1)    /* stride-2 dgrad as output-parity classes */                        \
  X(WGRAD_FAST, wgrad_fast, 1)          /* igemm WGRAD fast loader */                                         \
  X(GRAPHS, graphs, 4)                  /* 0 eager, 1 fwd + bwd hipGraphs, 2 fwd only, 3 bwd only, 4 auto */ \
  X(WGRAD_HALO, wgrad_halo, 224)        /* target workgroups of the halo WGRAD kernel (0 = igemm only) */   \
  X(HALO_CONV, halo_conv, 1)            /* halo FWD/DGRAD for 3x3 s1: 0 off, 1 auto, 2+k force cfg k */     \
  X(HALO_SPLIT, halo_split, 0)          /* halo FWD/DGRAD split-K: 0 auto, k forced */                        \
  X(BWD_STREAMS, bwd_streams, 1)        /* weight gradients on a side stream beside the dgrad/BN chain */    \
  X(CONV_C64, conv_c64, 1)              /* persistent 64->64 3x3 conv for layer1: 1 >= a tile per workgroup, 2 always */           \
  X(BN_FUSED_FIN, bn_fused_fin, 1)      /* BN coefficients folded into the apply kernels */                   \
  X(WGRAD_BATCH, wgrad_batch, 4)        /* up to this many 3x3 s1 wgrads of a bucket per launch */            \
  X(BN_MASK, bn_mask, 1)                /* ReLU mask bits from the forward drive the BN backward */          \
  X(BARRIER_SPIN, barrier_spin, 1)      /* dtc_barrier: 1 poll the event, 0 hipEventSynchronize */           \
  X(STEM_DIRECT, stem_direct, 1)        /* (plan time) direct stem conv, 0 = im2col + GEMM */                 \
  X(WGRAD_XCD, wgrad_xcd, 1)            /* wgrad_halo: tiles of one (problem, split) on one XCD */           \
  X(WGRAD_DIRECT, wgrad_direct, 1)      /* wgrad_halo: a one-split launch writes the scaled dw itself */     \
  X(IGEMM_TILE, igemm_tile, 0)          /* igemm tile: 0 auto, 1 64x64, 2 128x128, 3 64x256 (tuning) */     \
  X(IGEMM_SPLIT, igemm_split, 0)        /* igemm split-K: 0 auto, k forced (tuning) */                        \
  X(DGRAD_CLASS_ORDER, dgrad_class_order, 1) /* stride-2 dgrad classes heaviest first */                      \
  X(STEM_PROLOGUE, stem_prologue, 1)    /* input copy + BN slot zeroing in one launch */                      \
  X(SC_COMPACT, sc_compact, 1)          /* shortcut dx at the stride-2 grid, added by conv1's dgrad */        \
  X(STEM_BN_FUSE, stem_bn_fuse, 1)      /* stem BN backward apply inside the stem weight gradient */          \
  X(BN_RED_ELEMS, bn_red_elems, 16384)  /* bn_bwd_reduce: target elements per workgroup (tuning) */           \
  X(BN_RED_BLOCKS, bn_red_blocks, 256)  /* ... while keeping at least this many workgroups (tuning) */        \
  X(BN_FA_BLOCKS, bn_fa_blocks, 1024)   /* BN fin_apply: target workgroups per launch (tuning) */             \
  X(FORK_LAZY, fork_lazy, 1)            /* fork the wgrad stream only where a wgrad launches */               \
  X(SIDE_PRIO, side_prio, 1)            /* (side stream creation) weight-gradient stream at low priority */  \
  X(SC_FUSE, sc_fuse, 1)                /* projection shortcut inside conv1's forward: 1 layer4, 2/3 wider */ \
  X(STEM_WLDS, stem_wlds, 1)            /* stem forward weight staged in LDS */                               \
  X(HALO_S2, halo_s2, 1)                /* stride-2 3x3 FWD on the column-split halo kernel */                \
  X(WGRAD_S2, wgrad_s2, 1)              /* stride-2 wgrad (+ shortcut) on the halo kernel: 0 off, 1 all, 2 GEN */ \
  X(WGRAD_S2_WGS, wgrad_s2_wgs, 128)    /* stride-2 halo wgrad: target workgroups (split-K slab = wgs x tile) */ \
  X(C64_WGS, c64_wgs, 256)              /* conv_c64 (layer1) persistent grid size */                          \
  X(WGRAD_HALO_L1, wgrad_halo_l1, 0)    /* wgrad_halo target for the one-tile (layer1) geometry (0: wgrad_halo) */ \
  X(DGRAD_SCF, dgrad_scf, 1)            /* shortcut dgrad fused into conv1's parity-class dgrad */            \
  X(BN_CG, bn_cg, 1)                    /* small BN backward as one launch (bn_bwd_cg) ...                  */ \
  X(BN_CG_ELEMS, bn_cg_elems, 262144)   /* ... for tensors of at most this many elements                    */ \
  X(HEAD_FUSED, head_fused, 1)          /* head backward in one launch: 1 always, 2 at <= 64 images */       \
  X(XENT_FUSE, xent_fuse, 1)            /* CrossEntropyLoss backward inside the head backward kernel */     \
  X(COMM_ON_SIDE, comm_on_side, 1)      /* bucket all-reduces on the weight-gradient stream (no comm stream) */ \
  X(BUCKET_TAIL, bucket_tail, 1)        /* (plan time) close the open bucket (>= 1 MB) after layer2.0 */      \
  X(WGRAD_GEN, wgrad_gen, 1)            /* wgrad_halo general step geometry (224x224 model) */                \
  X(WGRAD_TRIM, wgrad_trim, 1)          /* wgrad_halo: no zero-fill DMA for last-round rows past the halo */  \
  X(HALO_GEN, halo_gen, 1)              /* conv_halo general tile geometry (224x224 model) */                 \
  X(BN_RED_UNROLL, bn_red_unroll, 4)    /* bn_bwd_reduce: rows per thread whose loads go together */          \
  X(C64_GEN, c64_gen, 1)                /* conv_c64 general tiles (224x224 layer1) */                         \
  X(SPLITK_INK, splitk_ink, 1)          /* conv split-K summed by the last workgroup per tile (no reduce launch) */ \
  X(COMM_PRIO, comm_prio, 0)            /* (communicator creation) its own stream: 0 normal, 1 most urgent */ \
  X(COMM_TAIL_INLINE, comm_tail_inline, 1) /* the last bucket's all-reduce on the compute stream (no fork / join) */ \
  X(DGRAD_S2H, dgrad_s2h, 1)            /* stride-2 3x3 dgrad (+ shortcut) as a halo sub-pixel conv: 1 K <= 256, 2 all */ \
  X(HALO_SMALL, halo_small, 1)          /* halo FWD/DGRAD: 64x64 double-buffered tiles where they give <= 512 workgroups */

enum {
#define DTC_OPT_ENUM(id, name, def) OPT_##id,
  DTC_OPTION_LIST(DTC_OPT_ENUM)
#undef DTC_OPT_ENUM
  OPT_COUNT
};
int option_get(int id);
int option_set(const char* name, int value);
int option_epoch();  // bumped by every option_set (captured graphs bake the options in)

// ------------------------------------------------------------------ convolution
struct ConvShape {
  int N, H, W, C;  // input NHWC
  int K, R, S;     // filters KRSC
  int stride, pad;
};
enum { CONV_FWD = 0, CONV_DGRAD = 1, CONV_WGRAD = 2 };
struct ConvPlan {
  int bm, bn, splits, num_kt;
  size_t slab_bytes;  // fp32 workspace the plan wants (0 = none)
};
ConvPlan plan_conv(const ConvShape& s, int mode);

// y = conv(x, w) (bf16 NHWC out); optional BN statistics of the bf16 output into
// stats (sum, sum of squares; exact fixed-point accumulators, DTC_STAT_WORDS(K) int64: common.h).
// `ts` (optional, every conv launcher): a DTC_PROF_SLOT_U64 slot receiving the entry times of the
// first workgroups and every workgroup's exit time in s_memrealtime ticks (graph-safe per-call timing).
// tick (optional): >= DTC_TICKS zeroed u32 arrival counters reserved for the launch stream (the executor's
// workspace: one set per stream); with it a split-K conv reduces its slab inside the kernel (the last
// workgroup of each output tile), else a separate reduction launch does. The counters are left zero.
#define DTC_TICKS 8192
int conv_fwd(const ConvShape& s, const u16* x, const u16* w, u16* y, int64_t* stats, float* slab,
             size_t slab_bytes, hipStream_t st, u64* ts = nullptr, unsigned* tick = nullptr);
// 3x3 stride-2 conv and the 1x1 stride-2 projection shortcut of the same input in one launch
bool conv_fwd_sc_ok(const ConvShape& s, const ConvShape& sc);
int conv_fwd_sc(const ConvShape& s, const ConvShape& sc, const u16* x, const u16* w, u16* y, int64_t* stats,
                const u16* wsc, u16* ysc, int64_t* stats_sc, hipStream_t st, u64* ts = nullptr);
// dx = conv_transpose(dy, w) (+ res), bf16 NHWC.
// bnb (optional): dx is the gradient of a post-ReLU BN output; store dz = dx * [bnb->ym > 0] instead
// and accumulate the BN-backward sums (bn_bwd_reduce's work) -- in the epilogue where the kernel
// supports it (conv_c64, conv_halo, split-K reduce), else by a bn_bwd_reduce pass after the conv.
// dx may alias res (in place: each element is read and written by the same lane).
// true when conv_dgrad(s) takes the stride-2 parity-class path (the one a compact residual needs)
bool dgrad_class_ok(const ConvShape& s);
// res_compact: res is [N][H/2][W/2][C] (a 1x1 stride-2 shortcut's dx at its only nonzero parity),
// added at the (even, even) pixels only -- stride-2 parity-class dgrads.
// dx = dgrad(dy, w) + dgrad_1x1_s2(dsc, wsc) for a projection block's 3x3 stride-2 conv1 and its shortcut
// in one parity-class launch (dsc [N][H/2][W/2][K], wsc [K][C])
bool conv_dgrad_sc_ok(const ConvShape& s);
// stride-2 3x3 pad-1 dgrad as a halo-tiled sub-pixel convolution (dgrad_s2.hip), optionally + the 1x1 stride-2
// shortcut's dgrad (dsc [N][H/2][W/2][K], wsc [K][C]) at the even / even pixels
bool dgrad_s2_halo_ok(const ConvShape& s);
int conv_dgrad_s2_halo(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* dsc, const u16* wsc,
                       hipStream_t st, u64* ts = nullptr);
int conv_dgrad_sc(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* dsc, const u16* wsc,
                  hipStream_t st, u64* ts = nullptr, const BnbArgs* bnb = nullptr);
int conv_dgrad(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* res, float* slab,
               size_t slab_bytes, hipStream_t st, u64* ts = nullptr, const BnbArgs* bnb = nullptr,
               int res_compact = 0, unsigned* tick = nullptr);
// dw[k][0:dw_cols] (row stride dw_ld) = scale * sum_pixels dy (x) im2col(x); fp32
int conv_wgrad(const ConvShape& s, const u16* x, const u16* dy, float* dw, int dw_cols, int dw_ld, float scale,
               float* slab, size_t slab_bytes, hipStream_t st, u64* ts = nullptr);
// Halo-tiled WGRAD for 3x3 / stride 1 / pad 1 (wgrad_halo.hip): split count it would use for s
// batched nprob at a time (0 = not applicable / disabled), and the launch writing
// slab[nprob][used][K][9C] (reduce separately).
constexpr int DTC_WG_BATCH = 4;
int wgrad_halo_splits(const ConvShape& s, int nprob = 1);
// dw (optional): when the launch uses ONE split its epilogue writes dw[i] = scale * sum directly (no
// slab, no reduce; *used_splits = 0 tells the caller), else slab[nprob][used][K][9C] as above.
// 3x3 stride-2 weight gradient (conv1 of a projection block) on the column-split halo kernel, and with
// dsc != null the block's 1x1 stride-2 shortcut's (dw_sc[k][c] from dsc) in the same launch; split-K over
// output pixels into slab ([splits][K][9C] then [splits][K][C]) + deterministic reduces.
int wgrad_s2_splits(const ConvShape& s);  // 0: no plan (option wgrad_s2 off or geometry)
size_t conv_wgrad_s2_slab_bytes(const ConvShape& s);
int conv_wgrad_s2(const ConvShape& s, const u16* x, const u16* dy, const u16* dsc, float* dw, float* dw_sc,
                  float scale, float* slab, size_t slab_bytes, hipStream_t st, u64* ts = nullptr);
int conv_wgrad_halo(const ConvShape& s, int nprob, const u16* const* x, const u16* const* dy, float* slab, int splits,
                    int* used_splits, hipStream_t st, u64* ts, float* const* dw = nullptr, float scale = 1.f);
// nprob (<= DTC_WG_BATCH) independent weight gradients of one 3x3 stride-1 geometry in one halo
// launch + one reduce launch: dw[i] = scale * wgrad(x[i], dy[i]). Returns DTC_EINVAL when the
// geometry has no halo plan or the slab is too small (callers then issue them one by one).
size_t conv_wgrad_batch_slab_bytes(const ConvShape& s, int nprob);
int conv_wgrad_batch(const ConvShape& s, int nprob, const u16* const* x, const u16* const* dy, float* const* dw,
                     float scale, float* slab, size_t slab_bytes, hipStream_t st, u64* ts = nullptr);
// Halo-tiled 3x3 / stride 1 FWD and DGRAD (conv_halo.hip): configuration for the pass (-1: not
// applicable), and the launch (FWD: stats optional; DGRAD: res optional).
// Persistent 64-channel 3x3 stride-1 FWD / DGRAD (conv_c64.hip).
bool conv_c64_ok(const ConvShape& s);
int conv_c64(const ConvShape& s, int mode, const u16* src, const u16* w, u16* out, const u16* res, int64_t* stats,
             hipStream_t st, u64* ts);
struct HaloPlan {
  int cfg, split;
  int gen = 0;  // 1: general tile geometry (rows of seg columns, 64-bit tile bases; conv_halo.hip)
};
HaloPlan conv_halo_plan(const ConvShape& s, int mode);
size_t conv_halo_slab_bytes(const ConvShape& s, int mode);  // fp32 split-K slab the plan needs
int conv_halo(const ConvShape& s, int mode, const HaloPlan& hp, const u16* src, const u16* w, u16* out,
              const u16* res, int64_t* stats, float* slab, size_t slab_bytes, hipStream_t st, u64* ts = nullptr,
              const u16* wsc = nullptr, u16* out2 = nullptr, int64_t* stats2 = nullptr, unsigned* tick = nullptr);
// out = bf16(sum_s slab[s] (+ res)) (+ the BN statistics of out): the separate split-K reduction
int splitk_reduce(const float* slab, int splits, int M, int Nc, u16* out, const u16* res, int64_t* stats,
                  hipStream_t st, u64* ts = nullptr);
// per slot i of ts[n][DTC_PROF_SLOT_U64]: acc[i] += (max end - min start, 1) if stamped; cells reset
int prof_accumulate(u64* ts, int n, u64* acc, hipStream_t st);

// fp32 mode (conv_f32.hip): fp32 in / fp32 out implicit GEMM on v_mfma_f32_16x16x4_f32.
// FWD: out = y (+ BN stats into `stats`); DGRAD: out = dx (+ res); WGRAD: dw[k][0:dw_cols] (row stride
// dw_ld; 0 = R*S*C) = scale * sum over pixels, via split-K slabs in `slab`. C and K multiples of 16.
int conv_f32(const ConvShape& s, int mode, const float* a, const float* b, float* out, const float* res,
             int64_t* stats, float* dw, int dw_cols, int dw_ld, float scale, float* slab, size_t slab_bytes,
             hipStream_t st, u64* ts = nullptr);
size_t f32_conv_workspace(const ConvShape& s, int mode);  // fp32 slab bytes the pass wants
int f32_stem_im2col(const float* x, float* cols, int N, int H, int W, hipStream_t st);  // [N*H*W][32]
int f32_stem_pack_weight(const float* w27, float* w32, int K, hipStream_t st);          // [K][27] -> [K][32]

// ------------------------------------------------------------------ batch norm (NHWC, C channels, M pixels)
// forward finalize: mean/invstd/scale/shift from stats; running-stat update; stats re-zeroed.
int bn_fwd_finalize(int64_t* stats, int C, int64_t count, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, int64_t* num_batches, float momentum, float eps,
                    float* mean, float* invstd, float* scale, float* shift, hipStream_t st);
// eval mode: scale/shift from running statistics (mean/invstd also written for reference)
int bn_eval_coef(int C, const float* gamma, const float* beta, const float* running_mean, const float* running_var,
                 float eps, float* mean, float* invstd, float* scale, float* shift, hipStream_t st);
// y = relu(x*scale + shift)
int bn_apply_relu(const u16* x, const float* scale, const float* shift, u16* y, int64_t M, int C, hipStream_t st);
// y = relu(x*scale + shift + res)            (identity shortcut)
int bn_apply_add_relu(const u16* x, const float* scale, const float* shift, const u16* res, u16* y, int64_t M,
                      int C, hipStream_t st);
// y = relu(x*scale + shift + x2*scale2 + shift2)   (projection shortcut: two BNs)
int bn_apply_dual_relu(const u16* x, const float* scale, const float* shift, const u16* x2, const float* scale2,
                       const float* shift2, u16* y, int64_t M, int C, hipStream_t st);
// y = x*scale + shift (no activation; eval helpers / tests)
int bn_apply(const u16* x, const float* scale, const float* shift, u16* y, int64_t M, int C, hipStream_t st);
// fp32-activation versions of the four (fp32 mode: the reference without --amp)
int bn_apply_relu(const float* x, const float* scale, const float* shift, float* y, int64_t M, int C, hipStream_t st);
int bn_apply_add_relu(const float* x, const float* scale, const float* shift, const float* res, float* y, int64_t M,
                      int C, hipStream_t st);
int bn_apply_dual_relu(const float* x, const float* scale, const float* shift, const float* x2, const float* scale2,
                       const float* shift2, float* y, int64_t M, int C, hipStream_t st);
int bn_apply(const float* x, const float* scale, const float* shift, float* y, int64_t M, int C, hipStream_t st);

// Fused finalize + apply: the coefficients are computed by the consumer from the statistic slots
// (bn.hip); the first pixel block writes the saved / running statistics (forward) or dgamma /
// dbeta (backward). The slots must be zeroed before their producers run (executor: memset node).
struct BnFwdArgs {
  const int64_t* stats = nullptr;  // DTC_STAT_WORDS(C): sum, sum of squares of the bf16 conv output
  int64_t count = 0;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* rmean = nullptr;
  float* rvar = nullptr;
  int64_t* nbt = nullptr;
  float momentum = 0.1f, eps = 1e-5f;
  float* mean = nullptr;    // saved for backward
  float* invstd = nullptr;
};
struct BnBwdArgs {
  const int64_t* acc = nullptr;  // [SLOTS][2][C] sum(dz), sum(dz*xhat)
  int64_t count = 0;
  const float* gamma = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  float gscale = 1.f;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
};
// mode: 1 relu, 2 add residual x2 + relu, 3 dual BN (x2 normalised by a2) + relu
// mask (optional): ReLU mask bits of y (byte o/8 for element offset o) for the mask-bit backward
int bn_fin_apply(int mode, const u16* x, const BnFwdArgs& a1, const u16* x2, const BnFwdArgs* a2, u16* y, int64_t M,
                 int C, hipStream_t st, uint8_t* mask = nullptr, u64* ts = nullptr);
// Mask-bit BN backward (the executor's default): dz = dy * mask bit is formed where it is used, never
// stored by the reduction. Reduce: sums only (dy, bits, x read: 4.125 B/element); apply: dx (and
// dzo = dz if non-null, may alias dy) from dy, bits, x. bn_mask_apply: dz alone (parity captures).
int bn_bwd_reduce_mask(const u16* dy, const uint8_t* mbits, const u16* x1, const float* mean1, const float* invstd1,
                       int64_t* acc1, const u16* x2, const float* mean2, const float* invstd2, int64_t* acc2, int64_t M,
                       int C, hipStream_t st, u64* ts = nullptr);
int bn_bwd_fin_apply_mask(const u16* dy, const uint8_t* mbits, u16* dzo, const u16* x1, const BnBwdArgs& a1, u16* dx1,
                          const u16* x2, const BnBwdArgs* a2, u16* dx2, int64_t M, int C, hipStream_t st,
                          u64* ts = nullptr);
int bn_mask_apply(const u16* dy, const uint8_t* mbits, u16* dz, int64_t M, int C, hipStream_t st);
// One-launch mask-bit BN backward of a small tensor (bn_bwd_cg_ok: M <= 4096 pixels, 2048 dual): reduce +
// coefficients + apply (dz, dx1 [, dx2], dgamma / dbeta x gscale) in one workgroup per 8 channels; the
// statistic slots are unused
bool bn_bwd_cg_ok(int64_t M, int C, bool dual);
int bn_bwd_cg(const u16* dy, const uint8_t* mbits, u16* dzo, const u16* x1, const BnBwdArgs& a1, u16* dx1,
              const u16* x2, const BnBwdArgs* a2, u16* dx2, int64_t M, int C, hipStream_t st, u64* ts = nullptr);
int bn_bwd_fin_apply(const u16* dz, const u16* x1, const BnBwdArgs& a1, u16* dx1, const u16* x2, const BnBwdArgs* a2,
                     u16* dx2, int64_t M, int C, hipStream_t st);
int bn_fin_apply(int mode, const float* x, const BnFwdArgs& a1, const float* x2, const BnFwdArgs* a2, float* y,
                 int64_t M, int C, hipStream_t st);
int bn_bwd_fin_apply(const float* dz, const float* x1, const BnBwdArgs& a1, float* dx1, const float* x2,
                     const BnBwdArgs* a2, float* dx2, int64_t M, int C, hipStream_t st);

// slot 0 <- the exact sum over the slots (lo carried into hi), the others zeroed (SyncBN's collective)
int bn_fold_slots(int64_t* slots, int C, hipStream_t st);
// backward: dz = dy * [y > 0] (mask optional); accumulates sum(dz), sum(dz*xhat1) [, sum(dz*xhat2)]
int bn_bwd_reduce(const u16* dy, const u16* ymask, const u16* x1, const float* mean1, const float* invstd1,
                  int64_t* acc1, const u16* x2, const float* mean2, const float* invstd2, int64_t* acc2, u16* dz,
                  int64_t M, int C, hipStream_t st);
int bn_bwd_reduce(const float* dy, const float* ymask, const float* x1, const float* mean1, const float* invstd1,
                  int64_t* acc1, const float* x2, const float* mean2, const float* invstd2, int64_t* acc2, float* dz,
                  int64_t M, int C, hipStream_t st);
// dgamma/dbeta (scaled by gscale) into the flat grad buffer; apply coefficients coef[3][C]; acc re-zeroed.
int bn_bwd_finalize(int64_t* acc, int C, int64_t count, const float* gamma, const float* mean,
                    const float* invstd, float gscale, float* dgamma, float* dbeta, float* coef, hipStream_t st);
// dx1 = A1*dz + B1*x1 + C1 [; dx2 = A2*dz + B2*x2 + C2]
int bn_bwd_apply(const u16* dz, const u16* x1, const float* coef1, u16* dx1, const u16* x2, const float* coef2,
                 u16* dx2, int64_t M, int C, hipStream_t st);
int bn_bwd_apply(const float* dz, const float* x1, const float* coef1, float* dx1, const float* x2, const float* coef2,
                 float* dx2, int64_t M, int C, hipStream_t st);

// ------------------------------------------------------------------ stem / head / loss
// x fp32 NCHW [N][3][H][W] -> im2col bf16 [N*H*W][64] (3x3 pad 1 taps, (r,s,c) order, zero padded)
int stem_im2col(const float* x, u16* cols, int N, int H, int W, hipStream_t st);
// w bf16 [64][27] -> [64][64] zero padded
int stem_pack_weight(const u16* w27, u16* w64, int K, hipStream_t st);
// Direct stem conv (stem.hip): im2col gathered into LDS per 256-pixel tile, one K=32 MFMA k-step.
// fwd: y [N*H*W][64] bf16 (+ BN statistics of the bf16 output into stats[SLOTS][2][64] if non-null)
// from fp32 NCHW x and the bf16 [64][27] weight; wgrad: dw27 [64][27] fp32 = scale * sum.
int stem_fwd(const float* x, const u16* w27, u16* y, int64_t* stats, int N, int H, int W, hipStream_t st,
             u64* ts = nullptr);
size_t stem_wgrad_slab_bytes(int64_t M);
int stem_wgrad(const float* x, const u16* dy, float* dw27, float scale, int N, int H, int W, float* slab,
               size_t slab_bytes, hipStream_t st, u64* ts = nullptr);
// stem weight gradient with the stem BN's backward apply fused: dc = A*(dy*bit) + B*c + Cc formed per
// tile in LDS from (dy, mask bits, the conv output c) and the BN's slots (a: as bn_bwd_fin_apply's)
int stem_wgrad_bn(const float* x, const u16* dy, const uint8_t* mbits, const u16* c, const BnBwdArgs& a, float* dw27,
                  float scale, int N, int H, int W, float* slab, size_t slab_bytes, hipStream_t st, u64* ts = nullptr);
// grad[k][0:ncols] (row stride ldo) = scale * sum_s slab[s][k][0:RSC] (igemm.hip's deterministic reduce)
int wgrad_reduce_to(const float* slab, int splits, int K, int RSC, int ncols, int ldo, float scale, float* dw,
                    hipStream_t st, u64* ts = nullptr);
int wgrad_reduce_pair(const float* slab, int splits, int K, int ld0, float* dw0, size_t stride, int ld1, float* dw1,
                      float scale, hipStream_t st, u64* ts = nullptr);
// feat[n][c] = bf16round(mean_hw act); logits[n][j] = feat . W[j] + b[j]
int head_fwd(const u16* act, int N, int HW, int C, const u16* wfc, const float* bfc, int ncls, float* feat,
             float* logits, hipStream_t st);
// mean cross entropy; lse per row
// the same plus loss * (*scale) into `scaled` and the loss into the host word `host` (optional), one launch
int xent_fwd_fused(const float* logits, const int64_t* labels, int N, int ncls, float* loss, float* lse,
                   const float* scale, float* scaled, float* host, hipStream_t st);
int xent_fwd(const float* logits, const int64_t* labels, int N, int ncls, float* loss, float* lse,
             hipStream_t st);
// dlogits = (softmax - onehot) * (*gscale) / N
int xent_bwd(const float* logits, const int64_t* labels, const float* lse, const float* gscale, int N, int ncls,
             float* dlogits, hipStream_t st);
// dW = scale*dlogits^T feat ; db = scale*sum dlogits ; dact[n][hw][c] = (dlogits . W)[c] / HW
size_t head_bwd_workspace(int N, int C, int ncls);
// fp32 mode: fp32 activations and fp32 Linear weights, no autocast rounding
int head_fwd(const float* act, int N, int HW, int C, const float* wfc, const float* bfc, int ncls, float* feat,
             float* logits, hipStream_t st);
// xa != nullptr: the CrossEntropyLoss backward is fused in -- dlogits is computed from (logits, labels,
// lse, gscale) exactly as xent_bwd does, used directly, and also stored into `dlogits` (an output then)
struct XentArgs {
  const float* logits = nullptr;
  const int64_t* labels = nullptr;
  const float* lse = nullptr;
  const float* gscale = nullptr;
};
int head_bwd(const float* dlogits, const float* feat, const float* wfc, int N, int HW, int C, int ncls, float scale,
             float* dw, float* db, float* dact, float* ws, size_t ws_bytes, hipStream_t st,
             const XentArgs* xa = nullptr);
int head_bwd(const float* dlogits, const float* feat, const u16* wfc, int N, int HW, int C, int ncls, float scale,
             float* dw, float* db, u16* dact, float* ws, size_t ws_bytes, hipStream_t st, const XentArgs* xa = nullptr);

// ------------------------------------------------------------------ optimizer / amp / casts
// Nesterov SGD over a flat buffer (torch.optim.SGD semantics, dampening 0).
int sgd_nesterov(float* p, const float* g, float* mom, u16* p_bf16, int64_t n, float lr, float wd, float mu,
                 const float* inv_scale, const int* found_inf, hipStream_t st);
int cast_f32_bf16(const float* src, u16* dst, int64_t n, hipStream_t st);
// zero an 8-byte aligned range (a kernel node, unlike hipMemsetAsync's fill dispatch)
int zero_bytes(void* p, size_t bytes, hipStream_t st);
// dst[0:bytes] = src[0:bytes] (16-B aligned) and zp[0:zbytes] = 0 (8-B aligned), one launch
int copy_and_zero(const void* src, void* dst, size_t bytes, void* zp, size_t zbytes, hipStream_t st);
// x[i] *= f (loopback test communicator)
int scale_f32(float* x, int64_t n, float f, hipStream_t st);
int scale_f64(double* x, int64_t n, double f, hipStream_t st);
int scale_i64(int64_t* x, int64_t n, int64_t f, hipStream_t st);
// thread-group communicator: every rank's buffer <- the rank-ordered sum of all (fp32 dtype 0 / int64 2 /
// fp64 3)
#define DTC_GROUP_MAX 8
struct GroupPtrs { void* p[DTC_GROUP_MAX]; };
int group_sum(const GroupPtrs& g, int w, int64_t n, int dtype, hipStream_t st);
// dst[i] += src[i] (DataParallel reduce-add of replicas sharing a device)
int add_f32(float* dst, const float* src, int64_t n, hipStream_t st);
int amp_check_finite(const float* g, int64_t n, int* found_inf, hipStream_t st);
int amp_scale(const float* x, const float* scale, float* out, int64_t n, hipStream_t st);  // out = x * (*scale)
int amp_update_scale(float* scale, float* inv_scale, int* growth_tracker, int* found_inf, float growth,
                     float backoff, int interval, hipStream_t st);

// ------------------------------------------------------------------ input pipeline
// gather + RandomCrop(pad) + RandomHorizontalFlip + ToTensor + Normalize: uint8 [N][h][w][3] ->
// fp32 [n][3][h][w]; crop = [n][2] offsets (NULL: centre), flip = [n] (NULL: none).
int cifar_augment(const uint8_t* images, const int64_t* targets, int64_t n_images, const int64_t* index,
                  const uint8_t* crop, const uint8_t* flip, int n, int h, int w, int pad, const float* mean,
                  const float* stdv, float* out, int64_t* labels, int* status, hipStream_t st);

}  // namespace dtc
