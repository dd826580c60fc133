// Halo-tiled weight gradient for 3x3 / stride 1 / pad 1 convolutions on bf16 MFMA (gfx950).
//
// Replaces the weight-gradient half of `nn.Conv2d.backward` (reference src/*/net.py:18-24,
// 29-35) for every 3x3 stride-1 conv of ResNet-18 (13 of the 20 convs). The generic WGRAD
// loader (igemm.hip) gives each workgroup one tap, so x and dy are re-read from L2 once per tap
// (9x); here a workgroup owns ALL nine taps of a 64-channel input slice:
//
//   D[(r,s,c)][k] (576 x 64) += sum over a 64-pixel step of x(p+r-1, q+s-1, c0+c) * dy(p, q, k0+k)
//
// Per step the x rows the 64 output pixels touch are staged ONCE as a zero-padded halo
// ((rows+2) x (W+2) pixels, 128-B rows of 64 channels, padding zero-filled by out-of-range
// buffer offsets) and every tap reads it shifted by r*(W+2)+s rows. L2->LDS traffic per step:
// <= 24 KiB halo + 8 KiB dy for 4.7 MFLOP (~180 FLOP/B, vs ~32 for one tap per workgroup).
// Operands are read with ds_read_b64_tr_b16 (pixels are the MFMA reduction index); the tr
// swizzle is a function of the LDS row, so shifted tap windows stay bank-conflict-free.
// 8 waves: 4 along the 576 rows (9 fragments each) x 2 along the 64 output channels.
// Pixel steps are split across workgroups; each writes an fp32 slab [split][K][RSC] that the
// shared deterministic wgrad_reduce kernel (igemm.hip) sums and scales.
// Batched launches (blockIdx.z = problem): up to DTC_WG_BATCH independent weight gradients of one
// geometry (the executor defers the 3x3 wgrads of a bucket and issues them together). The chip is
// filled by problems x splits workgroups, so each problem needs 1/P of the splits: the fp32 slab
// written and re-read per conv -- the cost that bounds this kernel beside the MFMAs -- drops P-fold.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "tile_common.h"

namespace dtc {

struct HaloParams {
  const u16* xs[DTC_WG_BATCH];   // per problem: NHWC [N][H][W][C]
  const u16* dys[DTC_WG_BATCH];  // per problem: NPQK [N][H][W][K] (stride 1, pad 1: P = H, Q = W)
  float* slab;     // [problem][splits][K][9*C]
  float* dws[DTC_WG_BATCH];  // direct: per problem dw [K][9*C] (one split: no slab, no reduce)
  float scale;     // direct: dw = scale * sum
  int direct;
  size_t slab_stride;  // floats per problem
  int N, H, W, C, K;
  uint32_t x_bytes;
  FastDiv fd_hw, fd_w;
  int steps_per_split, nsteps;
  int rs, hb, nh;  // output rows per image per step, halo rows per image block, halo rows per step
  int spi;         // pixels per image block of a step (rs * W)
  int xcd;         // 1: XCD-grouped decode of the workgroup id (wg_coords)
  u64* ts;
  // halo row pitch (stride 1: W + 2) and output dims (stride 1: H, W); stride 2 (ST = 2): the x halo is
  // column-split as in conv_halo.hip (padded column 2j at j, 2j + 1 at hwh + j), so the 64 output pixels
  // of a step read consecutive halo rows for every tap and the tr-read swizzle stays conflict-free
  int pitch, hwh, ho, wo;
  // SC (stride 2): the block's 1x1 stride-2 projection shortcut's weight gradient in the same launch --
  // dW_sc[k][c] = sum_p dsc[p][k] x[2p][c] is the centre tap (r, s) = (1, 1) of conv1's A operand
  // against a second dy tile (dsc): one extra 64-pixel DMA and 2 MFMAs per k-step and wave
  const u16* dsc;
  float* slab_sc;  // [splits][K][C] (or, direct, dw_sc)
  float* dw_sc;
  // general geometry (GEN kernels; stride 1, e.g. the 224x224 model's 224/112/56/28-wide rows): a step is
  // rs rows x seg columns of one image (rs * seg <= 64 real pixels; the remaining MFMA reduction slots of
  // the 64-pixel step carry zero dy), its halo (rs + 2) x (seg + 2) pixels; every step addresses x and dy
  // from a 64-bit per-step base, so an activation may exceed 2 GB (512 x 224 x 224 x 64 bf16 = 3.3 GB)
  int seg, spimg;      // pixels per row segment, steps per image
  // option wgrad_trim (round 6): a wave whose rows of the last halo DMA round all lie past the step's halo
  // (nh <= (NR - 1) * 64 + wave * 8) issues no DMA for them instead of a zero-filling one (layer1: 136 of 192
  // rows are halo, layer4: 144): fewer LDS-DMA bytes per step, its counted waits one instruction per stage lower
  int trim;
  FastDiv fd_spimg, fd_spr, fd_seg, fd_seg2;  // steps per image, segments per row, seg, seg + 2
};

// pixel (within the 64-pixel step) of k-step ks, lane block b = lane >> 4, tr read h, lane quad q
__device__ __forceinline__ int wg_pixel(int ks, int b, int h, int q) { return ks * 32 + 8 * b + q + 4 * h; }
// the trswz swizzle of LDS row r as an 8-B unit XOR (unit index bits 2 and 3)
__device__ __forceinline__ int wg_uswz(int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3); }

// (output tile, split, problem) of this workgroup. Workgroups are dispatched to the 8 XCDs round-robin
// by linear id, so with the plain grid decode the tiles of one (problem, split) -- which read the same
// x halo (tiles of one input-channel slice) and the same dy rows (tiles of one output-channel slice) --
// land on different XCDs and each XCD's L2 fetches those operands again. With xcd = 1 the linear id is
// renumbered so every XCD owns a contiguous range of (problem, split, tile) triples: the tiles of a
// (problem, split) run on one XCD at the same time and share its L2.
__device__ __forceinline__ void wg_coords(const HaloParams& p, int& tile, int& split, unsigned& z) {
  if (!p.xcd) {
    tile = blockIdx.x;
    split = blockIdx.y;
    z = blockIdx.z;
    return;
  }
  const unsigned T = gridDim.x * gridDim.y * gridDim.z;
  const unsigned L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned r = L & 7, q = T >> 3, rem = T & 7;
  const unsigned Lp = r * q + min(r, rem) + (L >> 3);
  tile = (int)(Lp % gridDim.x);
  const unsigned g = Lp / gridDim.x;
  split = (int)(g % gridDim.y);
  z = g / gridDim.y;
}

template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* ptr) {
  const uint64_t v = (uint64_t)(uintptr_t)ptr;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// LDS per pipeline stage: the halo (NR DMA rounds of 64 rows of 128 B) + the dy tile (64 pixels x 64
// channels). NS stages form a ring; NS - 1 of them are in flight while one is computed.
template <int NR, bool SC = false>
struct WgStage {
  static constexpr int HALO_ROWS = 64 * NR;
  static constexpr int HALO_BYTES = HALO_ROWS * 128;
  static constexpr int BYTES = HALO_BYTES + 64 * 128 * (SC ? 2 : 1);
};

// NS: pipeline stages in the LDS ring (2: wait for the next step's DMA at every step; 4: three
// steps of DMA in flight, a counted s_waitcnt per step). NR: halo DMA rounds per step.
// Wave layout: 4 waves along the 576 rows x 2 along the 64 output channels, each wave both 32-pixel halves
// of a step (9 A + 2 B fragment reads per 18 MFMAs), the fragment reads software-pipelined (compute()).
// (Removed variants, numbers in DESIGN.md: compiler-scheduled fragment reads -- option wgrad_ksplit=0, round 6;
// the pixel-split layouts -- round 5; a three-stage ring -- option wgrad_ring=3, round 6; the split-K summed by
// the last-arriving workgroup -- option wgrad_ink, round 6: a 64 x 576 fp32 tile per split made that one
// workgroup's serial sum slower than a reduce launch.)
// (Round 6 scheduling experiments, bit-identical and neutral, removed: waves 4-7 half a step behind waves 0-3 on a
// 5-stage ring, l1 wgrad 38.0 -> 38.6 us, in-step -0.45%; waves 4-7 at s_setprio 1, neutral;
// profiles/r06ac_sched_experiments.txt.)
template <int NS, int NR, int ST = 1, bool SC = false, bool GEN = false>
__global__ void __launch_bounds__(512) wgrad_halo_kernel(const HaloParams p) {
  typedef WgStage<NR, SC> SG;
  constexpr int PER = NR + 1 + (SC ? 1 : 0);  // LDS-DMA instructions per wave per stage (halo rounds + dy (+ dsc))
  static_assert(!SC || ST == 2, "shortcut fusion: stride 2");
  __shared__ __attribute__((aligned(1024))) char smem[NS * SG::BYTES];
  stamp_start(p.ts);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ktiles = p.K >> 6;
  int tile, split;
  unsigned z;
  wg_coords(p, tile, split, z);
  const int c0 = (tile / ktiles) * 64, k0 = (tile % ktiles) * 64;
  // problem pointers as scalar selects (a dynamically indexed kernarg array would land in VGPRs, and
  // the LDS-DMA buffer descriptor must be scalar)
  const u16* const px = uniform_ptr(z == 0 ? p.xs[0] : z == 1 ? p.xs[1] : z == 2 ? p.xs[2] : p.xs[3]);
  const u16* const pdy = uniform_ptr(z == 0 ? p.dys[0] : z == 1 ? p.dys[1] : z == 2 ? p.dys[2] : p.dys[3]);
  const int st_begin = split * p.steps_per_split;
  const int st_end = min(p.nsteps, st_begin + p.steps_per_split);
  const int W2 = p.pitch;

  // ---- halo DMA: round j covers LDS rows j*64 + wave*8 + lane/8, 16-B chunk lane%8
  int hrel[NR], hrow_in[NR], hcc[NR];
  bool hcol[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int hrow = j * 64 + wave * 8 + (lane >> 3);
    if constexpr (GEN) {  // halo row -> (row, column) of the step's input box, relative to its corner
      // stride 1: (rs + 2) x (seg + 2) box, row pitch seg + 2. Stride 2: (2 rs + 1) input rows x (2 seg + 1)
      // columns stored column-split (box column 2j at halo column j, 2j + 1 at hwh + j; pitch p.pitch)
      const int hr = (int)fdiv((uint32_t)hrow, p.fd_seg2), hc = hrow - hr * (int)p.fd_seg2.d;
      const int src_chunk = (lane & 7) ^ trswz(hrow);
      const int lc = ST == 1 ? hc : (hc < p.hwh ? 2 * hc : (hc < 2 * p.hwh - 1 ? 2 * (hc - p.hwh) + 1 : -1000000));
      hcol[j] = hrow < p.nh && lc >= 0;
      hrow_in[j] = hr - 1;
      hcc[j] = lc - 1;
      hrel[j] = ((hr * p.W + (lc >= 0 ? lc : 0)) * p.C + c0 + src_chunk * 8) * 2;
      continue;
    }
    hcc[j] = 0;
    const int ii = hrow / p.hb, rem = hrow - ii * p.hb;
    const int hr = rem / W2, wc = rem - hr * W2;
    const int src_chunk = (lane & 7) ^ trswz(hrow);
    // input column of this halo column (stride 2: column-split layout), -1 = padding / out of range
    const int col = ST == 1 ? wc - 1 : (wc < p.hwh ? 2 * wc - 1 : (wc < 2 * p.hwh ? 2 * (wc - p.hwh) : -1));
    hcol[j] = hrow < p.nh && col >= 0 && col < p.W;
    hrow_in[j] = hr - 1;  // input row relative to the step's first input row (ST x its first output row)
    hrel[j] = (((ii * p.H + hr - 1) * p.W + col) * p.C + c0 + src_chunk * 8) * 2;
  }
  // ---- dy DMA: row t = wave*8 + lane/8 of the 64-pixel step
  const int trow = wave * 8 + (lane >> 3);
  const int dcol = k0 + (((lane & 7) ^ trswz(trow)) * 8);
  // GEN: this lane's dy row of the step (pixel trow = (row, column) of the rs x seg segment; padded -> zero)
  uint32_t drel = 0x80000000u;
  if constexpr (GEN) {  // (output grid: wo columns; stride 1 wo = W)
    const int tr = (int)fdiv((uint32_t)trow, p.fd_seg), tc = trow - tr * p.seg;
    if (trow < p.rs * p.seg) drel = (uint32_t)(((tr * p.wo + tc) * p.K + dcol) * 2);
  }

  const bool trim = p.trim && (NR - 1) * 64 + wave * 8 >= p.nh;  // (wave-uniform)
  auto stage_gen = [&](char* sb, int step) {  // GEN: per-step 64-bit bases, zero-fill out of the image
    const int img = (int)fdiv((uint32_t)step, p.fd_spimg), r = step - img * p.spimg;
    const int yb = (int)fdiv((uint32_t)r, p.fd_spr), qs = r - yb * (int)p.fd_spr.d;
    const int y0 = yb * p.rs, q0 = qs * p.seg;  // first OUTPUT row / column of the step
    const int iy0 = ST * y0, iq0 = ST * q0;       // ... and the input pixel of its (0, 0) tap centre
    const u16* xb = px + ((int64_t)(img * p.H + iy0 - 1) * p.W + (iq0 - 1)) * p.C;  // the halo box corner
    const int64_t dro = ((int64_t)(img * p.ho + y0) * p.wo + q0) * p.K;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if (j == NR - 1 && trim) break;
      const bool ok = hcol[j] && (unsigned)(iy0 + hrow_in[j]) < (unsigned)p.H && (unsigned)(iq0 + hcc[j]) < (unsigned)p.W;
      buf_lds16(xb, 0x7ffffff0u, sb + (j * 64 + wave * 8) * 128, ok ? (uint32_t)hrel[j] : 0x80000000u);
    }
    buf_lds16(pdy + dro, 0x7ffffff0u, sb + SG::HALO_BYTES + wave * 1024, drel);
    if constexpr (SC) buf_lds16(p.dsc + dro, 0x7ffffff0u, sb + SG::HALO_BYTES + 8192 + wave * 1024, drel);
  };
  auto stage = [&](char* sb, int step) {
    if constexpr (GEN) {
      stage_gen(sb, step);
      return;
    }
    const int m0 = step * 64;
    const int n0 = (int)fdiv((uint32_t)m0, p.fd_hw);
    const int p0 = (int)fdiv((uint32_t)(m0 - n0 * (int)p.fd_hw.d), p.fd_w) * ST;  // first INPUT row
    const int base = ((n0 * p.H + p0) * p.W) * p.C * 2;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if (j == NR - 1 && trim) break;
      const bool ok = hcol[j] && (unsigned)(p0 + hrow_in[j]) < (unsigned)p.H;
      buf_lds16(px, p.x_bytes, sb + (j * 64 + wave * 8) * 128, ok ? (uint32_t)(base + hrel[j]) : 0x80000000u);
    }
    glds16(pdy + (size_t)(m0 + trow) * p.K + dcol, sb + SG::HALO_BYTES + wave * 1024);
    if constexpr (SC) glds16(p.dsc + (size_t)(m0 + trow) * p.K + dcol, sb + SG::HALO_BYTES + 8192 + wave * 1024);
  };

  // ---- per-lane halo rows of the pixels this lane reads (wg_pixel: t = ks*32 + 8*(lane>>4) + (lane&15)/4 (+4))
  int hm[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = wg_pixel(ks, lane >> 4, h, (lane & 15) >> 2);
      if constexpr (GEN) {  // padded slots (t >= rs * seg, zero dy) read any in-range halo row: row 0
        const int pr = t / p.seg, q = t - pr * p.seg;
        hm[ks][h] = t < p.rs * p.seg ? pr * (ST * W2) + q : 0;
        continue;
      }
      const int ii = t / p.spi, rem = t - ii * p.spi;
      const int pr = rem / p.wo, q = rem - pr * p.wo;
      hm[ks][h] = ii * p.hb + pr * (ST * W2) + q;
    }
  // halo row offset of tap t (stride 2: row r*pitch, column-split column shift)
  auto tap_off = [&](int tap) {
    const int ts = tap % 3;
    return (tap / 3) * W2 + (ST == 1 ? ts : (ts & 1) * p.hwh + (ts >> 1));
  };

  const int wm = wave >> 1, wn = wave & 1;  // wave row (144 of the 576 GEMM rows) and column half (32 channels)
  constexpr int NJ = 2;  // B fragments (16 output channels each) per wave
  f32x4 acc[9][NJ];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Per-lane LDS byte offsets (within a stage) of every fragment half a step reads, computed once:
  // A = the x halo read transposed at each tap's shift, B = the dy tile read transposed. The step
  // loop is unrolled by NS so each stage base is a constant the ds_read offset field absorbs: the
  // MFMA stream carries no address arithmetic.
  constexpr int NKS = 2;  // 32-pixel halves (k-steps) a wave computes
  uint32_t aoff[NKS][9][2], boff[NKS][NJ][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int row = wm * 144 + i * 16;  // GEMM row = tap*64 + channel
      const int tap = row >> 6, cin = row & 63;
      const int toff = tap_off(tap);
      const int unit = (cin >> 2) + (lane & 3);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ra = hm[ks][h] + toff;
        const int f = wg_uswz(ra);
        aoff[ks][i][h] = (uint32_t)(ra * 128 + ((unit ^ f) << 3));
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cin = wn * 32 + j * 16;
      const int li = lane & 15, q = li >> 2, pp = li & 3, g = lane >> 4;
      const int unit = (cin >> 2) + pp;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kr = wg_pixel(ks, g, h, q);
        const int f = wg_uswz(kr);
        boff[ks][j][h] = (uint32_t)(SG::HALO_BYTES + kr * 128 + ((unit ^ f) << 3));
      }
    }
  }
  // SC: the centre tap's A fragment of channels wm*16.. (the shortcut's 64 output rows, 16 per wave row)
  uint32_t aoff_sc[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ra = hm[ks][h] + tap_off(4);
      const int unit = ((wm * 16) >> 2) + (lane & 3);
      const int f = (((ra >> 1) & 1) << 2) | (((ra >> 3) & 1) << 3);
      aoff_sc[ks][h] = (uint32_t)(ra * 128 + ((unit ^ f) << 3));
    }
  f32x4 acc_sc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  typedef __attribute__((address_space(3))) bf16x4_t lds_v4;
  auto tr8 = [&](const char* sb, uint32_t o0, uint32_t o1) {
    const bf16x4_t t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(sb + o0));
    const bf16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(sb + o1));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto compute = [&](const char* sb) {
    // software-pipelined fragment reads: both k-steps' B fragments first, then the 18 A fragments through a
    // three-deep register ring -- fragment f + 2 is read before the MFMAs of f, and scheduling fences keep the
    // compiler from sinking the reads back next to their uses (without them each A fragment was read right
    // before its two MFMAs and waited for: lgkmcnt(0) every 2 MFMAs)
    bf16x8 bfr2[2][2], ar[3];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr2[ks][j] = tr8(sb, boff[ks][j][0], boff[ks][j][1]);
    ar[0] = tr8(sb, aoff[0][0][0], aoff[0][0][1]);
    ar[1] = tr8(sb, aoff[0][1][0], aoff[0][1][1]);
#pragma unroll
    for (int f = 0; f < 18; ++f) {
      __builtin_amdgcn_sched_barrier(0);
      if (f + 2 < 18) ar[(f + 2) % 3] = tr8(sb, aoff[(f + 2) / 9][(f + 2) % 9][0], aoff[(f + 2) / 9][(f + 2) % 9][1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[f % 9][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[f % 3], bfr2[f / 9][j], acc[f % 9][j], 0, 0, 0);
    }
    if constexpr (SC) {  // the shortcut (stride 2): centre-tap A fragment x the dsc tile, per k-step
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 af = tr8(sb, aoff_sc[ks][0], aoff_sc[ks][1]);
        bf16x8 bs[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) bs[j] = tr8(sb, boff[ks][j][0] + 8192, boff[ks][j][1] + 8192);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc_sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bs[j], acc_sc[j], 0, 0, 0);
      }
    }
  };

  // NS-stage LDS ring. Step k: wait until this wave's DMAs of stage k landed (the DMAs of the
  // NS - 2 younger stages may stay outstanding: a counted vmcnt; near the tail vmcnt(0)), barrier
  // (every wave's DMAs of stage k landed, and every wave finished computing stage k - 1, whose slot
  // is refilled next), issue stage k + NS - 1, compute stage k. A raw s_barrier is used:
  // __syncthreads() would also drain vmcnt to 0.
  if (st_begin < st_end) {
    const int nk = st_end - st_begin;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
      if (i < nk) stage(smem + i * SG::BYTES, st_begin + i);
    for (int it = 0; it < nk; it += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int k = it + u;
        if (k >= nk) break;
        if (NS > 2 && k + NS - 2 < nk) {
          if (trim) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (PER - 1)) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * PER) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (k + NS - 1 < nk) stage(smem + ((u + NS - 1) % NS) * SG::BYTES, st_begin + k + NS - 1);
        compute(smem + u * SG::BYTES);
      }
    }
  }

  // ---- epilogue: slab[split][k][tap*C + c0 + c] (4 consecutive c per lane: one 16-B store)
  const int RSC = 9 * p.C;
  // one split: the final weight gradient itself (scale * sum, exactly what wgrad_reduce would write)
  float* const slab = p.direct ? uniform_ptr(z == 0 ? p.dws[0] : z == 1 ? p.dws[1] : z == 2 ? p.dws[2] : p.dws[3])
                               : p.slab + z * p.slab_stride + (size_t)split * p.K * RSC;
  const float osc = p.direct ? p.scale : 1.f;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int row = wm * 144 + i * 16 + 4 * (lane >> 4);
    const int rsc = (row >> 6) * p.C + c0 + (row & 63);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kout = k0 + wn * 32 + j * 16 + (lane & 15);
      *(f32x4*)(slab + (size_t)kout * RSC + rsc) = acc[i][j] * osc;
    }
  }
  if constexpr (SC) {  // slab_sc[split][k][c] (direct: dw_sc)
    float* const ss = p.direct ? p.dw_sc : p.slab_sc + (size_t)split * p.K * p.C;
    const int c = c0 + wm * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kout = k0 + wn * 32 + j * 16 + (lane & 15);
      *(f32x4*)(ss + (size_t)kout * p.C + c) = acc_sc[j] * osc;
    }
  }
  stamp_end(p.ts);
}

// ---------------------------------------------------------------- host side
// Step geometry. Classic (gen = 0): 64-pixel steps of whole rows (rs = 64 / W) or whole images, tensors
// under 2 GB (32-bit offsets). General (gen = 1, option wgrad_gen): rs rows x seg columns of one image per
// step -- seg = W for rows of at most 64 pixels (rs = 64 / W, H a multiple of rs), else a 56- / 64- / 32-
// pixel segment that divides the row -- with 64-bit per-step bases: the 224x224 model's 224 / 112 / 56 / 28
// wide rows (56 real pixels per 64-slot step at every width).
struct WgGeom {
  int gen = 0, rs = 0, imgs = 1, seg = 0, spr = 1, spimg = 0, hb = 0, nh = 0;
  int64_t nsteps = 0;
};
static bool wg_geometry(const ConvShape& s, WgGeom& g) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0)) return false;
  const int hw = s.H * s.W;
  if (s.W <= 64 && 64 % s.W == 0 && (hw % 64 == 0 || 64 % hw == 0)) {
    g.gen = 0;
    if (hw % 64 == 0) {
      g.rs = 64 / s.W;
      g.imgs = 1;
    } else {
      g.rs = s.H;
      g.imgs = 64 / hw;
    }
    g.hb = (g.rs + 2) * (s.W + 2);
    g.nh = g.imgs * g.hb;
    g.nsteps = (int64_t)s.N * hw / 64;
    // whole 64-pixel steps only (multi-image steps need N a multiple of the images per step)
    if (g.nh <= 192 && ((int64_t)s.N * hw) % 64 == 0 && (uint64_t)s.N * hw * s.C * 2 < (1ull << 31)) return true;
  }
  if (option_get(OPT_WGRAD_GEN) == 0) return false;
  g = WgGeom{};
  g.gen = 1;
  if (s.W <= 64) {
    g.seg = s.W;
    g.rs = 64 / s.W;
    if (s.H % g.rs != 0) return false;
  } else {
    g.seg = s.W % 64 == 0 ? 64 : s.W % 56 == 0 ? 56 : s.W % 32 == 0 ? 32 : 0;
    if (g.seg == 0) return false;
    g.rs = 1;
  }
  g.spr = s.W / g.seg;
  g.spimg = (s.H / g.rs) * g.spr;
  g.hb = g.nh = (g.rs + 2) * (g.seg + 2);
  g.nsteps = (int64_t)s.N * g.spimg;
  return g.nh <= 192 && g.rs * g.seg <= 64 && g.nsteps < (1ll << 31) &&
         (int64_t)(g.rs + 2) * s.W * std::max(s.C, s.K) * 2 < (1ll << 31);
}

int wgrad_halo_splits(const ConvShape& s, int nprob) {
  int target = option_get(OPT_WGRAD_HALO);
  WgGeom g;
  if (target <= 0 || nprob < 1 || nprob > DTC_WG_BATCH || !wg_geometry(s, g)) return 0;
  const int tiles = (s.C / 64) * (s.K / 64);
  // option wgrad_halo_l1: the target of the one-tile (64 -> 64 channel, layer1) geometry, whose batch runs in the
  // backward's tail beside the stem chain (0: wgrad_halo's)
  if (tiles == 1 && option_get(OPT_WGRAD_HALO_L1) > 0) target = option_get(OPT_WGRAD_HALO_L1);
  int splits = std::max(1, target / (tiles * nprob));
  // >= 24 pixel steps (1536 pixels) per workgroup: a split's slab write and its share of the reduce are paid
  // once per workgroup. Binding only at <= 64 images per rank (config 3): layer1 / 2 / 3 at batch 32 run
  // 21 / 5 / 1 splits instead of 56 / 18 / 4 (layer3 writes dw directly, no reduce launch). In-process A/B
  // against the round-5 floor of 4 (profiles/r06be_*, r06bf_*): batch 32 +2.8% / +0.3%, batch 64 +0.8% / +1.1%
  // (13 of 14 rounds), batch 128 and 256 unchanged; floors of 48 / 64 lose 1-4%.
  splits = (int)std::min<int64_t>(splits, std::max<int64_t>(1, g.nsteps / 24));
  return splits;
}

int conv_wgrad_halo(const ConvShape& s, int nprob, const u16* const* x, const u16* const* dy, float* slab, int splits,
                    int* used_splits, hipStream_t st, u64* ts, float* const* dw, float scale) {
  WgGeom g;
  DTC_CHECK_ARG(wg_geometry(s, g) && splits > 0 && nprob >= 1 && nprob <= DTC_WG_BATCH,
                "wgrad_halo: unsupported geometry");
  const int rs = g.rs, imgs = g.imgs;
  HaloParams p{};
  for (int i = 0; i < nprob; ++i) {
    p.xs[i] = x[i];
    p.dys[i] = dy[i];
  }
  p.slab = slab;
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C; p.K = s.K;
  p.x_bytes = g.gen ? 0u : (uint32_t)((uint64_t)s.N * s.H * s.W * s.C * 2);
  p.fd_hw = make_fastdiv(s.H * s.W);
  p.fd_w = make_fastdiv(s.W);
  p.nsteps = (int)g.nsteps;
  p.steps_per_split = (p.nsteps + splits - 1) / splits;
  p.rs = rs;
  p.hb = g.hb;
  p.nh = g.nh;
  p.spi = rs * s.W;
  p.pitch = (g.gen ? g.seg : s.W) + 2;
  p.ho = s.H;
  p.wo = s.W;
  if (g.gen) {
    p.seg = g.seg;
    p.spimg = g.spimg;
    p.fd_spimg = make_fastdiv(g.spimg);
    p.fd_spr = make_fastdiv(g.spr);
    p.fd_seg = make_fastdiv(g.seg);
    p.fd_seg2 = make_fastdiv(p.pitch);
  }
  (void)imgs;
  p.ts = ts;
  p.xcd = option_get(OPT_WGRAD_XCD);
  p.trim = option_get(OPT_WGRAD_TRIM);
  const int used = (p.nsteps + p.steps_per_split - 1) / p.steps_per_split;
  p.slab_stride = (size_t)used * s.K * 9 * s.C;
  p.direct = used == 1 && dw != nullptr && option_get(OPT_WGRAD_DIRECT) != 0;
  dim3 grid((s.C / 64) * (s.K / 64), used, nprob);
  if (p.direct)
    for (int i = 0; i < nprob; ++i) p.dws[i] = dw[i];
  p.scale = scale;
  const int nr = (p.nh + 63) / 64;  // halo DMA rounds per step
  // 4-stage LDS ring (three steps of DMA in flight)
#define DTC_WGH(NR_, GEN_) DTC_KLAUNCH((wgrad_halo_kernel<4, NR_, 1, false, GEN_>), grid, dim3(512), 0, st, p)
  if (g.gen) {  // general geometry
    if (nr <= 2) { DTC_WGH(2, true); }
    else { DTC_WGH(3, true); }
  } else {
    if (nr <= 2) { DTC_WGH(2, false); }
    else { DTC_WGH(3, false); }
  }
#undef DTC_WGH
  DTC_LAUNCH_CHECK();
  *used_splits = p.direct ? 0 : used;
  return 0;
}

// ---------------------------------------------------------------- stride 2 (+ shortcut)
// conv1 of a projection block (3x3, stride 2, pad 1) and, optionally, its 1x1 stride-2 shortcut: one
// halo launch over the OUTPUT pixels, the x halo column-split (conv_halo.hip's s2 layout: row pitch
// 2 (Wo + 1) [+2 where 2 * pitch must be 8 mod 16 rows for the tr reads of a 64-pixel step spanning
// output rows]); 9 taps + the shortcut from one x halo per step instead of one im2col gather per tap.
static int s2_pitch_w(int wo) { return 2 * (wo + 1) + ((wo % 16) == 8 ? 2 : 0); }
static bool halo_geometry_s2(const ConvShape& s, int& rs, int& imgs, int& pitch, int& hb, int& nh) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0 && s.H % 2 == 0 &&
        s.W % 2 == 0))
    return false;
  const int ho = s.H / 2, wo = s.W / 2, hw = ho * wo;
  if (wo > 64 || 64 % wo != 0) return false;
  if (hw % 64 == 0) {
    rs = 64 / wo;
    imgs = 1;
  } else if (64 % hw == 0) {
    rs = ho;
    imgs = 64 / hw;
  } else {
    return false;
  }
  pitch = s2_pitch_w(wo);
  hb = (2 * rs + 1) * pitch;
  nh = imgs * hb;
  return nh <= 384 && ((int64_t)s.N * hw) % 64 == 0 && (uint64_t)s.N * s.H * s.W * s.C * 2 < (1ull << 31) &&
         (uint64_t)s.N * hw * s.K * 2 < (1ull << 31);
}

// General stride-2 geometry (GEN kernels; the 224x224 model's conv1 of layers 2-4): rs output rows x seg
// output columns per step (seg = the output row if <= 64 pixels, else a 56- / 64- / 32-pixel piece), the
// input box (2 rs + 1) x (2 seg + 1) stored column-split, 64-bit per-step bases.
struct WgGeomS2 {
  int rs = 0, seg = 0, spr = 0, spimg = 0, pitch = 0, nh = 0;
  int64_t nsteps = 0;
};
static bool wg_geometry_s2_gen(const ConvShape& s, WgGeomS2& g) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0 && s.H % 2 == 0 &&
        s.W % 2 == 0))
    return false;
  const int ho = s.H / 2, wo = s.W / 2;
  g.seg = wo <= 64 ? wo : wo % 64 == 0 ? 64 : wo % 56 == 0 ? 56 : wo % 32 == 0 ? 32 : 0;
  if (g.seg == 0) return false;
  g.rs = 64 / g.seg;
  while (g.rs > 1 && ho % g.rs != 0) --g.rs;
  g.pitch = s2_pitch_w(g.seg);
  g.nh = (2 * g.rs + 1) * g.pitch;
  g.spr = wo / g.seg;
  g.spimg = (ho / g.rs) * g.spr;
  g.nsteps = (int64_t)s.N * g.spimg;
  return g.nh <= 384 && 2 * g.rs * g.seg >= 64 && g.nsteps < (1ll << 31) &&
         (int64_t)(2 * g.rs + 2) * s.W * std::max(s.C, s.K) * 2 < (1ll << 31);
}

// option wgrad_s2: 0 off, 1 every stride-2 3x3 shape it tiles, 2 (default) the general-geometry shapes only
static bool wgrad_s2_plan(const ConvShape& s, bool& gen, int64_t& nsteps) {
  const int o = option_get(OPT_WGRAD_S2);
  if (o == 0) return false;
  int rs, imgs, pitch, hb, nh;
  if (halo_geometry_s2(s, rs, imgs, pitch, hb, nh)) {
    gen = false;
    nsteps = (int64_t)s.N * (s.H / 2) * (s.W / 2) / 64;
    return o == 1;
  }
  WgGeomS2 g;
  if (option_get(OPT_WGRAD_GEN) == 0 || !wg_geometry_s2_gen(s, g)) return false;
  gen = true;
  nsteps = g.nsteps;
  return true;
}

int wgrad_s2_splits(const ConvShape& s) {
  bool gen = false;
  int64_t nsteps = 0;
  if (!wgrad_s2_plan(s, gen, nsteps)) return 0;
  const int tiles = (s.C / 64) * (s.K / 64);
  int splits = std::max(1, std::max(16, option_get(OPT_WGRAD_S2_WGS)) / tiles);
  return (int)std::min<int64_t>(splits, std::max<int64_t>(1, nsteps / 4));  // (a floor of 8 / 16 / 24 steps: batch 256 -0.1 / -0.1 / -1.0%,
  // batch 32 -0.2 / 0.0 / -0.8%, batch 64 +1.5 / +1.5 / +1.2%: profiles/r06bg_*; kept at 4)
}

size_t conv_wgrad_s2_slab_bytes(const ConvShape& s) {
  const int sp = wgrad_s2_splits(s);
  return sp > 0 ? (size_t)sp * s.K * 10 * s.C * 4 : 0;  // 9 taps + the shortcut's [K][C]
}

int conv_wgrad_s2(const ConvShape& s, const u16* x, const u16* dy, const u16* dsc, float* dw, float* dw_sc,
                  float scale, float* slab, size_t slab_bytes, hipStream_t st, u64* ts) {
  int rs = 0, imgs = 0, pitch = 0, hb = 0, nh = 0;
  const int splits = wgrad_s2_splits(s);
  bool gen = false;
  int64_t gsteps = 0;
  DTC_CHECK_ARG(splits > 0 && wgrad_s2_plan(s, gen, gsteps) && x && dy && dw && (!dsc || dw_sc),
                "conv_wgrad_s2: unsupported geometry or arguments");
  WgGeomS2 gg;
  if (gen) {
    wg_geometry_s2_gen(s, gg);
    rs = gg.rs; imgs = 1; pitch = gg.pitch; hb = nh = gg.nh;
  } else {
    halo_geometry_s2(s, rs, imgs, pitch, hb, nh);
  }
  HaloParams p{};
  p.xs[0] = x;
  p.dys[0] = dy;
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C; p.K = s.K;
  p.x_bytes = (uint32_t)((uint64_t)s.N * s.H * s.W * s.C * 2);
  p.ho = s.H / 2;
  p.wo = s.W / 2;
  p.fd_hw = make_fastdiv(p.ho * p.wo);
  p.fd_w = make_fastdiv(p.wo);
  p.nsteps = (int)gsteps;
  p.steps_per_split = (p.nsteps + splits - 1) / splits;
  p.rs = rs;
  p.hb = hb;
  p.nh = nh;
  p.spi = rs * p.wo;
  p.pitch = pitch;
  p.hwh = p.wo + 1;
  if (gen) {
    p.x_bytes = 0;
    p.hwh = gg.seg + 1;
    p.seg = gg.seg;
    p.spimg = gg.spimg;
    p.fd_spimg = make_fastdiv(gg.spimg);
    p.fd_spr = make_fastdiv(gg.spr);
    p.fd_seg = make_fastdiv(gg.seg);
    p.fd_seg2 = make_fastdiv(gg.pitch);
  }
  p.ts = ts;
  p.xcd = option_get(OPT_WGRAD_XCD);
  p.trim = option_get(OPT_WGRAD_TRIM);
  const int used = (p.nsteps + p.steps_per_split - 1) / p.steps_per_split;
  p.direct = used == 1 && option_get(OPT_WGRAD_DIRECT) != 0;
  DTC_CHECK_ARG(p.direct || (slab && slab_bytes >= (size_t)used * s.K * 10 * s.C * 4), "conv_wgrad_s2: slab too small");
  p.slab = slab;
  p.slab_stride = (size_t)used * s.K * 9 * s.C;
  p.slab_sc = slab + p.slab_stride;  // [used][K][C] after the taps
  p.dws[0] = dw;
  p.dw_sc = dw_sc;
  p.dsc = dsc;
  p.scale = scale;
  const dim3 grid((s.C / 64) * (s.K / 64), used, 1);
  const int nr = (nh + 63) / 64;
#define DTC_WS2(NR_, SC_, G_) DTC_KLAUNCH((wgrad_halo_kernel<2, NR_, 2, SC_, G_>), grid, dim3(512), 0, st, p)
  if (gen) {
    if (nr <= 5) { if (dsc) DTC_WS2(5, true, true); else DTC_WS2(5, false, true); }
    else { if (dsc) DTC_WS2(6, true, true); else DTC_WS2(6, false, true); }
  } else {
    if (nr <= 5) { if (dsc) DTC_WS2(5, true, false); else DTC_WS2(5, false, false); }
    else { if (dsc) DTC_WS2(6, true, false); else DTC_WS2(6, false, false); }
  }
#undef DTC_WS2
  DTC_LAUNCH_CHECK();
  if (p.direct) return 0;  // dw (and dw_sc) written by the halo kernel
  // the taps' and the shortcut's slabs in one reduce launch (round 6: one launch per projection block fewer)
  if (dsc) return wgrad_reduce_pair(slab, used, s.K, 9 * s.C, dw, p.slab_stride, s.C, dw_sc, scale, st, ts);
  return wgrad_reduce_to(slab, used, s.K, 9 * s.C, 9 * s.C, 9 * s.C, scale, dw, st, ts);
}

}  // namespace dtc
