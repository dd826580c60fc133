// Halo-tiled 3x3 / stride 1 / pad 1 convolution, forward and data-gradient, on bf16 MFMA (gfx950).
//
// Replaces cuDNN's forward and data-gradient kernels for the 13 stride-1 3x3 convs of ResNet-18
// (reference src/*/net.py:18-24, 29-35; `nn.Conv2d(..., kernel_size=3, stride=1, padding=1)`).
// The generic implicit-GEMM loader (igemm.hip) gathers one im2col row per (pixel, tap), so each
// input pixel is fetched from L2 nine times. Here a workgroup owns an output tile of whole image
// rows (BN pixels) x BM output channels and, per 64-channel reduction chunk, stages the tile's
// zero-padded input HALO once ((rows+2) x (W+2) pixels per image slice, 128-B LDS rows of 64
// channels); the nine taps then read the same halo shifted by r*(W+2)+s rows. Weights of one
// (chunk, tap) step are BM rows of 128 B. L2->LDS bytes per output tile and chunk drop from
// 9*BN*128 + 9*BM*128 (im2col) to ~1.3*BN*128 + 9*BM*128.
//
//   mode   D = A x B (MFMA rows x cols)     A (rows, from LDS)                B (cols)
//   FWD    y[k][pixel]                       W[k][r][s][c-chunk]  row image    halo(x)  at +( r,  s)
//   DGRAD  dx[c][pixel]                      W[k-chunk][r][s][c]  tr image     halo(dy) at +(2-r,2-s)
//
// (dgrad of a stride-1 pad-1 3x3 conv is the same correlation with the taps mirrored and W
// transposed; the tr image is read with ds_read_b64_tr_b16, so W is never transposed in HBM.)
// Epilogues match igemm.hip: FWD rounds to bf16 and reduces the BN batch statistics of the
// rounded output into fp64 slots; DGRAD optionally adds the residual-branch gradient.
//
// Pipeline: weights double-buffered; the halo is double-buffered (NHB = 2: the next chunk's halo
// arrives in slices during the current chunk's first eight taps) or single (NHB = 1: reloaded
// at chunk boundaries, a bubble other resident workgroups hide). One s_waitcnt vmcnt(0) +
// s_barrier per step (the DMA for step it+1 overlaps the MFMAs of step it).
#include "common.h"
#include "kernels.h"
#include "tile_common.h"

namespace dtc {

// Halo LDS swizzle: 16-B chunk c of halo row r is stored at chunk c ^ hswz(r). Every 8 B-fragment
// lanes that share a reduction chunk read 8 halo rows that are distinct mod 8 (the per-lane pixel
// order below guarantees it for W = 4 and 8 too), so (row parity, chunk ^ hswz) spreads them over
// 8 different 16-B bank slots, and the chunk pair (q, q+1) read by one ds_read_b128 lane group
// lands on even / odd slots: conflict-free for EVERY tap shift (rowswz is only for aligned rows).
__device__ __forceinline__ int hswz(int r) { return ((r >> 1) & 3) << 1; }

// Pixel of B-fragment column j (0..15) within its 16-pixel block. ds_read_b128 serves lanes in
// groups {0-3,12-15,20-27}, ...: columns {4..11} and {0..3,12..15} must each map to halo rows
// distinct mod 8. Contiguous image rows (W >= 16) satisfy it as is; for W = 8 (halo pitch 10) the
// block's first image row goes to columns 4..11, for W = 4 (pitch 6) image rows 0 and 2 do.
__device__ __forceinline__ int frag_pixel(int j, int W) {
  if (W == 8) return (j >= 4 && j < 12) ? j - 4 : (j < 4 ? j + 8 : j);
  if (W == 4) return (j >= 4 && j < 8) ? j - 4 : (j < 4 ? j + 4 : j);
  return j;
}

struct HConvParams {
  const u16* src;  // FWD: x; DGRAD: dy. NHWC, Cin channels (Cin = reduction channels)
  const u16* w;    // KRSC [K][3][3][C] (C = conv input channels)
  u16* out;        // NHWC, Cout channels
  const u16* res;  // DGRAD: residual added in the epilogue (NHWC, Cout) or null
  int64_t* stats;   // FWD: BN statistics [SLOTS][2][Cout] or null
  float* slab;     // split-K: fp32 partial tiles [split][M][Cout]
  // split-K reduced IN the kernel (option splitk_ink): per output tile an arrival counter (zero between
  // launches: the last arriver resets it); the workgroup whose agent-scope add returns splits - 1 sums the
  // tile's partials in split order and runs the normal (non-split) epilogue. Null: the separate
  // splitk_reduce launch does it.
  unsigned* tick;
  u64* phase;      // phase probe buffer (DTC_PHASES builds; null otherwise)
  int N, H, W, Cin, Cout, C;
  uint32_t src_bytes;
  int rows;     // output rows per image slice
  int imgs;     // image slices per tile (imgs > 1: whole images, rows == H)
  int hb;       // halo rows per image slice: (rows + 2) * (W + 2)
  int nh;       // halo rows per tile
  int nhi;      // halo DMA instructions per wave (8 rows each, 4 waves)
  int tiles_y;  // H / rows
  int tiles_a;  // Cout / BM
  int nchunk;   // Cin / 64 chunks per split
  int xcd_remap;
  FastDiv fd_hb, fd_w2, fd_spx, fd_w;
  u64* ts;
  // output dims (Ho, Wo) and halo row pitch; stride 1: (H, W) and W + 2
  int Ho, Wo, pitch;
  // stride 2 (FWD, ST = 2): the halo is stored column-split -- padded input column 2j at halo column j,
  // 2j + 1 at hwh + j (hwh = Wo + 1) -- so the output pixels of a fragment read CONSECUTIVE halo rows
  // for every tap, as at stride 1 (bank-conflict-free with the stride-1 swizzle; the row pitch is
  // padded per geometry where a fragment spans output rows: tools/halo_banks.py)
  int hwh;
  // SC (stride-2 FWD): the block's 1x1 stride-2 projection shortcut reads exactly the centre tap's
  // pixels; its weight chunk [BM][64] is staged next to the ring and a second set of MFMAs on the
  // centre tap's B fragments accumulates the shortcut output tile (one read of x, one launch)
  const u16* wsc;  // [Cout][C]
  u16* out2;
  int64_t* stats2;
  // general tile geometry (GEN kernels, stride 1; option halo_gen): a tile is grs rows x gseg columns of one
  // image in BN slots (slot l < grs * gseg: row l / gseg, column l % gseg; the rest padded: read any halo
  // row, stored nowhere), its halo (grs + 2) x (gseg + 2) pixels addressed from a 64-bit per-tile base --
  // the 224x224 model's 224 / 112 / 56 / 28-wide rows (seg 56 or the row, activations past 2 GB)
  int gseg, grs, gtpi, gspr;
  FastDiv fd_gtpi, fd_gspr;
};

// s_waitcnt vmcnt(NIW + S(tap - 1) + S(tap - 2)) for the double-buffered halo's static slices S(k) = the halo DMA
// instructions issued at tap k (k < 8) -- the immediate must be a literal, so one asm per tap after unrolling
template <int NHI>
__host__ __device__ constexpr int halo_slice(int k) { return k < 0 || k > 7 ? 0 : (((k + 1) * NHI) >> 3) - ((k * NHI) >> 3); }
template <int NIW, int NHI>
__device__ __forceinline__ void wait_vm_slices(int tap) {
#define DTC_VMW(T_) \
  case T_: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIW + halo_slice<NHI>(T_ - 1) + halo_slice<NHI>(T_ - 2)) : "memory"); break
  switch (tap) {
    DTC_VMW(1); DTC_VMW(2); DTC_VMW(3); DTC_VMW(4); DTC_VMW(5); DTC_VMW(6); DTC_VMW(7); DTC_VMW(8);
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIW) : "memory");
  }
#undef DTC_VMW
}

template <int MODE, int BM, int BN, int WR, int WC, int NHB, int HCAP, int WS, int ST = 1, bool SC = false,
          bool GEN = false>
__global__ void __launch_bounds__(256, 2) conv_halo_kernel(const HConvParams p) {
  constexpr int FM = BM / (WR * 16);
  constexpr int FN = BN / (WC * 16);
  constexpr int WBYTES = BM * 128;
  constexpr int HBYTES = HCAP * 128;
  constexpr int NIW = BM / 32;       // weight DMA instructions per wave per step
  constexpr int NHI = HCAP / 32;     // max halo DMA instructions per wave
  constexpr int SCBYTES = SC ? WBYTES : 0;
  static_assert(WR * WC == 4 && HCAP % 32 == 0 && (WS == 2 || WS == 3), "shape");  // (launched with WS = 3)
  static_assert(ST == 1 || (ST == 2 && MODE == 0 && NHB == 1), "stride 2: forward, single halo buffer");
  static_assert(!SC || (ST == 2 && WS == 3), "shortcut fusion: stride-2 forward, 3-slot weight ring");
  static_assert(!GEN || ST == 1 || (MODE == 0 && NHB == 1), "general tile geometry: stride 2 is FWD only");
  __shared__ __attribute__((aligned(1024))) char smem[NHB * HBYTES + WS * WBYTES + SCBYTES];
  char* const wbase = smem + NHB * HBYTES;
  char* const scbase = wbase + WS * WBYTES;

  stamp_start(p.ts);
  phase_mark(p.phase, 0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int bid = blockIdx.x;
  if (p.xcd_remap && gridDim.x >= 16) {  // consecutive tile ids (same pixel tile) share an XCD's L2
    const int nwg = gridDim.x, x8 = bid & 7, q = nwg >> 3, rr = nwg & 7;
    bid = (x8 < rr ? x8 * (q + 1) : rr * (q + 1) + (x8 - rr) * q) + (bid >> 3);
  }
  const int ta = bid % p.tiles_a, tb = bid / p.tiles_a;
  const int a0 = ta * BM;
  const int split = blockIdx.y, c0 = split * p.nchunk;  // first reduction chunk of this split
  int n0, y0, q0 = 0;
  if constexpr (GEN) {
    n0 = (int)fdiv((uint32_t)tb, p.fd_gtpi);
    const int rem = tb - n0 * p.gtpi, yb = (int)fdiv((uint32_t)rem, p.fd_gspr);
    y0 = yb * p.grs;
    q0 = (rem - yb * p.gspr) * p.gseg;
  } else if (p.imgs == 1) {
    n0 = tb / p.tiles_y;
    y0 = (tb - n0 * p.tiles_y) * p.rows;
  } else {
    n0 = tb * p.imgs;
    y0 = 0;
  }
  const int W2 = p.pitch;
  const int px0 = (n0 * p.Ho + y0) * p.Wo + q0;
  const int M = p.N * p.Ho * p.Wo;
  // output pixel of tile slot l (M: a padded slot of the general geometry -- every epilogue skips pix >= M)
  auto slot_pix = [&](int l) -> int {
    if constexpr (GEN) {
      if (l >= p.grs * p.gseg) return M;
      const int r = l / p.gseg;
      return px0 + r * p.Wo + (l - r * p.gseg);
    }
    return px0 + l;
  };
  // GEN: the halo box corner (input row ST y0 - 1, column ST q0 - 1) as a 64-bit base; DMA offsets are relative
  const u16* const gsrc =
      GEN ? p.src + ((int64_t)(n0 * p.H + ST * y0 - 1) * p.W + (ST * q0 - 1)) * p.Cin : p.src;
  const int lrow = lane >> 3, pc = lane & 7;
  const int RSC = 9 * p.C;

  // ---- weight DMA: per-lane element offsets (add the step's tap / chunk term)
  int offW[NIW];
#pragma unroll
  for (int j = 0; j < NIW; ++j) {
    if constexpr (MODE == 0) {  // row image: LDS row = output channel, 64 input channels of one tap
      const int row = (wave + 4 * j) * 8 + lrow;
      offW[j] = (a0 + row) * RSC + (pc ^ rowswz(row)) * 8;
    } else {  // tr image(s): LDS row = k within the chunk, 64 output channels c per image
      const int ia = wave + 4 * j, img = ia >> 3, rowin = (ia & 7) * 8 + lrow;
      offW[j] = rowin * RSC + a0 + img * 64 + (pc ^ trswz(rowin)) * 8;
    }
  }
  auto stage_w = [&](char* dst, int cc, int tap) {
    // FWD pairs weight tap (r,s) with halo offset (r,s); DGRAD pairs weight tap (r,s) with (2-r,2-s):
    // the loop tap index t is the HALO offset, so DGRAD loads weight tap 8-t.
    const int wt = (MODE == 0) ? tap : 8 - tap;
    const int add = (MODE == 0) ? (wt * p.C + cc * 64) : (cc * 64 * RSC + wt * p.C);
#pragma unroll
    for (int j = 0; j < NIW; ++j) glds16(p.w + offW[j] + add, dst + (wave + 4 * j) * 1024);
  };

  // ---- halo DMA: instruction q of this wave fills LDS rows (wave + 4q)*8 .. +8
  uint32_t hoff[NHI];
#pragma unroll
  for (int q = 0; q < NHI; ++q) {
    const int hr = (wave + 4 * q) * 8 + lrow;
    uint32_t off = 0x80000000u;  // out of the buffer: the DMA writes zeros
    if (q < p.nhi && hr < p.nh) {
      const int i = (int)fdiv((uint32_t)hr, p.fd_hb), rem = hr - i * p.hb;
      const int hy = (int)fdiv((uint32_t)rem, p.fd_w2), hx = rem - hy * W2;
      int y, x;
      if constexpr (GEN) {  // box row hy; box (padded-local) column lc: stride 2 column-split as below
        const int lc = ST == 1 ? hx : (hx < p.hwh ? 2 * hx : (hx < 2 * p.hwh - 1 ? 2 * (hx - p.hwh) + 1 : -1));
        y = ST * y0 + hy - 1;
        x = ST * q0 + lc - 1;
        if (lc >= 0 && n0 < p.N && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W)
          off = (uint32_t)(((hy * p.W + lc) * p.Cin + (pc ^ hswz(hr)) * 8) * 2);
        hoff[q] = off;
        continue;
      } else if constexpr (ST == 1) {
        y = y0 + hy - 1;
        x = hx - 1;
      } else {  // column-split halo: input row 2*y0 - 1 + hy, padded column 2*hx or 2*(hx - hwh) + 1
        y = 2 * y0 + hy - 1;
        x = hx < p.hwh ? 2 * hx - 1 : (hx < 2 * p.hwh ? 2 * (hx - p.hwh) : -1);
      }
      const int n = n0 + i;
      if (n < p.N && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W)
        off = (uint32_t)((((n * p.H + y) * p.W + x) * p.Cin + (pc ^ hswz(hr)) * 8) * 2);
    }
    hoff[q] = off;
  }
  // (all: a full load skips instructions past the tile's halo; false: every instruction of [q_lo, q_hi) is issued
  // -- rows past the halo get zeros (out-of-range offset) in LDS rows nothing reads -- so a slice's instruction
  // count is a compile-time constant the counted waits below can leave in flight)
  auto stage_h = [&](char* dst, int cc, int q_lo, int q_hi, bool all = true) {
#pragma unroll
    for (int q = 0; q < NHI; ++q) {
      if (q >= q_lo && q < q_hi && (!all || q < p.nhi)) {
        const uint32_t o = hoff[q] == 0x80000000u ? 0x80000000u : hoff[q] + (uint32_t)(cc * 128);
        buf_lds16(gsrc, GEN ? 0x7ffffff0u : p.src_bytes, dst + (wave + 4 * q) * 1024, o);
      }
    }
  };

  // ---- B fragments: halo row of each of this lane's pixels (tap (0,0))
  const int wr = wave / WC, wc = wave % WC;
  const int arow0 = wr * (BM / WR), bcol0 = wc * (BN / WC);
  const int spx = p.rows * p.Wo;  // pixels per image slice
  const int fpx = ST == 1 && !GEN ? frag_pixel(lane & 15, p.W) : (lane & 15);
  int hbr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int l = bcol0 + j * 16 + fpx;
    if constexpr (GEN) {  // slot -> (row, column) of the tile; padded slots read halo row 0
      const int r = l / p.gseg;
      hbr[j] = l < p.grs * p.gseg ? r * (ST * W2) + (l - r * p.gseg) : 0;
      continue;
    }
    const int i = (int)fdiv((uint32_t)l, p.fd_spx), rem = l - i * spx;
    const int y = (int)fdiv((uint32_t)rem, p.fd_w), x = rem - y * p.Wo;
    hbr[j] = i * p.hb + y * (ST * W2) + x;
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // B-fragment LDS byte offsets (within a halo buffer) for every tap / k-step / fragment, computed
  // once: with the taps unrolled and the chunk loop unrolled by two, every buffer base is a
  // constant the ds_read offset field absorbs, so the MFMA stream carries no address arithmetic.
  // (k-step 1 reads chunk (4 + g) ^ h = ((g ^ h) ^ 4): its offset is the k-step-0 offset ^ 64)
  uint32_t boff[9][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int ts = t % 3;
      const int row = hbr[j] + (t / 3) * W2 + (ST == 1 ? ts : (ts & 1) * p.hwh + (ts >> 1));
      boff[t][j] = (uint32_t)(row * 128 + (((lane >> 4) ^ hswz(row)) << 4));
    }
  typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;

  // Small wave tiles (< 16 MFMAs per k-step): all 2*(FM+FN) fragments of a step are read first
  // (the LDS reads overlap each other and the first MFMAs instead of each MFMA pair waiting on its
  // own reads); sched_barrier keeps the compiler from sinking the reads back next to their uses.
  auto compute = [&](const char* hbuf, const char* wb, int tap) {
    if constexpr (FM * FN >= 16) {  // 16+ MFMAs per k-step hide its reads: k-step fragments only
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = *(const lds_bf16x8*)(hbuf + (boff[tap][j] ^ (uint32_t)(ks * 64)));
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if constexpr (MODE == 0) af[i] = frag_row(wb, arow0 + i * 16, ks, lane);
          else af[i] = frag_tr(wb, arow0 + i * 16, ks, lane);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      bf16x8 af[2][FM], bfr[2][FN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[ks][j] = *(const lds_bf16x8*)(hbuf + (boff[tap][j] ^ (uint32_t)(ks * 64)));
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if constexpr (MODE == 0) af[ks][i] = frag_row(wb, arow0 + i * 16, ks, lane);
          else af[ks][i] = frag_tr(wb, arow0 + i * 16, ks, lane);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    }
  };

  f32x4 acc2[SC ? FM : 1][SC ? FN : 1];
  if constexpr (SC) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // SC: the shortcut's weight chunk cc (rows a0.., the W row-image swizzle) into its slot
  auto stage_sc = [&](int cc) {
#pragma unroll
    for (int j = 0; j < NIW; ++j) {
      const int row = (wave + 4 * j) * 8 + lrow;
      glds16(p.wsc + (a0 + row) * p.C + cc * 64 + (pc ^ rowswz(row)) * 8, scbase + (wave + 4 * j) * 1024);
    }
  };
  auto compute_sc = [&](const char* hbuf) {  // centre tap (t = 4): the same B fragments, the W_sc chunk
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *(const lds_bf16x8*)(hbuf + (boff[4][j] ^ (uint32_t)(ks * 64)));
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_row(scbase, arow0 + i * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc2[i][j], 0, 0, 0);
    }
  };

  // ---- main loop: chunk pairs x 9 unrolled taps. Weights: a WS-slot ring; step (c, tap) reads slot
  // (c + tap) & 1 (WS = 2; 9 is odd) or tap % 3 (WS = 3; 9 = 3 x 3) -- static after the unrolling.
  // WS = 2: the next step's weights are issued right before this step's MFMAs and waited for with
  // vmcnt(0) at the next step. WS = 3: two steps of weights in flight; a step waits only until its
  // own weights (and any older halo DMA) landed: vmcnt(NIW) leaves the next step's NIW weight DMAs
  // outstanding, vmcnt(0) where nothing younger exists (the last step) or where the NHB = 1 halo
  // reload is the youngest DMA (a chunk's first step).
  // Halo: NHB = 2 double-buffers it (the next chunk's halo arrives in slices during the current
  // chunk's first eight taps; buffer c & 1), NHB = 1 reloads it at chunk boundaries.
  const int nsteps = p.nchunk * 9;
  stage_h(smem, c0, 0, NHI);
  stage_w(wbase, c0, 0);
  if constexpr (WS == 3) {
    if (nsteps > 1) stage_w(wbase + WBYTES, c0, 1);
  }
  for (int cc = 0; cc < p.nchunk; cc += 2) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int c = cc + half;
      if (c >= p.nchunk) break;
      const char* hbuf = smem + (NHB == 2 ? half * HBYTES : 0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int step = c * 9 + tap;
        if constexpr (WS == 3) {
          // NHB = 2: the next chunk's halo slices of the two previous steps may stay in flight as well (issued after
          // their step's weights, so younger than this step's weights; the chunk's first step needs them all)
          if (step + 1 < nsteps && !(NHB == 1 && tap == 0 && c > 0)) {
            if (NHB == 2 && tap >= 1 && c + 1 < p.nchunk) wait_vm_slices<NIW, NHI>(tap);
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIW) : "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (step == 0) phase_mark(p.phase, 1);
        if (c == 1 && tap == 0) phase_mark(p.phase, 2);
        if constexpr (WS == 3) {  // weights of step + 2 into the slot step - 1 used
          if (tap + 2 <= 8) stage_w(wbase + ((tap + 2) % 3) * WBYTES, c0 + c, tap + 2);
          else if (c + 1 < p.nchunk) stage_w(wbase + ((tap + 2) % 3) * WBYTES, c0 + c + 1, tap + 2 - 9);
          // SC: W_sc chunk c issued right after the centre tap's weights (step + 2 = (c, 4)): it is older
          // than the step-(c, 5) weights, so the centre step's counted vmcnt(NIW) covers it
          if constexpr (SC) {
            if (tap == 2) stage_sc(c0 + c);
          }
        } else {
          const int par = (half + tap) & 1;
          if (tap < 8) stage_w(wbase + (par ^ 1) * WBYTES, c0 + c, tap + 1);
          else if (c + 1 < p.nchunk) stage_w(wbase + (par ^ 1) * WBYTES, c0 + c + 1, 0);
        }
        if constexpr (NHB == 2) {
          if (c + 1 < p.nchunk && tap < 8) {  // next chunk's halo, slice `tap` of 8
            // static slices of the NHI instructions (WS = 3: counted in the waits above; rows past the halo zeroed)
            if constexpr (WS == 3) stage_h(smem + (half ^ 1) * HBYTES, c0 + c + 1, (tap * NHI) >> 3, ((tap + 1) * NHI) >> 3, false);
            else stage_h(smem + (half ^ 1) * HBYTES, c0 + c + 1, (tap * p.nhi) >> 3, ((tap + 1) * p.nhi) >> 3);
          }
        }
        compute(hbuf, wbase + (WS == 3 ? (tap % 3) : ((half + tap) & 1)) * WBYTES, tap);
        if constexpr (SC) {
          if (tap == 4) compute_sc(hbuf);
        }
        if (NHB == 1 && tap == 8 && c + 1 < p.nchunk) {  // every wave is done with the halo: refill it
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          stage_h(smem, c0 + c + 1, 0, NHI);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  phase_mark(p.phase, 3);
  __builtin_amdgcn_s_barrier();  // LDS reads done before the epilogue reuses smem
  asm volatile("" ::: "memory");

  // ---- epilogue: D[row = output channel][col = pixel], 4 consecutive channels per lane
  const int rq = (lane >> 4) * 4, cl = fpx;  // column -> pixel, as in the B fragments
  if (p.slab != nullptr) {  // split-K partial: fp32 [split][pixel][Cout], one 16-B store per fragment
    const size_t plane = (size_t)M * p.Cout;
    if (p.tick == nullptr) {  // the separate splitk_reduce launch sums the slab
      float* slab = p.slab + (size_t)split * plane;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int pix = slot_pix(bcol0 + j * 16 + cl);
        if (pix >= M) continue;
#pragma unroll
        for (int i = 0; i < FM; ++i)
          *(f32x4*)(slab + (size_t)pix * p.Cout + a0 + arow0 + i * 16 + rq) = acc[i][j];
      }
      phase_mark(p.phase, 4);
      stamp_end(p.ts);
      return;
    }
    // In-kernel reduction (MI355X_MICROARCH.md, inter-workgroup hand-off, "Valid forms" table row 1): every
    // partial is stored write-through (sc1) and every storing wave drains (vmcnt 0) before the workgroup
    // barrier; one lane then adds to the tile's arrival counter (agent scope, returning); the workgroup
    // whose add returns splits - 1 reads the other partials with sc1 loads (L2-served, never a stale L1
    // line). No workgroup waits for another: the others exit. Compiler ordering: the stores sit above an
    // asm vmcnt(0) with a memory clobber and a __syncthreads (a workgroup acq_rel fence to the compiler), the
    // partial loads below two more __syncthreads, so neither can move across the arrival add. No agent-scope
    // release / acquire fence: on gfx950 it lowers to buffer_wbl2 / buffer_inv of the XCD's L2,
    // ~1.7-6.5 us per workgroup (the guide's price table) -- the sc1 form above needs neither.
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.slab, 0, 0x7ffffff0, 0x00020000);
    const int nsplit = (int)gridDim.y;
    uint32_t eoff[FM][FN];  // byte offset of each fragment's 4 channels within one split's plane
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int pix = slot_pix(bcol0 + j * 16 + cl);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        eoff[i][j] = pix < M ? (uint32_t)(((size_t)pix * p.Cout + a0 + arow0 + i * 16 + rq) * 4) : 0x80000000u;
    }
    const uint32_t own = (uint32_t)((size_t)split * plane * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if (eoff[i][j] != 0x80000000u)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, own + eoff[i][j], 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* const flag = (unsigned*)smem;
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.tick + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = old == (unsigned)(nsplit - 1) ? 1u : 0u;
      if (last) __hip_atomic_store(p.tick + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *(volatile unsigned*)flag = last;
    }
    __syncthreads();
    const unsigned last = *(volatile unsigned*)flag;
    __syncthreads();  // the flag word is read by every wave before the epilogue reuses smem
    if (!last) {
      phase_mark(p.phase, 4);
      stamp_end(p.ts);
      return;
    }
    // the sum splitk_reduce forms: 0 + slab[0] + slab[1] + ... (same order, same bits), this workgroup's own
    // partial from its registers. The other splits' fragments are loaded GS splits at a time, every load of a
    // group in flight before its first add: one memory latency per group instead of one per split (the
    // 64 x 64 tiles of layer4 at small batch split four ways: their last arriver waited three latencies)
    constexpr int GS = FM * FN <= 4 ? 4 : (FM * FN <= 8 ? 2 : 1);
    f32x4 sum[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) sum[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int g0 = 0; g0 < nsplit; g0 += GS) {
      f32x4 part[GS][FM][FN];
#pragma unroll
      for (int u = 0; u < GS; ++u) {
        const int sp = g0 + u;
        const bool ld = sp < nsplit && sp != split;
        const uint32_t base = (uint32_t)((size_t)(ld ? sp : 0) * plane * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            part[u][i][j] = ld && eoff[i][j] != 0x80000000u
                                ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + eoff[i][j], 0, 16))
                                : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < GS; ++u) {
        const int sp = g0 + u;
        if (sp >= nsplit) break;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) sum[i][j] += sp == split ? acc[i][j] : part[u][i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = sum[i][j];
  }
  // 16-B epilogue accesses (MI355X guide T21 for the 16x16 MFMA layout; as conv_c64.hip): lanes l and l ^ 16 hold
  // channels rq.. and rq + 4.. of the same pixel, so one v_permlane16_swap per dword of a fragment pair (2q, 2q+1)
  // leaves 8 consecutive channels per lane -- one dwordx4 store instead of two dwordx2 (issue-bound epilogues).
  // Both lanes of a swap pair hold the same pixel, so a pixel's validity is uniform across each swap.
  // (the lane id through an opaque move: the epilogue's lane-dependent offsets are computed here, not hoisted
  // before the main loop and held across it -- the 64 x 256 kernels run at the 2-waves-per-SIMD register limit)
  int ln;
  asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
  const int r4 = ln >> 4;
  const int wch = (r4 & 1) * 16 + (r4 >> 1) * 8;  // this lane's first channel within a fragment pair (16 B)
  auto swap2 = [](uint32_t& x, uint32_t& y) {  // rows 1 / 3 of x <-> rows 0 / 2 of y
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  static_assert(FM % 2 == 0, "fragment pairs");
  if constexpr (MODE == 0) {
    float* red = (float*)smem;  // [WC][BM][2]
    auto epi_fwd = [&](f32x4 (&A)[SC ? FM : 1][SC ? FN : 1], f32x4 (&B)[FM][FN], bool second, u16* outp, int64_t* stp) {
      const bool want_stats = stp != nullptr;
      float s4[FM][4], q4[FM][4];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) s4[i][t] = q4[i][t] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int pix = slot_pix(bcol0 + j * 16 + cl);
        uint32_t pk[FM][2];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const f32x4 a = second ? A[SC ? i : 0][SC ? j : 0] : B[i][j];
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = round_bf(a[t]);
          if (pix < M) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              s4[i][t] += v[t];
              q4[i][t] += v[t] * v[t];
            }
          }
          pk[i][0] = pack_bf2(v[0], v[1]);
          pk[i][1] = pack_bf2(v[2], v[3]);
        }
#pragma unroll
        for (int q = 0; q < FM / 2; ++q) {
          uint32_t x0 = pk[2 * q][0], x1 = pk[2 * q][1], y0 = pk[2 * q + 1][0], y1 = pk[2 * q + 1][1];
          swap2(x0, y0);
          swap2(x1, y1);
          if (pix < M) *(uint4*)(outp + (size_t)pix * p.Cout + a0 + arow0 + q * 32 + wch) = uint4{x0, x1, y0, y1};
        }
      }
      if (want_stats) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int chl = arow0 + i * 16 + rq;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            s4[i][t] = row16_sum(s4[i][t]);
            q4[i][t] = row16_sum(q4[i][t]);
          }
          if ((lane & 15) == 0) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              red[(wc * BM + chl + t) * 2 + 0] = s4[i][t];
              red[(wc * BM + chl + t) * 2 + 1] = q4[i][t];
            }
          }
        }
        __syncthreads();
        if ((int)threadIdx.x < BM) {
          float s = 0.f, q = 0.f;
#pragma unroll
          for (int w = 0; w < WC; ++w) {
            s += red[(w * BM + threadIdx.x) * 2 + 0];
            q += red[(w * BM + threadIdx.x) * 2 + 1];
          }
          stat_add(stp, p.Cout, a0 + threadIdx.x, s, q);
        }
      }
    };
    epi_fwd(acc2, acc, false, p.out, p.stats);
    if constexpr (SC) {
      __syncthreads();  // the statistics staging area is reused
      epi_fwd(acc2, acc, true, p.out2, p.stats2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int pix = slot_pix(bcol0 + j * 16 + cl);
      const bool ok = pix < M;
      const size_t o = (size_t)(ok ? pix : 0) * p.Cout + a0 + arow0 + wch;  // + 32 q: fragment pair q
      uint4 rr[FM / 2];  // the residuals of all FM fragments in flight before the first store (16-B loads)
#pragma unroll
      for (int q = 0; q < FM / 2; ++q) rr[q] = p.res && ok ? *(const uint4*)(p.res + o + q * 32) : uint4{0u, 0u, 0u, 0u};
      uint32_t res2[FM][2];
#pragma unroll
      for (int q = 0; q < FM / 2; ++q) {  // back to the MFMA layout (the swap is an involution)
        uint32_t x0 = rr[q].x, x1 = rr[q].y, y0 = rr[q].z, y1 = rr[q].w;
        swap2(x0, y0);
        swap2(x1, y1);
        res2[2 * q][0] = x0; res2[2 * q][1] = x1;
        res2[2 * q + 1][0] = y0; res2[2 * q + 1][1] = y1;
      }
      uint32_t pk[FM][2];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (p.res) {
          v[0] += bf_lo(res2[i][0]); v[1] += bf_hi(res2[i][0]); v[2] += bf_lo(res2[i][1]); v[3] += bf_hi(res2[i][1]);
        }
        pk[i][0] = pack_bf2(v[0], v[1]);
        pk[i][1] = pack_bf2(v[2], v[3]);
      }
#pragma unroll
      for (int q = 0; q < FM / 2; ++q) {
        uint32_t x0 = pk[2 * q][0], x1 = pk[2 * q][1], y0 = pk[2 * q + 1][0], y1 = pk[2 * q + 1][1];
        swap2(x0, y0);
        swap2(x1, y1);
        if (ok) *(uint4*)(p.out + o + q * 32) = uint4{x0, x1, y0, y1};
      }
    }
  }
  phase_mark(p.phase, 4);
  stamp_end(p.ts);
}

// ---------------------------------------------------------------- host side
struct HaloCfg {
  int bm, bn, nhb, hcap, st;
};
// Template instances (launch_halo below). LDS: NHB * HCAP * 128 + WS * BM * 128 (+ BM * 128 with SC).
static const HaloCfg kHaloCfgs[] = {
    {64, 256, 1, 416, 1},   // 0: 70 KB, 2 WG/CU: big images / many tiles
    {64, 128, 2, 288, 1},   // 1: 90 KB: double-buffered halo, no chunk bubbles
    {64, 128, 1, 288, 1},   // 2: 53 KB, 3 WG/CU
    {128, 256, 1, 416, 1},  // 3: 86 KB: wide output-channel tiles
    {128, 128, 1, 288, 1},  // 4: 69 KB, 2 WG/CU: 64x64 per wave
    {128, 128, 2, 288, 1},  // 5: 106 KB: 64x64 per wave, double-buffered halo
    {64, 128, 2, 224, 1},   // 6: 72 KB, 2 WG/CU: double-buffered halo of up to 224 rows (2 images of 8x8)
    {64, 64, 2, 160, 1},    // 7: 56 KB: double-buffered halo of up to 160 rows (4 images of 4x4)
    // stride 2 (FWD, column-split halo; the 64-pixel tile of a 16-wide output needs 9 x 34 input halo rows)
    {64, 64, 1, 384, 2},    // 8: 80 KB with the shortcut slot, 2 WG/CU, 32x32 per wave
    {64, 128, 1, 768, 2},   // 9: 128 KB, 1 WG/CU, 64x32 per wave
    {128, 64, 1, 384, 2},   // 10: 112 KB, 1 WG/CU, 64x32 per wave
};
constexpr int kNumHaloCfgs = (int)(sizeof(kHaloCfgs) / sizeof(kHaloCfgs[0]));
constexpr int kFirstS2Cfg = 8;

// Halo row pitch of the column-split stride-2 layout: 2 (Wo + 1) input columns, +2 where a 16-pixel
// fragment spans output rows of width Wo = 8 mod 16 (the +1-output-row offset 2 * pitch must be 8 mod
// 16 rows there for the ds_read_b128 lane groups to hit distinct bank slots; tools/halo_banks.py).
static int s2_pitch(int wo) { return 2 * (wo + 1) + ((wo % 16) == 8 ? 2 : 0); }

// Output tile geometry: `rows` output rows of one image slice or `imgs` whole images per tile, the
// halo rows per slice (hb) and per tile (nh), the halo row pitch and (stride 2) the split point hwh.
struct HaloGeom {
  int rows, imgs, hb, nh, pitch, hwh, ho, wo;
};
static bool halo_geometry(const ConvShape& s, int st, int bn, int hcap, HaloGeom& g) {
  g.ho = s.H / st;
  g.wo = s.W / st;
  const int hw = g.ho * g.wo;
  if (hw >= bn) {
    if (bn % g.wo) return false;
    g.rows = bn / g.wo;
    if (g.ho % g.rows) return false;
    g.imgs = 1;
  } else {
    if (bn % hw) return false;
    g.imgs = bn / hw;
    g.rows = g.ho;
  }
  if (st == 1) {
    g.pitch = s.W + 2;
    g.hwh = 0;
    g.hb = (g.rows + 2) * g.pitch;
  } else {
    g.pitch = s2_pitch(g.wo);
    g.hwh = g.wo + 1;
    g.hb = (2 * g.rows + 1) * g.pitch;
  }
  g.nh = g.imgs * g.hb;
  return g.nh <= hcap;
}

static bool halo_shape_ok(const ConvShape& s, int st) {
  if (!(s.R == 3 && s.S == 3 && s.stride == st && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0)) return false;
  if (st == 2 && (s.H % 2 || s.W % 2)) return false;
  return (uint64_t)s.N * s.H * s.W * std::max(s.C, s.K) * 2 < (1ull << 31);
}

static int halo_tiles_b(const ConvShape& s, const HaloGeom& g) {
  return g.imgs == 1 ? s.N * (g.ho / g.rows) : (s.N + g.imgs - 1) / g.imgs;
}

// General tile geometry (stride 1, option halo_gen): gseg columns per row segment (the row if it has at most
// 64 pixels, else a 64- / 56- / 32-pixel piece of it), grs rows of segments per tile (the most that fit BN
// slots and divide H). Used where the classic whole-row / whole-image tiles do not fit (the 224x224 model).
struct HaloGen {
  int seg = 0, rs = 0, spr = 0, tpi = 0, nh = 0;
};
static bool halo_gen_geometry(const ConvShape& s, int bn, int hcap, HaloGen& g) {
  if (option_get(OPT_HALO_GEN) == 0) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0)) return false;
  g.seg = s.W <= 64 ? s.W : s.W % 64 == 0 ? 64 : s.W % 56 == 0 ? 56 : s.W % 32 == 0 ? 32 : 0;
  if (g.seg == 0 || g.seg > bn) return false;
  g.rs = std::min(bn / g.seg, s.H);
  while (g.rs > 1 && s.H % g.rs != 0) --g.rs;
  g.spr = s.W / g.seg;
  g.tpi = (s.H / g.rs) * g.spr;
  g.nh = (g.rs + 2) * (g.seg + 2);
  // at least half the slots real; 32-bit per-tile offsets and pixel indices
  return g.nh <= hcap && 2 * g.rs * g.seg >= bn && (int64_t)s.N * g.tpi < (1ll << 31) &&
         (int64_t)s.N * s.H * s.W < (1ll << 31) && (int64_t)(g.rs + 2) * s.W * std::max(s.C, s.K) * 2 < (1ll << 31);
}

// the same for the stride-2 forward (output grid Ho x Wo, column-split input box (2 rs + 1) x pitch)
static bool halo_gen_geometry_s2(const ConvShape& s, int bn, int hcap, HaloGen& g) {
  if (option_get(OPT_HALO_GEN) == 0) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0 && s.H % 2 == 0 &&
        s.W % 2 == 0))
    return false;
  const int ho = s.H / 2, wo = s.W / 2;
  g.seg = wo <= 64 ? wo : wo % 64 == 0 ? 64 : wo % 56 == 0 ? 56 : wo % 32 == 0 ? 32 : 0;
  if (g.seg == 0 || g.seg > bn) return false;
  g.rs = std::min(bn / g.seg, ho);
  while (g.rs > 1 && ho % g.rs != 0) --g.rs;
  g.spr = wo / g.seg;
  g.tpi = (ho / g.rs) * g.spr;
  g.nh = (2 * g.rs + 1) * s2_pitch(g.seg);
  return g.nh <= hcap && 2 * g.rs * g.seg >= bn && (int64_t)s.N * g.tpi < (1ll << 31) &&
         (int64_t)s.N * ho * wo < (1ll << 31) && (int64_t)(2 * g.rs + 1) * s.W * std::max(s.C, s.K) * 2 < (1ll << 31);
}

static bool cfg_fits(const ConvShape& s, int cfg, int cout) {
  HaloGeom g;
  const HaloCfg& c = kHaloCfgs[cfg];
  return cout % c.bm == 0 && halo_geometry(s, c.st, c.bn, c.hcap, g);
}

// Plan for pass `mode` (CONV_FWD / CONV_DGRAD): configuration (-1: not applicable / disabled) and
// split-K factor over the reduction chunks.
HaloPlan conv_halo_plan(const ConvShape& s, int mode) {
  HaloPlan hp{-1, 1};
  if (s.stride == 2) {  // FWD only, column-split halo (option halo_s2: 0 off, 1 auto, 2+k force config 8+k)
    const int o2 = option_get(OPT_HALO_S2);
    if (o2 == 0 || mode != CONV_FWD) return hp;
    if (!halo_shape_ok(s, 2) || !cfg_fits(s, kFirstS2Cfg, s.K)) {
      // general geometry (the 224x224 model): forced settings only (halo_s2 >= 2) -- at 224x224 the 64 x 64
      // column-split tiles (56 real slots, a 3 x 116-row input halo each) measured 1.3-1.8x the implicit GEMM's
      // 128 x 128 tiles (l2.0.conv1 419 vs 233 us at batch 64; -2% in-step), so auto keeps the GEMM
      HaloGen g;
      if (o2 >= 2 && s.K % 64 == 0 && halo_gen_geometry_s2(s, 64, 384, g)) {
        hp.cfg = kFirstS2Cfg;
        hp.gen = 1;
      }
      return hp;
    }
    // auto: only where the reduction has >= 2 chunks -- with one 64-channel chunk (layer2.0.conv1) the whole
    // halo must land before the first MFMA and the implicit GEMM's per-tap pipeline is faster (20 vs 28 us
    // at B=256; layer3 20.7 -> 19.6, layer4 22.2 -> 17.1, the shortcut-fused launches 29.2 -> 24.1 / 20.3)
    // (round 5: except where its 64 x 64 tiles give <= 512 workgroups -- config 3's per-rank batches: layer2.0's
    // forward + shortcut at B=32 8.5 vs 10.6 us, B=64 10.3 vs 12.9; conv_bench r05zc)
    const int64_t s2tiles = (int64_t)s.N * (s.H / 2) * (s.W / 2) / 64 * (s.K / 64);
    if (o2 == 1 && s.C < 128 && s2tiles > 512) return hp;
    const int cfg = o2 >= 2 ? std::min(kFirstS2Cfg + o2 - 2, kNumHaloCfgs - 1) : kFirstS2Cfg;
    if (cfg_fits(s, cfg, s.K)) hp.cfg = cfg;
    return hp;  // no split-K: the shortcut fusion and the BN statistics live in the epilogue
  }
  const int opt = option_get(OPT_HALO_CONV);
  if (opt == 0) return hp;
  const int cout = mode == CONV_FWD ? s.K : s.C;
  const int cin = mode == CONV_FWD ? s.C : s.K;
  const int nchunk = cin / 64;
  if (!halo_shape_ok(s, 1) || (opt == 1 && !cfg_fits(s, 0, cout) && !cfg_fits(s, 2, cout))) {
    // the general tile geometry: 64 x 256 tiles (4 rows of a 56-pixel segment at 224 / 112 / 56 wide rows), or
    // 64 x 128 where the tile count would leave CUs idle; no split-K (these layers have >= 1024 tiles)
    HaloGen g0, g2;
    const bool f0 = cout % 64 == 0 && halo_gen_geometry(s, 256, 416, g0);
    const bool f2 = cout % 64 == 0 && halo_gen_geometry(s, 128, 288, g2);
    if (f0 && (int64_t)s.N * g0.tpi * (cout / 64) >= 512) hp.cfg = 0;
    else if (f2) hp.cfg = 2;
    else if (f0) hp.cfg = 0;
    else return hp;
    hp.gen = 1;
    hp.split = 1;
    return hp;
  }
  auto tiles = [&](int cfg) {
    HaloGeom g;
    const HaloCfg& c = kHaloCfgs[cfg];
    halo_geometry(s, c.st, c.bn, c.hcap, g);
    return halo_tiles_b(s, g) * (cout / c.bm);
  };
  if (opt >= 2) {  // forced configuration opt-2 (tuning)
    const int cfg = std::min(opt - 2, kFirstS2Cfg - 1);
    if (!cfg_fits(s, cfg, cout)) return hp;
    hp.cfg = cfg;
  } else {
    // measured (tools/conv_bench.py, B=256): 64x256 tiles while they give >= 2 workgroups per CU
    // (layer1/2); else 64x128 tiles at 3 workgroups per CU, split-K up to ~2 workgroups per CU
    // (layer3: 512 tiles; layer4: 256 tiles x 2 splits)
    // round 5 (option halo_small, default on): 64 x 64 tiles with the double-buffered halo (config 7) wherever they
    // give at most 512 workgroups -- the small layers at every batch (tools/conv_bench.py, r05v / r05w, fwd / dgrad
    // us: layer4 at B=256 25.4 / 24.9 vs 27.1 / 27.5; layer3 at B=128 14.9 / 14.5 vs 18.5 / 18.8; at B=32 layer2
    // 8.6 / 8.3 vs 9.3 / 9.9, layer3 13.1 / 12.8 vs 14.9 / 15.5, layer4 15.9 / 15.4 vs 17.7 / 18.1); with more
    // tiles the 64 x 64 tile's weight re-streaming per FLOP loses (layer2 at B=256: 34.3 vs 23.5)
    if (cfg_fits(s, 0, cout) && tiles(0) >= 512) hp.cfg = 0;
    else if (option_get(OPT_HALO_SMALL) != 0 && cfg_fits(s, 7, cout) && tiles(7) <= 512) hp.cfg = 7;
    else if (cfg_fits(s, 2, cout)) hp.cfg = 2;
    else if (cfg_fits(s, 0, cout)) hp.cfg = 0;
    else return hp;
  }
  int split = option_get(OPT_HALO_SPLIT);
  if (split <= 0) {
    split = 1;
    while (tiles(hp.cfg) * split * 2 <= 512 && nchunk % (split * 2) == 0 && nchunk / (split * 2) >= 2) split *= 2;
  }
  if (nchunk % split != 0) split = 1;
  hp.split = split;
  return hp;
}

size_t conv_halo_slab_bytes(const ConvShape& s, int mode) {
  const HaloPlan hp = conv_halo_plan(s, mode);
  if (hp.cfg < 0 || hp.split <= 1) return 0;
  const int cout = mode == CONV_FWD ? s.K : s.C;
  return (size_t)hp.split * s.N * s.H * s.W * cout * 4;
}

template <int MODE, int WS>
static int launch_halo_ws(const HConvParams& p, int cfg, dim3 grid, hipStream_t st) {
  switch (cfg) {
    case 0: DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 256, 1, 4, 1, 416, WS>), grid, dim3(256), 0, st, p); break;
    case 1: DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 128, 1, 4, 2, 288, WS>), grid, dim3(256), 0, st, p); break;
    case 2: DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 128, 1, 4, 1, 288, WS>), grid, dim3(256), 0, st, p); break;
    case 3: DTC_KLAUNCH((conv_halo_kernel<MODE, 128, 256, 2, 2, 1, 416, WS>), grid, dim3(256), 0, st, p); break;
    case 4: DTC_KLAUNCH((conv_halo_kernel<MODE, 128, 128, 2, 2, 1, 288, WS>), grid, dim3(256), 0, st, p); break;
    case 5: DTC_KLAUNCH((conv_halo_kernel<MODE, 128, 128, 2, 2, 2, 288, WS>), grid, dim3(256), 0, st, p); break;
    case 6: DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 128, 1, 4, 2, 224, WS>), grid, dim3(256), 0, st, p); break;
    default: DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 64, 2, 2, 2, 160, WS>), grid, dim3(256), 0, st, p); break;
  }
  DTC_LAUNCH_CHECK();
  return 0;
}

// (The two-slot weight ring, option halo_wstages=2, is removed: 441 vs 451 us isolated in round 5 but -6.5% in the
// step at the round-6 kernels, 0 of 10 in-process rounds faster: profiles/r06bc_b256_misc.txt.)
template <int MODE>
static int launch_halo(const HConvParams& p, int cfg, dim3 grid, hipStream_t st) {
  return launch_halo_ws<MODE, 3>(p, cfg, grid, st);
}

// general tile geometry instances (3-slot weight ring): configurations 0 (64 x 256) and 2 (64 x 128); the
// stride-2 forward in configuration 8 (64 x 64), with or without the fused shortcut
template <int MODE>
static int launch_halo_gen(const HConvParams& p, int cfg, dim3 grid, hipStream_t st) {
  if (cfg == kFirstS2Cfg) {
    if (p.wsc)
      DTC_KLAUNCH((conv_halo_kernel<0, 64, 64, 2, 2, 1, 384, 3, 2, true, true>), grid, dim3(256), 0, st, p);
    else
      DTC_KLAUNCH((conv_halo_kernel<0, 64, 64, 2, 2, 1, 384, 3, 2, false, true>), grid, dim3(256), 0, st, p);
  } else if (cfg == 0)
    DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 256, 1, 4, 1, 416, 3, 1, false, true>), grid, dim3(256), 0, st, p);
  else
    DTC_KLAUNCH((conv_halo_kernel<MODE, 64, 128, 1, 4, 1, 288, 3, 1, false, true>), grid, dim3(256), 0, st, p);
  DTC_LAUNCH_CHECK();
  return 0;
}

// stride-2 forward instances (3-slot weight ring), with or without the fused shortcut
template <bool SC>
static int launch_halo_s2(const HConvParams& p, int cfg, dim3 grid, hipStream_t st) {
  switch (cfg) {
    case 8: DTC_KLAUNCH((conv_halo_kernel<0, 64, 64, 2, 2, 1, 384, 3, 2, SC>), grid, dim3(256), 0, st, p); break;
    case 9: DTC_KLAUNCH((conv_halo_kernel<0, 64, 128, 1, 4, 1, 768, 3, 2, SC>), grid, dim3(256), 0, st, p); break;
    default: DTC_KLAUNCH((conv_halo_kernel<0, 128, 64, 2, 2, 1, 384, 3, 2, SC>), grid, dim3(256), 0, st, p); break;
  }
  DTC_LAUNCH_CHECK();
  return 0;
}

static int conv_halo_general(const ConvShape& s, int mode, const HaloPlan& hp, const u16* src, const u16* w, u16* out,
                             const u16* res, int64_t* stats, float* slab, size_t slab_bytes, hipStream_t st, u64* ts,
                             const u16* wsc, u16* out2, int64_t* stats2) {
  DTC_CHECK_ARG(hp.cfg == 0 || hp.cfg == 2 || hp.cfg == kFirstS2Cfg, "conv_halo: general geometry configuration");
  const HaloCfg& c = kHaloCfgs[hp.cfg];
  const int ST = c.st;
  DTC_CHECK_ARG(ST == 1 || (mode == CONV_FWD && res == nullptr), "conv_halo: general stride 2 is FWD only");
  DTC_CHECK_ARG(wsc == nullptr || (ST == 2 && out2 != nullptr), "conv_halo: the shortcut fusion is stride-2 FWD");
  HaloGen g;
  DTC_CHECK_ARG(ST == 1 ? halo_gen_geometry(s, c.bn, c.hcap, g) : halo_gen_geometry_s2(s, c.bn, c.hcap, g),
                "conv_halo: general geometry does not fit config %d", hp.cfg);
  HConvParams p{};
  p.src = src; p.w = w; p.out = out; p.res = res; p.stats = stats;
  p.wsc = wsc; p.out2 = out2; p.stats2 = stats2;
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C;
  p.Cin = mode == CONV_FWD ? s.C : s.K;
  p.Cout = mode == CONV_FWD ? s.K : s.C;
  DTC_CHECK_ARG(p.Cout % c.bm == 0, "conv_halo: output channels %d not a multiple of %d", p.Cout, c.bm);
  p.rows = g.rs; p.imgs = 1; p.nh = g.nh; p.hb = g.nh;
  p.Ho = s.H / ST; p.Wo = s.W / ST;
  p.pitch = ST == 1 ? g.seg + 2 : s2_pitch(g.seg);
  p.hwh = ST == 1 ? 0 : g.seg + 1;
  p.gseg = g.seg; p.grs = g.rs; p.gtpi = g.tpi; p.gspr = g.spr;
  p.fd_gtpi = make_fastdiv(g.tpi);
  p.fd_gspr = make_fastdiv(g.spr);
  p.slab = nullptr;  // (no split-K: >= 1024 tiles at the sizes this geometry serves)
  p.src_bytes = 0;
  p.nhi = (p.nh + 31) / 32;
  p.tiles_y = p.Ho / g.rs;
  p.tiles_a = p.Cout / c.bm;
  p.nchunk = p.Cin / 64;
  p.xcd_remap = option_get(OPT_XCD_REMAP);
  p.fd_hb = make_fastdiv(p.hb);
  p.fd_w2 = make_fastdiv(p.pitch);
  p.fd_spx = make_fastdiv(g.rs * g.seg);
  p.fd_w = make_fastdiv(p.Wo);
  p.ts = ts;
  (void)slab; (void)slab_bytes;
  const int64_t ntiles = (int64_t)s.N * g.tpi * p.tiles_a;
  DTC_CHECK_ARG(ntiles < (1ll << 31), "conv_halo: too many tiles");
  const dim3 grid((unsigned)ntiles, 1);
  return mode == CONV_FWD ? launch_halo_gen<0>(p, hp.cfg, grid, st) : launch_halo_gen<1>(p, hp.cfg, grid, st);
}

#ifdef DTC_PHASES
u64* g_phase = nullptr;  // also read by conv_c64.hip's per-wave cycle stamps
extern "C" int dtc_probe_phase_buffer(void* buf) {  // diagnostic builds only (tools/phase_probe.py)
  g_phase = (u64*)buf;
  return 0;
}
#endif

int conv_halo(const ConvShape& s, int mode, const HaloPlan& hp, const u16* src, const u16* w, u16* out,
              const u16* res, int64_t* stats, float* slab, size_t slab_bytes, hipStream_t st, u64* ts,
              const u16* wsc, u16* out2, int64_t* stats2, unsigned* tick) {
  DTC_CHECK_ARG(hp.cfg >= 0 && hp.cfg < kNumHaloCfgs && (mode == CONV_FWD || mode == CONV_DGRAD),
                "conv_halo: unsupported configuration");
  const HaloCfg& c = kHaloCfgs[hp.cfg];
  if (hp.gen) return conv_halo_general(s, mode, hp, src, w, out, res, stats, slab, slab_bytes, st, ts, wsc, out2, stats2);
  DTC_CHECK_ARG(halo_shape_ok(s, c.st) && (c.st == 1 || mode == CONV_FWD), "conv_halo: unsupported shape / pass");
  DTC_CHECK_ARG(wsc == nullptr || (c.st == 2 && out2 != nullptr), "conv_halo: the shortcut fusion is stride-2 FWD");
  HConvParams p{};
  p.src = src; p.w = w; p.out = out; p.res = res; p.stats = stats;
  p.wsc = wsc; p.out2 = out2; p.stats2 = stats2;
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C;
  p.Cin = mode == CONV_FWD ? s.C : s.K;
  p.Cout = mode == CONV_FWD ? s.K : s.C;
  DTC_CHECK_ARG(p.Cout % c.bm == 0, "conv_halo: output channels %d not a multiple of %d", p.Cout, c.bm);
  HaloGeom g;
  DTC_CHECK_ARG(halo_geometry(s, c.st, c.bn, c.hcap, g), "conv_halo: geometry does not fit config %d", hp.cfg);
  p.rows = g.rows; p.imgs = g.imgs; p.nh = g.nh; p.hb = g.hb;
  p.Ho = g.ho; p.Wo = g.wo; p.pitch = g.pitch; p.hwh = g.hwh;
  const int M = s.N * g.ho * g.wo;
  int split = hp.split;
  if (split > 1 && (slab == nullptr || slab_bytes < (size_t)split * M * p.Cout * 4)) split = 1;
  DTC_CHECK_ARG((p.Cin / 64) % split == 0, "conv_halo: split %d does not divide the reduction", split);
  DTC_CHECK_ARG(split == 1 || c.st == 1, "conv_halo: stride 2 has no split-K");
  p.slab = split > 1 ? slab : nullptr;
  p.src_bytes = (uint32_t)((uint64_t)s.N * s.H * s.W * p.Cin * 2);
  p.nhi = (p.nh + 31) / 32;
  p.tiles_y = g.ho / p.rows;
  p.tiles_a = p.Cout / c.bm;
  p.nchunk = p.Cin / 64 / split;
  p.xcd_remap = option_get(OPT_XCD_REMAP);
  p.fd_hb = make_fastdiv(p.hb);
  p.fd_w2 = make_fastdiv(p.pitch);
  p.fd_spx = make_fastdiv(p.rows * g.wo);
  p.fd_w = make_fastdiv(g.wo);
  p.ts = ts;
#ifdef DTC_PHASES
  p.phase = g_phase;
#endif
  const dim3 grid(halo_tiles_b(s, g) * p.tiles_a, split);
  // split-K reduced in the kernel (the last workgroup of each tile) when the caller gave arrival counters
  // for the grid (tick: >= DTC_TICKS zeroed words, reserved for this stream) and option splitk_ink is on
  const bool ink = split > 1 && tick != nullptr && option_get(OPT_SPLITK_INK) != 0 && grid.x <= (unsigned)DTC_TICKS;
  p.tick = ink ? tick : nullptr;
  if (c.st == 2) {
    return wsc ? launch_halo_s2<true>(p, hp.cfg, grid, st) : launch_halo_s2<false>(p, hp.cfg, grid, st);
  }
  DTC_TRY(mode == CONV_FWD ? launch_halo<0>(p, hp.cfg, grid, st) : launch_halo<1>(p, hp.cfg, grid, st));
  if (split > 1 && !ink) return splitk_reduce(slab, split, M, p.Cout, out, res, stats, st, ts);
  return 0;
}

}  // namespace dtc
