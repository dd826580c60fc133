// Persistent 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels
// (ResNet-18 layer1: four convs, forward and data-gradient; reference src/*/net.py:18-24,
// `nn.Conv2d(64, 64, 3, 1, 1)`), bf16 MFMA on gfx950.
//
// layer1's reduction is a single 64-channel chunk x 9 taps, so a tile-per-workgroup kernel
// (conv_halo.hip) spends as long in its prologue / epilogue as in its 9 MFMA steps. Here one
// 4-wave workgroup per CU stays resident and walks output tiles of 256 pixels (whole image rows),
// each wave owning all 64 output channels x 64 pixels:
//   * the whole filter (64 x 9 x 64 = 72 KB) is loaded ONCE per workgroup and stays in LDS as nine
//     tap images (FWD: W rows, read with ds_read_b128; DGRAD: W^T, read with ds_read_b64_tr_b16);
//     with two 43 KB halo buffers beside it the workgroup uses 158 KB, one per CU;
//   * the zero-padded input halo of the NEXT tile is DMA'd into the other LDS buffer while the
//     current tile runs its 9 taps x 2 k-steps of MFMAs with no barrier in between;
//   * one barrier per tile; output stores are buffer stores (out-of-range lanes are dropped by
//     the descriptor bound), so every wave issues the same count and the halo wait is a counted
//     vmcnt that leaves the tile's stores in flight;
//   * FWD accumulates the BN batch statistics of the bf16-rounded outputs in registers across
//     all tiles of the workgroup and adds them to the fp64 slots once.
// Halo layout, swizzle and DGRAD tap mirroring are those of conv_halo.hip.
//
// General geometry (template flag GEN, option c64_gen; the 224x224 model's 224-wide layer1): rows whose
// width does not divide 256 are cut into 32-pixel segments and a tile is 8 rows x one segment of one image
// -- the LDS image of a tile is then exactly the classic 32-wide tile's (a 10 x 34 halo, the same B-fragment
// offsets) -- while HBM is addressed from a 64-bit per-tile base (the halo box corner / the tile's first
// pixel) with 32-bit offsets inside the box: activations past 2 GB (512 x 224 x 224 x 64 bf16 = 3.3 GB).
#include "common.h"
#include "kernels.h"
#include "tile_common.h"

namespace dtc {

__device__ __forceinline__ int c64_hswz(int r) { return ((r >> 1) & 3) << 1; }

struct C64Params {
  const u16* src;  // FWD: x, DGRAD: dy (NHWC, 64 channels)
  const u16* w;    // KRSC [64][3][3][64]
  u16* out;        // NHWC, 64 channels
  const u16* res;  // DGRAD residual or null
  int64_t* stats;   // FWD BN statistics [SLOTS][2][64] or null
  int N, H, W;
  uint32_t src_bytes, out_bytes;
  int rows, imgs, hb, nh, tiles_y, ntiles;
  FastDiv fd_hb, fd_w2, fd_spx, fd_w;
  // GEN: tiles per image and 32-pixel segments per row (a tile = rows 8*yb.. x columns 32*sb.. of image n)
  int tpi, spr;
  FastDiv fd_tpi, fd_spr;
  u64* ts;
  u64* phase;  // cycle-stamp buffer (DTC_PHASES builds; null otherwise)
};

// Cycle stamps (diagnostic builds only, tools/c64_stamps.py): every wave of workgroups < 1024 writes s_memtime
// (shader clock) at slot k of buf[wg][wave][32]; the stamp drains LDS reads (lgkmcnt(0)), so it is placed only
// where none are in flight. Its store adds one VMEM op, which only makes the counted halo waits stricter. The
// store goes through a buffer descriptor whose size is 0 without a buffer: a branch around the stamp made the
// compiler treat the halo DMA's descriptors as divergent.
#ifdef DTC_PHASES
extern u64* g_phase;
#define C64_STAMP(k, rt)                                                                                         \
  do {                                                                                                           \
    u64 t_;                                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                                           \
    if (rt) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));                                \
    else asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));                                       \
    __builtin_amdgcn_sched_barrier(0);                                                                           \
    typedef int i32x2_ __attribute__((ext_vector_type(2)));                                                      \
    __builtin_amdgcn_raw_buffer_store_b64(i32x2_{(int)(uint32_t)t_, (int)(uint32_t)(t_ >> 32)}, c64_phase_rsrc,   \
                                          ((blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (k)) * 8, 0, 0);        \
  } while (0)
#else
#define C64_STAMP(k, rt) \
  do {                   \
  } while (0)
#endif

constexpr int C64_HCAP = 344;                 // halo rows per buffer: 43 DMA wave-instructions of 8 rows
constexpr int C64_NHI = (C64_HCAP / 8 + 3) / 4;  // per wave (instruction ids wave + 4q < 43)
constexpr int C64_HBYTES = C64_HCAP * 128;
constexpr int C64_WBYTES = 9 * 8192;

// 16-B fragment at an LDS byte address (ds_read_b128 with that VGPR address)
__device__ __forceinline__ bf16x8 lds_frag(uint32_t addr) {
  typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;
  return *(const lds_bf16x8*)(size_t)addr;
}

// MODE 0: FWD (+ BN statistics), 1: DGRAD, 2: DGRAD + residual.
// (The compiler-scheduled fragment reads -- option c64_pf=0 -- are removed: the read-ahead below is faster.)
// Software pipelined over tiles: the epilogue of tile k-1 (bf16 rounding, statistics, stores) is
// issued in the same basic block as tile k's 288 MFMAs, so its VALU work fills MFMA issue gaps
// instead of running after them on the wave's single SIMD (one wave per SIMD: nothing else would
// hide it). Per-lane B-fragment LDS offsets for all nine taps and both k-steps, and the
// tile-invariant part of the halo DMA addressing, are computed once per workgroup.
constexpr int C64_SEG = 32, C64_GROWS = 8;  // GEN tile: 8 rows x 32 columns

template <int MODE, bool GEN = false>
__global__ void __launch_bounds__(256, 1) conv_c64_kernel(const C64Params p) {
  constexpr int FM = 4, FN = 4;  // wave tile: 64 channels x 64 pixels
  constexpr bool FWD = MODE == 0, RES = MODE == 2;
  __shared__ __attribute__((aligned(1024))) char smem[C64_WBYTES + 2 * C64_HBYTES];
  char* const halo = smem + C64_WBYTES;
  stamp_start(p.ts);
#ifdef DTC_PHASES
  const __amdgpu_buffer_rsrc_t c64_phase_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.phase, 0, p.phase != nullptr ? 1024 * 4 * 32 * 8 : 0, 0x00020000);
#endif
  C64_STAMP(16, true);
  C64_STAMP(0, false);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bcol0 = wave * 64;
  const int lrow = lane >> 3, pc = lane & 7;
  const int LW = GEN ? C64_SEG : p.W;  // width of the tile's LDS image
  const int W2 = LW + 2;
  const int M = p.N * p.H * p.W;
  // GEN: tile -> (image, first row, first column) and the 64-bit element index of its first pixel
  auto gen_tile = [&](int tile, int& n0, int& y0, int& q0) {
    n0 = (int)fdiv((uint32_t)tile, p.fd_tpi);
    const int rem = tile - n0 * p.tpi, yb = (int)fdiv((uint32_t)rem, p.fd_spr);
    y0 = yb * C64_GROWS;
    q0 = (rem - yb * p.spr) * C64_SEG;
  };
  auto gen_base = [&](int tile) -> int64_t {
    int n0, y0, q0;
    gen_tile(tile, n0, y0, q0);
    return ((int64_t)n0 * p.H + y0) * p.W + q0;
  };

  // ---- filter -> LDS, once: nine tap images of 64 rows x 128 B (read as MFMA A fragments per tap)
#pragma unroll
  for (int q = 0; q < 18; ++q) {
    const int g = wave + 4 * q;  // 72 wave-instructions: tap g/8, row group g%8
    const int tap = g >> 3, ia = g & 7, row = ia * 8 + lrow;
    const u16* src = FWD ? p.w + row * 576 + tap * 64 + (pc ^ rowswz(row)) * 8
                         : p.w + row * 576 + (8 - tap) * 64 + (pc ^ trswz(row)) * 8;
    glds16(src, smem + tap * 8192 + ia * 1024);
  }
  // ---- B fragments: LDS byte offsets within a halo buffer, per tap / k-step / fragment
  const int spx = p.rows * p.W;
  const int fpx = lane & 15;  // W >= 16: the 16 pixels of a fragment are contiguous in one image row
  uint32_t boff[9][2][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int l = bcol0 + j * 16 + fpx;
    const int i = (int)fdiv((uint32_t)l, p.fd_spx), rem = l - i * spx;
    const int y = (int)fdiv((uint32_t)rem, p.fd_w), x = rem - y * LW;
    const int hbr = i * p.hb + y * W2 + x;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int row = hbr + (t / 3) * W2 + (t % 3);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) boff[t][ks][j] = row * 128 + (((ks * 4 + (lane >> 4)) ^ c64_hswz(row)) << 4);
    }
  }
  // ---- halo DMA: tile-invariant per-lane parts (row decomposition, x range, swizzled channel chunk)
  int hrel[C64_NHI], hyy[C64_NHI], hii[C64_NHI], hxx[C64_NHI];
  bool hok[C64_NHI];
#pragma unroll
  for (int q = 0; q < C64_NHI; ++q) {
    const int g = wave + 4 * q;
    const int hr = g * 8 + lrow;
    const int i = (int)fdiv((uint32_t)hr, p.fd_hb), rem = hr - i * p.hb;
    const int hy = (int)fdiv((uint32_t)rem, p.fd_w2), hx = rem - hy * W2;
    hyy[q] = hy - 1;
    hii[q] = i;
    if constexpr (GEN) {  // box row hy, column hx: byte offset from the box corner (row y0 - 1, column q0 - 1)
      hok[q] = g < C64_HCAP / 8 && hr < p.nh;
      hxx[q] = hx - 1;
      hrel[q] = ((hy * p.W + hx) * 64 + (pc ^ c64_hswz(hr)) * 8) * 2;
    } else {
      hok[q] = g < C64_HCAP / 8 && hr < p.nh && (unsigned)(hx - 1) < (unsigned)p.W;
      hxx[q] = 0;
      hrel[q] = (((i * p.H + hy - 1) * p.W + hx - 1) * 64 + (pc ^ c64_hswz(hr)) * 8) * 2;
    }
  }
  auto stage_halo = [&](char* dst, int tile) {
    if constexpr (GEN) {
      int n0, y0, q0;
      gen_tile(tile, n0, y0, q0);
      const u16* const box = p.src + (((int64_t)n0 * p.H + y0 - 1) * p.W + (q0 - 1)) * 64;
#pragma unroll
      for (int q = 0; q < C64_NHI; ++q) {
        const int g = wave + 4 * q;
        if (g >= C64_HCAP / 8) break;
        const bool ok = hok[q] && (unsigned)(y0 + hyy[q]) < (unsigned)p.H && (unsigned)(q0 + hxx[q]) < (unsigned)p.W;
        buf_lds16(box, 0x7ffffff0u, dst + g * 1024, ok ? (uint32_t)hrel[q] : 0x80000000u);
      }
      return;
    }
    int n0, y0;
    if (p.imgs == 1) {
      n0 = (int)((unsigned)tile / (unsigned)p.tiles_y);
      y0 = (tile - n0 * p.tiles_y) * p.rows;
    } else {
      n0 = tile * p.imgs;
      y0 = 0;
    }
    const int tbase = (n0 * p.H + y0) * p.W * 128;
#pragma unroll
    for (int q = 0; q < C64_NHI; ++q) {
      const int g = wave + 4 * q;
      if (g >= C64_HCAP / 8) break;
      const bool ok = hok[q] && (unsigned)(y0 + hyy[q]) < (unsigned)p.H && n0 + hii[q] < p.N;
      buf_lds16(p.src, p.src_bytes, dst + g * 1024, ok ? (uint32_t)(tbase + hrel[q]) : 0x80000000u);
    }
  };
  // buffer descriptors of the output-side tensors; GEN: rebased at a tile's first pixel (tile_rsrc below)
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.out, 0, p.out_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(RES ? p.res : p.out), 0, RES ? p.out_bytes : 0, 0x00020000);
  // GEN: a descriptor starting `byte_base` bytes into a tensor (a tile's first pixel: 128 B per pixel of the
  // bf16 tensors, 8 B per pixel of the mask bits); offsets inside the tile stay 32-bit
  auto tile_rsrc = [&](const void* t, int64_t byte_base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)t + byte_base), 0, 0x7ffffff0u, 0x00020000);
  };
  const uint32_t halo_lds = __builtin_amdgcn_readfirstlane(lds_u32(halo));

  const int rq = (lane >> 4) * 4;
  // FWD: sum / sum of squares of the bf16 outputs
  float ssum[FM][4], ssq[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) ssum[i][t] = ssq[i][t] = 0.f;

  // DGRAD residual of one tile, loaded one tile AHEAD of its use: issued right after the tile's
  // halo wait, before the next halo DMA, so it has landed by the next iteration's halo wait and the
  // epilogue (interleaved with the following tile's MFMAs) never waits on it. Loading it inside the
  // epilogue stalled the wave's only SIMD on a full HBM latency per pixel-column group (and on the
  // younger halo DMA: vmcnt retires in order): 74 -> 26 us per layer1 dgrad at B=256.
  typedef int i32x2 __attribute__((ext_vector_type(2)));
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  // 16-B epilogue accesses (MI355X guide T21, for the 16x16 MFMA layout): lane l holds channels rq..rq+3 of
  // fragment i, and lane l ^ 16 the next four. One v_permlane16_swap per dword of a fragment pair (2p, 2p+1)
  // gives the lanes of rows 0 / 2 the 8 consecutive channels 32p + {0, 8}.. of fragment 2p and the lanes of rows
  // 1 / 3 those of fragment 2p + 1 -- one dwordx4 store per pair instead of two dwordx2 (the stores were
  // issue-bound: 8-B accesses move half the bytes per vector-memory instruction). The swap is an involution,
  // so a 16-B residual load is turned back into the MFMA layout the same way.
  const int r4 = lane >> 4;
  const int wch = (r4 & 1) * 16 + (r4 >> 1) * 8;  // this lane's first channel within a fragment pair (16 B)
  auto swap2 = [](uint32_t& x, uint32_t& y) {  // rows 1 / 3 of x <-> rows 0 / 2 of y
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  struct EpiOps {
    i32x4 r[FN][FM / 2];
  };
  // VMEM ops the previous tile's epilogue leaves in flight per wave at the halo wait: its stores
  constexpr int EPI_VM = FN * FM / 2;
  // byte offset of channel `ch` of pixel column j (pixel bcol0 + 16 j + lane % 16) of a tile
  auto epi_off_ch = [&](int tile, int j, int ch) {
    const int l = bcol0 + j * 16 + fpx;
    if constexpr (GEN) {  // slot l = row l / 32, column l % 32 of the tile; byte offset from its first pixel
      return (uint32_t)((((l >> 5) * p.W + (l & 31)) * 64 + ch) * 2);
    }
    const int pix = tile * 256 + l;  // tiles are 256 consecutive pixels
    return pix < M ? (uint32_t)((pix * 64 + ch) * 2) : 0x80000000u;
  };
  auto epi_off = [&](int tile, int j, int i) { return epi_off_ch(tile, j, i * 16 + rq); };
  auto prefetch = [&](EpiOps& o, int tile) {
    const __amdgpu_buffer_rsrc_t rr = GEN ? tile_rsrc(RES ? p.res : p.out, gen_base(tile) * 128) : rrsrc;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < FM / 2; ++q)
        o.r[j][q] = __builtin_amdgcn_raw_buffer_load_b128(rr, epi_off_ch(tile, j, q * 32 + wch), 0, 0);
  };

  // epilogue of one finished tile: exactly FM*FN buffer stores per wave; lanes of pixels past M, or
  // of no tile (have == false), are dropped by the descriptor bound
  auto epilogue_col = [&](const f32x4 (&a)[FM][FN], const EpiOps& o, int tile, bool have, int j) {
    const int pix = tile * 256 + bcol0 + j * 16 + fpx;
    const bool ok = have && (GEN || pix < M);  // GEN tiles have no slot past the tensor
    __amdgpu_buffer_rsrc_t ors = orsrc;
    if constexpr (GEN) ors = tile_rsrc(p.out, (have ? gen_base(tile) : 0) * 128);
    uint32_t rres[FM][2];  // RES: the residual of each fragment in the MFMA layout (packed bf16 x 4)
    if constexpr (RES) {
#pragma unroll
      for (int q = 0; q < FM / 2; ++q) {
        uint32_t x0 = (uint32_t)o.r[j][q].x, x1 = (uint32_t)o.r[j][q].y, y0 = (uint32_t)o.r[j][q].z,
                 y1 = (uint32_t)o.r[j][q].w;
        swap2(x0, y0);
        swap2(x1, y1);
        rres[2 * q][0] = x0; rres[2 * q][1] = x1;
        rres[2 * q + 1][0] = y0; rres[2 * q + 1][1] = y1;
      }
    }
    uint32_t packed[FM][2];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      float v[4] = {a[i][j][0], a[i][j][1], a[i][j][2], a[i][j][3]};
      if constexpr (RES) {
        v[0] += bf_lo(rres[i][0]); v[1] += bf_hi(rres[i][0]);
        v[2] += bf_lo(rres[i][1]); v[3] += bf_hi(rres[i][1]);
      }
      packed[i][0] = pack_bf2(v[0], v[1]);
      packed[i][1] = pack_bf2(v[2], v[3]);
      if constexpr (FWD) {  // statistics of the bf16-rounded outputs, read back from the packed words (a tile that
        // is not there -- the first iteration's -- holds zeros: no mask needed)
        const float r[4] = {bf_lo(packed[i][0]), bf_hi(packed[i][0]), bf_lo(packed[i][1]), bf_hi(packed[i][1])};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          ssum[i][t] += r[t];
          ssq[i][t] += r[t] * r[t];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < FM / 2; ++q) {  // fragment pair (2q, 2q + 1) -> one 16-B store per lane
      uint32_t x0 = packed[2 * q][0], x1 = packed[2 * q][1], y0 = packed[2 * q + 1][0], y1 = packed[2 * q + 1][1];
      swap2(x0, y0);
      swap2(x1, y1);
      const uint32_t o16 = ok ? epi_off_ch(tile, j, q * 32 + wch) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)x0, (int)x1, (int)y0, (int)y1}, ors, o16, 0, 0);
    }
  };
  auto epilogue = [&](const f32x4 (&a)[FM][FN], const EpiOps& o, int tile, bool have) {
#pragma unroll
    for (int j = 0; j < FN; ++j) epilogue_col(a, o, tile, have, j);
  };

  f32x4 accp[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) accp[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  EpiOps opp{}, opc{};  // residual of the previous / current tile (modes 2, 4)
  int tilep = 0;
  int k = 0;
  int tile = blockIdx.x;
  if (tile < p.ntiles) stage_halo(halo, tile);
  C64_STAMP(1, false);
  for (; tile < p.ntiles; tile += gridDim.x, ++k) {
    // this tile's halo (and the residual issued before it) have landed; the previous iteration's
    // epilogue VMEM ops (FM*FN stores, + the BN-backward y/x loads) were issued after it
    if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EPI_VM) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k < 6) C64_STAMP(2 + 2 * k, false);
    const uint32_t hb = halo_lds + (uint32_t)((k & 1) * C64_HBYTES);
    if constexpr (RES) prefetch(opc, tile);
    const int tn = tile + gridDim.x;
    if (tn < p.ntiles) stage_halo(halo + ((k + 1) & 1) * C64_HBYTES, tn);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 18 (tap, k-step) groups of FM + FN fragment reads and FM x FN MFMAs. The reads of group g + 1
    // go out before the MFMAs of group g (two register sets; scheduling fences keep the compiler
    // from sinking them back next to their uses), so with one wave per SIMD an LDS read's latency
    // hides behind the 16 MFMAs before it instead of stalling the SIMD once per group.
    bf16x8 af[2][FM], bfr[2][FN];
    auto load = [&](int g, int b) {
      const int t = g >> 1, ks = g & 1;
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[b][i] = FWD ? frag_row(smem + t * 8192, i * 16, ks, lane) : frag_tr(smem + t * 8192, i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[b][j] = lds_frag(hb + boff[t][ks][j]);
    };
    load(0, 0);
#pragma unroll
    for (int g = 0; g < 18; ++g) {
      __builtin_amdgcn_sched_barrier(0);
      if (g + 1 < 18) load(g + 1, (g + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[g & 1][i], bfr[g & 1][j], acc[i][j], 0, 0, 0);
      // the previous tile's epilogue, one pixel-column group after each odd tap's second k-step
      if ((g & 3) == 3) epilogue_col(accp, opp, tilep, k > 0, g >> 2);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) accp[i][j] = acc[i][j];
    tilep = tile;
    if constexpr (RES) opp = opc;
    if (k < 6) C64_STAMP(3 + 2 * k, false);
  }
  if (k > 0) epilogue(accp, opp, tilep, true);
  C64_STAMP(14, false);

  if constexpr (FWD) {
    int64_t* const sacc = p.stats;
    if (sacc != nullptr) {  // per-channel sums of this workgroup -> fp64 slot (once per workgroup)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
      float* red = (float*)halo;  // [4 waves][64 ch][2]
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float s = row16_sum(ssum[i][t]), q = row16_sum(ssq[i][t]);
          if ((lane & 15) == 0) {
            const int ch = i * 16 + rq + t;
            red[(wave * 64 + ch) * 2 + 0] = s;
            red[(wave * 64 + ch) * 2 + 1] = q;
          }
        }
      __syncthreads();
      if (threadIdx.x < 64) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          s += red[(w * 64 + threadIdx.x) * 2 + 0];
          q += red[(w * 64 + threadIdx.x) * 2 + 1];
        }
        stat_add(sacc, 64, threadIdx.x, s, q);
      }
    }
  }
  C64_STAMP(15, false);
  C64_STAMP(17, true);
  stamp_end(p.ts);
}

// ---------------------------------------------------------------- host side
static bool c64_classic_ok(const ConvShape& s);
// GEN geometry: 8 rows x 32-column segments (rows whose width does not divide 256, or tensors past 2 GB)
static bool c64_gen_ok(const ConvShape& s) {
  if (option_get(OPT_C64_GEN) == 0) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.C == 64 && s.K == 64)) return false;
  if (s.W % C64_SEG != 0 || s.H % C64_GROWS != 0) return false;
  const int64_t M = (int64_t)s.N * s.H * s.W;
  return M / 256 < (1ll << 31) && M < (1ll << 31) && (int64_t)C64_GROWS * s.W * 128 < (1ll << 31);
}
// option conv_c64: 0 off; 1 (auto) where every persistent workgroup gets at least one 256-pixel tile -- below
// that (batch 32 at 32x32: 128 tiles for 256 workgroups) the halo kernel's 64 x 64 tiles fill the chip (layer1
// fwd / dgrad at B=32 8.0 / 7.5 vs 9.4 / 8.7 us; equal at B=64, c64 ahead at B=128: tools/conv_bench.py r05y);
// 2 always
bool conv_c64_ok(const ConvShape& s) {
  const int o = option_get(OPT_CONV_C64);
  if (o == 0) return false;
  if (o == 1 && (int64_t)s.N * s.H * s.W / 256 < (int64_t)std::max(1, option_get(OPT_C64_WGS))) return false;
  return c64_classic_ok(s) || c64_gen_ok(s);
}
static bool c64_classic_ok(const ConvShape& s) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.C == 64 && s.K == 64)) return false;
  if (s.W < 16 || 256 % s.W != 0) return false;  // fragments of 16 contiguous pixels in one image row
  const int hw = s.H * s.W;
  int rows, imgs;
  if (hw >= 256) {
    rows = 256 / s.W;
    if (s.H % rows) return false;
    imgs = 1;
  } else {
    if (256 % hw) return false;
    imgs = 256 / hw;
    rows = s.H;
  }
  const int nh = imgs * (rows + 2) * (s.W + 2);
  const int64_t M = (int64_t)s.N * hw;
  return nh <= C64_HCAP && M % 256 == 0 && M * 128 < (1ll << 31);
}

int conv_c64(const ConvShape& s, int mode, const u16* src, const u16* w, u16* out, const u16* res, int64_t* stats,
             hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(conv_c64_ok(s) && (mode == CONV_FWD || mode == CONV_DGRAD), "conv_c64: unsupported shape");
  C64Params p{};
  p.src = src; p.w = w; p.out = out; p.res = res; p.stats = stats;
  p.N = s.N; p.H = s.H; p.W = s.W;
  const int64_t hw = (int64_t)s.H * s.W;
  const int64_t M = s.N * hw;
  const bool gen = !c64_classic_ok(s);
  const int lw = gen ? C64_SEG : s.W;  // the LDS tile width
  if (gen) {
    p.rows = C64_GROWS;
    p.imgs = 1;
    p.spr = s.W / C64_SEG;
    p.tpi = (s.H / C64_GROWS) * p.spr;
    p.fd_tpi = make_fastdiv(p.tpi);
    p.fd_spr = make_fastdiv(p.spr);
    p.src_bytes = p.out_bytes = 0x7ffffff0u;  // unused: every access goes through a per-tile base
  } else {
    if (hw >= 256) {
      p.rows = 256 / s.W;
      p.imgs = 1;
    } else {
      p.imgs = (int)(256 / hw);
      p.rows = s.H;
    }
    p.src_bytes = (uint32_t)(M * 128);
    p.out_bytes = (uint32_t)(M * 128);
  }
  p.hb = (p.rows + 2) * (lw + 2);
  p.nh = p.imgs * p.hb;
  p.tiles_y = s.H / p.rows;
  p.ntiles = (int)(M / 256);
  p.fd_hb = make_fastdiv(p.hb);
  p.fd_w2 = make_fastdiv(lw + 2);
  p.fd_spx = make_fastdiv(p.rows * lw);
  p.fd_w = make_fastdiv(lw);
  p.ts = ts;
#ifdef DTC_PHASES
  p.phase = g_phase;
#endif
  // persistent: one workgroup per CU by default (option c64_wgs), each walking ntiles / grid tiles with the
  // filter resident
  const int grid = std::min(p.ntiles, std::max(1, option_get(OPT_C64_WGS)));
  const int kmode = mode == CONV_FWD ? 0 : (res == nullptr ? 1 : 2);
#define DTC_C64(M_)                                                                        \
  if (gen) DTC_KLAUNCH((conv_c64_kernel<M_, true>), dim3(grid), dim3(256), 0, st, p); \
  else DTC_KLAUNCH((conv_c64_kernel<M_>), dim3(grid), dim3(256), 0, st, p)
  switch (kmode) {
    case 0: DTC_C64(0); break;
    case 1: DTC_C64(1); break;
    default: DTC_C64(2); break;
  }
#undef DTC_C64
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
