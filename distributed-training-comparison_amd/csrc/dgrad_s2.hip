// Data gradient of a 3x3 / stride 2 / pad 1 convolution (conv1 of ResNet-18's three projection blocks,
// reference src/*/net.py:18-19, 29-36) as a halo-tiled sub-pixel convolution on bf16 MFMA (gfx950), with the
// block's 1x1 stride-2 shortcut's data gradient fused.
//
// dx[n][2a+py][2b+px][c] = sum_k sum_(da,db) dy[n][a+da][b+db][k] W[k][r][s][c]   (+ dsc[n][a][b][k] Wsc[k][c]
// at py = px = 0), where an output parity class (py, px) meets the dy grid at offsets da, db in {0, 1}:
// py = 0 only at da = 0 (tap r = 1); py = 1 at da = 0 (r = 2) and da = 1 (r = 0); the same for columns. The
// four classes together use the nine taps once each. A workgroup owns BN consecutive dy-grid positions (whole
// dy rows of one image, or whole images) x 64 channels c, i.e. 4 BN output pixels, and per 64-channel chunk of
// the reduction (k) stages the positions' dy HALO ONCE -- (rows + 1) x (Wo + 1) dy pixels, the bottom / right
// neighbours zero-filled by the buffer descriptor -- instead of one im2col gather per (class, tap) as the
// implicit-GEMM parity classes (igemm.hip) do: the nine (offset, class, tap) steps read it at four offsets,
// each offset's B fragments read once for all the classes that use it. Weights: one W^T tap image [k][c] per
// step (3-slot LDS ring, read with ds_read_b64_tr_b16), the shortcut's Wsc^T as a tenth step against a dsc
// tile of the positions (class (0, 0) only). Epilogue: 16-B stores (permlane16 pair swap, conv_halo.hip).
#include "common.h"
#include "kernels.h"
#include "tile_common.h"

namespace dtc {

struct S2dParams {
  const u16* dy;   // [N][Ho][Wo][K]
  const u16* w;    // [K][3][3][C]
  u16* dx;         // [N][2 Ho][2 Wo][C]
  const u16* dsc;  // SC: [N][Ho][Wo][K]
  const u16* wsc;  // SC: [K][C]
  int N, Ho, Wo, C, K;
  int rows, imgs;  // dy rows per image slice; image slices per tile (imgs > 1: whole images, rows = Ho)
  int hb, nh;      // halo rows per slice ((rows + 1) x (Wo + 1)) and per tile
  int nchunk;      // K / 64
  int tiles_c;     // C / 64
  int npos;        // N * Ho * Wo
  uint32_t dy_bytes;
  FastDiv fd_hb, fd_w2, fd_spx, fd_wo, fd_hw;
  u64* ts;
};

// step t of a chunk: dy offset (da, db), output class (py, px), weight tap (r, s)
__device__ __forceinline__ constexpr int s2_da(int t) { return t >= 6 ? 1 : 0; }
__device__ __forceinline__ constexpr int s2_db(int t) { return (t == 4 || t == 5 || t == 8) ? 1 : 0; }
__device__ __forceinline__ constexpr int s2_cls(int t) {
  // 0: (0,0) tap (1,1) | 1: (0,1) (1,2) | 2: (1,0) (2,1) | 3: (1,1) (2,2) | 4: (0,1) (1,0) | 5: (1,1) (2,0)
  // 6: (1,0) (0,1) | 7: (1,1) (0,2) | 8: (1,1) (0,0)
  return t == 0 ? 0 : t == 1 ? 1 : t == 2 ? 2 : t == 3 ? 3 : t == 4 ? 1 : t == 5 ? 3 : t == 6 ? 2 : 3;
}
__device__ __forceinline__ constexpr int s2_tap(int t) {  // r * 3 + s
  return t == 0 ? 4 : t == 1 ? 5 : t == 2 ? 7 : t == 3 ? 8 : t == 4 ? 3 : t == 5 ? 6 : t == 6 ? 1 : t == 7 ? 2 : 0;
}

template <int FN, bool SC>
__global__ void __launch_bounds__(256, 2) dgrad_s2_kernel(const S2dParams p) {
  constexpr int FM = 2;             // wave tile: 32 channels (2 fragments) x 16 FN positions
  constexpr int BN = 32 * FN;       // positions per workgroup (2 waves along the positions)
  constexpr int HCAP = FN == 4 ? 224 : 128;
  constexpr int NHI = HCAP / 32;    // halo DMA instructions per wave
  constexpr int NST = SC ? 10 : 9;  // steps per chunk
  constexpr int HBYTES = HCAP * 128, WBYTES = 8192, DBYTES = SC ? BN * 128 : 0;
  __shared__ __attribute__((aligned(1024))) char smem[HBYTES + 3 * WBYTES + DBYTES];
  char* const halo = smem;
  char* const wring = smem + HBYTES;
  char* const dtile = wring + 3 * WBYTES;
  stamp_start(p.ts);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lrow = lane >> 3, pc = lane & 7;
  const int tc = blockIdx.x % p.tiles_c, tp = blockIdx.x / p.tiles_c;
  const int c0 = tc * 64;
  const int p0 = tp * BN;  // first position of the tile (flattened n, a, b)
  int n0, a0;
  if (p.imgs == 1) {
    n0 = (int)fdiv((uint32_t)p0, p.fd_hw);
    a0 = (int)fdiv((uint32_t)(p0 - n0 * (int)p.fd_hw.d), p.fd_wo);
  } else {
    n0 = (int)fdiv((uint32_t)p0, p.fd_hw);
    a0 = 0;
  }
  const int W2 = p.Wo + 1;
  const int RSC = 9 * p.C;

  // ---- weight DMA (W^T tap image: LDS row k, 64 channels c per row, tr swizzle): 2 instructions per wave
  int offW[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wave + 4 * j) * 8 + lrow;
    offW[j] = row * RSC + c0 + (pc ^ trswz(row)) * 8;
  }
  int offSc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wave + 4 * j) * 8 + lrow;
    offSc[j] = row * p.C + c0 + (pc ^ trswz(row)) * 8;
  }
  auto stage_w = [&](int slot, int gstep) {  // gstep = chunk * NST + step
    const int cc = gstep / NST, t = gstep - cc * NST;
    char* dst = wring + slot * WBYTES;
    if (SC && t == 9) {
#pragma unroll
      for (int j = 0; j < 2; ++j) glds16(p.wsc + (size_t)cc * 64 * p.C + offSc[j], dst + (wave + 4 * j) * 1024);
      return;
    }
    const int tap = t == 0 ? 4 : t == 1 ? 5 : t == 2 ? 7 : t == 3 ? 8 : t == 4 ? 3 : t == 5 ? 6 : t == 6 ? 1 : t == 7 ? 2 : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      glds16(p.w + (size_t)cc * 64 * RSC + tap * p.C + offW[j], dst + (wave + 4 * j) * 1024);
  };

  // ---- halo DMA: instruction q of this wave fills halo rows (wave + 4q) * 8 .. + 8
  uint32_t hoff[NHI];
#pragma unroll
  for (int q = 0; q < NHI; ++q) {
    const int hr = (wave + 4 * q) * 8 + lrow;
    uint32_t off = 0x80000000u;
    if (hr < p.nh) {
      const int i = (int)fdiv((uint32_t)hr, p.fd_hb), rem = hr - i * p.hb;
      const int ry = (int)fdiv((uint32_t)rem, p.fd_w2), rx = rem - ry * W2;
      const int n = n0 + i, a = a0 + ry;
      if (n < p.N && a < p.Ho && rx < p.Wo)
        off = (uint32_t)((((n * p.Ho + a) * p.Wo + rx) * p.K + (pc ^ ((((hr >> 1) & 3) << 1))) * 8) * 2);
    }
    hoff[q] = off;
  }
  // dsc tile (SC): row l = position p0 + l, row image (rowswz), 8 rows per wave-instruction
  constexpr int NDI = SC ? BN / 32 : 1;
  uint32_t doff[NDI];
#pragma unroll
  for (int q = 0; q < NDI; ++q) {
    const int l = (wave + 4 * q) * 8 + lrow;
    doff[q] = p0 + l < p.npos ? (uint32_t)(((p0 + l) * p.K + (pc ^ rowswz(l)) * 8) * 2) : 0x80000000u;
  }
  auto stage_halo = [&](int cc) {
#pragma unroll
    for (int q = 0; q < NHI; ++q)
      buf_lds16(p.dy, p.dy_bytes, halo + (wave + 4 * q) * 1024, hoff[q] == 0x80000000u ? hoff[q] : hoff[q] + cc * 128);
    if constexpr (SC) {
#pragma unroll
      for (int q = 0; q < NDI; ++q)
        buf_lds16(p.dsc, p.dy_bytes, dtile + (wave + 4 * q) * 1024, doff[q] == 0x80000000u ? doff[q] : doff[q] + cc * 128);
    }
  };

  // ---- B fragments: halo row of each of this lane's positions at offset (0, 0)
  const int wr = wave >> 1, wc = wave & 1;
  const int arow0 = wr * 32, bcol0 = wc * (BN / 2);
  const int spx = p.rows * p.Wo;
  int hbr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int l = bcol0 + j * 16 + (lane & 15);
    const int i = (int)fdiv((uint32_t)l, p.fd_spx), rem = l - i * spx;
    const int y = (int)fdiv((uint32_t)rem, p.fd_wo), x = rem - y * p.Wo;
    hbr[j] = i * p.hb + y * W2 + x;
  }
  auto boff = [&](int j, int da, int db) -> uint32_t {
    const int row = hbr[j] + da * W2 + db;
    return (uint32_t)(row * 128 + (((lane >> 4) ^ ((((row >> 1) & 3) << 1))) << 4));
  };
  typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;

  f32x4 acc[4][FM][FN];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = p.nchunk * NST;
  stage_halo(0);
  stage_w(0, 0);
  if (nsteps > 1) stage_w(1, 1);
  int slot = 0;  // ring slot of the current step
  for (int cc = 0; cc < p.nchunk; ++cc) {
    bf16x8 bfr[2][FN];
#pragma unroll
    for (int t = 0; t < NST; ++t) {
      const int g = cc * NST + t;
      // this step's weights (issued two steps ago) have landed; the next step's 2 DMAs may stay in flight.
      // A chunk's first step also waits for the halo reload (issued after the previous chunk's last step).
      if (t == 0 || g + 1 >= nsteps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (g + 2 < nsteps) stage_w(slot == 0 ? 2 : slot - 1, g + 2);  // the slot step g - 1 used
      const char* wb = wring + slot * WBYTES;
      bf16x8 af[2][FM];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i) af[ks][i] = frag_tr(wb, arow0 + i * 16, ks, lane);
      if (SC && t == 9) {  // the shortcut: class (0, 0), B = the dsc tile (row image)
        bf16x8 bs[2][FN];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < FN; ++j) bs[ks][j] = frag_row(dtile, bcol0 + j * 16, ks, lane);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bs[ks][j], acc[0][i][j], 0, 0, 0);
      } else {
        const int tt = t < 9 ? t : 0;
        if (tt == 0 || tt == 4 || tt == 6 || tt == 8) {  // a new dy offset: its B fragments, once for its classes
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const uint32_t o = boff(j, s2_da(tt), s2_db(tt));
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) bfr[ks][j] = *(const lds_bf16x8*)(halo + (o ^ (uint32_t)(ks * 64)));
          }
        }
        constexpr int dummy = 0;
        (void)dummy;
        const int cls = s2_cls(tt);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              if (cls == 0) acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[0][i][j], 0, 0, 0);
              else if (cls == 1) acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[1][i][j], 0, 0, 0);
              else if (cls == 2) acc[2][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[2][i][j], 0, 0, 0);
              else acc[3][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[3][i][j], 0, 0, 0);
            }
      }
      slot = slot == 2 ? 0 : slot + 1;
      if (t == NST - 1 && cc + 1 < p.nchunk) {  // every wave is done with the halo (and dsc tile): refill them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_halo(cc + 1);
      }
    }
  }

  // ---- epilogue: class (py, px) of position (n, a, b) -> dx pixel (n, 2a + py, 2b + px); 16-B stores
  int ln;
  asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
  const int r4 = ln >> 4;
  const int wch = (r4 & 1) * 16 + (r4 >> 1) * 8;
  const int H = 2 * p.Ho, W = 2 * p.Wo;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int pos = p0 + bcol0 + j * 16 + (ln & 15);
    const bool ok = pos < p.npos;
    const int n = (int)fdiv((uint32_t)(ok ? pos : 0), p.fd_hw);
    const int rem = (ok ? pos : 0) - n * (int)p.fd_hw.d;
    const int a = (int)fdiv((uint32_t)rem, p.fd_wo), b = rem - a * p.Wo;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int py = c >> 1, px = c & 1;
      uint32_t pk[FM][2];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        pk[i][0] = pack_bf2(acc[c][i][j][0], acc[c][i][j][1]);
        pk[i][1] = pack_bf2(acc[c][i][j][2], acc[c][i][j][3]);
      }
      uint32_t x0 = pk[0][0], x1 = pk[0][1], y0 = pk[1][0], y1 = pk[1][1];
      {
        const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        x0 = r0[0];
        y0 = r0[1];
        const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        x1 = r1[0];
        y1 = r1[1];
      }
      if (ok) {
        const size_t o = ((size_t)(n * H + 2 * a + py) * W + 2 * b + px) * p.C + c0 + arow0 + wch;
        *(uint4*)(p.dx + o) = uint4{x0, x1, y0, y1};
      }
    }
  }
  stamp_end(p.ts);
}

// ---------------------------------------------------------------- host side
// Tile geometry: BN consecutive dy-grid positions = whole dy rows of one image, or whole images.
static bool s2d_geometry(const ConvShape& s, int bn, int hcap, int& rows, int& imgs, int& hb, int& nh) {
  if (!(s.R == 3 && s.S == 3 && s.stride == 2 && s.pad == 1 && s.C % 64 == 0 && s.K % 64 == 0 && s.H % 2 == 0 &&
        s.W % 2 == 0))
    return false;
  const int ho = s.H / 2, wo = s.W / 2, hw = ho * wo;
  if (hw >= bn) {
    if (bn % wo || ho % (bn / wo)) return false;
    rows = bn / wo;
    imgs = 1;
  } else {
    if (bn % hw) return false;
    imgs = bn / hw;
    rows = ho;
  }
  hb = (rows + 1) * (wo + 1);
  nh = imgs * hb;
  return nh <= hcap && (uint64_t)s.N * hw * s.K * 2 < (1ull << 31) && (uint64_t)s.N * s.H * s.W * s.C * 2 < (1ull << 31);
}

// 128 positions per workgroup where that leaves >= 256 workgroups, else 64
static int s2d_bn(const ConvShape& s) {
  int rows, imgs, hb, nh;
  const int npos = s.N * (s.H / 2) * (s.W / 2);
  if (s2d_geometry(s, 128, 224, rows, imgs, hb, nh) && (int64_t)((npos + 127) / 128) * (s.C / 64) >= 256) return 128;
  if (s2d_geometry(s, 64, 128, rows, imgs, hb, nh)) return 64;
  return 0;
}

// option dgrad_s2h: 1 (auto) where it measured faster than the parity-class igemm -- output-gradient depth
// K <= 256 (conv_bench r05g, batch 256: layer2.0 28.2 -> 17.9 us, layer3.0 23.2 -> 20.5); layer4's K = 512 runs
// 4608-deep reductions on 256 workgroups with no split (27.0 us against the classes' 22.6); 2 every geometry
// and only where the tiles give >= 256 workgroups: with fewer (config 3's per-rank batches) the parity-class GEMM
// is ahead (B=32: l2.0.c1 8.4 vs 9.4 us, l3.0.c1 12.5 vs 15.0; B=64: 9.8 vs 10.0, 12.8 vs 15.2; conv_bench r05zc)
bool dgrad_s2_halo_ok(const ConvShape& s) {
  const int o = option_get(OPT_DGRAD_S2H);
  const int bn = s2d_bn(s);
  if (o == 0 || bn == 0) return false;
  if (o >= 2) return true;
  const int64_t wgs = ((int64_t)s.N * (s.H / 2) * (s.W / 2) + bn - 1) / bn * (s.C / 64);
  return s.K <= 256 && wgs >= 256;
}

int conv_dgrad_s2_halo(const ConvShape& s, const u16* dy, const u16* w, u16* dx, const u16* dsc, const u16* wsc,
                       hipStream_t st, u64* ts) {
  const int bn = s2d_bn(s);
  DTC_CHECK_ARG(bn > 0 && dy && w && dx && (!dsc || wsc), "conv_dgrad_s2_halo: unsupported geometry / args");
  S2dParams p{};
  p.dy = dy; p.w = w; p.dx = dx; p.dsc = dsc; p.wsc = wsc;
  p.N = s.N; p.Ho = s.H / 2; p.Wo = s.W / 2; p.C = s.C; p.K = s.K;
  s2d_geometry(s, bn, bn == 128 ? 224 : 128, p.rows, p.imgs, p.hb, p.nh);
  p.nchunk = s.K / 64;
  p.tiles_c = s.C / 64;
  p.npos = s.N * p.Ho * p.Wo;
  p.dy_bytes = (uint32_t)((uint64_t)p.npos * s.K * 2);
  p.fd_hb = make_fastdiv(p.hb);
  p.fd_w2 = make_fastdiv(p.Wo + 1);
  p.fd_spx = make_fastdiv(p.rows * p.Wo);
  p.fd_wo = make_fastdiv(p.Wo);
  p.fd_hw = make_fastdiv(p.Ho * p.Wo);
  p.ts = ts;
  const dim3 grid((unsigned)(((p.npos + bn - 1) / bn) * p.tiles_c));
  if (bn == 128) {
    if (dsc) DTC_KLAUNCH((dgrad_s2_kernel<4, true>), grid, dim3(256), 0, st, p);
    else DTC_KLAUNCH((dgrad_s2_kernel<4, false>), grid, dim3(256), 0, st, p);
  } else {
    if (dsc) DTC_KLAUNCH((dgrad_s2_kernel<2, true>), grid, dim3(256), 0, st, p);
    else DTC_KLAUNCH((dgrad_s2_kernel<2, false>), grid, dim3(256), 0, st, p);
  }
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
