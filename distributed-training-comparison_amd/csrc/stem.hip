// Direct stem convolution, forward and weight gradient: `self.conv1 = nn.Conv2d(3, 64, 3, 1, 1)`
// (reference src/*/net.py:91) + the BN statistics of its bf16 output, on bf16 MFMA (gfx950).
//
// The stem's reduction is 27 values per pixel (3 channels x 3 x 3 taps). Materialising them as an
// im2col matrix (stem_im2col: [pixels][64] bf16, 27 real columns) costs a 128-B write and a 128-B
// re-read per pixel in the forward and another re-read in the weight gradient, plus a K = 64 GEMM
// that multiplies 37 zero columns. Here each workgroup gathers its 256 pixels' 27 taps straight
// from the fp32 NCHW input (coalesced per tap, L2-resident: 12 B of input per pixel) into an LDS
// tile of 32 bf16 columns (27 + 5 zeros) and runs ONE 16x16x32 k-step per output fragment:
//   forward  y[pixel][k]  = bf16(sum_kk col[pixel][kk] * W[k][kk])      (+ BN sum / sum of squares)
//   wgrad    dW[k][kk]   += sum_pixel dy[pixel][kk'...]: D[k][kk] over 256-pixel tiles, fp32 slab
//                           per workgroup [64][32], summed by the deterministic wgrad_reduce.
// HBM per pixel: forward 128 B written (the conv output) instead of 128 + 128 + 128; weight
// gradient 128 B of dy read instead of 128 + 128. The weight is the bf16 shadow in KRSC order,
// [64][27] with kk = (r*3 + s)*3 + c -- the im2col column order of stem_im2col.
#include "common.h"
#include "kernels.h"
#include "tile_common.h"
#include "bn_coef.h"

namespace dtc {

// The 256-pixel tile's input rows (3 channels x rows h0-1 .. h1+1 x W+2 columns with the zero
// padding, fp32) staged once in LDS with coalesced loads; each thread then gathers its pixel's 27
// taps from LDS. Tiles that span two images (images under 256 pixels) or more rows than 24 KB
// hold (narrow images) gather from global memory instead.
constexpr int STEM_LDS_FLOATS = 5120;  // 20 KB: 224-wide rows fit 5 staged rows (3 x 5 x 226)

// pixel index decomposition without 64-bit or runtime-divisor divisions (M < 2^31, checked on the host)
struct StemGeom {
  int N, H, W;
  uint32_t M, HW;
  FastDiv fd_w, fd_hw, fd_w2;
};

struct StemTile {
  int n;       // image of the tile (-1: global gathers)
  int h0, rt;  // first output row, rows staged (h1 - h0 + 3)
};

// The tile's staging geometry (T.n = -1: global gathers instead).
template <int CAP>
__device__ __forceinline__ StemTile stem_tile(uint32_t pix0, const StemGeom& G) {
  const uint32_t last = min(pix0 + 255u, G.M - 1u);
  const int n = (int)fdiv(pix0, G.fd_hw), nl = (int)fdiv(last, G.fd_hw);
  StemTile T{n, (int)fdiv(pix0 - (uint32_t)n * G.HW, G.fd_w), 0};
  const int h1 = (int)fdiv(last - (uint32_t)nl * G.HW, G.fd_w);
  T.rt = h1 - T.h0 + 3;
  if (nl != n || T.rt * 3 * (G.W + 2) > CAP) T.n = -1;
  return T;
}

// Loads of the staged rows into registers (split from the LDS stores so that a caller can put other
// loads between the two). Every lane loads from a clamped valid address, then selects (a load under a
// divergent branch gets its own s_waitcnt: one latency per element); the trip count is uniform.
template <int CAP>
__device__ __forceinline__ void stem_stage_ld(const float* __restrict__ x, const StemTile& T, const StemGeom& G,
                                              float (&v)[CAP / 256]) {
  if (T.n < 0) return;
  const float* xn = x + (size_t)T.n * 3 * G.HW;
  const int W2 = G.W + 2, E = 3 * T.rt * W2, iters = (E + 255) >> 8;
#pragma unroll
  for (int i = 0; i < CAP / 256; ++i) {
    if (i < iters) {
      const int e = threadIdx.x + 256 * i;
      const int rr = (int)fdiv((uint32_t)e, G.fd_w2), col = e - rr * W2;  // staged row rr = c * rt + r
      const int c = rr >= T.rt ? (rr >= 2 * T.rt ? 2 : 1) : 0;
      const int ih = T.h0 - 1 + (rr - c * T.rt), iw = col - 1;
      const bool ok = e < E && (unsigned)ih < (unsigned)G.H && (unsigned)iw < (unsigned)G.W;
      const int ihc = min(max(ih, 0), G.H - 1), iwc = min(max(iw, 0), G.W - 1), cc = min(c, 2);
      const float a = xn[((size_t)cc * G.H + ihc) * G.W + iwc];
      v[i] = ok ? a : 0.f;
    }
  }
}

template <int CAP>
__device__ __forceinline__ void stem_stage_st(const StemTile& T, const StemGeom& G, const float (&v)[CAP / 256],
                                              float* xt) {
  if (T.n < 0) return;
  const int E = 3 * T.rt * (G.W + 2), iters = (E + 255) >> 8;
#pragma unroll
  for (int i = 0; i < CAP / 256; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (i < iters && e < E) xt[e] = v[i];
  }
}

// every load of the tile issued before the first LDS store (one memory latency, not one per row)
__device__ __forceinline__ StemTile stem_stage(const float* __restrict__ x, uint32_t pix0, const StemGeom& G,
                                               float* xt) {
  const StemTile T = stem_tile<STEM_LDS_FLOATS>(pix0, G);
  float v[STEM_LDS_FLOATS / 256];
  stem_stage_ld<STEM_LDS_FLOATS>(x, T, G, v);
  stem_stage_st<STEM_LDS_FLOATS>(T, G, v, xt);
  return T;
}

// the pixel's 27 taps (kk = (r*3+s)*3 + c) + 5 zeros, rounded to bf16, as 4 x 16 B
__device__ __forceinline__ void stem_taps(const float* __restrict__ x, const float* xt, const StemTile& T,
                                          uint32_t pix, const StemGeom& G, uint4 (&q)[4]) {
  float v[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = 0.f;
  if (pix < G.M) {
    const uint32_t nh = fdiv(pix, G.fd_w);  // n*H + h
    const int w = (int)(pix - nh * (uint32_t)G.W);
    const int n = (int)fdiv(pix, G.fd_hw);
    const int h = (int)(nh - (uint32_t)n * (uint32_t)G.H);
    if (T.n >= 0) {
      const int W2 = G.W + 2, per_c = T.rt * W2;
      const int base = (h - T.h0) * W2 + w;  // tap (r, s) of channel c: xt[c*per_c + base + r*W2 + s]
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
          for (int c = 0; c < 3; ++c) v[(r * 3 + s) * 3 + c] = xt[c * per_c + base + r * W2 + s];
    } else {
      const float* xn = x + (size_t)n * 3 * G.HW;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int ih = h + r - 1, iw = w + s - 1;
          const bool in = (unsigned)ih < (unsigned)G.H && (unsigned)iw < (unsigned)G.W;
#pragma unroll
          for (int c = 0; c < 3; ++c) v[(r * 3 + s) * 3 + c] = in ? xn[((size_t)c * G.H + ih) * G.W + iw] : 0.f;
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = pack8(v + j * 8);
}

static StemGeom stem_geom(int N, int H, int W) {
  StemGeom G;
  G.N = N; G.H = H; G.W = W;
  G.HW = (uint32_t)H * W;
  G.M = (uint32_t)((int64_t)N * H * W);
  G.fd_w = make_fastdiv(W);
  G.fd_hw = make_fastdiv(G.HW);
  G.fd_w2 = make_fastdiv(W + 2);
  return G;
}

// ---------------------------------------------------------------- forward
// 256 pixels per workgroup, 4 waves x (64 output channels x 64 pixels): 16 MFMAs per wave.
// LDS tile [256 pixels][4 x 16 B], chunk j of pixel p at j ^ ((p >> 2) & 3): the 16 lanes of a
// ds_read_b128 group read 16 consecutive pixels' same chunk -> 16 distinct 16-B bank slots.
// <= 40 KB LDS and <= 128 VGPRs: four workgroups per CU, so the 1024 tiles of a 256 x 32 x 32 batch
// are all resident at once and their load latencies overlap (a workgroup does little else).
// WL (option stem_wlds): the [64][27] bf16 weight is read once per workgroup with coalesced 4-B loads
// into LDS and the A fragments are gathered from there, instead of 32 scattered 2-B global loads per
// lane; the staged input rows are capped at 8 KB (STEM_BN_CAP) so the LDS stays at four per CU.
template <bool WL = false>
__global__ void __launch_bounds__(256, 4) stem_fwd_kernel(const float* __restrict__ x, const u16* __restrict__ w27,
                                                      u16* __restrict__ y, int64_t* __restrict__ stats, const StemGeom G,
                                                      u64* ts) {
  constexpr int CAP = WL ? 2048 : STEM_LDS_FLOATS;
  // cols (16 KB) + the staged input rows (20 KB; WL 8 KB); after the MFMAs the first 32 KB hold the
  // output tile [256 pixels][128 B] for 16-B coalesced stores
  __shared__ __attribute__((aligned(16))) char smem[(256 * 64 + CAP * 4) > 32768 ? (256 * 64 + CAP * 4) : 32768];
  __shared__ float red[4][64][2];
  __shared__ uint32_t wsh[WL ? 864 : 1];  // WL: the weight, 64 x 27 bf16 = 864 words
  uint4* const cols = (uint4*)smem;
  float* const xt = (float*)(smem + 256 * 64);
  char* const ot = smem;
  stamp_start(ts);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t pix0 = blockIdx.x * 256u;
  // A fragments W[k = i*16 + lane%16][kk = 8*(lane/16) + 0..7] (kk >= 27: 0): all 32 loads issued
  // before the input tile's, so the two latencies overlap
  uint32_t we[4][4];  // bf16 pairs
  if constexpr (!WL) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = i * 16 + (lane & 15), kk = 8 * (lane >> 4) + 2 * j;
        const uint32_t a = w27[k * 27 + min(kk, 26)], b = w27[k * 27 + min(kk + 1, 26)];  // branch-free
        we[i][j] = (kk < 27 ? a : 0u) | ((kk + 1 < 27 ? b : 0u) << 16);
      }
  }
  uint32_t wv[4];
  if constexpr (WL) {  // 864 words, coalesced (the weight is 4-B aligned: KRSC rows of 27 bf16 from an even offset)
    const uint32_t* w32 = (const uint32_t*)w27;
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = w32[min(t + 256 * u, 863)];
  }
  {
    const StemTile T = WL ? stem_tile<CAP>(pix0, G) : stem_tile<STEM_LDS_FLOATS>(pix0, G);
    float xv[CAP / 256];
    stem_stage_ld<CAP>(x, T, G, xv);
    stem_stage_st<CAP>(T, G, xv, xt);
    if constexpr (WL) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (t + 256 * u < 864) wsh[t + 256 * u] = wv[u];
    }
    __syncthreads();
    if constexpr (WL) {
      const u16* wl = (const u16*)wsh;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = i * 16 + (lane & 15), kk = 8 * (lane >> 4) + 2 * j;
          const uint32_t a = wl[k * 27 + min(kk, 26)], b = wl[k * 27 + min(kk + 1, 26)];
          we[i][j] = (kk < 27 ? a : 0u) | ((kk + 1 < 27 ? b : 0u) << 16);
        }
    }
    uint4 q[4];
    stem_taps(x, xt, T, pix0 + t, G, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) cols[t * 4 + (j ^ ((t >> 2) & 3))] = q[j];
  }
  __syncthreads();
  bf16x8 af[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    af[i] = __builtin_bit_cast(bf16x8, uint4{we[i][0], we[i][1], we[i][2], we[i][3]});
  f32x4 acc[4][4];
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const int p = wave * 64 + jn * 16 + (lane & 15);
    const bf16x8 bf = __builtin_bit_cast(bf16x8, cols[p * 4 + ((lane >> 4) ^ ((p >> 2) & 3))]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  // epilogue: lane holds channels k = i*16 + 4*(lane/16) + 0..3 of pixel wave*64 + jn*16 + lane%16
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[i][r] = ssq[i][r] = 0.f;
  __syncthreads();  // every wave done reading cols: the output tile goes over it
#pragma unroll
  for (int jn = 0; jn < 4; ++jn) {
    const int px = wave * 64 + jn * 16 + (lane & 15);
    const bool ok = pix0 + px < G.M;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = round_bf(acc[i][jn][r]);
        const float u = ok ? v[r] : 0.f;
        ssum[i][r] += u;
        ssq[i][r] += u * u;
      }
      // channels k..k+3, k = 16i + 4(lane/16): 16-B chunk k/8 of the pixel row, stored at chunk ^ (px & 7)
      const int k = i * 16 + 4 * (lane >> 4);
      *(uint2*)(ot + px * 128 + (((k >> 3) ^ (px & 7)) << 4) + (k & 7) * 2) =
          uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    }
  }
  __syncthreads();
  if (y != nullptr) {  // the tile is 256 consecutive pixels = one contiguous 32 KB block of y
    const uint32_t npx = min(256u, G.M - pix0);
    uint4* dst = (uint4*)(y + (size_t)pix0 * 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int g = t + 256 * j, px = g >> 3, c = g & 7;
      if ((uint32_t)px < npx) {
        const uint4 raw = *(const uint4*)(ot + px * 128 + ((c ^ (px & 7)) << 4));
        dst[g] = raw;
      }
    }
  }
  if (stats != nullptr) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row16_sum(ssum[i][r]), q = row16_sum(ssq[i][r]);
        if ((lane & 15) == 0) {
          const int ch = i * 16 + 4 * (lane >> 4) + r;
          red[wave][ch][0] = s;
          red[wave][ch][1] = q;
        }
      }
    __syncthreads();
    if (t < 64) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        s += red[w][t][0];
        q += red[w][t][1];
      }
      stat_add(stats, 64, t, s, q);
    }
  }
  stamp_end(ts);
}

int stem_fwd(const float* x, const u16* w27, u16* y, int64_t* stats, int N, int H, int W, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(x && w27 && (y || stats) && N > 0 && H > 0 && W > 0, "stem_fwd: bad args");
  const int64_t M = (int64_t)N * H * W;
  DTC_CHECK_ARG(M + 256 < (1ll << 31), "stem_fwd: more than 2^31 pixels");
  if (option_get(OPT_STEM_WLDS) != 0 && ((uintptr_t)w27 & 3) == 0)
    DTC_KLAUNCH((stem_fwd_kernel<true>), dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, x, w27, y,
                       stats, stem_geom(N, H, W), ts);
  else
    DTC_KLAUNCH((stem_fwd_kernel<false>), dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, x, w27, y,
                       stats, stem_geom(N, H, W), ts);
  DTC_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- weight gradient
// D[k][kk] (64 x 32) += sum over 256-pixel tiles of dy[p][k] * col[p][kk]. Both operands are
// [pixel][channel] LDS images read transposed (frag_tr: reduction = pixels): dy DMA'd global->LDS
// (256 rows of 128 B, trswz chunk swizzle), col built by the threads in the same layout (64 bf16
// columns, 32..63 zero). Wave w owns k = 16w..16w+15 x both 16-column kk blocks: 2 MFMAs per
// 32-pixel k-step, 16 per tile. Each workgroup walks `tiles` consecutive tiles and writes its fp32
// partial [64][32] to slab[blockIdx.x].
__global__ void __launch_bounds__(256) stem_wgrad_kernel(const float* __restrict__ x, const u16* __restrict__ dy,
                                                        float* __restrict__ slab, const StemGeom G, int tiles,
                                                        u64* ts) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 32768];  // dy tile, col tile
  __shared__ float xt[STEM_LDS_FLOATS];
  char* const dyt = smem;
  char* const colt = smem + 32768;
  stamp_start(ts);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t ntiles = (G.M + 255u) / 256u;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  // col rows: 128 B = 8 chunks of 16 B (chunks 4..7 zero), chunk j of row p at j ^ trswz(p)
  const int tsw = trswz(t);
  for (int it = 0; it < tiles; ++it) {
    const uint32_t tile = blockIdx.x * (uint32_t)tiles + it;
    if (tile >= ntiles) break;
    const uint32_t pix0 = tile * 256u;
    // dy tile: 32 wave-instructions of 8 rows (row = 8*g + lane/8, 16-B chunk lane%8, swizzled source)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = wave + 4 * u, row = g * 8 + (lane >> 3);
      const uint32_t p = pix0 + row < G.M ? pix0 + row : G.M - 1;  // rows past M: a valid row (zero taps)
      glds16(dy + (size_t)p * 64 + (((lane & 7) ^ trswz(row)) * 8), dyt + g * 1024);
    }
    const StemTile T = stem_stage(x, pix0, G, xt);
    __syncthreads();
    uint4 q[4];
    stem_taps(x, xt, T, pix0 + t, G, q);  // zeros past M
#pragma unroll
    for (int j = 0; j < 4; ++j) *(uint4*)(colt + t * 128 + ((j ^ tsw) << 4)) = q[j];
#pragma unroll
    for (int j = 4; j < 8; ++j) *(uint4*)(colt + t * 128 + ((j ^ tsw) << 4)) = uint4{0u, 0u, 0u, 0u};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const bf16x8 a = frag_tr(dyt, wave * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, frag_tr(colt, j * 16, ks, lane),
                                                                                 acc[j], 0, 0, 0);
    }
    __syncthreads();
  }
  // slab[blockIdx.x][k][kk]: lane holds k = 16*wave + 4*(lane/16) + r, kk = 16*j + lane%16
  float* out = slab + (size_t)blockIdx.x * 64 * 32;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(wave * 16 + 4 * (lane >> 4) + r) * 32 + j * 16 + (lane & 15)] = acc[j][r];
  stamp_end(ts);
}

static int stem_bn_grid(int64_t M, int& tiles);
size_t stem_wgrad_slab_bytes(int64_t M) {  // either weight-gradient kernel's partials
  const int64_t ntiles = (M + 255) / 256;
  int tiles = 0;
  const int64_t nwg = std::max<int64_t>(std::min<int64_t>(ntiles, 256), stem_bn_grid(M, tiles));
  return (size_t)nwg * 64 * 32 * 4;
}

int stem_wgrad(const float* x, const u16* dy, float* dw27, float scale, int N, int H, int W, float* slab,
               size_t slab_bytes, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(x && dy && dw27 && slab && N > 0 && H > 0 && W > 0, "stem_wgrad: bad args");
  const int64_t M = (int64_t)N * H * W;
  const int64_t ntiles = (M + 255) / 256;
  const int nwg0 = (int)std::min<int64_t>(ntiles, 256);  // one 90 KB workgroup per CU
  const int tiles = (int)((ntiles + nwg0 - 1) / nwg0);
  const int nwg = (int)((ntiles + tiles - 1) / tiles);
  DTC_CHECK_ARG(slab_bytes >= (size_t)nwg * 64 * 32 * 4, "stem_wgrad: slab workspace too small");
  DTC_CHECK_ARG(M + 256 < (1ll << 31), "stem_wgrad: more than 2^31 pixels");
  DTC_KLAUNCH(stem_wgrad_kernel, dim3(nwg), dim3(256), 0, st, x, dy, slab, stem_geom(N, H, W), tiles, ts);
  DTC_LAUNCH_CHECK();
  return wgrad_reduce_to(slab, nwg, 64, 32, 27, 27, scale, dw27, st, ts);
}


// ---------------------------------------------------------------- weight gradient + BN backward apply
// The stem BN's backward apply fused into the weight gradient (option stem_bn_fuse): the conv-output
// gradient dc = A*dz + B*c + Cc (dz = dy * ReLU bit; A, B, Cc from the BN's fp64 slots exactly as
// bn_bwd_fin_apply computes them, same fp32 expression, same bf16 rounding) is formed in registers and
// written into the LDS dy tile of stem_wgrad_kernel's layout. dc is consumed only by this weight
// gradient (the stem has no input gradient), so it never goes to HBM: the apply's 2 B/element write,
// the wgrad's 2 B/element re-read and one launch are gone; per pixel 128 B of dy + 128 B of c + 8 B of
// mask bits are read. A tile's loads (dy, c, bits, input rows) are issued one tile ahead, into
// registers, so they are in flight during the previous tile's taps and MFMAs; <= 80 KB of LDS keeps two
// workgroups on a CU.
constexpr int STEM_BN_CAP = 2048;  // staged input floats (8 KB): 32-wide images, 8 rows + halo = 1020

template <int CAP>
__global__ void __launch_bounds__(256, 2) stem_wgrad_bn_kernel(const float* __restrict__ x, const u16* __restrict__ dy,
                                                             const uint8_t* __restrict__ mbits,
                                                             const u16* __restrict__ cin, const BnBwdArgs a,
                                                             float* __restrict__ slab, const StemGeom G, int tiles,
                                                             u64* ts) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 32768];  // dc tile, col tile
  __shared__ float xt[CAP];
  __shared__ int64_t part[256];
  __shared__ float coef[3][64];
  char* const dyt = smem;
  char* const colt = smem + 32768;
  stamp_start(ts);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, c8 = t & 7, r0 = t >> 3;
  const uint32_t ntiles = (G.M + 255u) / 256u;
  const uint32_t tile0 = blockIdx.x * (uint32_t)tiles;
  // register image of one tile: pixel rows r0 + 32u, 16-B channel chunk c8 (coalesced: 8 lanes per row)
  uint4 vd[8], vc[8];
  uint32_t mk[8];
  float xv[CAP / 256];
  auto load = [&](uint32_t pix0, const StemTile& T) {
    stem_stage_ld<CAP>(x, T, G, xv);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t p = min(pix0 + r0 + 32u * u, G.M - 1u);  // rows past M: a valid row (zero taps)
      const size_t o = (size_t)p * 64 + c8 * 8;
      vd[u] = *(const uint4*)(dy + o);
      vc[u] = *(const uint4*)(cin + o);
      mk[u] = mbits[o >> 3];
    }
  };
  SlotFold f;
  fold_issue_bwd(a, 64, 0, f);  // the fold's loads first (in-order vmcnt), then the first tile's
  StemTile T = stem_tile<CAP>(tile0 * 256u, G);
  if (tile0 < ntiles) load(tile0 * 256u, T);
  fa_bwd_coef_from(a, f, 64, 0, part, coef[0], coef[1], coef[2]);
  float A[8], B[8], Cc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A[k] = coef[0][c8 * 8 + k];
    B[k] = coef[1][c8 * 8 + k];
    Cc[k] = coef[2][c8 * 8 + k];
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int tsw = trswz(t);
  for (int it = 0; it < tiles; ++it) {
    const uint32_t tile = tile0 + it;
    if (tile >= ntiles) break;
    const uint32_t pix0 = tile * 256u;
    // this tile's dc rows and input rows into LDS
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float d[8], c[8], v[8];
      unpack8(vd[u], d);
      unpack8(vc[u], c);
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = (mk[u] >> k) & 1u ? d[k] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = A[k] * d[k] + B[k] * c[k] + Cc[k];
      const int row = r0 + 32 * u;
      *(uint4*)(dyt + row * 128 + ((c8 ^ trswz(row)) << 4)) = pack8(v);
    }
    stem_stage_st<CAP>(T, G, xv, xt);
    const StemTile Tc = T;
    // the next tile's loads, in flight during this tile's taps and MFMAs
    if (it + 1 < tiles && tile + 1 < ntiles) {
      T = stem_tile<CAP>(pix0 + 256u, G);
      load(pix0 + 256u, T);
    }
    __syncthreads();
    uint4 q[4];
    stem_taps(x, xt, Tc, pix0 + t, G, q);  // zeros past M
    // chunks 0..3 of a col row (the 27 taps + 5 zeros); frag_tr never reads chunks 4..7
#pragma unroll
    for (int j = 0; j < 4; ++j) *(uint4*)(colt + t * 128 + ((j ^ tsw) << 4)) = q[j];
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const bf16x8 fa = frag_tr(dyt, wave * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, frag_tr(colt, j * 16, ks, lane), acc[j], 0, 0, 0);
    }
    __syncthreads();
  }
  float* out = slab + (size_t)blockIdx.x * 64 * 32;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(wave * 16 + 4 * (lane >> 4) + r) * 32 + j * 16 + (lane & 15)] = acc[j][r];
  stamp_end(ts);
}

static int stem_bn_grid(int64_t M, int& tiles) {
  const int64_t ntiles = (M + 255) / 256;
  const int nwg0 = (int)std::min<int64_t>(ntiles, 512);  // two ~78 KB workgroups per CU
  tiles = (int)((ntiles + nwg0 - 1) / nwg0);
  return (int)((ntiles + tiles - 1) / tiles);
}

int stem_wgrad_bn(const float* x, const u16* dy, const uint8_t* mbits, const u16* c, const BnBwdArgs& a, float* dw27,
                  float scale, int N, int H, int W, float* slab, size_t slab_bytes, hipStream_t st, u64* ts) {
  DTC_CHECK_ARG(x && dy && mbits && c && dw27 && slab && a.acc && a.gamma && a.mean && a.invstd && N > 0 && H > 0 &&
                    W > 0,
                "stem_wgrad_bn: bad args");
  const int64_t M = (int64_t)N * H * W;
  DTC_CHECK_ARG(M + 256 < (1ll << 31), "stem_wgrad_bn: more than 2^31 pixels");
  int tiles = 0;
  const int nwg = stem_bn_grid(M, tiles);
  DTC_CHECK_ARG(slab_bytes >= (size_t)nwg * 64 * 32 * 4, "stem_wgrad_bn: slab workspace too small");
  DTC_KLAUNCH(stem_wgrad_bn_kernel<STEM_BN_CAP>, dim3(nwg), dim3(256), 0, st, x, dy, mbits, c, a, slab,
                     stem_geom(N, H, W), tiles, ts);
  DTC_LAUNCH_CHECK();
  return wgrad_reduce_to(slab, nwg, 64, 32, 27, 27, scale, dw27, st, ts);
}

}  // namespace dtc
