// fp32 implicit-GEMM convolution on the f32-input MFMA (v_mfma_f32_16x16x4_f32) for gfx950.
//
// fp32 mode of the executor: the reference trains in plain fp32 when --amp is off
// (ddp/trainer.py:160-165, single/trainer.py:144-145), so nn.Conv2d (net.py:18-24, 29-35, 91) runs
// fp32 in / fp32 out there. gfx950 has no xf32 / TF32 MFMA: v_mfma_f32_16x16x4_f32 is exact f32
// (a k-ordered fmaf chain) at the fp32 vector rate (157 TF/s), so these kernels give fp32 results
// at the north_star's 1e-5 tolerance.
//
// One template serves the three passes as D[m][n] = sum_k A[m][k] B[k][n]:
//   mode   rows m            cols n         reduction k      A[m][k]                     B[k][n]
//   FWD    output pixel      out channel    (r, s, c)        x[pixel shifted by (r,s)][c] w[n][r][s][c]
//   DGRAD  input pixel       in channel     (r, s, k)        dy[pixel^-1(r,s)][k]         w[k][r][s][n]
//   WGRAD  out channel       (r, s, c)      pixel            dy[pixel][m]                 x[pixel shifted][c]
// Tiles of 64x64 outputs (4 waves, 2x2 fragments of 16x16 each), reduction stages of 16 staged in
// LDS as [16][64] k-major images (the MFMA reads A[l&15][k = l>>4] / B[k = l>>4][l&15] as single
// floats); the next stage's global loads are issued into registers before the current stage's
// MFMAs (register double buffering). FWD epilogue: fp32 output + per-channel (sum, sum^2) into the
// fp64 BatchNorm slots; DGRAD: fp32 output (+ residual); WGRAD: split-K fp32 slabs reduced in a
// fixed order by f32_wgrad_reduce (deterministic).
#include "common.h"
#include "kernels.h"
#include "tile_common.h"

namespace dtc {

enum { F32_FWD = 0, F32_DGRAD = 1, F32_WGRAD = 2 };

struct F32ConvParams {
  const float* src0;  // FWD x, DGRAD dy, WGRAD x
  const float* src1;  // FWD w, DGRAD w, WGRAD dy
  float* out;         // FWD y, DGRAD dx, WGRAD slab [split][K][RSC]
  const float* res;   // DGRAD residual (optional)
  int64_t* stats;      // FWD BN statistics slots (optional)
  int N, H, W, C, K, R, S, P, Q, stride, pad;
  int M;      // GEMM rows
  int NC;     // GEMM cols
  int RSC;
  int64_t red;          // reduction length
  int steps_per_split;  // reduction stages of 16 per split
  FastDiv fd_q, fd_pq;  // FWD/WGRAD: output Q, P*Q ; DGRAD: input W, H*W
  u64* ts;
};

constexpr int F32_BM = 64, F32_BN = 64, F32_KS = 16, F32_LD = 68;

template <int MODE>
__global__ void __launch_bounds__(256) conv_f32_kernel(const F32ConvParams p) {
  __shared__ float As[F32_KS][F32_LD];
  __shared__ float Bs[F32_KS][F32_LD];
  __shared__ float red[2][2][F32_BN];
  stamp_start(p.ts);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int tiles_m = (p.M + F32_BM - 1) / F32_BM;
  const int m0 = (blockIdx.x % tiles_m) * F32_BM;
  const int n0 = (blockIdx.x / tiles_m) * F32_BN;
  const int64_t nsteps = (p.red + F32_KS - 1) / F32_KS;
  const int64_t s_begin = (int64_t)blockIdx.y * p.steps_per_split;
  const int64_t s_end = min(nsteps, s_begin + p.steps_per_split);

  // ---- per-thread load coordinates (fixed over the reduction)
  // A: FWD/DGRAD thread -> (row = t/4, red chunk (t%4)*4); WGRAD thread -> (red row t/16, col chunk (t%16)*4)
  // B: FWD thread -> (col = t/4, red chunk (t%4)*4); DGRAD/WGRAD -> (red row t/16, col chunk (t%16)*4)
  int a_n = 0, a_h = 0, a_w = 0;  // A row's image / spatial position (FWD, DGRAD)
  bool a_ok = false;
  if constexpr (MODE != F32_WGRAD) {
    const int m = m0 + (t >> 2);
    a_ok = m < p.M;
    if (a_ok) {
      a_n = (int)fdiv((uint32_t)m, p.fd_pq);
      const int rem = m - a_n * (int)p.fd_pq.d;
      a_h = (int)fdiv((uint32_t)rem, p.fd_q);
      a_w = rem - a_h * (int)p.fd_q.d;
    }
  }

  auto load_a = [&](int64_t step) -> f32x4 {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if constexpr (MODE == F32_FWD) {
      if (!a_ok) return z;
      const int kr = (int)(step * F32_KS) + (t & 3) * 4;  // (r, s, c): C % 16 == 0 -> one tap per stage
      const int tap = kr / p.C, c = kr - tap * p.C;
      const int r = tap / p.S, s = tap - r * p.S;
      const int ih = a_h * p.stride - p.pad + r, iw = a_w * p.stride - p.pad + s;
      if ((unsigned)ih >= (unsigned)p.H || (unsigned)iw >= (unsigned)p.W) return z;
      return *(const f32x4*)(p.src0 + (((int64_t)a_n * p.H + ih) * p.W + iw) * p.C + c);
    } else if constexpr (MODE == F32_DGRAD) {
      if (!a_ok) return z;
      const int kr = (int)(step * F32_KS) + (t & 3) * 4;  // (r, s, k)
      const int tap = kr / p.K, k = kr - tap * p.K;
      const int r = tap / p.S, s = tap - r * p.S;
      int ph = a_h + p.pad - r, pw = a_w + p.pad - s;
      if (ph < 0 || pw < 0) return z;
      if (p.stride == 2) {
        if ((ph & 1) || (pw & 1)) return z;
        ph >>= 1;
        pw >>= 1;
      }
      if (ph >= p.P || pw >= p.Q) return z;
      return *(const f32x4*)(p.src0 + (((int64_t)a_n * p.P + ph) * p.Q + pw) * p.K + k);
    } else {  // WGRAD: A[kout][pixel] = dy[pixel][kout]
      const int64_t pix = step * F32_KS + (t >> 4);
      const int kout = m0 + (t & 15) * 4;
      if (pix >= p.red || kout >= p.M) return z;
      return *(const f32x4*)(p.src1 + pix * p.K + kout);
    }
  };
  auto load_b = [&](int64_t step) -> f32x4 {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if constexpr (MODE == F32_FWD) {  // w[col][red]
      const int col = n0 + (t >> 2);
      const int kr = (int)(step * F32_KS) + (t & 3) * 4;
      if (col >= p.NC) return z;
      return *(const f32x4*)(p.src1 + (int64_t)col * p.RSC + kr);
    } else if constexpr (MODE == F32_DGRAD) {  // w[k][r][s][col], red = (r, s, k)
      const int kr = (int)(step * F32_KS) + (t >> 4);
      const int col = n0 + (t & 15) * 4;
      if (col >= p.NC) return z;
      const int tap = kr / p.K, k = kr - tap * p.K;
      return *(const f32x4*)(p.src1 + ((int64_t)k * p.R * p.S + tap) * p.C + col);
    } else {  // WGRAD: x[pixel shifted by tap][c], col = (r, s, c)
      const int64_t pix = step * F32_KS + (t >> 4);
      const int col = n0 + (t & 15) * 4;
      if (pix >= p.red || col >= p.NC) return z;
      const int tap = col / p.C, c = col - tap * p.C;
      const int r = tap / p.S, s = tap - r * p.S;
      const int n = (int)fdiv((uint32_t)pix, p.fd_pq);
      const int rem = (int)pix - n * (int)p.fd_pq.d;
      const int pp = (int)fdiv((uint32_t)rem, p.fd_q);
      const int qq = rem - pp * (int)p.fd_q.d;
      const int ih = pp * p.stride - p.pad + r, iw = qq * p.stride - p.pad + s;
      if ((unsigned)ih >= (unsigned)p.H || (unsigned)iw >= (unsigned)p.W) return z;
      return *(const f32x4*)(p.src0 + (((int64_t)n * p.H + ih) * p.W + iw) * p.C + c);
    }
  };
  auto store_a = [&](const f32x4& v) {
    if constexpr (MODE != F32_WGRAD) {  // transpose: 4 reduction values of one row
      const int row = t >> 2, k = (t & 3) * 4;
      As[k + 0][row] = v[0];
      As[k + 1][row] = v[1];
      As[k + 2][row] = v[2];
      As[k + 3][row] = v[3];
    } else {
      *(f32x4*)&As[t >> 4][(t & 15) * 4] = v;
    }
  };
  auto store_b = [&](const f32x4& v) {
    if constexpr (MODE == F32_FWD) {
      const int col = t >> 2, k = (t & 3) * 4;
      Bs[k + 0][col] = v[0];
      Bs[k + 1][col] = v[1];
      Bs[k + 2][col] = v[2];
      Bs[k + 3][col] = v[3];
    } else {
      *(f32x4*)&Bs[t >> 4][(t & 15) * 4] = v;
    }
  };

  const int wr = wave >> 1, wc = wave & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (s_begin < s_end) {
    f32x4 ra = load_a(s_begin), rb = load_b(s_begin);
    for (int64_t st = s_begin; st < s_end; ++st) {
      __syncthreads();  // previous stage's fragment reads are done
      store_a(ra);
      store_b(rb);
      __syncthreads();
      if (st + 1 < s_end) {  // next stage's loads in flight during this stage's MFMAs
        ra = load_a(st + 1);
        rb = load_b(st + 1);
      }
#pragma unroll
      for (int kk = 0; kk < F32_KS / 4; ++kk) {
        const int kr = kk * 4 + (lane >> 4);
        float af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = As[kr][wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = Bs[kr][wc * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: D[row = 32 wr + 16 i + 4 (lane >> 4) + v][col = 32 wc + 16 j + (lane & 15)]
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  if constexpr (MODE == F32_WGRAD) {
    float* slab = p.out + (size_t)blockIdx.y * p.M * p.RSC;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wc * 32 + j * 16 + cl;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = m0 + wr * 32 + i * 16 + rq + v;
          if (row < p.M && col < p.NC) slab[(size_t)row * p.RSC + col] = acc[i][j][v];
        }
      }
  } else {
    float s[2] = {0.f, 0.f}, q[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wc * 32 + j * 16 + cl;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = m0 + wr * 32 + i * 16 + rq + v;
          float d = acc[i][j][v];
          if (row < p.M && col < p.NC) {
            const size_t o = (size_t)row * p.NC + col;
            if constexpr (MODE == F32_DGRAD) {
              if (p.res) d += p.res[o];
            }
            p.out[o] = d;
          }
          s[j] += d;  // rows beyond M hold exact zeros (their operands were zero-filled)
          q[j] += d * d;
        }
      }
    if constexpr (MODE == F32_FWD) {
      if (p.stats != nullptr) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          s[j] += __shfl_xor(s[j], 16, 64);
          s[j] += __shfl_xor(s[j], 32, 64);
          q[j] += __shfl_xor(q[j], 16, 64);
          q[j] += __shfl_xor(q[j], 32, 64);
          if (lane < 16) {
            red[wr][0][wc * 32 + j * 16 + lane] = s[j];
            red[wr][1][wc * 32 + j * 16 + lane] = q[j];
          }
        }
        __syncthreads();
        if (t < F32_BN && n0 + t < p.NC) {
          stat_add(p.stats, p.NC, n0 + t, red[0][0][t] + red[1][0][t], red[0][1][t] + red[1][1][t]);
        }
      }
    }
  }
  stamp_end(p.ts);
}

// dw[k][0:ncols] (row stride ld_out) = scale * sum_s slab[s][k][0:RSC], fixed split order
__global__ void __launch_bounds__(256) f32_wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K,
                                                              int RSC, int ncols, int ld_out, float scale,
                                                              float* __restrict__ dw, u64* ts) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int64_t plane = (int64_t)K * RSC;
  if (i < (int64_t)K * ncols) {
    const int k = (int)(i / ncols), c = (int)(i - (int64_t)k * ncols);
    float a = 0.f;
    for (int sp = 0; sp < splits; ++sp) a += slab[sp * plane + (int64_t)k * RSC + c];
    dw[(int64_t)k * ld_out + c] = a * scale;
  }
  stamp_end(ts);
}

// ---------------------------------------------------------------- stem (fp32): im2col + weight pack
// cols[pixel][32]: the 27 taps (r, s, c; c fastest = KRSC filter order) of NCHW fp32 input, 5 zeros
__global__ void __launch_bounds__(256) f32_stem_im2col_kernel(const float* __restrict__ x, float* __restrict__ cols,
                                                             int N, int H, int W) {
  const int64_t M = (int64_t)N * H * W;
  const int64_t pix = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (pix >= M) return;
  const int w = (int)(pix % W);
  const int h = (int)((pix / W) % H);
  const int n = (int)(pix / ((int64_t)W * H));
  const float* xn = x + (int64_t)n * 3 * H * W;
  float v[32];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int ih = h + r - 1, iw = w + s - 1;
      const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[(r * 3 + s) * 3 + c] = in ? xn[((int64_t)c * H + ih) * W + iw] : 0.f;
    }
#pragma unroll
  for (int k = 27; k < 32; ++k) v[k] = 0.f;
  f32x4* dst = (f32x4*)(cols + pix * 32);
#pragma unroll
  for (int q = 0; q < 8; ++q) dst[q] = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}

__global__ void f32_stem_pack_weight_kernel(const float* __restrict__ w27, float* __restrict__ w32, int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= K * 32) return;
  const int k = t >> 5, j = t & 31;
  w32[t] = j < 27 ? w27[k * 27 + j] : 0.f;
}

int f32_stem_im2col(const float* x, float* cols, int N, int H, int W, hipStream_t st) {
  DTC_CHECK_ARG(x && cols && N > 0 && H > 0 && W > 0, "f32_stem_im2col: bad args");
  const int64_t M = (int64_t)N * H * W;
  DTC_KLAUNCH(f32_stem_im2col_kernel, dim3((int)((M + 255) / 256)), dim3(256), 0, st, x, cols, N, H, W);
  DTC_LAUNCH_CHECK();
  return 0;
}

int f32_stem_pack_weight(const float* w27, float* w32, int K, hipStream_t st) {
  DTC_CHECK_ARG(w27 && w32 && K > 0, "f32_stem_pack_weight: bad args");
  DTC_KLAUNCH(f32_stem_pack_weight_kernel, dim3((K * 32 + 255) / 256), dim3(256), 0, st, w27, w32, K);
  DTC_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- host side
static int f32_fill(F32ConvParams& p, const ConvShape& s) {
  p.N = s.N; p.H = s.H; p.W = s.W; p.C = s.C; p.K = s.K; p.R = s.R; p.S = s.S;
  p.stride = s.stride; p.pad = s.pad;
  p.P = (s.H + 2 * s.pad - s.R) / s.stride + 1;
  p.Q = (s.W + 2 * s.pad - s.S) / s.stride + 1;
  p.RSC = s.R * s.S * s.C;
  DTC_CHECK_ARG(s.C % 16 == 0 && s.K % 16 == 0, "conv_f32: C (%d) and K (%d) must be multiples of 16", s.C, s.K);
  DTC_CHECK_ARG(s.stride == 1 || s.stride == 2, "conv_f32: stride must be 1 or 2");
  DTC_CHECK_ARG(s.N > 0 && p.P > 0 && p.Q > 0 && (int64_t)s.N * s.H * s.W < (1ll << 31), "conv_f32: bad geometry");
  return 0;
}

static int ceil_div_f(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

int f32_wgrad_splits(const ConvShape& s) {
  const int P = (s.H + 2 * s.pad - s.R) / s.stride + 1, Q = (s.W + 2 * s.pad - s.S) / s.stride + 1;
  const int64_t nsteps = ((int64_t)s.N * P * Q + F32_KS - 1) / F32_KS;
  const int tiles = ceil_div_f(s.K, F32_BM) * ceil_div_f((int64_t)s.R * s.S * s.C, F32_BN);
  int64_t splits = std::max<int64_t>(1, 512 / tiles);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, nsteps / 8));  // >= 8 stages per workgroup
  return (int)splits;
}

size_t f32_conv_workspace(const ConvShape& s, int mode) {
  if (mode != CONV_WGRAD) return 0;
  return (size_t)f32_wgrad_splits(s) * s.K * s.R * s.S * s.C * 4;
}

int conv_f32(const ConvShape& s, int mode, const float* a, const float* b, float* out, const float* res,
             int64_t* stats, float* dw_ld_or_null, int dw_cols, int dw_ld, float scale, float* slab,
             size_t slab_bytes, hipStream_t st, u64* ts) {
  F32ConvParams p{};
  DTC_TRY(f32_fill(p, s));
  p.ts = ts;
  if (mode == CONV_FWD) {
    p.src0 = a; p.src1 = b; p.out = out; p.stats = stats;
    p.M = s.N * p.P * p.Q;
    p.NC = s.K;
    p.red = p.RSC;
    p.fd_q = make_fastdiv(p.Q); p.fd_pq = make_fastdiv(p.P * p.Q);
    p.steps_per_split = (int)((p.red + F32_KS - 1) / F32_KS);
    dim3 grid(ceil_div_f(p.M, F32_BM) * ceil_div_f(p.NC, F32_BN), 1);
    DTC_KLAUNCH(conv_f32_kernel<F32_FWD>, grid, dim3(256), 0, st, p);
    DTC_LAUNCH_CHECK();
    return 0;
  }
  if (mode == CONV_DGRAD) {
    p.src0 = a; p.src1 = b; p.out = out; p.res = res;
    p.M = s.N * s.H * s.W;
    p.NC = s.C;
    p.red = (int64_t)s.R * s.S * s.K;
    p.fd_q = make_fastdiv(s.W); p.fd_pq = make_fastdiv(s.H * s.W);
    p.steps_per_split = (int)((p.red + F32_KS - 1) / F32_KS);
    dim3 grid(ceil_div_f(p.M, F32_BM) * ceil_div_f(p.NC, F32_BN), 1);
    DTC_KLAUNCH(conv_f32_kernel<F32_DGRAD>, grid, dim3(256), 0, st, p);
    DTC_LAUNCH_CHECK();
    return 0;
  }
  // WGRAD: a = x, b = dy
  DTC_CHECK_ARG(dw_ld_or_null != nullptr && slab != nullptr, "conv_f32 wgrad: null output / slab");
  p.src0 = a; p.src1 = b;
  p.M = s.K;
  p.NC = p.RSC;
  p.red = (int64_t)s.N * p.P * p.Q;
  p.fd_q = make_fastdiv(p.Q); p.fd_pq = make_fastdiv(p.P * p.Q);
  int splits = f32_wgrad_splits(s);
  while (splits > 1 && (size_t)splits * s.K * p.RSC * 4 > slab_bytes) --splits;
  DTC_CHECK_ARG((size_t)s.K * p.RSC * 4 <= slab_bytes, "conv_f32 wgrad: slab workspace too small");
  const int64_t nsteps = (p.red + F32_KS - 1) / F32_KS;
  p.steps_per_split = (int)((nsteps + splits - 1) / splits);
  splits = (int)((nsteps + p.steps_per_split - 1) / p.steps_per_split);
  p.out = slab;
  dim3 grid(ceil_div_f(p.M, F32_BM) * ceil_div_f(p.NC, F32_BN), splits);
  DTC_KLAUNCH(conv_f32_kernel<F32_WGRAD>, grid, dim3(256), 0, st, p);
  DTC_LAUNCH_CHECK();
  const int ncols = dw_cols > 0 ? dw_cols : p.RSC;
  const int ldo = dw_ld > 0 ? dw_ld : p.RSC;
  DTC_KLAUNCH(f32_wgrad_reduce_kernel, dim3(ceil_div_f((int64_t)s.K * ncols, 256)), dim3(256), 0, st, slab,
                     splits, s.K, p.RSC, ncols, ldo, scale, dw_ld_or_null, ts);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
