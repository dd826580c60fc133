// Stem im2col, global average pool + Linear, and cross-entropy for the ResNet-18 step.
//
//   stem_im2col / stem_pack_weight : `self.conv1 = nn.Conv2d(3, 64, 3, 1, 1)` (reference
//       src/*/net.py:91) lowered to a K=27 GEMM: the 3-channel input is gathered into a
//       zero-padded [pixels][64] bf16 matrix so the stem runs on the same MFMA kernel.
//   head_fwd / head_bwd : `F.avg_pool2d(out, 4)`, `view`, `self.linear` (net.py:113-115).
//       The pool is global over the last feature map (identical to avg_pool2d(4) at 32x32
//       inputs; at 224x224 this is the documented global-pool deviation, SURVEY §7 viii).
//   xent_fwd / xent_bwd : `nn.CrossEntropyLoss()` mean reduction (reference trainer.py:40,155).
#include "common.h"
#include "kernels.h"

namespace dtc {

__global__ void __launch_bounds__(256) stem_im2col_kernel(const float* __restrict__ x, u16* __restrict__ cols,
                                                         int N, int H, int W) {
  const int64_t total = (int64_t)N * H * W * 8;  // 8 chunks of 8 columns per pixel
  for (int64_t t = blockIdx.x * (int64_t)256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int chunk = (int)(t & 7);
    const int64_t pix = t >> 3;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const int n = (int)(pix / ((int64_t)W * H));
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = chunk * 8 + k;  // (r, s, c) with c fastest: KRSC filter order
      float val = 0.f;
      if (j < 27) {
        const int r = j / 9, s = (j / 3) % 3, c = j % 3;
        const int ih = h + r - 1, iw = w + s - 1;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          val = x[(((int64_t)n * 3 + c) * H + ih) * W + iw];
      }
      v[k] = val;
    }
    *(uint4*)(cols + pix * 64 + chunk * 8) = pack8(v);
  }
}

int stem_im2col(const float* x, u16* cols, int N, int H, int W, hipStream_t st) {
  DTC_CHECK_ARG(x && cols && N > 0 && H > 0 && W > 0, "stem_im2col: bad args");
  const int64_t total = (int64_t)N * H * W * 8;
  const int blocks = (int)std::min<int64_t>(8192, (total + 255) / 256);
  hipLaunchKernelGGL(stem_im2col_kernel, dim3(blocks), dim3(256), 0, st, x, cols, N, H, W);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void stem_pack_weight_kernel(const u16* __restrict__ w27, u16* __restrict__ w64, int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= K * 64) return;
  const int k = t >> 6, j = t & 63;
  w64[t] = j < 27 ? w27[k * 27 + j] : (u16)0;
}

int stem_pack_weight(const u16* w27, u16* w64, int K, hipStream_t st) {
  DTC_CHECK_ARG(w27 && w64 && K > 0, "stem_pack_weight: bad args");
  hipLaunchKernelGGL(stem_pack_weight_kernel, dim3((K * 64 + 255) / 256), dim3(256), 0, st, w27, w64, K);
  DTC_LAUNCH_CHECK();
  return 0;
}

// Pool: feat[n][c] = bf16(mean_p act[n][p][c]); one thread per (n, c).
__global__ void __launch_bounds__(256) head_pool_kernel(const u16* __restrict__ act, int N, int HW, int C,
                                                       float* __restrict__ feat) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= (int64_t)N * C) return;
  const int64_t n = i / C, c = i - n * C;
  const u16* a = act + n * HW * C + c;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf2f(a[(int64_t)p * C]);
  feat[i] = round_bf(s / (float)HW);  // avg_pool2d output is bf16 under autocast
}

// Linear: logits[n][j] = bf16(feat[n] . W[j] + bf16(b[j])); one thread per output, 16-byte loads.
__global__ void __launch_bounds__(256) head_fc_kernel(const float* __restrict__ feat, int N, int C,
                                                     const u16* __restrict__ wfc, const float* __restrict__ bfc,
                                                     int ncls, float* __restrict__ logits) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= (int64_t)N * ncls) return;
  const int64_t n = i / ncls, j = i - n * ncls;
  const f32x4* f = (const f32x4*)(feat + n * C);
  const uint4* w = (const uint4*)(wfc + j * C);
  float acc = 0.f;
#pragma unroll 4
  for (int c8 = 0; c8 < C / 8; ++c8) {
    float wv[8];
    unpack8(w[c8], wv);
    const f32x4 a = f[2 * c8], b = f[2 * c8 + 1];
    acc += a[0] * wv[0] + a[1] * wv[1] + a[2] * wv[2] + a[3] * wv[3] + b[0] * wv[4] + b[1] * wv[5] + b[2] * wv[6] +
           b[3] * wv[7];
  }
  logits[i] = round_bf(acc + round_bf(bfc[j]));  // bf16 linear under autocast
}

int head_fwd(const u16* act, int N, int HW, int C, const u16* wfc, const float* bfc, int ncls, float* feat,
             float* logits, hipStream_t st) {
  DTC_CHECK_ARG(act && wfc && bfc && feat && logits && N > 0 && HW > 0 && C > 0 && C % 8 == 0 && ncls > 0,
                "head_fwd: bad args");
  hipLaunchKernelGGL(head_pool_kernel, dim3((int)(((int64_t)N * C + 255) / 256)), dim3(256), 0, st, act, N, HW, C,
                     feat);
  DTC_LAUNCH_CHECK();
  hipLaunchKernelGGL(head_fc_kernel, dim3((int)(((int64_t)N * ncls + 255) / 256)), dim3(256), 0, st, feat, N, C, wfc,
                     bfc, ncls, logits);
  DTC_LAUNCH_CHECK();
  return 0;
}

// per-row log-sum-exp: one wave per row
__global__ void __launch_bounds__(256) xent_lse_kernel(const float* __restrict__ logits, int N, int ncls,
                                                      float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= N) return;
  const float* z = logits + (int64_t)b * ncls;
  float m = -INFINITY;
  for (int j = lane; j < ncls; j += 64) m = fmaxf(m, z[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < ncls; j += 64) s += expf(z[j] - m);
  s = wave_sum(s);
  if (lane == 0) lse[b] = m + logf(s);
}

// loss = mean_b (lse[b] - z[b][y_b]); one workgroup, fixed summation order
__global__ void __launch_bounds__(256) xent_mean_kernel(const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, int N, int ncls,
                                                       float* __restrict__ loss) {
  __shared__ float part[4];
  const int t = threadIdx.x;
  float acc = 0.f;
  for (int b = t; b < N; b += 256) {
    const int64_t y = labels[b];
    acc += (y >= 0 && y < ncls) ? (lse[b] - logits[(int64_t)b * ncls + y]) : NAN;
  }
  acc = wave_sum(acc);
  if ((t & 63) == 0) part[t >> 6] = acc;
  __syncthreads();
  if (t == 0) *loss = (part[0] + part[1] + part[2] + part[3]) / (float)N;
}

int xent_fwd(const float* logits, const int64_t* labels, int N, int ncls, float* loss, float* lse, hipStream_t st) {
  DTC_CHECK_ARG(logits && labels && loss && lse && N > 0 && ncls > 0, "xent_fwd: bad args");
  hipLaunchKernelGGL(xent_lse_kernel, dim3((N + 3) / 4), dim3(256), 0, st, logits, N, ncls, lse);
  DTC_LAUNCH_CHECK();
  hipLaunchKernelGGL(xent_mean_kernel, dim3(1), dim3(256), 0, st, logits, labels, lse, N, ncls, loss);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void __launch_bounds__(256) xent_bwd_kernel(const float* __restrict__ logits,
                                                      const int64_t* __restrict__ labels,
                                                      const float* __restrict__ lse, const float* __restrict__ gscale,
                                                      int N, int ncls, float* __restrict__ dl) {
  const int64_t total = (int64_t)N * ncls;
  const float g = (gscale ? *gscale : 1.f) / (float)N;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / ncls), j = (int)(i % ncls);
    const float p = expf(logits[i] - lse[b]);
    dl[i] = (p - (labels[b] == j ? 1.f : 0.f)) * g;
  }
}

int xent_bwd(const float* logits, const int64_t* labels, const float* lse, const float* gscale, int N, int ncls,
             float* dlogits, hipStream_t st) {
  DTC_CHECK_ARG(logits && labels && lse && dlogits && N > 0 && ncls > 0, "xent_bwd: bad args");
  const int64_t total = (int64_t)N * ncls;
  const int blocks = (int)std::min<int64_t>(1024, (total + 255) / 256);
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(blocks), dim3(256), 0, st, logits, labels, lse, gscale, N, ncls, dlogits);
  DTC_LAUNCH_CHECK();
  return 0;
}

// dW[j][c] = scale * sum_n dl[n][j] * feat[n][c]; db[j] = scale * sum_n dl[n][j]
// Stage 1: workgroup (64 channels, 16 classes, 32 images) -> partial slab [split][j][c] (plain stores).
constexpr int HB_IMGS = 32;
__global__ void __launch_bounds__(256) head_bwd_w_partial_kernel(const float* __restrict__ dl,
                                                                const float* __restrict__ feat, int N, int C,
                                                                int ncls, float* __restrict__ part) {
  __shared__ float dls[HB_IMGS][16];
  const int t = threadIdx.x;
  const int c = blockIdx.x * 64 + (t & 63);
  const int jq = (t >> 6) * 4;
  const int n0 = blockIdx.z * HB_IMGS;
  for (int e = t; e < HB_IMGS * 16; e += 256) {
    const int n = n0 + (e >> 4), j = blockIdx.y * 16 + (e & 15);
    dls[e >> 4][e & 15] = (n < N && j < ncls) ? dl[(int64_t)n * ncls + j] : 0.f;
  }
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int nn = min(HB_IMGS, N - n0);
  if (c < C) {
#pragma unroll 8
    for (int i = 0; i < nn; ++i) {
      const float fv = feat[(int64_t)(n0 + i) * C + c];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += dls[i][jq + q] * fv;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = blockIdx.y * 16 + jq + q;
      if (j < ncls) part[((int64_t)blockIdx.z * ncls + j) * C + c] = acc[q];
    }
  }
  // bias partial of this image block (the c-tile 0 workgroups): one thread per class
  if (blockIdx.x == 0 && t < 16) {
    const int j = blockIdx.y * 16 + t;
    float b = 0.f;
    for (int i = 0; i < nn; ++i) b += dls[i][t];
    if (j < ncls) part[(int64_t)gridDim.z * ncls * C + (int64_t)blockIdx.z * ncls + j] = b;
  }
}

// Stage 2: fixed-order sum over splits; thread per (j, c); db by the c == 0 threads.
__global__ void __launch_bounds__(256) head_bwd_w_reduce_kernel(const float* __restrict__ part, int splits,
                                                               const float* __restrict__ dl, int N, int C, int ncls,
                                                               float scale, float* __restrict__ dw,
                                                               float* __restrict__ db) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i >= (int64_t)ncls * C) return;
  float a = 0.f;
  for (int s = 0; s < splits; ++s) a += part[(int64_t)s * ncls * C + i];
  dw[i] = a * scale;
  const int64_t j = i / C, c = i - j * C;
  if (c == 0) {  // bias: fixed-order sum of the per-image-block partials
    const float* pb = part + (int64_t)splits * ncls * C;
    float b = 0.f;
    for (int s = 0; s < splits; ++s) b += pb[(int64_t)s * ncls + j];
    db[j] = b * scale;
  }
}

size_t head_bwd_workspace(int N, int C, int ncls) {
  return (size_t)((N + HB_IMGS - 1) / HB_IMGS) * ncls * (C + 1) * sizeof(float);
}

// dact[n][p][c] = (sum_j dl[n][j] * W[j][c]) / HW
__global__ void __launch_bounds__(256) head_bwd_x_kernel(const float* __restrict__ dl, const u16* __restrict__ wfc,
                                                        int HW, int C, int ncls, u16* __restrict__ dact) {
  extern __shared__ float row[];
  const int n = blockIdx.x, t = threadIdx.x;
  for (int j = t; j < ncls; j += 256) row[j] = dl[(int64_t)n * ncls + j];
  __syncthreads();
  const float inv = 1.f / (float)HW;
  u16* o = dact + (int64_t)n * HW * C;
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int j = 0; j < ncls; ++j) s += row[j] * bf2f(wfc[(int64_t)j * C + c]);
    const u16 v = f2bf(s * inv);
    for (int p = 0; p < HW; ++p) o[(int64_t)p * C + c] = v;
  }
}

int head_bwd(const float* dlogits, const float* feat, const u16* wfc, int N, int HW, int C, int ncls, float scale,
             float* dw, float* db, u16* dact, float* ws, size_t ws_bytes, hipStream_t st) {
  DTC_CHECK_ARG(dlogits && feat && wfc && dw && db && dact && N > 0 && HW > 0 && C > 0 && ncls > 0,
                "head_bwd: bad args");
  DTC_CHECK_ARG(ws && ws_bytes >= head_bwd_workspace(N, C, ncls), "head_bwd: workspace too small");
  const int splits = (N + HB_IMGS - 1) / HB_IMGS;
  hipLaunchKernelGGL(head_bwd_w_partial_kernel, dim3((C + 63) / 64, (ncls + 15) / 16, splits), dim3(256), 0, st,
                     dlogits, feat, N, C, ncls, ws);
  DTC_LAUNCH_CHECK();
  hipLaunchKernelGGL(head_bwd_w_reduce_kernel, dim3((int)(((int64_t)ncls * C + 255) / 256)), dim3(256), 0, st, ws,
                     splits, dlogits, N, C, ncls, scale, dw, db);
  DTC_LAUNCH_CHECK();
  hipLaunchKernelGGL(head_bwd_x_kernel, dim3(N), dim3(256), ncls * sizeof(float), st, dlogits, wfc, HW, C, ncls,
                     dact);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
