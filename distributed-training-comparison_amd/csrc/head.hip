// Stem im2col, global average pool + Linear, and cross-entropy for the ResNet-18 step.
//
//   stem_im2col / stem_pack_weight : `self.conv1 = nn.Conv2d(3, 64, 3, 1, 1)` (reference
//       src/*/net.py:91) lowered to a K=27 GEMM: the 3-channel input is gathered into a
//       zero-padded [pixels][64] bf16 matrix so the stem runs on the same MFMA kernel.
//   head_fwd / head_bwd : `F.avg_pool2d(out, 4)`, `view`, `self.linear` (net.py:113-115).
//       The pool is global over the last feature map (identical to avg_pool2d(4) at 32x32
//       inputs; at 224x224 this is the documented global-pool deviation, SURVEY §7 viii).
//   xent_fwd / xent_bwd : `nn.CrossEntropyLoss()` mean reduction (reference trainer.py:40,155).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace dtc {

__global__ void __launch_bounds__(256) stem_im2col_kernel(const float* __restrict__ x, u16* __restrict__ cols,
                                                         int N, int H, int W) {
  // One thread per output pixel: its 27 taps (r, s, c with c fastest: KRSC filter order) are read
  // from NCHW fp32 (per tap the lanes of a wave read consecutive pixels: coalesced) and written as
  // columns 0..31 of the pixel's row into LDS; the workgroup's 256 rows (32 KB) are then stored as
  // contiguous 16-B lanes, columns 32..63 as zeros.
  __shared__ uint4 rows[256 * 4];
  const int t = threadIdx.x;
  const int64_t M = (int64_t)N * H * W;
  const int64_t pix0 = (int64_t)blockIdx.x * 256, pix = pix0 + t;
  if (pix < M) {
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
#pragma unroll
    for (int q = 0; q < 4; ++q) rows[t * 4 + (q ^ (t & 3))] = pack8(v + q * 8);
  }
  __syncthreads();
  const int64_t nrow = std::min<int64_t>(256, M - pix0);
  uint4* dst = (uint4*)(cols + pix0 * 64);
  for (int e = t; e < nrow * 8; e += 256) {
    const int row = e >> 3, q = e & 7;
    dst[e] = q < 4 ? rows[row * 4 + (q ^ (row & 3))] : uint4{0u, 0u, 0u, 0u};
  }
}

int stem_im2col(const float* x, u16* cols, int N, int H, int W, hipStream_t st) {
  DTC_CHECK_ARG(x && cols && N > 0 && H > 0 && W > 0, "stem_im2col: bad args");
  const int64_t M = (int64_t)N * H * W;
  const int blocks = (int)((M + 255) / 256);
  DTC_KLAUNCH(stem_im2col_kernel, dim3(blocks), dim3(256), 0, st, x, cols, N, H, W);
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
  DTC_KLAUNCH(stem_pack_weight_kernel, dim3((K * 64 + 255) / 256), dim3(256), 0, st, w27, w64, K);
  DTC_LAUNCH_CHECK();
  return 0;
}

// Pool + Linear in one launch, one workgroup per image:
//   feat[n][c] = bf16(mean_p act[n][p][c])                 (avg_pool2d output is bf16 under autocast)
//   logits[n][j] = bf16(feat[n] . W[j] + bf16(b[j]))         (bf16 linear under autocast)
// The pool's threads own 8 channels each (16-B loads of consecutive channels, pixels split over
// the workgroup's row groups and combined in LDS in a fixed order). For the Linear eight lanes share
// a class row: lane r of the group reads 16-B chunks r, r + 8, ... (every load instruction covers
// eight whole 128-B row pieces: coalesced, all of a lane's loads in flight at once), FMAs them against
// the pooled features in LDS, and the group's partials meet in a fixed xor-shuffle tree; a wave takes
// eight classes per pass, the workgroup 32. Both reductions have a fixed order: deterministic.
template <typename T>
__global__ void __launch_bounds__(256) head_fwd_kernel(const T* __restrict__ act, int HW, int C,
                                                      const T* __restrict__ wfc, const float* __restrict__ bfc,
                                                      int ncls, float* __restrict__ feat, float* __restrict__ logits) {
  typedef Elt<T> E;
  extern __shared__ float hsm[];  // [C] feat, then [256 / (C/8)][C] pool partials
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int tpr = C >> 3, groups = max(1, 256 / tpr);
  float* fs = hsm;
  float* part = hsm + C;
  const T* a = act + (int64_t)n * HW * C;
  // bf16, C = 512, <= 128 classes (the model's head): every weight chunk and bias this lane's Linear needs
  // (four passes x eight 16-B chunks) is loaded FIRST, beside the pool's loads -- one memory latency for the
  // kernel instead of one per pass (each dependent global access costs ~1 us here)
  constexpr bool BF = std::is_same<T, u16>::value;
  const bool fast = BF && C == 512 && ncls <= 128;
  const int r8 = lane & 7;
  typename E::V wpf[BF ? 4 : 1][8];
  float bpf[4];
  if constexpr (BF) {
    if (fast) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = q * 32 + wave * 8 + (lane >> 3), jj = j < ncls ? j : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) wpf[q][u] = E::ld(wfc + (int64_t)jj * 512 + (r8 + 8 * u) * 8);
        bpf[q] = bfc[jj];
      }
    }
  }
  for (int c8 = t % tpr; c8 < tpr; c8 += 256) {  // (tpr > 256: threads loop over channel groups)
    const int g = t / tpr;
    if (g >= groups) break;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int p = g;
    for (; p + 3 * groups < HW; p += 4 * groups) {  // four pixels' loads in flight, then their adds in order
      typename E::V q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = E::ld(a + (int64_t)(p + u * groups) * C + c8 * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v[8];
        E::unpack(q[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += v[k];
      }
    }
    for (; p < HW; p += groups) {
      float v[8];
      E::unpack(E::ld(a + (int64_t)p * C + c8 * 8), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) part[g * C + c8 * 8 + k] = s[k];
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int g = 0; g < groups; ++g) s += part[g * C + c];
    const float f = E::round(s / (float)HW);
    fs[c] = f;
    feat[(int64_t)n * C + c] = f;
  }
  __syncthreads();
  // Linear: class j = pass * 32 + wave * 8 + (lane >> 3); lane r = lane & 7 of its group
  if constexpr (BF) {
    if (fast) {  // the same sums in the same order as the loop below, from the prefetched chunks
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = q * 32 + wave * 8 + (lane >> 3);
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float f[8];
          E::unpack(wpf[q][u], f);
          const float* fc = fs + (r8 + 8 * u) * 8;
#pragma unroll
          for (int k = 0; k < 8; ++k) acc += fc[k] * f[k];
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (j < ncls && r8 == 0) logits[(int64_t)n * ncls + j] = E::round(acc + E::round(bpf[q]));
      }
      return;
    }
  }
  const int nch = C >> 3;
  for (int j0 = 0; j0 < ncls; j0 += 32) {
    const int j = j0 + wave * 8 + (lane >> 3);
    const bool ok = j < ncls;
    const T* w = wfc + (int64_t)(ok ? j : 0) * C;
    float acc = 0.f;
    for (int c8 = r8; c8 < nch; c8 += 64) {  // (C > 512: further 64-chunk rounds)
      typename E::V wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (c8 + 8 * u < nch) wv[u] = E::ld(w + (c8 + 8 * u) * 8);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (c8 + 8 * u >= nch) break;
        float f[8];
        E::unpack(wv[u], f);
        const float* fc = fs + (c8 + 8 * u) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += fc[k] * f[k];
      }
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (ok && r8 == 0) logits[(int64_t)n * ncls + j] = E::round(acc + E::round(bfc[j]));
  }
}

template <typename T>
static int head_fwd_t(const T* act, int N, int HW, int C, const T* wfc, const float* bfc, int ncls, float* feat,
                      float* logits, hipStream_t st) {
  DTC_CHECK_ARG(act && wfc && bfc && feat && logits && N > 0 && HW > 0 && C > 0 && C % 32 == 0 && C <= 2048 &&
                    ncls > 0,
                "head_fwd: bad args");
  const int groups = std::max(1, 256 / (C / 8));
  const size_t lds = (size_t)(C + std::max(groups * C, 256)) * sizeof(float);
  DTC_KLAUNCH(head_fwd_kernel<T>, dim3(N), dim3(256), lds, st, act, HW, C, wfc, bfc, ncls, feat, logits);
  DTC_LAUNCH_CHECK();
  return 0;
}
int head_fwd(const u16* act, int N, int HW, int C, const u16* wfc, const float* bfc, int ncls, float* feat,
             float* logits, hipStream_t st) {
  return head_fwd_t<u16>(act, N, HW, C, wfc, bfc, ncls, feat, logits, st);
}
int head_fwd(const float* act, int N, int HW, int C, const float* wfc, const float* bfc, int ncls, float* feat,
             float* logits, hipStream_t st) {
  return head_fwd_t<float>(act, N, HW, C, wfc, bfc, ncls, feat, logits, st);
}

// Per-row log-sum-exp: sixteen lanes per row (one DPP row), lane l holding z[l], z[l + 16], ...: a per-lane
// max / sum over its values, then the 16-lane DPP tree (four VALU steps, no LDS permutes). The same function
// (same per-lane order, same tree) serves xent_lse_kernel and the one-launch xent_fwd_fused_kernel, so both
// produce bit-identical lse and loss.
__device__ __forceinline__ float row_lse16(const float* __restrict__ z, int ncls, int li) {
  float m = -INFINITY;
#pragma unroll 8
  for (int j = li; j < ncls; j += 16) m = fmaxf(m, z[j]);
  m = row16_max(m);
  float s = 0.f;
#pragma unroll 8
  for (int j = li; j < ncls; j += 16) s += expf(z[j] - m);
  s = row16_sum(s);
  return m + logf(s);
}

__global__ void __launch_bounds__(256) xent_lse_kernel(const float* __restrict__ logits, int N, int ncls,
                                                      float* __restrict__ lse) {
  const int li = threadIdx.x & 15;
  const int b = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (b >= N) return;  // (whole 16-lane rows retire together: the DPP tree never reads a retired lane)
  const float v = row_lse16(logits + (int64_t)b * ncls, ncls, li);
  if (li == 0) lse[b] = v;
}

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
  DTC_KLAUNCH(xent_lse_kernel, dim3((N + 15) / 16), dim3(256), 0, st, logits, N, ncls, lse);
  DTC_LAUNCH_CHECK();
  DTC_KLAUNCH(xent_mean_kernel, dim3(1), dim3(256), 0, st, logits, labels, lse, N, ncls, loss);
  DTC_LAUNCH_CHECK();
  return 0;
}

// The training step's loss in ONE launch (one 1024-thread workgroup, N <= XF_MAX_ROWS): the per-row
// log-sum-exp exactly as xent_lse_kernel computes it (row_lse16), the mean exactly as xent_mean_kernel
// sums it (same lanes, same order: bit-identical loss), then loss x scale (GradScaler.scale, amp_scale's
// multiply) and the loss stored into a pinned host word (the item() value: no copy launch). Replaces
// xent_lse + xent_mean + a device-to-host copy + amp_scale on the path to the per-step barrier.
constexpr int XF_MAX_ROWS = 4096;
__global__ void __launch_bounds__(1024) xent_fwd_fused_kernel(const float* __restrict__ logits,
                                                             const int64_t* __restrict__ labels, int N, int ncls,
                                                             float* __restrict__ loss, float* __restrict__ lse,
                                                             const float* __restrict__ scale, float* __restrict__ scaled,
                                                             float* host) {
  __shared__ float sterm[XF_MAX_ROWS];  // lse - logit[label] per row (xent_mean_kernel's term)
  __shared__ float part[4];
  const int t = threadIdx.x, li = t & 15, lane = t & 63;
  if (ncls <= 128) {
    // Every dependent global access costs ~1 us here, so each thread first issues ALL its loads -- four
    // rows' values (lane li: z[li + 16 k]) and labels -- and only then reduces: one memory latency per
    // four rounds of 64 rows. The folds match row_lse16 (same per-lane order, same DPP tree); the label's
    // logit is read from the lane holding it (a permute within the row) instead of reloaded.
    constexpr int RR = 4, KV = 8;
    for (int b0 = t >> 4; b0 < N; b0 += 64 * RR) {
      float v[RR][KV];
      int64_t y[RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        const int b = b0 + 64 * r, bb = b < N ? b : 0;
        const float* z = logits + (int64_t)bb * ncls;
#pragma unroll
        for (int k = 0; k < KV; ++k) v[r][k] = li + 16 * k < ncls ? z[li + 16 * k] : 0.f;
        y[r] = labels[bb];
      }
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        const int b = b0 + 64 * r;
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < KV; ++k)
          if (li + 16 * k < ncls) m = fmaxf(m, v[r][k]);
        m = row16_max(m);
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < KV; ++k)
          if (li + 16 * k < ncls) sum += expf(v[r][k] - m);
        sum = row16_sum(sum);
        const float l = m + logf(sum);
        const bool ok = y[r] >= 0 && y[r] < ncls;
        const int yl = ok ? (int)y[r] : 0;
        float cand = 0.f;
#pragma unroll
        for (int k = 0; k < KV; ++k) cand = (yl >> 4) == k ? v[r][k] : cand;
        const float zy = __shfl(cand, (lane & ~15) | (yl & 15));
        if (li == 0 && b < N) {
          lse[b] = l;
          sterm[b] = ok ? (l - zy) : NAN;
        }
      }
    }
  } else {
    for (int b = t >> 4; b < N; b += 64) {  // 64 rows per round, sixteen lanes each
      const float* z = logits + (int64_t)b * ncls;
      const float v = row_lse16(z, ncls, li);
      if (li == 0) {
        lse[b] = v;
        const int64_t y = labels[b];
        sterm[b] = (y >= 0 && y < ncls) ? (v - z[y]) : NAN;
      }
    }
  }
  __syncthreads();
  if (t < 256) {  // the mean exactly as xent_mean_kernel sums it
    float acc = 0.f;
    for (int b = t; b < N; b += 256) acc += sterm[b];
    acc = wave_sum(acc);
    if ((t & 63) == 0) part[t >> 6] = acc;
  }
  __syncthreads();
  if (t == 0) {
    const float l = (part[0] + part[1] + part[2] + part[3]) / (float)N;
    *loss = l;
    if (scaled) *scaled = l * *scale;
    if (host) *host = l;
  }
}

int xent_fwd_fused(const float* logits, const int64_t* labels, int N, int ncls, float* loss, float* lse,
                   const float* scale, float* scaled, float* host, hipStream_t st) {
  DTC_CHECK_ARG(logits && labels && loss && lse && N > 0 && N <= XF_MAX_ROWS && ncls > 0 && (!scaled || scale),
                "xent_fwd_fused: bad args (N=%d)", N);
  DTC_KLAUNCH(xent_fwd_fused_kernel, dim3(1), dim3(1024), 0, st, logits, labels, N, ncls, loss, lse, scale,
                     scaled, host);
  DTC_LAUNCH_CHECK();
  return 0;
}

// d loss / d logit = (softmax - onehot) * gscale / N: one definition for xent_bwd and the fused head backward
__device__ __forceinline__ float xent_gain(const float* gscale, int N) { return (gscale ? *gscale : 1.f) / (float)N; }
__device__ __forceinline__ float xent_grad(float z, float lse, bool hit, float g) {
  return (expf(z - lse) - (hit ? 1.f : 0.f)) * g;
}

__global__ void __launch_bounds__(256) xent_bwd_kernel(const float* __restrict__ logits,
                                                      const int64_t* __restrict__ labels,
                                                      const float* __restrict__ lse, const float* __restrict__ gscale,
                                                      int N, int ncls, float* __restrict__ dl) {
  const int64_t total = (int64_t)N * ncls;
  const float g = xent_gain(gscale, N);
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / ncls), j = (int)(i % ncls);
    dl[i] = xent_grad(logits[i], lse[b], labels[b] == j, g);
  }
}

int xent_bwd(const float* logits, const int64_t* labels, const float* lse, const float* gscale, int N, int ncls,
             float* dlogits, hipStream_t st) {
  DTC_CHECK_ARG(logits && labels && lse && dlogits && N > 0 && ncls > 0, "xent_bwd: bad args");
  const int64_t total = (int64_t)N * ncls;
  const int blocks = (int)std::min<int64_t>(1024, (total + 255) / 256);
  DTC_KLAUNCH(xent_bwd_kernel, dim3(blocks), dim3(256), 0, st, logits, labels, lse, gscale, N, ncls, dlogits);
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
// dact of one image: dact[p][c] = (1/HW) sum_j dl[j] W[j][c], the same value at every pixel p (the
// pool's backward). Wave w sums classes j = w, w + 4, ... for 8 consecutive channels per lane (16-B
// weight loads, eight rows in flight per lane); the four wave partials are added in LDS in a fixed
// order, and the pixel rows are stored as 16-B pieces. sm: ncls + 4 C floats. dln == nullptr: the caller
// already wrote the dlogits row into sm[0, ncls) (the barrier below orders it).
template <typename T>
__device__ __forceinline__ void head_dact_image(const float* __restrict__ dln, const T* __restrict__ wfc, int HW, int C,
                                                int ncls, T* __restrict__ o, float* sm) {
  typedef Elt<T> E;
  float* row = sm;
  float* red = sm + ncls;
  const int t = threadIdx.x, wv = t >> 6, l = t & 63, nch = C >> 3;
  constexpr bool BF = std::is_same<T, u16>::value;
  if constexpr (BF) {
    if (C == 512 && ncls <= 128) {  // all of this lane's weight rows (<= 32 x 16 B) in flight before any use
      typename E::V w8[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int j = wv + 4 * u;
        w8[u] = E::ld(wfc + (int64_t)(j < ncls ? j : 0) * C + l * 8);
      }
      if (dln)
        for (int j = t; j < ncls; j += 256) row[j] = dln[j];
      __syncthreads();
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 32; ++u) {  // classes wv, wv + 4, ...: the generic loop's order
        if (wv + 4 * u >= ncls) break;
        float f[8];
        E::unpack(w8[u], f);
        const float d = row[wv + 4 * u];
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += d * f[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) red[wv * C + l * 8 + k] = s[k];
      goto combine;
    }
  }
  if (dln)
    for (int j = t; j < ncls; j += 256) row[j] = dln[j];
  __syncthreads();
  for (int c8 = l; c8 < nch; c8 += 64) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const T* wc = wfc + c8 * 8;
    for (int j = wv; j < ncls; j += 32) {
      typename E::V w8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (j + 4 * u < ncls) w8[u] = E::ld(wc + (int64_t)(j + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j + 4 * u >= ncls) break;
        float f[8];
        E::unpack(w8[u], f);
        const float d = row[j + 4 * u];
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += d * f[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wv * C + c8 * 8 + k] = s[k];
  }
combine:
  __syncthreads();
  const float inv = 1.f / (float)HW;
  for (int idx = t; idx < HW * nch; idx += 256) {
    const int p = idx / nch, c8 = idx - p * nch;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 * 8 + k;
      v[k] = (((red[c] + red[C + c]) + red[2 * C + c]) + red[3 * C + c]) * inv;
    }
    E::st(o + (int64_t)p * C + c8 * 8, E::pack(v));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) head_bwd_x_kernel(const float* __restrict__ dl, const T* __restrict__ wfc,
                                                        int HW, int C, int ncls, T* __restrict__ dact) {
  extern __shared__ float hsx[];
  const int n = blockIdx.x;
  head_dact_image<T>(dl + (int64_t)n * ncls, wfc, HW, C, ncls, dact + (int64_t)n * HW * C, hsx);
}

// One launch for the whole head backward (the first kernels after the per-step barrier, when the GPU
// queue is empty, so every launch boundary here is exposed): workgroups [0, nw) compute dW / db, one
// (class, 256-channel) strip each, the four waves summing every fourth image (dl[n][j] is uniform, feat
// rows coalesced); workgroups [nw, nw + N) compute dact of one image each (head_bwd_x's work).
// XE: the CrossEntropyLoss backward fused in (xa.logits != nullptr): every dlogits value is computed where
// it is used, by xent_grad as xent_bwd computes it, and the dact workgroups also store their image's row
// into dl (the executor's dlogits buffer) -- one launch fewer right after the per-step barrier.
template <typename T, bool XE>
__global__ void __launch_bounds__(256) head_bwd_fused_kernel(float* __restrict__ dl,
                                                            const float* __restrict__ feat,
                                                            const T* __restrict__ wfc, int N, int HW, int C, int ncls,
                                                            float scale, float* __restrict__ dw,
                                                            float* __restrict__ db, T* __restrict__ dact, int nw,
                                                            XentArgs xa) {
  extern __shared__ float hsx[];
  const int t = threadIdx.x;
  // (a template parameter, not a runtime test: a branch inside the image loop below kept the compiler
  // from batching its loads -- 26.6 vs 10.9 us per launch at batch 256)
  constexpr bool xe = XE;
  const float xg = xe ? xent_gain(xa.gscale, N) : 0.f;
  if ((int)blockIdx.x < nw) {
    // dW[j][c..c+3] (float4 of feat per lane) and db[j]: wave w sums the images n = w, w + 4, ... (eight
    // rows in flight per lane), the four wave partials are added in LDS in a fixed order
    const int strips = (C + 255) / 256;
    const int j = blockIdx.x / strips, cb = (blockIdx.x - j * strips) * 256;
    const int wv = t >> 6, l = t & 63, c = cb + l * 4;
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b = 0.f;
    if constexpr (XE) {
      // dlogits column j for 256 images at a time into LDS (one image per thread: the gather of logits,
      // lse and labels is spread over the workgroup instead of serialised in each wave's image loop),
      // then the same per-wave image order n = wv, wv + 4, ... as below
      float* dcol = hsx + 4 * 260;
      for (int n0 = 0; n0 < N; n0 += 256) {
        const int nn = min(256, N - n0);
        if (t < nn) dcol[t] = xent_grad(xa.logits[(int64_t)(n0 + t) * ncls + j], xa.lse[n0 + t], xa.labels[n0 + t] == j, xg);
        __syncthreads();
        if (c < C) {
#pragma unroll 8
          for (int i = wv; i < nn; i += 4) {
            const float d = dcol[i];
            const f32x4 f = *(const f32x4*)(feat + (int64_t)(n0 + i) * C + c);
#pragma unroll
            for (int k = 0; k < 4; ++k) a[k] += d * f[k];
            b += d;
          }
        }
        __syncthreads();
      }
    } else if (c < C) {
#pragma unroll 8
      for (int n = wv; n < N; n += 4) {
        const float d = dl[(int64_t)n * ncls + j];
        const f32x4 f = *(const f32x4*)(feat + (int64_t)n * C + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += d * f[k];
        b += d;
      }
    }
    float* red = hsx;  // [4 waves][260]
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wv * 260 + l * 4 + k] = a[k];
    if (l == 0) red[wv * 260 + 256] = b;
    __syncthreads();
    if (wv == 0 && c < C) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = l * 4 + k;
        dw[(int64_t)j * C + c + k] = (((red[i] + red[260 + i]) + red[520 + i]) + red[780 + i]) * scale;
      }
    }
    if (t == 0 && cb == 0) db[j] = (((red[256] + red[516]) + red[776]) + red[1036]) * scale;
    return;
  }
  const int n = blockIdx.x - nw;
  if constexpr (XE) {
    const float ls = xa.lse[n];
    const int64_t lab = xa.labels[n];
    for (int j = t; j < ncls; j += 256) {
      const float d = xent_grad(xa.logits[(int64_t)n * ncls + j], ls, lab == j, xg);
      hsx[j] = d;
      dl[(int64_t)n * ncls + j] = d;
    }
  }
  head_dact_image<T>(xe ? nullptr : dl + (int64_t)n * ncls, wfc, HW, C, ncls, dact + (int64_t)n * HW * C, hsx);
}

template <typename T>
static int head_bwd_t(const float* dlogits, const float* feat, const T* wfc, int N, int HW, int C, int ncls,
                      float scale, float* dw, float* db, T* dact, float* ws, size_t ws_bytes, hipStream_t st,
                      const XentArgs* xa) {
  DTC_CHECK_ARG(dlogits && feat && wfc && dw && db && dact && N > 0 && HW > 0 && C > 0 && C % 8 == 0 && C <= 2048 &&
                    ncls > 0 && ncls <= 4096 && (!xa || (xa->logits && xa->labels && xa->lse)),
                "head_bwd: bad args");
  // head_dact_image / fused dW (+ the fused-xent dlogits column)
  const size_t dx_lds = (size_t)std::max(ncls + 4 * C, 4 * 260 + 256) * sizeof(float);
  // option head_fused: 1 (default) always, 2 at most 64 images. With the dW strips summed by four waves the one
  // launch is faster at batch 256 too (+0.45%, 4-round A/B r04m; the round-3 sequential strip loop was 1% slower)
  const int hf = option_get(OPT_HEAD_FUSED);
  if (ncls <= 1024 && (hf == 1 || (hf == 2 && N <= 64))) {
    const int nw = ncls * ((C + 255) / 256);
    if (xa)
      DTC_KLAUNCH((head_bwd_fused_kernel<T, true>), dim3(nw + N), dim3(256), dx_lds, st, (float*)dlogits, feat,
                         wfc, N, HW, C, ncls, scale, dw, db, dact, nw, *xa);
    else
      DTC_KLAUNCH((head_bwd_fused_kernel<T, false>), dim3(nw + N), dim3(256), dx_lds, st, (float*)dlogits, feat,
                         wfc, N, HW, C, ncls, scale, dw, db, dact, nw, XentArgs());
    DTC_LAUNCH_CHECK();
    return 0;
  }
  if (xa) DTC_TRY(xent_bwd(xa->logits, xa->labels, xa->lse, xa->gscale, N, ncls, (float*)dlogits, st));
  DTC_CHECK_ARG(ws && ws_bytes >= head_bwd_workspace(N, C, ncls), "head_bwd: workspace too small");
  const int splits = (N + HB_IMGS - 1) / HB_IMGS;
  DTC_KLAUNCH(head_bwd_w_partial_kernel, dim3((C + 63) / 64, (ncls + 15) / 16, splits), dim3(256), 0, st,
                     dlogits, feat, N, C, ncls, ws);
  DTC_LAUNCH_CHECK();
  DTC_KLAUNCH(head_bwd_w_reduce_kernel, dim3((int)(((int64_t)ncls * C + 255) / 256)), dim3(256), 0, st, ws,
                     splits, dlogits, N, C, ncls, scale, dw, db);
  DTC_LAUNCH_CHECK();
  DTC_KLAUNCH(head_bwd_x_kernel<T>, dim3(N), dim3(256), dx_lds, st, dlogits, wfc, HW, C, ncls, dact);
  DTC_LAUNCH_CHECK();
  return 0;
}
int head_bwd(const float* dlogits, const float* feat, const u16* wfc, int N, int HW, int C, int ncls, float scale,
             float* dw, float* db, u16* dact, float* ws, size_t ws_bytes, hipStream_t st, const XentArgs* xa) {
  return head_bwd_t<u16>(dlogits, feat, wfc, N, HW, C, ncls, scale, dw, db, dact, ws, ws_bytes, st, xa);
}
int head_bwd(const float* dlogits, const float* feat, const float* wfc, int N, int HW, int C, int ncls, float scale,
             float* dw, float* db, float* dact, float* ws, size_t ws_bytes, hipStream_t st, const XentArgs* xa) {
  return head_bwd_t<float>(dlogits, feat, wfc, N, HW, C, ncls, scale, dw, db, dact, ws, ws_bytes, st, xa);
}

}  // namespace dtc
