// On-device CIFAR input pipeline: one launch per batch does what the reference's DataLoader
// workers do per sample on the host (src/ddp/dataset.py:43-64, 95-98, 100-108):
//   Subset/DistributedSampler gather (index -> stored image, target)
//   transforms.RandomCrop(32, padding=4)   zero padding, crop at (i, j) in [0, 2*pad]
//   transforms.RandomHorizontalFlip()      applied after the crop
//   transforms.ToTensor()                  uint8 HWC -> float CHW, x / 255
//   transforms.Normalize(mean, std)        (x - mean[c]) / std[c]
// The valid/test transforms (dataset.py:49-54, 139-149) are the same launch with i = j = pad and
// no flip. Arithmetic follows the CPU transforms operation by operation (true division by 255,
// subtract, true division by std, all fp32), so the result is bit-identical to them.
//
// Layout: the dataset lives in HBM as uint8 [n_images][h][w][3] (CIFAR's own storage order,
// 3 KB per 32x32 image); the batch is written as fp32 NCHW [n][3][h][w], the model's input.
// One 256-thread workgroup per up to 4 output images: the source images are staged in LDS with
// coalesced dword loads (one HBM read per image), the normalize table (256 byte values x 3
// channels) is built once per workgroup, then every thread writes float4 runs along w.
// HBM-bound: h*w*3 B read + h*w*3*4 B written (+8 B index, +8 B label) per image.
#include "common.h"
#include "kernels.h"

namespace dtc {

constexpr int AUG_MAX_BYTES = 12 * 1024;  // staged source images (imgs*h*w*3 bytes) per workgroup
constexpr int AUG_IMGS = 4;                // images per workgroup (amortises the normalize table)

// normalize(u, c) depends only on the byte value and the channel: the workgroup tabulates it once
// (768 entries, the same fp32 operations as the transform), so the pixel loop is LDS lookups.
__global__ void __launch_bounds__(256) cifar_augment_kernel(
    const uint8_t* __restrict__ images, const int64_t* __restrict__ targets, int64_t n_images,
    const int64_t* __restrict__ index, const uint8_t* __restrict__ crop, const uint8_t* __restrict__ flip, int n,
    int h, int w, int pad, int imgs, float m0, float m1, float m2, float s0, float s1, float s2,
    float* __restrict__ out, int64_t* __restrict__ labels, int* __restrict__ status) {
  __shared__ uint32_t img[AUG_MAX_BYTES / 4];
  __shared__ float lut[3 * 256];
  const int tid = threadIdx.x;
  {
    const float t = (float)tid / 255.0f;
    lut[tid] = (t - m0) / s0;
    lut[256 + tid] = (t - m1) / s1;
    lut[512 + tid] = (t - m2) / s2;
  }
  const int hw = h * w;
  const int ndw = hw * 3 / 4;
  const int b0 = blockIdx.x * imgs;
  const int nb = min(imgs, n - b0);
  for (int q = 0; q < nb; ++q) {
    const int b = b0 + q;
    const int64_t src = index ? index[b] : (int64_t)b;
    const bool valid = src >= 0 && src < n_images;
    if (tid == 0) {
      if (labels) labels[b] = valid ? targets[src] : 0;
      const int ci = crop ? crop[2 * b] : pad, cj = crop ? crop[2 * b + 1] : pad;
      if (status && (!valid || ci > 2 * pad || cj > 2 * pad)) *status = 1;
    }
    const uint32_t* s = (const uint32_t*)(images + (valid ? src : 0) * (int64_t)hw * 3);
    uint32_t* d = img + q * ndw;
    for (int i = tid; i < ndw; i += 256) d[i] = valid ? s[i] : 0u;
  }
  __syncthreads();
  const int w4 = w >> 2;
  const int per_c = h * w4;
  const int per_img = 3 * per_c;
  for (int g = tid; g < nb * per_img; g += 256) {
    const int q = g / per_img;
    const int r0 = g - q * per_img;
    const int b = b0 + q;
    const int ci = crop ? crop[2 * b] : pad;
    const int cj = crop ? crop[2 * b + 1] : pad;
    const bool fl = flip ? flip[b] != 0 : false;
    const uint8_t* px = (const uint8_t*)(img + q * ndw);
    const int c = r0 / per_c;
    const int rem = r0 - c * per_c;
    const int oh = rem / w4;
    const int ow0 = (rem - oh * w4) * 4;
    const float* tab = lut + c * 256;
    const int y = ci + oh - pad;
    const bool yin = y >= 0 && y < h;
    f32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ow = ow0 + k;
      const int x = cj + (fl ? (w - 1 - ow) : ow) - pad;
      const unsigned u = (yin && x >= 0 && x < w) ? px[(y * w + x) * 3 + c] : 0u;
      v[k] = tab[u];
    }
    *(f32x4*)(out + (int64_t)b * 3 * hw + (int64_t)c * hw + oh * w + ow0) = v;
  }
}

int cifar_augment(const uint8_t* images, const int64_t* targets, int64_t n_images, const int64_t* index,
                  const uint8_t* crop, const uint8_t* flip, int n, int h, int w, int pad, const float* mean,
                  const float* stdv, float* out, int64_t* labels, int* status, hipStream_t st) {
  DTC_CHECK_ARG(images && out && mean && stdv && n > 0 && h > 0 && w > 0 && pad >= 0 && n_images > 0,
                "cifar_augment: bad args");
  DTC_CHECK_ARG(w % 4 == 0 && (int64_t)h * w * 3 <= AUG_MAX_BYTES,
                "cifar_augment: bad shape h=%d w=%d (w %% 4 == 0, h*w*3 <= %d)", h, w, AUG_MAX_BYTES);
  DTC_CHECK_ARG(!labels || targets, "cifar_augment: labels requested without targets");
  DTC_CHECK_ARG(stdv[0] != 0.f && stdv[1] != 0.f && stdv[2] != 0.f, "cifar_augment: zero std");
  const int imgs = (int)std::max<int64_t>(1, std::min<int64_t>(AUG_IMGS, AUG_MAX_BYTES / ((int64_t)h * w * 3)));
  DTC_KLAUNCH(cifar_augment_kernel, dim3((n + imgs - 1) / imgs), dim3(256), 0, st, images, targets, n_images,
                     index, crop, flip, n, h, w, pad, imgs, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2], out,
                     labels, status);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
