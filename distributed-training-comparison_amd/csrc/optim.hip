// Fused flat-bucket SGD (Nesterov momentum) and the GradScaler device-side kernels.
//
// Replaces `optim.SGD(params, lr, weight_decay, momentum=0.9, nesterov=True).step()`
// (reference src/ddp/trainer.py:92-98, 158/165) and the AMP helpers behind
// `GradScaler.step/update` (main.py:25, trainer.py:157-159). torch.optim.SGD, dampening 0:
//     d = g + wd*p ; buf = mu*buf + d   (first step: buf = d) ; d = d + mu*buf ; p -= lr*d
// The first-step special case needs no flag: buffers start at zero and mu*0 + d == d exactly.
// GradScaler semantics (torch._amp_update_scale_): a step whose gradients hold inf/NaN is
// skipped entirely; scale *= backoff on overflow, *= growth after `interval` clean steps.
// The step also refreshes the bf16 shadow of every parameter (the GEMM operand layout).
#include "common.h"
#include "kernels.h"

namespace dtc {

__global__ void __launch_bounds__(256) sgd_nesterov_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ m, u16* __restrict__ pb, int64_t n4,
                                                          float lr, float wd, float mu,
                                                          const float* __restrict__ inv_scale,
                                                          const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;  // GradScaler: skip the whole step
  const float is = inv_scale ? *inv_scale : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 pv = *(const f32x4*)(p + i * 4);
    const f32x4 gv = *(const f32x4*)(g + i * 4);
    f32x4 mv = *(const f32x4*)(m + i * 4);
    f32x4 d = gv * is + pv * wd;
    mv = mv * mu + d;
    d = d + mv * mu;
    pv = pv - d * lr;
    *(f32x4*)(p + i * 4) = pv;
    *(f32x4*)(m + i * 4) = mv;
    uint2 w;
    w.x = pack_bf2(pv[0], pv[1]);
    w.y = pack_bf2(pv[2], pv[3]);
    *(uint2*)(pb + i * 4) = w;
  }
}

int sgd_nesterov(float* p, const float* g, float* mom, u16* p_bf16, int64_t n, float lr, float wd, float mu,
                 const float* inv_scale, const int* found_inf, hipStream_t st) {
  DTC_CHECK_ARG(p && g && mom && p_bf16 && n > 0 && (n % 4) == 0, "sgd_nesterov: bad args (n=%lld)", (long long)n);
  const int64_t n4 = n / 4;
  const int blocks = (int)std::min<int64_t>(2048, (n4 + 255) / 256);
  DTC_KLAUNCH(sgd_nesterov_kernel, dim3(blocks), dim3(256), 0, st, p, g, mom, p_bf16, n4, lr, wd, mu, inv_scale,
                     found_inf);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ s, u16* __restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = f2bf(s[i]);
}

int cast_f32_bf16(const float* src, u16* dst, int64_t n, hipStream_t st) {
  DTC_CHECK_ARG(src && dst && n > 0, "cast_f32_bf16: bad args");
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  DTC_KLAUNCH(cast_f32_bf16_kernel, dim3(blocks), dim3(256), 0, st, src, dst, n);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void zero_kernel(uint2* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = uint2{0u, 0u};
}

// A kernel, not hipMemsetAsync: inside a captured graph a memset node is a separate (fill) dispatch
int zero_bytes(void* p, size_t bytes, hipStream_t st) {
  DTC_CHECK_ARG(p && bytes % 8 == 0 && ((uintptr_t)p & 7) == 0, "zero_bytes: 8-byte aligned ranges only");
  if (bytes == 0) return 0;
  const int64_t n = (int64_t)(bytes / 8);
  const int blocks = (int)std::min<int64_t>(1024, (n + 255) / 256);
  DTC_KLAUNCH(zero_kernel, dim3(blocks), dim3(256), 0, st, (uint2*)p, n);
  DTC_LAUNCH_CHECK();
  return 0;
}

// The executor's forward prologue: the caller's input copied into the executor's own buffer (the
// captured forward graph reads a fixed address) and the BN slots zeroed, in one launch.
__global__ void copy_zero_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16,
                                 uint2* __restrict__ z, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n8; i += stride) z[i] = uint2{0u, 0u};
}

int copy_and_zero(const void* src, void* dst, size_t bytes, void* zp, size_t zbytes, hipStream_t st) {
  DTC_CHECK_ARG(src && dst && zp && bytes % 16 == 0 && zbytes % 8 == 0 && ((uintptr_t)src & 15) == 0 &&
                    ((uintptr_t)dst & 15) == 0 && ((uintptr_t)zp & 7) == 0,
                "copy_and_zero: 16-byte aligned copy, 8-byte aligned zero range");
  const int64_t n16 = (int64_t)(bytes / 16), n8 = (int64_t)(zbytes / 8);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (std::max(n16, n8) + 255) / 256));
  DTC_KLAUNCH(copy_zero_kernel, dim3(blocks), dim3(256), 0, st, (const uint4*)src, (uint4*)dst, n16, (uint2*)zp,
                     n8);
  DTC_LAUNCH_CHECK();
  return 0;
}


template <typename T>
__global__ void scale_kernel(T* __restrict__ x, int64_t n, T f) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] *= f;
}

int scale_f32(float* x, int64_t n, float f, hipStream_t st) {
  DTC_CHECK_ARG(x && n > 0, "scale_f32: bad args");
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  DTC_KLAUNCH(scale_kernel<float>, dim3(blocks), dim3(256), 0, st, x, n, f);
  DTC_LAUNCH_CHECK();
  return 0;
}

int scale_f64(double* x, int64_t n, double f, hipStream_t st) {
  DTC_CHECK_ARG(x && n > 0, "scale_f64: bad args");
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  DTC_KLAUNCH(scale_kernel<double>, dim3(blocks), dim3(256), 0, st, x, n, f);
  DTC_LAUNCH_CHECK();
  return 0;
}

int scale_i64(int64_t* x, int64_t n, int64_t f, hipStream_t st) {
  DTC_CHECK_ARG(x && n > 0, "scale_i64: bad args");
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  DTC_KLAUNCH(scale_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, x, n, f);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void amp_scale_kernel(const float* __restrict__ x, const float* __restrict__ scale, float* __restrict__ out,
                                 int64_t n) {
  const float s = *scale;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = x[i] * s;
}

int amp_scale(const float* x, const float* scale, float* out, int64_t n, hipStream_t st) {
  DTC_CHECK_ARG(x && scale && out && n > 0, "amp_scale: bad args");
  const int blocks = (int)std::min<int64_t>(1024, (n + 255) / 256);
  DTC_KLAUNCH(amp_scale_kernel, dim3(blocks), dim3(256), 0, st, x, scale, out, n);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void add_f32_kernel(float* __restrict__ d, const float* __restrict__ s, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 a = ((f32x4*)d)[i];
    a += ((const f32x4*)s)[i];
    ((f32x4*)d)[i] = a;
  }
}

int add_f32(float* dst, const float* src, int64_t n, hipStream_t st) {
  DTC_CHECK_ARG(dst && src && n > 0 && n % 4 == 0 && ((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0,
                "add_f32: bad args (n %% 4 and 16-byte alignment required)");
  const int blocks = (int)std::min<int64_t>(2048, (n / 4 + 255) / 256);
  DTC_KLAUNCH(add_f32_kernel, dim3(blocks), dim3(256), 0, st, dst, src, n / 4);
  DTC_LAUNCH_CHECK();
  return 0;
}

// In-process thread-group communicator (comm.cpp): out_r[i] = sum_q in_q[i] for every rank r, the
// ranks' buffers summed in rank order (fixed; for two ranks the fp32 sum itself), read before written
// per element so the all-reduce is in place in every rank's buffer.
template <typename T>
__global__ void group_sum_kernel(GroupPtrs g, int w, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    T s = ((const T*)g.p[0])[i];
    for (int r = 1; r < w; ++r) s += ((const T*)g.p[r])[i];
    for (int r = 0; r < w; ++r) ((T*)g.p[r])[i] = s;
  }
}

int group_sum(const GroupPtrs& g, int w, int64_t n, int dtype, hipStream_t st) {
  DTC_CHECK_ARG(w >= 1 && w <= DTC_GROUP_MAX && n > 0 && (dtype == 0 || dtype == 2 || dtype == 3), "group_sum: bad args");
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  if (dtype == 0) DTC_KLAUNCH(group_sum_kernel<float>, dim3(blocks), dim3(256), 0, st, g, w, n);
  else if (dtype == 2) DTC_KLAUNCH(group_sum_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, g, w, n);
  else DTC_KLAUNCH(group_sum_kernel<double>, dim3(blocks), dim3(256), 0, st, g, w, n);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void amp_check_finite_kernel(const float* __restrict__ g, int64_t n, int* __restrict__ found) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) *found = 1;
}

// 16-B aligned gradients (the flat buffer): float4 loads, four in flight per thread per trip
__global__ void amp_check_finite4_kernel(const float* __restrict__ g, int64_t n, int* __restrict__ found) {
  const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * 256;
  const f32x4* __restrict__ g4 = (const f32x4*)g;
  bool bad = false;
  int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f32x4 a = g4[i], b = g4[i + stride], c = g4[i + 2 * stride], d = g4[i + 3 * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k)  // branch-free: the four tests OR-ed as integers
      bad |= (int)!isfinite(a[k]) | (int)!isfinite(b[k]) | (int)!isfinite(c[k]) | (int)!isfinite(d[k]);
  }
  for (; i < n4; i += stride) {
    const f32x4 a = g4[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) bad |= !isfinite(a[k]);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) bad |= !isfinite(g[(n4 << 2) + threadIdx.x]);
  if (__any(bad) && (threadIdx.x & 63) == 0) *found = 1;
}

int amp_check_finite(const float* g, int64_t n, int* found_inf, hipStream_t st) {
  DTC_CHECK_ARG(g && found_inf && n > 0, "amp_check_finite: bad args");
  if (((uintptr_t)g & 15) == 0) {
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n / 4 + 255) / 256));
    DTC_KLAUNCH(amp_check_finite4_kernel, dim3(blocks), dim3(256), 0, st, g, n, found_inf);
    DTC_LAUNCH_CHECK();
    return 0;
  }
  const int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  DTC_KLAUNCH(amp_check_finite_kernel, dim3(blocks), dim3(256), 0, st, g, n, found_inf);
  DTC_LAUNCH_CHECK();
  return 0;
}

__global__ void amp_update_scale_kernel(float* scale, float* inv_scale, int* tracker, int* found, float growth,
                                        float backoff, int interval) {
  float s = *scale;  // the three state words loaded together (one memory latency), then the update
  const int f = *found, tr = *tracker;
  if (f) {
    s *= backoff;
    *tracker = 0;
  } else {
    const int k = tr + 1;
    if (k >= interval) {
      const float ns = s * growth;
      if (isfinite(ns)) s = ns;
      *tracker = 0;
    } else {
      *tracker = k;
    }
  }
  *scale = s;
  if (inv_scale) *inv_scale = 1.f / s;
  *found = 0;
}

int amp_update_scale(float* scale, float* inv_scale, int* growth_tracker, int* found_inf, float growth, float backoff,
                     int interval, hipStream_t st) {
  DTC_CHECK_ARG(scale && growth_tracker && found_inf && interval > 0, "amp_update_scale: bad args");
  DTC_KLAUNCH(amp_update_scale_kernel, dim3(1), dim3(1), 0, st, scale, inv_scale, growth_tracker, found_inf,
                     growth, backoff, interval);
  DTC_LAUNCH_CHECK();
  return 0;
}

}  // namespace dtc
