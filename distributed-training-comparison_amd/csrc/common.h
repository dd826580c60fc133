// Shared device/host helpers for the MI355X (gfx950) ResNet-18 data-parallel step.
//
// Conventions used by every kernel in this library:
//   * activations are NHWC bf16 (raw 16-bit words, `u16`), channels innermost;
//   * master parameters / gradients are fp32 in one flat buffer (see resnet.cpp);
//   * conv weights are K x R x S x C ("KRSC"), so one output channel's filter is a
//     contiguous row of R*S*C elements: that row is the GEMM operand directly;
//   * every launch takes the caller's hipStream_t; nothing here allocates memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

typedef uint16_t u16;
typedef unsigned long long u64;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------- errors
namespace dtc {
int set_error(int code, const char* fmt, ...);
const char* last_error();
}  // namespace dtc

#define DTC_EINVAL (-1)
#define DTC_CHECK_ARG(cond, ...)                                   \
  do {                                                             \
    if (!(cond)) return ::dtc::set_error(DTC_EINVAL, __VA_ARGS__); \
  } while (0)
#define DTC_HIP(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::dtc::set_error((int)e_, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                              __FILE__, __LINE__);                                           \
  } while (0)
#define DTC_LAUNCH_CHECK() DTC_HIP(hipGetLastError())

// ---------------------------------------------------------------- launches
// Every kernel of the library is launched through DTC_KLAUNCH, which notes a launch on the stream a side stream
// was last forked from (resnet.cpp: a second fork from the same point -- a bucket's collective right after its
// weight-gradient flush -- then needs no second event record; a record costs the recording stream a ~2.7 us
// bubble before its next kernel, tools/probes/fork_gap.hip).
namespace dtc {
struct ForkWatch {
  hipStream_t st = nullptr;
  bool dirty = true;  // something was launched on st since the fork
};
inline thread_local ForkWatch g_fork_watch;
inline void note_launch(hipStream_t st) {
  if (st == g_fork_watch.st) g_fork_watch.dirty = true;
}
}  // namespace dtc
#define DTC_KLAUNCH(K, G, B, SH, ST, ...)          \
  do {                                            \
    ::dtc::note_launch(ST);                       \
    hipLaunchKernelGGL(K, G, B, SH, ST, __VA_ARGS__); \
  } while (0)
#define DTC_TRY(expr)      \
  do {                     \
    int r_ = (expr);       \
    if (r_ != 0) return r_; \
  } while (0)

// ---------------------------------------------------------------- bf16 <-> f32
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
// Round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950; keeps NaN a NaN).
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
// two values in one v_cvt_pk_bf16_f32 (the same round-to-nearest-even per value as f2bf)
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// unpack 8 bf16 held in a uint4 into floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
  f[4] = bf_lo(v.z); f[5] = bf_hi(v.z); f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]); v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]); v.w = pack_bf2(f[6], f[7]);
  return v;
}

// ---------------------------------------------------------------- activation element traits
// The executor runs activations either as bf16 (AMP: autocast rounding points) or as fp32 (the
// reference without --amp, ddp/trainer.py:160-165). Elementwise kernels are written once over
// 8-element vectors: V = the raw 8-element register image (16 B of bf16 or 32 B of fp32),
// round() = the autocast rounding of an intermediate (identity in fp32 mode).
template <typename T>
struct Elt;
template <>
struct Elt<u16> {
  typedef uint4 V;
  static __device__ __forceinline__ V ld(const u16* p) { return *(const uint4*)p; }
  static __device__ __forceinline__ void st(u16* p, const V& v) { *(uint4*)p = v; }
  static __device__ __forceinline__ void unpack(const V& v, float* f) { unpack8(v, f); }
  static __device__ __forceinline__ V pack(const float* f) { return pack8(f); }
  static __device__ __forceinline__ float round(float x) { return round_bf(x); }
  static __device__ __forceinline__ float cvt(u16 v) { return bf2f(v); }
  static __device__ __forceinline__ u16 from(float f) { return f2bf(f); }
  // ReLU mask of 8 packed outputs (>= 0 after the ReLU): bit k = element k > 0
  static __device__ __forceinline__ uint32_t mask8(const V& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) b |= (((w[k] & 0x7fffu) != 0u) ? 1u : 0u) << (2 * k) | (((w[k] & 0x7fff0000u) != 0u) ? 2u : 0u) << (2 * k);
    return b;
  }
};
struct F32x8 {
  f32x4 a, b;
};
template <>
struct Elt<float> {
  typedef F32x8 V;
  static __device__ __forceinline__ V ld(const float* p) { return V{*(const f32x4*)p, *(const f32x4*)(p + 4)}; }
  static __device__ __forceinline__ void st(float* p, const V& v) {
    *(f32x4*)p = v.a;
    *(f32x4*)(p + 4) = v.b;
  }
  static __device__ __forceinline__ void unpack(const V& v, float* f) {
    f[0] = v.a[0]; f[1] = v.a[1]; f[2] = v.a[2]; f[3] = v.a[3];
    f[4] = v.b[0]; f[5] = v.b[1]; f[6] = v.b[2]; f[7] = v.b[3];
  }
  static __device__ __forceinline__ V pack(const float* f) {
    return V{f32x4{f[0], f[1], f[2], f[3]}, f32x4{f[4], f[5], f[6], f[7]}};
  }
  static __device__ __forceinline__ float round(float x) { return x; }
  static __device__ __forceinline__ float cvt(float v) { return v; }
  static __device__ __forceinline__ float from(float f) { return f; }
  static __device__ __forceinline__ uint32_t mask8(const V& v) {
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) b |= (v.a[k] > 0.f ? 1u : 0u) << k | (v.b[k] > 0.f ? 1u : 0u) << (k + 4);
    return b;
  }
};

// ---------------------------------------------------------------- fast unsigned division
// q = (umulhi(n, m) + n) >> s, exact for n < 2^31 (pixel indices here are < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) { f.d = 1; f.m = 0; f.s = 0; return f; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  f.s = l;
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// ---------------------------------------------------------------- wave reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sum over the 16 lanes of a DPP row (e.g. the 16 pixel columns of an MFMA 16x16 output
// fragment); every lane of the row receives the sum. Four VALU adds with DPP operands.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false)));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- BN statistic accumulators
// A BN's batch sums (sum x, sum x^2 in the forward; sum dz, sum dz * xhat in the backward) are built from
// one fp32 partial per producing workgroup and channel. They are accumulated EXACTLY, in integer fixed
// point: a partial v is split into hi = floor(v * 2^8) and lo = floor(frac(v * 2^8) * 2^44) and both are
// added with int64 atomics into one of DTC_STAT_SLOTS slots (blockIdx.x mod slots: spreads the atomic
// contention). Integer addition is associative, so the totals -- and every BN coefficient computed from
// them -- do not depend on the order in which the workgroups' adds arrive: the training step is
// bit-reproducible run to run, as the reference's cudnn.deterministic = True asks (src/ddp/utils.py:12-13).
// (Rounds 1-5 added fp64 partials with fp64 atomics: a sum that rounds depends on the arrival order.)
// Bits of v below 2^-52 are dropped (deterministically; fp64 atomics kept 53 bits of the running total). A
// partial that is not finite or not below 2^40 in magnitude is not added: it sets the header's flag word,
// and every consumer then produces NaN coefficients (the AMP GradScaler skips such a step, as an fp16
// overflow makes the reference's GradScaler skip it). Range: totals below 2^55, at most 2^15 partials per
// slot and channel (2^18 per BN) -- batch 512 at 224x224 makes ~2^17.
// Layout per BN, int64 words: [DTC_STAT_HDR header, word 0 = flag][DTC_STAT_SLOTS][2 stats][2 words: hi, lo][C]
#ifndef DTC_STAT_SLOTS  // (overridable at build time for A/B builds)
#define DTC_STAT_SLOTS 8  // 16: +4.5% BN family time (the apply kernels' slot-fold loads), 32: +12%; 4: the same
#endif                     // BN time, conv epilogues slower (atomic contention) -- round 6, profiles/r06c_lab_slots.txt
#ifndef DTC_STAT_HDR
#define DTC_STAT_HDR 16  // one 128-B line: keeps every (slot, statistic, word) row line-aligned
#endif
#define DTC_STAT_WORDS(C) ((size_t)DTC_STAT_HDR + (size_t)DTC_STAT_SLOTS * 4 * (size_t)(C))

// word (slot k, statistic j, part w) of channel 0
__host__ __device__ __forceinline__ size_t stat_word(int k, int j, int w, int C) {
  return (size_t)DTC_STAT_HDR + ((size_t)k * 4 + j * 2 + w) * (size_t)C;
}

__device__ __forceinline__ void stat_add1(int64_t* __restrict__ base, size_t o, int C, float v) {
  const double d = (double)v * 256.0;
  if (fabs(d) < 0x1p48) {  // false for NaN / inf too
    const double h = floor(d);
    __hip_atomic_fetch_add(base + o, (int64_t)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(base + o + C, (int64_t)((d - h) * 0x1p44), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_fetch_or(base, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// this workgroup's partials (s, q) of channel c into slot blockIdx.x mod DTC_STAT_SLOTS
__device__ __forceinline__ void stat_add(int64_t* __restrict__ base, int C, int c, float s, float q) {
  const int k = blockIdx.x & (DTC_STAT_SLOTS - 1);
  stat_add1(base, stat_word(k, 0, 0, C) + c, C, s);
  stat_add1(base, stat_word(k, 1, 0, C) + c, C, q);
}

// total of one statistic from its summed hi / lo words (exact int64 sums over the slots) and the flag
__host__ __device__ __forceinline__ double stat_total(int64_t hi, int64_t lo, int64_t flag) {
  if (flag != 0) return __builtin_nan("");
  return (double)(hi + (lo >> 44)) * 0x1p-8 + (double)(lo & ((1ll << 44) - 1)) * 0x1p-52;
}
// conv call-timing slot (u64): start cell l at [DTC_PROF_LINE * l], end cell l at
// [DTC_PROF_LINE * (DTC_PROF_LINES + l)], l < DTC_PROF_LINES (one 128-B line per cell)
#define DTC_PROF_LINE 16
#define DTC_PROF_LINES 64
#define DTC_PROF_SLOT_U64 (DTC_PROF_LINE * DTC_PROF_LINES * 2)

