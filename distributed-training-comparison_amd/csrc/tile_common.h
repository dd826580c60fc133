// Device helpers shared by the implicit-GEMM kernels (igemm.hip, wgrad_halo.hip): LDS-DMA
// loaders, the LDS swizzles, MFMA fragment readers and the call-timing stamps.
#pragma once
#include "common.h"

namespace dtc {

// LDS-DMA (16 B per lane, lane-linear LDS destination at a wave-uniform base) is issued through
// inline asm on purpose. With the builtins, hipcc treats the DMA as a pending write to LDS and
// emits `s_waitcnt vmcnt(0)` before the next ds_read of ANY LDS buffer, i.e. it drains the
// prefetch of step k+1 before the MFMAs of step k can read their operands (measured in the .s of
// every pipelined kernel here). hipcc neither counts nor waits for an asm DMA: completion is each
// kernel's own counted `s_waitcnt vmcnt(N)` followed by an s_barrier before the data is read.
// M0 (the DMA's LDS base) is compiler-reserved: saved and restored inside the same statement.
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// 16-byte LDS-DMA through a buffer descriptor over [base, base + bytes): an offset outside the
// range loads zeros.
__device__ __forceinline__ void buf_lds16(const void* base, uint32_t bytes, char* lds_dst, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_u32(lds_dst));
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(r), "s"(dst)
      : "memory");
}

// Call-timing stamps (kernel entry / exit only, one lane per workgroup; nothing on the loop).
// Slot layout (u64, one 128-B line per cell): DTC_PROF_LINES start cells, then DTC_PROF_LINES end
// cells. Dispatch order is not guaranteed, so the start is the min over the entries of the first
// DTC_PROF_LINES workgroups (the earliest dispatched among them in practice), each in its own
// line; the end is the max over all workgroups' exits, spread over the end lines. No contention.
__device__ __forceinline__ void stamp_start(u64* ts) {
  if (ts != nullptr && threadIdx.x == 0) {
    const unsigned lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (lin < DTC_PROF_LINES) atomicMin(ts + DTC_PROF_LINE * lin, (u64)__builtin_amdgcn_s_memrealtime());
  }
}
__device__ __forceinline__ void stamp_end(u64* ts) {
  if (ts != nullptr && threadIdx.x == 0) {
    const unsigned lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    atomicMax(ts + DTC_PROF_LINE * (DTC_PROF_LINES + (lin & (DTC_PROF_LINES - 1))),
              (u64)__builtin_amdgcn_s_memrealtime());
  }
}

// Phase probe (diagnostic builds only: `make phases` -> libdtc_amd_phases.so, -DDTC_PHASES): lane 0 of each
// workgroup writes s_memrealtime (100 MHz, chip-wide) at marked points of a kernel into buf[wg][8]
// (plain vector stores); tools/phase_probe.py reads them. In the product build the marks are empty.
#ifdef DTC_PHASES
constexpr unsigned DTC_PHASE_WGS = 16384;
__device__ __forceinline__ void phase_mark(u64* buf, int k) {
  // wave 0 only, as a wave-uniform branch (a lane-divergent one here would make the compiler treat the
  // buffer descriptors of the surrounding LDS-DMA asm as divergent); its 64 lanes store the same word
  if (buf != nullptr && __builtin_amdgcn_readfirstlane(threadIdx.x) == 0) {
    const unsigned lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (lin < DTC_PHASE_WGS) buf[lin * 8 + k] = (u64)__builtin_amdgcn_s_memrealtime();
  }
}
#else
__device__ __forceinline__ void phase_mark(u64*, int) {}
#endif

__device__ __forceinline__ int rowswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int trswz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

// 16-byte LDS-DMA from a per-lane global address (global_load_lds_dwordx4).
__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_u32(lds_wave_base));
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

// Row-image fragment: lane holds row (lane&15), reduction chunk (ks*4 + lane>>4).
__device__ __forceinline__ bf16x8 frag_row(const char* region, int row0, int ks, int lane) {
  const int row = row0 + (lane & 15);
  const int ch = (ks * 4 + (lane >> 4)) ^ rowswz(row);
  uint4 v = *(const uint4*)(region + row * 128 + (ch << 4));
  return __builtin_bit_cast(bf16x8, v);
}

// Tr-image fragment: lane holds column (cb + lane&15), reduction rows ks*32 + 8*(lane>>4) + 0..7.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 frag_tr(const char* region, int cb, int ks, int lane) {
  const int img = cb >> 6, cin = cb & 63;
  const int i = lane & 15, q = i >> 2, pp = i & 3, g = lane >> 4;
  const int unit = (cin >> 2) + pp;
  const char* base = region + img * 8192;
  const int kr0 = ks * 32 + g * 8 + q;
  const int kr1 = kr0 + 4;
  const int f0 = (((kr0 >> 1) & 1) << 2) | (((kr0 >> 3) & 1) << 3);
  const int f1 = (((kr1 >> 1) & 1) << 2) | (((kr1 >> 3) & 1) << 3);
  typedef __attribute__((address_space(3))) bf16x4_t lds_v4;
  bf16x4_t t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(base + kr0 * 128 + ((unit ^ f0) << 3)));
  bf16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(base + kr1 * 128 + ((unit ^ f1) << 3)));
  return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace dtc
