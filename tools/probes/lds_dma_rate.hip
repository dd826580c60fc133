// Probe: what one halo refill costs a wave (round 6, conv_c64 stamps: ~1900 cycles per tile for 11 LDS-DMA pieces
// of 1 KiB per wave). Every CU runs one 4-wave workgroup (as conv_c64); each wave moves NP pieces of 1 KiB per round
// into LDS, ROUNDS rounds, and stamps s_memtime (shader clock) around the issue and around the completion:
//   mode 0  buffer_load_dwordx4 ... lds, M0 set per piece (conv_c64's buf_lds16)
//   mode 1  global_load_dwordx4 into VGPRs, then ds_write_b128 after the wait
//   mode 2  global_load_dwordx4 into VGPRs only (the fetch alone)
// Source: "l2" = every workgroup reads the same 64 KiB (L2-resident), "hbm" = each (workgroup, round) its own
// 44 KiB of a 2 GiB buffer. Prints per-round medians over waves: issue cycles, issue-to-landed cycles.
// Build: hipcc --offload-arch=gfx950 -O3 lds_dma_rate.hip -o lds_dma_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

typedef unsigned long long u64;
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int NP = 11, ROUNDS = 16, PIECE = 1024;

__device__ __forceinline__ u64 stamp() {
  u64 t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

__device__ __forceinline__ void lds_dma(const __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(r), "s"(lds_dst)
      : "memory");
}

template <int MODE>
__global__ void __launch_bounds__(256, 1) probe(const char* src, uint32_t src_bytes, int hbm, u64* out) {
  __shared__ __attribute__((aligned(1024))) char lds[4 * NP * PIECE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  u64 issue = 0, done = 0;
  for (int r = 0; r < ROUNDS; ++r) {
    const size_t region = hbm ? ((size_t)blockIdx.x * ROUNDS + r) * (4 * NP * PIECE) : 0;
    const char* base = src + region;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 4 * NP * PIECE, 0x00020000);
    __builtin_amdgcn_s_barrier();
    const u64 t0 = stamp();
    i32x4 v[NP];
    if constexpr (MODE == 0) {
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int g = wave + 4 * q;
        lds_dma(rs, g * PIECE + lane * 16, __builtin_amdgcn_readfirstlane(lds_base + g * PIECE));
      }
    } else {
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int g = wave + 4 * q;
        v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, g * PIECE + lane * 16, 0, 0);
      }
    }
    const u64 t1 = stamp();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (MODE == 1) {
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int g = wave + 4 * q;
        *(__attribute__((address_space(3))) i32x4*)(size_t)(lds_base + g * PIECE + lane * 16) = v[q];
      }
    }
    if constexpr (MODE == 2) {  // keep the loads alive
      int s = 0;
#pragma unroll
      for (int q = 0; q < NP; ++q) s += v[q].x ^ v[q].w;
      if (s == 0x7fffffff) lds[lane] = 1;
    }
    const u64 t2 = stamp();
    if (r >= 2) {
      issue += t1 - t0;
      done += t2 - t0;
    }
  }
  if (lane == 0) {
    out[(blockIdx.x * 4 + wave) * 2 + 0] = issue / (ROUNDS - 2);
    out[(blockIdx.x * 4 + wave) * 2 + 1] = done / (ROUNDS - 2);
  }
  if (lds[threadIdx.x * 7 % sizeof(lds)] == 123 && lane == 999) out[0] = 0;  // LDS contents observable
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int nwg = ncu;
  const size_t bytes = (size_t)nwg * ROUNDS * 4 * NP * PIECE;
  char* src;
  u64* out;
  CK(hipMalloc(&src, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipMalloc(&out, nwg * 4 * 2 * sizeof(u64)));
  std::vector<u64> h(nwg * 4 * 2);
  const char* mn[3] = {"LDS-DMA (buffer_load ... lds)", "global_load_b128 + ds_write_b128", "global_load_b128 only"};
  for (int hbm = 0; hbm < 2; ++hbm)
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(nwg), dim3(256), 0, 0, src, (uint32_t)bytes, hbm, out);
        if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(nwg), dim3(256), 0, 0, src, (uint32_t)bytes, hbm, out);
        if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(nwg), dim3(256), 0, 0, src, (uint32_t)bytes, hbm, out);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(h.data(), out, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
      std::vector<u64> is, dn;
      for (int i = 0; i < nwg * 4; ++i) {
        is.push_back(h[2 * i]);
        dn.push_back(h[2 * i + 1]);
      }
      std::sort(is.begin(), is.end());
      std::sort(dn.begin(), dn.end());
      printf("%-4s %-34s %d pieces x 1 KiB per wave, %d waves: issue %6llu cyc (p90 %6llu)  landed %6llu cyc (p90 %6llu)"
             "  -> %.1f B/clk/CU\n",
             hbm ? "hbm" : "l2", mn[mode], NP, nwg * 4, is[is.size() / 2], is[is.size() * 9 / 10], dn[dn.size() / 2],
             dn[dn.size() * 9 / 10], 4.0 * NP * PIECE / (double)dn[dn.size() / 2]);
    }
  return 0;
}
