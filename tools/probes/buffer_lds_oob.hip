// Probe: does an out-of-range buffer_load ... lds (raw buffer, stride 0) write zeros into LDS
// or leave LDS untouched? Prints "zero-fill" or "skip" per lane class.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* g, unsigned nbytes, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 0xDEADBEEFu;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, 0, nbytes, 0x00020000);
  // lanes 0..31 in range, lanes 32..63 out of range (offset 0x80000000)
  unsigned voff = threadIdx.x < 32 ? threadIdx.x * 16 : 0x80000000u;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
int main() {
  unsigned *g, *o, h[256];
  hipMalloc(&g, 4096); hipMalloc(&o, 1024);
  unsigned init[1024]; for (int i = 0; i < 1024; ++i) init[i] = 0x11110000u + i;
  hipMemcpy(g, init, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, 512, o);
  hipMemcpy(h, o, 1024, hipMemcpyDeviceToHost);
  printf("in-range lane0 dw0=%08x (expect 11110000)\n", h[0]);
  printf("out-of-range lane32 dw0=%08x -> %s\n", h[128], h[128] == 0 ? "zero-fill" : (h[128] == 0xDEADBEEFu ? "skip" : "other"));
  printf("lane63 dw3=%08x\n", h[255]);
  return 0;
}
