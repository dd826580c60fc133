// Probe: the main-stream bubble a side-stream fork costs (round 6). Two busy kernels K1, K2 on stream A with,
// between them, one of:
//   0  nothing
//   1  hipEventRecord(e, A) + hipStreamWaitEvent(B, e) + a busy kernel on B  (resnet.cpp fork_side today)
//   2  K1 launched with hipExtLaunchKernelGGL(..., stop event e) + hipStreamWaitEvent(B, e) + kernel on B
//   3  hipEventRecord(e, A) alone (no waiter)
//   4  K1 launched with a stop event, no waiter (the cost of the event on a kernel nobody waits for)
// Each kernel stamps its first workgroup's start and every workgroup's end (s_memrealtime, 100 MHz) into
// device memory with vector stores; the gap = K2 first start - K1 last end. Median over 40 repetitions.
// Build: hipcc --offload-arch=gfx950 -O2 fork_gap.hip -o fork_gap
#include <hip/hip_ext.h>
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

// out[0] = min start (via per-workgroup stores, reduced on the host), per workgroup: start, end
__global__ void busy(unsigned long long* out, int ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < (unsigned long long)ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t0;
    out[2 * blockIdx.x + 1] = t;
  }
}

int main() {
  const int nwg = 512, reps = 40, ticks = 3000;  // 30 us per workgroup: the host is ahead of K1's end
  unsigned long long *k1, *k2, *kb;
  CK(hipMalloc(&k1, nwg * 16));
  CK(hipMalloc(&k2, nwg * 16));
  CK(hipMalloc(&kb, 64 * 16));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  std::vector<unsigned long long> h1(2 * nwg), h2(2 * nwg), hb(2 * 64);
  const char* names[5] = {"nothing", "eventRecord+wait+side kernel", "ExtLaunch stop event+wait+side kernel",
                          "eventRecord only", "ExtLaunch stop event only"};
  for (int mode = 0; mode < 5; ++mode) {
    std::vector<double> gaps;
    int early = 0;  // side kernel started before K1 ended (the wait was not honoured)
    for (int r = 0; r < reps + 5; ++r) {
      if (mode == 2 || mode == 4) {
        hipExtLaunchKernelGGL(busy, dim3(nwg), dim3(64), 0, A, nullptr, ev, 0, k1, ticks);
      } else {
        hipLaunchKernelGGL(busy, dim3(nwg), dim3(64), 0, A, k1, ticks);
      }
      CK(hipGetLastError());
      if (mode == 1 || mode == 3) CK(hipEventRecord(ev, A));
      if (mode == 1 || mode == 2) {
        CK(hipStreamWaitEvent(B, ev, 0));
        hipLaunchKernelGGL(busy, dim3(64), dim3(64), 0, B, kb, ticks / 4);
      }
      hipLaunchKernelGGL(busy, dim3(nwg), dim3(64), 0, A, k2, ticks);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h1.data(), k1, nwg * 16, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), k2, nwg * 16, hipMemcpyDeviceToHost));
      unsigned long long e1 = 0, s2 = ~0ull;
      for (int i = 0; i < nwg; ++i) {
        e1 = std::max(e1, h1[2 * i + 1]);
        s2 = std::min(s2, h2[2 * i]);
      }
      if (r >= 5) gaps.push_back(((double)s2 - (double)e1) * 0.01);  // 100 MHz -> us
      if (mode == 1 || mode == 2) {
        CK(hipMemcpy(hb.data(), kb, 64 * 16, hipMemcpyDeviceToHost));
        unsigned long long sb = ~0ull;
        for (int i = 0; i < 64; ++i) sb = std::min(sb, hb[2 * i]);
        if (sb < e1) ++early;
      }
    }
    std::sort(gaps.begin(), gaps.end());
    printf("%-40s gap K1 end -> K2 start: median %6.2f us  p10 %6.2f  p90 %6.2f  side started before K1 end: %d\n",
           names[mode], gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10], early);
  }
  return 0;
}
