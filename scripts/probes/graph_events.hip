// Probe (diagnostic, not shipped): does a stream capture of the engine's launch pattern --
// hipEventRecord, hipExtLaunchKernelGGL with start / stop events, plain launches, D2H
// copies into pinned memory -- instantiate and replay, and do the events then time it?
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); } } while (0)
__global__ void k_spin(unsigned* p, int n) {
  unsigned v = threadIdx.x;
  for (int i = 0; i < n; ++i) v = v * 1664525u + 1013904223u;
  if (v == 7u) p[0] = v;
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(p + 1, 1u);
}
int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* d;
  CK(hipMalloc(&d, 4096));
  CK(hipMemset(d, 0, 4096));
  unsigned* h;
  CK(hipHostMalloc((void**)&h, 4096, 0));
  hipEvent_t ev[9];
  for (auto& x : ev) CK(hipEventCreate(&x));
  auto seq = [&](bool ext) {
    CK(hipEventRecord(ev[0], st));
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, st, d, 2000);
    if (ext) { hipExtLaunchKernelGGL(k_spin, dim3(1024), dim3(256), 0, st, ev[7], ev[8], 0, d, 20000); CK(hipGetLastError()); }
    else hipLaunchKernelGGL(k_spin, dim3(1024), dim3(256), 0, st, d, 20000);
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, st, d, 2000);
    CK(hipEventRecord(ev[5], st));
    CK(hipMemcpyAsync(h, d, 256, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(h + 64, d + 64, 256, hipMemcpyDeviceToHost, st));
  };
  for (int ext = 0; ext < 2; ++ext) {
    // eager
    for (int r = 0; r < 5; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      seq(ext);
      auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(st));
      auto t2 = std::chrono::steady_clock::now();
      float a = -1, b = -1;
      CK(hipEventElapsedTime(&a, ev[0], ev[5]));
      if (ext) CK(hipEventElapsedTime(&b, ev[7], ev[8]));
      printf("eager ext=%d: launch %.1f us, total %.1f us, ev0-5 %.1f us, ev7-8 %.1f us, count %u\n", ext,
             std::chrono::duration<double, std::micro>(t1 - t0).count(), std::chrono::duration<double, std::micro>(t2 - t0).count(),
             a * 1e3, b * 1e3, h[1]);
    }
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    seq(ext);
    CK(hipStreamEndCapture(st, &g));
    if (!g) { printf("capture ext=%d failed\n", ext); continue; }
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    printf("graph ext=%d: %zu nodes\n", ext, nn);
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    for (int r = 0; r < 6; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(x, st));
      auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(st));
      auto t2 = std::chrono::steady_clock::now();
      float a = -1, b = -1;
      CK(hipEventElapsedTime(&a, ev[0], ev[5]));
      if (ext) CK(hipEventElapsedTime(&b, ev[7], ev[8]));
      printf("graph ext=%d: launch %.1f us, total %.1f us, ev0-5 %.1f us, ev7-8 %.1f us, count %u\n", ext,
             std::chrono::duration<double, std::micro>(t1 - t0).count(), std::chrono::duration<double, std::micro>(t2 - t0).count(),
             a * 1e3, b * 1e3, h[1]);
    }
    // events recorded outside the graph around it
    for (int r = 0; r < 4; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipEventRecord(ev[1], st));
      CK(hipGraphLaunch(x, st));
      CK(hipEventRecord(ev[2], st));
      CK(hipStreamSynchronize(st));
      auto t2 = std::chrono::steady_clock::now();
      float a = -1;
      CK(hipEventElapsedTime(&a, ev[1], ev[2]));
      printf("graph+outer events ext=%d: total %.1f us, outer %.1f us\n", ext,
             std::chrono::duration<double, std::micro>(t2 - t0).count(), a * 1e3);
    }
    CK(hipGraphExecDestroy(x));
    CK(hipGraphDestroy(g));
  }
  printf("probe done\n");
  return 0;
}
