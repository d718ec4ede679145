// Prefetch-depth microbenchmark for the scan's structure on MI355X: persistent 256-thread
// workgroups, one 8 KiB wave-tile per wave per iteration (16 B per lane per 1 KiB row),
// staged into the wave's LDS region, then a synthetic processing phase of R dependent
// LDS-read + VALU rounds (the scan's per-tile work is a latency chain of this kind).  The
// next tile(s) are prefetched into registers: depth 1 (the scan today) or depth 2.  LDS
// padding sets the workgroups per CU.  Prints GB/s of the streamed bytes.
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_depth.hip -o mb_depth && ./mb_depth
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kTile = 8192;

template <int D, int R, int PADKB>
__global__ __launch_bounds__(256) void k(const uint4* __restrict__ in, uint32_t ntiles, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s_all[4][kTile + 64];
  __shared__ uint8_t s_pad[PADKB * 1024 + 4];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4* s = reinterpret_cast<uint4*>(s_all[wv]);
  const uint32_t nwaves = gridDim.x * 4;
  uint32_t t = blockIdx.x * 4 + wv;
  uint4 a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3, b4, b5, b6, b7;
#define LD(x, tt) { const uint4* p = in + (size_t)(tt) * (kTile / 16); x##0 = p[lane]; x##1 = p[64 + lane]; x##2 = p[128 + lane]; x##3 = p[192 + lane]; x##4 = p[256 + lane]; x##5 = p[320 + lane]; x##6 = p[384 + lane]; x##7 = p[448 + lane]; }
#define ST(x) { s[lane] = x##0; s[64 + lane] = x##1; s[128 + lane] = x##2; s[192 + lane] = x##3; s[256 + lane] = x##4; s[320 + lane] = x##5; s[384 + lane] = x##6; s[448 + lane] = x##7; }
  uint32_t acc = s_pad[lane];
  if (t < ntiles) LD(a, t);
  if (D == 2 && t + nwaves < ntiles) LD(b, t + nwaves);
  auto work = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t v = (uint32_t)lane * 4u;
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(s_all[wv] + (v & (kTile - 4)));
      v = (w ^ (v * 2654435761u)) + (uint32_t)r * 68u + (uint32_t)lane * 4u;
      acc += w;
    }
    asm volatile("" ::: "memory");
  };
  for (; t < ntiles;) {
    ST(a);
    const uint32_t tn = t + (uint32_t)D * nwaves;
    if (tn < ntiles) LD(a, tn);
    work();
    t += nwaves;
    if (D == 2) {
      if (t >= ntiles) break;
      ST(b);
      const uint32_t tn2 = t + 2u * nwaves;
      if (tn2 < ntiles) LD(b, tn2);
      work();
      t += nwaves;
    }
  }
  if (acc == 0x12345u) out[0] = acc;
}

template <int D, int R, int PADKB>
int run(const uint4* d, uint32_t ntiles, uint32_t* out, size_t bytes) {
  int occ = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k<D, R, PADKB>, 256, 0));
  int dev = 0, ncu = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t grid = (uint32_t)(ncu * occ);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k<D, R, PADKB>), dim3(grid), dim3(256), 0, 0, d, ntiles, out);
  CHK(hipEventRecord(e0, 0));
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k<D, R, PADKB>), dim3(grid), dim3(256), 0, 0, d, ntiles, out);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("depth %d  R %3d  wg/CU %d  %.3f ms  %7.1f GB/s\n", D, R, occ, ms, bytes / (ms * 1e-3) / 1e9);
  return 0;
}

int main() {
  const size_t bytes = 4ull << 30;
  const uint32_t ntiles = (uint32_t)(bytes / kTile);
  uint4* d = nullptr;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&d, bytes));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(d, 0x41, bytes));
  // 4 WG/CU (pad 0: 33 KB each), 3 WG/CU (pad 20 KB), 2 WG/CU (pad 48 KB)
  run<1, 0, 0>(d, ntiles, out, bytes);
  run<2, 0, 0>(d, ntiles, out, bytes);
  run<1, 32, 0>(d, ntiles, out, bytes);
  run<2, 32, 0>(d, ntiles, out, bytes);
  run<1, 64, 0>(d, ntiles, out, bytes);
  run<2, 64, 0>(d, ntiles, out, bytes);
  run<1, 96, 0>(d, ntiles, out, bytes);
  run<2, 96, 0>(d, ntiles, out, bytes);
  run<1, 32, 20>(d, ntiles, out, bytes);
  run<2, 32, 20>(d, ntiles, out, bytes);
  run<1, 64, 20>(d, ntiles, out, bytes);
  run<2, 64, 20>(d, ntiles, out, bytes);
  run<1, 64, 48>(d, ntiles, out, bytes);
  run<2, 64, 48>(d, ntiles, out, bytes);
  run<1, 128, 20>(d, ntiles, out, bytes);
  run<2, 128, 20>(d, ntiles, out, bytes);
  return 0;
}
