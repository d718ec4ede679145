// Streaming microbenchmark for the scan kernel's access pattern on MI355X: how fast can
// 16 KiB tiles be read and newline-counted under different work distributions?
//   hipcc --offload-arch=gfx950 -O3 scripts/mb_stream.hip -o mb_stream && ./mb_stream
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t zcount(uint32_t x) {
  const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
  return __popc(z);
}
__device__ __forceinline__ uint32_t count4(uint4 v) {
  return zcount(v.x ^ 0x0A0A0A0Au) + zcount(v.y ^ 0x0A0A0A0Au) + zcount(v.z ^ 0x0A0A0A0Au) +
         zcount(v.w ^ 0x0A0A0A0Au);
}

constexpr int TILE = 16384;

// V0: one tile per workgroup, grid = tiles (coalesced 16 B per lane, 4 loads per lane)
__global__ __launch_bounds__(256) void v0(const uint4* in, uint32_t* out) {
  const uint4* p = in + (size_t)blockIdx.x * (TILE / 16);
  uint32_t c = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) c += count4(p[v * 256 + threadIdx.x]);
  c = __reduce_add_sync(~0ull, c);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[blockIdx.x & 1023], c);
}
// V1: persistent, static round robin (tile = blockIdx + k*grid)
__global__ __launch_bounds__(256) void v1(const uint4* in, uint32_t* out, uint32_t ntiles) {
  uint32_t c = 0;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p = in + (size_t)t * (TILE / 16);
#pragma unroll
    for (int v = 0; v < 4; ++v) c += count4(p[v * 256 + threadIdx.x]);
  }
  c = __reduce_add_sync(~0ull, c);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[blockIdx.x & 1023], c);
}
// V2: persistent, ticket groups (32 counters) + LDS broadcast of the ticket
__global__ __launch_bounds__(256) void v2(const uint4* in, uint32_t* out, uint32_t ntiles, uint32_t* ctr,
                                          uint32_t G, uint32_t stride) {
  __shared__ uint32_t s_t;
  const uint32_t g = blockIdx.x % G;
  uint32_t c = 0;
  for (;;) {
    if (threadIdx.x == 0) s_t = atomicAdd(&ctr[g * stride], 1u);
    __syncthreads();
    const uint32_t t = s_t * G + g;
    __syncthreads();
    if (t >= ntiles) break;
    const uint4* p = in + (size_t)t * (TILE / 16);
#pragma unroll
    for (int v = 0; v < 4; ++v) c += count4(p[v * 256 + threadIdx.x]);
  }
  c = __reduce_add_sync(~0ull, c);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[blockIdx.x & 1023], c);
}
// V3: V2 + LDS staging + per-thread 64 B contiguous reads + 3 barriers per tile
__global__ __launch_bounds__(256) void v3(const uint4* in, uint32_t* out, uint32_t ntiles, uint32_t* ctr) {
  __shared__ uint4 s_tile[TILE / 16 + 20];
  __shared__ uint32_t s_t, s_w[4];
  const uint32_t g = blockIdx.x & 31;
  uint32_t c = 0;
  for (;;) {
    if (threadIdx.x == 0) s_t = atomicAdd(&ctr[g], 1u);
    __syncthreads();
    const uint32_t t = s_t * 32 + g;
    if (t >= ntiles) break;
    const uint4* p = in + (size_t)t * (TILE / 16);
#pragma unroll
    for (int v = 0; v < 4; ++v) s_tile[v * 256 + threadIdx.x] = p[v * 256 + threadIdx.x];
    __syncthreads();
    uint32_t cc = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) cc += count4(s_tile[threadIdx.x * 4 + v]);
    cc = __reduce_add_sync(~0ull, cc);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = cc;
    __syncthreads();
    c += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(&out[blockIdx.x & 1023], c);
}
// ALU calibration: dependent integer ops per lane; reports the effective shader clock
__global__ __launch_bounds__(256) void alu(uint32_t* out, uint32_t iters) {
  uint32_t x = threadIdx.x, y = blockIdx.x;
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) { x = x * 1664525u + y; y ^= x >> 7; }
  }
  if (x == 0x12345678u && y == 1u) out[0] = x;
}
// V4: persistent static, 2 tiles in flight per workgroup (register double buffer)
__global__ __launch_bounds__(256) void v4(const uint4* in, uint32_t* out, uint32_t ntiles) {
  uint32_t c = 0;
  uint32_t t = blockIdx.x;
  uint4 a[4];
  if (t < ntiles) {
    const uint4* p = in + (size_t)t * (TILE / 16);
#pragma unroll
    for (int v = 0; v < 4; ++v) a[v] = p[v * 256 + threadIdx.x];
  }
  for (; t < ntiles; t += gridDim.x) {
    uint4 b[4];
    const uint32_t tn = t + gridDim.x;
    if (tn < ntiles) {
      const uint4* p = in + (size_t)tn * (TILE / 16);
#pragma unroll
      for (int v = 0; v < 4; ++v) b[v] = p[v * 256 + threadIdx.x];
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) c += count4(a[v]);
#pragma unroll
    for (int v = 0; v < 4; ++v) a[v] = b[v];
  }
  c = __reduce_add_sync(~0ull, c);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[blockIdx.x & 1023], c);
}

int main(int argc, char** argv) {
  const bool quick = argc > 1;
  const size_t bytes = (size_t)4 << 30;
  const uint32_t ntiles = (uint32_t)(bytes / TILE);
  uint8_t* d;
  uint32_t *out, *ctr;
  CHK(hipMalloc(&d, bytes));
  CHK(hipMalloc(&out, 4096 * 4));
  CHK(hipMalloc(&ctr, 1 << 20));
  std::vector<uint8_t> h(1 << 26);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (i % 431 == 430) ? '\n' : (uint8_t)('a' + i % 26);
  for (size_t o = 0; o < bytes; o += h.size()) CHK(hipMemcpy(d + o, h.data(), h.size(), hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const uint4* in = (const uint4*)d;
  auto run = [&](const char* name, auto launch) {
    float best = 1e9;
    for (int r = 0; r < 8; ++r) {
      (void)hipMemset(out, 0, 4096 * 4);
      (void)hipMemset(ctr, 0, 1 << 20);
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2 && ms < best) best = ms;
    }
    printf("%-40s %8.3f ms  %7.1f GB/s\n", name, best, bytes / best / 1e6);
  };
  if (quick) {  // calibration line for scripts/gpu_abl.sh
    run("calib v1 persistent static x4/CU", [&] { hipLaunchKernelGGL(v1, dim3(cus * 4), dim3(256), 0, 0, in, out, ntiles); });
    run("calib v4 register double buffer x4/CU", [&] { hipLaunchKernelGGL(v4, dim3(cus * 4), dim3(256), 0, 0, in, out, ntiles); });
    {
      const uint32_t iters = 20000;
      hipLaunchKernelGGL(alu, dim3(cus * 8), dim3(256), 0, 0, out, iters);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(alu, dim3(cus * 8), dim3(256), 0, 0, out, iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      // 8 waves/CU over 4 SIMDs = 2 waves per SIMD; each dependent op ~1 issue per 1 cycle
      // per wave (2 waves interleave): ops per SIMD = 2 * iters * 16 * 3
      printf("calib alu %.3f ms  ~%.2f G wave-ops/s per SIMD\n", ms, 2.0 * iters * 16 * 3 / (ms * 1e6));
    }
    return 0;
  }
  run("v0 one tile per WG", [&] { hipLaunchKernelGGL(v0, dim3(ntiles), dim3(256), 0, 0, in, out); });
  for (int occ : {4, 8}) {
    char n[96];
    snprintf(n, 96, "v1 persistent static x%d/CU", occ);
    run(n, [&] { hipLaunchKernelGGL(v1, dim3(cus * occ), dim3(256), 0, 0, in, out, ntiles); });
    for (uint32_t G : {32u, 64u, 128u, 256u}) for (uint32_t stride : {1u, 16u, 64u, 1024u}) {
      snprintf(n, 96, "v2 tickets G=%u stride=%uB x%d/CU", G, stride * 4, occ);
      run(n, [&] { hipLaunchKernelGGL(v2, dim3(cus * occ), dim3(256), 0, 0, in, out, ntiles, ctr, G, stride); });
    }
  }
  return 0;
}
