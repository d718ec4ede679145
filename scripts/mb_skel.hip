// Skeleton microbenchmark of the k_scan structure (persistent grid, a wave owns a tile from
// load to record, next tile prefetched in registers): which part of the structure costs
// bandwidth.  Variants: tile size per wave, LDS staging on/off, halo loads on/off, per-tile
// 16-B record on/off, workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/mb_skel.hip -o scripts/mb_skel
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t any_nl(const uint4& v) {
  const uint32_t m = 0xFEFEFEFFu, c = 0x0A0A0A0Au;
  return (((v.x ^ c) + m) | ((v.y ^ c) + m) | ((v.z ^ c) + m) | ((v.w ^ c) + m)) & 0x80808080u;
}

template <int ROWS, bool LDS, bool HALO, int REC>  // REC 0 none, 1 at the tile's end, 2 deferred before the next loads
__global__ __launch_bounds__(256) void skel(const uint8_t* __restrict__ in, uint32_t ntiles, uint4* rec, uint32_t* out) {
  constexpr int TILE = ROWS * 1024;
  __shared__ __attribute__((aligned(16))) uint8_t s_all[4][LDS ? TILE + 64 : 16];
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  uint8_t* s_tile = s_all[wv];
  const uint32_t nwaves = gridDim.x * 4;
  uint4 pf0, pf1, pf2, pf3, pf4, pf5, pf6, pf7;  // named: an array went to scratch
  uint4 pfh = make_uint4(0, 0, 0, 0);
  uint32_t tile = blockIdx.x * 4 + wv;
#define PF(r) if (ROWS > r) pf##r = gp[r * 64 + lane];
#define LOAD(tl)                                                                    \
  {                                                                                 \
    const uint4* gp = reinterpret_cast<const uint4*>(in + (size_t)(tl) * TILE);     \
    PF(0) PF(1) PF(2) PF(3) PF(4) PF(5) PF(6) PF(7)                                 \
    if (HALO && lane < 4 && (tl) + 1 < ntiles) pfh = gp[TILE / 16 + lane];          \
  }
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  // BUF: rows and halo by buffer loads; every lane, every tile (no branches: exact vmcnt
  // bookkeeping); a missing next tile is an empty resource (loads return 0)
#define BLD(r) if (ROWS > r) { const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rsl, (r * 64 + lane) * 16, 0, 0); pf##r = make_uint4(x[0], x[1], x[2], x[3]); }
#define BLOAD(tl)                                                                                        \
  {                                                                                                      \
    const bool ok = (tl) < ntiles;                                                                       \
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(                                \
        const_cast<uint8_t*>(in) + (size_t)(ok ? (tl) : 0) * TILE, 0, ok ? TILE + 64 : 0, 0x00020000);    \
    BLD(0) BLD(1) BLD(2) BLD(3) BLD(4) BLD(5) BLD(6) BLD(7)                                              \
    const u4v h = __builtin_amdgcn_raw_buffer_load_b128(rsl, lane < 4 ? TILE + lane * 16 : 0x7FFFFFF0, 0, 0); \
    pfh = make_uint4(h[0], h[1], h[2], h[3]);                                                            \
  }
  if (REC >= 10) { BLOAD(tile); } else if (tile < ntiles) LOAD(tile);
  uint32_t acc = 0;
  uint32_t d_s = 0, d_tile = ~0u;  // REC 2: the previous tile's record, stored before the next loads
  for (; tile < ntiles; tile += nwaves) {
    uint32_t nlc = 0;
    if (LDS) {
      uint4* l = reinterpret_cast<uint4*>(s_tile);
#define ST(r) if (ROWS > r) l[r * 64 + lane] = pf##r;
      ST(0) ST(1) ST(2) ST(3) ST(4) ST(5) ST(6) ST(7)
      if (HALO && (REC >= 10 || lane < 4)) l[TILE / 16 + (lane & 3)] = pfh;
      if (REC == 2 && d_tile != ~0u && lane == 0) rec[d_tile] = make_uint4(d_s, d_tile, 0, 0);
      if (REC >= 10) { BLOAD(tile + nwaves); } else if (tile + nwaves < ntiles) LOAD(tile + nwaves);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint4 xs[ROWS];
#pragma unroll
      for (int v = 0; v < ROWS; ++v)  // rotated chunk order: conflict-free ds_read_b128
        xs[v] = *reinterpret_cast<const uint4*>(s_tile + lane * ROWS * 16 + 16 * ((v + (lane >> 1)) & (ROWS - 1)));
#pragma unroll
      for (int v = 0; v < ROWS; ++v) nlc |= any_nl(xs[v]) ? (1u << v) : 0u;
    } else {
#define AN(r) if (ROWS > r) nlc |= any_nl(pf##r) ? (1u << r) : 0u;
      AN(0) AN(1) AN(2) AN(3) AN(4) AN(5) AN(6) AN(7)
      if (tile + nwaves < ntiles) LOAD(tile + nwaves);
    }
    const uint32_t c = __popc(nlc);
    acc += c;
    if (REC) {
      uint32_t s = c;
      if (REC != 4) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
      }
      if (REC == 3) acc += s;
      if (REC == 5 && lane < 8) rec[(size_t)tile * 8 + lane] = make_uint4(s, tile, lane, 0);
      if (REC == 6 && lane == 0) rec[(size_t)(blockIdx.x * 4 + wv) * (ntiles / nwaves + 1) + tile / nwaves] = make_uint4(s, tile, 0, 0);
      if (REC == 9 || REC == 10) {  // branch-free: every lane stores, lanes past 0 land out of range (dropped)
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(rec, 0, (int)(ntiles * 16u), 0x00020000);
        const u4v v = {s, tile, 0u, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, lane == 0 ? (int)(tile * 16u) : 0x7FFFFFF0, 0, 0);
      }
      if (REC == 7 && lane == 0) { typedef unsigned int u4v __attribute__((ext_vector_type(4))); u4v v = {s, tile, 0u, 0u}; __builtin_nontemporal_store(v, reinterpret_cast<u4v*>(&rec[tile])); }
      if (REC == 8 && lane == 0 && ((tile / nwaves) & 7) == 0) rec[tile] = make_uint4(s, tile, 0, 0);
      if ((REC == 1 || REC == 4) && lane == 0) rec[tile] = make_uint4(s, tile, 0, 0);
      d_s = s;
      d_tile = tile;
    }
    asm volatile("" ::: "memory");
  }
  if (REC == 2 && d_tile != ~0u && lane == 0) rec[d_tile] = make_uint4(d_s, d_tile, 0, 0);
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)4 << 30;
  uint8_t* d;
  uint32_t* out;
  uint4* rec;
  CHK(hipMalloc(&d, bytes + 65536));
  CHK(hipMalloc(&out, 4096 * 4));
  CHK(hipMalloc(&rec, (bytes / 1024 + 16) * 16));  // 16 B per KiB of input: REC 5 (128 B per 8 KiB tile), 1 record per tile down to 1 KiB tiles
  std::vector<uint8_t> h(1 << 26);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (i % 431 == 430) ? '\n' : (uint8_t)('a' + i % 26);
  for (size_t o = 0; o < bytes; o += h.size()) CHK(hipMemcpy(d + o, h.data(), h.size(), hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2 && ms < best) best = ms;
    }
    printf("%-48s %8.3f ms  %7.1f GB/s\n", name, best, bytes / best / 1e6);
    fflush(stdout);
  };
#define RUN(ROWS, LDS, HALO, REC, BPC)                                                                   \
  run(#ROWS "KiB lds=" #LDS " halo=" #HALO " rec=" #REC " x" #BPC "/CU", [&] {                        \
    hipLaunchKernelGGL((skel<ROWS, LDS, HALO, REC>), dim3(cus * BPC), dim3(256), 0, 0, d,              \
                       (uint32_t)(bytes / (ROWS * 1024)), rec, out);                                     \
  })
  for (int rep = 0; rep < 2; ++rep) {
    RUN(8, true, true, 0, 4);
    RUN(8, true, true, 1, 4);
    RUN(8, true, true, 9, 4);
    RUN(8, true, true, 10, 4);
  }
  return 0;
}
