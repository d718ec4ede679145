// klf_kernels.hip — CDNA4 (gfx950) kernels of the klogs filter path.
//
// Pipeline over one device batch (streams laid out as 256-B-aligned segments):
//   K1 k_scan      newline scan + RFC3339Nano parse + since mask per line + fused
//                  single-literal grep over 4 KiB wave-tiles, staged per tile;
//                  k_tsum/k_tbase tile line bases; k_scatter -> global line index
//   K2 k_match     general pattern sets: Aho-Corasick DFA + Glushkov bit-parallel NFA
//   K3 k_mcount    per-stream matched counts (chunk partials; parsed / since_ok come
//                  from k_tbase's prefixes)
//      k_tail      kubelet tail rule -> per-stream candidate window (one block / stream)
//      k_wprefix   exclusive prefix of window sizes
//   K4 k_csum / k_cscan / k_cgather   output offsets (reduce-then-scan over 1024-line
//                  blocks) + content gather copy
// Semantics: SPEC.md (kubelet logs.go ReadLogs / tail.go FindTailLineStartIndex /
// Go time.Parse(RFC3339Nano) / bytes.Contains / regexp.Match).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "klf_kernels.hpp"
#include "klf_ts.hpp"

namespace klf {
namespace {

#ifndef KLF_TIMELINE
#define KLF_TIMELINE 0
#endif
__device__ uint32_t g_abl_waves;  // timing builds: k_scan waves finished so far
#if KLF_TIMELINE
// Diagnostic build only: per tile {claim, loaded, A published, prefix known, done,
// look-back rounds, spins, cu/xcc} stamps (s_memtime), dumped by the engine.
__device__ uint64_t g_timeline[300000 * 8];
__device__ uint32_t g_lb_rounds, g_lb_spins;
#define KLF_STAMP(tile, k) do { if (threadIdx.x == 0 && (tile) < 300000) g_timeline[(size_t)(tile) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define KLF_STAMP(tile, k) do { } while (0)
#endif
// Diagnostic build only (KLF_TIMELINE): k_verify's phases per hit thread, slot k of its global
// thread id (s_memtime; 0 = phase not reached)
#if KLF_TIMELINE
#define KLF_VSTAMP(k) do { const uint32_t vg_ = (blockIdx.x * blockDim.x + threadIdx.x) % 300000u; \
  g_timeline[(size_t)vg_ * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define KLF_VSTAMP(k) do { } while (0)
#endif

// ------------------------------------------------------------------ small helpers ---

template <class T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}
template <class T>
__device__ __forceinline__ T wave_incl_scan_add(T x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(x, d, 64);
    if (lane >= d) x += o;
  }
  return x;
}

// 32-bit wave scans / reductions on DPP (row_shr within 16-lane rows, then the row totals
// through v_readlane): no LDS round trips (the generic __shfl versions above lower to
// ds_bpermute, ~100 cycles each, six in a chain).  Exact-type overloads: every u32 call
// site picks these.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {  // lanes with no source read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_incl_scan_add(uint32_t x, int lane) {
  x += dpp0<0x111>(x);  // row_shr:1
  x += dpp0<0x112>(x);  // row_shr:2
  x += dpp0<0x114>(x);  // row_shr:4
  x += dpp0<0x118>(x);  // row_shr:8
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
  const uint32_t r1 = r0 + (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
  const uint32_t r2 = r1 + (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
  const int row = lane >> 4;
  return x + (row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) + (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
         (uint32_t)__builtin_amdgcn_readlane((int)x, 47) + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  x = mx(x, dpp0<0x111>(x));
  x = mx(x, dpp0<0x112>(x));
  x = mx(x, dpp0<0x114>(x));
  x = mx(x, dpp0<0x118>(x));
  return mx(mx((uint32_t)__builtin_amdgcn_readlane((int)x, 15), (uint32_t)__builtin_amdgcn_readlane((int)x, 31)),
            mx((uint32_t)__builtin_amdgcn_readlane((int)x, 47), (uint32_t)__builtin_amdgcn_readlane((int)x, 63)));
}

__device__ __forceinline__ uint32_t wave_incl_scan_max(uint32_t x, int lane) {
  auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  x = mx(x, dpp0<0x111>(x));  // row_shr:1 (lanes without a source read 0)
  x = mx(x, dpp0<0x112>(x));
  x = mx(x, dpp0<0x114>(x));
  x = mx(x, dpp0<0x118>(x));
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
  const uint32_t r1 = mx(r0, (uint32_t)__builtin_amdgcn_readlane((int)x, 31));
  const uint32_t r2 = mx(r1, (uint32_t)__builtin_amdgcn_readlane((int)x, 47));
  const int row = lane >> 4;
  return mx(x, row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}

__device__ __forceinline__ uint32_t find_seg_by_tile(const SegDesc* segs, uint32_t n, uint32_t tile) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].tile0 <= tile) lo = mid; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t find_seg_by_line(const SegOut* so, uint32_t n, uint64_t l) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (so[mid].line_lo <= l) lo = mid; else hi = mid;
  }
  return lo;
}

// Byte source for the general timestamp parser (k_fixup): global memory, -1 past the
// end of the stream.
struct GlobalBytes {
  const uint8_t* seg;  // global stream base
  int64_t p0;          // stream offset of the line start
  int64_t seg_len;
  __device__ __forceinline__ int operator()(uint32_t i) const {
    const int64_t q = p0 + (int64_t)i;
    return q < seg_len ? (int)seg[q] : -1;
  }
};
__device__ __forceinline__ uint16_t make_meta(bool ok, bool since_ok, uint32_t plen) {
  if (!ok) return 0;
  const uint32_t pl = plen < kPlenEscape ? plen : kPlenEscape;
  return (uint16_t)(Meta::kParsed | (since_ok ? Meta::kSince : 0) | (pl << 2));
}

// ============================================================== K1: the scan ==
// Streaming scan with no inter-workgroup waiting and no workgroup barriers in the loop.
// The unit of work is an 8 KiB WAVE-TILE owned by one wave from load to record (static
// round robin over a persistent grid); the next wave-tile is in flight in registers
// (32 VGPRs) while this one is processed from the wave's LDS region.
//   * line ends: per lane 128 contiguous bytes; a SWAR any-test per 16-B chunk (2-3 VALU
//     per dword), exact byte positions only for chunks that hit (a line ends every few
//     hundred bytes, so most chunks never take the exact step);
//   * in-wave scan (DPP) of the per-lane event counts -> local line numbers; the line
//     starts go to a per-wave LDS list (slot j = j-th line starting in the tile);
//   * one parse pass over the list, one line per lane: the canonical kubelet prefix
//     "YYYY-MM-DDTHH:MM:SS.nnnnnnnnnZ " (logs.go timeFormatOut) in SWAR (v_perm digit
//     packing, u24 multiply-adds, since compared as (day, second of day, ns)); any other
//     shape is DEFERRED to k_fixup, which runs the general Go time.Parse restatement;
//   * fused single literal (--grep): rare-byte anchor any-test per chunk, candidates
//     verified from LDS, the hit's line found by binary search in the list;
//   * slots (u32: start offset in the tile, defer bit, literal-hit bit, u16 meta) are
//     written once per tile; tiles with more starts than kSlots use a global pool.
//   K1b/K1c  device scan of the per-tile line counts -> tile line bases, stream ranges.
//   K1d      k_scatter: slots -> global line_off (u64) / meta (u16) / match bitmap.

constexpr uint32_t kSlotOff = 0x3FFFu, kSlotDefer = 0x4000u, kSlotHit = 0x8000u;
constexpr uint32_t kCtrDefer = 5;  // counters[5]: some line of this run was deferred
constexpr uint32_t kTsInline = 16u;  // TileStat.flags: the tile's single line slot is its pool_base word
constexpr uint32_t kTsHitInline = 32u;  // TileStat.flags (general sets): its 1-2 prefilter hits are pool_base's halves
// Kept runs of one tile (a selected line carries a >= 20-B prefix, so at most kTile / 20
// + 2 runs: the carried-in line's and those of the lines starting in the tile) and its
// 16-B output chunks (513 at most, in groups of 8: 16-B LDS accesses).
constexpr int kTcRuns = kTile / 20 + 8;     // + the two sentinels
constexpr int kTcChunks = kTile / 16 + 8;

// ---- planned dense compaction (RunArgs::plan_runs: no patterns, --tail -1) ---------------
// With every line decided where it starts (parsed and since_ok: SPEC.md S3/S4 with tail -1)
// the scan lists each tile's kept runs of the lines starting in it, and the tile's output
// offset and carried-in run follow from a scan over tile aggregates (k_cmid / k_cmove, no
// line-index pass).  A range's aggregate is a function of the state entering it:
//   bytes  kept bytes of the lines starting in the range,
//   has    some line starts in the range,
//   span   bytes from the range start to its first line start (the range when !has): the
//          entering line's part, kept from its content start on when that line is kept,
//   sel / crel   the line open at the range end: kept?, its content start - the range end.
// A stream's first tile lists its line 0 at offset 0 (span 0), so nothing carries across
// streams.  Deferred lines (non-canonical prefixes, decided later by fix_tile) void the
// plan: the run then lists its tiles from the line slots (k_tkeep).
struct FAgg {
  uint64_t bytes;  // (the blocks before a k_cmove block: the whole output so far, past 4 GiB)
  uint32_t span;
  int32_t crel;
  bool has, sel;
};
struct FPre {
  uint64_t off;
  int32_t crel;  // content start of the open line - the boundary
  bool sel;
};
// a content start before the boundary: kept from the boundary on, however far back (-1)
__device__ __forceinline__ int32_t f_sat(int32_t crel) { return crel < 0 ? -1 : crel; }
__device__ __forceinline__ uint32_t f_carried(uint32_t span, bool sel, int32_t crel) {
  const int32_t lo = crel > 0 ? crel : 0;
  return (sel && (int32_t)span > lo) ? (uint32_t)((int32_t)span - lo) : 0u;
}
// X then Y
__device__ __forceinline__ FAgg f_combine(const FAgg& x, const FAgg& y) {
  FAgg z;
  z.bytes = x.bytes + y.bytes + (x.has ? f_carried(y.span, x.sel, x.crel) : 0u);
  z.has = x.has || y.has;
  z.span = x.has ? x.span : x.span + y.span;
  if (y.has) { z.sel = y.sel; z.crel = y.crel; }
  else { z.sel = x.sel; z.crel = f_sat(x.crel - (int32_t)y.span); }  // !y.has: y.span = its length
  return z;
}
__device__ __forceinline__ FPre f_apply(const FPre& p, const FAgg& z) {
  FPre r;
  r.off = p.off + z.bytes + f_carried(z.span, p.sel, p.crel);
  if (z.has) { r.sel = z.sel; r.crel = z.crel; }
  else { r.sel = p.sel; r.crel = f_sat(p.crel - (int32_t)z.span); }
  return r;
}
// a tile's plan (the scan -> trec[tile] until k_cmove rewrites it): x = bytes | span << 14
// | has << 28 | sel << 29, y = crel (16 bits signed) | nsel << 16, z = own runs (or
// kRunsRecompute), w = kPlanTag
constexpr uint32_t kPlanTag = 0x504C414Eu;
constexpr uint32_t kRunsShifted = 0x4000u;  // TRec.nruns: runs 1.. shift by TRec.nsel (run 0 = carried)
__device__ __forceinline__ bool planned(const RunArgs& a) { return a.plan_runs && !a.counters[kCtrDefer]; }
__device__ __forceinline__ FAgg plan_agg(const uint4& r) {
  FAgg a;
  a.bytes = r.x & 0x3FFFu;
  a.span = (r.x >> 14) & 0x3FFFu;
  a.has = (r.x >> 28) & 1u;
  a.sel = (r.x >> 29) & 1u;
  a.crel = (int32_t)(int16_t)(uint16_t)(r.y & 0xFFFFu);
  return a;
}
__device__ __forceinline__ FAgg wave_incl_scan_fagg(FAgg x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    FAgg y;
    y.bytes = __shfl_up(x.bytes, d, 64);
    y.span = (uint32_t)__shfl_up((int)x.span, d, 64);
    y.crel = __shfl_up(x.crel, d, 64);
    const int fl = __shfl_up((x.has ? 1 : 0) | (x.sel ? 2 : 0), d, 64);
    y.has = fl & 1;
    y.sel = (fl & 2) != 0;
    if (lane >= d) x = f_combine(y, x);
  }
  return x;
}

// Any-test: nonzero when some byte of the 16 equals the byte replicated in c4.  One
// v_xad_u32 per dword ((x ^ c4) - 0x01..01: bit 7 of an equal byte is set) and 3-input
// ORs; it also flags bytes with (x ^ c) >= 0x81 (non-ASCII text) and bytes above a true
// match (borrow) -- false flags only send the chunk to the exact test.
__device__ __forceinline__ uint32_t xad(uint32_t x, uint32_t c, uint32_t d) {  // (x ^ c) + d
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(c), "v"(d));
  return r;
}
__device__ __forceinline__ uint32_t any_eq16(const uint4& v, uint32_t c4) {
  const uint32_t m = 0xFEFEFEFFu;  // -0x01010101
  return (xad(v.x, c4, m) | xad(v.y, c4, m) | xad(v.z, c4, m) | xad(v.w, c4, m)) & 0x80808080u;
}
// exact: bit i set iff byte i of the 16 bytes equals the byte in c4
__device__ __forceinline__ uint32_t eq_mask16(const uint4& v, uint32_t c4) {
  auto z = [c4](uint32_t x) {
    const uint32_t y = x ^ c4;
    const uint32_t f = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;  // 0x80 per equal byte
    return (f * 0x00204081u) >> 28;  // flags 7,15,23,31 -> bits 0..3 (no carries)
  };
  return z(v.x) | (z(v.y) << 4) | (z(v.z) << 8) | (z(v.w) << 12);
}

// eq_mask16 for '\n' (any byte with bit 7 clear): bit 7 of x ^ c is bit 7 of x, so an
// equal byte is ~((((x & 0x7F..) ^ c) + 0x7F..) | x) & 0x80..: and, xad, one 3-input op
// per dword instead of six
__device__ __forceinline__ uint32_t nor_and(uint32_t a, uint32_t b, uint32_t c) {  // ~(a | b) & c
  uint32_t r;  // (v_bitop3 table: bit a*4 + b*2 + c; the compiler emits or, not, and)
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x02" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}
__device__ __forceinline__ uint32_t eq_mask16_nl(const uint4& v) {
  auto z = [](uint32_t x) {
    const uint32_t t = xad(x & 0x7F7F7F7Fu, 0x0A0A0A0Au, 0x7F7F7F7Fu);
    const uint32_t f = nor_and(t, x, 0x80808080u);  // 0x80 per '\n'
    return (f * 0x00204081u) >> 28;  // flags 7,15,23,31 -> bits 0..3 (no carries)
  };
  return z(v.x) | (z(v.y) << 4) | (z(v.z) << 8) | (z(v.w) << 12);
}

template <class T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const T o = __shfl_xor(x, d, 64);
    x = o > x ? o : x;
  }
  return x;
}

// A wave's own LDS writes are visible to its later LDS reads (the LDS executes one wave's
// instructions in order); this keeps the compiler from reordering across the point and
// waits for the writes to land.  No workgroup barrier is involved.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(256) void k_tiles(const SegDesc* segs, uint32_t nsegs, uint32_t ntiles,
                                               uint32_t* tile_seg) {
  for (uint32_t tile = blockIdx.x * 256 + threadIdx.x; tile < ntiles; tile += gridDim.x * 256)
    tile_seg[tile] = find_seg_by_tile(segs, nsegs, tile);
}

// v_mul_hi_u32_u24: bits 32..47 of the product of the low 24 bits of a and b (no intrinsic;
// the 64-bit C++ form only lowers to it when a is known to fit in 24 bits)
__device__ __forceinline__ uint32_t mul_hi_u24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "s"(b), "v"(a));
  return r;
}
// v_mul_u32_u24 / v_bfe_u32 as single instructions: __umul24 keeps an explicit 24-bit mask
// in front of the multiply, and a bfe feeding an xor is split into shift + and
__device__ __forceinline__ uint32_t mul_u24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(b), "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t bfe_u32(uint32_t a, uint32_t off, uint32_t width) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "n"(off), "n"(width));
  return r;
}
// w >> ((h >> 8) & 31) in one instruction (the shift amount as an SDWA byte select; the
// compiler emits a separate shift for it)
__device__ __forceinline__ uint32_t shr_byte1(uint32_t w, uint32_t h) {
  uint32_t r;
  asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
      : "=v"(r) : "v"(h), "v"(w));
  return r;
}
#ifndef KLF_PARSE_UNALIGNED
#define KLF_PARSE_UNALIGNED 1  // the timestamp prefix read with unaligned 16-B LDS loads
#endif
// Canonical kubelet prefix at LDS byte offset o (bytes o .. o + 30 valid): true with
// since_ok set when the line starts "YYYY-MM-DDTHH:MM:SS.nnnnnnnnnZ " with a valid date,
// year 1970..2099 (where the Gregorian leap rule is y % 4 == 0).  The 23 digits are packed
// big-endian (p0..p5: first digit in the top byte), so for valid dates the digit strings
// order like the instants and since is one lexicographic compare against the cutoff's
// digits (RunArgs::since_dig): no day / second arithmetic.  Only days 29..31 (and 00)
// need the month's length.  The value equals Go time.Parse's for exactly these inputs;
// false sends the line to the general parser.
__device__ __forceinline__ bool parse_fast(const uint8_t* lds, uint32_t o, const uint32_t (&cut)[6], bool& since_ok) {
  uint32_t w[8];
  if (KLF_PARSE_UNALIGNED) {
    // two 16-B reads at the line start itself: gfx950 LDS serves unaligned ds_read_b128
    // (the HSA default unaligned access mode), so no byte alignment in VALU
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 x0, x1;
    __builtin_memcpy(&x0, lds + o, 16);
    __builtin_memcpy(&x1, lds + o + 16, 16);
    w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
    w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
  } else {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(lds);
    const uint32_t base = o >> 2, sh = o & 3u;
    uint32_t prev = s32[base];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t nx = s32[base + j + 1];
      w[j] = __builtin_amdgcn_alignbyte(nx, prev, sh);
      prev = nx;
    }
  }
  // separators: '-' 4, '-' 7, 'T' 10, ':' 13, ':' 16, '.' 19, 'Z' 29, ' ' 30
  const uint32_t sep = ((w[1] ^ 0x2D00002Du) & 0xFF0000FFu) | ((w[2] ^ 0x00540000u) & 0x00FF0000u) |
                       ((w[3] ^ 0x00003A00u) & 0x0000FF00u) | ((w[4] ^ 0x2E00003Au) & 0xFF0000FFu) |
                       ((w[7] ^ 0x00205A00u) & 0x00FFFF00u);
  // the 23 digits in 6 dwords, big-endian (one pad '0' before the last digit)
  const uint32_t p0 = __builtin_amdgcn_perm(0u, w[0], 0x00010203u);                   // Y Y Y Y
  const uint32_t p1 = __builtin_amdgcn_perm(w[2], w[1], 0x01020405u);                 // M M D D
  const uint32_t p2 = __builtin_amdgcn_perm(w[3], w[2], 0x03040607u);                 // h h m m
  const uint32_t p3 = __builtin_amdgcn_perm(w[5], w[4], 0x01020405u);                 // s s n0 n1
  const uint32_t p4 = __builtin_amdgcn_perm(w[6], w[5], 0x02030405u);                 // n2 n3 n4 n5
  const uint32_t p5 = __builtin_amdgcn_perm(w[7], w[6], 0x02030C04u) | 0x00003000u;  // n6 n7 0 n8
  // digit check: high nibble 3 everywhere, low nibble <= 9 (no cross-byte carry once the
  // high nibbles are 3)
  const uint32_t hi = ((p0 ^ 0x30303030u) | (p1 ^ 0x30303030u) | (p2 ^ 0x30303030u) | (p3 ^ 0x30303030u) |
                       (p4 ^ 0x30303030u) | (p5 ^ 0x30303030u)) & 0xF0F0F0F0u;
  const uint32_t lo = ((p0 + 0x06060606u) | (p1 + 0x06060606u) | (p2 + 0x06060606u) | (p3 + 0x06060606u) |
                       (p4 + 0x06060606u) | (p5 + 0x06060606u)) & 0x40404040u;
  if ((sep | hi | lo) != 0u) return false;
  // field ranges on the big-endian digit pairs (all bytes are digits here)
  if (p0 - 0x31393730u > 0x32303939u - 0x31393730u) return false;        // year 1970..2099
  if ((p1 >> 16) - 0x3031u > 0x3132u - 0x3031u) return false;            // month 01..12
  if ((p2 >> 16) > 0x3233u || (p2 & 0xFFFFu) > 0x3539u || (p3 >> 16) > 0x3539u) return false;  // hh mm ss
  if ((p1 & 0xFFFFu) - 0x3031u > 0x3238u - 0x3031u) {  // day outside 01..28: the month's length
    const uint32_t day = ((p1 >> 8) & 15u) * 10u + (p1 & 15u);
    const uint32_t month = ((p1 >> 24) & 15u) * 10u + ((p1 >> 16) & 15u);
    const uint32_t yy = ((p0 >> 8) & 15u) * 10u + (p0 & 15u);  // year mod 100 (100 = 0 mod 4)
    const uint32_t dim = month == 2u ? 28u + ((yy & 3u) == 0u ? 1u : 0u) : 30u + ((month + (month >> 3)) & 1u);
    if (day - 1u >= dim) return false;
  }
  // lexicographic: the line's digits >= the cutoff's (not Before(since))
  const uint64_t a0 = (uint64_t)p0 << 32 | p1, a1 = (uint64_t)p2 << 32 | p3, a2 = (uint64_t)p4 << 32 | p5;
  const uint64_t c0 = (uint64_t)cut[0] << 32 | cut[1], c1 = (uint64_t)cut[2] << 32 | cut[3],
                 c2 = (uint64_t)cut[4] << 32 | cut[5];
  since_ok = a0 > c0 || (a0 == c0 && (a1 > c1 || (a1 == c1 && a2 >= c2)));
  return true;
}

#ifndef KLF_ABL
#define KLF_ABL 0
#endif
#ifndef KLF_SCAN_NT
// the scan's prefetch rows as non-temporal loads (read once; L1 bypassed): C5 k_scan
// 6.33 -> 6.09-6.12 ms, C2 0.92-0.93 -> 0.89-0.92, C4 7.72 -> 7.64 (same box, two rounds
// each, gpurun_out/r5d, r5e)
#define KLF_SCAN_NT 1
#endif
#ifndef KLF_SCAN_PRIO
#define KLF_SCAN_PRIO 0  // s_setprio level while a wave stages its tile and issues the next one
#endif
#ifndef KLF_NL_MASK
#define KLF_NL_MASK 1  // the exact newline positions with the three-op test (eq_mask16_nl)
#endif
#ifndef KLF_SCAN_BALLOT
#define KLF_SCAN_BALLOT 1  // per-lane 0/1 counts (sparse lines) summed / ranked by ballots
#endif
#ifndef KLF_SCAN_PACKSUM
#define KLF_SCAN_PACKSUM 1  // the tile's parsed / since_ok counts in one wave reduction
#endif
#ifndef KLF_VERIFY_PAR
#define KLF_VERIFY_PAR 0  // k_verify: 1 loads a needle's dwords 1..7 at once (C4: 468 vs 452 us, more VGPRs, r6e)
#endif
#ifndef KLF_HIT_INLINE
#define KLF_HIT_INLINE 0  // 1: a tile's 1-2 prefilter hits in its TileStat (C4 k_scan +2.8 %, r6e)
#endif
#ifndef KLF_TS_INLINE
#define KLF_TS_INLINE 1  // a tile where one line starts keeps its slot in the TileStat (no record store)
#endif
#ifndef KLF_SCAN_SUMSKIP
// no count reductions on tiles where no line starts (C5: ~half its tiles): 6.33 -> 6.29 ms
#define KLF_SCAN_SUMSKIP 1
#endif
typedef uint32_t klf_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const klf_v4u v = __builtin_nontemporal_load(reinterpret_cast<const klf_v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
#ifndef KLF_CG_NT
#define KLF_CG_NT 0
#endif
#ifndef KLF_CG_GRID
#define KLF_CG_GRID 8  // k_cgather workgroups per CU
#endif
#ifndef KLF_CG_PF2
#define KLF_CG_PF2 1  // C3 compaction 7.12 -> 6.78 ms (U=2 on top: 7.81)
#endif
#ifndef KLF_COPY_U
#define KLF_COPY_U 1
#endif
#ifndef KLF_ANY_BATCH
#define KLF_ANY_BATCH 8  // chunk reads in flight in the scan's newline any-test
#endif
#ifndef KLF_SCAN_OCC
// plain / literal scans: waves per SIMD the launch bounds ask for.  3 leaves the compiler
// up to 168 VGPRs: C3's plain scan 1.84 -> 1.67 ms, C2's literal scan unchanged within the
// box spread (0.90-0.94 ms either way), 5: no better (same box, scripts/r3_check15.sh)
#define KLF_SCAN_OCC 3
#endif
// Scan variants: no patterns, the fused single literal, general sets through the fused
// q-gram prefilter (QS = sampling stride).
constexpr int kScanPlain = 0, kScanLit = 1, kScanGen = 2;

// The tile descriptors come in as separate __restrict__ const parameters so that their
// (wave-uniform) reads compile to scalar loads: a vector load of them would be ordered
// behind the in-flight prefetch by vmcnt and stall every tile on the next tile's bytes.
// General sets: QS sampling stride, QK bits per gram, QQ gram bytes (3 or 4), QA (stride 8
// only) the short needles' anchor test (DevPatterns::qf_anc_*).
__device__ __forceinline__ void copy_tile_runs(const uint8_t* s_buf, uint32_t* s_run, uint16_t* s_map, uint32_t nr,
                                               uint32_t kept, uint64_t obase, uint8_t* out, int lane);

// FUSE (plain scan only; RunArgs::fuse): the one-pass compaction of runs without patterns and
// with --tail -1.  Each wave owns a contiguous range of fuse_range tiles (a multiple of
// kScanGroup) and compacts their kept bytes in place: the range's output starts where its
// input starts (output <= input), so no offset depends on another wave.  A range's output is
// one extent per stream it touches (fuse_ext[fuse_ext0[range] + k] = {start, length});
// the bytes before the range's first line start belong to a line that started in an earlier
// range: the wave leaves that many bytes free in front of its output and k_fcarry fills them
// from the state the earlier ranges left (fuse_rinfo) once every range has been scanned.
// A dense tile or a deferred line voids the pass (counters[kCtrFuseBad]: the host reruns
// the two-pass compaction).
template <int MODE, int QS, int QK, int QQ = 4, bool QA = false, bool FUSE = false>
__global__ __launch_bounds__(kThreads, MODE == kScanGen ? 3 : KLF_SCAN_OCC) void k_scan(RunArgs a, const uint32_t* __restrict__ tseg,
                                                               const SegDesc* __restrict__ segs) {
  static_assert(!FUSE || MODE == kScanPlain, "the fused compaction runs in the plain scan");
  constexpr bool LIT = MODE == kScanLit;
  constexpr bool GEN = MODE == kScanGen;
  constexpr bool ANC = GEN && QA;
  static_assert(QQ == 3 || QQ == 4, "3- or 4-byte grams");
  constexpr int kWaves = kThreads / 64;
  constexpr int kRows = kTile / 1024;  // 1 KiB rows: 16 B per lane per row
  // (FUSE: 16 B of front pad, which copy_tile_runs' unaligned windows read)
  constexpr int kPad = FUSE ? 16 : 0;
  __shared__ __attribute__((aligned(16))) uint8_t s_tile_all[kWaves][kPad + kTile + kHalo];
  __shared__ __attribute__((aligned(16))) uint32_t s_frun_all[FUSE ? kWaves : 1][FUSE ? kTcRuns : 1];
  __shared__ __attribute__((aligned(16))) uint16_t s_fmap_all[FUSE ? kWaves : 1][FUSE ? kTcChunks : 8];
  __shared__ __attribute__((aligned(16))) uint32_t s_list_all[kWaves][kSlotStride];
  __shared__ __attribute__((aligned(16))) uint32_t s_lit[kMaxFusedLiteral / 4 + 1];  // literal, zero padded
  // the TileStats of the wave's current tile group: LDS for the plain / literal scans (a
  // register quad there spills), a register quad for GEN (LDS is what bounds its occupancy)
  __shared__ uint4 s_gstat[GEN ? 1 : kWaves][kScanGroup];
  __shared__ uint32_t s_qf[GEN ? kQfWords : 1];  // q-gram bitmap of the needles
  __shared__ uint32_t s_h2[GEN ? kWaves : 1][1];  // a tile's inline hits (kTsHitInline): two u16
  // wv is wave-uniform; readfirstlane tells the compiler so (tile indices stay in SGPRs and
  // the descriptor reads stay scalar loads)
  const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
  uint8_t* s_tile = s_tile_all[wv] + kPad;
  uint32_t* s_list = s_list_all[wv];
  uint32_t* err_flag = a.counters + 2;
  for (uint32_t i = t; i < kMaxFusedLiteral / 4 + 1; i += kThreads)
    s_lit[i] = (LIT && i < (a.lit_len + 3) / 4) ? a.lit_words[i] : 0u;
  if (GEN)
    for (uint32_t i = t; i < kQfWords; i += kThreads) s_qf[i] = a.pats.qf_bitmap[i];
  __syncthreads();  // the kernel's only block barrier
  const uint32_t nwaves = gridDim.x * kWaves;
  // Timing builds (KLF_ABL != 0, scripts/variant.sh): the first launch is the full scan;
  // from the second launch on (a wave knows once every wave of an earlier launch has
  // finished) the ablated scan runs and stores nothing, so the first launch's records feed
  // the downstream kernels (identical batches) and no ablation can misdirect them.
  // KLF_ABL bits: 2 no literal anchor test, 64 staging + any-test only, 1 no timestamp
  // parse, 128 no line list / parse / literal, 4 no prefilter fast pass, 8 prefilter
  // probes only; 4096 = nothing removed (the scan without its stores).
  const bool abl = (KLF_ABL != 0) &&
                   __hip_atomic_load(&g_abl_waves, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nwaves;
#define ABL(x) ((KLF_ABL & (x)) && abl)

  // the prefetch registers are named (an array here was put on the scratch stack)
  static_assert(kRows == 8, "KLF_ROWS lists the 8 prefetch rows");
#define KLF_ROWS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define KLF_DECL(r) uint4 pf##r;
  KLF_ROWS(KLF_DECL)
#undef KLF_DECL
// non-temporal prefetch loads in the literal / general scans (not the plain one: C3's
// k_tcopy re-reads the input, 5.15 -> 5.18 ms with them)
#define KLF_LOAD(r) pf##r = (KLF_SCAN_NT && MODE != kScanPlain) ? ld_nt(&gp[r * 64 + lane]) : gp[r * 64 + lane];
#define KLF_STORE(r) l[r * 64 + lane] = pf##r;
  uint4 pfh = make_uint4(0, 0, 0, 0);
  // A wave takes groups of kScanGroup consecutive tiles (group g, g + nwaves, ...): their
  // TileStats go out together as one whole-line store into the compact tstat array.
  // (FUSE: the wave's own range of consecutive tiles instead)
  auto next_tile = [&](uint32_t x) -> uint32_t {
    return (FUSE || (x % kScanGroup) != kScanGroup - 1) ? x + 1 : x + 1 + kScanGroup * (nwaves - 1);
  };
  const uint32_t gw = blockIdx.x * kWaves + wv;
  uint32_t tile = FUSE ? gw * a.fuse_range : gw * kScanGroup;
  const uint32_t tile_end = FUSE ? (tile + a.fuse_range < a.ntiles ? tile + a.fuse_range : a.ntiles) : a.ntiles;
  const uint32_t range_t0 = tile;
  uint4 stv = make_uint4(0, 0, 0, 0);  // GEN: lane k holds the group's TileStat k
  // The segment of the prefetched tile travels with it (scalar registers): a stride of
  // nwaves tiles stays inside one stream for all but the last tiles of a long stream, so
  // the dependent descriptor loads (tseg -> segs, scalar-cache misses at this stride) leave
  // the path that issues the next prefetch.
  uint32_t pf_s = 0;
  SegDesc pf_sd{};
  if (tile < a.ntiles) {
    pf_s = tseg[tile];
    pf_sd = segs[pf_s];
    const uint4* gp = reinterpret_cast<const uint4*>(a.bytes + pf_sd.base + (uint64_t)(tile - pf_sd.tile0) * kTile);
    KLF_ROWS(KLF_LOAD)
    if (lane < kHalo / 16) pfh = (KLF_SCAN_NT && MODE != kScanPlain) ? ld_nt(&gp[kTile / 16 + lane]) : gp[kTile / 16 + lane];
  }
  // Each tile ends with exactly one unconditional store instruction (the first two 128-B
  // lines of its record region, through a buffer descriptor so that an ablated launch can
  // drop it): a dropped store here gives the loop entry the same count behind the first
  // prefetch, so the compiler's wait for the prefetched rows (vmcnt in issue order) stops
  // short of the previous tile's store instead of waiting for it to complete.
  {
    const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(a.slots, 0, 0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0x7FFF0000u, 0, 0);
  }
  bool any_defer = false;
  uint32_t wp_cur = 0, wp_end = 0;  // the wave's pool chunk (wave_pool): next free slot, end
  // FUSE state of the wave's range (wave-uniform): whether the line open at the current tile
  // start is decided (a line started in this range's part of the stream, or the part began
  // at the stream's start), that line's kept bit and content start - the tile start (f_sat),
  // the output position, the current extent
  bool fz_known = false, fz_sel = false, fz_res_set = false;
  int32_t fz_crel = -1;
  uint64_t fz_obase = 0, fz_estart = 0, fz_res = 0, fz_part = 0, fz_rbase = 0;
  uint32_t fz_ext = 0;
  if (FUSE && tile < tile_end) {
    fz_rbase = pf_sd.base + (uint64_t)(tile - pf_sd.tile0) * kTile;
    fz_ext = a.fuse_ext0[gw];
  }
  // closes the current extent (a range part that saw no line start: all of it is left to
  // k_fcarry, the extent empty at its end)
  auto fz_close = [&]() __attribute__((always_inline)) {
    if (!fz_res_set) {
      fz_res = fz_part;
      fz_res_set = true;
      fz_estart = fz_obase = fz_rbase + fz_part;
    }
    if (lane == 0) {
      a.fuse_ext[2 * (size_t)fz_ext] = fz_estart;
      a.fuse_ext[2 * (size_t)fz_ext + 1] = fz_obase - fz_estart;
    }
  };
  for (; tile < tile_end; tile = next_tile(tile)) {
    const uint32_t s = pf_s;
    const SegDesc sd = pf_sd;
    const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
    const int64_t seg_len = (int64_t)sd.len;
    const int32_t tile_len = (int32_t)(seg_len - rel_lo < kTile ? seg_len - rel_lo : kTile);
    const bool first = rel_lo == 0;
    const bool last = rel_lo + kTile >= seg_len;
    const uint8_t* segp = a.bytes + sd.base;

    // ---- stage this tile in the wave's LDS region, then start loading the next one ----
    if (KLF_SCAN_PRIO) __builtin_amdgcn_s_setprio(KLF_SCAN_PRIO);  // A/B: the prefetch issue first
    {
      uint4* l = reinterpret_cast<uint4*>(s_tile);
      KLF_ROWS(KLF_STORE)
      if (lane < kHalo / 16) l[kTile / 16 + lane] = pfh;
      const uint32_t nx = next_tile(tile);
      if (nx < tile_end) {
        if (nx - sd.tile0 >= sd.ntiles) {
          pf_s = tseg[nx];
          pf_sd = segs[pf_s];
        }
        const uint4* gp = reinterpret_cast<const uint4*>(a.bytes + pf_sd.base + (uint64_t)(nx - pf_sd.tile0) * kTile);
        KLF_ROWS(KLF_LOAD)
        if (lane < kHalo / 16) pfh = (KLF_SCAN_NT && MODE != kScanPlain) ? ld_nt(&gp[kTile / 16 + lane]) : gp[kTile / 16 + lane];
      }
    }
    if (KLF_SCAN_PRIO) __builtin_amdgcn_s_setprio(0);
    wave_lds_sync();

    // ---- any-tests over my 128 bytes: 8 chunks of 16 B, read rotated (chunk (v + lane/2)
    // mod 8) so that every 16-lane group of a ds_read_b128 covers all 64 banks once ----
    const uint32_t my0 = (uint32_t)lane * kLaneBytes;
    const int nvalid_s = tile_len - (int)my0;
    const int nvalid = nvalid_s <= 0 ? 0 : (nvalid_s >= kLaneBytes ? kLaneBytes : nvalid_s);
    // the byte of the anchor test: the fused literal's rarest byte, or the short needles'
    // anchor (loose short needles: bytes tested OR 0x20)
    const uint32_t pat = ANC ? a.pats.qf_anc_byte : a.lit_anchor_byte * 0x01010101u;
    const uint32_t afold = ANC ? a.pats.qf_anc_fold : 0u;
    auto or4 = [](const uint4& x, uint32_t f) { return make_uint4(x.x | f, x.y | f, x.z | f, x.w | f); };
    uint32_t nlc = 0, anc = 0;
    {
      const uint32_t rot = ((uint32_t)lane >> 1) & 7u;
      // KLF_ANY_BATCH reads in flight before the first test (8: one LDS round trip, not
      // eight; 4: two round trips, 16 fewer VGPRs)
#pragma unroll
      for (int v0 = 0; v0 < 8; v0 += KLF_ANY_BATCH) {
        uint4 xs[KLF_ANY_BATCH];
#pragma unroll
        for (int v = 0; v < KLF_ANY_BATCH; ++v)
          xs[v] = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * (((uint32_t)(v0 + v) + rot) & 7u));
#pragma unroll
        for (int v = 0; v < KLF_ANY_BATCH; ++v) {
          const uint32_t c = ((uint32_t)(v0 + v) + rot) & 7u;
          nlc |= any_eq16(xs[v], 0x0A0A0A0Au) ? (1u << c) : 0u;
          if (LIT && !ABL(2)) anc |= any_eq16(xs[v], pat) ? (1u << c) : 0u;
          if (ANC) anc |= any_eq16(afold ? or4(xs[v], afold) : xs[v], pat) ? (1u << c) : 0u;
        }
      }
      if (nvalid < kLaneBytes) {
        const uint32_t vm = (1u << ((nvalid + 15) >> 4)) - 1u;
        nlc &= vm;
        anc &= vm;
      }
    }
    if (ABL(64)) {  // timing build: staging + any-test only
      asm volatile("" ::"v"(nlc | anc) : "memory");
      continue;
    }
    auto clip = [&](uint32_t e, uint32_t c) -> uint32_t {  // bytes of chunk c past the tile's end
      const int nv = nvalid - 16 * (int)c;
      return nv >= 16 ? e : (nv <= 0 ? 0u : (e & ((1u << nv) - 1u)));
    };
    // ---- exact line-end positions in the chunks that hit: a 128-bit event mask ----
    uint32_t em[4] = {0u, 0u, 0u, 0u};
    for (uint32_t m = nlc; m; m &= m - 1u) {
      const uint32_t c = (uint32_t)__builtin_ctz(m);
      const uint4 x = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * c);
      const uint32_t e = clip(KLF_NL_MASK ? eq_mask16_nl(x) : eq_mask16(x, 0x0A0A0A0Au), c) << ((c & 1u) * 16u);
      const uint32_t q = c >> 1;
      em[0] |= q == 0 ? e : 0u;
      em[1] |= q == 1 ? e : 0u;
      em[2] |= q == 2 ? e : 0u;
      em[3] |= q == 3 ? e : 0u;
    }
    // the stream's end is an event too (it closes the last line); it starts no line
    uint32_t st[4] = {em[0], em[1], em[2], em[3]};
    if (last && nvalid > 0 && (int)my0 + nvalid == tile_len) {
      const uint32_t eb = (uint32_t)nvalid - 1u, q = eb >> 5, bit = 1u << (eb & 31u);
      bool nl_at_end = false;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((uint32_t)k == q) {
          nl_at_end = (em[k] & bit) != 0u;
          em[k] |= bit;
          st[k] &= ~bit;
        }
      if (!abl) a.segout[s].frag = nl_at_end ? 0 : 1;
    }
    const uint32_t cnt = (uint32_t)(__popc(em[0]) + __popc(em[1]) + __popc(em[2]) + __popc(em[3]));
    // (at most one event per lane -- lines of 128 B and more: a ballot's rank is the scan)
    const uint32_t incl = (KLF_SCAN_BALLOT && !__any(cnt > 1u))
                              ? cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(__ballot(cnt != 0u) >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)__ballot(cnt != 0u), 0u))
                              : wave_incl_scan_add(cnt, lane);
    const uint32_t agg = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // Local line k = the line after the tile's k-th event (k = 0: the line open at the
    // tile start).  Lines starting here: k in [k0, k1), slot j = k - k0.
    const uint32_t k0 = first ? 0 : 1;
    const uint32_t k1 = last ? agg : agg + 1;
    const uint32_t nlines = k1 > k0 ? k1 - k0 : 0;
    const bool dense = nlines > (uint32_t)kSlots;
    uint32_t pool_base = 0;
    if (dense) {
      uint32_t pb = 0;
      if (lane == 0 && !abl) {
        pb = atomicAdd(&a.counters[kCtrPool], (nlines + 31u) & ~31u);  // (whole 128-B lines: the waves' chunks stay aligned)
        if ((uint64_t)pb + nlines > a.pool_cap) atomicOr(err_flag, 1u);
      }
      pool_base = (uint32_t)__builtin_amdgcn_readlane((int)pb, 0);
    }
    const bool pool_ok = !dense || (uint64_t)pool_base + nlines <= a.pool_cap;
    uint32_t* const trec = a.slots + (size_t)tile * kRecStride;  // this tile's record region
    uint32_t* gslot = dense ? a.pool + pool_base : trec + kRecHead;

    // The per-tile work on the line list, instantiated for the LDS list (normal tiles) and
    // the global pool (dense tiles).
    uint32_t n_parsed = 0, n_since = 0, n_defer = 0, carry = 0, n_hit = 0;
    auto work = [&](uint32_t* list) __attribute__((always_inline)) {
      // ---- line starts -> list[j] = start offset in the tile ----
      if (first && lane == 0) list[0] = 0u;
      {
        uint32_t kk = incl - cnt;  // events before my bytes
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          for (uint32_t ev = em[q]; ev; ev &= ev - 1u) {
            const uint32_t b = (uint32_t)__builtin_ctz(ev);
            ++kk;
            if ((st[q] >> b) & 1u) list[kk - k0] = my0 + 32u * q + b + 1u;
          }
        }
      }
      if (dense) __threadfence_block();
      wave_lds_sync();
      // ---- timestamp + since: one line per lane ----
      for (uint32_t b0 = 0; b0 < nlines; b0 += 64) {
        const uint32_t j = b0 + (uint32_t)lane;
        if (j < nlines) {
          const uint32_t off = list[j];
          bool so = false, fast = false;
          if (ABL(1)) {
            fast = so = true;
          } else if (rel_lo + (int64_t)off + 31 <= seg_len) {
            fast = parse_fast(s_tile, off, a.since_dig, so);
          }
          if (FUSE && !fast) {  // the one-pass compaction decides every line here: Go time.Parse
            TsResult tr;
            uint32_t plen = 0;
            const bool ok = parse_line_prefix(GlobalBytes{segp, rel_lo + (int64_t)off, seg_len}, tr, plen);
            const bool so2 = ok && !time_before(tr.sec, tr.nsec, a.since_sec, a.since_nsec);
            list[j] = off | ((uint32_t)make_meta(ok, so2, ok ? plen : 0u) << 16);
            if (ok && plen >= kPlenEscape) atomicOr(&a.counters[kCtrFuseBad], 1u);  // (a prefix longer than the meta holds)
            n_parsed += ok ? 1u : 0u;
            n_since += so2 ? 1u : 0u;
          } else {
            list[j] = fast ? (off | ((uint32_t)make_meta(true, so, 31) << 16)) : (off | kSlotDefer);
            n_parsed += fast ? 1u : 0u;
            n_since += (fast && so) ? 1u : 0u;
            n_defer += fast ? 0u : 1u;
          }
        }
      }
      // ---- planned dense compaction: the tile's own kept runs and aggregate (FAgg above).
      // Two rounds of 64 lines, each ending in one buffer store of the runs (lanes without a
      // run, or past the record, dropped) and the plan in one more: a fixed store count per
      // tile (see the record stores below).  Tiles with more lines leave their runs to
      // k_tcopy (kRunsRecompute).
      if constexpr (MODE == kScanPlain && FUSE) {
        // ---- one-pass compaction: this tile's kept runs (the carried-in line's, then the
        // lines starting here), copied to the range's output at once (a dense tile voids
        // the pass) ----
        if (!dense) {
        wave_lds_sync();
        if (__any(n_defer != 0) && lane == 0) a.counters[kCtrFuseBad] = 1u;  // decided later: rerun
        const uint64_t tin = sd.base + (uint64_t)rel_lo;  // the tile's input = output position
        if (first) {  // a stream starts here: nothing carried in
          if (tile != range_t0) {
            fz_close();
            ++fz_ext;
          } else {
            fz_res_set = true;
          }
          fz_known = true;
          fz_sel = false;
          fz_crel = -1;
          fz_obase = fz_estart = tin;
          fz_part = 0;
        }
        const uint32_t span = nlines ? (list[0] & kSlotOff) : (uint32_t)tile_len;
        uint32_t clen = 0, csrc = 0;
        if (fz_known) {
          clen = f_carried(span, fz_sel, fz_crel);
          csrc = fz_crel > 0 ? (uint32_t)fz_crel : 0u;
        } else if (nlines) {  // the range's first line start: the bytes before it are k_fcarry's
          fz_res = fz_part + span;
          fz_res_set = true;
          fz_obase = fz_estart = tin + span;
        }
        uint32_t* s_frun = s_frun_all[wv];
        uint32_t nr = 0, dacc = 0, lsel = 0;
        int32_t lcrel = -1;
        for (uint32_t b0 = 0; b0 < nlines; b0 += 64) {
          const uint32_t j = b0 + (uint32_t)lane;
          uint32_t src = 0, len = 0;
          if (j < nlines) {
            const uint32_t v = list[j], off = v & kSlotOff, mt = v >> 16;
            const bool sel = !(v & kSlotDefer) && (mt & Meta::kParsed) && (mt & Meta::kSince);
            const uint32_t c = off + (mt >> 2);
            const uint32_t e = j + 1 < nlines ? (list[j + 1] & kSlotOff) : (uint32_t)tile_len;
            if (sel && e > c) { src = c; len = e - c; }
            if (j + 1 == nlines) { lsel = sel ? 1u : 0u; lcrel = f_sat((int32_t)c - tile_len); }
          }
          const uint32_t incl = wave_incl_scan_add(len, lane);
          const uint64_t bm = __ballot(len != 0);
          const uint32_t idx = nr + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
          if (len) s_frun[1 + idx] = src | ((clen + dacc + incl - len) << 16);
          nr += (uint32_t)__popcll(bm);
          dacc += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (clen && lane == 0) s_frun[0] = csrc;  // (output offset 0)
        const uint32_t kept = clen + dacc;
        if (kept) {
          if (fz_obase + kept + 16 > a.out_cap) {
            if (lane == 0) a.counters[kCtrFuseBad] = 1u;
          } else {
            copy_tile_runs(s_tile, clen ? s_frun : s_frun + 1, s_fmap_all[wv], nr + (clen ? 1u : 0u), kept, fz_obase,
                           a.out, lane);
          }
          fz_obase += kept;
        }
        if (nlines) {
          const uint32_t lastl = (nlines - 1u) & 63u;
          fz_sel = __builtin_amdgcn_readlane((int)lsel, (int)lastl) != 0;
          fz_crel = __builtin_amdgcn_readlane(lcrel, (int)lastl);
          fz_known = true;
        } else if (fz_known) {
          fz_crel = f_sat(fz_crel - tile_len);
        }
        fz_part += (uint64_t)tile_len;
        }
      } else if constexpr (MODE == kScanPlain) {
        if (a.plan_runs) {
          if (dense) __threadfence_block();
          wave_lds_sync();
          typedef uint32_t u32x4p __attribute__((ext_vector_type(4)));
          const bool fits = nlines <= 128u && !abl;
          const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
              a.truns + (size_t)tile * kRunSlots, 0, fits ? kRunSlots * 4 : 0, 0x00020000);
          uint32_t nr = 0, dacc = 0, ns = 0, lsel = 0;
          int32_t lcrel = -1;
          // one round of 64 lines: the run word and its store offset (dropped: none)
          auto round = [&](uint32_t b0, uint32_t& w, uint32_t& o) __attribute__((always_inline)) {
            const uint32_t j = b0 + (uint32_t)lane;
            uint32_t src = 0, len = 0;
            bool sel = false, starts = false;
            if (j < nlines) {
              const uint32_t v = list[j], off = v & kSlotOff, mt = v >> 16;
              sel = !(v & kSlotDefer) && (mt & Meta::kParsed) && (mt & Meta::kSince);
              const uint32_t c = off + (mt >> 2);
              const uint32_t e = j + 1 < nlines ? (list[j + 1] & kSlotOff) : (uint32_t)tile_len;
              if (sel && e > c) { src = c; len = e - c; }
              // (a line starting at the tile end -- the last byte is '\n' -- starts the next
              // tile, whose list does not hold it: counted here, in its stream)
              starts = off <= (uint32_t)tile_len;
              if (j + 1 == nlines) { lsel = sel ? 1u : 0u; lcrel = f_sat((int32_t)c - tile_len); }
            }
            const uint32_t incl = wave_incl_scan_add(len, lane);
            const uint64_t bm = __ballot(len != 0);
            const uint32_t idx = nr + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
            // slot 0 is the carried-in run's (k_cmove)
            w = src | ((dacc + incl - len) << 16);
            o = len ? 4u * (idx + 1u) : 0x7FFF0000u;
            nr += (uint32_t)__popcll(bm);
            dacc += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            ns += (uint32_t)__popcll(__ballot(sel && starts));
          };
          uint32_t w0 = 0, o0 = 0x7FFF0000u, w1 = 0, o1 = 0x7FFF0000u;
          round(0u, w0, o0);
          __builtin_amdgcn_raw_buffer_store_b32(w0, rr, o0, 0, 0);
          if (nlines > 64u) round(64u, w1, o1);  // (its store issues either way: a fixed count)
          __builtin_amdgcn_raw_buffer_store_b32(w1, rr, o1, 0, 0);
          for (uint32_t b0 = 128u; b0 < nlines; b0 += 64) {  // (no runs stored)
            uint32_t w, o;
            round(b0, w, o);
          }
          const uint32_t lastl = nlines ? ((nlines - 1u) & 63u) : 0u;
          const uint32_t psel = nlines ? (uint32_t)__builtin_amdgcn_readlane((int)lsel, (int)lastl) : 0u;
          const int32_t pcrel = nlines ? __builtin_amdgcn_readlane(lcrel, (int)lastl) : -1;
          const uint32_t span = nlines ? (list[0] & kSlotOff) : (uint32_t)tile_len;
          const uint32_t px = (dacc & 0x3FFFu) | ((span & 0x3FFFu) << 14) | ((nlines ? 1u : 0u) << 28) | (psel << 29);
          const uint32_t py = ((uint32_t)(uint16_t)(int16_t)pcrel) | (ns << 16);
          const uint32_t pz = (fits && nr + 1u <= (uint32_t)kRunSlots) ? nr : (uint32_t)kRunsRecompute;
          const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(a.trec + tile, 0, abl ? 0 : 16, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4p{px, py, pz, kPlanTag}, pr, lane ? 0x7FFF0000u : 0u, 0, 0);
        }
      }
      // number of listed line starts at or before tile offset pos
      auto starts_upto = [&](int32_t pos) __attribute__((always_inline)) -> int {
        int lo = 0, hi = pos < 0 ? 0 : (int)nlines;  // pos < 0: in the carried-in line
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((list[mid] & kSlotOff) <= (uint32_t)pos) lo = mid + 1; else hi = mid;
        }
        return lo;
      };
      // a final (literal) hit starting at tile offset pos -> its line's hit bit
      auto attribute = [&](int32_t pos) __attribute__((always_inline)) {
        const int lo = starts_upto(pos);
        if (lo > 0) {  // the line starts in this tile: deferred lines are searched by k_fixup
          const uint32_t v = list[lo - 1];
          const uint32_t mt = v >> 16;
          if (!(v & kSlotDefer) && (mt & Meta::kParsed) && (uint32_t)pos >= (v & kSlotOff) + (mt >> 2)) {
            atomicOr(&list[lo - 1], kSlotHit);
            ++n_hit;
          }
        } else {  // carried in from an earlier tile: k_scatter decides (furthest hit wins)
          const uint32_t c1 = (uint32_t)(pos + 1 + (int32_t)kCarryBias);  // pos >= -kCarryBias
          carry = carry > c1 ? carry : c1;
        }
      };
      // ---- fused single-literal grep ----
      // Anchor hits (the literal's rarest byte) name candidate starts p = anchor - ka.  A
      // tile owns the starts inside it: anchors whose start lies in the previous tile are
      // left to that tile, which scans its halo.
      if (LIT) {
        if (dense) __threadfence_block();
        wave_lds_sync();
        const uint32_t m = a.lit_len, ka = a.lit_anchor;
        auto check = [&](int32_t pos) __attribute__((always_inline)) {
          if (pos < 0 || pos >= tile_len || rel_lo + pos + (int64_t)m > seg_len) return;
          bool eq = true;
          if ((uint32_t)pos + m + 4 <= (uint32_t)(kTile + kHalo)) {  // 4 bytes per LDS read
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s_tile);
            const uint32_t sh = (uint32_t)pos & 3u;
            uint32_t wi = (uint32_t)pos >> 2;
            uint32_t prev = s32[wi];
            for (uint32_t k = 0; k < m && eq; k += 4) {
              const uint32_t nx = s32[++wi];
              const uint32_t got = __builtin_amdgcn_alignbyte(nx, prev, sh);
              prev = nx;
              const uint32_t nb = m - k < 4 ? m - k : 4;
              const uint32_t msk = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1);
              eq = ((got ^ s_lit[k >> 2]) & msk) == 0;
            }
          } else {
            const uint8_t* lit = reinterpret_cast<const uint8_t*>(s_lit);
            for (uint32_t k = 0; k < m && eq; ++k) {
              const uint32_t o = (uint32_t)pos + k;
              const uint8_t c = o < (uint32_t)(kTile + kHalo) ? s_tile[o] : segp[rel_lo + o];
              eq = c == lit[k];
            }
          }
          if (!eq) return;
          attribute(pos);
        };
        for (uint32_t cm = anc; cm; cm &= cm - 1u) {
          const uint32_t c = (uint32_t)__builtin_ctz(cm);
          const uint4 x = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * c);
          for (uint32_t e = clip(eq_mask16(x, pat), c); e; e &= e - 1u)
            check((int32_t)(my0 + 16u * c + (uint32_t)__builtin_ctz(e)) - (int32_t)ka);
        }
        if (lane == 63 && ka > 0 && !last) {  // halo anchors -> starts in this tile's tail
          for (uint32_t jj = 0; jj < ka; ++jj) {
            const int64_t q = rel_lo + kTile + jj;
            if (q >= seg_len) break;
            const uint8_t c = jj < (uint32_t)kHalo ? s_tile[kTile + jj] : segp[q];
            if (c == a.lit_anchor_byte) check((int32_t)(kTile + jj) - (int32_t)ka);
          }
        }
        carry = wave_max(carry);
      }
      if (dense) __threadfence_block();
      wave_lds_sync();
    };
    if (ABL(128)) {  // timing build: no line list / parse / literal
    } else if (!dense) {
      work(s_list);
    } else if (pool_ok && !abl) {
      if (FUSE && lane == 0) a.counters[kCtrFuseBad] = 1u;  // (a dense tile: the two-pass rerun)
      work(gslot);
    }

    uint32_t tile_hits = 0;
    bool hinl = false;  // GEN: the tile's hits inline (kTsHitInline)
    uint32_t hit2 = 0;
    // ---- general sets: fused q-gram prefilter ----
    // Samples p = 0 mod QS of the tile (each needle's chosen window is q + QS - 1 long, so
    // every occurrence spans exactly one sample whose gram lies in the window) probe the
    // LDS bitmap (one word, two bits per gram).  The few bitmap hits are appended to a global list
    // (one atomic per wave and tile) and verified by k_verify once the line index exists:
    // the scan keeps no verification code, and the latency-bound bucket walks run with
    // the whole GPU's parallelism.
    if (GEN) {
      const uint32_t fold = a.pats.qf_fold;
      const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s_tile);
      // bit 0 of the result: gram g has all K bits of its bitmap word set (qf_f / qf_hash /
      // qf_bits): the multiplies, the word read, and the bit positions as byte / word selects
      // or low bits of the products (SDWA operands of the shifts)
      struct Probe {
        uint32_t h, p, m, a;  // a: byte offset of the bitmap word in LDS (qf_bucket * 4)
      };
      constexpr bool kMidIdx = QQ == 3 && QK == 2;  // word from h bits 18..29 (qf_bucket)
      constexpr bool K3 = QK == 3 || QK == (int)kQfTwoLevel;  // three bits per gram
      constexpr bool TWO = QK == (int)kQfTwoLevel;            // pair stage first (stride 4 only)
      static_assert(!TWO || QS == 4, "the two-level probe runs at stride 4");
      // (the 24-bit multiplies ignore bits 24..31 of f: no mask)
      auto probe = [&](uint32_t g) __attribute__((always_inline)) -> Probe {
        const uint32_t gf = g | fold;
        const uint32_t f = K3 ? gf ^ bfe_u32(gf, 13, 11) : gf;
        Probe r;
        r.h = mul_u24(f, 0x9E3779u);
        if (QQ == 4) r.h = mad_u24(gf >> 8, 0x7F4A7Du, r.h);  // + bytes 1..3 * C2
        r.p = K3 ? mul_hi_u24(f, 0xC2B2AEu) : 0u;  // K = 2: both bits from h (qf_bits)
        r.m = K3 ? mul_u24(f, 0x5BD1E9u) : 0u;
        r.a = TWO ? (((r.h >> 21) << 2) + kQfPairWords * 4u)  // the Bloom half, 11-bit word
              : kMidIdx ? ((r.h >> 16) & ((kQfWords - 1u) << 2)) : ((r.h >> (32 - kQfBucketBits)) << 2);
        return r;
      };
      auto word = [&](const Probe& r) __attribute__((always_inline)) -> uint32_t {
        return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(s_qf) + r.a);
      };
      auto test = [&](uint32_t w, const Probe& r) __attribute__((always_inline)) -> uint32_t {
        uint32_t t = K3 ? (w >> ((r.m >> 24) & 31u)) & (w >> (r.p & 31u))
                        : shr_byte1(w, r.h) & (w >> ((r.h >> 16) & 31u));
        if (K3) t &= w >> ((r.h >> 16) & 31u);
        if (TWO) t &= shr_byte1(w, r.m);  // the fourth bit: m bits 8..12 (qf_bits)
        return t;
      };
      auto hbits = [&](uint32_t g) __attribute__((always_inline)) -> uint32_t {
        const Probe r = probe(g);
        return test(word(r), r);
      };
      // the samples of chunk c (16 B) -> their grams, in order (QS = 8: dwords 0 and 2;
      // QS = 6: the grid's bytes 0, 6 and 12, qf_sampled)
      auto chunk_grams = [&](uint32_t c, auto&& f) __attribute__((always_inline)) {
        const uint32_t o0 = my0 + 16u * c;
        const uint4 x = *reinterpret_cast<const uint4*>(s_tile + o0);
        if constexpr (QS == 6) {
          f(x.x, 0);
          f(__builtin_amdgcn_alignbyte(x.z, x.y, 2u), 6);
          f(x.w, 12);
          return;
        }
        const uint32_t w4 = QS < 4 ? s32[(o0 >> 2) + 4] : 0u;
        const uint32_t w[5] = {x.x, x.y, x.z, x.w, w4};
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int o = 0; o < 4; o += (QS < 4 ? QS : 4)) {
            if ((4 * d + o) % QS != 0) continue;
            f(o == 0 ? w[d] : __builtin_amdgcn_alignbyte(w[d + 1], w[d], o), 4 * d + o);
          }
      };
      // fast pass: one OR-accumulated bit per chunk (no positions); most tiles stop here
      uint32_t chit = 0;
      const uint32_t rot = ((uint32_t)lane >> 1) & 7u;
      uint32_t hq0 = 0, hq1 = 0, hq2 = 0, hq3 = 0;
      uint32_t xh = 0xFFFFFFFFu;  // a hit at this tile offset (the compacted stage 2), beside hq
      if (TWO) {
        // stage 1: the exact set of the probed grams' low two bytes (pair words [0, 2048)):
        // sv bit i = the sample at my0 + 4i passes (each chunk's four dwords, two chunks per
        // step with their eight word reads in flight).  The raw bytes probe: for a folded set
        // the host lists every case variant of a pair (p with p | 0x2020 in the set), so the
        // stage has no fold OR and the word's bit is the sample's own low five bits.  Step v
        // puts chunk (v + rot) & 7 at bits 4v.. (constant shifts); one rotate at the end
        uint32_t sv = 0;
#pragma unroll
        for (int v = 0; v < (ABL(4) ? 0 : 8); v += 2) {
          const uint32_t ca = ((uint32_t)v + rot) & 7u, cb = ((uint32_t)v + 1u + rot) & 7u;
          const uint4 xa = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * ca);
          const uint4 xb = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * cb);
          const uint32_t g[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
          uint32_t w[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            w[k] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(s_qf) +
                                                      ((KLF_PAIR_SWZ ? bfe_u32(g[k], 5, 11) ^ (g[k] & 31u) : bfe_u32(g[k], 5, 11)) << 2));
#pragma unroll
          for (int k = 0; k < 8; ++k)
            sv |= __builtin_amdgcn_ubfe(w[k], g[k], 1u) << (4 * v + k);  // bit g mod 32 (v_bfe_u32 reads offset[4:0])
        }
        sv = __builtin_amdgcn_alignbit(sv, sv, 32u - 4u * rot);  // rotate left by 4 rot (shift mod 32): chunk c at bits 4c..
        // samples at or past the tile's end (4i >= nvalid) do not count
        sv &= nvalid >= kLaneBytes ? ~0u : ((1u << ((uint32_t)(nvalid + 3) >> 2)) - 1u);
        // stage 2: the survivors' 3-bit probe into the Bloom half.  The ~1.4 % survivors
        // (~30 per tile) are compacted over the wave first, so that one round of 64 lanes
        // probes them all (each lane's own walk took as many dependent LDS round trips as
        // the busiest lane had survivors); a hit's tile offset goes to xh.  Past 64
        // survivors each lane walks its own: a hit's byte position 4i -> its 32-B group
        // q = i / 8, bit 4i mod 32
        if (ABL(16)) sv = 0u;  // (KLF_ABL 16: no stage 2)
        const uint32_t scnt = (uint32_t)__popc(sv);
        const uint32_t sincl = wave_incl_scan_add(scnt, lane);
        const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane((int)sincl, 63);
        // (the list: the last 32 words of the wave's slot list, free unless more than
        // kSlotStride - 32 lines start in the tile; a 512-B LDS array of its own cost a third
        // of the workgroups: 7.7 -> 10.4 ms)
        if (stot <= 64u && nlines <= (uint32_t)kSlotStride - 32u) {
          if (stot) {
            uint16_t* sl = reinterpret_cast<uint16_t*>(s_list + kSlotStride - 32);
            uint32_t k = sincl - scnt;
            for (uint32_t m = sv; m; m &= m - 1u) sl[k++] = (uint16_t)(((uint32_t)lane << 5) | (uint32_t)__builtin_ctz(m));
            wave_lds_sync();
            if ((uint32_t)lane < stot) {
              const uint32_t e = sl[lane];  // sample e & 31 of lane e >> 5: tile offset 4 e
              if (hbits(s32[e]) & 1u) xh = 4u * e;
            }
            wave_lds_sync();  // (the next tile rewrites the list)
          }
        } else {
          for (uint32_t m = sv; m; m &= m - 1u) {
            const uint32_t i = (uint32_t)__builtin_ctz(m);
            if (hbits(s32[(my0 >> 2) + i]) & 1u) {
              const uint32_t q = i >> 3, b = 1u << ((4u * i) & 31u);
              hq0 |= q == 0 ? b : 0u;
              hq1 |= q == 1 ? b : 0u;
              hq2 |= q == 2 ? b : 0u;
              hq3 |= q == 3 ? b : 0u;
            }
          }
        }
      } else if (QS == 4 || QS == 6) {
        // stride 4: a chunk's samples are its four dwords (the grid: bytes 0, 6, 12).  Two
        // chunks per step, their bitmap reads issued before the first test (one LDS round
        // trip per step, not one per probe)
        constexpr int kPer = QS == 4 ? 4 : 3;
#pragma unroll
        for (int v = 0; v < (ABL(4) ? 0 : 8); v += 2) {
          const uint32_t ca = ((uint32_t)v + rot) & 7u, cb = ((uint32_t)v + 1u + rot) & 7u;
          const uint4 xa = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * ca);
          const uint4 xb = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * cb);
          uint32_t g[2 * kPer];
          if constexpr (QS == 4) {
            g[0] = xa.x; g[1] = xa.y; g[2] = xa.z; g[3] = xa.w;
            g[4] = xb.x; g[5] = xb.y; g[6] = xb.z; g[7] = xb.w;
          } else {
            g[0] = xa.x; g[1] = __builtin_amdgcn_alignbyte(xa.z, xa.y, 2u); g[2] = xa.w;
            g[3] = xb.x; g[4] = __builtin_amdgcn_alignbyte(xb.z, xb.y, 2u); g[5] = xb.w;
          }
          Probe r[2 * kPer];
          uint32_t w[2 * kPer];
#pragma unroll
          for (int k = 0; k < 2 * kPer; ++k) r[k] = probe(g[k]);
#pragma unroll
          for (int k = 0; k < 2 * kPer; ++k) w[k] = word(r[k]);
          uint32_t acc_a = 0, acc_b = 0;
#pragma unroll
          for (int k = 0; k < 2 * kPer; ++k) {
            const uint32_t t = test(w[k], r[k]);
            if (k < kPer) acc_a |= t; else acc_b |= t;
          }
          chit |= ((acc_a & 1u) << ca) | ((acc_b & 1u) << cb);
        }
      } else {
#pragma unroll
        for (int v = 0; v < (ABL(4) ? 0 : 8); ++v) {
          const uint32_t c = ((uint32_t)v + rot) & 7u;
          uint32_t acc = 0;
          chunk_grams(c, [&](uint32_t g, int) __attribute__((always_inline)) { acc |= hbits(g); });
          chit |= (acc & 1u) << c;
        }
      }
      // chunks with a possible hit: the sample positions (past the tile's end clipped)
      if (!TWO && __any(chit != 0)) {
        for (uint32_t m = chit; m; m &= m - 1u) {
          const uint32_t c = (uint32_t)__builtin_ctz(m);
          uint32_t hm = 0;
          chunk_grams(c, [&](uint32_t g, int pos) __attribute__((always_inline)) { hm |= (hbits(g) & 1u) << pos; });
          hm = clip(hm, c) << ((c & 1u) * 16u);
          const uint32_t q = c >> 1;
          hq0 |= q == 0 ? hm : 0u;
          hq1 |= q == 1 ? hm : 0u;
          hq2 |= q == 2 ? hm : 0u;
          hq3 |= q == 3 ? hm : 0u;
        }
      }
      // short needles: every anchor byte whose dword passes a pre-check is a hit (its
      // bucket entries name the anchor's offset in the needle); anchors are rare
      if (ANC && __any(anc != 0)) {
        const uint32_t npre = a.pats.qf_anc_n;
        for (uint32_t cm = anc; cm; cm &= cm - 1u) {
          const uint32_t c = (uint32_t)__builtin_ctz(cm);
          const uint4 x = *reinterpret_cast<const uint4*>(s_tile + my0 + 16u * c);
          uint32_t am = 0;
          for (uint32_t e = clip(eq_mask16(afold ? or4(x, afold) : x, pat), c); e; e &= e - 1u) {
            const uint32_t pos = my0 + 16u * c + (uint32_t)__builtin_ctz(e);
            const uint32_t w = __builtin_amdgcn_alignbyte(s32[(pos >> 2) + 1], s32[pos >> 2], pos & 3u) | fold;
            bool ok = false;
            for (uint32_t j = 0; j < npre; ++j) ok |= (w & a.pats.qf_anc_pre[2 * j + 1]) == a.pats.qf_anc_pre[2 * j];
            am |= ok ? 1u << (pos & 15u) : 0u;
          }
          am <<= (c & 1u) * 16u;
          const uint32_t q = c >> 1;
          hq0 |= q == 0 ? am : 0u;
          hq1 |= q == 1 ? am : 0u;
          hq2 |= q == 2 ? am : 0u;
          hq3 |= q == 3 ? am : 0u;
        }
      }
      if (ABL(8)) {  // timing build: probes only
        asm volatile("" ::"v"(hq0 | hq1 | hq2 | hq3 | xh));
        hq0 = hq1 = hq2 = hq3 = 0;
        xh = 0xFFFFFFFFu;
      }
      // (the count only where some lane has a hit: ~1.5 % of C5's tiles)
      if (__any((hq0 | hq1 | hq2 | hq3) != 0u || xh != 0xFFFFFFFFu) && (!abl || (KLF_ABL & (65536 | 131072)))) {
        const uint32_t nh = (uint32_t)(__popc(hq0) + __popc(hq1) + __popc(hq2) + __popc(hq3)) + (xh != 0xFFFFFFFFu ? 1u : 0u);
        // tile-owned slots (u16 tile offsets, no atomics); only a tile with more than
        // kHitSlots hits spills the rest to the global list
        const uint32_t ih = wave_incl_scan_add(nh, lane);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)ih, 63);
        uint32_t ob = 0;
        if (tot > kHitSlots) {
          if (lane == 63) ob = atomicAdd(&a.counters[kCtrHits], tot - kHitSlots);
          ob = (uint32_t)__builtin_amdgcn_readlane((int)ob, 63);
        }
        uint16_t* hs = a.hslots + (size_t)tile * kHitSlots;
        // one or two hits of a tile that keeps no line slot in its TileStat go to its
        // pool_base halves (KLF_HIT_INLINE): no 2-B stores into a half-written 64-B slot line
        // (C4: ~1.4 M tiles with hits per step)
        hinl = KLF_HIT_INLINE && tot <= 2u && !dense && nlines != 1u;
        uint16_t* hd = hinl ? reinterpret_cast<uint16_t*>(s_h2[GEN ? wv : 0]) : hs;
        uint32_t k = ih - nh;
        if (xh != 0xFFFFFFFFu) {
          if (k < kHitSlots) {
            hd[k] = (uint16_t)xh;
          } else if ((uint64_t)ob + (k - kHitSlots) < a.qhits_cap) {
            a.qhits[ob + (k - kHitSlots)] = sd.base + (uint64_t)rel_lo + xh;
          } else {
            atomicOr(&a.counters[kCtrHitsOver], 1u);
          }
          ++k;
        }
        const uint32_t hq[4] = {hq0, hq1, hq2, hq3};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          for (uint32_t m = hq[q]; m; m &= m - 1u, ++k) {
            const uint32_t off = my0 + 32u * q + (uint32_t)__builtin_ctz(m);
            if (k < kHitSlots) {
              hd[k] = (uint16_t)off;
            } else if ((uint64_t)ob + (k - kHitSlots) < a.qhits_cap) {
              a.qhits[ob + (k - kHitSlots)] = sd.base + (uint64_t)rel_lo + off;
            } else {
              atomicOr(&a.counters[kCtrHitsOver], 1u);
            }
          }
        tile_hits = tot < kHitSlots ? tot : kHitSlots;
        if (hinl) {
          wave_lds_sync();
          const uint32_t h2 = s_h2[GEN ? wv : 0][0];  // (hit 0 in the low half, hit 1 in the high)
          hit2 = tot > 1u ? h2 : (h2 & 0xFFFFu);
        }
      }
    }

    // ---- per-tile record: the first 64 slots and the TileStat, two store instructions
    // on every path (see the loop entry) ----
#if KLF_SCAN_PACKSUM
    // one reduction for both counts (each <= 8,193 per tile: 16 bits apiece, no carry from
    // the low half) and a ballot for the deferred lines, whose count nothing reads
    // (at most one line per lane -- 64 lines or fewer: two ballots' popcounts)
    const uint32_t pq = (KLF_SCAN_BALLOT && nlines <= 64u)
                            ? (uint32_t)__popcll(__ballot(n_parsed != 0u)) | ((uint32_t)__popcll(__ballot(n_since != 0u)) << 16)
                            : wave_sum(n_parsed | (n_since << 16));
    const uint32_t pp = pq & 0xFFFFu, qq = pq >> 16;
    const uint32_t dd = __any(n_defer != 0) ? 1u : 0u;
#elif KLF_SCAN_SUMSKIP  // A/B: no reductions on tiles where no line starts (wave-uniform)
    uint32_t pp = 0, qq = 0, dd = 0;
    if (nlines) { pp = wave_sum(n_parsed); qq = wave_sum(n_since); dd = wave_sum(n_defer); }
#else
    const uint32_t pp = wave_sum(n_parsed), qq = wave_sum(n_since), dd = wave_sum(n_defer);
#endif
    any_defer |= dd != 0;
    {
      // A tile's line slots: one line start -> the slot in its TileStat (kTsInline); two or
      // more -> appended to the wave's own chunk of the pool (RunArgs::wave_pool, round 6: a
      // sequential stream of whole lines per wave, where the 1,152-B-stride record regions
      // took a 128-B store per tile however few its slots), 16-B aligned, TileStat bit 0 and
      // pool_base as for a dense tile (whose slots the line list wrote to the pool itself).
      // 16 B per lane: narrower per-lane stores cost several times more per byte.
      const bool inl = KLF_TS_INLINE && !dense && nlines == 1u;
      const bool pooled = a.wave_pool && !dense && nlines >= 2u;
      // (timing builds: KLF_ABL 65536 drops only the slot stores, 131072 only the TileStat stores)
      const bool no_slots = (abl && !(KLF_ABL & (65536 | 131072))) || ABL(65536);
      uint32_t pb = dense ? pool_base : 0u, nunits = 0;
      uint32_t* sdst = trec;  // the record region (a.wave_pool == 0: unit 0 the TileStat copy)
      if (pooled && !no_slots) {
        // 16-B granules; a run of 16 slots or more starts on a 128-B line and fills whole
        // lines (a run straddling lines left partly written lines behind: C3 +1.6 %, r6f)
        const bool whole = nlines > 12u;
        const uint32_t need = whole ? (nlines + 31u) & ~31u : (nlines + 3u) & ~3u;
        if (whole) wp_cur = (wp_cur + 31u) & ~31u;  // (chunks start 128-B aligned: see below)
        if (wp_cur + need > wp_end) {  // (wave-uniform) a new chunk
          const uint32_t ch = need > a.pool_chunk ? need : a.pool_chunk;
          uint32_t b = 0;
          if (lane == 0) b = atomicAdd(&a.counters[kCtrPool], ch);
          b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
          wp_cur = b;
          wp_end = (uint64_t)b + ch <= a.pool_cap ? b + ch : b;  // (past the pool: no room, the run is redone)
          if (wp_end == b && lane == 0) atomicOr(err_flag, 1u);
        }
        if (wp_cur + need <= wp_end) {
          pb = wp_cur;
          wp_cur += need;
          nunits = need / 4u;
          sdst = a.pool + pb;
        }
      } else if (!a.wave_pool && !no_slots && !dense && nlines > 1u - (KLF_TS_INLINE ? 0u : 1u)) {
        nunits = ((kRecHead + nlines + 31u) & ~31u) / 4u;  // the record region (whole 128-B lines)
      }
      const uint32_t w0 = agg, w1 = (dense || pooled) ? pb : (inl ? s_list[0] : (hinl ? hit2 : 0u));
      const uint32_t w2 = (pp & 0xFFFFu) | (qq << 16);
      const bool hh = LIT && __any(n_hit != 0);  // some line starting here holds the literal
      const uint32_t w3 = (((dense || (pooled && nunits)) ? 1u : 0u) | (carry ? 2u : 0u) | (dd ? 4u : 0u) | (hh ? 8u : 0u) |
                           (inl ? kTsInline : 0u) | (hinl ? kTsHitInline : 0u)) |
                          ((uint32_t)(uint16_t)(GEN ? tile_hits : carry) << 16);  // GEN: hit slots used
      const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(sdst, 0, (int)(nunits * 16u), 0x00020000);
      typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
      const uint32_t ushift = a.wave_pool ? 0u : 1u;  // (the record region: unit 0 the TileStat)
      for (uint32_t u = (uint32_t)lane; u < (nunits > 64u ? 128u : 64u); u += 64) {  // one or two stores
        const uint32_t us = u - ushift;  // (u = 0 of a record: -1)
        const uint32_t li = u < ushift ? 0u : (4u * us < (uint32_t)kSlotStride - 4u ? 4u * us : (uint32_t)kSlotStride - 4u);
        const uint4 sl = *reinterpret_cast<const uint4*>(s_list + li);
        const u32x4v v = u >= ushift ? u32x4v{sl.x, sl.y, sl.z, sl.w} : u32x4v{w0, w1, w2, w3};
        __builtin_amdgcn_raw_buffer_store_b128(v, rrs, 16u * u, 0, 0);
      }
      // the group's TileStats, one 128-B store at its last tile (lanes past it dropped)
      const uint32_t gk = tile % kScanGroup, g0 = tile - gk;
      if (GEN) {
        if ((uint32_t)lane == gk) stv = make_uint4(w0, w1, w2, w3);
      } else {
        if (lane == 0) s_gstat[wv][gk] = make_uint4(w0, w1, w2, w3);
        wave_lds_sync();
      }
      const bool gend = gk == kScanGroup - 1 || tile + 1 >= a.ntiles;
      const uint32_t ng = a.ntiles - g0 < kScanGroup ? a.ntiles - g0 : kScanGroup;
      const __amdgpu_buffer_rsrc_t srs =
          __builtin_amdgcn_make_buffer_rsrc(a.tstat + g0, 0, (gend && (!abl || (KLF_ABL & 65536))) && !ABL(131072) ? (int)(16u * ng) : 0, 0x00020000);
      const uint4 gs = GEN ? stv : s_gstat[GEN ? 0 : wv][lane & (kScanGroup - 1)];
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{gs.x, gs.y, gs.z, gs.w}, srs, 16u * (uint32_t)lane, 0, 0);
    }
    asm volatile("" ::: "memory");  // the next stage overwrites the LDS region read above
  }
  if (any_defer && lane == 0 && !abl) a.counters[kCtrDefer] = 1u;
  if (FUSE && range_t0 < tile_end) {  // the range's last extent and the state it leaves
    fz_close();
    if (lane == 0) {
      uint64_t* ri = a.fuse_rinfo + 4 * (size_t)gw;
      ri[0] = fz_res;
      ri[1] = (fz_known ? 1u : 0u) | (fz_sel ? 2u : 0u);
      ri[2] = (uint64_t)(int64_t)fz_crel;
      ri[3] = fz_part;
    }
  }
  if (KLF_ABL != 0 && lane == 0) atomicAdd(&g_abl_waves, 1u);
#undef ABL
}

// ---- K1e: general parse of the deferred lines (non-canonical timestamp shapes) ---------
// One wave per tile that reported deferred lines: Go time.Parse(RFC3339Nano) restated
// (klf_ts.hpp) from global memory, since, and — with a fused literal — bytes.Contains over
// the whole content of the line (its hits were not attributed by the scan).  The slot
// keeps its defer bit (k_scatter then leaves carried hits of the line alone) and the
// tile's parsed / since_ok counts are corrected before the tile-base scan.
__device__ bool contains_bytes(const uint8_t* p, int64_t n, const uint8_t* lit, uint32_t m) {
  if ((int64_t)m > n) return false;
  for (int64_t i = 0; i + (int64_t)m <= n; ++i) {
    if (p[i] != lit[0]) continue;
    uint32_t k = 1;
    while (k < m && p[i + k] == lit[k]) ++k;
    if (k == m) return true;
  }
  return false;
}

__device__ bool ac_match(const DevPatterns& P, const uint8_t* p, int64_t n);
__device__ bool rx_match(const DevPatterns& P, uint32_t r, const uint8_t* p, int64_t n);
// the whole general set on one (non-empty) content: AC over the literals, every regex
__device__ bool general_match(const DevPatterns& P, const uint8_t* p, int64_t n) {
  if (P.ac_states && ac_match(P, p, n)) return true;
  for (uint32_t r = 0; r < P.rx_count; ++r)
    if (rx_match(P, r, p, n)) return true;
  return false;
}

// ---- per-pattern counts (KLF_FILTER_PATTERN_COUNTS) -------------------------------------
// Line l of segment s matches compiled pattern cid: count it once.  The (line, cid) pairs
// go through an open-addressing set (key + 1, 0 = empty; atomicCAS), so the several
// occurrences the prefilter verifies in one line, and the deferred lines the fix-up
// re-matches, add one line each.
__device__ void count_pair(const RunArgs& a, uint64_t l, uint32_t s, uint32_t cid) {
  const uint64_t key = ((l << 20) | cid) + 1;
  const uint32_t mask = (1u << a.pairs_log2) - 1u;
  uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & mask;
  for (int probe = 0; probe < 128; ++probe) {
    const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(&a.pairs[h]), 0ull, key);
    if (prev == 0ull) {
      atomicAdd(&a.pcount[(size_t)s * a.pats.n_cids + cid], 1u);
      return;
    }
    if (prev == key) return;
    h = (h + 1u) & mask;
  }
  atomicAdd(&a.counters[kCtrPairsOver], 1u);  // failed inserts: the host re-runs with a set sized from them
}

// Every pattern of the set on one content (deferred lines, the fallback matcher): counts
// each matching pattern of line l; true when one matches.  AC reports every literal that
// ends at each position (dictionary links), every regex runs on its own.
__device__ bool general_count(const RunArgs& a, const uint8_t* p, int64_t n, uint64_t l, uint32_t s) {
  const DevPatterns& P = a.pats;
  bool any = false;
  if (P.ac_states) {
    uint32_t st = 0;
    for (int64_t i = 0; i < n; ++i) {
      st = P.ac_next[(size_t)st * P.ac_classes + P.ac_class[p[i]]];
      if (!P.ac_accept[st]) continue;
      any = true;
      for (uint32_t t = P.ac_out[st] >= 0 ? st : P.ac_dict[st]; t; t = P.ac_dict[t]) count_pair(a, l, s, (uint32_t)P.ac_out[t]);
    }
  }
  for (uint32_t r = 0; r < P.rx_count; ++r)
    if (rx_match(P, r, p, n)) {
      any = true;
      count_pair(a, l, s, P.n_lits + r);
    }
  return any;
}

// A tile's line slots: dense tiles in the pool, a tile where exactly one line starts in its
// TileStat's pool_base word (kTsInline, round 6: no 128-B record store for it; C5's most
// common tile), every other tile in its record region.
__device__ __forceinline__ uint32_t* slot_list(const RunArgs& a, const TileStat& ts, uint32_t tile) {
  // (a.slots is null with the wave pool: a tile left with neither belongs to a run whose
  // pool overflowed, which is redone -- its readers get in-bounds garbage)
  return (ts.flags & 1u) ? a.pool + ts.pool_base
         : (ts.flags & kTsInline) ? reinterpret_cast<uint32_t*>(a.tstat + tile) + 1
         : a.slots ? a.slots + (size_t)tile * kRecStride + kRecHead : a.pool;
}
// slot j of a tile whose TileStat is at hand: an inline slot without a second load
__device__ __forceinline__ uint32_t slot_at(const RunArgs& a, const TileStat& ts, uint32_t tile, uint32_t j) {
  return (ts.flags & kTsInline) ? ts.pool_base : slot_list(a, ts, tile)[j];
}

// One wave: the deferred lines of `tile` (TileStat ts) through the general parse; their
// slots are rewritten in place and the parsed / since_ok counts the tile gains are
// returned (wave-uniform).
__device__ void fix_tile(const RunArgs& a, uint32_t tile, const TileStat& ts, int lane, uint32_t& add_p,
                         uint32_t& add_q) {
  const uint32_t s = a.tile_seg[tile];
  const SegDesc sd = a.segs[s];
  const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
  const int64_t seg_len = (int64_t)sd.len;
  const bool first = rel_lo == 0, last = rel_lo + kTile >= seg_len;
  const uint32_t k0 = first ? 0 : 1, k1 = last ? ts.events : ts.events + 1;
  const uint32_t nlines = k1 > k0 ? k1 - k0 : 0;
  uint32_t* list = slot_list(a, ts, tile);
  const uint8_t* segp = a.bytes + sd.base;
  uint32_t dp = 0, dq = 0;
  for (uint32_t j = lane; j < nlines; j += 64) {
    const uint32_t sl = list[j];
    if (!(sl & kSlotDefer)) continue;
    const uint32_t off = sl & kSlotOff;
    const int64_t p0 = rel_lo + off;
    TsResult r;
    uint32_t plen = 0;
    const bool ok = parse_line_prefix(GlobalBytes{segp, p0, seg_len}, r, plen);
    const bool so = ok && !time_before(r.sec, r.nsec, a.since_sec, a.since_nsec);
    uint32_t hit = 0;
    const bool gen = a.grep_mode == kGrepGeneral && a.pats.qf_on;  // the scan attributed none
    if ((a.grep_mode == kGrepLit1 || gen) && ok) {
      const int64_t cs = p0 + plen;
      int64_t ce;
      if (j + 1 < nlines) {
        ce = rel_lo + (int64_t)(list[j + 1] & kSlotOff) - 1;  // the line's '\n'
      } else {
        ce = cs;
        while (ce < seg_len && segp[ce] != '\n') ++ce;
      }
      if (ce > cs && !gen && contains_bytes(segp + cs, ce - cs, a.lit, a.lit_len)) hit = kSlotHit;
      if (ce > cs && gen && general_match(a.pats, segp + cs, ce - cs)) hit = kSlotHit;
    }
    list[j] = off | kSlotDefer | hit | ((uint32_t)make_meta(ok, so, plen) << 16);
    dp += ok ? 1u : 0u;
    dq += so ? 1u : 0u;
  }
  add_p = wave_sum(dp);
  add_q = wave_sum(dq);
}

// ---- K1b/K1c: tile line bases (exclusive scan of TileStat.events) -------------------
// Two passes over the compact TileStats (the scan writes them 8 tiles to a 128-B line), a
// thread owning R consecutive tiles (block: 256 R tiles):
//   k_tindex<R, 0>  the deferred lines' general parse (fix_tile; it corrects the tiles'
//                   counts in place), then each block's totals;
//   k_tindex<R, 1>  the earlier blocks' totals + the block scan of events / parsed /
//                   since_ok / prefilter hits -> tile line bases, the streams' line and
//                   count ranges (prefix differences at their first and last tile: no
//                   same-address atomics), the flattened hit list, and zeroed match-bitmap
//                   words whose first line falls in the block's line range (the bitmap is
//                   only ever OR-ed into by the kernels after this one).

// TileStat.carry_off is the tile's hit-slot count with the q-gram prefilter (GEN scan)
__device__ __forceinline__ uint32_t tile_hits(const RunArgs& a, const TileStat& ts) {
  return (a.grep_mode == kGrepGeneral && a.pats.qf_on) ? ts.carry_off : 0u;
}

#ifndef KLF_FLAT_BATCH
#define KLF_FLAT_BATCH 1  // k_tindex<R, 1>: hits flattened per thread at once (4: C4 71.6 -> 85.5 us, its
#endif                    // VGPRs past 128 cost the kernel a wave per SIMD, r6v)
#ifndef KLF_TINDEX_WAVES
#define KLF_TINDEX_WAVES 4  // k_tindex: min waves per SIMD (<16, 1>: 130 -> 128 VGPRs, C4 75 -> 63 us, C5 38 -> 30, r6y)
#endif
template <int R, int PASS>
__global__ __launch_bounds__(256, KLF_TINDEX_WAVES) void k_tindex(RunArgs a) {
  __shared__ uint32_t s_wt[4][4];
  __shared__ uint64_t s_w64[4][4];
  __shared__ uint64_t s_base[4];
  __shared__ uint32_t s_ndef;
  __shared__ uint32_t s_def[PASS == 0 ? 256 : 1];
  __shared__ uint32_t s_fix[PASS == 0 ? 256 : 1][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t bid = blockIdx.x;
  const uint32_t tb = bid * (256u * R) + (uint32_t)t * R;  // my first tile
  TileStat ts[R];
  uint32_t sg[R];
  {  // whole 16-B loads through buffer descriptors (tiles past the end read as zero): plain
     // loads get narrowed to the fields used, four instructions per record that each touch
     // 64 scattered lines
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(a.tstat, 0, (int)(a.ntiles * 16u), 0x00020000);
    // (tile_seg has room for whole 16-B groups past its end; entries there are never used)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(a.tile_seg, 0, (int)(((a.ntiles + 3u) & ~3u) * 4u), 0x00020000);
    typedef uint32_t u32x4t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32x4t q = __builtin_amdgcn_raw_buffer_load_b128(rt, (tb + r) * 16u, 0, 0);
      ts[r].events = q.x;
      ts[r].pool_base = q.y;
      ts[r].parsed = (uint16_t)q.z;
      ts[r].since_ok = (uint16_t)(q.z >> 16);
      ts[r].flags = (uint16_t)q.w;
      ts[r].carry_off = (uint16_t)(q.w >> 16);
    }
#pragma unroll
    for (int r = 0; r < R; r += 4) {
      const u32x4t q = __builtin_amdgcn_raw_buffer_load_b128(rs, (tb + r) * 4u, 0, 0);
      sg[r] = q.x;
      sg[r + 1] = q.y;
      sg[r + 2] = q.z;
      sg[r + 3] = q.w;
    }
  }
  // deferred lines (non-canonical timestamp prefixes; rare): per round every thread hands
  // its next tile that has them to the block (<= 256 per round), the waves run them
  uint32_t dmask = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (PASS == 0 && tb + r < a.ntiles && (ts[r].flags & 4u)) dmask |= 1u << r;
  while (PASS == 0 && __syncthreads_or(dmask != 0u)) {
    if (t == 0) s_ndef = 0;
    __syncthreads();
    uint32_t slot = ~0u;
    const uint32_t rr = dmask ? (uint32_t)__builtin_ctz(dmask) : 0u;
    if (dmask) {
      slot = atomicAdd(&s_ndef, 1u);  // < 256: one entry per thread and round
      s_def[slot] = tb + rr;
    }
    __syncthreads();
    const uint32_t nd = s_ndef;
    for (uint32_t k = wv; k < nd; k += 4) {
      const uint32_t tile = s_def[k];
      uint32_t dp, dq;
      fix_tile(a, tile, a.tstat[tile], lane, dp, dq);
      if (lane == 0) { s_fix[k][0] = dp; s_fix[k][1] = dq; }
    }
    __syncthreads();
    if (slot != ~0u) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((uint32_t)r == rr) {
          ts[r].parsed = (uint16_t)(ts[r].parsed + s_fix[slot][0]);
          ts[r].since_ok = (uint16_t)(ts[r].since_ok + s_fix[slot][1]);
          // the corrected counts for every later kernel (only their word: fix_tile rewrote an
          // inline slot in pool_base, which ts[r] holds from before)
          reinterpret_cast<uint32_t*>(a.tstat + tb + r)[2] = (uint32_t)ts[r].parsed | ((uint32_t)ts[r].since_ok << 16);
        }
      dmask &= dmask - 1u;
    }
  }
  // the thread's and the block's totals (block-local: < 2^32)
  uint32_t v = 0, p = 0, q = 0, h = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) { v += ts[r].events; p += ts[r].parsed; q += ts[r].since_ok; h += tile_hits(a, ts[r]); }
  const uint32_t iv = wave_incl_scan_add(v, lane), ip = wave_incl_scan_add(p, lane), iq = wave_incl_scan_add(q, lane),
                 ih = wave_incl_scan_add(h, lane);
  if (lane == 63) { s_wt[0][wv] = iv; s_wt[1][wv] = ip; s_wt[2][wv] = iq; s_wt[3][wv] = ih; }
  __syncthreads();
  uint32_t ov = iv - v, op = ip - p, oq = iq - q, oh = ih - h;
  for (int k = 0; k < wv; ++k) { ov += s_wt[0][k]; op += s_wt[1][k]; oq += s_wt[2][k]; oh += s_wt[3][k]; }
  if (PASS == 0) {  // the block's totals
    if (t < 4) a.bsum[4 * (size_t)bid + t] = s_wt[t][0] + s_wt[t][1] + s_wt[t][2] + s_wt[t][3];
    return;
  }
  {  // the earlier blocks' totals
    uint64_t xv = 0, xp = 0, xq = 0, xh = 0;
    for (uint32_t b = t; b < bid; b += 256) {
      xv += a.bsum[4 * (size_t)b];
      xp += a.bsum[4 * (size_t)b + 1];
      xq += a.bsum[4 * (size_t)b + 2];
      xh += a.bsum[4 * (size_t)b + 3];
    }
    xv = wave_sum(xv);
    xp = wave_sum(xp);
    xq = wave_sum(xq);
    xh = wave_sum(xh);
    if (lane == 0) { s_w64[0][wv] = xv; s_w64[1][wv] = xp; s_w64[2][wv] = xq; s_w64[3][wv] = xh; }
    __syncthreads();
    if (t < 4) s_base[t] = s_w64[t][0] + s_w64[t][1] + s_w64[t][2] + s_w64[t][3];
    __syncthreads();
  }
  const uint32_t s_prev = tb > 0 && tb - 1 < a.ntiles ? a.tile_seg[tb - 1] : ~0u;
  const uint32_t s_next = tb + R < a.ntiles ? a.tile_seg[tb + R] : ~0u;
  const uint64_t blk_lo = s_base[0];
  const uint64_t blk_hi = s_base[0] + s_wt[0][0] + s_wt[0][1] + s_wt[0][2] + s_wt[0][3];
  const uint32_t blk_h = s_wt[3][0] + s_wt[3][1] + s_wt[3][2] + s_wt[3][3];
  // tile bases and hit counts go through LDS so that both outputs are written coalesced
  __shared__ uint32_t s_tbl[256 * R];   // block-local tile line base (< 2^32)
  __shared__ uint8_t s_thit[256 * R];   // tile hit slots (<= kHitSlots)
  __shared__ uint32_t s_tseg[256 * R];  // tile -> stream (for the flattened hits)
  __shared__ uint32_t s_hpre[256];      // inclusive prefix of the threads' hit slots
  s_hpre[t] = oh + h;
  uint32_t lv = ov;
  uint64_t bv = s_base[0] + ov, bp = s_base[1] + op, bq = s_base[2] + oq;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t tile = tb + r;
    s_tbl[t * R + r] = lv;
    s_thit[t * R + r] = (uint8_t)(tile < a.ntiles ? tile_hits(a, ts[r]) : 0u);
    s_tseg[t * R + r] = sg[r];
    if (tile < a.ntiles) {
      const uint32_t s = sg[r];
      const uint32_t sp = r ? sg[r - 1] : s_prev, sn = r + 1 < R ? sg[r + 1] : s_next;
      const uint32_t nx = tile + 1 < a.ntiles ? sn : ~0u;
      if (sp != s) { a.segout[s].line_lo = bv; a.segout[s].p_lo = bp; a.segout[s].q_lo = bq; }
      if (nx != s) {
        a.segout[s].line_hi = bv + ts[r].events;
        a.segout[s].p_hi = bp + ts[r].parsed;
        a.segout[s].q_hi = bq + ts[r].since_ok;
      }
    }
    lv += ts[r].events;
    bv += ts[r].events;
    bp += ts[r].parsed;
    bq += ts[r].since_ok;
  }
  __syncthreads();
  const uint32_t t0 = bid * (256u * R);
  for (uint32_t k = (uint32_t)t; k < 256u * R; k += 256)
    if (t0 + k < a.ntiles) a.tile_base[t0 + k] = blk_lo + s_tbl[k];
  // the block's hit slots, in tile order: hit k -> its thread (prefix search), then tile
  // (KLF_FLAT_BATCH hits per thread at once: their hit-slot loads in flight together)
  const uint64_t hb = s_base[3];
  constexpr int FB = KLF_FLAT_BATCH;
  for (uint32_t k0 = (uint32_t)t; k0 < blk_h; k0 += 256u * FB) {
    uint32_t ftile[FB], fj[FB], fseg[FB], off[FB];
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const uint32_t k = k0 + 256u * (uint32_t)u;
      ftile[u] = ~0u;
      fj[u] = 0;
      fseg[u] = 0;
      if (k >= blk_h || hb + k >= a.hflat_cap) continue;
      uint32_t lo = 0, hi = 255;  // the first thread whose inclusive prefix exceeds k
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_hpre[mid] > k) hi = mid; else lo = mid + 1;
      }
      uint32_t j = k - (lo ? s_hpre[lo - 1] : 0u), r = 0;
      while (j >= s_thit[lo * R + r]) j -= s_thit[lo * R + r++];
      ftile[u] = t0 + lo * R + r;
      fj[u] = j;
      // (+ the tile's stream in bits 48..63 when it fits: k_verify skips its tile_seg load;
      // the owning thread's registers hold it, passed through LDS)
      fseg[u] = s_tseg[lo * R + r];
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      // {tile, its hit's tile offset << 32}: inline hits from the TileStat (L2: this kernel
      // just read it), the others from the tile's hit slots
      off[u] = 0;
      if (ftile[u] == ~0u) continue;
      if (KLF_HIT_INLINE) {
        const TileStat& tsh = a.tstat[ftile[u]];
        off[u] = (tsh.flags & kTsHitInline) ? ((tsh.pool_base >> (16u * fj[u])) & 0xFFFFu)
                                            : (uint32_t)a.hslots[(size_t)ftile[u] * kHitSlots + fj[u]];
      } else {
        off[u] = a.hslots[(size_t)ftile[u] * kHitSlots + fj[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < FB; ++u)
      if (ftile[u] != ~0u)
        a.hflat[hb + k0 + 256u * (uint32_t)u] = (uint64_t)ftile[u] | ((uint64_t)off[u] << 32) |
                                                 ((uint64_t)(fseg[u] < 0xFFFFu ? fseg[u] : 0xFFFFu) << 48);
  }
  if (t == 0 && (bid + 1) * (256u * R) >= a.ntiles) {  // the last block knows the totals
    // More lines than the line index holds: raised here, before any kernel that indexes
    // by global line (k_verify runs beside k_scatter, whose own check comes too late for
    // it; bits / meta / line_off past cap_lines are outside their allocations).
    if (blk_hi > a.cap_lines) atomicOr(&a.counters[2], 1u);
    if (a.hflat) {
      const uint64_t tot = hb + blk_h;
      a.counters[kCtrFlatHits] = (uint32_t)(tot < 0xFFFFFFFFull ? tot : 0xFFFFFFFFull);
      if (tot > a.hflat_cap) atomicOr(&a.counters[kCtrHitsOver], 1u);
    }
  }
  if (a.grep_mode != kGrepNone && a.bits) {  // bitmap words whose first line is in [blk_lo, blk_hi)
    const uint64_t w0 = (blk_lo + 31) / 32, w1 = (blk_hi + 31) / 32;
    for (uint64_t w = w0 + t; w < w1 && w * 32 < a.cap_lines; w += 256) a.bits[w] = 0u;
  }
}

// ---- K1d: scatter staged slots into the global line arrays --------------------------
// One wave per group of 64 consecutive tiles (one lane per tile reads the tile's record
// into the wave's LDS table; ~20 lines per 8 KiB tile would leave most lanes of a
// wave-per-tile idle), then the lanes walk the group's lines, each line finding its tile by
// binary search over the LDS prefix.  The walk loads kScatterBatch lines' slots before
// storing any of them: the kernel is latency-bound on those dependent loads otherwise.
constexpr int kScatterGroup = 64;
constexpr int kScatterBatch = 8;
struct ScatterEnt {
  uint64_t base;     // global line index of the tile's slot 0 (= tile line k0)
  uint64_t rel_lo;   // tile start, stream-relative
  uint32_t src;      // index of slot 0 in slots[] (normal) or pool[] (dense, bit 31 set)
  uint32_t seg;      // stream segment
  uint32_t pad[2];
};

struct ScatterLds {
  ScatterEnt ent[4][kScatterGroup];
  uint32_t pre[4][kScatterGroup];  // inclusive line-count prefix of the group's tiles
};
// Block bid of nb (k_scatter alone, or the first nb blocks of k_scatter_verify).
__device__ __forceinline__ void scatter_body(RunArgs& a, uint32_t bid, uint32_t nb, ScatterLds& L) {
  auto& s_ent = L.ent;
  auto& s_pre = L.pre;
  // lazy line index (grep none, --tail -1): launched after k_tailw, and only the line gather
  // needs the index; the dense path lists lines from the slots (the host builds the index
  // on demand: klf_result_lines, klf_retail, klf_result_last_unparsed)
  if (a.lazy_index && a.counters[kCtrDense]) return;
  // the windowed index's pre-count pass of a general set: only deferred lines (fix_tile's
  // matches) carry slot hit bits there, and without a deferred line there is nothing to do
  if (a.scatter_mode == 1 && a.grep_mode == kGrepGeneral && !a.counters[kCtrDefer]) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* err_flag = a.counters + 2;
  const uint32_t ngroups = (a.ntiles + kScatterGroup - 1) / kScatterGroup;
  // the window pass visits only the groups k_tailw listed per stream (flat index f over
  // their concatenation: the stream by a search of the prefix)
  const bool wpass = a.scatter_mode == 2;
  const uint64_t F = wpass ? (a.counters[2] ? 0 : a.wgrp[2 * a.nsegs]) : ngroups;  // (overflow: no list)
  // small batches: P waves per group, each writing a P-th of the group's lines (C1: 128
  // groups of ~5,400 lines were 128 waves walking their lines 64 at a time)
  // (P from the grid: up to 8; RunArgs::scatter_split overrides it, tests)
  uint32_t P = a.scatter_split;
  if (P == 0) {
    const uint64_t w = (uint64_t)nb * 4 / (F ? F : 1);
    P = w < 1 ? 1u : (w > 8 ? 8u : (uint32_t)w);
  }
  for (uint64_t fp = bid * 4 + wv; fp < F * P; fp += nb * 4) {
    const uint64_t f = fp / P;
    const uint32_t part = (uint32_t)(fp - f * P);
    uint32_t g = (uint32_t)f;
    if (wpass) {
      uint32_t lo = 0, hi = a.nsegs;  // the last stream whose prefix is <= f
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.wgrp[a.nsegs + mid] <= f) lo = mid; else hi = mid;
      }
      g = (uint32_t)(a.wgrp[lo] & 0xFFFFFFFFull) + (uint32_t)(f - a.wgrp[a.nsegs + lo]);
      if (g >= ngroups) continue;
    }
    const uint32_t tile = g * kScatterGroup + lane;
    uint32_t n = 0;
    if (tile < a.ntiles) {
      const TileStat ts = a.tstat[tile];
      const uint32_t s = a.tile_seg[tile];
      const SegDesc sd = a.segs[s];
      const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
      const bool first = rel_lo == 0, last = rel_lo + kTile >= (int64_t)sd.len;
      const uint32_t k0 = first ? 0 : 1, k1 = last ? ts.events : ts.events + 1;
      n = k1 > k0 ? k1 - k0 : 0;
      const uint64_t base = a.tile_base[tile];
      if (a.scatter_mode == 1 && !(ts.flags & 12u)) n = 0;  // (no deferred line, no literal hit here)
      if (a.scatter_mode == 2) {  // lines of the tail window and the one after it (its end)
        const SegOut& so = a.segout[s];
        const uint64_t f = base + k0;
        if (so.win_hi <= so.win_lo || f > so.win_hi || f + n <= so.win_lo) n = 0;
      }
      ScatterEnt e;
      e.base = base + k0;
      e.rel_lo = (uint64_t)rel_lo;
      // slot 0's source: the pool (bit 31), the TileStat itself (bit 30: kTsInline), the record
      e.src = (ts.flags & 1u) ? (ts.pool_base | 0x80000000u) : (ts.flags & kTsInline) ? 0x40000000u : 0u;
      e.seg = s;
      e.pad[0] = e.pad[1] = 0;
      s_ent[wv][lane] = e;
      if ((ts.flags & 2u) && base < a.cap_lines && a.scatter_mode != 2 && part == 0) {
        // literal hit inside the line carried in from an earlier tile: that line's start
        // is the last staged start of the nearest earlier tile of the stream that has one
        // (the window pass skips it: the pre-count pass set those bits already)
        int64_t cs = -1;
        for (uint32_t pt = tile; pt > sd.tile0;) {
          --pt;
          const TileStat pst = a.tstat[pt];
          const int64_t prel = (int64_t)(pt - sd.tile0) * kTile;
          const uint32_t pk0 = prel == 0 ? 0 : 1;
          const uint32_t pn = pst.events + 1 > pk0 ? pst.events + 1 - pk0 : 0;  // never the stream's last tile
          if (pn == 0) continue;
          const uint32_t v = slot_at(a, pst, pt, pn - 1);
          const uint32_t mt = v >> 16;
          // a deferred line had its whole content searched by k_fixup
          if ((mt & Meta::kParsed) && !(v & kSlotDefer)) cs = prel + (int64_t)(v & kSlotOff) + (mt >> 2);
          break;
        }
        if (cs >= 0 && rel_lo + (int64_t)ts.carry_off - 1 - (int64_t)kCarryBias >= cs)
          atomicOr(&a.bits[base >> 5], 1u << (base & 31));
      }
      if (last && part == 0) {
        const uint64_t lend = base + ts.events;
        if (lend <= a.cap_lines) a.line_off[lend + s] = sd.len;
        else atomicOr(err_flag, 1u);
      }
    }
    const uint32_t incl = wave_incl_scan_add(n, lane);
    s_pre[wv][lane] = incl;
    const uint32_t gtotal = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // this wave's part of the group's lines: [lb, total)
    const uint32_t lb = (uint32_t)((uint64_t)gtotal * part / P), total = (uint32_t)((uint64_t)gtotal * (part + 1) / P);
    wave_lds_sync();
    for (uint32_t l0 = lb; l0 < total; l0 += 64 * kScatterBatch) {
      uint32_t sl[kScatterBatch], kk[kScatterBatch], jj[kScatterBatch];
#pragma unroll
      for (int u = 0; u < kScatterBatch; ++u) {
        const uint32_t l = l0 + (uint32_t)(u * 64 + lane);
        sl[u] = 0;
        kk[u] = 0;
        jj[u] = 0;
        if (l < total) {
          uint32_t lo = 0, hi = kScatterGroup - 1;  // first tile whose inclusive prefix exceeds l
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[wv][mid] > l) hi = mid; else lo = mid + 1;
          }
          const uint32_t j = l - (lo ? s_pre[wv][lo - 1] : 0u);
          const uint32_t src = s_ent[wv][lo].src;
          const uint32_t* sp = (src & 0x80000000u) ? a.pool + (src & 0x7FFFFFFFu)
                               : (src & 0x40000000u) ? reinterpret_cast<const uint32_t*>(a.tstat + g * kScatterGroup + lo) + 1
                               : a.slots ? a.slots + (size_t)(g * kScatterGroup + lo) * kRecStride + kRecHead : a.pool;
          sl[u] = sp[j];
          kk[u] = lo;
          jj[u] = j;
        }
      }
#pragma unroll
      for (int u = 0; u < kScatterBatch; ++u) {
        const uint32_t l = l0 + (uint32_t)(u * 64 + lane);
        if (l >= total) continue;
        const ScatterEnt& e = s_ent[wv][kk[u]];
        const uint64_t li = e.base + jj[u];
        if (li >= a.cap_lines) { atomicOr(err_flag, 1u); continue; }
#if KLF_ABL & 16384  // timing build: slot contents ignored (no line selected downstream)
        a.line_off[li + e.seg] = e.rel_lo;
        a.meta[li] = (uint16_t)(sl[u] & 0u);
#else
        if (a.scatter_mode != 1) {  // (the pre-count pass: match bits only; k_mcount and
          a.line_off[li + e.seg] = e.rel_lo + (sl[u] & kSlotOff);  // k_tailw read no more,
          a.meta[li] = (uint16_t)(sl[u] >> 16);  // the window pass writes the lines it keeps)
        }
        if (sl[u] & kSlotHit) atomicOr(&a.bits[li >> 5], 1u << (li & 31));
#endif
      }
    }
    asm volatile("" ::: "memory");  // the next group rewrites the wave's LDS tables
  }
}
__global__ __launch_bounds__(256) void k_scatter(RunArgs a) {
  __shared__ ScatterLds L;
  scatter_body(a, blockIdx.x, gridDim.x, L);
}

// ============================================= K2: general pattern sets (per line) ==
__device__ bool ac_match(const DevPatterns& P, const uint8_t* p, int64_t n) {
  uint32_t st = 0;
  for (int64_t i = 0; i < n; ++i) {
    st = P.ac_next[(size_t)st * P.ac_classes + P.ac_class[p[i]]];
    if (P.ac_accept[st]) return true;
  }
  return false;
}

__device__ bool rx_match(const DevPatterns& P, uint32_t r, const uint8_t* p, int64_t n) {
  const uint32_t fl = P.rx_flags[r];
  if (n == 0) return (fl & 2u) != 0;
  if (fl & 1u) return true;
  const uint64_t first = P.rx_first[r], lastm = P.rx_last[r];
  const uint64_t* B = P.rx_b + (size_t)r * P.rx_classes;
  const uint64_t* F = P.rx_follow + (size_t)r * 64;
  uint64_t d = P.rx_init0[r];
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t c = d & B[P.rx_class[p[i]]];
    if (c & lastm) return true;
    uint64_t nd = first, m = c;
    while (m) {
      const int q = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      nd |= F[q];
    }
    d = nd;
  }
  return (d & P.rx_end[r]) != 0;
}

__device__ __forceinline__ uint32_t line_plen(const RunArgs& a, uint16_t meta, const uint8_t* segp,
                                              uint64_t start, uint64_t end) {
  uint32_t plen = meta >> 2;
  if (plen == kPlenEscape) {  // long prefix: find the first space again
    plen = 0;
    for (uint64_t q = start; q < end; ++q)
      if (segp[q] == ' ') { plen = (uint32_t)(q - start) + 1; break; }
  }
  return plen;
}

// K2a: verification of the prefilter's bitmap hits.  One lane per hit: the sample's gram
// (global bytes), the 16-B entries of its bucket, the needle compare (first dword from the
// entry), then the line of the occurrence start (segment + line-index binary searches).
// A literal starting inside a parsed line's content is a match; a regex factor queues
// (line, regex) for k_nfa.  The occurrence may start before the sample's tile.
__device__ __forceinline__ uint32_t gword(const uint8_t* p) {  // 4 bytes at any alignment
  const uintptr_t a0 = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a0 & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a0 & 3));
}

// One bitmap hit: the sample at tile offset p of `tile` (stream s).  The occurrence start
// x = p - k may lie before the tile: an occurrence holds no '\n', so it is then in the
// tile's carried-in line.  Inside the tile, its line comes from the tile's own staged
// line starts (slots, meta in the high half) instead of a search of the whole index.
// The bucket walk of one hit whose bucket [e0, e1) is known (the loads before it are
// batched over several hits by k_verify).
// NFA candidates of one wave, staged in LDS and appended to the global queue with one
// atomic per wave at the end (k_verify): one counter that every candidate of the run
// incremented serialized them at the memory side (C5: ~67 K candidates).
constexpr uint32_t kVerifyQ = 256;  // candidates staged per wave (more: pushed directly)
struct VerifyQ {
  uint32_t* n;        // LDS: staged count
  uint64_t (*buf)[2];  // LDS: [kVerifyQ] {line | regex << 40, occurrence}
};
__device__ __forceinline__ void push_candidate(const RunArgs& a, const VerifyQ& q, uint64_t key, uint64_t x) {
  const uint32_t k = atomicAdd(q.n, 1u);  // (LDS)
  if (k < kVerifyQ) {
    q.buf[k][0] = key;
    q.buf[k][1] = x;
    return;
  }
  const uint32_t qi = atomicAdd(&a.counters[kCtrQueue], 1u);
  if (qi < a.cand_cap) {
    a.cand[2 * (size_t)qi] = key;
    a.cand[2 * (size_t)qi + 1] = x;
  } else {
    atomicOr(&a.counters[kCtrQOver], 1u);
  }
}
#ifndef KLF_VERIFY_ENT
#define KLF_VERIFY_ENT 4  // bucket entries loaded at once by the walk (1: one at a time)
#endif
constexpr int kVerifyEnt = KLF_VERIFY_ENT;
__device__ void verify_hit_from(const RunArgs& a, uint32_t tile, uint32_t s, const SegDesc& sd, int32_t p,
                                uint32_t gs, uint32_t e0, uint32_t e1, const VerifyQ& vq) {
  const DevPatterns& P = a.pats;
  const uint8_t* segp = a.bytes + sd.base;
  const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
  // one bucket entry past its pre-check (below): the full compare, the line, the candidate
  auto entry = [&](const uint4 E) {
    const uint32_t m = E.y & 0xFFFFu, ko = (E.y >> 16) & 0xFFu;
    const uint32_t lm = (E.y & kQfLoose) ? 0x20202020u : 0u;
    auto msk_of = [&](uint32_t k) { return m - k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (m - k))) - 1u); };
    const int32_t x = p - (int32_t)ko;
    if (rel_lo + x < 0 || rel_lo + x + (int64_t)m > (int64_t)sd.len) return;
    // the needle's dwords, then dwords 1..7 with every load in flight at once (KLF_VERIFY_PAR),
    // the rest of a needle longer than 32 bytes dword by dword
    const uint8_t* q = segp + rel_lo + x;
    bool eq = (((gword(q) | lm) ^ P.qf_nbytes[E.x]) & msk_of(0)) == 0;
    if (!KLF_VERIFY_PAR) {  // dword by dword, each load after the previous compare
      for (uint32_t k = 4; k < m && eq; k += 4)
        eq = (((gword(q + k) | lm) ^ P.qf_nbytes[E.x + (k >> 2)]) & msk_of(k)) == 0;
    } else if (eq && m > 4) {
      const uintptr_t qa = reinterpret_cast<uintptr_t>(q);
      const uint32_t* qw = reinterpret_cast<const uint32_t*>(qa & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(qa & 3);
      uint32_t d[9], want[8];
#pragma unroll
      for (int k = 1; k < 9; ++k) d[k] = (4u * (uint32_t)k < m + 4u) ? qw[k] : 0u;  // (read slack past the batch)
#pragma unroll
      for (int k = 1; k < 8; ++k) want[k] = 4u * (uint32_t)k < m ? P.qf_nbytes[E.x + (uint32_t)k] : 0u;
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (4u * (uint32_t)k < m)
          eq = eq && ((((__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh)) | lm) ^ want[k]) & msk_of(4u * (uint32_t)k)) == 0;
      for (uint32_t k = 32; k < m && eq; k += 4)
        eq = (((gword(q + k) | lm) ^ P.qf_nbytes[E.x + (k >> 2)]) & msk_of(k)) == 0;
    }
    if (!eq) return;
#if KLF_ABL & 32
    atomicOr(&a.counters[13], x);  // timing build: bucket walk only
    return;
#endif
    KLF_VSTAMP(2);  // (a matching entry)
    // the occurrence's line: global index, start (stream offset), meta
    const TileStat ts = a.tstat[tile];
    const bool first = rel_lo == 0, last = rel_lo + kTile >= (int64_t)sd.len;
    const uint32_t k0 = first ? 0 : 1, k1 = last ? ts.events : ts.events + 1;
    const uint32_t nl = k1 > k0 ? k1 - k0 : 0;
    int lo = 0, hi = x < 0 ? 0 : (int)nl;  // starts <= x
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int32_t)(slot_at(a, ts, tile, (uint32_t)mid) & kSlotOff) <= x) lo = mid + 1; else hi = mid;
    }
    const uint64_t l = a.tile_base[tile] + (lo > 0 ? k0 + (uint32_t)lo - 1 : 0);
    if (l >= a.cap_lines) {  // (k_tindex raises the overflow first; never index past the arrays)
      atomicOr(&a.counters[2], 1u);
      return;
    }
    KLF_VSTAMP(3);  // (its tile's line search done)
    // the line's meta and start from its slot: the tile's own, or for the line carried in
    // from an earlier tile the last one listed by the nearest earlier tile that lists one
    // (k_scatter may still be running: the global line index is not read here)
    uint32_t v = 0;
    int64_t vrel = rel_lo;
    if (lo > 0 || (KLF_ABL & 524288)) {  // (timing build 524288: no walk back, a wrong slot)
      v = slot_at(a, ts, tile, lo > 0 ? (uint32_t)lo - 1 : 0u);
    } else {
      for (uint32_t pt = tile; pt > sd.tile0;) {  // the stream's first tile lists line 0
        --pt;
        const TileStat pst = a.tstat[pt];
        const int64_t prel = (int64_t)(pt - sd.tile0) * kTile;
        const uint32_t pk0 = prel == 0 ? 0u : 1u;
        const uint32_t pn = pst.events + 1 - pk0;  // an earlier tile is never the stream's last
        if (pn == 0) continue;
        v = slot_at(a, pst, pt, pn - 1);
        vrel = prel;
        break;
      }
    }
    const uint16_t mt = (uint16_t)(v >> 16);
    const uint64_t ls = (uint64_t)vrel + (v & kSlotOff);
    KLF_VSTAMP(4);  // (the line's start slot, walked back to)
    if (!(mt & Meta::kParsed)) return;
    if (!(E.y & kQfRegex)) {  // literal: a match when it starts inside the content
      // (a parsed line's first space ends its prefix: the stream end bounds the search)
      const uint32_t plen = (mt >> 2) == kPlenEscape ? line_plen(a, mt, segp, ls, sd.len) : mt >> 2;
      if ((uint64_t)(rel_lo + x) >= ls + plen) {
        atomicOr(&a.bits[l >> 5], 1u << (l & 31));
        if (a.count_pats) count_pair(a, l, s, E.z);
      }
      return;
    }
    if (!a.count_pats && ((a.bits[l >> 5] >> (l & 31)) & 1u)) return;  // counting: every regex decides
    KLF_VSTAMP(5);  // (bitmap checked)
    if (a.win_index) {
      // windowed line index (no full k_scatter): the candidate line's start, end and meta for
      // k_nfa_win / k_nfa.  Its end is the next line start: this tile's next slot, else the
      // first start a later tile of the stream lists, else the stream end (every writer of
      // these entries writes the same values)
      uint64_t le = sd.len;
      if ((uint32_t)lo < nl) {
        le = (uint64_t)rel_lo + (slot_at(a, ts, tile, (uint32_t)lo) & kSlotOff);
      } else if (!(KLF_ABL & 262144)) {  // (timing build 262144: no walk forward)
        for (uint32_t pt = tile + 1; pt < sd.tile0 + sd.ntiles; ++pt) {
          const TileStat pst = a.tstat[pt];
          const int64_t prel = (int64_t)(pt - sd.tile0) * kTile;
          const uint32_t pk1 = prel + kTile >= (int64_t)sd.len ? pst.events : pst.events + 1;
          if (pk1 <= 1u) continue;  // (k0 = 1: no line starts in tile pt)
          le = (uint64_t)prel + (slot_at(a, pst, pt, 0) & kSlotOff);
          break;
        }
      }
      a.line_off[l + s] = ls;
      a.line_off[l + s + 1] = le;
      a.meta[l] = mt;
    }
    KLF_VSTAMP(6);  // (the line's bounds written)
    // {line | regex << 40, the occurrence (stream offset) | stream << 40}
    push_candidate(a, vq, l | ((uint64_t)E.z << 40), (uint64_t)(rel_lo + x) | ((uint64_t)s << 40));
  };
  // the bucket walk, four entries loaded at once: the pre-check (round 6) compares the
  // needle's bytes at its sampled offset with the sample dword gs already in a register, so
  // entries of other grams sharing the bucket (C4: a bucket of a common gram lists dozens of
  // needles) end without a further access -- the walk's cost is its entry loads, in flight
  // together instead of one after the other
  for (uint32_t eb = e0; eb < e1; eb += kVerifyEnt) {
    uint4 Eb[kVerifyEnt];
    uint32_t pass = 0;
#pragma unroll
    for (int j = 0; j < kVerifyEnt; ++j) Eb[j] = eb + (uint32_t)j < e1 ? P.qf_ent[eb + (uint32_t)j] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < kVerifyEnt; ++j) {
      const uint32_t m = Eb[j].y & 0xFFFFu, ko = (Eb[j].y >> 16) & 0xFFu;
      const uint32_t lm = (Eb[j].y & kQfLoose) ? 0x20202020u : 0u;
      const uint32_t mk = m - ko >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (m - ko))) - 1u);
      if (eb + (uint32_t)j < e1 && (((gs | lm) ^ Eb[j].w) & mk) == 0u) pass |= 1u << j;
    }
    while (pass) {  // (register select, no dynamic index into Eb: that would go to scratch)
      const int j = __builtin_ctz(pass);
      pass &= pass - 1u;
      uint4 E = Eb[0];
#pragma unroll
      for (int i = 1; i < kVerifyEnt; ++i)
        if (j == i) E = Eb[i];
      entry(E);
    }
  }
}

__device__ void verify_hit(const RunArgs& a, uint32_t tile, uint32_t s, int32_t p, const VerifyQ& vq) {
  const DevPatterns& P = a.pats;
  const SegDesc sd = a.segs[s];
  const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
  const uint32_t gs = gword(a.bytes + sd.base + rel_lo + p);
  const uint32_t g = (gs | P.qf_fold) & P.qf_mask;
  const uint32_t b = qf_bucket(g, P.qf_w24, P.qf_k);
  verify_hit_from(a, tile, s, sd, p, gs, P.qf_head[b], P.qf_head[b + 1], vq);
}

// Thread per hit: the flattened tile hit slots (k_tindex), then the spilled hits.  The
// chain of dependent loads before a hit's bucket walk (slot -> offset, stream ->
// descriptor -> gram -> bucket) runs for kVerifyBatch hits at once: the kernel is bound
// by that latency (most hits are prefilter false positives that end at the bucket).
constexpr int kVerifyBatch = 4;
struct VerifyLds {
  uint32_t qn[4];
  uint64_t qbuf[4][kVerifyQ][2];
};
__device__ __forceinline__ void verify_body(RunArgs& a, uint32_t bid, uint32_t nb, VerifyLds& L) {
  auto& s_qn = L.qn;
  auto& s_qbuf = L.qbuf;
  if (a.counters[2] || a.counters[kCtrHitsOver]) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s_qn[wv] = 0;
  wave_lds_sync();
  const VerifyQ vq{&s_qn[wv], s_qbuf[wv]};
  const uint32_t gid = bid * blockDim.x + threadIdx.x, stride = nb * blockDim.x;
  const uint32_t nf = a.counters[kCtrFlatHits];
  const DevPatterns& P = a.pats;
  if (gid < nf) KLF_VSTAMP(0);
  for (uint32_t i0 = gid; i0 < nf; i0 += kVerifyBatch * stride) {
    uint32_t tile[kVerifyBatch], sg[kVerifyBatch], e0[kVerifyBatch], e1[kVerifyBatch];
    int32_t pp[kVerifyBatch];
    SegDesc sd[kVerifyBatch];
#pragma unroll
    for (int u = 0; u < kVerifyBatch; ++u) {
      const uint32_t i = i0 + (uint32_t)u * stride;
      const uint64_t hf = a.hflat[i < nf ? i : i0];
      tile[u] = (uint32_t)hf;
      pp[u] = (int32_t)((hf >> 32) & 0xFFFFu);
      sg[u] = (uint32_t)(hf >> 48);
      if (sg[u] == 0xFFFFu) sg[u] = a.tile_seg[tile[u]];  // (streams past 65,534)
    }
#pragma unroll
    for (int u = 0; u < kVerifyBatch; ++u) sd[u] = a.segs[sg[u]];
    uint32_t gg[kVerifyBatch];
#pragma unroll
    for (int u = 0; u < kVerifyBatch; ++u) {
      const int64_t rel_lo = (int64_t)(tile[u] - sd[u].tile0) * kTile;
      gg[u] = gword(a.bytes + sd[u].base + rel_lo + pp[u]);
    }
#pragma unroll
    for (int u = 0; u < kVerifyBatch; ++u) {
      const uint32_t b = qf_bucket((gg[u] | P.qf_fold) & P.qf_mask, P.qf_w24, P.qf_k);
      e0[u] = P.qf_head[b];
      e1[u] = P.qf_head[b + 1];
    }
    KLF_VSTAMP(1);  // (the batch's hits, streams, grams and buckets loaded)
#pragma unroll
    for (int u = 0; u < kVerifyBatch; ++u)
      if (i0 + (uint32_t)u * stride < nf) {
#if KLF_ABL & 16
        if (pp[u] == 0x7FFF) atomicOr(&a.counters[13], sg[u]);  // timing build: no verification work
        continue;
#endif
        verify_hit_from(a, tile[u], sg[u], sd[u], pp[u], gg[u], e0[u], e1[u], vq);
      }
  }
  const uint32_t nh = a.counters[kCtrHits] < a.qhits_cap ? a.counters[kCtrHits] : a.qhits_cap;
  for (uint32_t i = gid; i < nh; i += stride) {
    const uint64_t pos = a.qhits[i];
    uint32_t lo = 0, hi = a.nsegs;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.segs[mid].base <= pos) lo = mid; else hi = mid;
    }
    const uint64_t rel = pos - a.segs[lo].base;
    const uint32_t tile = a.segs[lo].tile0 + (uint32_t)(rel / kTile);
    verify_hit(a, tile, lo, (int32_t)(rel % kTile), vq);
  }
  if (gid == 0) a.counters[kCtrVerified] = nf + nh;
  if (gid < nf) KLF_VSTAMP(7);
  // the wave's staged candidates: one queue reservation, then coalesced stores
  wave_lds_sync();
  const uint32_t nq = s_qn[wv] < kVerifyQ ? s_qn[wv] : kVerifyQ;
  if (nq) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.counters[kCtrQueue], nq);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
    for (uint32_t k = (uint32_t)lane; k < nq; k += 64) {
      if ((uint64_t)base + k < a.cand_cap) {
        a.cand[2 * ((size_t)base + k)] = s_qbuf[wv][k][0];
        a.cand[2 * ((size_t)base + k) + 1] = s_qbuf[wv][k][1];
      } else {
        atomicOr(&a.counters[kCtrQOver], 1u);
      }
    }
  }
}
#ifndef KLF_VERIFY_WAVES
#define KLF_VERIFY_WAVES 4  // k_verify / k_scatter_verify: min waves per SIMD (<= 128 VGPRs; 1 -> 129: C4 339 vs 295 us)
#endif
__global__ __launch_bounds__(256, KLF_VERIFY_WAVES) void k_verify(RunArgs a) {
  __shared__ VerifyLds L;
  verify_body(a, blockIdx.x, gridDim.x, L);
}
// Regex sets: k_scatter (bandwidth-bound) and k_verify (latency-bound: a chain of dependent
// loads per hit) as one launch, blocks [0, nsb) scattering, the rest verifying, so the two
// overlap on the chip without a second stream (k_verify reads the line slots, not the
// global line index).
__global__ __launch_bounds__(256, KLF_VERIFY_WAVES) void k_scatter_verify(RunArgs a, uint32_t nsb) {
  __shared__ union {
    ScatterLds s;
    VerifyLds v;
  } L;
  if (blockIdx.x < nsb) scatter_body(a, blockIdx.x, nsb, L.s);
  else verify_body(a, blockIdx.x - nsb, gridDim.x - nsb, L.v);
}

// K2b: the prefiltered regex stage.  One lane per queued (batch offset, regex) candidate:
// the offset's stream and line (binary searches over the segment table and the line
// index), then the Glushkov NFA of that regex over the line's content.  Lines already
// matched are skipped.  LDS: the regex tables (byte classes, B[regex][class],
// follow[regex][position < maxpos], first/last/init0/end) are staged once per block;
// content is read 16 B at a time and the 16 class / B lookups of a block are issued
// before the state recurrence walks it (only the follow lookups depend on the state).
struct NfaTables {
  const uint8_t* cls;
  const uint64_t* b;      // [rx][classes]
  const uint64_t* fol;    // [rx][fstride]
  const uint64_t* vec;    // [rx][4]: first, last, init0, end
  uint32_t classes, fstride;
};

// Runs regex r over p[0, n) from entered set d.  inject: unanchored search (first is
// entered at every boundary); without it only the given set is followed and the run
// stops as soon as it dies out.  Sets hit on a match; returns the entered set at the end.
__device__ __forceinline__ uint64_t nfa_chunk(const NfaTables& T, uint32_t r, const uint8_t* p, uint64_t n,
                                              uint64_t d, bool inject, bool& hit) {
  const uint64_t* V = T.vec + 4 * (size_t)r;
  const uint64_t first = inject ? V[0] : 0ull, lastm = V[1];
  const uint64_t* B = T.b + (size_t)r * T.classes;
  const uint64_t* F = T.fol + (size_t)r * T.fstride;
  const uintptr_t a0 = reinterpret_cast<uintptr_t>(p);
  const uint4* q = reinterpret_cast<const uint4*>(a0 & ~(uintptr_t)15);
  uint32_t skip = (uint32_t)(a0 & 15);  // bytes of the first block before p
  uint64_t left = n;
  while (left) {
    if (!inject && d == 0) return 0;
    const uint4 v = *q++;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint64_t bm[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) bm[j] = B[T.cls[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu]];
    const uint32_t j0 = skip;
    const uint32_t j1 = (uint64_t)(16 - skip) < left ? 16u : skip + (uint32_t)left;
    left -= j1 - j0;
    skip = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      if (j < j0 || j >= j1) continue;
      const uint64_t c = d & bm[j];
      if (c & lastm) { hit = true; return 0; }
      uint64_t nd = first;
      for (uint64_t m = c; m; m &= m - 1) nd |= F[__ffsll((unsigned long long)m) - 1];
      d = nd;
    }
  }
  return d;
}

// One wave decides regex r on content p[0, n): the content is cut into <= 64 chunks
// (16-B multiples), every lane runs its chunk from the fresh state (init0 for chunk 0,
// `first` otherwise; every reachable state contains `first`).  The transition is a union
// homomorphism (delta(A u B) = delta(A) u delta'(B), delta' without the injection of
// `first`), so the partial matches crossing chunk boundaries are then followed by extra
// runs of delta' from the boundary states, rounds until no extra state survives a chunk.
__device__ bool nfa_wave(const NfaTables& T, uint32_t r, const uint8_t* p, uint64_t n, int lane) {
  const uint64_t* V = T.vec + 4 * (size_t)r;
  const uint64_t first = V[0];
  uint64_t L = (n + 63) / 64;
  L = (L + 15) & ~15ull;
  const uint32_t nc = (uint32_t)((n + L - 1) / L);
  const bool mine = (uint32_t)lane < nc;
  const uint64_t lo = mine ? (uint64_t)lane * L : 0, hi = mine ? (lo + L < n ? lo + L : n) : 0;
  bool hit = false;
  uint64_t e = 0;
  if (mine) e = nfa_chunk(T, r, p + lo, hi - lo, lane == 0 ? V[2] : first, true, hit);
  if (__any(hit)) return true;
  uint64_t fin = (uint32_t)lane == nc - 1 ? e : 0;  // entered set after the last byte
  uint64_t x = __shfl_up(e & ~first, 1, 64);
  if (lane == 0 || !mine) x = 0;
  for (int round = 0; round < 64 && __any(x != 0); ++round) {
    uint64_t y = 0;
    if (x) y = nfa_chunk(T, r, p + lo, hi - lo, x, false, hit);
    if (__any(hit)) return true;
    if ((uint32_t)lane == nc - 1) fin |= y;
    x = __shfl_up(y, 1, 64);
    if (lane == 0 || !mine) x = 0;
  }
  const uint64_t f = __shfl(fin, (int)nc - 1, 64);
  return (f & V[3]) != 0;
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_nfa(RunArgs a) {
  extern __shared__ uint64_t s_nfa[];
  if (a.counters[2] || a.counters[kCtrQOver] || a.counters[kCtrHitsOver]) return;  // k_match decides
  const uint32_t nq = a.counters[kCtrQueue] < a.cand_cap ? a.counters[kCtrQueue] : a.cand_cap;
  if (nq == 0 || blockIdx.x * (blockDim.x / 64) >= nq) return;  // one wave per candidate
  const DevPatterns& P = a.pats;
  const uint32_t R = P.rx_count, C = P.rx_classes, FS = LDS ? P.rx_maxpos : 64;
  NfaTables T;
  if (LDS) {
    uint64_t* sb = s_nfa;                      // [R][C]
    uint64_t* sf = sb + (size_t)R * C;          // [R][FS]
    uint64_t* sv = sf + (size_t)R * FS;         // [R][4]
    uint8_t* sc = reinterpret_cast<uint8_t*>(sv + 4 * (size_t)R);
    for (uint32_t i = threadIdx.x; i < R * C; i += blockDim.x) sb[i] = P.rx_b[i];
    for (uint32_t i = threadIdx.x; i < R * FS; i += blockDim.x) sf[i] = P.rx_follow[(size_t)(i / FS) * 64 + i % FS];
    for (uint32_t i = threadIdx.x; i < R; i += blockDim.x) {
      sv[4 * i] = P.rx_first[i];
      sv[4 * i + 1] = P.rx_last[i];
      sv[4 * i + 2] = P.rx_init0[i];
      sv[4 * i + 3] = P.rx_end[i];
    }
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) sc[i] = P.rx_class[i];
    __syncthreads();
    T = NfaTables{sc, sb, sf, sv, C, FS};
  } else {
    T = NfaTables{P.rx_class, P.rx_b, P.rx_follow, P.rx_vec, C, 64};
  }
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < nq; i += nw) {
    const uint64_t e = a.cand[2 * (size_t)i];
    const uint64_t l = e & ((1ull << 40) - 1);
    const uint32_t r = (uint32_t)(e >> 40);
    if (P.rx_pre[r] != kRxPreNone) continue;  // bounded window: k_nfa_win
    const uint32_t s = (uint32_t)(a.cand[2 * (size_t)i + 1] >> 40);  // (k_verify: the stream)
    if (!a.count_pats && ((a.bits[l >> 5] >> (l & 31)) & 1u)) continue;
    const uint16_t m = a.meta[l];
    if (!(m & Meta::kParsed)) continue;
    const uint8_t* segp = a.bytes + a.segs[s].base;
    const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
    const uint32_t plen = line_plen(a, m, segp, ls, le);
    uint64_t cs = ls + plen, ce = le;
    if (ce > cs && segp[ce - 1] == '\n') --ce;
    if (ce <= cs) continue;  // factor-bearing regexes never match empty content
    const bool hit = (P.rx_flags[r] & 1u) || nfa_wave(T, r, segp + cs, ce - cs, lane);
    if (hit && lane == 0) {
      atomicOr(&a.bits[l >> 5], 1u << (l & 31));
      if (a.count_pats) count_pair(a, l, s, P.n_lits + r);
    }
  }
}

// Per-pattern counts of the lines k_fixup decided (non-canonical timestamp prefix, general
// sets): k_fixup runs before the tile line bases exist, so the counting pass over those
// lines runs here, one wave per tile that deferred a line, once the line index is built.
__global__ __launch_bounds__(256) void k_fixcount(RunArgs a) {
  if (!a.counters[kCtrDefer] || a.counters[2]) return;
  if (a.win_index) {  // the deferred lines' bounds need the whole index: the host reruns with it
    if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[kCtrRedo] = 1u;
    return;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t tile = blockIdx.x * 4 + wv; tile < a.ntiles; tile += gridDim.x * 4) {
    const TileStat ts = a.tstat[tile];
    if (!(ts.flags & 4u)) continue;
    const uint32_t s = a.tile_seg[tile];
    const SegDesc sd = a.segs[s];
    const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
    const bool first = rel_lo == 0, last = rel_lo + kTile >= (int64_t)sd.len;
    const uint32_t k0 = first ? 0 : 1, k1 = last ? ts.events : ts.events + 1;
    const uint32_t nlines = k1 > k0 ? k1 - k0 : 0;
    const uint32_t* list = slot_list(a, ts, tile);
    const uint8_t* segp = a.bytes + sd.base;
    for (uint32_t j = lane; j < nlines; j += 64) {
      const uint32_t sl = list[j];
      if (!(sl & kSlotDefer) || !(sl & kSlotHit)) continue;  // only deferred lines that matched
      const uint64_t l = a.tile_base[tile] + k0 + j;
      if (l >= a.cap_lines) continue;  // overflowing run (counters[2]): rerun with the exact size
      const uint16_t m = a.meta[l];
      const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
      const uint64_t cs = ls + line_plen(a, m, segp, ls, le);
      uint64_t ce = le;
      if (ce > cs && segp[ce - 1] == '\n') --ce;
      if (ce > cs) general_count(a, segp + cs, (int64_t)(ce - cs), l, s);
    }
  }
}

// K2c: the windowed NFA (regexes whose factor set bounds the match start, rx_pre): one
// thread per candidate occurrence x.  Matches holding that occurrence start in
// [x - rx_pre, x]; the run enters `first` only up to x and stops as soon as the entered
// set dies (or at the content's end, where the EOT closure decides).  Every match holds
// its first factor occurrence and every occurrence is a candidate, so the union of the
// windows decides the line (klf_patterns.cpp nfa_window is the host twin).  Tens of bytes
// per candidate instead of the whole (1-32 KiB) line.
template <bool LDS>
__global__ __launch_bounds__(256) void k_nfa_win(RunArgs a) {
  extern __shared__ uint64_t s_nfa[];
  if (a.counters[2] || a.counters[kCtrQOver] || a.counters[kCtrHitsOver]) return;
  const uint32_t nq = a.counters[kCtrQueue] < a.cand_cap ? a.counters[kCtrQueue] : a.cand_cap;
  if (nq == 0) return;
  const DevPatterns& P = a.pats;
  const uint32_t R = P.rx_count, C = P.rx_classes, FS = LDS ? P.rx_maxpos : 64;
  NfaTables T;
  if (LDS) {
    uint64_t* sb = s_nfa;
    uint64_t* sf = sb + (size_t)R * C;
    uint64_t* sv = sf + (size_t)R * FS;
    uint8_t* sc = reinterpret_cast<uint8_t*>(sv + 4 * (size_t)R);
    for (uint32_t i = threadIdx.x; i < R * C; i += blockDim.x) sb[i] = P.rx_b[i];
    for (uint32_t i = threadIdx.x; i < R * FS; i += blockDim.x) sf[i] = P.rx_follow[(size_t)(i / FS) * 64 + i % FS];
    for (uint32_t i = threadIdx.x; i < R; i += blockDim.x) {
      sv[4 * i] = P.rx_first[i];
      sv[4 * i + 1] = P.rx_last[i];
      sv[4 * i + 2] = P.rx_init0[i];
      sv[4 * i + 3] = P.rx_end[i];
    }
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) sc[i] = P.rx_class[i];
    __syncthreads();
    T = NfaTables{sc, sb, sf, sv, C, FS};
  } else {
    T = NfaTables{P.rx_class, P.rx_b, P.rx_follow, P.rx_vec, C, 64};
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += gridDim.x * blockDim.x) {
    const uint64_t e = a.cand[2 * (size_t)i];
    const uint64_t l = e & ((1ull << 40) - 1);
    const uint32_t r = (uint32_t)(e >> 40);
    const uint32_t pre = P.rx_pre[r];
    if (pre == kRxPreNone) continue;  // k_nfa runs those over the whole line
    if (!a.count_pats && ((a.bits[l >> 5] >> (l & 31)) & 1u)) continue;
    const uint16_t m = a.meta[l];
    if (!(m & Meta::kParsed)) continue;
    const uint64_t xs = a.cand[2 * (size_t)i + 1];
    const uint32_t s = (uint32_t)(xs >> 40);  // (k_verify: the stream, no search of the segments)
    const uint64_t x = xs & ((1ull << 40) - 1);
    const uint8_t* segp = a.bytes + a.segs[s].base;
    const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
    const uint64_t cs = ls + line_plen(a, m, segp, ls, le);
    uint64_t ce = le;
    if (ce > cs && segp[ce - 1] == '\n') --ce;
    if (x < cs || x >= ce) continue;  // an occurrence in the timestamp prefix: no match holds it
    bool hit = (P.rx_flags[r] & 1u) != 0;
    if (!hit && !(KLF_ABL & 32768)) {  // (timing build 32768: no window runs)
      const uint64_t* V = T.vec + 4 * (size_t)r;
      const uint64_t first = V[0], lastm = V[1];
      const uint64_t* B = T.b + (size_t)r * T.classes;
      const uint64_t* F = T.fol + (size_t)r * T.fstride;
      const uint64_t ws = x - cs > pre ? x - pre : cs;
      uint64_t d = ws == cs ? V[2] : first;
      uint64_t p = ws;  // the next byte to run
      // the window's bytes 16 at a time (aligned loads; segments are 256-B aligned and the
      // batch has read slack past its end): one load round trip per 16 bytes, not per byte
      for (uint64_t q = ws & ~15ull; q < ce && d && !hit; q += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(segp + q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (q + j != p || p >= ce || !d || hit) continue;
          const uint64_t c = d & B[T.cls[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu]];
          if (c & lastm) { hit = true; continue; }
          uint64_t nd = p + 1 <= x ? first : 0ull;
          for (uint64_t mm = c; mm; mm &= mm - 1) nd |= F[__ffsll((unsigned long long)mm) - 1];
          d = nd;
          ++p;
        }
      }
      if (!hit && p == ce) hit = (d & V[3]) != 0;
    }
    if (hit) {
      atomicOr(&a.bits[l >> 5], 1u << (l & 31));
      if (a.count_pats) count_pair(a, l, s, P.n_lits + r);
    }
  }
}

// Per line: kGrepAll marks every parsed line; general sets are evaluated here when the
// prefilter is off or its lists overflowed, and with match_all (an always-pattern in the
// set, run with per-pattern counts) every parsed line is marked after the matchers.
__global__ __launch_bounds__(256) void k_match(RunArgs a) {
  if (a.counters[2]) return;
  const bool prefiltered =
      a.grep_mode == kGrepGeneral && a.pats.qf_on && !a.counters[kCtrQOver] && !a.counters[kCtrHitsOver];
  if (prefiltered && !a.match_all) return;
  if (a.win_index) {  // every line's index is needed: the host reruns with the whole index
    if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[kCtrRedo] = 1u;
    return;
  }
  const uint64_t L = a.segout[a.nsegs - 1].line_hi;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < L; l += stride) {
    const uint16_t m = a.meta[l];
    if (!(m & Meta::kParsed)) continue;
    bool hit = a.grep_mode == kGrepAll || (prefiltered && a.match_all);
    if (!hit) {
      const uint32_t s = find_seg_by_line(a.segout, a.nsegs, l);
      const uint8_t* segp = a.bytes + a.segs[s].base;
      const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
      const uint32_t plen = line_plen(a, m, segp, ls, le);
      uint64_t cs = ls + plen, ce = le;
      if (ce > cs && segp[ce - 1] == '\n') --ce;
      const uint8_t* p = segp + cs;
      const int64_t n = (int64_t)(ce - cs);
      if (a.count_pats) {
        hit = general_count(a, p, n, l, s);
      } else {
        if (a.pats.ac_states) hit = ac_match(a.pats, p, n);
        for (uint32_t r = 0; !hit && r < a.pats.rx_count; ++r) hit = rx_match(a.pats, r, p, n);
      }
      hit |= a.match_all != 0;
    }
    if (hit) atomicOr(&a.bits[l >> 5], 1u << (l & 31));
  }
}

// ============================================================== K3: per-stream counts ==
// parsed / since_ok come from k_tbase's prefixes.  matched = popcount of the match
// bitmap per stream: one partial per 8192-line chunk for the stream the chunk starts in
// (mpart[c], no atomics), the chunk's lines of the next stream as one block atomic, and
// per-thread atomics only for streams shorter than a chunk.  k_tail adds the partials of
// the chunks that start inside its stream.
__device__ __forceinline__ uint32_t word_range_mask(uint64_t w, uint64_t lo, uint64_t hi) {
  // bits of word w (lines 32w .. 32w+31) inside [lo, hi)
  const uint64_t l0 = w * 32;
  uint32_t m = ~0u;
  if (l0 < lo) m &= lo - l0 >= 32 ? 0u : (~0u << (lo - l0));
  if (l0 + 32 > hi) m &= hi <= l0 ? 0u : ((1u << (hi - l0)) - 1u);
  return m;
}

__global__ __launch_bounds__(256) void k_mcount(RunArgs a) {
  __shared__ uint64_t s_acc[2][4];
  if (a.counters[2]) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint64_t L = a.segout[a.nsegs - 1].line_hi;
  const uint64_t nchunks = (L + kMatchChunk - 1) / kMatchChunk;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint64_t l0 = c * kMatchChunk;
    const uint32_t s0 = find_seg_by_line(a.segout, a.nsegs, l0);
    const uint64_t hi0 = a.segout[s0].line_hi;
    const uint64_t w = c * (kMatchChunk / 32) + t;
    uint64_t v0 = 0, v1 = 0;
    if (w * 32 < L) {
      const uint32_t word = a.bits[w] & word_range_mask(w, 0, L);
      v0 = __popc(word & word_range_mask(w, 0, hi0));
      uint32_t rest = word & ~word_range_mask(w, 0, hi0);
      for (uint32_t s = s0 + 1; rest && s < a.nsegs; ++s) {
        const uint32_t part = rest & word_range_mask(w, a.segout[s].line_lo, a.segout[s].line_hi);
        rest &= ~part;
        if (s == s0 + 1) v1 += __popc(part);
        else if (part) atomicAdd((unsigned long long*)&a.segout[s].matched, (unsigned long long)__popc(part));
      }
    }
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    __syncthreads();
    if (lane == 0) { s_acc[0][wv] = v0; s_acc[1][wv] = v1; }
    __syncthreads();
    if (t == 0) {
      a.mpart[c] = s_acc[0][0] + s_acc[0][1] + s_acc[0][2] + s_acc[0][3];
      const uint64_t x1 = s_acc[1][0] + s_acc[1][1] + s_acc[1][2] + s_acc[1][3];
      if (x1) atomicAdd((unsigned long long*)&a.segout[s0 + 1].matched, (unsigned long long)x1);
    }
  }
}

// ==================================================== K3: tail window (one block/stream) ==
__device__ __forceinline__ bool gbit(const RunArgs& a, uint64_t l) {
  return a.grep_mode == kGrepNone ? true : ((a.bits[l >> 5] >> (l & 31)) & 1u);
}

__device__ uint32_t block_incl_scan_u32(uint32_t x, uint32_t* s_w, uint32_t* total) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t inc = wave_incl_scan_add(x, lane);
  __syncthreads();
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t pre = 0;
  for (int k = 0; k < wv; ++k) pre += s_w[k];
  *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  return inc + pre;
}

__device__ uint64_t block_sum_u64(uint64_t x, uint64_t* s_w) {
  const int t = threadIdx.x;
  x = wave_sum(x);
  __syncthreads();
  if ((t & 63) == 0) s_w[t >> 6] = x;
  __syncthreads();
  return s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

constexpr uint64_t kNone = ~0ull;

// The k-th (k >= 1) set bit of the match bitmap counted backwards from hi - 1 within
// [lo, hi): 256 words (8192 lines) per step, one word per thread (thread 0 = top word).
__device__ uint64_t select_back_bits(const uint32_t* bits, uint64_t lo, uint64_t hi, uint64_t k, uint32_t* s_w,
                                     uint64_t* s_res) {
  const int t = threadIdx.x;
  __syncthreads();
  if (t == 0) *s_res = kNone;
  if (hi <= lo || k == 0) { __syncthreads(); return kNone; }
  const int64_t wlo = (int64_t)(lo >> 5), whi = (int64_t)((hi - 1) >> 5);
  uint64_t cum = 0;
  for (int64_t top = whi; top >= wlo; top -= 256) {
    const int64_t w = top - t;
    uint32_t word = 0;
    if (w >= wlo) word = bits[w] & word_range_mask((uint64_t)w, lo, hi);
    const uint32_t c = (uint32_t)__popc(word);
    uint32_t tot;
    const uint32_t incl = block_incl_scan_u32(c, s_w, &tot);
    if (cum + tot >= k) {
      if (c && cum + incl >= k && cum + incl - c < k) {
        const uint32_t needc = (uint32_t)(k - (cum + incl - c));
        for (uint32_t i = 1; i < needc; ++i) word &= ~(1u << (31 - __clz(word)));
        *s_res = (uint64_t)w * 32 + (31 - __clz(word));
      }
      break;
    }
    cum += tot;
  }
  __syncthreads();
  return *s_res;
}

// kubelet tail (SPEC.md S4) over G = matching lines (all lines without patterns):
// start = the `need`-th G line from the end, need = |G| - max(0, T - n) <= n + 1.  The
// window [start, hi) then holds need G lines; all G lines are parsed when patterns are
// given (the bitmap only marks parsed lines), so the n-th parsed G line at/after start is
// the window's second-to-last G line exactly when need = n + 1 (the trailing fragment is
// then the (n+1)-th and is cut); otherwise every selected line of the window is in.
__device__ __forceinline__ void tail_body(RunArgs& a) {
  __shared__ uint32_t s_w[4];
  __shared__ uint64_t s_w64[4];
  __shared__ uint64_t s_res;
  const uint32_t s = blockIdx.x;
  const int t = threadIdx.x;
  if (a.counters[2]) return;
  SegOut& so = a.segout[s];
  const uint64_t lo = so.line_lo, hi = so.line_hi;
  const bool grep = a.grep_mode != kGrepNone;
  uint64_t matched = hi - lo;
  if (grep) {
    uint64_t v = 0;
    const uint64_t c0 = (lo + kMatchChunk - 1) / kMatchChunk, c1 = (hi + kMatchChunk - 1) / kMatchChunk;
    for (uint64_t c = c0 + t; c < c1; c += 256) v += a.mpart[c];
    matched = block_sum_u64(v, s_w64) + so.matched;
  }
  __syncthreads();
  if (t == 0) {
    so.parsed = so.p_hi - so.p_lo;
    so.since_ok = so.q_hi - so.q_lo;
    so.matched = matched;
  }
  if (a.tail < 0) {
    if (t == 0) { so.win_lo = lo; so.win_hi = hi; }
    return;
  }
  const uint64_t n = (uint64_t)a.tail;
  const uint64_t gsize = matched;
  const uint64_t gfrag = (so.frag && hi > lo && gbit(a, hi - 1)) ? 1 : 0;
  const uint64_t T = gsize - gfrag;
  const uint64_t k = T > n ? T - n : 0;
  const uint64_t need = gsize - k;
  if (need == 0 || n == 0) {  // n = 0 emits nothing (ReadLogs stops before the first line)
    if (t == 0) { so.win_lo = hi; so.win_hi = hi; }
    return;
  }
  uint64_t start, end = hi;
  if (grep) {
    start = select_back_bits(a.bits, lo, hi, need, s_w, &s_res);
    if (need == n + 1) end = select_back_bits(a.bits, start, hi - 1, 1, s_w, &s_res) + 1;
  } else {
    start = hi - need;
    if (need == n + 1) {  // cut the fragment only if every line of the window is parsed
      uint32_t bad = 0;
      for (uint64_t l = start + t; l < hi; l += 256) bad |= (a.meta[l] & Meta::kParsed) ? 0u : 1u;
      if (__syncthreads_or(bad) == 0) end = hi - 1;
    }
  }
  if (t == 0) { so.win_lo = start; so.win_hi = end; }
}

__device__ __forceinline__ void wprefix_body(RunArgs& a) {
  __shared__ uint64_t s_w64[4];
  if (a.counters[2]) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint64_t carry = 0;
  for (uint32_t b = 0; b < a.nsegs; b += 256) {
    const uint32_t s = b + t;
    const uint64_t v = s < a.nsegs ? a.segout[s].win_hi - a.segout[s].win_lo : 0;
    const uint64_t inc = wave_incl_scan_add(v, lane);
    __syncthreads();
    if (lane == 63) s_w64[wv] = inc;
    __syncthreads();
    uint64_t pre = 0;
    for (int k = 0; k < wv; ++k) pre += s_w64[k];
    const uint64_t tot = s_w64[0] + s_w64[1] + s_w64[2] + s_w64[3];
    if (s < a.nsegs) a.wpre[s] = carry + pre + inc - v;
    carry += tot;
  }
  const uint64_t nb0 = (carry + kCompactLines - 1) / kCompactLines;
  const uint32_t nb = (uint32_t)(nb0 < a.max_cblocks ? nb0 : a.max_cblocks);
  // Compaction path: tile copy (k_tkeep / k_tcopy) when at least a quarter of the lines
  // can be selected (every window line that is since_ok and matching at most), else the
  // line gather (k_csum / k_cscan / k_cgather), which touches only the selected lines.
  uint64_t est = 0;
  for (uint32_t s = t; s < a.nsegs; s += 256) {
    const SegOut& so = a.segout[s];
    uint64_t w = so.win_hi - so.win_lo;
    w = w < so.since_ok ? w : so.since_ok;
    if (a.grep_mode != kGrepNone) w = w < so.matched ? w : so.matched;
    est += w;
  }
  est = block_sum_u64(est, s_w64);
  const uint64_t L = a.segout[a.nsegs - 1].line_hi;
  const bool dense = a.compact_mode == 2 || (a.compact_mode == 0 && L > 0 && est * 4 >= L);
  if (t == 0) {
    a.wpre[a.nsegs] = carry;
    a.counters[3] = nb;
    a.counters[kCtrDense] = dense ? 1u : 0u;
  }
}

// Re-tail (klf_retail): clears what k_mcount .. k_cgather accumulate into the segment
// records, leaving the line index, the parse/since counts and the match bitmap of the run.
__global__ __launch_bounds__(256) void k_retail_init(RunArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.counters[kCtrTailDone] = 0;  // k_tailw's tickets
    a.counters[kCtrPlanDone] = 0;  // k_cplan's
    a.counters[kCtrOutShort] = 0;
  }
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < a.nsegs; s += gridDim.x * 256) {
    SegOut& so = a.segout[s];
    so.matched = 0;
    so.win_lo = so.win_hi = 0;
    so.sel_lo = so.sel_hi = 0;
    so.out_lo = so.out_hi = 0;
  }
}

// Zeroes the run's counters and per-stream records (one launch instead of memsets).
__global__ __launch_bounds__(256) void k_init(RunArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < kNumCounters) a.counters[i] = 0;
  const uint32_t nw = a.nsegs * (uint32_t)(sizeof(SegOut) / 8);
  uint64_t* so = reinterpret_cast<uint64_t*>(a.segout);
  for (uint32_t k = i; k < nw; k += gridDim.x * 256) so[k] = 0;
}

// ======================================================= K4: compaction + gather copy ==
// Reduce-then-scan over blocks of kCompactLines window lines (no inter-block waiting):
//   k_csum    per block: selected content bytes and selected lines -> csum[3 * blk]
//   k_cscan   one block: exclusive scan of the block sums (in place)
//   k_cgather per block: in-block scan + block base -> output offsets, stream output
//             ranges, gather copy of the selected contents (prefix stripped)
// Thread t of a block owns window lines blk * kCompactLines + 4t .. 4t + 3.
struct WinLines {
  uint64_t src[4];
  uint32_t len[4], seg[4];
  bool first[4], last[4], sel[4];  // sel: selected (a fragment's content may be empty)
  uint64_t bytes;
  uint32_t nsel;
};

// s_lo: a stream at or before the one holding window line w0 (0 = unknown; k_csum
// records each block's first stream so that k_cgather's search starts there)
__device__ __forceinline__ void window_lines(const RunArgs& a, uint64_t w0, uint64_t W, WinLines& r,
                                             uint32_t s_lo = 0) {
  uint32_t s = 0;
  {
    const uint64_t wq = w0 < W ? w0 : (W ? W - 1 : 0);
    uint32_t lo = s_lo, hi = a.nsegs;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.wpre[mid] <= wq) lo = mid; else hi = mid;
    }
    s = lo;
  }
  r.bytes = 0;
  r.nsel = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t wj = w0 + j;
    r.len[j] = 0; r.src[j] = 0; r.first[j] = r.last[j] = r.sel[j] = false; r.seg[j] = s;
    if (wj >= W) continue;
    while (wj >= a.wpre[s + 1]) ++s;
    r.seg[j] = s;
    r.first[j] = wj == a.wpre[s];
    r.last[j] = wj + 1 == a.wpre[s + 1];
    const uint64_t l = a.segout[s].win_lo + (wj - a.wpre[s]);
    const uint16_t m = a.meta[l];
    const bool sel = (m & Meta::kParsed) && (m & Meta::kSince) && gbit(a, l);
    r.sel[j] = sel;
    if (sel) {
      const uint8_t* segp = a.bytes + a.segs[s].base;
      const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
      const uint32_t plen = line_plen(a, m, segp, ls, le);
      r.src[j] = a.segs[s].base + ls + plen;
      r.len[j] = (uint32_t)(le - ls - plen);
      r.bytes += r.len[j];
      ++r.nsel;
    }
  }
}

constexpr uint32_t kCsegBoundary = 0x80000000u;  // cseg flag: block holds a stream's first/last window line

// (compaction blocks b0, b0 + bstep, ...: k_cplan's grid, or all of them in one block)
__device__ __forceinline__ void csum_body(RunArgs& a, uint32_t b0, uint32_t bstep) {
  __shared__ uint64_t s_wb[4], s_wc[4];
  __shared__ uint32_t s_wf[4];
  if (a.counters[2] || a.counters[kCtrDense]) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint64_t W = a.wpre[a.nsegs];
  const uint32_t nblocks = a.counters[3];
  for (uint32_t blk = b0; blk < nblocks; blk += bstep) {
    WinLines r;
    window_lines(a, (uint64_t)blk * kCompactLines + (uint64_t)t * 4, W, r);
    const uint64_t b = wave_sum(r.bytes), c = wave_sum((uint64_t)r.nsel);
    // does the block hold a stream's first or last window line? (k_cgather records the
    // stream's output range there, so such a block gets a copy chunk even with no bytes)
    const bool bnd = __any(r.first[0] || r.first[1] || r.first[2] || r.first[3] || r.last[0] || r.last[1] ||
                           r.last[2] || r.last[3]);
    __syncthreads();
    if (lane == 0) { s_wb[wv] = b; s_wc[wv] = c; s_wf[wv] = bnd ? 1u : 0u; }
    __syncthreads();
    if (t == 0) {
      a.csum[3 * blk] = s_wb[0] + s_wb[1] + s_wb[2] + s_wb[3];
      a.csum[3 * blk + 1] = s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
      a.cseg[blk] = r.seg[0] | ((s_wf[0] | s_wf[1] | s_wf[2] | s_wf[3]) ? kCsegBoundary : 0u);
    }
  }
}

// Exclusive prefixes of the block sums (bytes, lines) and of the copy chunks per block
// (ceil(bytes / kCopyChunk); 0 or 1 for an empty block): long selected lines spread their copy over many
// workgroups instead of the one that owns their 1024-line block.
__device__ __forceinline__ void cscan_body(RunArgs& a) {
  __shared__ uint64_t s_wb[4], s_wc[4], s_wk[4];
  if (a.counters[2] || a.counters[kCtrDense]) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nb = a.counters[3];
  __shared__ uint32_t s_lg;
  const uint32_t per = (nb + 255) / 256;
  const uint32_t i0 = t * per, i1 = i0 + per < nb ? i0 + per : nb;
  uint64_t b = 0, c = 0, k = 0;
  for (uint32_t i = i0; i < i1; ++i) { b += a.csum[3 * i]; c += a.csum[3 * i + 1]; }
  const uint64_t ib = wave_incl_scan_add(b, lane), ic = wave_incl_scan_add(c, lane);
  if (lane == 63) { s_wb[wv] = ib; s_wc[wv] = ic; }
  __syncthreads();
  if (t == 0) {  // this run's copy chunk (kCopyChunksTarget)
    const uint64_t total = s_wb[0] + s_wb[1] + s_wb[2] + s_wb[3];
    uint32_t lg = kCopyChunkMinLog2;
    while ((1ull << lg) < kCopyChunk && (total >> lg) >= kCopyChunksTarget) ++lg;
    s_lg = lg;
    a.counters[kCtrChunkLog2] = lg;
  }
  __syncthreads();
  const uint32_t lg = s_lg;
  // a block with no output bytes gets a chunk only when it holds a stream boundary (C2:
  // hundreds of empty blocks in the --since window, two of them with work)
  auto chunks = [&](uint64_t bytes, uint32_t i) -> uint64_t {
    return bytes ? (bytes + (1ull << lg) - 1) >> lg : ((a.cseg[i] & kCsegBoundary) ? 1 : 0);
  };
  for (uint32_t i = i0; i < i1; ++i) k += chunks(a.csum[3 * i], i);
  const uint64_t ik = wave_incl_scan_add(k, lane);
  if (lane == 63) s_wk[wv] = ik;
  __syncthreads();
  uint64_t pb = ib - b, pc = ic - c, pk = ik - k;
  for (int w = 0; w < wv; ++w) { pb += s_wb[w]; pc += s_wc[w]; pk += s_wk[w]; }
  for (uint32_t i = i0; i < i1; ++i) {
    const uint64_t xb = a.csum[3 * i], xc = a.csum[3 * i + 1];
    a.csum[3 * i] = pb;
    a.csum[3 * i + 1] = pc;
    a.csum[3 * i + 2] = pk;
    const uint64_t nk = chunks(xb, i);
    for (uint64_t k = 0; k < nk && pk + k < a.cmap_cap; ++k) a.cmap[pk + k] = i;  // chunk -> block
    pb += xb;
    pc += xc;
    pk += nk;
  }
  if (t == 255) {
    a.csum[3 * nb] = pb;  // total output bytes
    a.csum[3 * nb + 2] = pk;
    a.counters[kCtrCopyChunks] = (uint32_t)pk;
  }
}

// 16 bytes starting at byte offset o (0..15) of the 32-byte window w[0..7].
__device__ __forceinline__ uint4 extract16(const uint4& lo, const uint4& hi, uint32_t o) {
  const uint32_t q = o >> 2, r = (o & 3u) * 8u;
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t x[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)  // x[k] = w[q + k] without dynamic register indexing
    x[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[(k + 3) & 7];
  uint32_t y[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = (uint32_t)((((uint64_t)x[k + 1] << 32) | x[k]) >> r);
  return make_uint4(y[0], y[1], y[2], y[3]);
}
__device__ __forceinline__ uint32_t byte_mask(int b0, int b1, int k) {
  // bytes [b0, b1) of the chunk that fall in dword k, as a byte mask
  int lo = b0 - 4 * k, hi = b1 - 4 * k;
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
  const uint32_t mh = hi >= 4 ? ~0u : ((1u << (8 * hi)) - 1u);
  const uint32_t ml = lo >= 4 ? ~0u : ((1u << (8 * lo)) - 1u);
  return mh & ~ml;
}

// Copies the block's selected contents (LDS tables, output range [ob0, ob1)) with one
// 16-B output chunk per thread and step: coalesced 16-B stores; each line piece of a chunk
// is read as an aligned 32-byte window and byte-shifted into place.  Chunks shared with a
// neighbouring block are written bytewise (only this block's bytes).
__device__ void block_gather_copy(const uint64_t* s_src, const uint64_t* s_dst, const uint32_t* s_len,
                                  const uint16_t* s_map, uint64_t ob0, uint64_t ob1, const uint8_t* __restrict__ src,
                                  uint8_t* __restrict__ dst) {
  if (ob1 <= ob0) return;
  const uint64_t c0 = ob0 >> 4, c1 = (ob1 + 15) >> 4;
  // U output chunks per thread and step, their source loads all in flight before the
  // first is merged (the copy is latency-bound otherwise: a 16-B chunk per round trip)
  constexpr int U = KLF_COPY_U;
  auto piece = [&](uint32_t (&o)[4], int64_t ad0, const uint4& va, const uint4& vb, int b0, int b1)
      __attribute__((always_inline)) {
    if (ad0 >= 16) {
      const uint64_t base = (uint64_t)ad0 & ~15ull;
      const uint4 v = extract16(va, vb, (uint32_t)(ad0 - (int64_t)base));
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t m = byte_mask(b0, b1, k);
        o[k] = (vv[k] & m) | (o[k] & ~m);
      }
    } else {
      for (int b = b0; b < b1; ++b) {
        const uint32_t byte = src[ad0 + b];
        o[b >> 2] = (o[b >> 2] & ~(0xFFu << (8 * (b & 3)))) | (byte << (8 * (b & 3)));
      }
    }
  };
  for (uint64_t cb = c0 + threadIdx.x; cb < c1; cb += (uint64_t)U * blockDim.x) {
    uint4 va[U], vb[U], wa[U], wb[U];
    int liu[U], li2u[U];
    uint64_t pend0[U];
    int64_t a0[U], a1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // locate the first piece of every chunk, issue its loads
      const uint64_t c = cb + (uint64_t)u * blockDim.x;
      va[u] = vb[u] = make_uint4(0, 0, 0, 0);
      liu[u] = 0;
      pend0[u] = 0;
      a0[u] = 0;
      if (c >= c1) continue;
      const uint64_t d0 = c << 4;
      const uint64_t hi = d0 + 16 < ob1 ? d0 + 16 : ob1;
      const int li = s_map[c - c0];  // the line holding the chunk's first byte in [ob0, ob1)
      liu[u] = li;
      pend0[u] = s_dst[li] + s_len[li] < hi ? s_dst[li] + s_len[li] : hi;
      a0[u] = (int64_t)s_src[li] - (int64_t)s_dst[li] + (int64_t)d0;  // source of chunk byte 0
      if (a0[u] >= 16) {
        const uint4* wp = reinterpret_cast<const uint4*>(src + ((uint64_t)a0[u] & ~15ull));
        va[u] = wp[0];
        vb[u] = wp[1];
      }
      // the chunk's second piece (a line ends inside it: ~1 chunk in 8 at 120-B lines, so
      // almost every wave step has a lane with one) is loaded now too, not after the first
      // merge: one memory round trip per step instead of two
      wa[u] = wb[u] = make_uint4(0, 0, 0, 0);
      li2u[u] = li;
      a1[u] = 0;
      if (KLF_CG_PF2 && pend0[u] < hi) {
        int l2 = li + 1;
        while (s_len[l2] == 0) ++l2;  // the bytes at pend0 < hi belong to a later non-empty line
        li2u[u] = l2;
        a1[u] = (int64_t)s_src[l2] - (int64_t)s_dst[l2] + (int64_t)d0;
        if (a1[u] >= 16) {
          const uint4* wp = reinterpret_cast<const uint4*>(src + ((uint64_t)a1[u] & ~15ull));
          wa[u] = wp[0];
          wb[u] = wp[1];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t c = cb + (uint64_t)u * blockDim.x;
      if (c >= c1) continue;
      const uint64_t d0 = c << 4;
      const uint64_t lo = d0 > ob0 ? d0 : ob0, hi = d0 + 16 < ob1 ? d0 + 16 : ob1;
      uint32_t o[4] = {0, 0, 0, 0};
      piece(o, a0[u], va[u], vb[u], (int)(lo - d0), (int)(pend0[u] - d0));
      int li = liu[u];
      uint64_t pos = pend0[u];
      if (KLF_CG_PF2 && pos < hi) {
        li = li2u[u];
        const uint64_t pend = s_dst[li] + s_len[li] < hi ? s_dst[li] + s_len[li] : hi;
        piece(o, a1[u], wa[u], wb[u], (int)(pos - d0), (int)(pend - d0));
        pos = pend;
      }
      while (pos < hi) {  // further lines inside the chunk (short lines)
        while (s_dst[li] + s_len[li] <= pos) ++li;
        const uint64_t pend = s_dst[li] + s_len[li] < hi ? s_dst[li] + s_len[li] : hi;
        const int64_t ad0 = (int64_t)s_src[li] - (int64_t)s_dst[li] + (int64_t)d0;
        uint4 xa = make_uint4(0, 0, 0, 0), xb = xa;
        if (ad0 >= 16) {
          const uint4* wp = reinterpret_cast<const uint4*>(src + ((uint64_t)ad0 & ~15ull));
          xa = wp[0];
          xb = wp[1];
        }
        piece(o, ad0, xa, xb, (int)(pos - d0), (int)(pend - d0));
        pos = pend;
      }
      if (lo == d0 && hi == d0 + 16) {
#if KLF_CG_NT  // streaming store (written once, never re-read by this kernel)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v = {o[0], o[1], o[2], o[3]};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + d0));
#else
        *reinterpret_cast<uint4*>(dst + d0) = make_uint4(o[0], o[1], o[2], o[3]);
#endif
      } else {
        for (uint64_t pos = lo; pos < hi; ++pos) {
          const int b = (int)(pos - d0);
          dst[pos] = (uint8_t)(o[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
  }
}

__device__ __forceinline__ void cgather_body(RunArgs& a) {
  __shared__ uint64_t s_src[kCompactLines];
  __shared__ uint64_t s_dst[kCompactLines];
  __shared__ uint32_t s_len[kCompactLines];
  __shared__ uint16_t s_map[kCopyChunk / 16 + 1];
  __shared__ uint64_t s_wb[4], s_wc[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (a.counters[2] || a.counters[kCtrDense]) return;
  const uint64_t W = a.wpre[a.nsegs];
  __shared__ uint32_t s_mx[4];
  const uint32_t nblocks = a.counters[3], nchunks = a.counters[kCtrCopyChunks];
  const uint64_t cs = 1ull << a.counters[kCtrChunkLog2];  // this run's copy chunk (k_cscan)
  for (uint32_t w = blockIdx.x; w < nchunks; w += gridDim.x) {
    uint32_t blk;  // the compaction block of copy chunk w (k_cscan's map; search past its end)
    if (w < a.cmap_cap) {
      blk = a.cmap[w];
    } else {
      uint32_t lo = 0, hi = nblocks;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.csum[3 * mid + 2] <= w) lo = mid; else hi = mid;
      }
      blk = lo;
    }
    const uint32_t sub = w - (uint32_t)a.csum[3 * blk + 2];
    WinLines r;
    window_lines(a, (uint64_t)blk * kCompactLines + (uint64_t)t * 4, W, r, a.cseg[blk] & ~kCsegBoundary);
    const uint64_t ib = wave_incl_scan_add(r.bytes, lane);
    const uint64_t ic = wave_incl_scan_add((uint64_t)r.nsel, lane);
    __syncthreads();  // the previous chunk's copy is done with the LDS tables
    if (lane == 63) { s_wb[wv] = ib; s_wc[wv] = ic; }
    __syncthreads();
    uint64_t ob = a.csum[3 * blk] + ib - r.bytes, oc = a.csum[3 * blk + 1] + ic - r.nsel;
    // the block's selected lines only, compacted (k: selected lines of the block before
    // this one): a window block holds mostly unselected lines when a pattern is given (C2:
    // ~1 in 100), whose zero-length entries the chunk walks below stepped over one by one
    uint32_t k = (uint32_t)(ic - r.nsel);
    for (int w = 0; w < wv; ++w) { ob += s_wb[w]; oc += s_wc[w]; k += (uint32_t)s_wc[w]; }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (sub == 0 && r.first[j]) { a.segout[r.seg[j]].out_lo = ob; a.segout[r.seg[j]].sel_lo = oc; }
      if (r.sel[j]) {
        s_src[k] = r.src[j];
        s_dst[k] = ob;
        s_len[k] = r.len[j];
        ++k;
      }
      ob += r.len[j];
      oc += r.sel[j] ? 1 : 0;  // = k_csum's count (an empty fragment is still a line out)
      if (sub == 0 && r.last[j]) { a.segout[r.seg[j]].out_hi = ob; a.segout[r.seg[j]].sel_hi = oc; }
    }
    const uint32_t nsel_blk = (uint32_t)(s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3]);
    const uint64_t ob0 = a.csum[3 * blk];
    const uint64_t ob1 = ob0 + s_wb[0] + s_wb[1] + s_wb[2] + s_wb[3];
    const uint64_t c0 = ob0 + (uint64_t)sub * cs;
    const uint64_t c1 = c0 + cs < ob1 ? c0 + cs : ob1;
    // chunk map: 16-B output chunk k of [c0 & ~15, c1) -> the line holding its first byte
    // of [c0, c1) (every byte of the range is in exactly one line, so every chunk gets
    // exactly one writer).  Each line marks the first chunk that starts inside it, then a
    // block max-scan fills the rest (lines ascend with their output offsets): O(1) work
    // per thread whatever the line lengths.
    {
      const uint64_t cb0 = c0 >> 4;
      const uint32_t nmap = c1 > c0 ? (uint32_t)(((c1 + 15) >> 4) - cb0) : 0u;
      for (uint32_t k = (uint32_t)t; k < nmap; k += kThreads) s_map[k] = 0;
      __syncthreads();
      for (uint32_t i = (uint32_t)t; i < nsel_blk; i += kThreads) {
        const uint64_t d = s_dst[i], e = d + s_len[i];
        const uint64_t lo = d > c0 ? d : c0, hi = e < c1 ? e : c1;
        if (lo >= hi) continue;
        if (lo == c0) {
          s_map[0] = (uint16_t)i;  // c0 (16-B aligned or not) lies in line i
        } else {
          const uint64_t k = (lo + 15) >> 4;  // the first chunk starting inside the line
          if ((k << 4) < hi) s_map[k - cb0] = (uint16_t)i;
        }
      }
      __syncthreads();
      const uint32_t per = (nmap + kThreads - 1) / kThreads;
      const uint32_t m0 = (uint32_t)t * per, m1 = m0 + per < nmap ? m0 + per : nmap;
      uint32_t mx = 0;
      for (uint32_t k = m0; k < m1; ++k) mx = mx > s_map[k] ? mx : s_map[k];
      const uint32_t im = wave_incl_scan_max(mx, lane);
      if (lane == 63) s_mx[wv] = im;
      __syncthreads();
      uint32_t run = __shfl_up(im, 1);
      run = lane ? run : 0u;
      for (int k = 0; k < wv; ++k) run = run > s_mx[k] ? run : s_mx[k];
      for (uint32_t k = m0; k < m1; ++k) {
        run = run > s_map[k] ? run : s_map[k];
        s_map[k] = (uint16_t)run;
      }
    }
    __syncthreads();
    if (c1 + 16 > a.out_cap) {  // the buffer is too small: the host grows it and reruns
      if (t == 0) atomicOr(&a.counters[kCtrOutShort], 1u);
      continue;
    }
    if (!(KLF_ABL & 1024)) block_gather_copy(s_src, s_dst, s_len, s_map, c0, c1, a.bytes, a.out);
  }
}


// ============================================ K4': dense compaction (tile copy) ==
// When most lines are selected (e.g. C3: -l only, every line out) the output is the input
// minus the timestamp prefixes: a byte compaction.  It runs over the scan's 8 KiB tiles:
//   k_tkeep   wave per tile: the tile's lines (tile_base .. + events) -> its kept runs
//             (content bytes of selected lines inside the tile, with their offsets in the
//             tile's output), kept bytes and selected lines starting in it (TRec + runs)
//   k_ksum / k_kbase   reduce-then-scan of those -> each tile's output / selected-line
//             offsets, stream output ranges at the streams' first / last tiles
//   k_tcopy   wave per tile with kept bytes, the next tile's bytes and runs in flight in
//             registers: the tile goes to LDS (coalesced 16-B loads), and every 16-B output
//             chunk of the tile's output range is assembled from LDS (any alignment: five
//             dword reads + v_alignbyte) and stored with one 16-B store (coalesced across
//             the wave); only the two chunks shared with the neighbouring tiles are stored
//             bytewise.
// Input read once, output written once, the line index read once.
//
// Runs without patterns (grep none) list the lines from the scan's own per-tile line slots
// instead of the global line index (4 B per line instead of 18): line l0 + j of a tile is
// its slot j - k0 (k0 = 1 when line l0 is carried in from an earlier tile), the carried-in
// line's start and meta are the last slot of the nearest earlier tile of the stream that
// lists one (the k_scatter rule), and a line ends where the next one starts.  With
// --tail -1 the dense path then needs no line index at all (RunArgs::lazy_index).
struct TileLines {
  uint32_t s;
  SegDesc sd;
  int64_t rel_lo;  // tile start, stream-relative
  int32_t tlen;    // bytes of the stream in the tile
  uint64_t l0;     // global index of the tile's first line (the one holding its byte 0)
  uint32_t nl;     // lines holding bytes of the tile
  // grep none: the tile's slots; the carried-in line's start (stream offset) and slot word
  const uint32_t* sl;
  uint32_t k0, cslot;
  int64_t cstart;
};
__device__ __forceinline__ const uint32_t* tile_slot_list(const RunArgs& a, const TileStat& ts, uint32_t tile) {
  return slot_list(a, ts, tile);
}
// (wave-uniform) the slot fields of g, grep-none runs only.  The stream's first tile lists
// its line 0 at offset 0, so the walk back always ends at a tile with a slot.
__device__ __forceinline__ void tile_slots(const RunArgs& a, const TileStat* __restrict__ tstat, TileLines& g,
                                           uint32_t tile, const TileStat& ts) {
  g.sl = tile_slot_list(a, ts, tile);
  g.k0 = g.rel_lo == 0 ? 0u : 1u;
  g.cstart = g.rel_lo;
  g.cslot = 0;
  for (uint32_t pt = tile; g.k0 && pt > g.sd.tile0;) {
    --pt;
    const TileStat pst = tstat[pt];
    const int64_t prel = (int64_t)(pt - g.sd.tile0) * kTile;
    const uint32_t pk0 = prel == 0 ? 0u : 1u;
    const uint32_t pn = pst.events + 1 > pk0 ? pst.events + 1 - pk0 : 0u;  // never the stream's last tile
    if (pn == 0) continue;
    g.cslot = tile_slot_list(a, pst, pt)[pn - 1];
    g.cstart = prel + (int64_t)(g.cslot & kSlotOff);
    break;
  }
}
__device__ __forceinline__ TileLines tile_lines(const RunArgs& a, uint32_t tile) {
  TileLines g;
  g.s = a.tile_seg[tile];
  g.sd = a.segs[g.s];
  g.rel_lo = (int64_t)(tile - g.sd.tile0) * kTile;
  const int64_t rem = (int64_t)g.sd.len - g.rel_lo;
  g.tlen = (int32_t)(rem < kTile ? rem : kTile);
  const TileStat ts = a.tstat[tile];
  g.l0 = a.tile_base[tile];
  g.nl = rem <= kTile ? ts.events : ts.events + 1;  // the stream's end closes the last line
  if (a.grep_mode == kGrepNone) tile_slots(a, a.tstat, g, tile, ts);
  return g;
}

// The kept run of line j of tile g (lane = line): the line's index data is loaded first
// (LineData, all loads of a line in one round trip; k_tkeep loads the next tile's first
// lines ahead), then tested.  has = non-empty run.
struct LineData {
  uint64_t s0, le;  // line start / end (stream offsets)
  uint32_t bw;      // match bitmap word of the line
  uint32_t m;       // meta
};
struct LineRun {
  uint32_t src, len;  // tile offset of the run, bytes
  bool has, starts;   // non-empty run; a selected line starting in the tile
};
// Line l0 + j's data; l clamped into the index (lines past the tile are loaded but unused).
// Grep none: from the tile's slots (j clamped into the tile; the tile's last line is cut at
// the tile end, all the run needs).
__device__ __forceinline__ LineData load_line(const RunArgs& a, const TileLines& g, uint32_t j) {
  LineData d;
  d.bw = ~0u;
  if (a.grep_mode == kGrepNone) {
    const uint32_t jj = j < g.nl ? j : (g.nl ? g.nl - 1 : 0u);
    const uint32_t v = jj < g.k0 ? g.cslot : g.sl[jj - g.k0];
    d.m = v >> 16;
    d.s0 = jj < g.k0 ? (uint64_t)g.cstart : (uint64_t)(g.rel_lo + (int64_t)(v & kSlotOff));
    d.le = (uint64_t)(g.rel_lo + (jj + 1 < g.nl ? (int64_t)(g.sl[jj + 1 - g.k0] & kSlotOff) : (int64_t)g.tlen));
    return d;
  }
  uint64_t l = g.l0 + j;
  l = l < a.cap_lines ? l : a.cap_lines - 1;
  d.m = a.meta[l];
  d.s0 = a.line_off[l + g.s];
  d.le = a.line_off[l + g.s + 1];
  d.bw = a.bits[l >> 5];
  return d;
}
__device__ __forceinline__ LineRun eval_line(const RunArgs& a, const TileLines& g, uint64_t wlo, uint64_t whi,
                                             uint32_t j, const LineData& d) {
  LineRun r{0u, 0u, false, false};
  const uint64_t l = g.l0 + j;
  const bool sel = j < g.nl && l >= wlo && l < whi && (d.m & Meta::kParsed) && (d.m & Meta::kSince) &&
                   ((d.bw >> (l & 31)) & 1u);
  if (!sel) return r;
  // (a selected line is parsed: its prefix ends at its first space, so the stream end
  // bounds the search as well as the line end)
  const uint64_t cs = d.s0 + line_plen(a, (uint16_t)d.m, a.bytes + g.sd.base, d.s0, g.sd.len);
  const int64_t lo = (int64_t)cs > g.rel_lo ? (int64_t)cs : g.rel_lo;
  const int64_t hi = (int64_t)d.le < g.rel_lo + g.tlen ? (int64_t)d.le : g.rel_lo + g.tlen;
  r.has = hi > lo;
  r.src = r.has ? (uint32_t)(lo - g.rel_lo) : 0u;
  r.len = r.has ? (uint32_t)(hi - lo) : 0u;
  r.starts = (int64_t)d.s0 >= g.rel_lo && (int64_t)d.s0 < g.rel_lo + g.tlen;
  return r;
}

// Lists the tile's runs: to `runs` (at most cap entries; the count is returned whatever
// it is), with each run's offset in the tile's output.  *kept, *nsel: totals.  pre: the
// lane's line of the first group, already loaded (null: load it here).
__device__ __forceinline__ uint32_t list_runs(const RunArgs& a, const TileLines& g, uint64_t wlo, uint64_t whi,
                                              uint32_t* runs, uint32_t cap, int lane, uint32_t* kept, uint32_t* nsel,
                                              const LineData* pre = nullptr) {
  uint32_t nr = 0, dacc = 0, ns = 0;
  for (uint32_t j0 = 0; j0 < g.nl; j0 += 64) {
    const uint32_t j = j0 + (uint32_t)lane;
    const LineData d = (j0 == 0 && pre) ? *pre : load_line(a, g, j);
    const LineRun r = eval_line(a, g, wlo, whi, j, d);
    const uint32_t incl = wave_incl_scan_add(r.len, lane);
    const uint64_t bm = __ballot(r.has);
    if (r.has) {
      const uint32_t idx = nr + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
      if (idx < cap) runs[idx] = r.src | ((dacc + incl - r.len) << 16);
    }
    nr += (uint32_t)__popcll(bm);
    dacc += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    ns += (uint32_t)__popcll(__ballot(r.starts));
  }
  *kept = dacc;
  *nsel = ns;
  return nr;
}

// The per-tile descriptors come in as __restrict__ const parameters: their wave-uniform
// reads compile to scalar loads (lgkmcnt), so waiting for them never waits for the
// vector memory traffic in flight.  A wave takes kTkBatch tiles per round: the first 64
// lines' index data of all of them is loaded before any is listed (vmcnt counts loads and
// the previous round's record stores in issue order, so a round costs one memory round
// trip, not one per tile).
constexpr int kTkBatch = 4;
__device__ __forceinline__ void tkeep_body(RunArgs& a, const uint32_t* __restrict__ tseg,
                                           const SegDesc* __restrict__ segs, const TileStat* __restrict__ tstat,
                                           const uint64_t* __restrict__ tbase, const SegOut* __restrict__ sout) {
  if (a.counters[2] || !a.counters[kCtrDense] || planned(a)) return;  // (planned: the scan listed the runs)
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t t0 = (blockIdx.x * 4 + wv) * kTkBatch; t0 < a.ntiles; t0 += nw * kTkBatch) {
    TileLines g[kTkBatch];
    LineData pre[kTkBatch];
    if (a.grep_mode == kGrepNone) {
      // the batch's descriptors in phases, every load of a phase in flight together: the
      // tiles' and their predecessors' records, then the carried-in lines' slots (the last
      // slot of tile - 1; a tile without line starts before it sends the walk further back)
      TileStat ts[kTkBatch], tp[kTkBatch];
#pragma unroll
      for (int u = 0; u < kTkBatch; ++u) {
        const uint32_t tile = t0 + u < a.ntiles ? t0 + u : a.ntiles - 1;
        g[u].s = tseg[tile];
      }
#pragma unroll
      for (int u = 0; u < kTkBatch; ++u) {
        const uint32_t tile = t0 + u < a.ntiles ? t0 + u : a.ntiles - 1;
        g[u].sd = segs[g[u].s];
        g[u].l0 = tbase[tile];
        ts[u] = tstat[tile];
        tp[u] = tstat[tile > 0 ? tile - 1 : 0];
      }
      uint32_t cs[kTkBatch];
#pragma unroll
      for (int u = 0; u < kTkBatch; ++u) {
        const uint32_t tile = t0 + u < a.ntiles ? t0 + u : a.ntiles - 1;
        g[u].rel_lo = (int64_t)(tile - g[u].sd.tile0) * kTile;
        const int64_t rem = (int64_t)g[u].sd.len - g[u].rel_lo;
        g[u].tlen = (int32_t)(rem < kTile ? rem : kTile);
        g[u].nl = rem <= kTile ? ts[u].events : ts[u].events + 1;
        g[u].sl = tile_slot_list(a, ts[u], tile);
        g[u].k0 = g[u].rel_lo == 0 ? 0u : 1u;
        g[u].cstart = g[u].rel_lo;  // (the carried-in line: set below, lane 0 reloads it)
        g[u].cslot = 0;
        const uint32_t pk0 = g[u].rel_lo == kTile ? 0u : 1u;  // tile - 1 the stream's first
        const uint32_t pn = tp[u].events + 1 > pk0 ? tp[u].events + 1 - pk0 : 0u;
        cs[u] = (g[u].k0 && pn) ? tile_slot_list(a, tp[u], tile - 1)[pn - 1] : 0u;
        pre[u] = load_line(a, g[u], (uint32_t)lane);  // (own slots only: load_line reads cslot later)
      }
#pragma unroll
      for (int u = 0; u < kTkBatch; ++u) {
        const uint32_t tile = t0 + u < a.ntiles ? t0 + u : a.ntiles - 1;
        if (!g[u].k0) continue;
        const uint32_t pk0 = g[u].rel_lo == kTile ? 0u : 1u;
        if (tp[u].events + 1 > pk0) {  // the common case: tile - 1 lists a line start
          g[u].cslot = cs[u];
          g[u].cstart = g[u].rel_lo - kTile + (int64_t)(cs[u] & kSlotOff);
        } else {
          TileLines h = g[u];
          h.rel_lo -= kTile;
          tile_slots(a, tstat, h, tile - 1, tp[u]);  // tile - 1 carries the same line in
          g[u].cslot = h.cslot;
          g[u].cstart = h.cstart;
        }
        if ((uint32_t)lane < g[u].k0) pre[u] = load_line(a, g[u], (uint32_t)lane);  // lane 0: the carried-in line
      }
    } else {
#pragma unroll
      for (int u = 0; u < kTkBatch; ++u) {
        const uint32_t tile = t0 + u < a.ntiles ? t0 + u : a.ntiles - 1;
        g[u].s = tseg[tile];
        g[u].sd = segs[g[u].s];
        g[u].rel_lo = (int64_t)(tile - g[u].sd.tile0) * kTile;
        const int64_t rem = (int64_t)g[u].sd.len - g[u].rel_lo;
        g[u].tlen = (int32_t)(rem < kTile ? rem : kTile);
        g[u].l0 = tbase[tile];
        const TileStat ts = tstat[tile];
        g[u].nl = rem <= kTile ? ts.events : ts.events + 1;
        pre[u] = load_line(a, g[u], (uint32_t)lane);
      }
    }
#pragma unroll
    for (int u = 0; u < kTkBatch; ++u) {
      const uint32_t tile = t0 + u;
      if (tile >= a.ntiles) break;
      const uint64_t wlo = sout[g[u].s].win_lo, whi = sout[g[u].s].win_hi;
      uint32_t kept, nsel;
      // (no run table, a.truns null: --tail runs do not map one; k_tcopy lists the runs again)
      const uint32_t nr = list_runs(a, g[u], wlo, whi, a.truns ? a.truns + (size_t)tile * kRunSlots : nullptr,
                                    a.truns ? (uint32_t)kRunSlots : 0u, lane, &kept, &nsel, &pre[u]);
      if (lane == 0) {
        TRec rec;
        rec.src = g[u].sd.base + (uint64_t)g[u].rel_lo;
        rec.kept = kept;
        rec.nruns = (a.truns && nr <= (uint32_t)kRunSlots) ? (uint16_t)nr : kRunsRecompute;
        rec.nsel = (uint16_t)nsel;
        a.trec[tile] = rec;
      }
    }
  }
}

// Planned runs (the scan's plans, FAgg above): the tile aggregates' ordered reduce-then-scan,
// 256 threads x R consecutive tiles per block.  bsum per block: bytes, then span | has << 32
// | sel << 33 | crel << 34 (16 bits), then the selected lines.
__device__ __forceinline__ uint64_t pack_blk(const FAgg& b) {
  return (uint64_t)b.span | ((uint64_t)b.has << 32) | ((uint64_t)b.sel << 33) | ((uint64_t)(uint16_t)(int16_t)b.crel << 34);
}
__device__ __forceinline__ FAgg unpack_blk(uint64_t bytes, uint64_t v) {
  FAgg b;
  b.bytes = bytes;
  b.span = (uint32_t)v;
  b.has = (v >> 32) & 1u;
  b.sel = (v >> 33) & 1u;
  b.crel = (int32_t)(int16_t)(uint16_t)(v >> 34);
  return b;
}
constexpr FAgg kFAggNone{0u, 0u, -1, false, false};
// the ordered total of the block's thread values (every thread gets it); s_a / s_n: [4]
__device__ __forceinline__ FAgg block_fagg_total(FAgg x, uint64_t n, FAgg* s_a, uint64_t* s_n, uint64_t* total_n) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const FAgg w = wave_incl_scan_fagg(x, lane);
  const uint64_t wn = wave_sum(n);
  __syncthreads();
  if (lane == 63) s_a[wv] = w;
  if (lane == 0) s_n[wv] = wn;
  __syncthreads();
  FAgg b = s_a[0];
  for (int k = 1; k < 4; ++k) b = f_combine(b, s_a[k]);
  *total_n = s_n[0] + s_n[1] + s_n[2] + s_n[3];
  return b;
}
template <int R>
__device__ __forceinline__ void ksum_plan(RunArgs& a) {
  __shared__ FAgg s_a[4];
  __shared__ uint64_t s_n[4];
  const uint4* rec = reinterpret_cast<const uint4*>(a.trec);
  const uint32_t t0 = blockIdx.x * (256 * R) + threadIdx.x * R;
  FAgg acc = kFAggNone;
  uint64_t ns = 0;
  for (int r = 0; r < R; ++r)
    if (t0 + r < a.ntiles) {
      const uint4 q = rec[t0 + r];
      acc = f_combine(acc, plan_agg(q));
      ns += q.y >> 16;
    }
  uint64_t tn;
  const FAgg b = block_fagg_total(acc, ns, s_a, s_n, &tn);
  if (threadIdx.x == 0) {
    a.bsum[4 * blockIdx.x] = b.bytes;
    a.bsum[4 * blockIdx.x + 1] = pack_blk(b);
    a.bsum[4 * blockIdx.x + 2] = tn;
  }
}
template <int R>
__device__ __forceinline__ void kbase_plan(RunArgs& a) {
  __shared__ FAgg s_a[4];
  __shared__ uint64_t s_n[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // the aggregate of the blocks before this one (each thread a consecutive range of them)
  FPre cur{0ull, -1, false};
  uint64_t nc = 0;
  {
    const uint32_t nb = blockIdx.x, per = (nb + 255) / 256;
    FAgg acc = kFAggNone;
    uint64_t ns = 0;
    for (uint32_t k = t * per; k < nb && k < (t + 1) * per; ++k) {
      acc = f_combine(acc, unpack_blk(a.bsum[4 * k], a.bsum[4 * k + 1]));
      ns += a.bsum[4 * k + 2];
    }
    uint64_t tn;
    const FAgg b = block_fagg_total(acc, ns, s_a, s_n, &tn);
    cur = f_apply(cur, b);
    nc = tn;
  }
  // this thread's tiles: their aggregate, then the exclusive ordered scan over the threads
  const uint4* rec = reinterpret_cast<const uint4*>(a.trec);
  const uint32_t t0 = blockIdx.x * (256 * R) + (uint32_t)t * R;
  FAgg acc = kFAggNone;
  uint64_t ns = 0;
  for (int r = 0; r < R; ++r)
    if (t0 + r < a.ntiles) {
      const uint4 q = rec[t0 + r];
      acc = f_combine(acc, plan_agg(q));
      ns += q.y >> 16;
    }
  const FAgg incl = wave_incl_scan_fagg(acc, lane);
  const uint64_t nincl = wave_incl_scan_add(ns, lane);
  __syncthreads();
  if (lane == 63) { s_a[wv] = incl; s_n[wv] = nincl; }
  __syncthreads();
  for (int k = 0; k < wv; ++k) { cur = f_apply(cur, s_a[k]); nc += s_n[k]; }
  {
    FAgg ex;  // lanes before mine (lane 0: none)
    ex.bytes = __shfl_up(incl.bytes, 1, 64);
    ex.span = (uint32_t)__shfl_up((int)incl.span, 1, 64);
    ex.crel = __shfl_up(incl.crel, 1, 64);
    const int fl = __shfl_up((incl.has ? 1 : 0) | (incl.sel ? 2 : 0), 1, 64);
    ex.has = fl & 1;
    ex.sel = (fl & 2) != 0;
    if (lane) cur = f_apply(cur, ex);
    nc += nincl - ns;
  }
  // the tiles: output base, carried-in run, the copy record k_tcopy reads (TRec with the
  // runs' destination shift in place of the selected lines), run slot 0
  for (int r = 0; r < R; ++r) {
    const uint32_t tile = t0 + r;
    if (tile >= a.ntiles) break;
    const uint4 q = rec[tile];
    const FAgg x = plan_agg(q);
    const uint32_t carried = f_carried(x.span, cur.sel, cur.crel);
    const uint32_t lo = cur.crel > 0 ? (uint32_t)cur.crel : 0u;
    const uint32_t kept = (uint32_t)x.bytes + carried, nsel = q.y >> 16, own = q.z;
    const uint32_t s = a.tile_seg[tile];
    const SegDesc sd = a.segs[s];
    const uint64_t src = sd.base + (uint64_t)(tile - sd.tile0) * kTile;
    a.kbase[2 * tile] = cur.off;
    a.kbase[2 * tile + 1] = nc;
    const uint32_t nruns = own == kRunsRecompute ? (uint32_t)kRunsRecompute : ((own + 1u) | kRunsShifted);
    reinterpret_cast<uint4*>(a.trec)[tile] = make_uint4((uint32_t)src, (uint32_t)(src >> 32), kept, nruns | (carried << 16));
    if (own != kRunsRecompute) a.truns[(size_t)tile * kRunSlots] = lo;  // (length: up to run 1's destination)
    if (tile == sd.tile0) { a.segout[s].out_lo = cur.off; a.segout[s].sel_lo = nc; }
    if (tile + 1 == sd.tile0 + sd.ntiles) { a.segout[s].out_hi = cur.off + kept; a.segout[s].sel_hi = nc + nsel; }
    cur = f_apply(cur, x);
    nc += nsel;
  }
}

// Reduce-then-scan of the tiles' (kept bytes, selected lines): 256 x R tiles per block.
template <int R>
__device__ __forceinline__ void ksum_body(RunArgs& a) {
  __shared__ uint64_t s_w[2][4];
  if (a.counters[2] || !a.counters[kCtrDense]) return;
  if (planned(a)) { ksum_plan<R>(a); return; }
  const uint32_t t0 = blockIdx.x * (256 * R) + threadIdx.x;
  uint64_t b = 0, c = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (t0 + r * 256 < a.ntiles) {
      const TRec k = a.trec[t0 + r * 256];
      b += k.kept;
      c += k.nsel;
    }
  b = wave_sum(b);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) { s_w[0][threadIdx.x >> 6] = b; s_w[1][threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int k = threadIdx.x;
    a.bsum[2 * blockIdx.x + k] = s_w[k][0] + s_w[k][1] + s_w[k][2] + s_w[k][3];
  }
}

template <int R>
__device__ __forceinline__ void kbase_body(RunArgs& a) {
  __shared__ uint64_t s_w[2][2][4];
  __shared__ uint64_t s_base[2];
  if (a.counters[2] || !a.counters[kCtrDense]) return;
  if (blockIdx.x * (256u * R) >= a.ntiles) return;  // launched on k_cgather's grid (k_cmove)
  if (planned(a)) { kbase_plan<R>(a); return; }
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t t0 = blockIdx.x * (256 * R) + t;
  {
    uint64_t b = 0, c = 0;
    for (uint32_t k = t; k < blockIdx.x; k += 256) { b += a.bsum[2 * k]; c += a.bsum[2 * k + 1]; }
    b = wave_sum(b);
    c = wave_sum(c);
    if (lane == 0) { s_w[0][0][wv] = b; s_w[0][1][wv] = c; }
    __syncthreads();
    if (t < 2) s_base[t] = s_w[0][t][0] + s_w[0][t][1] + s_w[0][t][2] + s_w[0][t][3];
    __syncthreads();
  }
  uint64_t cb = s_base[0], cc = s_base[1];
  for (int r = 0; r < R; ++r) {
    const uint32_t tile = t0 + r * 256;
    uint32_t kb = 0, kc = 0;
    if (tile < a.ntiles) {
      const TRec k = a.trec[tile];
      kb = k.kept;
      kc = k.nsel;
    }
    const uint64_t ib = wave_incl_scan_add((uint64_t)kb, lane), ic = wave_incl_scan_add((uint64_t)kc, lane);
    const int pb = r & 1;
    if (lane == 63) { s_w[pb][0][wv] = ib; s_w[pb][1][wv] = ic; }
    __syncthreads();
    uint64_t ob = cb + ib - kb, oc = cc + ic - kc;
    for (int w = 0; w < wv; ++w) { ob += s_w[pb][0][w]; oc += s_w[pb][1][w]; }
    cb += s_w[pb][0][0] + s_w[pb][0][1] + s_w[pb][0][2] + s_w[pb][0][3];
    cc += s_w[pb][1][0] + s_w[pb][1][1] + s_w[pb][1][2] + s_w[pb][1][3];
    if (tile < a.ntiles) {
      a.kbase[2 * tile] = ob;
      a.kbase[2 * tile + 1] = oc;
      const uint32_t s = a.tile_seg[tile];
      const SegDesc& sd = a.segs[s];
      if (tile == sd.tile0) { a.segout[s].out_lo = ob; a.segout[s].sel_lo = oc; }
      if (tile + 1 == sd.tile0 + sd.ntiles) { a.segout[s].out_hi = ob + kb; a.segout[s].sel_hi = oc + kc; }
    }
  }
}

// ---- the launches after the matchers (fewer kernel boundaries: each costs ~5 us) ----------
// k_tailw: the kubelet tail rule per stream (block per stream); the last block to finish
// (ticket) then runs the window prefix over all streams and picks the compaction path.
// The last tiles of [t0, t0 + nt) whose tile_base (the line open at its start) is <= ka /
// <= kb, else t0: block-wide searches, 256 sample points per level (tile_base ascends),
// both keys' loads in flight together (one memory round trip per level).
__device__ void last_tiles_le(const RunArgs& a, uint32_t t0, uint32_t nt, uint64_t ka, uint64_t kb,
                              uint32_t& ra, uint32_t& rb) {
  uint32_t lo[2] = {t0, t0}, span[2] = {nt, nt};
  const uint64_t key[2] = {ka, kb};
  bool done[2] = {nt <= 1, nt <= 1};
  while (!done[0] || !done[1]) {
    uint32_t step[2];
    bool p[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      step[q] = (span[q] + 255u) / 256u;
      const uint32_t k = threadIdx.x * step[q];
      p[q] = !done[q] && k < span[q] && a.tile_base[lo[q] + k] <= key[q];
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t c = (uint32_t)__syncthreads_count(p[q]);  // the true samples are a prefix
      if (done[q]) continue;
      if (c == 0) { done[q] = true; continue; }  // (first level only: sample 0 of a later level is true)
      lo[q] += (c - 1u) * step[q];
      span[q] = step[q] < t0 + nt - lo[q] ? step[q] : t0 + nt - lo[q];
      done[q] = span[q] <= 1;
    }
  }
  ra = lo[0];
  rb = lo[1];
}
// win_index: the scatter groups holding stream s's window lines [win_lo, win_hi] (the
// window scatter's tiles), so that k_scatter's window pass visits only those.  Line l > the
// stream's first has its start slot in the tile of the newline that ends line l - 1: the
// last tile whose base (the line open at its start) is <= l - 1.  (Not "one tile before the
// last base <= l": a long line leaves every tile it covers with base l and no slot.)  The
// range ends at the last tile whose base is <= win_hi.
__device__ __forceinline__ void win_groups_body(RunArgs& a) {
  const uint32_t s = blockIdx.x;
  const SegDesc sd = a.segs[s];
  const SegOut& so = a.segout[s];
  uint64_t packed = 0;
  if (so.win_hi > so.win_lo && sd.ntiles) {
    uint32_t ta, tb;
    const bool first = so.win_lo <= so.line_lo;
    last_tiles_le(a, sd.tile0, sd.ntiles, first ? so.line_lo : so.win_lo - 1u, so.win_hi, ta, tb);
    if (first) ta = sd.tile0;
    packed = (uint64_t)(ta / kScatterGroup) | (uint64_t)(tb / kScatterGroup + 1u) << 32;
  }
  if (threadIdx.x == 0) a.wgrp[s] = packed;
}
__device__ __forceinline__ void win_groups_prefix(RunArgs& a) {
  __shared__ uint64_t s_w64[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint64_t carry = 0;
  for (uint32_t b = 0; b < a.nsegs; b += 256) {
    const uint32_t s = b + t;
    const uint64_t pk = s < a.nsegs ? a.wgrp[s] : 0;
    const uint64_t v = (pk >> 32) - (pk & 0xFFFFFFFFull);
    const uint64_t inc = wave_incl_scan_add(v, lane);
    __syncthreads();
    if (lane == 63) s_w64[wv] = inc;
    __syncthreads();
    uint64_t pre = 0;
    for (int k = 0; k < wv; ++k) pre += s_w64[k];
    if (s < a.nsegs) a.wgrp[a.nsegs + s] = carry + pre + inc - v;
    carry += s_w64[0] + s_w64[1] + s_w64[2] + s_w64[3];
  }
  if (t == 0) a.wgrp[2 * a.nsegs] = carry;
}
__global__ __launch_bounds__(256) void k_tailw(RunArgs a) {
  __shared__ uint32_t s_last;
  tail_body(a);
  __syncthreads();
  if (a.win_index && !a.counters[2]) {
    win_groups_body(a);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    __threadfence();  // this block's stream records before its ticket
    s_last = atomicAdd(&a.counters[kCtrTailDone], 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (s_last) {
    __threadfence();  // every block's records, seen through their tickets
    wprefix_body(a);
    if (a.win_index && !a.counters[2]) {
      __syncthreads();
      win_groups_prefix(a);
    }
    if (a.plan_mode == 2) {  // a small --tail selection: the gather's block sums and prefix here
      __syncthreads();
      csum_body(a, 0, 1);
      __syncthreads();
      cscan_body(a);
    }
  }
}
// Then three launches serve either compaction path (k_wprefix's choice, counters[kCtrDense]):
//   k_cplan   line gather: per-block selected bytes (k_csum) | tile copy: kept runs (k_tkeep)
//   k_cmid    block prefix (k_cscan, block 0)               | tile block sums (k_ksum)
//   k_cmove   gather copy (k_cgather)                       | tile output bases (k_kbase)
// and k_tcopy (tile copy) last.
__global__ __launch_bounds__(256) void k_cplan(RunArgs a, const uint32_t* __restrict__ tseg,
                                               const SegDesc* __restrict__ segs, const TileStat* __restrict__ tstat,
                                               const uint64_t* __restrict__ tbase, const SegOut* __restrict__ sout) {
  if (a.counters[kCtrDense]) tkeep_body(a, tseg, segs, tstat, tbase, sout);
  else csum_body(a, blockIdx.x, gridDim.x);
  if (a.plan_mode == 1) {  // the last block to finish runs k_cmid's prefix (not launched)
    __shared__ uint32_t s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();  // this block's sums (thread 0 wrote them) before its ticket
      s_last = atomicAdd(&a.counters[kCtrPlanDone], 1u) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (s_last) {
      __threadfence();
      cscan_body(a);
    }
  }
}
__global__ __launch_bounds__(256) void k_cmid(RunArgs a) {
  if (a.counters[kCtrDense]) ksum_body<16>(a);
  else if (blockIdx.x == 0) cscan_body(a);
}
__global__ __launch_bounds__(256) void k_cmove(RunArgs a) {
  if (a.counters[kCtrDense]) kbase_body<16>(a);
  else cgather_body(a);
}

#ifndef KLF_TC_ABL
#define KLF_TC_ABL 0  // timing builds: 1 no copy loop, 2 no map and no copy, 4 no tile loads
#endif
#ifndef KLF_COPY_UNALIGNED
#define KLF_COPY_UNALIGNED 1  // copy_tile_runs' 16-B windows as one unaligned LDS read (0: five dwords + v_alignbyte)
#endif
// The compaction copy of one tile, one wave: the tile's bytes in LDS (s_buf; 16 B readable
// before it and 32 B after it), its kept runs s_run[0, nr) (u32: tile offset of the run's
// first byte | its offset in the tile's output << 16, ascending), `kept` output bytes at
// out + obase.  s_run needs two spare entries (sentinels), s_map (nch + 8 entries) is
// scratch.  Every 16-B output chunk holding only this tile's bytes is built from <= 2 runs
// (five dword LDS reads + v_alignbyte each, branch-free blend) and stored once; the two
// edge chunks shared with the neighbouring tiles are stored bytewise in one instruction.
__device__ __forceinline__ void copy_tile_runs(const uint8_t* s_buf, uint32_t* s_run, uint16_t* s_map, uint32_t nr,
                                               uint32_t kept, uint64_t obase, uint8_t* out, int lane) {
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s_buf - 16);  // dword k = s_buf[4k - 16]
  const uint32_t o15 = (uint32_t)(obase & 15u);
  const uint32_t nch = (uint32_t)(((obase + kept + 15) >> 4) - (obase >> 4));
  // chunk c covers output [16 * (obase / 16 + c), +16); its first byte inside this tile's
  // output, x0(c) = (c ? 16c - o15 : 0), lies in exactly one run.  The map (u16): run k
  // marks the first chunk whose x0 is at or past its start; several short runs may mark
  // one chunk, and as the runs ascend the last of them (the one holding x0) is the one
  // whose successor marks a later chunk: it alone stores (no LDS atomics).  Then a
  // running max over the chunks.
    // two sentinel runs past the last (start = kept) spare the bounds checks below
    if (lane < 2) s_run[nr + lane] = kept << 16;
    for (uint32_t c = 8 * (uint32_t)lane; c < nch; c += 512) *reinterpret_cast<uint4*>(&s_map[c]) = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
    auto mark = [&](uint32_t d) { return d ? (d + o15 + 15) >> 4 : 0u; };
    for (uint32_t k = lane; k < nr; k += 64) {
      const uint32_t c = mark(s_run[k] >> 16);
      // (the sentinel run nr marks chunk nch exactly: a chunk it shares is past the output)
      if (c < nch && mark(s_run[k + 1] >> 16) != c) s_map[c] = (uint16_t)k;
    }
    wave_lds_sync();
    // running max: 8 consecutive entries per lane (one 16-B LDS access), one wave scan of
    // the lanes' maxima
    for (uint32_t c0 = 0, carry = 0; c0 < nch; c0 += 512) {
      const uint32_t c = c0 + 8 * (uint32_t)lane;
      const uint4 pk = *reinterpret_cast<const uint4*>(&s_map[c]);
      uint32_t v[8] = {pk.x & 0xFFFFu, pk.x >> 16, pk.y & 0xFFFFu, pk.y >> 16,
                       pk.z & 0xFFFFu, pk.z >> 16, pk.w & 0xFFFFu, pk.w >> 16};
      auto mx = [](uint32_t x, uint32_t y) { return x > y ? x : y; };
#pragma unroll
      for (int q = 1; q < 8; ++q) v[q] = mx(v[q], v[q - 1]);
      const uint32_t incl = mx(wave_incl_scan_max(v[7], lane), carry);
      uint32_t pre = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xF, 0xF, false);  // wave_shr:1
      pre = mx(lane ? pre : 0u, carry);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = mx(v[q], pre);
      if (c < nch)
        *reinterpret_cast<uint4*>(&s_map[c]) =
            make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
      carry = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    wave_lds_sync();
    if (KLF_TC_ABL & 1) return;
    uint8_t* outc = out + ((obase >> 4) << 4);
    // Every store goes through a per-tile buffer descriptor over the tile's output chunks
    // (wave-uniform): lanes with nothing to store pass an offset past its range and the
    // hardware drops them, so there is no branch around any store and each tile issues
    // exactly 8 + 1 store instructions.  The compiler then counts them: the wait for the
    // next tile's prefetched rows no longer waits for this tile's stores to complete.
    const uint64_t ob_u = (uint64_t)(uintptr_t)outc;
    const uint32_t ob_lo = __builtin_amdgcn_readfirstlane((uint32_t)ob_u);
    const uint32_t ob_hi = __builtin_amdgcn_readfirstlane((uint32_t)(ob_u >> 32));
    const uint32_t nout = __builtin_amdgcn_readfirstlane(kept ? nch * 16u : 0u);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>((uint64_t)ob_lo | ((uint64_t)ob_hi << 32)), 0, (int)nout, 0x00020000);
    constexpr uint32_t kDrop = 0x7FFFFFF0u;
    // 16 B of run r's bytes as they land on the chunk whose byte 0 is tile output x0: the
    // LDS window at any alignment (five dword reads + v_alignbyte; +16: the front pad)
    auto window = [&](uint32_t r, uint32_t x0, uint32_t (&y)[4]) __attribute__((always_inline)) {
      const int32_t va = (int32_t)(r & 0xFFFFu) + (int32_t)x0 - (int32_t)(r >> 16) + 16;
      if (KLF_COPY_UNALIGNED) {
        // one unaligned 16-B LDS read (gfx950, HSA default unaligned mode; parse_fast reads
        // the same way): consecutive lanes read consecutive 16 B, where five dword reads at a
        // 4-dword lane stride hit every bank four times (C3: 2.04x conflict cycles)
        typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));
        u32x4w v;
        __builtin_memcpy(&v, reinterpret_cast<const uint8_t*>(s32) + va, 16);
        y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
        return;
      }
      const int32_t wa = va >> 2;
      const uint32_t w0 = s32[wa], w1 = s32[wa + 1], w2 = s32[wa + 2], w3 = s32[wa + 3], w4 = s32[wa + 4];
      y[0] = __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)va);
      y[1] = __builtin_amdgcn_alignbyte(w2, w1, (uint32_t)va);
      y[2] = __builtin_amdgcn_alignbyte(w3, w2, (uint32_t)va);
      y[3] = __builtin_amdgcn_alignbyte(w4, w3, (uint32_t)va);
    };
    // Chunk bytes [b0, b1) (tile output x0 + b - b0 ...) of a chunk spanning any number of
    // runs, starting with run k: piecewise (the head and tail chunks, and chunks of three
    // or more runs).  o[] bytes outside [b0, b1) are left as they were.
    auto pieces = [&](uint32_t k, uint32_t xs, uint32_t xe, uint32_t xc, uint32_t (&o)[4]) __attribute__((always_inline)) {
      // xc = tile output position of chunk byte 0 (may be "negative": unsigned wrap)
      for (uint32_t x = xs; x < xe; ++k) {
        const uint32_t r = s_run[k];
        const uint32_t e = s_run[k + 1] >> 16;
        const uint32_t pe = e < xe ? e : xe;
        uint32_t y[4];
        window(r, xc, y);
        const int b0 = (int)(x - xc), b1 = (int)(pe - xc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t mm = byte_mask(b0, b1, q);
          o[q] = (y[q] & mm) | (o[q] & ~mm);
        }
        x = pe;
      }
    };
    // interior chunks (all 16 bytes from this tile): c in [c_lo, c_end), x0 = 16c - o15;
    // at most 512 of them: eight rounds of 64 lanes
    const uint32_t c_lo = o15 ? 1u : 0u, c_end = (kept + o15) >> 4;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t c = c_lo + (uint32_t)lane + 64u * (uint32_t)u;
      uint32_t o[4] = {0u, 0u, 0u, 0u};
      if (c < c_end) {
      const uint32_t x0 = 16 * c - o15, x1 = x0 + 16;
      const uint32_t k = s_map[c];
      const uint32_t r0 = s_run[k], r1 = s_run[k + 1], d2 = s_run[k + 2] >> 16;
      if (x1 <= d2) {  // at most two runs: both windows, blended where run k + 1 starts
        uint32_t y0[4], y1[4];
        window(r0, x0, y0);
        const uint32_t d1 = r1 >> 16;
        const bool two = d1 < x1;
        window(two ? r1 : r0, x0, y1);
        const int32_t split8 = 8 * (two ? (int32_t)(d1 - x0) : 16);  // bits of the chunk from run k
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int32_t sq = split8 - 32 * q;
          const uint32_t lo = sq <= 0 ? 0u : sq >= 32 ? ~0u : ((1u << sq) - 1u);
          o[q] = (y0[q] & lo) | (y1[q] & ~lo);
        }
      } else {
        pieces(k, x0, x1, x0, o);
      }
      }
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 ov = {o[0], o[1], o[2], o[3]};
      // (non-temporal stores and / or loads measured no faster: C3 step 5.50-5.56 ms against
      // 5.14-5.41, gpurun_out/r4r)
      __builtin_amdgcn_raw_buffer_store_b128(ov, orsrc, c < c_end ? 16u * c : kDrop, 0, 0);
    }
    // head / tail chunks shared with the neighbouring tiles: only this tile's bytes, one
    // byte per lane (lanes 0-15 the head chunk, 16-31 the tail chunk; a chunk holding both
    // ends is the head's), so both go out in ONE byte-store instruction
    {
      const uint32_t ct = (kept + o15) >> 4, i = (uint32_t)lane & 15u;
      bool act = false;
      uint32_t c = 0, xe = 0;
      if (lane < 16 && o15) {
        act = true;
        xe = kept < 16 - o15 ? kept : 16 - o15;
      } else if (lane >= 16 && lane < 32 && ((kept + o15) & 15u) && (ct > 0 || !o15)) {
        act = true;
        c = ct;
        xe = kept;
      }
      // tile output position of chunk byte i (wraps below 0 for the head chunk's bytes
      // that belong to the previous tile: then x >= xe)
      const uint32_t x = 16 * c - o15 + i;
      const bool st = act && x < xe;
      uint8_t b = 0;
      if (st) {
        uint32_t k = s_map[c];
        while ((s_run[k + 1] >> 16) <= x) ++k;  // the sentinels end the walk
        const uint32_t r = s_run[k];
        b = s_buf[(r & 0xFFFFu) + x - (r >> 16)];
      }
      __builtin_amdgcn_raw_buffer_store_b8(b, orsrc, st ? 16u * c + i : kDrop, 0, 0);
    }
}

// LDS per wave: the tile (16 B of front pad, 8 KiB, 32 B of back pad: the unaligned reads of
// a piece start up to 15 B before its chunk and end up to 20 B after it), the kept runs
// (a selected line carries a >= 20-B prefix, so at most kTile / 20 + 2 runs), and the
// chunk -> first run map.
// Workgroups of kTcWaves waves (no workgroup barrier: each wave owns its tiles and LDS).
// Measured on C3 (same box): 4-wave workgroups, 12 waves per CU, 5.52 ms per step;
// 2-wave (14 per CU) 5.70, 1-wave (14 per CU) 5.73 -- more copy waves per CU slow it.
#ifndef KLF_TC_WAVES
#define KLF_TC_WAVES 4
#endif
constexpr int kTcWaves = KLF_TC_WAVES;
__global__ __launch_bounds__(64 * kTcWaves) void k_tcopy(RunArgs a, const uint4* __restrict__ trec,
                                               const uint64_t* __restrict__ kbase, const uint32_t* __restrict__ truns) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf_all[kTcWaves][kTile + 48];
  __shared__ uint32_t s_run_all[kTcWaves][kTcRuns];
  __shared__ __attribute__((aligned(16))) uint16_t s_map_all[kTcWaves][kTcChunks];
  if (a.counters[2] || !a.counters[kCtrDense]) return;
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* s_buf = s_buf_all[wv] + 16;
  uint32_t* s_run = s_run_all[wv];
  uint16_t* s_map = s_map_all[wv];
  const uint32_t stride = gridDim.x * kTcWaves;
  // software pipeline: tile t's bytes and runs are in registers while tile t - stride is
  // copied; the records run one tile further ahead
  // (named registers: an array here is put on the scratch stack)
#define KLF_TC_ROWS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define KLF_TC_DECL(q) uint4 v##q = make_uint4(0, 0, 0, 0);
#define KLF_TC_LOAD(q) v##q = gp[q * 64 + lane];
#define KLF_TC_STORE(q) l[q * 64 + lane] = v##q;
  KLF_TC_ROWS(KLF_TC_DECL)
  uint32_t rw0 = 0, rw1 = 0;
  auto load_rec = [&](uint32_t t) __attribute__((always_inline)) {  // one scalar 16-B load
    const uint4 q = trec[t];
    TRec r;
    r.src = (uint64_t)q.x | ((uint64_t)q.y << 32);
    r.kept = q.z;
    r.nruns = (uint16_t)(q.w & 0xFFFFu);
    // nsel becomes the destination shift of runs 1.. (planned runs: run 0 is the carried-in
    // line's, set by k_cmove after the scan listed the others), else 0
    const bool shifted = r.nruns != kRunsRecompute && (r.nruns & kRunsShifted);
    r.nsel = shifted ? (uint16_t)(q.w >> 16) : (uint16_t)0;
    if (r.nruns != kRunsRecompute) r.nruns = (uint16_t)(r.nruns & ~kRunsShifted);
    return r;
  };
  auto issue = [&](uint32_t t, const TRec& r) __attribute__((always_inline)) {
    if (r.kept == 0) return;
    const uint4* gp = reinterpret_cast<const uint4*>(a.bytes + r.src);
    if (!(KLF_TC_ABL & 4)) { KLF_TC_ROWS(KLF_TC_LOAD) }
    if (r.nruns != kRunsRecompute) {
      const uint32_t* rp = truns + (size_t)t * kRunSlots;
      rw0 = (uint32_t)lane < r.nruns ? rp[lane] : 0u;
      rw1 = (uint32_t)lane + 64 < r.nruns ? rp[lane + 64] : 0u;
    }
  };
  uint32_t tile = blockIdx.x * kTcWaves + wv;
  TRec rec{}, nrec{};
  uint64_t ob = 0, nob = 0;
  if (tile < a.ntiles) {
    rec = load_rec(tile);
    ob = kbase[2 * tile];
    issue(tile, rec);
  }
  if (tile + stride < a.ntiles) {
    nrec = load_rec(tile + stride);
    nob = kbase[2 * (tile + stride)];
  }
  {  // nine dropped stores behind the first loads: the loop is entered with the same count
     // of stores after the prefetched rows as every iteration ends with (the waits for the
     // rows are computed over both paths)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0, 0x00020000);
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < 8; ++u) __builtin_amdgcn_raw_buffer_store_b128(z, none, 0x7FFF0000u + 16u * u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, none, 0x7FFF0100u, 0, 0);
  }
  for (; tile < a.ntiles; tile += stride) {
    const TRec cr = rec;
    const uint64_t obase = ob;
    if (cr.kept) {
      uint4* l = reinterpret_cast<uint4*>(s_buf);
      KLF_TC_ROWS(KLF_TC_STORE)
      if (cr.nruns != kRunsRecompute) {
        const uint32_t sh = (uint32_t)cr.nsel << 16;
        if ((uint32_t)lane < cr.nruns) s_run[lane] = rw0 + (lane ? sh : 0u);
        if ((uint32_t)lane + 64 < cr.nruns) s_run[lane + 64] = rw1 + sh;
      }
    }
    // the next tile's loads go out before this tile's copy
    rec = nrec;
    ob = nob;
    const uint32_t nt = tile + stride;
    if (nt < a.ntiles) issue(nt, rec);
    if (nt + stride < a.ntiles) {
      nrec = load_rec(nt + stride);
      nob = kbase[2 * (nt + stride)];
    }
    // (no early exit for a tile with nothing kept: every iteration issues the same nine
    // stores, so the compiler's vmcnt waits for the prefetched rows count past them)
    uint32_t nr = cr.nruns;
    if (nr == kRunsRecompute) {  // more runs than the record holds: list them again here
      const TileLines g = tile_lines(a, tile);
      uint32_t kept, nsel;
      nr = list_runs(a, g, a.segout[g.s].win_lo, a.segout[g.s].win_hi, s_run, kTcRuns, lane, &kept, &nsel);
    }
    if (KLF_TC_ABL & 2) continue;
    if (obase + cr.kept + 16 > a.out_cap) {  // the buffer is too small: the host grows it and reruns
      if (lane == 0) atomicOr(&a.counters[kCtrOutShort], 1u);
      continue;
    }
    copy_tile_runs(s_buf, s_run, s_map, nr, cr.kept, obase, a.out, lane);
    asm volatile("" ::: "memory");  // the next tile rewrites the wave's LDS
  }
#undef KLF_TC_ROWS
#undef KLF_TC_DECL
#undef KLF_TC_LOAD
#undef KLF_TC_STORE
}

// One-pass compaction, second kernel (one wave per range): the bytes in front of a range's
// first line start belong to the line open at the range start, which started in an earlier
// range.  Its state (kept?, content start) is the one the nearest earlier range with a line
// start left (the ranges in between lie inside that line); the kept part of those bytes is
// copied from the input to just in front of the range's output, whose first extent grows by
// it.  (A carried part is at most one line: copied a byte per lane.)
__global__ __launch_bounds__(256) void k_fcarry(RunArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.fuse_nranges || a.counters[kCtrFuseBad] || a.counters[2]) return;
  const uint32_t t0 = r * a.fuse_range;
  if (t0 >= a.ntiles) return;
  const SegDesc sd = a.segs[a.tile_seg[t0]];
  if (t0 == sd.tile0) return;  // a stream starts here: nothing carried in
  const uint64_t* ri = a.fuse_rinfo;
  const uint64_t res = ri[4 * (size_t)r];
  if (res == 0) return;
  int64_t back = 0;
  bool sel = false;
  int64_t crel = -1;
  for (uint32_t k = r; k-- > 0;) {
    const uint64_t fl = ri[4 * (size_t)k + 1];
    if (fl & 1u) {
      sel = (fl & 2u) != 0;
      crel = (int64_t)ri[4 * (size_t)k + 2];
      break;
    }
    back += (int64_t)ri[4 * (size_t)k + 3];  // (a whole range inside the line)
  }
  if (crel >= 0) crel -= back;  // relative to this range's start (f_sat: before it = -1)
  const uint64_t lo = crel > 0 ? (uint64_t)crel : 0u;
  const uint64_t clen = (sel && res > lo) ? res - lo : 0u;
  if (clen == 0) return;
  const uint64_t rbase = sd.base + (uint64_t)(t0 - sd.tile0) * kTile;
  const uint8_t* src = a.bytes + rbase + lo;
  uint8_t* dst = a.out + rbase + res - clen;
  // A range inside one long line carries up to the whole range (fuse_range tiles): the
  // middle goes as aligned 16-B stores, each built from two aligned 16-B loads of the
  // source (which may read up to 16 B past the carried bytes: inside the batch, whose
  // allocation has kAllocSlack bytes past its last stream); bytewise only up to the first
  // aligned destination chunk and after the last.
  uint64_t head = (16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u;
  head = head < clen ? head : clen;
  const uint64_t nmid = (clen - head) >> 4;
  for (uint64_t i = (uint64_t)lane; i < head; i += 64) dst[i] = src[i];
  {
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src + head);
    const uint4* sb = reinterpret_cast<const uint4*>(sa & ~(uintptr_t)15);
    const uint32_t so = (uint32_t)(sa & 15u);
    uint4* db = reinterpret_cast<uint4*>(dst + head);
    for (uint64_t k = (uint64_t)lane; k < nmid; k += 64) {
      const uint4 x0 = sb[k];
      db[k] = so ? extract16(x0, sb[k + 1], so) : x0;
    }
  }
  for (uint64_t i = head + (nmid << 4) + (uint64_t)lane; i < clen; i += 64) dst[i] = src[i];
  if (lane == 0) {
    uint64_t* ex = a.fuse_ext + 2 * (size_t)a.fuse_ext0[r];
    ex[0] -= clen;
    ex[1] += clen;
  }
}

// Data statistics for the prefilter's layout and window choice (one-off, first batch): the
// 2-grams at even offsets of a sample of the batch and every byte, counted per block in LDS
// (65,536 u16 pair counters, two per dword: a block's 1,024 dwords add at most 2,048 to one
// counter) and added to the global histogram once per nonzero counter and block.  Global
// atomics per sample serialised on the hot pairs of log text (`""`, `  `): 257 us for
// C5's 1 MiB sample.
constexpr uint32_t kGhDwords = 1024;  // sampled dwords per block
__global__ __launch_bounds__(256) void k_gramhist(const uint8_t* bytes, const SegDesc* segs, uint32_t nsegs,
                                                  uint64_t sample, uint32_t fold, uint32_t* hist) {
  __shared__ uint32_t s_p[32768];
  __shared__ uint32_t s_b[256];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < 32768u; i += 256u) s_p[i] = 0;
  s_b[t] = 0;
  __syncthreads();
  const uint32_t nseg = nsegs < 16 ? nsegs : 16;
  const uint32_t step = nsegs / nseg;
  const uint64_t per = sample / 4;  // dwords per segment sample
  const uint64_t w0b = (uint64_t)blockIdx.x * kGhDwords, w1b = w0b + kGhDwords;
  for (uint64_t w = w0b + t; w < w1b && w < per * nseg; w += 256u) {
    const SegDesc sd = segs[(uint32_t)(w / per) * step];
    const uint64_t o = (w % per) * 4;
    if (o + 8 > sd.len) continue;
    const uint32_t x = *reinterpret_cast<const uint32_t*>(bytes + sd.base + o);
    const uint32_t g = x | fold;
    const uint32_t lo = g & 0xFFFFu, hi = g >> 16;
    atomicAdd(&s_p[lo >> 1], 1u << ((lo & 1u) * 16u));
    atomicAdd(&s_p[hi >> 1], 1u << ((hi & 1u) * 16u));
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(&s_b[(x >> (8 * k)) & 0xFFu], 1u);
  }
  __syncthreads();
  for (uint32_t i = t; i < 32768u; i += 256u) {
    const uint32_t v = s_p[i];
    if (v & 0xFFFFu) atomicAdd(&hist[kGramHistPairs + 2u * i], v & 0xFFFFu);
    if (v >> 16) atomicAdd(&hist[kGramHistPairs + 2u * i + 1u], v >> 16);
  }
  if (s_b[t]) atomicAdd(&hist[t], s_b[t]);
}

// Capture assembly: block b copies 1 MiB of piece b / kAsmBlocks (pieces are 64 MiB
// device chunks); 16-B loads, four in flight per thread.
constexpr uint32_t kAsmSpan = 1u << 20;
__global__ __launch_bounds__(256) void k_assemble(const AsmPiece* __restrict__ pieces, uint32_t n,
                                                  uint8_t* __restrict__ batch, uint32_t per) {
  const uint32_t pi = blockIdx.x / per, sub = blockIdx.x % per;
  if (pi >= n) return;
  const AsmPiece p = pieces[pi];
  const uint64_t lo = (uint64_t)sub * kAsmSpan;
  if (lo >= p.len) return;
  const uint64_t m = (p.len - lo < kAsmSpan ? p.len - lo : kAsmSpan) / 16;
  const uint4* s = reinterpret_cast<const uint4*>(p.src + lo);
  uint4* d = reinterpret_cast<uint4*>(batch + p.dst + lo);
  for (uint64_t i = threadIdx.x; i < m; i += 4 * 256) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < m) v[k] = s[i + k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + k * 256 < m) d[i + k * 256] = v[k];
  }
}

__global__ __launch_bounds__(256) void k_lastbad(const uint16_t* __restrict__ meta, uint64_t lo, uint64_t hi,
                                                 unsigned long long* res) {
  uint64_t best = 0;
  for (uint64_t l = lo + (uint64_t)blockIdx.x * 256 + threadIdx.x; l < hi; l += (uint64_t)gridDim.x * 256)
    if (!(meta[l] & Meta::kParsed)) best = l + 1;
  if (best) atomicMax(res, (unsigned long long)best);
}

}  // namespace

hipError_t launch_assemble(const AsmPiece* pieces, uint32_t n, uint8_t* batch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  constexpr uint32_t per = (64u << 20) / kAsmSpan;  // = the engine's staging chunk / span
  hipLaunchKernelGGL(k_assemble, dim3(n * per), dim3(256), 0, st, pieces, n, batch, per);
  return hipGetLastError();
}

hipError_t launch_lastbad(const RunArgs& a, uint64_t lo, uint64_t hi, uint64_t* res, hipStream_t st) {
  hipError_t e = hipMemsetAsync(res, 0, 8, st);
  if (e != hipSuccess || hi <= lo) return e;
  const uint64_t nb = (hi - lo + 255) / 256;
  hipLaunchKernelGGL(k_lastbad, dim3((uint32_t)(nb < 2048 ? nb : 2048)), dim3(256), 0, st, a.meta, lo, hi,
                     reinterpret_cast<unsigned long long*>(res));
  return hipGetLastError();
}

hipError_t dump_timeline(void* host, size_t bytes) {
#if KLF_TIMELINE
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_timeline), bytes, 0, hipMemcpyDeviceToHost);
#else
  (void)host; (void)bytes;
  return hipErrorNotSupported;
#endif
}
hipError_t clear_timeline() {
#if KLF_TIMELINE
  void* p;
  hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_timeline));
  if (e != hipSuccess) return e;
  return hipMemset(p, 0, sizeof(uint64_t) * 300000 * 8);
#else
  return hipSuccess;
#endif
}

// Diagnostic (klf_debug_clock): the clock a VALU-bound loop holds on this board.  Per
// workgroup the shader-clock and 100 MHz real-time deltas around the loop (s_memtime /
// s_memrealtime reads) go to out[2 b], out[2 b + 1]; out[2 nblocks] only keeps the loop
// alive.  Nothing else reads the buffer.
__global__ __launch_bounds__(256) void k_clock(uint64_t* out, uint32_t iters) {
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x, y = x ^ 0x9E3779B9u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i) {
    x = x * 1664525u + 1013904223u;
    y = (y ^ (x >> 7)) + (x << 3);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  if ((x ^ y) == 0x7E57C10Cu) out[2 * gridDim.x] = y;
}
hipError_t clock_probe(int num_cus, uint32_t iters, uint32_t reps, uint64_t* out, hipStream_t st) {
  const uint32_t nb = (uint32_t)num_cus * 4;
  for (uint32_t r = 0; r < reps; ++r) {  // back to back: the last one is read
    hipLaunchKernelGGL(k_clock, dim3(nb), dim3(256), 0, st, out, iters);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_gramhist(const uint8_t* bytes, const SegDesc* segs, uint32_t nsegs, uint64_t sample, uint32_t fold,
                           uint32_t* hist, hipStream_t st) {
  hipError_t e = hipMemsetAsync(hist, 0, kGramHistWords * 4, st);
  if (e != hipSuccess) return e;
  const uint32_t nseg = nsegs < 16 ? nsegs : 16;
  const uint64_t dwords = nseg * (sample / 4);
  const uint32_t grid = (uint32_t)((dwords + kGhDwords - 1) / kGhDwords);
  hipLaunchKernelGGL(k_gramhist, dim3(grid ? grid : 1), dim3(256), 0, st, bytes, segs, nsegs, sample, fold, hist);
  return hipGetLastError();
}

// A first run's line density without a mid-run readback (literal and pattern-less runs; the
// prefiltered sets take it from k_gramhist's sample): block b counts the newlines of one
// 8 KiB tile spread evenly over the batch and writes {newlines, bytes} to out[2 b].
__global__ __launch_bounds__(256) void k_nlsample(const uint8_t* __restrict__ bytes, const SegDesc* __restrict__ segs,
                                                  uint32_t nsegs, uint32_t ntiles, uint32_t* __restrict__ out) {
  __shared__ uint32_t s_w[4];
  const uint32_t tile = (uint32_t)((uint64_t)blockIdx.x * ntiles / gridDim.x);
  const uint32_t s = find_seg_by_tile(segs, nsegs, tile);
  const SegDesc sd = segs[s];
  const uint64_t rel = (uint64_t)(tile - sd.tile0) * kTile;
  const uint32_t valid = (uint32_t)(sd.len - rel < (uint64_t)kTile ? sd.len - rel : (uint64_t)kTile);
  const uint32_t o = threadIdx.x * 32u;
  uint32_t nl = 0;
  if (o < valid) {
    const uint4* p = reinterpret_cast<const uint4*>(bytes + sd.base + rel + o);
    const uint4 x0 = p[0], x1 = p[1];  // (past the stream end: masked below; the batch has read slack)
    const uint32_t m = eq_mask16_nl(x0) | (eq_mask16_nl(x1) << 16);
    const uint32_t n = valid - o;
    nl = (uint32_t)__popc(n >= 32u ? m : (m & ((1u << n) - 1u)));
  }
  nl = wave_sum(nl);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = nl;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    out[2 * blockIdx.x + 1] = valid;
  }
}

hipError_t launch_nlsample(const uint8_t* bytes, const SegDesc* segs, uint32_t nsegs, uint32_t ntiles, uint32_t blocks,
                           uint32_t* out, hipStream_t st) {
  if (ntiles == 0 || blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_nlsample, dim3(blocks), dim3(256), 0, st, bytes, segs, nsegs, ntiles, out);
  return hipGetLastError();
}

size_t nfa_lds_bytes(const DevPatterns& P) {
  return 8ull * P.rx_count * (P.rx_classes + P.rx_maxpos + 4) + 256;
}

// KLF_SCAN_EVENTS=0 (A/B builds): no dispatch timestamps on k_scan / k_tcopy
static bool env_off(const char* name) {
  const char* v = getenv(name);
  return v && !strcmp(v, "0");
}

// the scan's timing events for the current launch_pipeline call (ev[7], ev[8]), else null
thread_local hipEvent_t t_scan_ev[2] = {nullptr, nullptr};

template <int MODE, int QS, int QK = 3, int QQ = 4, bool QA = false, bool FUSE = false>
int scan_occupancy() {
  static int occ = 0;  // queried once per variant: the host query delays the launch
  if (occ == 0) {
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan<MODE, QS, QK, QQ, QA, FUSE>, kThreads, 0);
    occ = occ < 1 ? 1 : (occ > 8 ? 8 : occ);
    if (getenv("KLF_DIAG"))
      fprintf(stderr, "[klf] k_scan<%d,%d,%d,%d,%d,%d>: %d blocks per CU\n", MODE, QS, QK, QQ, (int)QA, (int)FUSE, occ);
  }
  return occ;
}
template <int MODE, int QS, int QK = 3, int QQ = 4, bool QA = false, bool FUSE = false>
hipError_t launch_scan(const RunArgs& a, hipStream_t st, int num_cus) {
  const int occ = scan_occupancy<MODE, QS, QK, QQ, QA, FUSE>();
  uint32_t grid = (uint32_t)(num_cus * occ);
  if (grid > a.ntiles) grid = a.ntiles;
  if (FUSE) grid = (a.fuse_nranges + kThreads / 64 - 1) / (kThreads / 64);  // a wave per range
  if (t_scan_ev[0])  // the dispatch's own start / end timestamps (no event record beside it)
    hipExtLaunchKernelGGL((k_scan<MODE, QS, QK, QQ, QA, FUSE>), dim3(grid), dim3(kThreads), 0, st, t_scan_ev[0],
                          t_scan_ev[1], 0, a, a.tile_seg, a.segs);
  else
    hipLaunchKernelGGL((k_scan<MODE, QS, QK, QQ, QA, FUSE>), dim3(grid), dim3(kThreads), 0, st, a, a.tile_seg,
                       a.segs);
  return hipGetLastError();
}
template <int QS, int QQ>
hipError_t launch_gen_q(const RunArgs& a, hipStream_t st, int num_cus) {
  if constexpr (QS == 4)
    if (a.pats.qf_k == kQfTwoLevel)  // the two-level probe (stride 4, no anchor)
      return launch_scan<kScanGen, 4, (int)kQfTwoLevel, QQ>(a, st, num_cus);
  if (QS == 8 && a.pats.qf_anc_on)  // short needles anchored (only beside stride-8 probes)
    return a.pats.qf_k == 2 ? launch_scan<kScanGen, QS, 2, QQ, true>(a, st, num_cus)
                            : launch_scan<kScanGen, QS, 3, QQ, true>(a, st, num_cus);
  return a.pats.qf_k == 2 ? launch_scan<kScanGen, QS, 2, QQ>(a, st, num_cus)
                          : launch_scan<kScanGen, QS, 3, QQ>(a, st, num_cus);
}
template <int QS>
hipError_t launch_gen(const RunArgs& a, hipStream_t st, int num_cus) {
  return a.pats.qf_w24 ? launch_gen_q<QS, 4>(a, st, num_cus) : launch_gen_q<QS, 3>(a, st, num_cus);
}

static hipError_t launch_tail_stage(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus, uint32_t& m);

int fuse_waves(int num_cus) {
  return num_cus * scan_occupancy<kScanPlain, 1, 3, 4, false, true>() * (kThreads / 64);
}

hipError_t launch_scatter(const RunArgs& a, hipStream_t st, int num_cus) {
#ifndef KLF_SCATTER_GRID
#define KLF_SCATTER_GRID 8  // k_scatter workgroups per CU at most
#endif
  // up to 8 waves per 64-tile group (scatter_body splits a group's lines over them)
  uint32_t sg = ((a.ntiles + kScatterGroup - 1) / kScatterGroup * 8 + 3) / 4;
  if (sg > (uint32_t)num_cus * KLF_SCATTER_GRID) sg = num_cus * KLF_SCATTER_GRID;
  if (sg == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter, dim3(sg), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_pipeline(const RunArgs& a0, hipStream_t st, hipEvent_t* ev, int num_cus, int phase,
                           uint32_t* ev_mask) {
  RunArgs a = a0;
  hipError_t e;
  uint32_t m_local = 0;
  uint32_t& m = ev_mask ? *ev_mask : m_local;
#define KLF_TRY(x) do { e = (x); if (e != hipSuccess) return e; } while (0)
#define KLF_REC(k) do { KLF_TRY(hipEventRecord(ev[k], st)); m |= 1u << (k); } while (0)
  // phases: 0 all; 1 through the tile index, 2 the rest (a first run's line count between
  // them); 3 through k_scan, 4 the rest (the host joins the literal automaton's thread while
  // the scan runs: nothing before k_tindex reads it)
  if (phase != 2 && phase != 4) {
  if (ev) KLF_REC(0);
  {
    const uint32_t nw = a.nsegs * (uint32_t)(sizeof(SegOut) / 8);
    uint32_t g = (nw + 255) / 256;
    g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
    hipLaunchKernelGGL(k_init, dim3(g), dim3(256), 0, st, a);
    KLF_TRY(hipGetLastError());
  }
  if (a.build_tiles) {
    const uint32_t g = (a.ntiles + 255) / 256;
    hipLaunchKernelGGL(k_tiles, dim3(g < 4096 ? g : 4096), dim3(256), 0, st, a.segs, a.nsegs, a.ntiles,
                       a.tile_seg);
    KLF_TRY(hipGetLastError());
  }
  // ev[1] only with stage times: each event record idles the GPU for a few us, and the
  // scan's own time is then taken from ev[0] (k_init in front of it: ~2 us)
  if (ev && a.stage_times) KLF_REC(1);
  {
    // k_scan alone (the roofline kernel): ev[7] / ev[8] carry the dispatch's own timestamps
    const bool no_ev = env_off("KLF_SCAN_EVENTS");  // A/B (read per launch: tests toggle it)
    t_scan_ev[0] = ev && !no_ev ? ev[7] : nullptr;
    t_scan_ev[1] = ev && !no_ev ? ev[8] : nullptr;
    if (t_scan_ev[0]) m |= (1u << 7) | (1u << 8);
    if (a.grep_mode == kGrepLit1)
      KLF_TRY((launch_scan<kScanLit, 1>(a, st, num_cus)));
    else if (a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.qf_stride == 4)
      KLF_TRY((launch_gen<4>(a, st, num_cus)));
    else if (a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.qf_stride == 6)
      KLF_TRY((launch_gen<6>(a, st, num_cus)));
    else if (a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.qf_stride == 8)
      KLF_TRY((launch_gen<8>(a, st, num_cus)));
    else if (a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.qf_stride == 2)
      KLF_TRY((launch_gen<2>(a, st, num_cus)));
    else if (a.grep_mode == kGrepGeneral && a.pats.qf_on)
      KLF_TRY((launch_gen<1>(a, st, num_cus)));
    else if (a.fuse)
      KLF_TRY((launch_scan<kScanPlain, 1, 3, 4, false, true>(a, st, num_cus)));
    else
      KLF_TRY((launch_scan<kScanPlain, 1>(a, st, num_cus)));
    t_scan_ev[0] = t_scan_ev[1] = nullptr;  // (no event record behind it: each idles the GPU ~6 us)
  }
  if (phase == 3) return hipSuccess;
  }  // phase != 2, 4
  if (phase != 2) {
  {
    if (!a.tindex_wide) {
      hipLaunchKernelGGL((k_tindex<4, 0>), dim3((a.ntiles + 1023) / 1024), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
      hipLaunchKernelGGL((k_tindex<4, 1>), dim3((a.ntiles + 1023) / 1024), dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((k_tindex<16, 0>), dim3((a.ntiles + 4095) / 4096), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
      hipLaunchKernelGGL((k_tindex<16, 1>), dim3((a.ntiles + 4095) / 4096), dim3(256), 0, st, a);
    }
    KLF_TRY(hipGetLastError());
    KLF_TRY(hipGetLastError());
  }
  if (phase == 1) return hipSuccess;
  }  // phase != 2: the tile index
  // Regex sets: k_scatter and k_verify as one launch (k_scatter_verify; measured with two
  // streams: C5 -0.10 ms per step); a literal set's heavier verification (C4: 1,024 literals)
  // contends with the scatter instead (+0.08 ms), so literal-only sets keep the serial order.
#ifndef KLF_SV_FUSED
#define KLF_SV_FUSED 1  // regex sets: k_scatter and k_verify as one launch (0: two, for traces)
#endif
  const bool fused_sv = KLF_SV_FUSED && a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.rx_count;
  if (fused_sv) {
    uint32_t nsb = ((a.ntiles + kScatterGroup - 1) / kScatterGroup + 3) / 4;
    if (nsb > (uint32_t)num_cus * 4) nsb = num_cus * 4;
    if (nsb == 0) nsb = 1;
    RunArgs w = a;  // windowed index: the scatter part is the pre-count pass (deferred lines only)
    if (a.win_index) w.scatter_mode = 1;
    hipLaunchKernelGGL(k_scatter_verify, dim3(nsb + num_cus * 8), dim3(256), 0, st, w, nsb);
    KLF_TRY(hipGetLastError());
  } else if (a.win_index) {  // tiles with deferred lines now: their match bits come from the slots
    RunArgs w = a;
    w.scatter_mode = 1;
    KLF_TRY(launch_scatter(w, st, num_cus));
  } else if (!a.lazy_index) {
    KLF_TRY(launch_scatter(a, st, num_cus));
  }
  if (ev && a.stage_times && !fused_sv) KLF_REC(2);  // ~5 us of idle GPU each
  if (a.grep_mode == kGrepGeneral && a.pats.qf_on) {
    if (!fused_sv) {
      hipLaunchKernelGGL(k_verify, dim3(num_cus * 8), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
    }
    if (ev && a.stage_times && fused_sv) KLF_REC(2);
    if (a.count_pats) {
      hipLaunchKernelGGL(k_fixcount, dim3(num_cus * 2), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
    }
  }
  if (a.grep_mode == kGrepGeneral && a.pats.qf_on && a.pats.rx_count) {
    const size_t lds = nfa_lds_bytes(a.pats);
    if (lds <= kNfaMaxLds) {
      if (a.pats.rx_unbounded < a.pats.rx_count)
        hipLaunchKernelGGL(k_nfa_win<true>, dim3(num_cus * 2), dim3(256), lds, st, a);
      KLF_TRY(hipGetLastError());
      if (a.pats.rx_unbounded) hipLaunchKernelGGL(k_nfa<true>, dim3(num_cus * 4), dim3(256), lds, st, a);
    } else {
      if (a.pats.rx_unbounded < a.pats.rx_count)
        hipLaunchKernelGGL(k_nfa_win<false>, dim3(num_cus * 2), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
      if (a.pats.rx_unbounded) hipLaunchKernelGGL(k_nfa<false>, dim3(num_cus * 4), dim3(256), 0, st, a);
    }
    KLF_TRY(hipGetLastError());
  }
  // (skip_match: a prefiltered set launches no k_match; an overflowed hit list or NFA queue,
  // whose lines k_match would decide, makes the host redo the run with it)
  if ((a.grep_mode == kGrepGeneral || a.grep_mode == kGrepAll) && !a.skip_match) {
    hipLaunchKernelGGL(k_match, dim3(num_cus * 8), dim3(256), 0, st, a);
    KLF_TRY(hipGetLastError());
  }
  if (ev && a.stage_times) KLF_REC(3);  // ~5 us of idle GPU each
  KLF_TRY(launch_tail_stage(a, st, ev, num_cus, m));
  if (ev) KLF_REC(5);
#undef KLF_TRY
#undef KLF_REC
  return hipSuccess;
}

// Matched counts, kubelet tail window, window prefix, compaction + copy (the stages after
// the matchers): shared by launch_pipeline and launch_retail.
static hipError_t launch_tail_stage(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus, uint32_t& m) {
  hipError_t e;
#define KLF_TRY(x) do { e = (x); if (e != hipSuccess) return e; } while (0)
  if (a.grep_mode != kGrepNone) {
    const uint64_t nchunks = a.cap_lines / kMatchChunk + 1;
    // (16 blocks per CU: each 8,192-line chunk is a load, a block reduction and two barriers,
    // latency more than bytes -- C4's 11,700 chunks took 12 rounds of 4 blocks per CU, 24 us)
    const uint32_t g = (uint32_t)(nchunks < (uint64_t)num_cus * 16 ? nchunks : (uint64_t)num_cus * 16);
    hipLaunchKernelGGL(k_mcount, dim3(g), dim3(256), 0, st, a);
    KLF_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_tailw, dim3(a.nsegs), dim3(256), 0, st, a);
  KLF_TRY(hipGetLastError());
  if (a.lazy_index && !a.fuse) KLF_TRY(launch_scatter(a, st, num_cus));  // (exits at once on the dense path)
  if (a.win_index) {  // the tail windows' lines
    RunArgs w = a;
    w.scatter_mode = 2;
    KLF_TRY(launch_scatter(w, st, num_cus));
  }
  if (ev && a.stage_times) {  // ~5 us of idle GPU each
    KLF_TRY(hipEventRecord(ev[4], st));
    m |= 1u << 4;
  }
  if (a.fuse) {  // the scan compacted every range: only the bytes carried into them are left
    hipLaunchKernelGGL(k_fcarry, dim3((a.fuse_nranges + 3) / 4), dim3(256), 0, st, a);
    KLF_TRY(hipGetLastError());
    return hipSuccess;
  }
  {
    const uint32_t gt = (a.ntiles + 4 * kTkBatch - 1) / (4 * kTkBatch);
    uint32_t gp = (uint32_t)num_cus * 8;
    if (a.plan_mode == 1) {  // one ticket per block: a grid of one block per CU at most
      gp = (uint32_t)num_cus;
      if (a.grep_mode == kGrepNone && a.tail >= 0) {  // (<= S (N + 1) window lines without patterns)
        const uint64_t wmax = (uint64_t)a.nsegs * ((uint64_t)a.tail + 1) / kCompactLines + 1;
        gp = wmax < gp ? (uint32_t)wmax : gp;
      }
    }
    if (a.plan_mode != 2) {
      hipLaunchKernelGGL(k_cplan, dim3(a.compact_mode != 1 && gt < gp ? gt : gp), dim3(256), 0, st, a, a.tile_seg,
                         a.segs, a.tstat, a.tile_base, a.segout);
      KLF_TRY(hipGetLastError());
    }
    const uint32_t nb = (a.ntiles + 4095) / 4096;
    if (a.plan_mode == 0) {
      hipLaunchKernelGGL(k_cmid, dim3(nb), dim3(256), 0, st, a);
      KLF_TRY(hipGetLastError());
    }
    const uint32_t gg = (uint32_t)num_cus * KLF_CG_GRID;
    hipLaunchKernelGGL(k_cmove, dim3(nb > gg ? nb : gg), dim3(kThreads), 0, st, a);
    KLF_TRY(hipGetLastError());
  }
  // (skip_tcopy: a --tail run that has not taken the dense path before launches no k_tcopy;
  // the host launches it after the fact when this one did, launch_tcopy)
  if (a.compact_mode != 1 && !a.skip_tcopy) KLF_TRY(launch_tcopy(a, st, ev, num_cus, &m));
#undef KLF_TRY
  return hipSuccess;
}

hipError_t launch_tcopy(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus, uint32_t* ev_mask) {
  const uint32_t gk = (a.ntiles + kTcWaves - 1) / kTcWaves;
  // persistent grid: one resident generation of blocks, so every wave's prefetch
  // pipeline runs over its whole share of tiles
  static int occ = 0;
  if (occ == 0) {
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_tcopy, 64 * kTcWaves, 0);
    occ = occ < 1 ? 1 : (occ > 32 ? 32 : occ);
    if (getenv("KLF_DIAG")) fprintf(stderr, "[klf] k_tcopy: %d blocks of %d waves per CU\n", occ, kTcWaves);
  }
  const uint32_t gc = (uint32_t)num_cus * (uint32_t)occ;
  if (ev && !env_off("KLF_SCAN_EVENTS")) {  // ev[9] / ev[10]: the dispatch's own timestamps
    hipExtLaunchKernelGGL(k_tcopy, dim3(gk < gc ? gk : gc), dim3(64 * kTcWaves), 0, st, ev[9], ev[10], 0, a,
                          reinterpret_cast<const uint4*>(a.trec), a.kbase, a.truns);
    if (ev_mask) *ev_mask |= (1u << 9) | (1u << 10);
  } else {
    hipLaunchKernelGGL(k_tcopy, dim3(gk < gc ? gk : gc), dim3(64 * kTcWaves), 0, st, a,
                       reinterpret_cast<const uint4*>(a.trec), a.kbase, a.truns);
  }
  return hipGetLastError();
}

hipError_t launch_retail(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus, uint32_t* ev_mask) {
  uint32_t m_local = 0;
  uint32_t& m = ev_mask ? *ev_mask : m_local;
  hipError_t e = hipEventRecord(ev[0], st);
  if (e != hipSuccess) return e;
  m |= 1u;
  hipLaunchKernelGGL(k_retail_init, dim3((a.nsegs + 255) / 256 < 1024 ? (a.nsegs + 255) / 256 : 1024), dim3(256), 0,
                     st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = launch_tail_stage(a, st, ev, num_cus, m)) != hipSuccess) return e;
  if ((e = hipEventRecord(ev[5], st)) == hipSuccess) m |= 1u << 5;
  return e;
}

}  // namespace klf
