// klf_kernels.hip — CDNA4 (gfx950) kernels of the klogs filter path.
//
// Pipeline over one device batch (streams laid out as 256-B-aligned segments):
//   K1 k_scan      newline scan + line index (decoupled look-back over 16 KiB tiles),
//                  RFC3339Nano parse + since mask per line, fused single-literal grep
//   K2 k_match     general pattern sets: Aho-Corasick DFA + Glushkov bit-parallel NFA
//   K3 k_count     per-stream parsed / since_ok / matched counts
//      k_tail      kubelet tail rule -> per-stream candidate window (one block / stream)
//      k_wprefix   exclusive prefix of window sizes
//   K4 k_compact   output offsets (look-back over 1024-line blocks) + content gather copy
// Semantics: SPEC.md (kubelet logs.go ReadLogs / tail.go FindTailLineStartIndex /
// Go time.Parse(RFC3339Nano) / bytes.Contains / regexp.Match).
#include <hip/hip_runtime.h>

#include "klf_kernels.hpp"
#include "klf_ts.hpp"

namespace klf {
namespace {

// ------------------------------------------------------------------ small helpers ---

__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  // high bit of each byte set iff that byte is 0 (exact, no false positives)
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t pack4(uint32_t z) {
  return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}
// 64-bit mask: bit i set iff byte i of the 64 bytes in w equals the byte in `pat`
// (pat = byte * 0x01010101).
__device__ __forceinline__ uint64_t eq_mask64(const uint32_t* w, uint32_t pat) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) lo |= pack4(zero_bytes(w[j] ^ pat)) << (4 * j);
#pragma unroll
  for (int j = 0; j < 8; ++j) hi |= pack4(zero_bytes(w[8 + j] ^ pat)) << (4 * j);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t atomic_load_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void atomic_store_u64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint64_t kFlagA = 1ull << 62;  // aggregate published
constexpr uint64_t kFlagP = 2ull << 62;  // inclusive prefix published
constexpr uint64_t kFlagMask = 3ull << 62;
constexpr uint32_t kSpinLimit = 1u << 24;

// ---- scan summary monoid -----------------------------------------------------------
// (count of line-end events, IND = a line starts inside the span, P = the line open at
// the span's end has a parseable prefix).
// combine(a, b) with a before b.  Packed u32 (thread/block level) and u64 (tiles).
constexpr uint32_t kInd32 = 1u << 16, kP32 = 1u << 17;
__device__ __forceinline__ uint32_t comb32(uint32_t a, uint32_t b) {
  const uint32_t cnt = (a & 0xFFFFu) + (b & 0xFFFFu);
  const uint32_t pb = (b & kInd32) ? (b & kP32) : (a & kP32);
  return cnt | ((a | b) & kInd32) | pb;
}
constexpr uint64_t kCnt64 = (1ull << 59) - 1;
constexpr uint64_t kP64 = 1ull << 59, kInd64 = 1ull << 61;
__device__ __forceinline__ uint64_t comb64(uint64_t a, uint64_t b) {
  const uint64_t cnt = ((a & kCnt64) + (b & kCnt64)) & kCnt64;
  const uint64_t pb = (b & kInd64) ? (b & kP64) : (a & kP64);
  return cnt | ((a | b) & kInd64) | pb;
}
__device__ __forceinline__ uint64_t widen(uint32_t x) {
  return (uint64_t)(x & 0xFFFFu) | ((x & kInd32) ? kInd64 : 0) | ((x & kP32) ? kP64 : 0);
}

__device__ __forceinline__ uint32_t wave_incl_scan_summary(uint32_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(x, d, 64);
    if (lane >= d) x = comb32(o, x);
  }
  return x;
}

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

// Decoupled look-back of one tile over a chain of u64 words, run by ONE WAVE: each
// round reads 64 predecessors at once, waits until all of them have published
// (aggregate or inclusive), stops at the nearest inclusive prefix and folds the window
// with an ordered shuffle reduction (earlier tiles sit at higher lanes).  Returns the
// exclusive prefix (no flag bits) in every lane.  `agg` has no flag bits.  Spins are
// bounded: a timeout sets counters[2] bit 1 so the host reports an error instead of the
// GPU hanging.
template <class Comb>
__device__ uint64_t lookback_wave(uint64_t* st, uint32_t idx, uint64_t agg, uint64_t ident, Comb comb,
                                  uint32_t* err_flag, int lane) {
  if (idx == 0) {
    if (lane == 0) atomic_store_u64(&st[0], agg | kFlagP);
    return ident;
  }
  if (lane == 0) atomic_store_u64(&st[idx], agg | kFlagA);
  uint64_t acc = ident;
  int64_t hi = (int64_t)idx - 1;
  for (;;) {
    const int64_t j = hi - lane;
    uint64_t w = kFlagP | ident;  // before tile 0: acts as an empty inclusive prefix
    bool ready = j < 0;
    uint32_t spins = 0;
    for (;;) {
      if (!ready) {
        w = atomic_load_u64(&st[j]);
        ready = (w & kFlagMask) != 0;
      }
      if (__all(ready)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        if (lane == 0) atomicOr(err_flag, 2u);
        return acc;
      }
    }
    const uint64_t pmask = __ballot((w & kFlagMask) == kFlagP);
    const int plane = pmask ? __ffsll((unsigned long long)pmask) - 1 : 64;
    uint64_t v = lane <= plane ? (w & ~kFlagMask) : ident;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t o = __shfl_down(v, d, 64);
      if (lane + d < 64) v = comb(o, v);
    }
    acc = comb(__shfl(v, 0, 64), acc);
    if (plane < 64) break;
    hi -= 64;
  }
  if (lane == 0) atomic_store_u64(&st[idx], comb(acc, agg) | kFlagP);
  return acc;
}

struct SumComb {
  __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return (a + b) & ~kFlagMask; }
};
struct ScanComb {
  __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return comb64(a, b); }
};

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

// Byte source for the timestamp parser: the tile's LDS image (tile + halo) when the
// byte is there, global memory otherwise; -1 past the end of the stream.
struct LineBytes {
  const uint8_t* lds;   // LDS image; lds[0] = stream byte rel_lo
  const uint8_t* seg;   // global stream base
  int64_t p0;           // stream offset of the line start
  int64_t rel_lo;
  int64_t seg_len;
  __device__ __forceinline__ int operator()(uint32_t i) const {
    const int64_t q = p0 + (int64_t)i;
    if (q >= seg_len) return -1;
    const int64_t o = q - rel_lo;
    if (o >= 0 && o < kTile + kHalo) return lds[o];
    return seg[q];
  }
};
struct GlobalBytes {
  const uint8_t* seg;
  int64_t p0;
  int64_t end;
  __device__ __forceinline__ int operator()(uint32_t i) const {
    const int64_t q = p0 + (int64_t)i;
    return q < end ? seg[q] : -1;
  }
};

// Cold-path parse (kept out of line so the hot loop's register budget stays at 64).
__device__ __attribute__((noinline)) bool parse_at_cold(const uint8_t* lds, const uint8_t* seg, int64_t p0,
                                                       int64_t rel_lo, int64_t seg_len, uint32_t* plen) {
  TsResult r;
  LineBytes gb{lds, seg, p0, rel_lo, seg_len};
  return parse_line_prefix(gb, r, *plen);
}

__device__ __forceinline__ uint16_t make_meta(bool ok, bool since_ok, uint32_t plen) {
  if (!ok) return 0;
  const uint32_t pl = plen < kPlenEscape ? plen : kPlenEscape;
  return (uint16_t)(Meta::kParsed | (since_ok ? Meta::kSince : 0) | (pl << 2));
}

// ============================================================== K1: the scan kernel ==
// Persistent 256-thread workgroups, one 16 KiB tile at a time; thread t owns bytes
// [64t, 64t+64).  Per tile:
//   1. claim (ticket groups, below) and stage tile + halo in LDS;
//   2. line-end events ('\n', and the stream's last byte) -> counts -> block reduce ->
//      publish the tile's AGGREGATE immediately (the chain is a plain line count, so a
//      successor's look-back never waits on our parsing);
//   3. parse every line starting in the tile into LDS (meta + tile-relative offset);
//   4. look-back -> the tile's first global line index;
//   5. coalesced copy-out of line_off / meta; fused literal grep on the rare first+last
//      byte candidates.  Whether a hit lies in the content (after the first ' ') comes
//      from the line's plen; for a line begun in an earlier tile, from a backward scan
//      to its start and a re-parse (rare).
// Tiles with more than kMaxTileLines line starts (< 16 B per line: never kubelet
// output) take a slower per-thread path with the same results.

constexpr int kMaxTileLines = 1024;

// 4-bit mask of the zero bytes of x (exact): bit k set iff byte k of x is 0.
__device__ __forceinline__ uint32_t zmask4(uint32_t x) {
  const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 per zero byte
  return (z * 0x00204081u) >> 28;
}
__device__ __forceinline__ uint64_t eq_mask64_words(const uint32_t* w, uint32_t pat) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) lo |= zmask4(w[j] ^ pat) << (4 * j);
#pragma unroll
  for (int j = 0; j < 8; ++j) hi |= zmask4(w[8 + j] ^ pat) << (4 * j);
  return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void k_tiles(const SegDesc* segs, uint32_t nsegs, uint32_t ntiles,
                                               uint32_t* tile_seg) {
  for (uint32_t tile = blockIdx.x * 256 + threadIdx.x; tile < ntiles; tile += gridDim.x * 256)
    tile_seg[tile] = find_seg_by_tile(segs, nsegs, tile);
}

// Canonical kubelet prefix "YYYY-MM-DDTHH:MM:SS.nnnnnnnnnZ " (k8s logs.go timeFormatOut):
// 9 dword LDS reads instead of ~31 dependent byte reads.  Accepts exactly the inputs of
// this shape the general parser accepts (same value); anything else -> general parser.
__device__ __forceinline__ bool parse_fast_lds(const uint8_t* lds, uint32_t o, TsResult& r) {
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(lds);
  const uint32_t base = o >> 2, sh = (o & 3) * 8;
  uint32_t w[8];
  uint32_t prev = s32[base];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t nx = s32[base + j + 1];
    w[j] = sh ? (uint32_t)((((uint64_t)nx << 32) | prev) >> sh) : prev;
    prev = nx;
  }
#define KLF_B(k) ((w[(k) >> 2] >> (8 * ((k) & 3))) & 0xFFu)
  if (KLF_B(4) != '-' || KLF_B(7) != '-' || KLF_B(10) != 'T' || KLF_B(13) != ':' || KLF_B(16) != ':' ||
      KLF_B(19) != '.' || KLF_B(29) != 'Z' || KLF_B(30) != ' ')
    return false;
  // digits, folded as they are read (no per-byte array: keeps the register budget)
  bool ok = true;
  auto dig = [&](int k) -> uint32_t {
    const uint32_t v = KLF_B(k) - '0';
    ok &= v < 10;
    return v;
  };
  const int64_t year = dig(0) * 1000 + dig(1) * 100 + dig(2) * 10 + dig(3);
  const int month = (int)(dig(5) * 10 + dig(6)), day = (int)(dig(8) * 10 + dig(9));
  const int hour = (int)(dig(11) * 10 + dig(12)), minute = (int)(dig(14) * 10 + dig(15));
  const int second = (int)(dig(17) * 10 + dig(18));
  uint32_t ns = 0;
#pragma unroll
  for (int k = 20; k < 29; ++k) ns = ns * 10 + dig(k);
#undef KLF_B
  if (!ok) return false;
  if (month < 1 || month > 12 || hour >= 24 || minute >= 60 || second >= 60) return false;
  if (day < 1 || day > days_in_month(month, year)) return false;
  r.sec = days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + second;
  r.nsec = (int32_t)ns;
  r.len = 30;
  return true;
}

// General RFC3339Nano parse, out of line: non-canonical prefixes are rare, and keeping the
// byte-at-a-time parser out of the hot loop keeps the loop's register budget.
__device__ __attribute__((noinline)) bool parse_general_cold(const uint8_t* lds, const uint8_t* segp, int64_t p0,
                                                            int64_t rel_lo, int64_t seg_len, TsResult* r,
                                                            uint32_t* plen) {
  LineBytes gb{lds, segp, p0, rel_lo, seg_len};
  return parse_line_prefix(gb, *r, *plen);
}

// Parse of the line starting at stream offset p0: fast path from LDS, else general.
__device__ __forceinline__ bool parse_line_at(const uint8_t* lds, const uint8_t* segp, int64_t p0, int64_t rel_lo,
                                              int64_t seg_len, int64_t ssec, int32_t snsec, bool* since_ok,
                                              uint32_t* plen) {
  TsResult r;
  const int64_t o = p0 - rel_lo;
  bool ok;
  if (o >= 0 && o + 36 <= kTile + kHalo && p0 + 31 <= seg_len && parse_fast_lds(lds, (uint32_t)o, r)) {
    ok = true;
    *plen = 31;
  } else {
    LineBytes gb{lds, segp, p0, rel_lo, seg_len};
    ok = parse_line_prefix(gb, r, *plen);
  }
  *since_ok = ok && !time_before(r.sec, r.nsec, ssec, snsec);
  return ok;
}

// Rare path: content start of the line containing stream offset `pos` when that line
// began before `rel_lo` (scan back for its '\n', then parse).  -1 if unparseable.
__device__ __attribute__((noinline)) int64_t carried_content_start(const uint8_t* lds, const uint8_t* segp,
                                                                  int64_t rel_lo, int64_t seg_len,
                                                                  int64_t from) {
  int64_t ls = 0;
  for (int64_t q = from; q >= 0; --q) {
    const int64_t o = q - rel_lo;
    const uint8_t c = (o >= 0 && o < kTile + kHalo) ? lds[o] : segp[q];
    if (c == '\n') { ls = q + 1; break; }
  }
  uint32_t plen = 0;
  TsResult r;
  LineBytes gb{lds, segp, ls, rel_lo, seg_len};
  if (!parse_line_prefix(gb, r, plen)) return -1;
  return ls + plen;
}

#ifndef KLF_ABLATE
#define KLF_ABLATE 0
#endif

#ifndef KLF_SCAN_OCC
#define KLF_SCAN_OCC 6
#endif
template <bool LIT>
__global__ __launch_bounds__(kThreads, KLF_SCAN_OCC) void k_scan(RunArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTile + kHalo];
  __shared__ uint16_t s_meta[kMaxTileLines + 1];
  __shared__ uint16_t s_loff[kMaxTileLines + 1];
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_red[4][2];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_ticket;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t* err_flag = a.counters + 2;
  // Ticket groups: group g hands out tiles g, g+G, g+2G, ... in claim order.  One atomic
  // word saturates near 88 claims/us (MI355X_MICROARCH.md, row "dequeue"); G padded words
  // keep claims off the critical path.  A tile is claimed only when it is about to be
  // processed (a claimed-but-idle tile would stall every later look-back).  Deadlock-free
  // while every group keeps a resident workgroup: the lowest unfinished tile is either
  // being processed (its look-back needs only lower, finished tiles) or is the next
  // claim of its group, whose workgroups are then idle and claim it.
  const uint32_t g = blockIdx.x % kScanGroups;
  uint32_t* ctr = a.counters + kCtrScanGroups + g * kCtrStride;
  for (;;) {
    if (t == 0) s_ticket = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_ticket * kScanGroups + g;
    if (tile >= a.ntiles) break;
    const uint32_t s = a.tile_seg[tile];
    const SegDesc sd = a.segs[s];
    const int64_t rel_lo = (int64_t)(tile - sd.tile0) * kTile;
    const int64_t seg_len = (int64_t)sd.len;
    const int64_t tile_len = seg_len - rel_lo < kTile ? seg_len - rel_lo : kTile;
    const bool first = rel_lo == 0;
    const bool last = rel_lo + kTile >= seg_len;
    const uint8_t* segp = a.bytes + sd.base;

    // ---- 1. stage tile + halo in LDS (coalesced 16 B per lane) ----
    {
      const uint4* gp = reinterpret_cast<const uint4*>(segp + rel_lo);
      uint4* l = reinterpret_cast<uint4*>(s_tile);
#pragma unroll
      for (int v = 0; v < kTile / (kThreads * 16); ++v) l[v * kThreads + t] = gp[v * kThreads + t];
      if (t < kHalo / 16) l[kTile / 16 + t] = gp[kTile / 16 + t];
    }
    __syncthreads();

    // ---- 2. events of my 64 bytes -> counts -> publish the aggregate ----
    const int64_t nvalid_s = tile_len - (int64_t)t * kBytesPerThread;
    const int nvalid = nvalid_s <= 0 ? 0 : (nvalid_s >= 64 ? 64 : (int)nvalid_s);
    const uint64_t vm = nvalid >= 64 ? ~0ull : ((1ull << nvalid) - 1);
    const int64_t rel0 = rel_lo + (int64_t)t * kBytesPerThread;
    uint64_t nl, cand = 0;
    {
      uint32_t w[16];
      const uint4* l = reinterpret_cast<const uint4*>(s_tile + t * kBytesPerThread);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const uint4 x = l[v];
        w[4 * v] = x.x; w[4 * v + 1] = x.y; w[4 * v + 2] = x.z; w[4 * v + 3] = x.w;
      }
      nl = eq_mask64_words(w, 0x0A0A0A0Au) & vm;
      if (LIT) cand = eq_mask64_words(w, a.lit[0] * 0x01010101u) & vm;
    }
    const bool has_end = last && nvalid > 0 && rel0 + nvalid == seg_len;
    const int eb = nvalid - 1;
    uint64_t ev = nl, starts = nl;
    if (has_end) {
      ev |= 1ull << eb;
      starts &= ~(1ull << eb);
    }
    const bool reset = first && t == 0;
    const uint32_t cnt = (uint32_t)__popcll(ev);
    const uint32_t incl = wave_incl_scan_add(cnt, lane);
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t wexcl = 0, agg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < wv) wexcl += s_wsum[k];
      agg += s_wsum[k];
    }
    const uint32_t texcl = wexcl + incl - cnt;  // events of the tile before my bytes
    const bool staged = agg <= (uint32_t)kMaxTileLines;
    if (t == 0 && tile != 0) atomic_store_u64(&a.status[tile], (uint64_t)agg | kFlagA);

    // ---- 3. parse the lines starting in my bytes (into LDS when the tile fits) ----
    uint32_t n_parsed = 0, n_since = 0;
    if (staged) {
      if (reset) {
        bool so;
        uint32_t plen = 0;
        const bool ok = KLF_ABLATE >= 2 ? true : parse_line_at(s_tile, segp, rel0, rel_lo, seg_len, a.since_sec, a.since_nsec, &so, &plen);
        s_meta[0] = make_meta(ok, so, plen);
        s_loff[0] = 0;
        n_parsed += ok;
        n_since += so;
      }
      for (uint64_t m = starts; m;) {
        const int q = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint32_t k = texcl + (uint32_t)__popcll(ev & ((2ull << q) - 1));
        const int64_t p0 = rel0 + q + 1;
        bool so = true;
        uint32_t plen = 31;
        const bool ok = KLF_ABLATE >= 2 ? true : parse_line_at(s_tile, segp, p0, rel_lo, seg_len, a.since_sec, a.since_nsec, &so, &plen);
        s_meta[k] = make_meta(ok, so, plen);
        s_loff[k] = (uint16_t)(p0 - rel_lo);
        n_parsed += ok;
        n_since += so;
      }
    }

    // ---- 4. look-back: global index of the tile's first line ----
#if KLF_ABLATE >= 1
    if (t == 0) s_excl = 0;
#else
    if (wv == 0) {
      const uint64_t ex = lookback_wave(a.status, tile, (uint64_t)agg, 0ull, SumComb(), err_flag, lane);
      if (lane == 0) s_excl = ex;
    }
#endif
    __syncthreads();
    const uint64_t tile_lines = s_excl;
    const uint64_t lines_before = tile_lines + texcl;

    // ---- 5. write-out ----
    if (staged) {  // coalesced: local line k -> global tile_lines + k
      const uint32_t k0 = first ? 0 : 1;
      const bool tile_has_end = last;  // the stream's final event lies in this tile
      const uint32_t k1 = tile_has_end ? agg : agg + 1;
      for (uint32_t k = k0 + t; k < k1; k += kThreads) {
        const uint64_t l = tile_lines + k;
        if (l < a.cap_lines) {
          a.meta[l] = s_meta[k];
          a.line_off[l + s] = (uint64_t)rel_lo + s_loff[k];
        } else {
          atomicOr(err_flag, 1u);
        }
      }
    } else {  // dense tile: parse and write per thread
      if (reset) {
        bool so;
        uint32_t plen = 0;
        const bool ok = parse_line_at(s_tile, segp, rel0, rel_lo, seg_len, a.since_sec, a.since_nsec, &so, &plen);
        if (lines_before < a.cap_lines) {
          a.line_off[lines_before + s] = 0;
          a.meta[lines_before] = make_meta(ok, so, plen);
        } else {
          atomicOr(err_flag, 1u);
        }
        n_parsed += ok;
        n_since += so;
      }
      for (uint64_t m = starts; m;) {
        const int q = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint64_t l = lines_before + (uint64_t)__popcll(ev & ((2ull << q) - 1));
        const int64_t p0 = rel0 + q + 1;
        bool so;
        uint32_t plen = 0;
        const bool ok = parse_line_at(s_tile, segp, p0, rel_lo, seg_len, a.since_sec, a.since_nsec, &so, &plen);
        if (l < a.cap_lines) {
          a.line_off[l + s] = (uint64_t)p0;
          a.meta[l] = make_meta(ok, so, plen);
        } else {
          atomicOr(err_flag, 1u);
        }
        n_parsed += ok;
        n_since += so;
      }
    }
    if (reset) a.segout[s].line_lo = lines_before;
    if (has_end) {
      const uint64_t lend = lines_before + cnt;
      if (lend <= a.cap_lines) a.line_off[lend + s] = (uint64_t)seg_len;
      else atomicOr(err_flag, 1u);
      a.segout[s].line_hi = lend;
      a.segout[s].frag = (nl >> eb) & 1 ? 0 : 1;
    }

    // ---- fused single-literal grep (rare path: first-byte candidates) ----
    if (LIT && cand) {
      const uint32_t m = a.lit_len;
      {  // last-byte filter from the LDS window at +m-1 (word by word)
        const uint32_t off = (uint32_t)t * kBytesPerThread + m - 1;
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s_tile);
        const uint32_t base = off >> 2, sh = (off & 3) * 8;
        const uint32_t pat = a.lit[m - 1] * 0x01010101u;
        uint32_t prev = s32[base], lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t nx = s32[base + j + 1];
          const uint32_t wj = sh ? (uint32_t)((((uint64_t)nx << 32) | prev) >> sh) : prev;
          prev = nx;
          if (j < 8) lo |= zmask4(wj ^ pat) << (4 * j);
          else hi |= zmask4(wj ^ pat) << (4 * (j - 8));
        }
        cand &= ((uint64_t)hi << 32) | lo;
      }
      int64_t carried_cs = -2;  // content start of the line carried into my bytes (lazy)
      while (cand) {
        const int b = __ffsll((unsigned long long)cand) - 1;
        cand &= cand - 1;
        const int64_t pos = rel0 + b;
        if (pos + (int64_t)m > seg_len) continue;
        bool eq = true;
        for (uint32_t k = 1; k + 1 < m && eq; ++k) eq = s_tile[t * kBytesPerThread + b + k] == a.lit[k];
        if (!eq) continue;
        const uint64_t below = b == 0 ? 0 : ((1ull << b) - 1);
        const uint64_t E = ev & below;
        int64_t cs;  // content start of the hit's line, -1 = unparseable
        if (E || reset || (staged && (texcl > 0 || first))) {
          // the line starts inside this tile: its local index is the events before it
          const uint32_t kl = texcl + (uint32_t)__popcll(E);
          const int64_t p0 = E ? rel0 + (63 - __clzll(E)) + 1 : (reset ? rel0 : -1);
          if (staged) {
            const uint16_t mt = s_meta[kl];
            cs = (mt & Meta::kParsed) ? (int64_t)rel_lo + s_loff[kl] + (mt >> 2) : -1;
          } else if (p0 >= 0) {
            bool so;
            uint32_t plen = 0;
            cs = parse_line_at(s_tile, segp, p0, rel_lo, seg_len, 0, 0, &so, &plen) ? p0 + plen : -1;
          } else {
            if (carried_cs == -2) carried_cs = carried_content_start(s_tile, segp, rel_lo, seg_len, rel0 - 1);
            cs = carried_cs;
          }
        } else {
          if (carried_cs == -2) carried_cs = carried_content_start(s_tile, segp, rel_lo, seg_len, rel0 - 1);
          cs = carried_cs;
        }
        if (cs >= 0 && pos >= cs && cs <= pos) {
          const uint64_t l = lines_before + (uint64_t)__popcll(E);
          if (l < a.cap_lines) atomicOr(&a.bits[l >> 5], 1u << (l & 31));
        }
      }
    }

    // ---- per-tile counters ----
    const uint32_t pp = wave_sum(n_parsed), qq = wave_sum(n_since);
    if (lane == 0) { s_red[wv][0] = pp; s_red[wv][1] = qq; }
    __syncthreads();
    if (t == 0) {
      a.tile_cnt[2 * (size_t)tile] = s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0];
      a.tile_cnt[2 * (size_t)tile + 1] = s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1];
    }
    __syncthreads();  // LDS is reused by the next tile
  }
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

__global__ __launch_bounds__(256) void k_match(RunArgs a) {
  if (a.counters[2]) return;
  const uint64_t L = a.segout[a.nsegs - 1].line_hi;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < L; l += stride) {
    const uint16_t m = a.meta[l];
    if (!(m & Meta::kParsed)) continue;
    bool hit = a.grep_mode == kGrepAll;
    if (!hit) {
      const uint32_t s = find_seg_by_line(a.segout, a.nsegs, l);
      const uint8_t* segp = a.bytes + a.segs[s].base;
      const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
      const uint32_t plen = line_plen(a, m, segp, ls, le);
      uint64_t cs = ls + plen, ce = le;
      if (ce > cs && segp[ce - 1] == '\n') --ce;
      const uint8_t* p = segp + cs;
      const int64_t n = (int64_t)(ce - cs);
      if (a.pats.ac_states) hit = ac_match(a.pats, p, n);
      for (uint32_t r = 0; !hit && r < a.pats.rx_count; ++r) hit = rx_match(a.pats, r, p, n);
    }
    if (hit) atomicOr(&a.bits[l >> 5], 1u << (l & 31));
  }
}

// ============================================================== K3: per-stream counts ==
// Block-level segmented reduction: one atomic per (block, stream) when the block lies
// in one stream, per-thread atomics otherwise.
__device__ void seg_reduce_add(uint32_t seg, uint64_t v, uint64_t* dst_base, size_t stride_words,
                               uint32_t* s_seg, uint64_t* s_acc) {
  const int t = threadIdx.x;
  __syncthreads();
  if (t == 0) { s_seg[0] = seg; s_seg[1] = 0; }
  __syncthreads();
  if (seg != s_seg[0]) atomicOr(&s_seg[1], 1u);
  __syncthreads();
  if (s_seg[1] == 0) {
    const uint64_t ws = wave_sum(v);
    if ((t & 63) == 0) s_acc[t >> 6] = ws;
    __syncthreads();
    if (t == 0) {
      const uint64_t tot = s_acc[0] + s_acc[1] + s_acc[2] + s_acc[3];
      if (tot) atomicAdd((unsigned long long*)(dst_base + (size_t)seg * stride_words), (unsigned long long)tot);
    }
  } else if (v) {
    atomicAdd((unsigned long long*)(dst_base + (size_t)seg * stride_words), (unsigned long long)v);
  }
}

__global__ __launch_bounds__(256) void k_count(RunArgs a, uint32_t nblk_tiles, uint64_t nwords) {
  __shared__ uint32_t s_seg[2];
  __shared__ uint64_t s_acc[4];
  if (a.counters[2]) return;
  const size_t stride = sizeof(SegOut) / 8;
  if (blockIdx.x < nblk_tiles) {
    // parsed / since_ok from the per-tile records: one tile per thread
    const uint32_t tile = blockIdx.x * 256 + threadIdx.x;
    const uint32_t tclamp = tile < a.ntiles ? tile : a.ntiles - 1;
    const uint32_t s = find_seg_by_tile(a.segs, a.nsegs, tclamp);
    const uint64_t p = tile < a.ntiles ? a.tile_cnt[2 * (size_t)tile] : 0;
    const uint64_t q = tile < a.ntiles ? a.tile_cnt[2 * (size_t)tile + 1] : 0;
    seg_reduce_add(s, p, &a.segout[0].parsed, stride, s_seg, s_acc);
    seg_reduce_add(s, q, &a.segout[0].since_ok, stride, s_seg, s_acc);
  } else {
    // matched = popcount of the match bitmap per stream: one 32-line word per thread
    if (a.grep_mode == kGrepNone) return;
    const uint64_t L = a.segout[a.nsegs - 1].line_hi;
    const uint64_t wi = (uint64_t)(blockIdx.x - nblk_tiles) * 256 + threadIdx.x;
    const uint64_t l0 = wi * 32;
    const uint64_t lc = l0 < L ? l0 : (L ? L - 1 : 0);
    uint32_t s = find_seg_by_line(a.segout, a.nsegs, lc);
    uint64_t v = 0;
    uint32_t word = (wi < nwords && l0 < L) ? a.bits[wi] : 0;
    if (word) {
      // split the word at stream boundaries
      for (;;) {
        const uint64_t hi = a.segout[s].line_hi;
        if (hi >= l0 + 32 || s + 1 >= a.nsegs) { v += __popc(word); break; }
        const uint32_t nb = (uint32_t)(hi - l0);
        const uint32_t part = nb >= 32 ? word : (word & ((1u << nb) - 1));
        if (part) atomicAdd((unsigned long long*)&a.segout[s].matched, (unsigned long long)__popc(part));
        word &= ~((nb >= 32) ? ~0u : ((1u << nb) - 1));
        ++s;
        if (!word) break;
      }
    }
    seg_reduce_add(s, v, &a.segout[0].matched, stride, s_seg, s_acc);
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

__global__ __launch_bounds__(256) void k_tail(RunArgs a) {
  __shared__ uint32_t s_w[4];
  __shared__ uint64_t s_found;
  const uint32_t s = blockIdx.x;
  const int t = threadIdx.x;
  if (a.counters[2]) return;
  SegOut& so = a.segout[s];
  const uint64_t lo = so.line_lo, hi = so.line_hi;
  if (a.tail < 0) {
    if (t == 0) { so.win_lo = lo; so.win_hi = hi; }
    return;
  }
  const uint64_t n = (uint64_t)a.tail;
  const bool grep = a.grep_mode != kGrepNone;
  const uint64_t gsize = grep ? so.matched : hi - lo;
  const uint64_t gfrag = (so.frag && hi > lo && gbit(a, hi - 1)) ? 1 : 0;
  const uint64_t T = gsize - gfrag;
  const uint64_t k = T > n ? T - n : 0;
  const uint64_t need = gsize - k;  // G lines at / after the start: <= n + 1
  if (need == 0) {
    if (t == 0) { so.win_lo = hi; so.win_hi = hi; }
    return;
  }
  // backward: the need-th G line from the end
  if (t == 0) s_found = lo;
  uint64_t cum = 0;
  for (uint64_t end = hi; end > lo;) {
    const uint64_t cs = end - lo > 256 ? end - 256 : lo;
    const uint64_t l = cs + t;
    const uint32_t g = (l < end && gbit(a, l)) ? 1u : 0u;
    uint32_t tot;
    const uint32_t pre = block_incl_scan_u32(g, s_w, &tot);
    if (cum + tot >= need) {
      const uint64_t needc = need - cum;
      if (g && (uint64_t)(tot - pre + 1) == needc) s_found = l;
      break;
    }
    cum += tot;
    end = cs;
  }
  __syncthreads();
  const uint64_t start = s_found;
  // forward: the n-th parsed G line at / after start bounds the window
  if (t == 0) s_found = hi;
  cum = 0;
  if (n == 0) {
    if (t == 0) s_found = start;
  } else {
    for (uint64_t b = start; b < hi; b += 256) {
      const uint64_t l = b + t;
      const uint32_t pg = (l < hi && gbit(a, l) && (a.meta[l] & Meta::kParsed)) ? 1u : 0u;
      uint32_t tot;
      const uint32_t pre = block_incl_scan_u32(pg, s_w, &tot);
      if (cum + tot >= n) {
        if (pg && cum + pre == n) s_found = l + 1;
        break;
      }
      cum += tot;
    }
  }
  __syncthreads();
  if (t == 0) { so.win_lo = start; so.win_hi = s_found; }
}

__global__ __launch_bounds__(256) void k_wprefix(RunArgs a) {
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
  if (t == 0) {
    a.wpre[a.nsegs] = carry;
    const uint64_t nb = (carry + kCompactLines - 1) / kCompactLines;
    a.counters[3] = (uint32_t)(nb < a.max_cblocks ? nb : a.max_cblocks);
  }
}

// ======================================================= K4: compaction + gather copy ==
__global__ __launch_bounds__(kThreads) void k_compact(RunArgs a) {
  __shared__ uint64_t s_src[kCompactLines];
  __shared__ uint64_t s_dst[kCompactLines];
  __shared__ uint32_t s_len[kCompactLines];
  __shared__ uint64_t s_wb[4], s_wc[4];
  __shared__ uint64_t s_exb, s_exc;
  __shared__ uint32_t s_ticket;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (a.counters[2]) return;
  const uint64_t W = a.wpre[a.nsegs];
  const uint32_t nblocks = a.counters[3];
  uint64_t* stb = a.cstatus;
  uint64_t* stc = a.cstatus + a.max_cblocks;
  for (;;) {
    if (t == 0) s_ticket = atomicAdd(&a.counters[1], 1u);
    __syncthreads();
    const uint32_t blk = s_ticket;
    if (blk >= nblocks) break;
    const uint64_t w0 = (uint64_t)blk * kCompactLines + (uint64_t)t * 4;
    // segment of my first line
    uint32_t s = 0;
    {
      const uint64_t wq = w0 < W ? w0 : (W ? W - 1 : 0);
      uint32_t lo = 0, hi = a.nsegs;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.wpre[mid] <= wq) lo = mid; else hi = mid;
      }
      s = lo;
    }
    uint64_t src[4], blen = 0;
    uint32_t len[4], seg_of[4];
    uint32_t nsel = 0;
    bool is_first[4], is_last[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t wj = w0 + j;
      len[j] = 0; src[j] = 0; is_first[j] = is_last[j] = false; seg_of[j] = s;
      if (wj >= W) continue;
      while (wj >= a.wpre[s + 1]) ++s;
      seg_of[j] = s;
      is_first[j] = wj == a.wpre[s];
      is_last[j] = wj + 1 == a.wpre[s + 1];
      const uint64_t l = a.segout[s].win_lo + (wj - a.wpre[s]);
      const uint16_t m = a.meta[l];
      const bool sel = (m & Meta::kParsed) && (m & Meta::kSince) && gbit(a, l);
      if (sel) {
        const uint8_t* segp = a.bytes + a.segs[s].base;
        const uint64_t ls = a.line_off[l + s], le = a.line_off[l + s + 1];
        const uint32_t plen = line_plen(a, m, segp, ls, le);
        src[j] = a.segs[s].base + ls + plen;
        len[j] = (uint32_t)(le - ls - plen);
        blen += len[j];
        ++nsel;
      }
    }
    // block scans (bytes, selected lines)
    const uint64_t ib = wave_incl_scan_add(blen, lane);
    const uint64_t ic = wave_incl_scan_add((uint64_t)nsel, lane);
    if (lane == 63) { s_wb[wv] = ib; s_wc[wv] = ic; }
    __syncthreads();
    uint64_t pb = 0, pc = 0, tb = 0, tc = 0;
    for (int k = 0; k < 4; ++k) {
      if (k < wv) { pb += s_wb[k]; pc += s_wc[k]; }
      tb += s_wb[k]; tc += s_wc[k];
    }
    if (wv == 0) {
      const uint64_t xb = lookback_wave(stb, blk, tb, 0ull, SumComb(), a.counters + 2, lane);
      const uint64_t xc = lookback_wave(stc, blk, tc, 0ull, SumComb(), a.counters + 2, lane);
      if (lane == 0) { s_exb = xb; s_exc = xc; }
    }
    __syncthreads();
    uint64_t ob = s_exb + pb + ib - blen;  // my exclusive byte offset
    uint64_t oc = s_exc + pc + ic - nsel;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = t * 4 + j;
      if (is_first[j]) { a.segout[seg_of[j]].out_lo = ob; a.segout[seg_of[j]].sel_lo = oc; }
      s_src[i] = src[j];
      s_dst[i] = ob;
      s_len[i] = len[j];
      ob += len[j];
      oc += len[j] ? 1 : 0;
      if (is_last[j]) { a.segout[seg_of[j]].out_hi = ob; a.segout[seg_of[j]].sel_hi = oc; }
    }
    __syncthreads();
    // gather copy: each wave takes lines round-robin, 64 lanes per line
    for (int i = wv; i < kCompactLines; i += 4) {
      const uint32_t n = s_len[i];
      if (!n) continue;
      const uint8_t* sp = a.bytes + s_src[i];
      uint8_t* dp = a.out + s_dst[i];
      for (uint32_t k = lane; k < n; k += 64) dp[k] = sp[k];
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_pipeline(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus) {
  hipError_t e;
#define KLF_TRY(x) do { e = (x); if (e != hipSuccess) return e; } while (0)
  KLF_TRY(hipEventRecord(ev[0], st));
  KLF_TRY(hipMemsetAsync(a.counters, 0, kNumCounters * sizeof(uint32_t), st));
  KLF_TRY(hipMemsetAsync(a.status, 0, (size_t)a.ntiles * 8, st));
  KLF_TRY(hipMemsetAsync(a.segout, 0, (size_t)a.nsegs * sizeof(SegOut), st));
  KLF_TRY(hipMemsetAsync(a.cstatus, 0, (size_t)a.max_cblocks * 2 * 8, st));
  if (a.grep_mode != kGrepNone) KLF_TRY(hipMemsetAsync(a.bits, 0, (size_t)(a.cap_lines / 32 + 1) * 4, st));
  if (a.build_tiles) {
    const uint32_t g = (a.ntiles + 255) / 256;
    hipLaunchKernelGGL(k_tiles, dim3(g < 4096 ? g : 4096), dim3(256), 0, st, a.segs, a.nsegs, a.ntiles,
                       a.tile_seg);
    KLF_TRY(hipGetLastError());
  }
  KLF_TRY(hipEventRecord(ev[1], st));
  {
    int occ = 0;
    if (a.grep_mode == kGrepLit1)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan<true>, kThreads, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan<false>, kThreads, 0);
    occ = occ < 1 ? 1 : (occ > 8 ? 8 : occ);
    uint32_t grid = (uint32_t)(num_cus * occ);
    grid = grid / kScanGroups * kScanGroups;
    if (grid < kScanGroups) grid = kScanGroups;
    if (a.grep_mode == kGrepLit1)
      hipLaunchKernelGGL(k_scan<true>, dim3(grid), dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL(k_scan<false>, dim3(grid), dim3(kThreads), 0, st, a);
  }
  KLF_TRY(hipGetLastError());
  KLF_TRY(hipEventRecord(ev[2], st));
  if (a.grep_mode == kGrepGeneral || a.grep_mode == kGrepAll) {
    hipLaunchKernelGGL(k_match, dim3(num_cus * 8), dim3(256), 0, st, a);
    KLF_TRY(hipGetLastError());
  }
  KLF_TRY(hipEventRecord(ev[3], st));
  const uint32_t nblk_tiles = (a.ntiles + 255) / 256;
  const uint64_t nwords = a.cap_lines / 32 + 1;
  const uint32_t nblk_words = a.grep_mode == kGrepNone ? 0 : (uint32_t)((nwords + 255) / 256);
  hipLaunchKernelGGL(k_count, dim3(nblk_tiles + nblk_words), dim3(256), 0, st, a, nblk_tiles, nwords);
  KLF_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_tail, dim3(a.nsegs), dim3(256), 0, st, a);
  KLF_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_wprefix, dim3(1), dim3(256), 0, st, a);
  KLF_TRY(hipGetLastError());
  KLF_TRY(hipEventRecord(ev[4], st));
  hipLaunchKernelGGL(k_compact, dim3(num_cus * 4), dim3(kThreads), 0, st, a);
  KLF_TRY(hipGetLastError());
  KLF_TRY(hipEventRecord(ev[5], st));
#undef KLF_TRY
  return hipSuccess;
}

}  // namespace klf
