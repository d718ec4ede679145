// klf_kernels.hpp — device-side data structures and host launchers of the filter path.
// Kernels live in klf_kernels.hip; the engine (klf_engine.cpp) only sees this header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace klf {

// Work decomposition of the scan: a tile = one wave x 128 contiguous bytes per lane; a
// 256-thread workgroup runs 4 independent waves.
constexpr int kThreads = 256;
constexpr int kLaneBytes = 128;
constexpr int kTile = 64 * kLaneBytes;        // 8 KiB wave-tile
constexpr int kHalo = 64;                     // LDS bytes staged past the tile (timestamp window)
constexpr int kMaxFusedLiteral = 256;
constexpr uint64_t kSegAlign = 256;                 // segment base alignment in the batch buffer
constexpr uint64_t kAllocSlack = kTile + kHalo + 1024;
constexpr uint32_t kPlenEscape = 16383;             // meta plen field saturates here
constexpr int kCompactLines = 1024;                 // lines per compaction block
constexpr uint32_t kNumCounters = 64;               // zeroed by k_init each run
constexpr uint32_t kCtrPool = 4;                    // counters[4]: dense-tile pool allocator
constexpr uint32_t kMatchChunk = 8192;              // lines per k_mcount partial (256 words)

constexpr int kSlots = kTile / 32 + 2;  // staged line slots per tile (>= 8 KiB / 32-byte kubelet line + 1)
constexpr uint32_t kScanSmallTiles = 1u << 20;  // tile-scan blocks of 1,024 tiles up to this many tiles (8 GiB), 4,096 above
constexpr int kSlotStride = (kSlots + 3) & ~3;  // u32 slots of a tile's LDS line list
// Per-tile record region in HBM: the scan's TileStat (4 words) then the line slots, 128-B
// aligned and written as whole 128-B lines (a 16-B record store or a slot run ending
// inside a line is a partial-line write, read-modify-written by HBM3E: measured at ~0.3 ms
// per 4 M tiles).  k_tsum copies the TileStats into the compact `tstat` array.
constexpr int kRecHead = 4;
constexpr uint32_t kScanGroup = 8;  // consecutive tiles per wave turn: 8 TileStats = one 128-B line of tstat
constexpr int kRecStride = (kRecHead + kSlots + 31) & ~31;  // u32 words (1,152 B)

// q-gram prefilter of general pattern sets (klf_patterns.hpp CompiledSet::qf_*)
constexpr int kQfBucketBits = 12;                    // bitmap words = verification buckets
constexpr uint32_t kQfWords = 1u << kQfBucketBits;   // bitmap: 4096 words = 16 KiB of LDS
constexpr uint32_t kQfMinNeedle = 3;                 // shorter literal / factor: no prefilter
constexpr uint32_t kQfMaxFactor = 32;                // regex factors are cut to this length
constexpr uint32_t kMaxRegexSet = 1024;              // = klf_patterns.hpp kMaxRegexes
constexpr uint32_t kCtrQueue = 6;                   // counters[6]: NFA candidate queue length
constexpr uint32_t kCtrQOver = 7;                    // counters[7]: queue overflow -> k_match
constexpr uint32_t kHitSlots = 32;                   // prefilter hits a tile records itself
constexpr uint32_t kCtrHits = 8;                     // counters[8]: spilled prefilter hits
constexpr uint32_t kCtrRedo = 20;                    // counters[20]: a windowed-index run needs the whole index (rerun)
constexpr uint32_t kCtrHitsOver = 9;                 // counters[9]: hit list overflow -> k_match
constexpr uint32_t kCtrFlatHits = 12;                // counters[12]: hit slots flattened by k_tbase
constexpr uint32_t kCtrCopyChunks = 11;              // counters[11]: output copy chunks (k_cgather)
#ifndef KLF_COPY_CHUNK_KB
#define KLF_COPY_CHUNK_KB 128  // measured on C3: 64 KiB 7.75 ms, 128 KiB 7.25, 256 KiB 8.39
#endif
constexpr uint64_t kCopyChunk = KLF_COPY_CHUNK_KB * 1024;  // output bytes per k_cgather work item (at most)
// k_cscan picks the copy chunk per run: the smallest power of two >= 4 KiB (one 16-B
// store per thread of a workgroup) that keeps the output within kCopyChunksTarget chunks,
// up to kCopyChunk: a small output (tail-limited runs: C2, C5) is then spread over the
// whole chip instead of a few workgroups walking 128 KiB each.
constexpr uint32_t kCopyChunkMinLog2 = 12;
#ifndef KLF_COPY_CHUNKS_TARGET
#define KLF_COPY_CHUNKS_TARGET 1024
#endif
constexpr uint32_t kCopyChunksTarget = KLF_COPY_CHUNKS_TARGET;  // one resident generation of k_cmove workgroups (4 per CU)
constexpr uint32_t kCtrChunkLog2 = 16;               // counters[16]: log2 of this run's copy chunk
constexpr uint32_t kCtrTailDone = 18;                // counters[18]: k_tailw blocks done
constexpr uint32_t kCtrPlanDone = 26;                // counters[26]: k_cplan blocks done (plan_mode 1)
constexpr uint32_t kCtrVerified = 10;                // counters[10]: hits k_verify walked (diagnostics)
constexpr uint32_t kCtrDense = 14;                   // counters[14]: dense compaction (k_tkeep / k_tcopy)
constexpr uint32_t kCtrFuseBad = 24;                 // counters[24]: the one-pass compaction was voided (rerun)
constexpr uint32_t kCtrOutShort = 22;                // counters[22]: the output did not fit out_cap
constexpr uint32_t kCtrPairsOver = 15;               // counters[15]: failed (line, pattern) pair inserts (set full)
constexpr uint32_t kQfRegex = 1u << 24;              // entry flags: regex factor (else literal)
constexpr uint32_t kQfLoose = 1u << 25;              //   compare OR 0x20 per byte
constexpr uint32_t kQfAnchored = 1u << 26;           //   a short needle reached through its anchor (no bitmap bits)
constexpr size_t kNfaMaxLds = 64 * 1024;            // k_nfa stages its tables in LDS up to this
constexpr uint32_t kCarryBias = 256;
constexpr uint32_t kRxPreNone = 0xFFFFFFFFu;         // rx_pre: no bound (= klf_patterns.hpp kRxPreUnbounded)                 // TileStat.carry_off = hit offset + 1 + bias
// Blocked Bloom filter, one 32-bit bitmap word per probe, K = 2 or 3 bits per gram.  The
// multiplies see f = bytes 0..2 of the gram (K = 3: folded, f ^ f >> 13, so that byte 2
// reaches the low product bits too):
//   h    = f * C1 (+ bytes 1..3 * C2 for 4-byte grams): 24-bit multiply(-add)s, low 32
//          bits; word = h >> 20, also the verification bucket;
//   m    = f * C4, p = the high half of f * C3 (v_mul_hi_u32_u24) (K = 3 only);
//   bits = K = 2: h bits 8..12 and 16..20 (byte selects of h: no second multiply; the C5
//          set's hits on C5 data 115 vs 96 per 32 MiB with m's bytes); K = 3: p bits 0..4,
//          h bits 16..20, m bits 24..28 (m bits 16..20 in place of p: 11x the C4 hits).
// The scan takes every bit position as a byte / word select of a product (SDWA operands of
// the shifts) or its low bits, so a probe costs about 10 VALU (K = 2) / 13 (K = 3); the
// previous design cost ~14 / ~18.  Measured on the C4 / C5 sets and data (host emulation,
// tools in tests/test_prefilter.py): 0.9 / 0.01 bitmap hits per 8 KiB tile (before: 2.2 /
// 0.017).
// Two-level layout (qf_k = kQfTwoLevel, large sets at stride 4): the samples first test an
// exact set of the probed grams' low two bytes (bitmap words [0, kQfPairWords): bit
// (g & 0xFFFF), over raw bytes: a folded set lists every case variant of its pairs, so the
// scan probes the data's bytes as they are); only the survivors (~5 % of log text for the 1,024-literal C4 set) take the
// 3-bit probe, into a Bloom filter of the remaining kQfPairWords words (11-bit buckets).
constexpr uint32_t kQfTwoLevel = 5;
constexpr uint32_t kQfPairWords = 2048;
// The pair set's word of pair p (bit p & 31): p >> 5.  Its bank bits are the first byte's
// top three bits and the second byte's low two: on ASCII text about a dozen of the 32 banks,
// ~2x the LDS-active cycles in bank conflicts (C4, pmc_c4).  KLF_PAIR_SWZ=1 folds p's low
// five bits into them (all 32 banks) for one more VALU per sample: C4 k_scan 7.60 -> 7.97 ms
// (same box, two rounds, gpurun_out/r5k) -- the pair stage is bound by its instructions, not
// by the conflicts.
#ifndef KLF_PAIR_SWZ
#define KLF_PAIR_SWZ 0
#endif
__host__ __device__ inline uint32_t qf_pair_word(uint32_t p) {
  return KLF_PAIR_SWZ ? (((p >> 5) ^ (p & 31u)) & (kQfPairWords - 1u)) : ((p >> 5) & (kQfPairWords - 1u));
}
__host__ __device__ inline bool qf_k3(uint32_t k) { return k == 3 || k == kQfTwoLevel; }
__host__ __device__ inline uint32_t qf_f(uint32_t g, uint32_t k) {
  const uint32_t g24 = g & 0xFFFFFFu;
  return qf_k3(k) ? g24 ^ (g24 >> 13) : g24;
}
__host__ __device__ inline uint32_t qf_hash(uint32_t g, uint32_t w24, uint32_t k) {  // w24 = 24 (q = 4) or 0 (q = 3)
  const uint32_t hi = w24 ? (g >> 8) & 0xFFFFFFu : 0u;
  return qf_f(g, k) * 0x9E3779u + hi * 0x7F4A7Du;
}
__host__ __device__ inline uint32_t qf_word(uint32_t h) { return h >> (32 - kQfBucketBits); }
// The bitmap word (= verification bucket) of gram g: h's top 12 bits, or for 3-byte grams
// with two bits (no bit position taken from h) bits 18..29, whose LDS byte offset
// (h >> 16) & 0x3FFC is one SDWA AND -- a VALU fewer per probe; the C5 set's bitmap hits
// on C5 data are unchanged (96 per 32 MiB either way).  (Bits 34..45 of a second product,
// v_mul_hi_u32_u24: 54x the hits -- a product's top bits follow the gram's top byte.)
__host__ __device__ inline uint32_t qf_bucket(uint32_t g, uint32_t w24, uint32_t k) {
  if (w24 == 0 && k == 2) return (qf_hash(g, w24, k) >> 18) & (kQfWords - 1u);
  if (k == kQfTwoLevel) return qf_hash(g, w24, k) >> 21;  // [0, kQfPairWords)
  return qf_word(qf_hash(g, w24, k));
}
// the Bloom bitmap word of gram g (two-level: behind the pair words)
__host__ __device__ inline uint32_t qf_bloom_word(uint32_t g, uint32_t w24, uint32_t k) {
  return (k == kQfTwoLevel ? kQfPairWords : 0u) + qf_bucket(g, w24, k);
}
__host__ __device__ inline uint32_t qf_bits(uint32_t g, uint32_t h, uint32_t k) {
  const uint32_t f = qf_f(g, k);
  const uint32_t m = f * 0x5BD1E9u;
  if (!qf_k3(k)) return (1u << ((h >> 8) & 31u)) | (1u << ((h >> 16) & 31u));
  const uint32_t p = (uint32_t)(((uint64_t)f * 0xC2B2AEu) >> 32);
  const uint32_t b3 = (1u << ((m >> 24) & 31u)) | (1u << (p & 31u)) | (1u << ((h >> 16) & 31u));
  return k == kQfTwoLevel ? b3 | (1u << ((m >> 8) & 31u)) : b3;  // two-level: a fourth bit (survivors only)
}
// The whole probe of a (folded, masked) gram against the bitmap (host emulation; the scan
// computes the same from its LDS copy)
__host__ __device__ inline bool qf_pass(const uint32_t* bm, uint32_t gq, uint32_t w24, uint32_t k) {
  if (k == kQfTwoLevel && !((bm[qf_pair_word(gq & 0xFFFFu)] >> (gq & 31u)) & 1u)) return false;
  const uint32_t h = qf_hash(gq, w24, k), bits = qf_bits(gq, h, k);
  return (bm[qf_bloom_word(gq, w24, k)] & bits) == bits;
}
// Data statistics of the window choice (k_gramhist over a sample of the first batch): a
// byte histogram, then the exact 2-gram counts (fold applied) at even offsets
constexpr uint32_t kGramHistPairs = 256;  // first word of the 2-gram counts
constexpr uint32_t kGramHistWords = kGramHistPairs + 65536;
constexpr uint64_t kGramHistSample = 64u << 10;  // bytes sampled per segment (<= 16 segments)
constexpr uint32_t kQfK2MaxGrams = 1536;
// The prefilter's sampled positions (tile / stream offsets; tiles and streams start
// 16-B aligned): p = 0 mod S, except S = 6, the grid p mod 16 in {0, 6, 12}: three samples
// per 16-B chunk whose gaps never exceed 6, so every run of 6 consecutive positions holds
// one (windows of q + 5 bytes, as a stride of 6 would need) at 3/4 the samples of stride 4.
__host__ __device__ inline bool qf_sampled(uint64_t p, uint32_t S) {
  if (S == 6) {
    const uint32_t r = (uint32_t)(p & 15u);
    return r == 0 || r == 6 || r == 12;
  }
  return p % S == 0;
}
__host__ __device__ inline double qf_samples_per_tile(uint32_t S) { return S == 6 ? 8192.0 * 3 / 16 : 8192.0 / S; }  // up to this many sampled grams K = 2 bits, else 3

// Dense compaction: per-tile copy record written by k_tkeep, read by k_ksum / k_kbase /
// k_tcopy (16 B), and up to kRunSlots kept runs per tile (u32: tile offset of the run's
// first byte | its offset in the tile's output << 16); a tile with more runs has
// nruns = kRunsRecompute and k_tcopy lists them again from the line index.
constexpr int kRunSlots = 128;
constexpr uint16_t kRunsRecompute = 0xFFFF;
struct TRec {
  uint64_t src;    // batch offset of the tile's first byte
  uint32_t kept;   // content bytes of selected lines inside the tile
  uint16_t nruns;  // kept runs (or kRunsRecompute)
  uint16_t nsel;   // selected lines starting in the tile
};
static_assert(sizeof(TRec) == 16, "TRec is one 16-B record");

// Per-tile record of the scan (K1a), 16 B.
struct TileStat {
  uint32_t events;     // line-end events in the tile
  uint32_t pool_base;  // dense tiles: first pool slot; a tile where one line starts (bit4): that slot
  uint16_t parsed, since_ok;
  uint16_t flags;      // bit0 dense (slots in the pool), bit1 literal hit in the carried-in line,
                       // bit2 some line deferred to k_fixup, bit3 literal hit in a line starting here,
                       // bit4 the tile's single slot is pool_base (no record region written),
                       // bit5 (general sets) its 1-2 prefilter hits are pool_base's u16 halves
  uint16_t carry_off;  // literal: 1 + kCarryBias + tile offset of the furthest hit in the
                       // carried-in line (0 = none); general sets: hit slots used
};
static_assert(sizeof(TileStat) == 16, "TileStat is one 16-B store");

// One segment (= one non-empty stream) of the device batch.
struct SegDesc {
  uint64_t base;    // byte offset of the stream in the batch buffer (256-aligned)
  uint64_t len;     // stream length (> 0)
  uint32_t tile0;   // first global tile of the stream
  uint32_t ntiles;  // ceil(len / kTile)
};

// Per-segment results, written by the kernels, read back by the host in one copy.
struct SegOut {
  uint64_t line_lo, line_hi;   // global line indices [lo, hi) of the stream
  uint64_t parsed, since_ok, matched;
  uint64_t win_lo, win_hi;     // candidate window after the tail rule
  uint64_t sel_lo, sel_hi;     // selected-line chain values at the window ends
  uint64_t out_lo, out_hi;     // output byte offsets [lo, hi) in the output buffer
  uint64_t frag;               // 1 when the stream ends without '\n'
  uint64_t p_lo, p_hi;         // parsed-line prefix at the stream's first / past its last tile
  uint64_t q_lo, q_hi;         // since_ok-line prefix, same
};

// Line-meta word (u16): bit0 parsed, bit1 since_ok, bits 2..15 content offset (plen),
// saturating at kPlenEscape (then recomputed from the bytes).
struct Meta {
  static constexpr uint16_t kParsed = 1, kSince = 2;
};

enum GrepMode : uint32_t { kGrepNone = 0, kGrepNever = 1, kGrepAll = 2, kGrepLit1 = 3, kGrepGeneral = 4 };

struct DevPatterns {  // device copies of CompiledSet tables (kGrepGeneral)
  const uint8_t* ac_class = nullptr;
  const uint32_t* ac_next = nullptr;
  const uint8_t* ac_accept = nullptr;
  const int32_t* ac_out = nullptr;    // [states] literal id ending here, -1 none
  const uint32_t* ac_dict = nullptr;  // [states] dictionary link (0 none)
  uint32_t ac_states = 0, ac_classes = 0;
  uint32_t n_cids = 0, n_lits = 0;    // compiled pattern ids: literals, then regexes
  const uint8_t* rx_class = nullptr;
  const uint64_t* rx_b = nullptr;
  const uint64_t* rx_follow = nullptr;
  const uint64_t* rx_first = nullptr;
  const uint64_t* rx_last = nullptr;
  const uint64_t* rx_init0 = nullptr;
  const uint64_t* rx_end = nullptr;
  const uint64_t* rx_vec = nullptr;   // [rx_count][4]: first, last, init0, end
  const uint32_t* rx_flags = nullptr;
  const uint32_t* rx_pre = nullptr;   // [rx_count] match start -> first factor occurrence bound
  uint32_t rx_count = 0, rx_classes = 0, rx_maxpos = 64;
  uint32_t rx_unbounded = 0;          // regexes without a bound (k_nfa runs their whole lines)
  // q-gram prefilter (qf_on): bitmap, buckets, needles
  uint32_t qf_on = 0, qf_stride = 1, qf_fold = 0, qf_mask = ~0u;
  uint32_t qf_w24 = 24, qf_k = 3;     // probe: 4-byte grams (24) or 3-byte (0); bits per gram
  const uint32_t* qf_bitmap = nullptr;
  const uint32_t* qf_head = nullptr;
  const uint4* qf_ent = nullptr;
  const uint32_t* qf_nbytes = nullptr;
  // short needles anchored on a rare byte (klf_patterns.hpp CompiledSet::qf_anc_*)
  uint32_t qf_anc_on = 0, qf_anc_byte = 0, qf_anc_fold = 0, qf_anc_n = 0;  // anc_byte replicated x4
  const uint32_t* qf_anc_pre = nullptr;  // [qf_anc_n] {want, mask}
};

struct RunArgs {
  // batch
  const uint8_t* bytes;
  const SegDesc* segs;
  uint32_t nsegs;
  uint32_t ntiles;
  uint32_t* tile_seg;   // [ntiles] tile -> segment (filled by k_tiles when build_tiles)
  uint32_t build_tiles;
  uint32_t tindex_wide;  // k_tindex with 4,096 tiles per block (batches above kScanSmallTiles; tests force it)
  // filter
  int64_t since_sec;
  int32_t since_nsec;
  // the cutoff as the canonical prefix's 23 digits (YYYYMMDDhhmmss + 9 fraction digits),
  // packed like parse_fast's p0..p5 (big-endian digit order, a '0' pad before the last
  // digit); before 1970: 1970-01-01T00:00:00Z, from 2100 on: all '9'
  uint32_t since_dig[6];
  int64_t tail;
  uint32_t grep_mode;
  uint32_t match_all;  // kGrepGeneral: the set also matches every content (k_match marks every parsed line)
  const uint8_t* lit;  // kGrepLit1 literal (device)
  uint32_t lit_len;
  uint32_t lit_anchor; // index of the literal's rarest byte (scan anchor)
  uint32_t lit_anchor_byte;  // that byte
  const uint32_t* lit_words;  // the literal as little-endian dwords (zero padded)
  DevPatterns pats;
  // workspace (device)
  TileStat* tstat;      // [ntiles]
  uint32_t* slots;      // [ntiles * kRecStride] per-tile records: TileStat, then staged line slots
  uint32_t* pool;       // [pool_cap] slots of dense tiles, and (wave_pool) of every tile where two or
                        // more lines start, appended to per-wave chunks of pool_chunk slots
  uint64_t pool_cap;
  uint32_t wave_pool;   // 1: slots in the pool (a.slots unused, null); 0: per-tile record regions
  uint32_t pool_chunk;  // slots a wave reserves at a time (counters[kCtrPool] is the allocator)
  uint64_t* tile_base;  // [ntiles] global line index of each tile's line 0
  uint64_t* bsum;       // [4 * (ntiles / 1024 + 1)] scan block sums (events, parsed, since_ok, hits)
  uint64_t* mpart;      // [cap_lines / kMatchChunk + 1] matched-line partial per line chunk
  uint64_t* csum;       // [3 * (max compaction blocks + 1)] per-block (bytes, lines), then their
                        // prefixes and the prefix of copy chunks
  uint32_t* cmap;       // [cmap_cap] compaction block of every copy chunk (k_cscan -> k_cgather)
  uint64_t cmap_cap;
  uint32_t* cseg;       // [max compaction blocks] stream of each block's first window line
  uint32_t* counters;   // [kNumCounters]: 1 compact ticket, 2 error flags, 3 compact blocks,
                        // 4 dense-tile pool
  uint64_t* line_off;   // [cap_lines + nsegs]
  uint16_t* meta;       // [cap_lines]
  uint32_t* bits;       // [cap_lines / 32 + 1]
  uint64_t cap_lines;
  SegOut* segout;       // [nsegs]
  uint64_t* wpre;       // [nsegs + 1] exclusive prefix of window sizes
  uint64_t* wgrp;       // win_index: [nsegs] the scatter groups [ga, gb) holding each stream's
                        // tail window (ga | gb << 32), then [nsegs + 1] their exclusive prefix
  uint8_t* out;         // output bytes
  uint64_t out_cap;     // bytes of `out`: a copy that would pass it is skipped and flagged
                        // (counters[kCtrOutShort]); the host grows the buffer and reruns the tail stage
  uint32_t max_cblocks; // compaction block capacity
  uint32_t stage_times; // record the inner stage events (ev[2..4])
  uint64_t* cand;       // [2 * cand_cap] NFA candidates: {global line index | regex << 40,
                        //  stream offset of the factor occurrence | stream << 40}
  uint32_t cand_cap;
  uint16_t* hslots;     // [ntiles * kHitSlots] prefilter hits (tile offsets of the samples)
  uint64_t* hflat;      // [hflat_cap] prefilter hits {tile | tile offset << 32 | stream << 48 (0xFFFF: look it up)}, by k_tindex
  uint64_t hflat_cap;
  uint64_t* qhits;      // [qhits_cap] spilled hits (batch byte offsets of the samples)
  uint32_t qhits_cap;
  // dense compaction (most lines selected): per tile kept bytes / selected lines, their
  // exclusive prefixes (out offset, selected-line offset per tile)
  struct TRec* trec;    // [ntiles] per-tile copy record (k_tkeep)
  uint32_t* truns;      // [ntiles * kRunSlots] the tiles' kept runs (k_tkeep -> k_tcopy)
  uint64_t* kbase;      // [2 * ntiles]
  uint32_t compact_mode;  // 0 auto, 1 line gather (sparse), 2 tile copy (dense)
  // grep none with --tail -1: k_scatter goes after k_tailw and builds the global line index
  // only for the line gather; the dense path lists its lines from the scan's slots
  uint32_t lazy_index;
  // the scan plans the dense compaction (kept runs per tile + tile aggregates; needs truns):
  // k_tkeep's listing pass is skipped unless a line was deferred
  uint32_t plan_runs;
  // literal patterns and prefiltered regex sets (round 6): the global line index is built
  // after k_tailw for the lines of the tail windows only (k_scatter mode 2); tiles with
  // deferred lines or single-literal hits before k_mcount (mode 1: their match bits come
  // from the slots); k_verify writes the NFA candidate lines' bounds and meta
  uint32_t win_index;
  uint32_t scatter_mode;  // k_scatter: 0 every tile, 1 tiles with deferred lines, 2 tiles meeting a window
  uint32_t scatter_split; // k_scatter: waves per 64-tile group (small batches: a group's lines split over them; 0 = 1)
  uint32_t skip_match;    // prefiltered set: k_match not launched (an overflow redoes the run with it)
  uint32_t skip_tcopy;    // --tail run: k_tcopy not launched (the host launches it when the run went dense)
  // line gather's block sums / prefix (a --tail run, always the sparse path): 0 k_cplan,
  // k_cmid, k_cmove; 1 k_cplan's last block runs the prefix (no k_cmid); 2 k_tailw's last
  // block runs both (no k_cplan, no k_cmid: the line index exists before k_tailw)
  uint32_t plan_mode;
  // per-pattern counts (KLF_FILTER_PATTERN_COUNTS): pcount[segment * n_cids + cid] lines,
  // each (line, cid) counted once through the `pairs` hash set (open addressing, u64 keys)
  uint32_t count_pats;
  uint32_t* pcount;
  uint64_t* pairs;
  uint32_t pairs_log2;
  // one-pass compaction (no patterns, --tail -1; k_scan<plain, FUSE> + k_fcarry): each wave
  // compacts its own range of fuse_range consecutive tiles in place; fuse_ext0[range] = the
  // range's first extent, fuse_ext[2 e .. 2 e + 1] = {output start, length} of extent e (one
  // per stream the range touches), fuse_rinfo[4 range ..] = {bytes before the range's first
  // line start, known | sel << 1 at its end, the open line's content start - the range end,
  // bytes of its last stream part}
  uint32_t fuse;
  uint32_t fuse_range;
  uint32_t fuse_nranges;
  const uint32_t* fuse_ext0;
  uint64_t* fuse_ext;
  uint64_t* fuse_rinfo;
};

// Enqueues the whole pipeline on `stream`; `ev` (6 events) brackets the stages for
// per-kernel timing: ev[0] start, ev[1] after the workspace memsets, ev[2] after the
// scan, ev[3] after the general matcher, ev[4] after counts+tail+window prefix, ev[5]
// after compaction.  Returns a hipError_t.
// ev may be null: no event records.
// phase: 0 the whole pipeline; 1 up to the tile index (k_init .. k_tindex: the line arrays
// are not touched, a.bits may be null); 2 the rest (k_scatter on), after the host sized
// the line arrays from phase 1's line count (an engine's first run).
// ev_mask (nullable): bit k is set for every ev[k] recorded on the stream (ev[7] / ev[8]: the
// scan's dispatch timestamps), so that the host queries only the pairs the run recorded.
// k_scatter alone: the global line index of a run (an engine's lazy index, on demand).
hipError_t launch_scatter(const RunArgs& a, hipStream_t stream, int num_cus);
hipError_t launch_pipeline(const RunArgs& a, hipStream_t stream, hipEvent_t* ev, int num_cus, int phase = 0,
                           uint32_t* ev_mask = nullptr);
// Re-runs matched counts, tail and compaction of the last pipeline with a.tail changed.
hipError_t launch_retail(const RunArgs& a, hipStream_t stream, hipEvent_t* ev, int num_cus,
                         uint32_t* ev_mask = nullptr);
// Data statistics (kGramHistWords u32, zeroed here) of the first `sample` bytes of each of
// up to 16 segments: byte counts, and the 2-grams at even offsets (folded like the
// prefilter's grams).
// Diagnostic: reps back-to-back launches of a VALU loop (num_cus x 4 workgroups); out
// (2 num_cus x 4 + 1 u64) gets the last launch's per-workgroup shader / real-time deltas.
hipError_t clock_probe(int num_cus, uint32_t iters, uint32_t reps, uint64_t* out, hipStream_t stream);
hipError_t launch_tcopy(const RunArgs& a, hipStream_t st, hipEvent_t* ev, int num_cus, uint32_t* ev_mask);
hipError_t launch_nlsample(const uint8_t* bytes, const SegDesc* segs, uint32_t nsegs, uint32_t ntiles, uint32_t blocks,
                           uint32_t* out, hipStream_t st);
hipError_t launch_gramhist(const uint8_t* bytes, const SegDesc* segs, uint32_t nsegs, uint64_t sample, uint32_t fold,
                           uint32_t* hist, hipStream_t stream);
// Staged capture (klf_run): device chunks of the early H2D -> their places in the batch.
struct AsmPiece {
  const uint8_t* src;  // device chunk (16-B aligned)
  uint64_t dst;        // batch byte offset (16-B aligned)
  uint64_t len;        // bytes (a multiple of 16)
};
hipError_t launch_assemble(const AsmPiece* pieces, uint32_t n, uint8_t* batch, hipStream_t stream);
// Global index of the last line in [lo, hi) whose meta has no parsed bit, +1 (0 = none),
// atomically max-ed into *res (zeroed here).  Needs the latest run's meta (a.meta).
hipError_t launch_lastbad(const RunArgs& a, uint64_t lo, uint64_t hi, uint64_t* res, hipStream_t stream);
// waves of a full-occupancy launch of the one-pass compaction scan (RunArgs::fuse): the host
// cuts the batch into that many tile ranges
int fuse_waves(int num_cus);
// Diagnostic builds (-DKLF_TIMELINE=1): per-tile scan timeline; hipErrorNotSupported otherwise.
hipError_t dump_timeline(void* host, size_t bytes);
hipError_t clear_timeline();

}  // namespace klf
