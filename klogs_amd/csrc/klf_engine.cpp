// klf_engine.cpp — the C ABI of include/klf.h: staging, device workspace, the run,
// result views.  One engine = one GPU = one HIP stream (one process per GPU; the
// multi-GPU split happens above, in the host, by stream sharding — DESIGN.md §5).
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/klf.h"
#include "../../include/klf_debug.h"
#include "klf_copypool.hpp"
#include "klf_kernels.hpp"
#include "klf_patterns.hpp"
#include "klf_ts.hpp"

using klf::SegDesc;
using klf::SegOut;

namespace {

// time spent growing device buffers (KLF_DIAG: the first run's allocation share)
static std::atomic<uint64_t> g_alloc_ns{0};
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool borrowed = false;  // p lies in an engine's workspace block (not freed here)
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    if (p && !borrowed) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    borrowed = false;
    size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    g_alloc_ns += ns;
    static const bool diag = getenv("KLF_DIAG_ALLOC") != nullptr;
    if (diag) fprintf(stderr, "[klf] alloc %zu B: %.1f us\n", want, ns / 1e3);
    return e;
  }
  void release() {
    if (p && !borrowed) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    borrowed = false;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// An engine's first run maps its workspace buffers as one allocation (each hipMalloc costs
// tens of us of host time, ~20 of them add up in a one-shot run): buffers not yet mapped
// get 256-B aligned pieces of one block; later growth maps a buffer of its own.
// Maps the missing buffers of `req` into one block (an engine's first run: one allocation);
// a buffer that later outgrows its slice gets its own allocation, and the block is freed
// once no buffer borrows from it any more (`users`: the buffers mapped into it).
static hipError_t ensure_all(DevBuf& block, std::vector<DevBuf*>& users,
                             const std::vector<std::pair<DevBuf*, size_t>>& req) {
  size_t total = 0;
  for (auto& r : req)
    if (!r.first->p) total += (std::max<size_t>(r.second, 256) + 255) & ~(size_t)255;
  if (total && !block.p) {
    hipError_t h = block.ensure(total);
    if (h != hipSuccess) return h;
    size_t off = 0;
    for (auto& r : req) {
      if (r.first->p) continue;
      const size_t n = (std::max<size_t>(r.second, 256) + 255) & ~(size_t)255;
      r.first->p = static_cast<uint8_t*>(block.p) + off;
      r.first->cap = n;
      r.first->borrowed = true;
      users.push_back(r.first);
      off += n;
    }
  }
  for (auto& r : req)
    if (hipError_t h = r.first->ensure(r.second); h != hipSuccess) return h;
  if (block.p) {
    const uint8_t* lo = static_cast<const uint8_t*>(block.p);
    users.erase(std::remove_if(users.begin(), users.end(),
                               [&](DevBuf* b) {
                                 const uint8_t* q = static_cast<const uint8_t*>(b->p);
                                 return !(b->borrowed && q >= lo && q < lo + block.cap);
                               }),
                users.end());
    if (users.empty()) block.release();  // (every buffer outgrew its slice)
  }
  return hipSuccess;
}

// Pinned host buffer (hipHostMalloc): per-run readbacks land here with one async DMA each
// and a single stream sync (a pageable destination costs a staged copy and a wait per call).
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    const size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    else p = nullptr;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct klf_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  int num_cus = 256;
  klf::CompiledSet cs;
  std::string err;
  uint64_t gen = 0;
  // Staging (host path).  Each stream fills a pinned host chunk
  // (hipHostMalloc, pooled across runs); a chunk that fills is DMA'd at once on the copy
  // stream into a pooled 64 MiB device chunk, so the H2D overlaps the rest of the capture.
  // klf_run DMAs the partly filled last chunk of every stream straight into the batch and
  // one kernel (k_assemble) moves the device chunks into their places in the batch.
  // Per-stream records are heap objects that never move (klf_stage on different ids runs
  // concurrently while the table grows).
  std::mutex mu;
  struct StageChunk {
    uint8_t* p = nullptr;
    size_t used = 0;
    bool pinned = false;
  };
  struct StagedStream {
    std::vector<uint8_t*> dchunks;  // full chunks already DMA'd (device, kStageChunk each)
    StageChunk cur;                 // pinned chunk being filled (p = null: none)
    uint64_t len = 0;
  };
  std::vector<std::unique_ptr<StagedStream>> staged;
  std::vector<StageChunk> chunk_pool;  // free pinned chunks (used = 0)
  std::vector<uint8_t*> dchunk_pool;   // free device chunks
  struct Inflight {
    StageChunk c;
    hipEvent_t ev;
  };
  std::deque<Inflight> inflight;       // pinned chunks whose H2D may still be running
  std::vector<hipEvent_t> ev_pool;
  hipStream_t copy_stream = nullptr;   // early H2D of full chunks
  hipEvent_t copy_done = nullptr;
  bool ran = false;                    // klf_run since the last klf_reset (stage -> ESTATE)
  std::unique_ptr<klf::CopyPool> copier;  // started by the first klf_stage (device-resident runs never stage)
  std::once_flag copier_once;
  std::once_flag copy_stream_once;     // the copy stream: created by the first klf_stage / klf_run
  hipError_t copy_stream_err = hipSuccess;
  DevBuf d_asm;                        // k_assemble piece table
  DevBuf d_scratch;                    // small query results (klf_result_last_unparsed)
  DevBuf d_ac_out, d_ac_dict, d_pcount, d_pairs;  // per-pattern counts
  uint32_t pairs_log2 = 20;            // (line, pattern) pair set: 2^20 entries, grows on overflow
  uint32_t n_user = 0;                 // patterns as given to klf_open
  // a set with an always-pattern beside others (CompiledSet::also_all_pending): the patterns,
  // compiled in full on the first run that asks for per-pattern counts
  std::vector<std::vector<uint8_t>> pend_pats;
  std::vector<uint32_t> pend_kinds;
  bool tune_later = true;
  int counts_code = KLF_OK;            // that compile failed: counts unavailable (the filter is kAll's)
  std::string counts_err;
  // device pattern tables
  DevBuf d_lit, d_ac_class, d_ac_next, d_ac_accept, d_rx_class, d_rx_b, d_rx_follow, d_rx_vec, d_rx_flags, d_rx_pre;
  DevBuf d_qf_bitmap, d_qf_head, d_qf_ent, d_qf_nbytes, d_cand, d_rx_vec4, d_qhits, d_hslots, d_hist, d_hflat, d_qf_anc;
  HostBuf h_hist;  // gram / byte statistics of the first batch (pinned readback)
  uint32_t cand_cap = 1u << 22;  // NFA candidate queue (32 MiB); overflow -> k_match
  uint64_t hits_cap_max = 1u << 26;  // prefilter hit list (512 MiB at most); overflow -> k_match
  klf::DevPatterns dpats;
  // workspace
  std::vector<SegDesc> last_segs;  // tile_seg cache key
  DevBuf d_tile_seg;
  DevBuf d_cmap, d_cseg;
  DevBuf d_block;  // the first run's workspace buffers (ensure_all), freed last
  std::vector<DevBuf*> block_users;  // the buffers still mapped into d_block
  DevBuf d_block2;  // the first run's line arrays, slot pool / records and output (sized after its sample)
  std::vector<DevBuf*> block2_users;
  DevBuf d_batch, d_segs, d_tstat, d_slots, d_pool, d_tile_base, d_bsum, d_cstatus, d_counters, d_line_off,
      d_meta, d_bits, d_wpre, d_out, d_mpart, d_trec, d_truns, d_kbase;
  // one-pass compaction (RunArgs::fuse): range table, extents, range states; d_out2 the
  // contiguous device copy klf_result_device_out makes of a fused result on demand
  DevBuf d_fext0, d_fext, d_frinfo, d_out2;
  uint32_t fuse_range = 0, fuse_nranges = 0, fuse_next = 0;  // the layout d_fext0 was made for
  std::vector<uint32_t> fuse_ext0;
  // the segment table the extent table was built for: its own cache key (last_segs follows
  // every run, fused or not, and a failed run may leave it behind d_fext0)
  std::vector<SegDesc> fuse_segs;
  uint64_t pool_cap = 1 << 20;
  // lines per input byte of the last run (0: no run yet): sizes the line arrays of the next
  // runs (the first run sizes them from its own tile index, between two launch phases)
  double line_density = 0.0;
  bool dense_tail_seen = false;  // a --tail run took the dense compaction (keep its run table)
  HostBuf h_rb;  // run readback: the counters (kCtrBytes), the SegOut table, a one-pass run's extents
  HostBuf h_stage;  // pinned staging of the prefilter tables (upload_prefilter)
  HostBuf h_acblk;  // the automaton thread's tables (pinned), uploaded on the launch stream at the join
  size_t ac_total = 0, ac_off[5] = {0, 0, 0, 0, 0}, ac_cap[5] = {0, 0, 0, 0, 0};
  // The literals' Aho-Corasick automaton (deferred lines, the fallback matcher): klf_open
  // starts a host thread that builds it and uploads it as one block (d_acblk, one
  // synchronous copy); ensure_ac joins it before the first launch that may read it, so the
  // build overlaps the first run's sampling and needle placement
  std::thread ac_thread;
  bool ac_pending = false;  // the automaton is built (or being built) but not yet uploaded
  std::vector<std::vector<uint8_t>> ac_lits;
  klf::AcTables ac_tabs;
  hipError_t ac_err = hipSuccess;
  DevBuf d_acblk;
  hipEvent_t stage_ev = nullptr;  // the staged copies have drained
  bool stage_ev_pending = false;
  // KLF_GRAPH=1: small batches replay their launch sequence as a HIP graph (round 6): ~12
  // launches cost ~35-45 us of host time.  Opt-in: measured on C1 (64 MiB) the run went
  // 104 -> ~95 us, the device being the bound, while the first capture costs 5-7 ms (most
  // of it creating cap_stream), which a short-lived engine pays in full.  A sequence is
  // captured (on cap_stream: the engine's own stream may be the null stream) the second
  // time the same arguments run; graph_off after a capture that failed.
  hipStream_t cap_stream = nullptr;
  hipGraphExec_t gexec = nullptr;
  std::vector<uint8_t> gkey, gprev;  // the captured arguments; the previous eager run's
  bool graph_off = false;
  hipEvent_t ev[11] = {};  // [7], [8]: k_scan's dispatch (hipExtLaunchKernel start / stop); [9], [10]: k_tcopy's; [6] unused
  klf::RunArgs last_args{};  // arguments of the latest completed run (klf_retail)
  // the latest run's global line index is still to be built (lazy index, dense path): the
  // k_scatter launch that builds it
  std::vector<klf::RunArgs> index_pending;
  uint64_t last_gen = 0;     // gen of that run's result
};

struct klf_result {
  klf_engine* e = nullptr;
  uint64_t gen = 0;
  uint32_t n_streams = 0;
  std::vector<int64_t> seg_of;       // stream id -> segment (-1 = empty stream)
  std::vector<SegOut> so;            // per segment
  std::vector<uint64_t> seg_base;    // per segment (device byte offset)
  bool has_bits = false;
  uint64_t total_lines = 0, total_out = 0;
  double ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t ev_mask = 0;              // the timing events the run recorded
  int index_mode = KLF_INDEX_FULL;   // how much of the line index the run itself wrote
  // lazily filled host copies
  bool have_out = false, have_lines = false, have_bits = false;
  std::vector<uint8_t> out;
  std::vector<uint64_t> line_off;
  std::vector<uint32_t> bits;
  std::vector<std::vector<uint8_t>> stream_bits;
  std::vector<uint8_t> have_stream_bits;
  // per-pattern counts (KLF_FILTER_PATTERN_COUNTS): [segment][compiled id]
  bool counted = false, pcount_ok = false;
  std::vector<uint32_t> pcount;
  // a one-pass compaction run: each segment's output is the extents fx[2 k], fx[2 k + 1]
  // (d_out offset, length) for k in [fx_first[s], fx_first[s + 1]); so[s].out_lo / out_hi
  // are then the segment's place in the concatenated (host) output
  bool fused = false, have_dev = false;
  int compaction = KLF_COMPACT_GATHER;
  std::vector<uint64_t> fx;
  std::vector<uint32_t> fx_first;
};

// The run's counters and its per-stream records share one allocation (d_counters: the
// counters, then the records from byte kCtrBytes on), so that one D2H copy reads both back.
constexpr size_t kCtrBytes = klf::kNumCounters * 4;
static SegOut* segout_of(klf_engine* e) {
  return reinterpret_cast<SegOut*>(e->d_counters.as<uint8_t>() + kCtrBytes);
}

static int set_err(klf_engine* e, int code, const std::string& m) {
  if (e) e->err = m;
  return code;
}

// The since cutoff as the scan compares it (RunArgs::since_dig): the 23 digits of its
// canonical UTC prefix, packed like parse_fast's p0..p5.  The fast path only accepts years
// 1970..2099, so an earlier cutoff passes every such line (1970-01-01T00:00:00Z) and a
// later one none (all '9').
static void since_digits(int64_t sec, int64_t nsec, uint32_t out[6]) {
  sec += nsec / 1000000000;  // (nsec normalised into [0, 1e9))
  nsec %= 1000000000;
  if (nsec < 0) {
    nsec += 1000000000;
    --sec;
  }
  char d[48];
  if (sec < 0) {
    memcpy(d, "19700101000000000000000", 23);
  } else if (sec >= 4102444800LL) {  // 2100-01-01T00:00:00Z
    memset(d, '9', 23);
  } else {
    const int64_t z = sec / 86400 + 719468, era = z / 146097;  // civil from days (proleptic Gregorian)
    const int64_t doe = z - era * 146097, yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100), mp = (5 * doy + 2) / 153;
    const int64_t day = doy - (153 * mp + 2) / 5 + 1, month = mp < 10 ? mp + 3 : mp - 9;
    const int64_t year = yoe + era * 400 + (month <= 2 ? 1 : 0), sod = sec % 86400;
    snprintf(d, sizeof d, "%04d%02d%02d%02d%02d%02d%09d", (int)year, (int)month, (int)day, (int)(sod / 3600),
             (int)(sod / 60 % 60), (int)(sod % 60), (int)nsec);
  }
  auto be = [&](char a, char b, char c, char e) {
    return (uint32_t)(uint8_t)a << 24 | (uint32_t)(uint8_t)b << 16 | (uint32_t)(uint8_t)c << 8 | (uint8_t)e;
  };
  out[0] = be(d[0], d[1], d[2], d[3]);      // YYYY
  out[1] = be(d[4], d[5], d[6], d[7]);      // MMDD
  out[2] = be(d[8], d[9], d[10], d[11]);    // hhmm
  out[3] = be(d[12], d[13], d[14], d[15]);  // ss n0 n1
  out[4] = be(d[16], d[17], d[18], d[19]);  // n2..n5
  out[5] = be(d[20], d[21], '0', d[22]);    // n6 n7 pad n8
}
static int hip_err(klf_engine* e, hipError_t h, const char* where) {
  return set_err(e, KLF_EHIP, std::string(where) + ": " + hipGetErrorString(h));
}
#define HIPCHK(e, x, where) do { hipError_t _h = (x); if (_h != hipSuccess) return hip_err(e, _h, where); } while (0)

extern "C" const char* klf_strerror(int code) {
  switch (code) {
    case KLF_OK: return "ok";
    case KLF_EINVAL: return "invalid argument";
    case KLF_ENOMEM: return "out of memory";
    case KLF_EHIP: return "HIP runtime error";
    case KLF_EPATTERN: return "pattern outside the supported RE2 subset";
    case KLF_ETOOBIG: return "pattern set exceeds engine limits";
    case KLF_ESTATE: return "call out of order";
    case KLF_EIO: return "write to a stream's file failed";
    default: return "unknown error";
  }
}

extern "C" const char* klf_last_error(const klf_engine* e) { return e ? e->err.c_str() : ""; }

template <class T>
static hipError_t upload(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
  hipError_t h = b.ensure(std::max<size_t>(v.size() * sizeof(T), 16));
  if (h != hipSuccess || v.empty()) return h;
  h = hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st);
  if (h != hipSuccess) return h;
  return hipStreamSynchronize(st);
}
// Several tables through one pinned staging buffer: async copies in stream order, no sync
// (the staging buffer is rewritten only after the stream has drained it: the next
// staged upload waits for the previous one's event)
struct StagedUpload {
  HostBuf& stage;
  hipStream_t st;
  hipEvent_t done;
  size_t off = 0;
  std::vector<std::pair<DevBuf*, std::pair<size_t, size_t>>> items;  // (buffer, (offset, bytes))
  template <class T>
  hipError_t add(DevBuf& b, const std::vector<T>& v) {
    hipError_t h = b.ensure(std::max<size_t>(v.size() * sizeof(T), 16));
    if (h != hipSuccess) return h;
    items.push_back({&b, {off, v.size() * sizeof(T)}});
    off += (v.size() * sizeof(T) + 255) & ~(size_t)255;
    return hipSuccess;
  }
  template <class T>
  void fill(size_t k, const std::vector<T>& v) {
    if (!v.empty()) memcpy(stage.as<uint8_t>() + items[k].second.first, v.data(), v.size() * sizeof(T));
  }
};

// The prefilter tables that the layout choice (place_needles) rewrites: bitmap, buckets,
// anchor pre-checks, and the scalar layout fields of the device pattern set.
static hipError_t upload_prefilter(klf_engine* e) {
  const auto& cs = e->cs;
  hipStream_t st = e->stream;
  hipError_t h;
  std::vector<uint32_t> anc = cs.qf_anc_pre;
  if (anc.empty()) anc.assign(2, 0u);
  std::vector<uint32_t> pre = cs.rx_pre;  // the chosen needle set's match-start bounds
  if (pre.empty()) pre.assign(std::max<uint32_t>(cs.rx_count, 1u), klf::kRxPreUnbounded);
  // one pinned staging buffer, six async copies, no host sync (first-run latency)
  if (e->stage_ev_pending && (h = hipEventSynchronize(e->stage_ev)) != hipSuccess) return h;
  StagedUpload u{e->h_stage, st, e->stage_ev};
  if ((h = u.add(e->d_qf_bitmap, cs.qf_bitmap)) != hipSuccess || (h = u.add(e->d_qf_head, cs.qf_head)) != hipSuccess ||
      (h = u.add(e->d_qf_ent, cs.qf_ent)) != hipSuccess || (h = u.add(e->d_qf_anc, anc)) != hipSuccess ||
      (h = u.add(e->d_qf_nbytes, cs.qf_nbytes)) != hipSuccess || (h = u.add(e->d_rx_pre, pre)) != hipSuccess)
    return h;
  if ((h = e->h_stage.ensure(u.off + 256)) != hipSuccess) return h;
  u.fill(0, cs.qf_bitmap);
  u.fill(1, cs.qf_head);
  u.fill(2, cs.qf_ent);
  u.fill(3, anc);
  u.fill(4, cs.qf_nbytes);
  u.fill(5, pre);
  for (auto& it : u.items)
    if (it.second.second &&
        (h = hipMemcpyAsync(it.first->p, e->h_stage.as<uint8_t>() + it.second.first, it.second.second,
                            hipMemcpyHostToDevice, st)) != hipSuccess)
      return h;
  if ((h = hipEventRecord(e->stage_ev, st)) != hipSuccess) return h;
  e->stage_ev_pending = true;
  klf::DevPatterns& P = e->dpats;
  if (cs.rx_count) {  // (k_nfa_win / k_nfa split)
    P.rx_pre = e->d_rx_pre.as<uint32_t>();
    P.rx_unbounded = (uint32_t)std::count(pre.begin(), pre.end(), klf::kRxPreUnbounded);
  }
  P.qf_stride = cs.qf_stride;
  P.qf_mask = cs.qf_mask;
  P.qf_w24 = cs.qf_q == 4 ? 24u : 0u;
  P.qf_k = cs.qf_k;
  P.qf_bitmap = e->d_qf_bitmap.as<uint32_t>();
  P.qf_head = e->d_qf_head.as<uint32_t>();
  P.qf_ent = e->d_qf_ent.as<uint4>();
  P.qf_nbytes = e->d_qf_nbytes.as<uint32_t>();
  P.qf_anc_on = cs.qf_anc_on ? 1u : 0u;
  P.qf_anc_byte = cs.qf_anc_byte * 0x01010101u;
  P.qf_anc_fold = cs.qf_anc_fold;
  P.qf_anc_n = (uint32_t)(cs.qf_anc_pre.size() / 2);
  P.qf_anc_pre = e->d_qf_anc.as<uint32_t>();
  return hipSuccess;
}

// Host tables -> device buffers through the pinned staging buffer: one memcpy each into it,
// async copies in stream order, no host sync (the next staged upload waits for this one's
// event before it rewrites the buffer).  klf_open's pattern tables go up this way.
struct TableItem {
  DevBuf* dst;
  const void* src;
  size_t bytes;
};
static hipError_t stage_tables(klf_engine* e, const std::vector<TableItem>& items) {
  hipError_t h;
  if (e->stage_ev_pending && (h = hipEventSynchronize(e->stage_ev)) != hipSuccess) return h;
  e->stage_ev_pending = false;
  size_t total = 0;
  for (auto& it : items) {
    if ((h = it.dst->ensure(std::max<size_t>(it.bytes, 16))) != hipSuccess) return h;
    total += (it.bytes + 255) & ~(size_t)255;
  }
  if ((h = e->h_stage.ensure(total + 256)) != hipSuccess) return h;
  size_t off = 0;
  for (auto& it : items) {
    if (it.bytes) {
      memcpy(e->h_stage.as<uint8_t>() + off, it.src, it.bytes);
      if ((h = hipMemcpyAsync(it.dst->p, e->h_stage.as<uint8_t>() + off, it.bytes, hipMemcpyHostToDevice, e->stream)) !=
          hipSuccess)
        return h;
    }
    off += (it.bytes + 255) & ~(size_t)255;
  }
  if ((h = hipEventRecord(e->stage_ev, e->stream)) != hipSuccess) return h;
  e->stage_ev_pending = true;
  return hipSuccess;
}
template <class T>
static TableItem item(DevBuf& b, const std::vector<T>& v) {
  return TableItem{&b, v.data(), v.size() * sizeof(T)};
}

// The compiled set's matcher tables to the device (the prefilter layout only when it is
// placed already: tune_later = the first batch's statistics will place it).
static hipError_t upload_pattern_tables(klf_engine* e, bool tune_later) {
  const auto& cs = e->cs;
  hipError_t h;
  std::vector<TableItem> items;
  std::vector<uint8_t> padded;
  std::vector<uint64_t> vec, vec4;
  std::vector<uint32_t> pre0;
  if (cs.mode == klf::CompiledSet::kLiteral1) {
    padded = cs.literal;
    padded.resize((cs.literal.size() + 3) / 4 * 4 + 4, 0);  // bytes, then dword view at +0
    items.push_back(item(e->d_lit, padded));
  } else if (cs.mode == klf::CompiledSet::kGeneral) {
    klf::DevPatterns& P = e->dpats;
    if (cs.ac_states) {
      for (auto x : {item(e->d_ac_class, cs.ac_class), item(e->d_ac_next, cs.ac_next), item(e->d_ac_accept, cs.ac_accept),
                     item(e->d_ac_out, cs.ac_out), item(e->d_ac_dict, cs.ac_dict)})
        items.push_back(x);
      P.ac_states = cs.ac_states;
      P.ac_classes = cs.ac_classes;
    }
    if (cs.rx_count) {
      // first | last | init0 | end, each [rx_count]; and [rx][4] interleaved for k_nfa
      for (const auto* v : {&cs.rx_first, &cs.rx_last, &cs.rx_init0, &cs.rx_end}) vec.insert(vec.end(), v->begin(), v->end());
      for (uint32_t r = 0; r < cs.rx_count; ++r)
        for (const auto* v : {&cs.rx_first, &cs.rx_last, &cs.rx_init0, &cs.rx_end}) vec4.push_back((*v)[r]);
      pre0 = cs.rx_pre.empty() ? std::vector<uint32_t>(cs.rx_count, klf::kRxPreUnbounded) : cs.rx_pre;
      for (auto x : {item(e->d_rx_class, cs.rx_class), item(e->d_rx_b, cs.rx_b), item(e->d_rx_follow, cs.rx_follow),
                     item(e->d_rx_vec, vec), item(e->d_rx_flags, cs.rx_flags), item(e->d_rx_pre, pre0),
                     item(e->d_rx_vec4, vec4)})
        items.push_back(x);
      P.rx_unbounded = (uint32_t)std::count(pre0.begin(), pre0.end(), klf::kRxPreUnbounded);
      P.rx_count = cs.rx_count;
      P.rx_classes = cs.rx_classes;
      P.rx_maxpos = std::max<uint32_t>(1, cs.rx_maxpos);
    }
  }
  if (!items.empty() && (h = stage_tables(e, items)) != hipSuccess) return h;
  if (cs.mode == klf::CompiledSet::kGeneral) {  // device pointers of the staged tables
    klf::DevPatterns& P = e->dpats;
    if (cs.ac_states) {
      P.ac_class = e->d_ac_class.as<uint8_t>();
      P.ac_next = e->d_ac_next.as<uint32_t>();
      P.ac_accept = e->d_ac_accept.as<uint8_t>();
      P.ac_out = e->d_ac_out.as<int32_t>();
      P.ac_dict = e->d_ac_dict.as<uint32_t>();
    }
    if (cs.rx_count) {
      const uint64_t* v = e->d_rx_vec.as<uint64_t>();
      P.rx_class = e->d_rx_class.as<uint8_t>();
      P.rx_b = e->d_rx_b.as<uint64_t>();
      P.rx_follow = e->d_rx_follow.as<uint64_t>();
      P.rx_first = v;
      P.rx_last = v + cs.rx_count;
      P.rx_init0 = v + 2 * cs.rx_count;
      P.rx_end = v + 3 * cs.rx_count;
      P.rx_flags = e->d_rx_flags.as<uint32_t>();
      P.rx_pre = e->d_rx_pre.as<uint32_t>();
      P.rx_vec = e->d_rx_vec4.as<uint64_t>();
    }
    if (cs.qf_on) {
      if (!tune_later && (h = upload_prefilter(e)) != hipSuccess) return h;
      P.qf_on = 1;
      P.qf_fold = cs.qf_fold;
    }
  }
  return hipSuccess;
}

// the automaton thread: build, then one block on the device and one copy
// The literal automaton's thread: builds the tables, lays them out as one pinned block and
// maps the device block.  The upload itself is left to the join (ensure_ac), on the launch
// stream: a copy from this thread would go to HIP's null stream, where it queues behind a
// scan already running on that stream (an engine opened without a stream) and the join
// then waits for the scan (advisor r04).
static void ac_build_upload(klf_engine* e) {
  klf::build_ac(e->ac_lits, e->ac_tabs);
  const klf::AcTables& t = e->ac_tabs;
  hipError_t h = hipSetDevice(e->device);
  const std::pair<const void*, size_t> parts[5] = {
      {t.cls.data(), t.cls.size()}, {t.next.data(), t.next.size() * 4}, {t.accept.data(), t.accept.size()},
      {t.out.data(), t.out.size() * 4}, {t.dict.data(), t.dict.size() * 4}};
  size_t total = 0;
  for (int k = 0; k < 5; ++k) {
    e->ac_off[k] = total;
    e->ac_cap[k] = (std::max<size_t>(parts[k].second, 256) + 255) & ~(size_t)255;
    total += e->ac_cap[k];
  }
  e->ac_total = total;
  if (h == hipSuccess) h = e->h_acblk.ensure(total);
  if (h == hipSuccess) {
    memset(e->h_acblk.p, 0, total);
    for (int k = 0; k < 5; ++k) memcpy(e->h_acblk.as<uint8_t>() + e->ac_off[k], parts[k].first, parts[k].second);
  }
  if (h == hipSuccess) h = e->d_acblk.ensure(total);
  e->ac_err = h;
}

// Joins the automaton thread (if any) and points the device patterns at its tables.
static int ensure_ac(klf_engine* e) {
  if (e->ac_thread.joinable()) e->ac_thread.join();
  if (!e->ac_pending) return KLF_OK;
  e->ac_pending = false;
  if (e->ac_err != hipSuccess) return hip_err(e, e->ac_err, "Aho-Corasick tables");
  // the upload, ordered on the launch stream before the first kernel that reads it (the
  // pinned block stays until klf_close)
  HIPCHK(e, hipMemcpyAsync(e->d_acblk.p, e->h_acblk.p, e->ac_total, hipMemcpyHostToDevice, e->stream),
         "upload Aho-Corasick tables");
  DevBuf* dst[5] = {&e->d_ac_class, &e->d_ac_next, &e->d_ac_accept, &e->d_ac_out, &e->d_ac_dict};
  for (int k = 0; k < 5; ++k) {
    dst[k]->release();
    dst[k]->p = e->d_acblk.as<uint8_t>() + e->ac_off[k];
    dst[k]->cap = e->ac_cap[k];
    dst[k]->borrowed = true;
  }
  klf::CompiledSet& cs = e->cs;
  klf::AcTables& t = e->ac_tabs;
  cs.ac_states = t.states;
  cs.ac_classes = t.classes;
  cs.ac_class = std::move(t.cls);
  cs.ac_next = std::move(t.next);
  cs.ac_accept = std::move(t.accept);
  cs.ac_out = std::move(t.out);
  cs.ac_dict = std::move(t.dict);
  klf::DevPatterns& P = e->dpats;
  P.ac_states = cs.ac_states;
  P.ac_classes = cs.ac_classes;
  P.ac_class = e->d_ac_class.as<uint8_t>();
  P.ac_next = e->d_ac_next.as<uint32_t>();
  P.ac_accept = e->d_ac_accept.as<uint8_t>();
  P.ac_out = e->d_ac_out.as<int32_t>();
  P.ac_dict = e->d_ac_dict.as<uint32_t>();
  return KLF_OK;
}

extern "C" int klf_open(const klf_config* cfg, klf_engine** out) {
  if (!cfg || !out || (cfg->n_patterns && !cfg->patterns)) return KLF_EINVAL;
  *out = nullptr;
  auto* e = new (std::nothrow) klf_engine();
  if (!e) return KLF_ENOMEM;
  // 1) patterns (host only; errors surface before any device work)
  std::vector<std::vector<uint8_t>> pats;
  std::vector<uint32_t> kinds;
  for (uint32_t i = 0; i < cfg->n_patterns; ++i) {
    const klf_pattern& p = cfg->patterns[i];
    if (p.len && !p.bytes) { delete e; return KLF_EINVAL; }
    pats.emplace_back(p.bytes, p.bytes + p.len);
    kinds.push_back(p.kind);
  }
  int code = KLF_OK;
  std::string err;
  const auto t_open0 = std::chrono::steady_clock::now();
  // the prefilter layout waits for the first batch's statistics (the first run places the
  // needles), unless tuning is off (KLF_QF_TUNE=0: placed here, from byte-class estimates)
  const char* tune_env = getenv("KLF_QF_TUNE");
  const bool tune_later = !(tune_env && strcmp(tune_env, "0") == 0);
  const bool compiled = klf::compile_set(pats, kinds, e->cs, err, code, !tune_later, true, true);
  e->tune_later = tune_later;
  e->ac_lits.swap(e->cs.ac_lits);  // (the automaton thread's input; built after the device setup)
  if (compiled && e->cs.also_all_pending) {
    e->pend_pats = pats;
    e->pend_kinds = kinds;
  }
  if (getenv("KLF_DIAG"))
    fprintf(stderr, "[klf] open: pattern compile %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_open0).count());
  if (!compiled) {
    // keep the engine alive so the caller can read klf_last_error; report failure
    e->err = err;
    *out = e;
    return code;
  }
  // 2) device
  e->device = cfg->device;
  e->n_user = cfg->n_patterns;
  e->dpats.n_cids = e->cs.n_cids;
  e->dpats.n_lits = e->cs.n_lits;
  hipError_t h = hipSetDevice(cfg->device);
  if (h != hipSuccess) { e->err = std::string("hipSetDevice: ") + hipGetErrorString(h); *out = e; return KLF_EHIP; }
  const bool diag_open = getenv("KLF_DIAG") != nullptr;
  auto open_mark = [&](const char* what) {
    if (diag_open)
      fprintf(stderr, "[klf] open: %s at %.1f us\n", what,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_open0).count());
  };
  open_mark("device set");
  int ncu = 0;  // (one attribute query: hipGetDeviceProperties fills the whole struct, ~ms)
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && ncu > 0)
    e->num_cus = ncu;
  open_mark("attribute");
  // the caller's stream, else HIP's null stream: it exists from device init, while a new
  // stream costs ~5 ms of host time when it brings up a hardware queue (MI355X), which a
  // one-shot klogs invocation would pay in full
  e->stream = static_cast<hipStream_t>(cfg->hip_stream);
  open_mark("stream");
  for (auto& x : e->ev) {
    h = hipEventCreate(&x);
    if (h != hipSuccess) { e->err = "hipEventCreate failed"; *out = e; return KLF_EHIP; }
  }
  if (getenv("KLF_DIAG"))
    fprintf(stderr, "[klf] open: events done at %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_open0).count());
  if ((h = hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming)) != hipSuccess) {
    *out = e;
    return hip_err(e, h, "staging event");
  }
  if (getenv("KLF_DIAG"))
    fprintf(stderr, "[klf] open: device setup done at %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_open0).count());
  // 3) pattern tables to the device
  if ((h = upload_pattern_tables(e, tune_later)) != hipSuccess) {
    *out = e;
    return hip_err(e, h, "upload pattern tables");
  }
  if (const char* cc = getenv("KLF_CAND_CAP"))  // tests: force the queue-overflow fallback
    e->cand_cap = (uint32_t)std::max(1L, std::min(atol(cc), 1L << 28));
  if (const char* pl = getenv("KLF_PAIRS_LOG2"))  // tests: a small per-pattern pair set (grows on overflow)
    e->pairs_log2 = (uint32_t)std::max(4L, std::min(atol(pl), 28L));
  if (const char* hc = getenv("KLF_HITS_CAP"))  // tests: force the hit-list overflow fallback
    e->hits_cap_max = (uint64_t)std::max(1L, std::min(atol(hc), 1L << 28));
  if (!e->ac_lits.empty()) {
    e->ac_pending = true;
    try {
      e->ac_thread = std::thread(ac_build_upload, e);
    } catch (...) {  // no thread: build it here
      ac_build_upload(e);
    }
  }
  if (getenv("KLF_DIAG"))
    fprintf(stderr, "[klf] open: total %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_open0).count());
  *out = e;
  return KLF_OK;
}

static void release_staged(klf_engine* e);
static void free_chunk(klf_engine::StageChunk& c);

extern "C" void klf_close(klf_engine* e) {
  if (!e) return;
  if (e->ac_thread.joinable()) e->ac_thread.join();
  (void)hipStreamSynchronize(e->stream);
  if (e->copy_stream) (void)hipStreamSynchronize(e->copy_stream);
  for (DevBuf* b : {&e->d_lit, &e->d_ac_class, &e->d_ac_next, &e->d_ac_accept, &e->d_rx_class, &e->d_rx_b,
                    &e->d_rx_follow, &e->d_rx_vec, &e->d_rx_flags, &e->d_rx_pre, &e->d_qf_bitmap, &e->d_qf_head,
                    &e->d_qf_ent, &e->d_qf_nbytes, &e->d_qf_anc, &e->d_rx_vec4, &e->d_qhits, &e->d_hslots, &e->d_hist, &e->d_hflat, &e->d_cand, &e->d_batch, &e->d_segs, &e->d_tstat,
                    &e->d_slots, &e->d_pool, &e->d_tile_base, &e->d_bsum, &e->d_cstatus, &e->d_counters, &e->d_cmap, &e->d_cseg,
                    &e->d_line_off, &e->d_meta, &e->d_bits, &e->d_wpre, &e->d_out, &e->d_tile_seg, &e->d_mpart, &e->d_trec, &e->d_truns, &e->d_kbase,
                    &e->d_fext0, &e->d_fext, &e->d_frinfo, &e->d_out2})
    b->release();
  e->d_asm.release();
  e->d_scratch.release();
  e->h_rb.release();
  e->h_acblk.release();
  e->h_hist.release();
  e->h_stage.release();
  for (DevBuf* b : {&e->d_ac_out, &e->d_ac_dict, &e->d_pcount, &e->d_pairs}) b->release();
  e->d_block.release();
  e->d_block2.release();
  e->d_acblk.release();
  e->copier.reset();
  {
    std::lock_guard<std::mutex> g(e->mu);
    release_staged(e);
    for (auto& c : e->chunk_pool) free_chunk(c);
    e->chunk_pool.clear();
    for (uint8_t* d : e->dchunk_pool) (void)hipFree(d);
    e->dchunk_pool.clear();
    for (auto x : e->ev_pool) (void)hipEventDestroy(x);
    e->ev_pool.clear();
  }
  for (auto& x : e->ev)
    if (x) (void)hipEventDestroy(x);
  if (e->copy_done) (void)hipEventDestroy(e->copy_done);
  if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
  if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
  if (e->cap_stream) (void)hipStreamDestroy(e->cap_stream);
  if (e->stage_ev) (void)hipEventDestroy(e->stage_ev);
  delete e;
  (void)hipGetLastError();  // nothing above reports: leave no sticky error for the next engine
}

// ------------------------------------------------------------------------ staging ---

static constexpr size_t kStageChunk = 64u << 20;  // pinned staging chunk = device chunk
static constexpr size_t kMaxInflight = 8;         // pinned chunks with an H2D in flight (512 MiB)

// The copy stream of the host staging path (and its event), made on first use: a
// device-resident caller (klf_run_device) never pays for it.
static hipError_t ensure_copy_stream(klf_engine* e) {
  std::call_once(e->copy_stream_once, [e] {
    hipError_t h = hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking);
    if (h == hipSuccess) h = hipEventCreateWithFlags(&e->copy_done, hipEventDisableTiming);
    e->copy_stream_err = h;
  });
  return e->copy_stream_err;
}

static void grow_table(klf_engine* e, size_t n) {  // caller holds e->mu
  while (e->staged.size() < n) e->staged.emplace_back(new klf_engine::StagedStream());
}

extern "C" int klf_set_streams(klf_engine* e, uint32_t n) {
  if (!e) return KLF_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (e->ran) return set_err(e, KLF_ESTATE, "klf_set_streams after klf_run: klf_reset first");
  if (n < e->staged.size()) return set_err(e, KLF_ESTATE, "cannot shrink the stream table; klf_reset first");
  try {
    grow_table(e, n);
  } catch (...) {
    return set_err(e, KLF_ENOMEM, "stream table");
  }
  return KLF_OK;
}

static void free_chunk(klf_engine::StageChunk& c) {
  if (!c.p) return;
  if (c.pinned) (void)hipHostFree(c.p);
  else free(c.p);
  c.p = nullptr;
}

// A free pinned chunk: the pool, else a chunk whose H2D has finished, else (with
// kMaxInflight chunks in flight) the oldest one once its DMA is done, else a new one.
static bool take_chunk(klf_engine* e, klf_engine::StageChunk* c) {
  klf_engine::Inflight wait{};
  bool have_wait = false;
  {
    std::lock_guard<std::mutex> g(e->mu);
    while (!e->inflight.empty() && hipEventQuery(e->inflight.front().ev) == hipSuccess) {
      e->chunk_pool.push_back(e->inflight.front().c);
      e->ev_pool.push_back(e->inflight.front().ev);
      e->inflight.pop_front();
    }
    if (!e->chunk_pool.empty()) {
      *c = e->chunk_pool.back();
      e->chunk_pool.pop_back();
      c->used = 0;
      return true;
    }
    if (e->inflight.size() >= kMaxInflight) {
      wait = e->inflight.front();
      e->inflight.pop_front();
      have_wait = true;
    }
  }
  if (have_wait) {
    (void)hipEventSynchronize(wait.ev);
    {
      std::lock_guard<std::mutex> g(e->mu);
      e->ev_pool.push_back(wait.ev);
    }
    *c = wait.c;
    c->used = 0;
    return true;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, kStageChunk, hipHostMallocDefault) == hipSuccess && p) {
    c->p = static_cast<uint8_t*>(p);
    c->pinned = true;
  } else {
    (void)hipGetLastError();
    c->p = static_cast<uint8_t*>(malloc(kStageChunk));
    c->pinned = false;
    if (!c->p) return false;
  }
  c->used = 0;
  return true;
}

// The stream's full pinned chunk -> a device chunk, DMA'd now on the copy stream (the
// capture keeps running meanwhile); the pinned chunk returns to the pool when the DMA ends.
static int ship_chunk(klf_engine* e, klf_engine::StagedStream* s) {
  uint8_t* d = nullptr;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(e->mu);
    if (!e->dchunk_pool.empty()) {
      d = e->dchunk_pool.back();
      e->dchunk_pool.pop_back();
    }
    if (!e->ev_pool.empty()) {
      ev = e->ev_pool.back();
      e->ev_pool.pop_back();
    }
  }
  hipError_t h = hipSuccess;
  if (!d) h = hipMalloc(reinterpret_cast<void**>(&d), kStageChunk);
  if (h != hipSuccess) {  // hand the event back; the error string is shared with other stagers
    std::lock_guard<std::mutex> g(e->mu);
    if (ev) e->ev_pool.push_back(ev);
    return hip_err(e, h, "device staging chunk");
  }
  if (!ev) h = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (h == hipSuccess) h = hipMemcpyAsync(d, s->cur.p, kStageChunk, hipMemcpyHostToDevice, e->copy_stream);
  if (h == hipSuccess) h = hipEventRecord(ev, e->copy_stream);
  std::lock_guard<std::mutex> g(e->mu);
  if (h != hipSuccess) {
    e->dchunk_pool.push_back(d);
    if (ev) e->ev_pool.push_back(ev);
    return hip_err(e, h, "early H2D");
  }
  s->dchunks.push_back(d);
  e->inflight.push_back({s->cur, ev});
  s->cur = klf_engine::StageChunk{};
  return KLF_OK;
}

extern "C" int klf_stage(klf_engine* e, uint32_t id, const uint8_t* p, size_t n) {
  if (!e || (n && !p)) return KLF_EINVAL;
  klf_engine::StagedStream* dst;
  {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->ran) return set_err(e, KLF_ESTATE, "klf_stage after klf_run: klf_reset first");
    try {
      grow_table(e, (size_t)id + 1);
    } catch (...) {
      return set_err(e, KLF_ENOMEM, "stream table");
    }
    dst = e->staged[id].get();  // stable: the table holds pointers, only the table moves
  }
  if (hipError_t h = ensure_copy_stream(e); h != hipSuccess) return hip_err(e, h, "copy stream");
  std::call_once(e->copier_once, [e] {
    int nw = 3;  // staging copy workers (+ the calling thread)
    if (const char* v = getenv("KLF_STAGE_THREADS")) nw = std::max(0, std::min(atoi(v), 32));
    e->copier.reset(new klf::CopyPool(nw));
  });
  while (n) {
    if (!dst->cur.p && !take_chunk(e, &dst->cur)) {
      std::lock_guard<std::mutex> g(e->mu);
      return set_err(e, KLF_ENOMEM, "pinned staging chunk");
    }
    const size_t k = std::min(n, kStageChunk - dst->cur.used);
    e->copier->copy(dst->cur.p + dst->cur.used, p, k);
    dst->cur.used += k;
    dst->len += k;
    p += k;
    n -= k;
    if (dst->cur.used == kStageChunk) {
      const int rc = ship_chunk(e, dst);
      if (rc) return rc;
    }
  }
  return KLF_OK;
}

static void release_staged(klf_engine* e) {  // caller holds e->mu; no H2D may be in flight
  for (auto& s : e->staged) {
    for (uint8_t* d : s->dchunks) e->dchunk_pool.push_back(d);
    if (s->cur.p) {
      s->cur.used = 0;
      e->chunk_pool.push_back(s->cur);
    }
  }
  for (auto& f : e->inflight) {
    e->chunk_pool.push_back(f.c);
    e->ev_pool.push_back(f.ev);
  }
  e->inflight.clear();
  e->staged.clear();
  e->ran = false;
}

extern "C" int klf_reset(klf_engine* e) {
  if (!e) return KLF_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  if (e->copy_stream) (void)hipStreamSynchronize(e->copy_stream);  // early DMAs read the pinned chunks
  (void)hipStreamSynchronize(e->stream);       // k_assemble reads the device chunks
  release_staged(e);
  return KLF_OK;
}

extern "C" int klf_layout(uint32_t n, const uint64_t* lens, uint64_t* seg_base, uint64_t* total) {
  if ((n && (!lens || !seg_base)) || !total) return KLF_EINVAL;
  uint64_t off = 0;
  for (uint32_t i = 0; i < n; ++i) {
    seg_base[i] = off;
    off = align_up(off + lens[i], klf::kSegAlign);
  }
  *total = off + klf::kAllocSlack;
  return KLF_OK;
}

// -------------------------------------------------------------------------- run ---

// Waits for the run's readback by polling the stream: a blocking sync sleeps and wakes
// tens of microseconds after the last copy lands (measured ~50 us between batches of a
// capture loop), a poll returns within a microsecond or two.  The poll is bounded: past
// the expected run time (`spin_us`, the batch's bytes at ~2 TB/s plus a margin) the
// thread yields between polls for a while and then blocks, so one engine per GPU in one
// process does not keep a host core busy per GPU through a long run, and a hung kernel
// leaves the thread asleep in the runtime instead of spinning.
static hipError_t wait_stream(hipStream_t st, uint64_t spin_us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    const hipError_t h = hipStreamQuery(st);
    if (h != hipErrorNotReady) return h;
    if ((i & 63) == 63) {
      const uint64_t us = (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                              std::chrono::steady_clock::now() - t0).count();
      if (us > spin_us + 20000) return hipStreamSynchronize(st);
      if (us > spin_us) std::this_thread::yield();
    }
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

// Output bigger than the buffer (counters[kCtrOutShort], from k_cmove / k_tcopy, which
// skipped the copies that would not fit but still wrote every stream's output range): grow
// the buffer to the run's output and rerun the tail stage over the line index and bitmap
// still in HBM (k_mcount .. k_tcopy, tens of us), then read the stream records back.
static hipError_t grow_out_retail(klf_engine* e, klf::RunArgs& a, std::vector<SegOut>& so) {
  a.plan_runs = 0;  // the tile plans were consumed (k_cmove rewrote them): list the runs again
  a.skip_tcopy = 0;
  a.plan_mode = 0;  // (k_cplan / k_cmid / k_cmove, whichever path the window takes)
  for (int k = 0; k < 2; ++k) {
    uint64_t need = 0;
    for (auto& s : so) need = std::max(need, s.out_hi);
    hipError_t h = e->d_out.ensure(need + 64);
    if (h != hipSuccess) return h;
    a.out = e->d_out.as<uint8_t>();
    a.out_cap = e->d_out.cap;
    if ((h = klf::launch_retail(a, e->stream, e->ev, e->num_cus)) != hipSuccess) return h;
    uint32_t* rb = static_cast<uint32_t*>(e->h_rb.p);  // counters, then the stream records
    if ((h = hipMemcpyAsync(rb, e->d_counters.p, kCtrBytes + so.size() * sizeof(SegOut), hipMemcpyDeviceToHost,
                            e->stream)) != hipSuccess)
      return h;
    if ((h = hipStreamSynchronize(e->stream)) != hipSuccess) return h;
    memcpy(so.data(), reinterpret_cast<uint8_t*>(rb) + kCtrBytes, so.size() * sizeof(SegOut));
    if (!rb[klf::kCtrOutShort]) return hipSuccess;
  }
  return hipErrorOutOfMemory;  // the ranges did not settle (cannot happen: they do not depend on the buffer)
}

// One steady run's launch sequence (launch_pipeline, phase 0, no events inside: a graph's
// event nodes are not re-recorded by a replay) as a replayed graph, bracketed by ev[0] /
// ev[5] on the engine stream.  Returns false when the run should launch eagerly instead:
// a first sighting of these arguments, or a capture that failed (then never again).
static bool launch_graph(klf_engine* e, const klf::RunArgs& a, uint32_t& ev_mask) {
  const uint8_t* k = reinterpret_cast<const uint8_t*>(&a);
  std::vector<uint8_t> key(k, k + sizeof(a));
  key.insert(key.end(), reinterpret_cast<const uint8_t*>(&e->num_cus),
             reinterpret_cast<const uint8_t*>(&e->num_cus) + sizeof(e->num_cus));
  if (!e->gexec || key != e->gkey) {
    if (key != e->gprev) {  // first sighting: eager, remembered
      e->gprev = std::move(key);
      return false;
    }
    if (e->gexec) {
      (void)hipGraphExecDestroy(e->gexec);
      e->gexec = nullptr;
      e->gkey.clear();
    }
    if (!e->cap_stream && hipStreamCreateWithFlags(&e->cap_stream, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      e->graph_off = true;
      return false;
    }
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(e->cap_stream, hipStreamCaptureModeRelaxed) == hipSuccess;
    if (ok) {
      const hipError_t h = klf::launch_pipeline(a, e->cap_stream, nullptr, e->num_cus, 0, nullptr);
      ok = hipStreamEndCapture(e->cap_stream, &g) == hipSuccess && h == hipSuccess && g;
    }
    if (ok) ok = hipGraphInstantiate(&e->gexec, g, nullptr, nullptr, 0) == hipSuccess;
    if (g) (void)hipGraphDestroy(g);
    if (!ok) {
      (void)hipGetLastError();
      if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
      e->gexec = nullptr;
      e->graph_off = true;
      if (getenv("KLF_DIAG")) fprintf(stderr, "[klf] graph capture failed: eager launches from here on\n");
      return false;
    }
    e->gkey = std::move(key);
  }
  if (hipEventRecord(e->ev[0], e->stream) != hipSuccess) return false;
  if (hipGraphLaunch(e->gexec, e->stream) != hipSuccess) {
    (void)hipGetLastError();
    e->graph_off = true;
    return false;
  }
  ev_mask = 1u;
  if (hipEventRecord(e->ev[5], e->stream) == hipSuccess) ev_mask |= 1u << 5;
  return true;
}

static int run_device_impl(klf_engine* e, const uint8_t* d_bytes, uint32_t n_streams, const uint64_t* seg_base,
                           const uint64_t* lens, const klf_filter* f, klf_result** out) {
  if (!e || !f || !out || (n_streams && (!seg_base || !lens))) return KLF_EINVAL;
  if (f->tail < -1) return set_err(e, KLF_EINVAL, "tail must be >= -1");
  if (f->since.nsec < 0 || f->since.nsec >= 1000000000) return set_err(e, KLF_EINVAL, "since.nsec out of range");
  if (reinterpret_cast<uintptr_t>(d_bytes) % 16) return set_err(e, KLF_EINVAL, "device bytes must be 16-B aligned");
  *out = nullptr;
  const auto t_run0 = std::chrono::steady_clock::now();
  const uint64_t alloc0 = g_alloc_ns.load();
  uint64_t tune_ns = 0;
  // KLF_DIAG: wall-clock marks through the run (the first run's cost breakdown)
  static const bool diag_marks = getenv("KLF_DIAG") != nullptr;
  std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> marks;
  auto mark = [&](const char* what) {
    if (diag_marks) marks.emplace_back(what, std::chrono::steady_clock::now());
  };
  HIPCHK(e, hipSetDevice(e->device), "hipSetDevice");
  std::unique_ptr<klf_result> rp(new (std::nothrow) klf_result());  // freed on every error return
  klf_result* r = rp.get();
  if (!r) return KLF_ENOMEM;
  r->e = e;
  r->gen = ++e->gen;
  // the contiguous copy of an earlier one-pass result (klf_result_device_out): that result
  // is stale from here on (KLF_ESTATE), so is the copy
  if (e->d_out2.p) e->d_out2.release();
  r->n_streams = n_streams;
  r->seg_of.assign(n_streams, -1);
  if (e->cs.also_all_pending && (f->flags & KLF_FILTER_PATTERN_COUNTS)) {
    if (const int rc = ensure_ac(e); rc != KLF_OK) return rc;
    // the first run asking for per-pattern counts of a set with an always-pattern: compile
    // the other patterns now (klf_open kept the set as kAll); if that fails the filter stays
    // kAll's and the counts are reported unavailable
    klf::CompiledSet full;
    std::string cerr;
    int ccode = KLF_OK;
    if (klf::compile_set(e->pend_pats, e->pend_kinds, full, cerr, ccode, !e->tune_later, false)) {
      e->cs = std::move(full);
      e->dpats.n_cids = e->cs.n_cids;
      e->dpats.n_lits = e->cs.n_lits;
      HIPCHK(e, upload_pattern_tables(e, e->tune_later), "upload pattern tables");
    } else {
      e->cs.also_all_pending = false;
      e->counts_code = ccode;
      e->counts_err = "per-pattern counts unavailable: " + cerr;
    }
  }
  auto mode = e->cs.mode;
  // a set with an always-pattern (also_all) filters as kAll; its other patterns are
  // evaluated only when the run counts per pattern
  if (e->cs.also_all && !(f->flags & KLF_FILTER_PATTERN_COUNTS)) mode = klf::CompiledSet::kAll;
  r->has_bits = mode != klf::CompiledSet::kNone;

  std::vector<SegDesc> segs;
  uint64_t total_bytes = 0, ntiles = 0, cap = 0;
  for (uint32_t i = 0; i < n_streams; ++i) {
    if (!lens[i]) continue;
    if (seg_base[i] % klf::kSegAlign) return set_err(e, KLF_EINVAL, "seg_base must be 256-B aligned");
    SegDesc d;
    d.base = seg_base[i];
    d.len = lens[i];
    d.tile0 = (uint32_t)ntiles;
    d.ntiles = (uint32_t)((lens[i] + klf::kTile - 1) / klf::kTile);
    r->seg_of[i] = (int64_t)segs.size();
    segs.push_back(d);
    r->seg_base.push_back(d.base);
    ntiles += d.ntiles;
    total_bytes += lens[i];
    cap += lens[i] / 32 + 2;  // kubelet lines carry a >= 31-byte prefix; overflow -> exact rerun
  }
  if (ntiles >= (1ull << 32)) return set_err(e, KLF_EINVAL, "batch too large");
  const uint32_t nsegs = (uint32_t)segs.size();
  // the line arrays: from the last run's line density (+25 %) once there is one, else the
  // 32-B estimate above (1 G lines for 32 GiB: gigabytes of line index for a first run)
  auto learned_cap = [&]() {
    return (uint64_t)(e->line_density * (double)total_bytes * 1.25) + 2ull * nsegs + 4096;
  };
  if (e->line_density > 0.0) cap = std::min<uint64_t>(cap, learned_cap());
  // asked-for per-pattern counts are reported even when every stream is empty (all zero)
  r->counted = (f->flags & KLF_FILTER_PATTERN_COUNTS) != 0;
  r->pcount_ok = true;  // no segment reads pcount
  if (nsegs == 0) { e->last_gen = r->gen; *out = rp.release(); return KLF_OK; }
  r->pcount_ok = false;
  // tests: a line capacity clamped on every attempt forces the overflow error below
  uint64_t cap_clamp = ~0ull;
  if (const char* v = getenv("KLF_DEBUG_CAP_CLAMP")) cap_clamp = std::max(1L, atol(v));
  cap = std::min(cap, cap_clamp);

  hipStream_t st = e->stream;
  bool same_layout = segs.size() == e->last_segs.size() && e->d_tile_seg.cap >= ntiles * 4 &&
                     memcmp(segs.data(), e->last_segs.data(), segs.size() * sizeof(SegDesc)) == 0;
  mark("pre-segs");
  if (!same_layout) {
    HIPCHK(e, e->d_segs.ensure(nsegs * sizeof(SegDesc)), "alloc segs");
    mark("segs alloc");
    // (a pageable source: the runtime stages it before the call returns, so `segs` may go
    // out of scope with no stream sync, which would wait for klf_open's table uploads)
    HIPCHK(e, hipMemcpyAsync(e->d_segs.p, segs.data(), nsegs * sizeof(SegDesc), hipMemcpyHostToDevice, st),
           "H2D segs");
    mark("segs copy");
    HIPCHK(e, e->d_tile_seg.ensure(ntiles * 4 + 16), "alloc tile_seg");  // + whole 16-B loads past the end
  }
  mark("segs");
  // First batch of a prefiltered set: the data's own gram statistics (k_gramhist over a
  // sample) place the needles' sampling windows.  The sample's readback is in flight while
  // the host maps the workspace below; the layout and its upload follow the sync.  The
  // sample's newline share also sizes the first run's line arrays (no phase-1 readback).
  bool tune_pending = false;
  std::chrono::steady_clock::time_point t_tune0;
  if (mode == klf::CompiledSet::kGeneral && e->cs.qf_on && !e->cs.qf_tuned) {
    e->cs.qf_tuned = true;
    t_tune0 = std::chrono::steady_clock::now();
    const char* tune = getenv("KLF_QF_TUNE");
    if (!tune || strcmp(tune, "0") != 0) {
      const size_t nh = klf::kGramHistWords;
      HIPCHK(e, e->d_hist.ensure(nh * 4), "alloc hist");
      HIPCHK(e, e->h_hist.ensure(nh * 4), "alloc hist readback");
      HIPCHK(e, klf::launch_gramhist(d_bytes, e->d_segs.as<SegDesc>(), nsegs, klf::kGramHistSample, e->cs.qf_fold,
                                     e->d_hist.as<uint32_t>(), st), "gram histogram");
      HIPCHK(e, hipMemcpyAsync(e->h_hist.p, e->d_hist.p, nh * 4, hipMemcpyDeviceToHost, st), "D2H hist");
      tune_pending = true;
    }
  }
  // Any other first run (literals, no patterns, unprefiltered sets): the line density from a
  // newline count over 64 tiles spread over the batch, read back while the workspace is
  // mapped -- instead of a readback between the scan and the rest of the pipeline (the
  // scan's time plus the host's array setup in series: C2's first run 1.16 ms vs 1.01 warm)
  bool nl_pending = false;
  uint32_t nl_blocks = 0;
  // (a first batch whose 32-B-rule line arrays take at most ~2 GB maps them as they are: no
  // sample, no sync before the scan -- C1 / C2; lines under 32 B overflow and rerun exactly)
  const bool small_first = e->line_density == 0.0 && cap * 11 <= (2ull << 30) && !getenv("KLF_TWO_PHASE") &&
                           !getenv("KLF_DEBUG_NL_SCALE");
  if (!tune_pending && e->line_density == 0.0 && !small_first && !getenv("KLF_TWO_PHASE")) {
    nl_blocks = (uint32_t)std::min<uint64_t>(ntiles, 64);
    HIPCHK(e, e->d_hist.ensure((size_t)nl_blocks * 8), "alloc line sample");
    HIPCHK(e, e->h_hist.ensure((size_t)nl_blocks * 8), "alloc line sample readback");
    HIPCHK(e, klf::launch_nlsample(d_bytes, e->d_segs.as<SegDesc>(), nsegs, (uint32_t)ntiles, nl_blocks,
                                   e->d_hist.as<uint32_t>(), st), "line sample");
    HIPCHK(e, hipMemcpyAsync(e->h_hist.p, e->d_hist.p, (size_t)nl_blocks * 8, hipMemcpyDeviceToHost, st),
           "D2H line sample");
    nl_pending = nl_blocks > 0;
  }
  double est_density = 0.0;  // lines per byte of the first batch's sample (0: none)
  auto finish_tune = [&]() -> int {
    HIPCHK(e, hipStreamSynchronize(st), "sync hist");
    const auto t_hist = std::chrono::steady_clock::now();
    const uint32_t* hv = e->h_hist.as<uint32_t>();
    klf::DataStats ds;
    ds.bytes.assign(256, 0);
    for (int c = 0; c < 256; ++c) {
      ds.bytes[c] = hv[c];
      ds.nbytes += ds.bytes[c];
    }
    ds.pair.assign(hv + klf::kGramHistPairs, hv + klf::kGramHistPairs + 65536);
    for (auto& c : ds.pair) c *= 2;  // counted at every 2nd position
    klf::stats_finish(ds);
    if (ds.nbytes) est_density = (double)(ds.bytes['\n'] + 1) / (double)ds.nbytes;
    klf::place_needles(e->cs, &ds);
    const auto t_place = std::chrono::steady_clock::now();
    if (getenv("KLF_DIAG"))
      fprintf(stderr, "[klf] prefilter layout from %llu sampled bytes: %s\n", (unsigned long long)ds.nbytes,
              e->cs.qf_layout.c_str());
    HIPCHK(e, upload_prefilter(e), "upload prefilter tables");
    if (getenv("KLF_DIAG"))
      fprintf(stderr, "[klf] first-batch tuning: statistics %.1f us (with the workspace mapped meanwhile), layout %.1f us, uploads %.1f us\n",
              std::chrono::duration<double, std::micro>(t_hist - t_tune0).count(),
              std::chrono::duration<double, std::micro>(t_place - t_hist).count(),
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_place).count());
    tune_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_tune0).count();
    mark("first-batch tuning");
    return KLF_OK;
  };
  std::vector<std::pair<DevBuf*, size_t>> ws = {
      {&e->d_tstat, ntiles * sizeof(klf::TileStat)},
      {&e->d_tile_base, ntiles * 8}, {&e->d_bsum, (ntiles / 1024 + 2) * 4 * 8},
      {&e->d_counters, kCtrBytes + nsegs * sizeof(SegOut)} /* + the stream records */,
      {&e->d_wpre, (3 * (size_t)nsegs + 2) * 8} /* + wgrp */};
  // the dense compaction's per-tile run table (512 B per tile: 2.1 GB for 32 GiB) only for
  // runs without a --tail limit or after a --tail run took the dense path (k_tcopy lists
  // the runs itself without it)
  const bool want_truns = f->tail < 0 || e->dense_tail_seen;
  if (want_truns) ws.push_back({&e->d_truns, ntiles * klf::kRunSlots * 4});
  uint32_t compact_mode = 0;  // tests: force either compaction path
  if (const char* v = getenv("KLF_COMPACT")) compact_mode = !strcmp(v, "sparse") ? 1u : !strcmp(v, "dense") ? 2u : 0u;
  // A --tail run selects at most S (N + 1) lines: up to 2^20 of them the line gather is the
  // path (round 6; it copies any selection, long lines spread over copy chunks), so the tile
  // copy's per-tile tables (32 B per tile: 134 MB for 32 GiB) are neither mapped nor walked
  else if (f->tail >= 0 && (uint64_t)nsegs * ((uint64_t)f->tail + 1) <= (1ull << 20)) compact_mode = 1;
  if (compact_mode != 1) {
    ws.push_back({&e->d_trec, ntiles * sizeof(klf::TRec)});
    ws.push_back({&e->d_kbase, ntiles * 16});
  }
  // One-pass compaction (no patterns, --tail -1): the fused scan compacts each wave's tile
  // range in place.  The ranges (a multiple of kScanGroup tiles each, one per wave of a
  // full-occupancy launch) and each range's first extent (one extent per stream it touches).
  const bool fuse_try = mode == klf::CompiledSet::kNone && f->tail < 0 && compact_mode == 0 &&
                        !(getenv("KLF_FUSE") && !strcmp(getenv("KLF_FUSE"), "0"));
  bool fuse_ok = fuse_try;
  uint64_t seg_end = 0;  // past the last input byte (the fused output is laid out like the input)
  for (const auto& d : segs) seg_end = std::max<uint64_t>(seg_end, d.base + d.len);
  auto seg_of_tile = [&](uint64_t t) -> uint32_t {
    uint32_t lo = 0, hi = nsegs;  // the last segment whose tile0 <= t
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (segs[mid].tile0 <= t) lo = mid; else hi = mid;
    }
    return lo;
  };
  if (fuse_try) {
    const uint64_t waves = (uint64_t)std::max(1, klf::fuse_waves(e->num_cus));
    uint64_t R = (ntiles + waves - 1) / waves;
    R = (R + klf::kScanGroup - 1) / klf::kScanGroup * klf::kScanGroup;
    if (const char* v = getenv("KLF_DEBUG_FUSE_RANGE"))  // tests: short ranges (many range seams)
      R = std::max<uint64_t>(klf::kScanGroup, (uint64_t)atol(v) / klf::kScanGroup * klf::kScanGroup);
    const uint32_t nr = (uint32_t)((ntiles + R - 1) / R);
    const bool same_fuse_layout = segs.size() == e->fuse_segs.size() &&
                                  memcmp(segs.data(), e->fuse_segs.data(), segs.size() * sizeof(SegDesc)) == 0;
    if (!same_fuse_layout || e->fuse_range != (uint32_t)R || e->fuse_nranges != nr) {
      e->fuse_segs.clear();  // (invalid until the table below is on its way)
      e->fuse_ext0.assign(nr + 1, 0);
      for (uint32_t q = 0; q < nr; ++q) {
        const uint64_t t0 = (uint64_t)q * R, t1 = std::min<uint64_t>(t0 + R, ntiles) - 1;
        e->fuse_ext0[q + 1] = e->fuse_ext0[q] + (seg_of_tile(t1) - seg_of_tile(t0) + 1);
      }
      HIPCHK(e, e->d_fext0.ensure((nr + 1) * 4), "alloc fuse ranges");
      HIPCHK(e, hipMemcpyAsync(e->d_fext0.p, e->fuse_ext0.data(), (nr + 1) * 4, hipMemcpyHostToDevice, st),
             "H2D fuse ranges");
      e->fuse_range = (uint32_t)R;
      e->fuse_nranges = nr;
      e->fuse_next = e->fuse_ext0[nr];
      e->fuse_segs = segs;
    }
    HIPCHK(e, e->d_fext.ensure((size_t)e->fuse_next * 16), "alloc fuse extents");
    HIPCHK(e, e->d_frinfo.ensure((size_t)e->fuse_nranges * 32), "alloc fuse range states");
  }
  e->index_pending.clear();
  // lazy line index (grep none, --tail -1; KLF_LAZY_INDEX=0 turns it off)
  const bool full_index = (f->flags & KLF_FILTER_FULL_INDEX) != 0;
  // KLF_FILTER_NO_TIMING: no event in the launch sequence (launch_pipeline records none)
  hipEvent_t* const evs = (f->flags & KLF_FILTER_NO_TIMING) ? nullptr : e->ev;
  const bool lazy_index = mode == klf::CompiledSet::kNone && f->tail < 0 && !full_index &&
                          !(getenv("KLF_LAZY_INDEX") && !strcmp(getenv("KLF_LAZY_INDEX"), "0"));
  // (a run that needs every line's index -- k_match's fallback -- turns it off)
  bool win_ok = !full_index;
  // The output buffer: sized for the whole input up front when the run keeps about as much
  // as it reads (no --tail limit: C3-like), else grown
  // on demand -- the compaction skips a copy that would not fit, the host grows the buffer
  // to the run's output and reruns the tail stage (first runs only: the buffer is kept).
  // A --tail run then never maps an input-sized buffer (34 GB for C4 / C5).
  uint64_t out_need = 0;  // the output buffer (mapped below, with a first run's line arrays)
  if (f->tail < 0) out_need = std::max<uint64_t>(total_bytes, fuse_try ? seg_end : 0) + 64;
  else if (!e->d_out.p) {  // a first --tail run: room for a typical tail window (no rerun to grow)
    uint64_t first = 64ull << 20;
    if (const char* v = getenv("KLF_DEBUG_OUT_INIT")) first = (uint64_t)std::max(1L, atol(v));  // tests: force growth
    out_need = std::min<uint64_t>(total_bytes + 64, first);
  }
  const bool need_cand = mode == klf::CompiledSet::kGeneral && e->cs.qf_on && e->cs.rx_count;
  if (need_cand) ws.push_back({&e->d_cand, (size_t)e->cand_cap * 16});
  const bool need_hits = mode == klf::CompiledSet::kGeneral && e->cs.qf_on;
  // bitmap hits: < 1 per 8 KiB tile on log text (C4's 1,024 literals: 0.41, C5 0.02),
  // kHitSlots per tile recorded in place; spills beyond 1 per 8 KiB of input -> k_match decides
  const uint32_t qhits_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(total_bytes / 8192, 1u << 16),
                                                          e->hits_cap_max);
  // flattened hit slots: up to 1 per 4 KiB of input (2 per tile); more -> k_match decides
  // (round 5 mapped 1 per 512 B: 537 MB for 32 GiB, in every first run's workspace)
  const uint64_t hflat_cap = std::min<uint64_t>(std::max<uint64_t>(total_bytes / 4096, 1u << 20),
                                                (uint64_t)ntiles * klf::kHitSlots);
  if (need_hits) {
    ws.push_back({&e->d_qhits, (size_t)qhits_cap * 8});
    ws.push_back({&e->d_hslots, (size_t)ntiles * klf::kHitSlots * 2});
    ws.push_back({&e->d_hflat, (size_t)hflat_cap * 8});
  }
  HIPCHK(e, ensure_all(e->d_block, e->block_users, ws), "alloc workspace");

  const bool count = (f->flags & KLF_FILTER_PATTERN_COUNTS) && mode == klf::CompiledSet::kGeneral && e->cs.n_cids;
  r->counted = (f->flags & KLF_FILTER_PATTERN_COUNTS) != 0;
  mark("workspace");
  if (tune_pending) {
    const int rc = finish_tune();
    if (rc != KLF_OK) return rc;
  }
  if (nl_pending) {
    HIPCHK(e, hipStreamSynchronize(st), "sync line sample");
    const uint32_t* hv = e->h_hist.as<uint32_t>();
    uint64_t nl = 0, nb = 0;
    for (uint32_t b = 0; b < nl_blocks; ++b) { nl += hv[2 * b]; nb += hv[2 * b + 1]; }
    if (nb) est_density = (double)(nl + nl_blocks) / (double)nb;  // (+1 per tile: a margin, never 0)
    if (const char* v = getenv("KLF_DEBUG_NL_SCALE")) est_density *= atof(v);  // tests: force an underestimate
    mark("line sample");
  }
  // a first run with the sample's line density: the line arrays from it (x2 + a margin:
  // an overflow reruns with exact sizes), in one launch phase
  const bool density_cap = e->line_density == 0.0 && est_density > 0.0 && !getenv("KLF_TWO_PHASE");
  // Where the scan keeps the slots of tiles with two or more line starts (round 6): long lines
  // (under one per KiB: C5) -> per-wave chunks of the pool, no record regions allocated at all
  // (C5 k_scan -1.4 %, cold 8.6 -> 8.3 ms); shorter lines -> the per-tile record regions,
  // 1,152 B per tile, written as whole lines (C2 / C3 / C4 ran 0.7-1.5 % faster on them,
  // r6g).  KLF_WAVE_POOL=1 / 0 forces either.
  const double dens = e->line_density > 0.0 ? e->line_density : est_density;
  const char* wpv = getenv("KLF_WAVE_POOL");
  const bool wave_pool = wpv ? strcmp(wpv, "0") != 0 : (dens > 0.0 && dens * 1024.0 < 1.0);
  if (density_cap)
    cap = std::min<uint64_t>(cap, (uint64_t)(est_density * (double)total_bytes * 2.0) + 2ull * nsegs + 65536);
  // the buffers indexed by global line (and the compaction's per-block tables) for capacity c
  auto line_sizes = [&](uint64_t c) {
    const uint64_t mcb = c / klf::kCompactLines + 2;
    // >= sum over blocks of ceil(bytes / chunk) (>= 1 each): the block prefix's chunk keeps
    // the output within kCopyChunksTarget chunks unless it is the largest, kCopyChunk
    const uint64_t cmc = mcb + std::max<uint64_t>(total_bytes / klf::kCopyChunk, klf::kCopyChunksTarget) + 2;
    return std::vector<std::pair<DevBuf*, size_t>>{
        {&e->d_line_off, (c + nsegs + 1) * 8}, {&e->d_meta, c * 2 + 16}, {&e->d_bits, (c / 32 + 1) * 4},
        {&e->d_cstatus, (mcb + 1) * 3 * 8}, {&e->d_cmap, cmc * 4}, {&e->d_cseg, (mcb + 1) * 4},
        {&e->d_mpart, (c / klf::kMatchChunk + 2) * 8}};
  };
  auto pool_need = [&](uint64_t c, uint32_t& chunk) -> uint64_t {  // the slot pool (wave_pool: see the scan)
    chunk = 256;
    if (!wave_pool) return e->pool_cap;
    const uint64_t nwaves = (uint64_t)e->num_cus * 16;
    const uint64_t per_wave = (c + 2 * ntiles) / nwaves;
    while (chunk < 4096 && chunk * 4 < per_wave) chunk *= 2;
    return std::max<uint64_t>(e->pool_cap, c + 3 * ntiles + nwaves * chunk + 1024);
  };
  {
    // A first run maps its line arrays, slot pool / records and output buffer as one more
    // allocation, now that their sizes are known (each hipMalloc costs 1-26 us of host time
    // with the GPU idle: ~10 of them per first run); later runs grow single buffers
    std::vector<std::pair<DevBuf*, size_t>> ws2;
    if (out_need) ws2.push_back({&e->d_out, out_need});
    if (!wave_pool) ws2.push_back({&e->d_slots, ntiles * klf::kRecStride * 4});
    if (e->line_density == 0.0) {
      for (auto& x : line_sizes(cap)) ws2.push_back(x);
      uint32_t ch = 0;
      ws2.push_back({&e->d_pool, pool_need(cap, ch) * 4});
    }
    HIPCHK(e, ensure_all(e->d_block2, e->block2_users, ws2), "alloc line arrays / output");
    mark("line arrays / output");
  }
  uint32_t pool_chunk = 256;  // (per attempt, below: the wave pool's chunk size)
  bool force_match = false;   // an overflowed hit list / NFA queue: redo the run with k_match
  // every RunArgs field but the line arrays (alloc_lines) of a run over the whole batch
  auto fill_args = [&](klf::RunArgs& a, int attempt) {
    memset(static_cast<void*>(&a), 0, sizeof(a));
    a.bytes = d_bytes;
    a.segs = e->d_segs.as<SegDesc>();
    a.nsegs = nsegs;
    a.ntiles = (uint32_t)ntiles;
    a.tile_seg = e->d_tile_seg.as<uint32_t>();
    a.build_tiles = (!same_layout && attempt == 0) ? 1u : 0u;
    // tests: KLF_DEBUG_TINDEX_WIDE=1 runs the large-batch tile index on any batch
    a.tindex_wide = (ntiles > klf::kScanSmallTiles || getenv("KLF_DEBUG_TINDEX_WIDE")) ? 1u : 0u;
    a.since_sec = f->since.sec;
    a.since_nsec = f->since.nsec;
    since_digits(f->since.sec, f->since.nsec, a.since_dig);
    a.tail = f->tail;
    a.grep_mode = (uint32_t)mode;
    a.match_all = e->cs.also_all ? 1u : 0u;
    a.lit = e->d_lit.as<uint8_t>();
    a.lit_len = (uint32_t)e->cs.literal.size();
    a.lit_anchor = e->cs.literal_anchor;
    a.lit_anchor_byte = e->cs.literal.empty() ? 0u : e->cs.literal[e->cs.literal_anchor];
    a.lit_words = e->d_lit.as<uint32_t>();
    memcpy(static_cast<void*>(&a.pats), &e->dpats, sizeof(a.pats));
    a.tstat = e->d_tstat.as<klf::TileStat>();
    a.slots = wave_pool ? nullptr : e->d_slots.as<uint32_t>();
    a.pool = e->d_pool.as<uint32_t>();
    a.pool_cap = e->pool_cap;
    a.wave_pool = wave_pool ? 1u : 0u;
    a.pool_chunk = pool_chunk;
    a.tile_base = e->d_tile_base.as<uint64_t>();
    a.bsum = e->d_bsum.as<uint64_t>();
    a.counters = e->d_counters.as<uint32_t>();
    a.segout = segout_of(e);
    a.wpre = e->d_wpre.as<uint64_t>();
    a.wgrp = a.wpre + nsegs + 1;
    a.out = e->d_out.as<uint8_t>();
    a.out_cap = e->d_out.p ? e->d_out.cap : 0;
    a.stage_times = (f->flags & KLF_FILTER_STAGE_TIMES) && evs ? 1u : 0u;
    a.cand = need_cand ? e->d_cand.as<uint64_t>() : nullptr;
    a.cand_cap = need_cand ? e->cand_cap : 0;
    a.qhits = need_hits ? e->d_qhits.as<uint64_t>() : nullptr;
    a.hslots = need_hits ? e->d_hslots.as<uint16_t>() : nullptr;
    a.hflat = need_hits ? e->d_hflat.as<uint64_t>() : nullptr;
    a.hflat_cap = need_hits ? hflat_cap : 0;
    a.qhits_cap = need_hits ? qhits_cap : 0;
    a.trec = e->d_trec.as<klf::TRec>();
    a.truns = want_truns ? e->d_truns.as<uint32_t>() : nullptr;
    a.kbase = e->d_kbase.as<uint64_t>();
    a.compact_mode = compact_mode;
    a.lazy_index = lazy_index ? 1u : 0u;
    a.plan_runs = (lazy_index && want_truns && compact_mode != 1 &&
                   !(getenv("KLF_PLAN_RUNS") && !strcmp(getenv("KLF_PLAN_RUNS"), "0"))) ? 1u : 0u;
    // windowed line index: literal patterns, and (round 6) prefiltered regex sets, whose
    // candidate lines get their bounds from k_verify; per-pattern counts too (k_fixcount's
    // deferred lines, like k_match's fallback, ask for a rerun with the whole index)
    const bool win_rx = !(getenv("KLF_WIN_INDEX_RX") && !strcmp(getenv("KLF_WIN_INDEX_RX"), "0"));
    a.win_index = (win_ok &&
                   (mode == klf::CompiledSet::kLiteral1 ||
                    (mode == klf::CompiledSet::kGeneral && e->cs.qf_on && !e->cs.also_all &&
                     ((e->cs.rx_count == 0 && !count) || win_rx))) &&
                   !(getenv("KLF_WIN_INDEX") && !strcmp(getenv("KLF_WIN_INDEX"), "0"))) ? 1u : 0u;
    a.scatter_mode = 0;
    // no launch of kernels that would exit at once (each costs ~4 us plus its boundary):
    // k_match beside a working prefilter, k_tcopy in a --tail run before any went dense
    a.skip_match = (mode == klf::CompiledSet::kGeneral && e->cs.qf_on && !e->cs.also_all && !force_match &&
                    !(getenv("KLF_SKIP_IDLE") && !strcmp(getenv("KLF_SKIP_IDLE"), "0"))) ? 1u : 0u;
    a.skip_tcopy = (f->tail >= 0 && !e->dense_tail_seen && compact_mode == 0 &&
                    !(getenv("KLF_SKIP_IDLE") && !strcmp(getenv("KLF_SKIP_IDLE"), "0"))) ? 1u : 0u;
    // waves per scatter group (0: k_scatter picks it from its grid; tests force a split)
    a.scatter_split = getenv("KLF_SCATTER_SPLIT") ? (uint32_t)std::max(0L, atol(getenv("KLF_SCATTER_SPLIT"))) : 0u;
    // a --tail run's sparse gather with fewer launches (RunArgs::plan_mode), without patterns
    // (a window of at most S (N + 1) lines, the line index built before k_tailw): k_tailw
    // plans a window of at most 4 compaction blocks itself (C1: k_tailw +4.7 us for k_cplan
    // 4.8 + k_cmid 5.0), else k_cplan's last block runs the prefix (7.5 us).  A grep run's
    // window spans every line between its N + 1 matches: its block sums need k_cplan's
    // whole grid (C5 with the prefix in k_cplan's last block: 15.9 -> 24.1 us, r6t).
    // (KLF_PLAN_MODE=0 / 1 / 2 forces one, tests)
    a.plan_mode = 0;
    if (compact_mode == 1 && f->tail >= 0 && (mode == klf::CompiledSet::kNone || getenv("KLF_PLAN_MODE"))) {
      const bool index_first = !a.win_index && !lazy_index;
      a.plan_mode = index_first && mode == klf::CompiledSet::kNone &&
                    (uint64_t)nsegs * ((uint64_t)f->tail + 1) <= 4ull * klf::kCompactLines ? 2u : 1u;
      if (const char* v = getenv("KLF_PLAN_MODE")) a.plan_mode = std::min<uint32_t>((uint32_t)atoi(v), index_first ? 2u : 1u);
    }
    a.count_pats = count ? 1u : 0u;
    a.pcount = count ? e->d_pcount.as<uint32_t>() : nullptr;
    a.pairs = count ? e->d_pairs.as<uint64_t>() : nullptr;
    a.pairs_log2 = e->pairs_log2;
    if (fuse_ok) {
      a.fuse = 1;
      a.plan_runs = 0;
      a.fuse_range = e->fuse_range;
      a.fuse_nranges = e->fuse_nranges;
      a.fuse_ext0 = e->d_fext0.as<uint32_t>();
      a.fuse_ext = e->d_fext.as<uint64_t>();
      a.fuse_rinfo = e->d_frinfo.as<uint64_t>();
    }
  };
  bool overflow = false, pairs_over = false;
  uint32_t ev_mask = 0;
  const bool graph_on = getenv("KLF_GRAPH") && strcmp(getenv("KLF_GRAPH"), "0") != 0;  // (opt-in)
  const uint64_t graph_max = (getenv("KLF_GRAPH_MAX_MB") ? (uint64_t)std::max(0L, atol(getenv("KLF_GRAPH_MAX_MB"))) : 256ull) << 20;
  for (int attempt = 0, line_reruns = 0, pair_reruns = 0; attempt < 4; ++attempt) {
    if (count) {
      HIPCHK(e, e->d_pcount.ensure((size_t)nsegs * e->cs.n_cids * 4), "alloc pcount");
      HIPCHK(e, e->d_pairs.ensure((size_t)8 << e->pairs_log2), "alloc pairs");
      HIPCHK(e, hipMemsetAsync(e->d_pcount.p, 0, (size_t)nsegs * e->cs.n_cids * 4, st), "zero pcount");
      HIPCHK(e, hipMemsetAsync(e->d_pairs.p, 0, (size_t)8 << e->pairs_log2, st), "zero pairs");
    }
    // An engine's first run sizes its line arrays from its own line count: the pipeline
    // runs up to the tile index, the count is read back, the arrays are allocated, the
    // rest follows (one extra sync, first runs only).
    const bool two_phase = attempt == 0 && e->line_density == 0.0 && !density_cap && !small_first && !getenv("KLF_ONE_PHASE");
    // the arrays indexed by global line (and the compaction's per-block tables)
    auto alloc_lines = [&](klf::RunArgs& x, uint64_t c) -> hipError_t {
      const uint64_t mcb = c / klf::kCompactLines + 2;
      const uint64_t cmc = mcb + std::max<uint64_t>(total_bytes / klf::kCopyChunk, klf::kCopyChunksTarget) + 2;
      hipError_t h;
      for (auto& q : line_sizes(c))
        if ((h = q.first->ensure(q.second)) != hipSuccess) return h;
      x.line_off = e->d_line_off.as<uint64_t>();
      x.meta = e->d_meta.as<uint16_t>();
      x.bits = e->d_bits.as<uint32_t>();
      x.csum = e->d_cstatus.as<uint64_t>();
      x.cmap = e->d_cmap.as<uint32_t>();
      x.cmap_cap = cmc;
      x.cseg = e->d_cseg.as<uint32_t>();
      x.mpart = e->d_mpart.as<uint64_t>();
      x.cap_lines = c;
      x.max_cblocks = (uint32_t)mcb;
      return hipSuccess;
    };
    // the pool: every tile where two or more lines start (16-B aligned: <= 3 spare slots each),
    // dense tiles, and the waves' partly used last chunks (wave_pool); an overflow reruns
    // with the count the scan reserved
    e->pool_cap = pool_need(cap, pool_chunk);
    if (e->pool_cap >= (1ull << 31)) return set_err(e, KLF_EINVAL, "batch too large (line slot pool)");
    HIPCHK(e, e->d_pool.ensure(e->pool_cap * 4), "alloc pool");
    klf::RunArgs a;
    fill_args(a, attempt);
    if (attempt == 0 && getenv("KLF_DEBUG_POOL_CAP"))  // tests: a first attempt whose pool overflows
      a.pool_cap = std::min<uint64_t>(a.pool_cap, (uint64_t)std::max(1L, atol(getenv("KLF_DEBUG_POOL_CAP"))));
    ev_mask = 0;  // the events this attempt records (the timing queries read only those)
    r->so.resize(nsegs);
    uint32_t counters[32];
    // (+ a one-pass run's extents, read back with the counters: one sync on e->stream)
    const size_t rb_ext = fuse_ok ? (size_t)e->fuse_next * 16 : 0;
    HIPCHK(e, e->h_rb.ensure(kCtrBytes + nsegs * sizeof(SegOut) + rb_ext), "alloc readback");
    // the literal automaton (klf_open's thread) is read from k_tindex on (deferred lines)
    auto join_ac = [&]() -> int {
      if (const int rc = ensure_ac(e); rc != KLF_OK) return rc;
      memcpy(static_cast<void*>(&a.pats), &e->dpats, sizeof(a.pats));
      mark("automaton");
      return KLF_OK;
    };
    if (two_phase) {
      if (const int rc = join_ac(); rc != KLF_OK) return rc;
      a.cap_lines = 1ull << 40;  // phase 1 indexes no line array (k_tindex: no overflow, no bitmap)
      HIPCHK(e, klf::launch_pipeline(a, st, evs, e->num_cus, 1, &ev_mask), "launch");
      uint8_t* rb1 = e->h_rb.as<uint8_t>();
      HIPCHK(e, hipMemcpyAsync(rb1, e->d_counters.p, kCtrBytes + nsegs * sizeof(SegOut), hipMemcpyDeviceToHost, st),
             "D2H counters + records");
      HIPCHK(e, hipStreamSynchronize(st), "sync phase 1");
      mark("phase 1 (launch + sync)");
      memcpy(counters, rb1, sizeof(counters));
      memcpy(r->so.data(), rb1 + kCtrBytes, nsegs * sizeof(SegOut));
      if (counters[2]) {  // the dense-tile pool overflowed: a whole rerun (as below)
        e->pool_cap = std::max<uint64_t>(e->pool_cap, (uint64_t)counters[klf::kCtrPool] + (uint64_t)e->num_cus * 16 * 4096);
        e->line_density = (double)(r->so[nsegs - 1].line_hi + 1) / (double)total_bytes;
        cap = std::min<uint64_t>(cap, r->so[nsegs - 1].line_hi + 2);
        continue;
      }
      // the same margin later runs size by (their line density estimate), so that they fit
      e->line_density = (double)(r->so[nsegs - 1].line_hi + 1) / (double)total_bytes;
      // phase 1 knows the exact line count: size the arrays to it (the 32-B estimate is
      // short for lines under 32 B); a capacity still below it (only KLF_DEBUG_CAP_CLAMP)
      // fails here, before phase 2's kernels index the arrays (advisor r03)
      const uint64_t need = r->so[nsegs - 1].line_hi + 2;
      cap = std::min<uint64_t>(std::max<uint64_t>(std::min<uint64_t>(cap, learned_cap()), need), cap_clamp);
      if (need > cap) {
        overflow = true;
        break;
      }
      HIPCHK(e, alloc_lines(a, cap), "alloc line arrays");
      mark("line arrays");
      if (a.grep_mode != klf::CompiledSet::kNone)  // (phase 1's k_tindex zeroes it otherwise)
        HIPCHK(e, hipMemsetAsync(a.bits, 0, (cap / 32 + 1) * 4, st), "zero bits");
      HIPCHK(e, klf::launch_pipeline(a, st, evs, e->num_cus, 2, &ev_mask), "launch");
      mark("phase 2 launched");
    } else if (e->ac_pending) {  // joined while the scan runs
      HIPCHK(e, alloc_lines(a, cap), "alloc line arrays");
      HIPCHK(e, klf::launch_pipeline(a, st, evs, e->num_cus, 3, &ev_mask), "launch");
      if (const int rc = join_ac(); rc != KLF_OK) return rc;
      HIPCHK(e, klf::launch_pipeline(a, st, evs, e->num_cus, 4, &ev_mask), "launch");
    } else {
      HIPCHK(e, alloc_lines(a, cap), "alloc line arrays");
      mark("line arrays");
      // KLF_GRAPH=1: a small batch (KLF_GRAPH_MAX_MB, default 256) replays a graph
      const bool graph = !e->graph_off && !a.stage_times && total_bytes <= graph_max && graph_on;
      if (!(graph && launch_graph(e, a, ev_mask)))
        HIPCHK(e, klf::launch_pipeline(a, st, evs, e->num_cus, 0, &ev_mask), "launch");
    }
    mark("launched");
    uint8_t* rb = e->h_rb.as<uint8_t>();
    HIPCHK(e, hipMemcpyAsync(rb, e->d_counters.p, kCtrBytes + nsegs * sizeof(SegOut), hipMemcpyDeviceToHost, st),
           "D2H counters + records");
    if (a.fuse)
      HIPCHK(e, hipMemcpyAsync(rb + kCtrBytes + nsegs * sizeof(SegOut), e->d_fext.p, rb_ext,
                               hipMemcpyDeviceToHost, st), "D2H extents");
    HIPCHK(e, wait_stream(st, 1000 + total_bytes / 2000000), "sync");
    mark("pipeline done");
    memcpy(counters, rb, sizeof(counters));
    memcpy(r->so.data(), rb + kCtrBytes, nsegs * sizeof(SegOut));
    e->last_segs = segs;
    if (getenv("KLF_DIAG"))
      fprintf(stderr, "[klf] hits=%u spilled=%u hits_over=%u nfa_queue=%u queue_over=%u deferred=%u\n",
              counters[klf::kCtrVerified], counters[klf::kCtrHits], counters[klf::kCtrHitsOver],
              counters[klf::kCtrQueue], counters[klf::kCtrQOver], counters[5]);
    overflow = (counters[2] & 1u) != 0;
    if (overflow) {  // more lines (or dense-tile slots) than estimated: rerun with exact sizes
      if (line_reruns++) break;
      cap = std::min(std::max<uint64_t>(cap, r->so[nsegs - 1].line_hi + 2), cap_clamp);
      e->pool_cap = std::max<uint64_t>(e->pool_cap, (uint64_t)counters[klf::kCtrPool] + (uint64_t)e->num_cus * 16 * 4096);
      continue;
    }
    if (a.skip_match && (counters[klf::kCtrQOver] || counters[klf::kCtrHitsOver])) {  // k_match decides: redo with it
      force_match = true;
      continue;
    }
    if (a.skip_tcopy && counters[klf::kCtrDense]) {  // the dense path without its copy: launch it now
      uint32_t* rb1 = e->h_rb.as<uint32_t>();
      HIPCHK(e, klf::launch_tcopy(a, st, nullptr, e->num_cus, nullptr), "launch tile copy");
      HIPCHK(e, hipMemcpyAsync(rb1, e->d_counters.p, sizeof(counters), hipMemcpyDeviceToHost, st), "D2H counters");
      HIPCHK(e, hipStreamSynchronize(st), "sync tile copy");
      counters[klf::kCtrOutShort] = rb1[klf::kCtrOutShort];
      a.skip_tcopy = 0;  // (klf_retail from this run launches it)
    }
    if (a.fuse && counters[klf::kCtrFuseBad]) {  // a deferred line or a dense tile: the two-pass rerun
      fuse_ok = false;
      continue;
    }
    if (a.win_index && counters[klf::kCtrRedo]) {  // k_match needed the whole index: rerun with it
      win_ok = false;
      continue;
    }
    pairs_over = count && counters[klf::kCtrPairsOver] != 0;
    if (pairs_over && pair_reruns < 2 && e->pairs_log2 < 28) {  // the pair set filled: a larger one
      // distinct pairs <= the set's capacity + the failed inserts; size for load <= 1/2
      ++pair_reruns;
      const uint64_t need = 2 * (((uint64_t)1 << e->pairs_log2) + counters[klf::kCtrPairsOver]);
      uint32_t lg = e->pairs_log2 + 1;
      while (lg < 28 && ((uint64_t)1 << lg) < need) ++lg;
      e->pairs_log2 = lg;
      continue;
    }
    if (counters[klf::kCtrOutShort]) {  // the output did not fit: grow, rerun the tail stage
      HIPCHK(e, grow_out_retail(e, a, r->so), "grow output");
      if (getenv("KLF_DIAG")) fprintf(stderr, "[klf] output buffer grown to %zu B\n", e->d_out.cap);
    }
    if (a.fuse) {  // the extents, in stream order (ranges ascend, and so do a range's streams)
      r->fused = true;
      r->fx.resize((size_t)e->fuse_next * 2);
      memcpy(r->fx.data(), rb + kCtrBytes + nsegs * sizeof(SegOut), (size_t)e->fuse_next * 16);
      r->fx_first.assign(nsegs + 1, e->fuse_next);
      for (uint32_t q = e->fuse_nranges; q-- > 0;) {
        const uint32_t s0 = seg_of_tile((uint64_t)q * e->fuse_range);
        for (uint32_t k = e->fuse_ext0[q]; k < e->fuse_ext0[q + 1]; ++k) r->fx_first[s0 + (k - e->fuse_ext0[q])] = k;
      }
      uint64_t acc = 0;
      for (uint32_t sg = 0; sg < nsegs; ++sg) {
        r->so[sg].sel_lo = 0;  // --tail -1, no patterns: every parsed line since the cutoff
        r->so[sg].sel_hi = r->so[sg].since_ok;
        r->so[sg].out_lo = acc;
        for (uint32_t k = r->fx_first[sg]; k < r->fx_first[sg + 1]; ++k) acc += r->fx[2 * (size_t)k + 1];
        r->so[sg].out_hi = acc;
      }
    }
    e->last_args = a;
    const bool on_demand = a.lazy_index && (counters[klf::kCtrDense] || a.fuse);
    if (on_demand || a.win_index) e->index_pending.push_back(a);
    r->index_mode = on_demand ? KLF_INDEX_ON_DEMAND : a.win_index ? KLF_INDEX_WINDOWS : KLF_INDEX_FULL;
    r->compaction = a.fuse ? KLF_COMPACT_ONEPASS : counters[klf::kCtrDense] ? KLF_COMPACT_TILES : KLF_COMPACT_GATHER;
    e->last_gen = r->gen;
    e->line_density = (double)(r->so[nsegs - 1].line_hi + 1) / (double)total_bytes;
    if (f->tail >= 0 && counters[klf::kCtrDense]) e->dense_tail_seen = true;
    break;
  }
  if (count && !overflow && !pairs_over) {
    r->pcount.resize((size_t)nsegs * e->cs.n_cids);
    HIPCHK(e, hipMemcpy(r->pcount.data(), e->d_pcount.p, r->pcount.size() * 4, hipMemcpyDeviceToHost), "D2H pcount");
    r->pcount_ok = true;
  }
  if (getenv("KLF_DIAG")) {
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_run0).count();
    fprintf(stderr, "[klf] run %.1f us: allocations %.1f us, first-batch tuning %.1f us\n", us,
            (g_alloc_ns.load() - alloc0) / 1e3, tune_ns / 1e3);
    std::string m = "[klf] run marks (us):";
    auto prev = t_run0;
    for (auto& x : marks) {
      m += std::string(" ") + x.first + " " + std::to_string((int)std::chrono::duration<double, std::micro>(x.second - prev).count()) + ";";
      prev = x.second;
    }
    fprintf(stderr, "%s\n", m.c_str());
  }
  if (overflow)  // the exact rerun overflowed too: never hand out the aborted run's records
    return set_err(e, KLF_ENOMEM, "line index / dense-tile pool overflow after the exact rerun");
  if (const char* path = getenv("KLF_TIMELINE_OUT")) {  // diagnostic builds only
    std::vector<uint64_t> tl(300000 * 8);
    if (klf::dump_timeline(tl.data(), tl.size() * 8) == hipSuccess) {
      if (FILE* f = fopen(path, "wb")) {
        fwrite(tl.data(), 8, std::min<size_t>(tl.size(), ntiles * 8), f);
        fclose(f);
      }
      (void)klf::clear_timeline();
    }
  }
  // only the event pairs this run recorded (ev_mask): a pair it did not record would fail
  // the query (or time an earlier run).  Timing is diagnostic: a recorded pair that fails to
  // read leaves -1 in its slot (KLF_DIAG says so) and the filter result stands.
  auto elapsed = [&](int k0, int k1, int slot) {
    if (!((ev_mask >> k0 & 1u) && (ev_mask >> k1 & 1u))) return;
    float ms = 0.f;
    const hipError_t h = hipEventElapsedTime(&ms, e->ev[k0], e->ev[k1]);
    if (h == hipSuccess) {
      r->ms[slot] = ms;
      return;
    }
    (void)hipGetLastError();  // (the failed query's error is not the next call's)
    r->ms[slot] = -1.0;
    if (getenv("KLF_DIAG"))
      fprintf(stderr, "[klf] timing events %d/%d unreadable: %s\n", k0, k1, hipGetErrorString(h));
  };
  static const int kPairs[6][3] = {{1, 2, 0}, {2, 3, 1}, {3, 4, 2}, {4, 5, 3}, {0, 5, 4}, {0, 1, 5}};
  const auto t_q0 = std::chrono::steady_clock::now();
  for (const auto& q : kPairs) elapsed(q[0], q[1], q[2]);
  elapsed(7, 8, 6);   // k_scan's dispatch alone
  elapsed(9, 10, 7);  // k_tcopy's dispatch alone (dense copy)
  if (diag_marks)
    fprintf(stderr, "[klf] timing queries %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_q0).count());
  r->ev_mask = ev_mask;
  r->total_lines = r->so[nsegs - 1].line_hi;
  for (auto& s : r->so) r->total_out = std::max(r->total_out, s.out_hi);
  *out = rp.release();
  return KLF_OK;
}

extern "C" int klf_run_device(klf_engine* e, const uint8_t* d_bytes, uint32_t n, const uint64_t* seg_base,
                              const uint64_t* lens, const klf_filter* f, klf_result** out) {
  return run_device_impl(e, d_bytes, n, seg_base, lens, f, out);
}

static int ensure_index(klf_engine* e);

extern "C" int klf_retail(klf_engine* e, klf_result* prev, int64_t tail, klf_result** out) {
  if (!e || !prev || !out || prev->e != e || tail < -1) return KLF_EINVAL;
  *out = nullptr;
  if (prev->gen != e->gen || e->last_gen != prev->gen) return set_err(e, KLF_ESTATE, "klf_retail: not the latest run");
  if (int rc = ensure_index(e)) return rc;
  HIPCHK(e, hipSetDevice(e->device), "hipSetDevice");
  auto* r = new (std::nothrow) klf_result();
  if (!r) return KLF_ENOMEM;
  r->e = e;
  r->n_streams = prev->n_streams;
  r->seg_of = prev->seg_of;
  r->seg_base = prev->seg_base;
  r->has_bits = prev->has_bits;
  r->total_lines = prev->total_lines;
  r->counted = prev->counted;
  r->pcount_ok = prev->pcount_ok;
  r->pcount = prev->pcount;
  const uint32_t nsegs = (uint32_t)prev->so.size();
  r->so.resize(nsegs);
  if (nsegs) {
    klf::RunArgs a = e->last_args;
    a.tail = tail;
    a.stage_times = 0;
    a.fuse = 0;  // (the two-pass compaction, over the line index)
    a.plan_runs = 0;  // (plans assume --tail -1 and are consumed by the run)
    a.skip_tcopy = 0;  // (another window may take the dense path)
    a.plan_mode = 0;   // (and may be larger: the gather's plan over the whole grid)
    hipStream_t st = e->stream;
    uint32_t rmask = 0;
    hipError_t h = klf::launch_retail(a, st, e->ev, e->num_cus, &rmask);
    uint32_t short_out = 0;
    if (h == hipSuccess) h = e->h_rb.ensure(kCtrBytes + nsegs * sizeof(SegOut));
    if (h == hipSuccess)
      h = hipMemcpyAsync(e->h_rb.p, e->d_counters.p, kCtrBytes + nsegs * sizeof(SegOut), hipMemcpyDeviceToHost, st);
    if (h == hipSuccess) h = hipStreamSynchronize(st);
    if (h == hipSuccess) {
      memcpy(r->so.data(), e->h_rb.as<uint8_t>() + kCtrBytes, nsegs * sizeof(SegOut));
      short_out = static_cast<uint32_t*>(e->h_rb.p)[klf::kCtrOutShort];
      r->compaction = static_cast<uint32_t*>(e->h_rb.p)[klf::kCtrDense] ? KLF_COMPACT_TILES : KLF_COMPACT_GATHER;
    }
    if (h == hipSuccess && short_out) h = grow_out_retail(e, a, r->so);  // a larger window than the buffer holds
    if (h == hipSuccess) e->last_args = a;
    if (h != hipSuccess) { delete r; return hip_err(e, h, "klf_retail"); }
    if ((rmask & 1u) && (rmask >> 5 & 1u)) {
      float ms = 0.f;
      if ((h = hipEventElapsedTime(&ms, e->ev[0], e->ev[5])) != hipSuccess) { delete r; return hip_err(e, h, "klf_retail timing"); }
      r->ms[4] = ms;
    }
    if ((rmask >> 9 & 1u) && (rmask >> 10 & 1u)) {
      float ms = 0.f;
      if ((h = hipEventElapsedTime(&ms, e->ev[9], e->ev[10])) != hipSuccess) { delete r; return hip_err(e, h, "klf_retail timing"); }
      r->ms[7] = ms;
    }
    r->ev_mask = rmask;
  }
  for (auto& s : r->so) r->total_out = std::max(r->total_out, s.out_hi);
  r->gen = ++e->gen;  // prev's output buffer is rewritten: prev is stale from here on
  e->last_gen = r->gen;
  *out = r;
  return KLF_OK;
}

extern "C" int klf_run(klf_engine* e, const klf_filter* f, klf_result** out) {
  if (!e || !f || !out) return KLF_EINVAL;
  HIPCHK(e, hipSetDevice(e->device), "hipSetDevice");
  HIPCHK(e, ensure_copy_stream(e), "copy stream");
  std::lock_guard<std::mutex> g(e->mu);
  const uint32_t n = (uint32_t)e->staged.size();
  std::vector<uint64_t> lens(n), base(n);
  for (uint32_t i = 0; i < n; ++i) lens[i] = e->staged[i]->len;
  uint64_t total = 0;
  klf_layout(n, lens.data(), base.data(), &total);
  HIPCHK(e, e->d_batch.ensure(total), "alloc batch");
  uint8_t* batch = e->d_batch.as<uint8_t>();
  std::vector<klf::AsmPiece> pieces;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t off = base[i];
    for (uint8_t* d : e->staged[i]->dchunks) {
      pieces.push_back({d, off, kStageChunk});
      off += kStageChunk;
    }
  }
  if (!pieces.empty()) HIPCHK(e, upload(e->d_asm, pieces, e->stream), "upload pieces");
  // early DMAs done -> k_assemble moves the device chunks into place, while the copy
  // stream DMAs every stream's partly filled last chunk straight to its place
  HIPCHK(e, hipEventRecord(e->copy_done, e->copy_stream), "record copy");
  HIPCHK(e, hipStreamWaitEvent(e->stream, e->copy_done, 0), "wait copy");
  if (!pieces.empty())
    HIPCHK(e, klf::launch_assemble(e->d_asm.as<klf::AsmPiece>(), (uint32_t)pieces.size(), batch, e->stream),
           "assemble");
  for (uint32_t i = 0; i < n; ++i) {
    const auto& s = *e->staged[i];
    if (s.cur.p && s.cur.used)
      HIPCHK(e, hipMemcpyAsync(batch + base[i] + s.dchunks.size() * kStageChunk, s.cur.p, s.cur.used,
                               hipMemcpyHostToDevice, e->copy_stream), "H2D tail");
  }
  HIPCHK(e, hipEventRecord(e->copy_done, e->copy_stream), "record tail");
  HIPCHK(e, hipStreamWaitEvent(e->stream, e->copy_done, 0), "wait tail");
  e->ran = true;
  return run_device_impl(e, batch, n, base.data(), lens.data(), f, out);
}

// ---------------------------------------------------------------------- results ---

static int check_result(klf_result* r, uint32_t id) {
  if (!r || id >= r->n_streams) return KLF_EINVAL;
  if (r->e->gen != r->gen) return KLF_ESTATE;  // workspace reused by a later run
  return KLF_OK;
}

// The latest run's global line index, built now if that run left it out (lazy index).
static int ensure_index(klf_engine* e) {
  if (e->index_pending.empty()) return KLF_OK;
  HIPCHK(e, hipSetDevice(e->device), "hipSetDevice");
  for (auto& x : e->index_pending) {
    x.lazy_index = 0;
    x.win_index = 0;
    x.scatter_mode = 0;
    HIPCHK(e, klf::launch_scatter(x, e->stream, e->num_cus), "launch line index");
  }
  HIPCHK(e, hipStreamSynchronize(e->stream), "sync line index");
  e->index_pending.clear();
  e->last_args.lazy_index = 0;
  e->last_args.win_index = 0;
  return KLF_OK;
}

static void fill_counts(const klf_result* r, int64_t s, const uint64_t len, klf_counts* c) {
  if (!c) return;
  memset(c, 0, sizeof(*c));
  if (s < 0) return;
  const SegOut& so = r->so[s];
  const auto mode = r->e->cs.mode;
  c->lines = so.line_hi - so.line_lo;
  c->parsed = so.parsed;
  c->since_ok = so.since_ok;
  c->matched = mode == klf::CompiledSet::kNone ? c->lines : so.matched;
  c->selected = so.sel_hi - so.sel_lo;
  c->out_bytes = len;
}

extern "C" int klf_result_stream(klf_result* r, uint32_t id, const uint8_t** bytes, uint64_t* len, klf_counts* counts) {
  int rc = check_result(r, id);
  if (rc) return rc;
  klf_engine* e = r->e;
  if (bytes && !r->have_out) {  // counts only: no D2H
    r->out.resize(r->total_out + 1);
    if (r->total_out && !r->fused) {
      HIPCHK(e, hipMemcpyAsync(r->out.data(), e->d_out.p, r->total_out, hipMemcpyDeviceToHost, e->stream), "D2H out");
      HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
    } else if (r->total_out) {  // one copy per extent, into the stream's place
      const uint8_t* d = e->d_out.as<uint8_t>();
      for (size_t sg = 0; sg < r->so.size(); ++sg) {
        uint64_t o = r->so[sg].out_lo;
        for (uint32_t k = r->fx_first[sg]; k < r->fx_first[sg + 1]; ++k) {
          const uint64_t n = r->fx[2 * (size_t)k + 1];
          if (n) HIPCHK(e, hipMemcpyAsync(r->out.data() + o, d + r->fx[2 * (size_t)k], n, hipMemcpyDeviceToHost, e->stream),
                        "D2H out");
          o += n;
        }
      }
      HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
    }
    r->have_out = true;
  }
  const int64_t s = r->seg_of[id];
  uint64_t n = 0, off = 0;
  if (s >= 0) { off = r->so[s].out_lo; n = r->so[s].out_hi - r->so[s].out_lo; }
  if (bytes) *bytes = r->out.data() + off;
  if (len) *len = n;
  fill_counts(r, s, n, counts);
  return KLF_OK;
}

static bool write_all(int fd, const uint8_t* p, uint64_t n) {  // io.Copy's write loop
  while (n) {
    const ssize_t k = ::write(fd, p, (size_t)std::min<uint64_t>(n, 1u << 30));
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (k == 0) {
      errno = EIO;
      return false;
    }
    p += k;
    n -= (uint64_t)k;
  }
  return true;
}

// §8f-3: device output -> per-stream files.  The output is one buffer in stream order;
// it crosses PCIe once, through 64 MiB pinned chunks taken from the staging pool, with
// the DMA of the next piece in flight while the host writes the current one.
//
// A page-cache write(2) is a host memcpy under the file's inode lock (≈ 7 GB/s on one
// core, measured), far below the pinned D2H, so with several streams each worker thread
// owns whole streams (files), with its own HIP stream and pinned chunk: files are written
// in parallel and each file still sees one sequential write(2) sequence.  One descriptor
// shared by several streams must see them in stream order: that case (and small outputs)
// runs on the calling thread alone.
namespace {
// a stream's output: [lo, hi) of the concatenated output, in d_out as `parts` ({offset,
// length}: one part, or a fused run's extents)
struct WPiece {
  uint64_t lo, hi;
  int fd;
  uint32_t id;
  std::vector<std::pair<uint64_t, uint64_t>> parts;
};

struct WErr { std::atomic<int> id{-1}; int err = 0; std::string what; std::mutex mu; };

// D2H each part of the stream's output in two halves of `buf` (double-buffered on `st`) and
// write(2) each half to fd.  Returns false with `werr` set on the first failure.
bool copy_part(klf_engine* e, const uint8_t* d_out, const WPiece& q, uint64_t dlo, uint64_t n, uint8_t* buf,
               uint64_t half, hipStream_t st, hipEvent_t ev[2], WErr& werr, uint64_t& total);
bool copy_piece(klf_engine* e, const uint8_t* d_out, const WPiece& q, uint8_t* buf, uint64_t half,
                hipStream_t st, hipEvent_t ev[2], WErr& werr, uint64_t& total) {
  for (const auto& pt : q.parts)
    if (pt.second && !copy_part(e, d_out, q, pt.first, pt.second, buf, half, st, ev, werr, total)) return false;
  return true;
}
bool copy_part(klf_engine* e, const uint8_t* d_out, const WPiece& q, uint64_t dlo, uint64_t n, uint8_t* buf,
               uint64_t half, hipStream_t st, hipEvent_t ev[2], WErr& werr, uint64_t& total) {
  auto fail = [&](int err, const std::string& what) {
    int exp = -1;
    if (werr.id.compare_exchange_strong(exp, (int)q.id)) { werr.err = err; werr.what = what; }
    return false;
  };
  const uint64_t nk = (n + half - 1) / half;
  auto issue = [&](uint64_t k) {
    const uint64_t o = k * half, m = std::min(half, n - o);
    return hipMemcpyAsync(buf + (k & 1) * half, d_out + dlo + o, m, hipMemcpyDeviceToHost, st) == hipSuccess &&
           hipEventRecord(ev[k & 1], st) == hipSuccess;
  };
  if (!issue(0)) return fail(0, "D2H");
  for (uint64_t k = 0; k < nk; ++k) {
    if (werr.id.load() >= 0) return false;  // another worker failed: stop early
    if (k + 1 < nk && !issue(k + 1)) return fail(0, "D2H");
    if (hipEventSynchronize(ev[k & 1]) != hipSuccess) return fail(0, "D2H sync");
    const uint64_t o = k * half, m = std::min(half, n - o);
    if (!write_all(q.fd, buf + (k & 1) * half, m)) return fail(errno, "write");
    total += m;
  }
  (void)e;
  return true;
}
}  // namespace

extern "C" int klf_result_write(klf_result* r, const int* fds, uint32_t n_fds, uint64_t* written) {
  if (written) *written = 0;
  if (!r || (n_fds && !fds) || n_fds != r->n_streams) return KLF_EINVAL;
  klf_engine* e = r->e;
  if (e->gen != r->gen) return KLF_ESTATE;
  std::vector<WPiece> pcs;
  for (uint32_t i = 0; i < n_fds; ++i) {
    const int64_t s = r->seg_of[i];
    if (fds[i] < 0 || s < 0 || r->so[s].out_hi == r->so[s].out_lo) continue;
    WPiece q{r->so[s].out_lo, r->so[s].out_hi, fds[i], i, {}};
    if (r->fused) {
      for (uint32_t k = r->fx_first[s]; k < r->fx_first[s + 1]; ++k) q.parts.emplace_back(r->fx[2 * (size_t)k], r->fx[2 * (size_t)k + 1]);
    } else {
      q.parts.emplace_back(q.lo, q.hi - q.lo);
    }
    pcs.push_back(std::move(q));
  }
  if (pcs.empty()) return KLF_OK;
  std::sort(pcs.begin(), pcs.end(), [](const WPiece& a, const WPiece& b) { return a.lo < b.lo; });
  uint64_t out_bytes = 0;
  for (const auto& q : pcs) out_bytes += q.hi - q.lo;
  auto eio = [&](const WErr& w) {
    return set_err(e, KLF_EIO, "write stream " + std::to_string(w.id.load()) + ": " + w.what +
                                   (w.err ? std::string(": ") + strerror(w.err) : std::string()));
  };
  if (r->have_out) {  // already on the host (klf_result_stream ran)
    uint64_t total = 0;
    for (const auto& q : pcs) {
      if (!write_all(q.fd, r->out.data() + q.lo, q.hi - q.lo))
        return set_err(e, KLF_EIO, "write stream " + std::to_string(q.id) + ": " + strerror(errno));
      total += q.hi - q.lo;
    }
    if (written) *written = total;
    return KLF_OK;
  }
  int nthr = 8;
  if (const char* v = getenv("KLF_WRITE_THREADS")) nthr = std::max(1, atoi(v));
  nthr = (int)std::min<size_t>((size_t)nthr, pcs.size());
  {
    std::vector<int> f;
    for (const auto& q : pcs) f.push_back(q.fd);
    std::sort(f.begin(), f.end());
    if (std::adjacent_find(f.begin(), f.end()) != f.end()) nthr = 1;  // shared fd: stream order
  }
  if (out_bytes < (8u << 20)) nthr = 1;
  HIPCHK(e, hipStreamSynchronize(e->stream), "sync before write");  // d_out complete
  const uint8_t* d_out = e->d_out.as<uint8_t>();
  WErr werr;
  std::atomic<size_t> next{0};
  std::vector<uint64_t> totals((size_t)nthr, 0);
  std::atomic<int> setup_fail{0};
  auto worker = [&](int t) {
    klf_engine::StageChunk c;
    hipStream_t st = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ok = hipSetDevice(e->device) == hipSuccess && take_chunk(e, &c) &&
              hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      setup_fail = 1;
    } else {
      for (size_t j; (j = next.fetch_add(1)) < pcs.size();)
        if (!copy_piece(e, d_out, pcs[j], c.p, kStageChunk / 2, st, ev, werr, totals[(size_t)t])) break;
    }
    if (st) (void)hipStreamSynchronize(st);  // no DMA into a chunk handed back below
    for (auto& x : ev)
      if (x) (void)hipEventDestroy(x);
    if (st) (void)hipStreamDestroy(st);
    if (c.p) {
      std::lock_guard<std::mutex> g(e->mu);
      c.used = 0;
      e->chunk_pool.push_back(c);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthr; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  if (setup_fail && werr.id.load() < 0 && next.load() < pcs.size())
    return set_err(e, KLF_ENOMEM, "write worker setup (pinned chunk / HIP stream)");
  if (werr.id.load() >= 0) return eio(werr);
  uint64_t total = 0;
  for (auto x : totals) total += x;
  if (written) *written = total;
  return KLF_OK;
}

extern "C" int klf_result_lines(klf_result* r, uint32_t id, const uint64_t** off, uint64_t* n_lines) {
  int rc = check_result(r, id);
  if (rc) return rc;
  klf_engine* e = r->e;
  const int64_t s = r->seg_of[id];
  static const uint64_t kZero = 0;
  if (s < 0) {
    if (off) *off = &kZero;
    if (n_lines) *n_lines = 0;
    return KLF_OK;
  }
  if (!r->have_lines) {
    if (int rc2 = ensure_index(e)) return rc2;
    const size_t nwords = r->total_lines + r->so.size();
    r->line_off.resize(nwords);
    HIPCHK(e, hipMemcpyAsync(r->line_off.data(), e->d_line_off.p, nwords * 8, hipMemcpyDeviceToHost, e->stream), "D2H lines");
    HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
    r->have_lines = true;
  }
  if (off) *off = r->line_off.data() + r->so[s].line_lo + (uint64_t)s;
  if (n_lines) *n_lines = r->so[s].line_hi - r->so[s].line_lo;
  return KLF_OK;
}

extern "C" int klf_result_match_bits(klf_result* r, uint32_t id, const uint8_t** bits, uint64_t* nbytes) {
  int rc = check_result(r, id);
  if (rc) return rc;
  if (!r->has_bits) return KLF_EINVAL;
  klf_engine* e = r->e;
  if (!r->have_bits) {
    if (int rc2 = ensure_index(e)) return rc2;
    const size_t nw = r->total_lines / 32 + 1;
    r->bits.assign(nw, 0);
    if (!r->so.empty()) {
      HIPCHK(e, hipMemcpyAsync(r->bits.data(), e->d_bits.p, nw * 4, hipMemcpyDeviceToHost, e->stream), "D2H bits");
      HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
    }
    r->have_bits = true;
    r->stream_bits.assign(r->n_streams, {});
    r->have_stream_bits.assign(r->n_streams, 0);
  }
  if (!r->have_stream_bits[id]) {
    const int64_t s = r->seg_of[id];
    auto& v = r->stream_bits[id];
    if (s >= 0) {
      const uint64_t lo = r->so[s].line_lo, n = r->so[s].line_hi - lo;
      v.assign((n + 7) / 8, 0);
      for (uint64_t i = 0; i < n; ++i) {
        const uint64_t l = lo + i;
        if ((r->bits[l >> 5] >> (l & 31)) & 1u) v[i >> 3] |= (uint8_t)(1u << (i & 7));
      }
    }
    r->have_stream_bits[id] = 1;
  }
  if (bits) *bits = r->stream_bits[id].data();
  if (nbytes) *nbytes = r->stream_bits[id].size();
  return KLF_OK;
}

extern "C" int klf_result_pattern_counts(klf_result* r, uint32_t id, uint64_t* counts, uint32_t cap, uint32_t* n) {
  if (!r || id >= r->n_streams || (cap && !counts)) return KLF_EINVAL;
  klf_engine* e = r->e;
  if (n) *n = e->n_user;
  if (!r->counted) return set_err(e, KLF_ESTATE, "the run did not ask for per-pattern counts (KLF_FILTER_PATTERN_COUNTS)");
  if (e->counts_code != KLF_OK) return set_err(e, e->counts_code, e->counts_err);
  const auto& cs = e->cs;
  const int64_t s = r->seg_of[id];
  const bool general = cs.mode == klf::CompiledSet::kGeneral;
  if (general && !r->pcount_ok)
    return set_err(e, KLF_ETOOBIG, "per-pattern counts: the (line, pattern) pair set overflowed");
  for (uint32_t u = 0; u < std::min(cap, e->n_user); ++u) {
    const int32_t m = u < cs.user_map.size() ? cs.user_map[u] : klf::CompiledSet::kCidNever;
    uint64_t v = 0;
    if (s >= 0) {
      const SegOut& so = r->so[s];
      if (m == klf::CompiledSet::kCidAlways) v = so.parsed;
      else if (m >= 0 && cs.mode == klf::CompiledSet::kLiteral1) v = so.matched;  // the one literal
      else if (m >= 0 && general) v = r->pcount[(size_t)s * cs.n_cids + (size_t)m];
    }
    counts[u] = v;
  }
  return KLF_OK;
}

extern "C" int klf_result_last_unparsed(klf_result* r, uint32_t id, uint64_t* rank) {
  int rc = check_result(r, id);
  if (rc) return rc;
  if (!rank) return KLF_EINVAL;
  *rank = 0;
  const int64_t s = r->seg_of[id];
  if (s < 0) return KLF_OK;
  klf_engine* e = r->e;
  const SegOut& so = r->so[s];
  const uint64_t hi = so.line_hi - (so.frag ? 1 : 0);  // newline-terminated lines only
  if (hi <= so.line_lo) return KLF_OK;
  if (int rc2 = ensure_index(e)) return rc2;
  HIPCHK(e, e->d_scratch.ensure(64), "alloc scratch");
  uint64_t v = 0;
  HIPCHK(e, klf::launch_lastbad(e->last_args, so.line_lo, hi, e->d_scratch.as<uint64_t>(), e->stream), "lastbad");
  HIPCHK(e, hipMemcpyAsync(&v, e->d_scratch.p, 8, hipMemcpyDeviceToHost, e->stream), "D2H lastbad");
  HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
  if (v) *rank = hi - (v - 1);
  return KLF_OK;
}

extern "C" int klf_result_device_out(klf_result* r, uint32_t id, const uint8_t** d_out, uint64_t* off, uint64_t* len) {
  if (r && r->fused && !r->have_dev && check_result(r, id) == KLF_OK) {  // one contiguous copy, on demand
    klf_engine* e = r->e;
    HIPCHK(e, hipSetDevice(e->device), "hipSetDevice");
    HIPCHK(e, e->d_out2.ensure(r->total_out + 64), "alloc contiguous output");
    const uint8_t* d = e->d_out.as<uint8_t>();
    for (size_t sg = 0; sg < r->so.size(); ++sg) {
      uint64_t o = r->so[sg].out_lo;
      for (uint32_t k = r->fx_first[sg]; k < r->fx_first[sg + 1]; ++k) {
        const uint64_t n = r->fx[2 * (size_t)k + 1];
        if (n) HIPCHK(e, hipMemcpyAsync(e->d_out2.as<uint8_t>() + o, d + r->fx[2 * (size_t)k], n, hipMemcpyDeviceToDevice,
                                        e->stream), "D2D contiguous output");
        o += n;
      }
    }
    HIPCHK(e, hipStreamSynchronize(e->stream), "sync");
    r->have_dev = true;
  }
  int rc = check_result(r, id);
  if (rc) return rc;
  const int64_t s = r->seg_of[id];
  if (d_out) *d_out = r->fused ? r->e->d_out2.as<uint8_t>() : r->e->d_out.as<uint8_t>();
  if (off) *off = s >= 0 ? r->so[s].out_lo : 0;
  if (len) *len = s >= 0 ? r->so[s].out_hi - r->so[s].out_lo : 0;
  return KLF_OK;
}

extern "C" int klf_result_timing(const klf_result* r, double* ms, uint32_t cap, uint32_t* n) {
  if (!r || (cap && !ms)) return KLF_EINVAL;
  const uint32_t k = std::min<uint32_t>(cap, 8);
  for (uint32_t i = 0; i < k; ++i) ms[i] = r->ms[i];
  if (n) *n = k;
  return KLF_OK;
}

extern "C" int klf_result_index_mode(const klf_result* r) { return r ? r->index_mode : KLF_EINVAL; }
extern "C" int klf_result_compaction(const klf_result* r) { return r ? r->compaction : KLF_EINVAL; }

extern "C" int klf_result_totals(const klf_result* r, klf_counts* t) {
  if (!r || !t) return KLF_EINVAL;
  memset(t, 0, sizeof(*t));
  for (uint32_t i = 0; i < r->n_streams; ++i) {
    const int64_t s = r->seg_of[i];
    if (s < 0) continue;
    klf_counts c;
    fill_counts(r, s, r->so[s].out_hi - r->so[s].out_lo, &c);
    t->lines += c.lines;
    t->parsed += c.parsed;
    t->since_ok += c.since_ok;
    t->matched += c.matched;
    t->selected += c.selected;
    t->out_bytes += c.out_bytes;
  }
  return KLF_OK;
}

extern "C" void klf_result_free(klf_result* r) { delete r; }

// ------------------------------------------------------------------ follow mode ---

struct klf_follow {
  klf_engine* e = nullptr;
  klf_filter f{};
  std::mutex mu;  // guards the carry table's growth (feeds of different ids run concurrently)
  std::vector<std::unique_ptr<std::string>> carry;
};

static std::string* follow_carry(klf_follow* w, uint32_t id) {
  std::lock_guard<std::mutex> g(w->mu);
  while (w->carry.size() <= id) w->carry.emplace_back(new std::string());
  return w->carry[id].get();
}

extern "C" int klf_follow_open(klf_engine* e, const klf_filter* f, klf_follow** out) {
  if (!e || !f || !out) return KLF_EINVAL;
  *out = nullptr;
  auto* w = new (std::nothrow) klf_follow();
  if (!w) return KLF_ENOMEM;
  w->e = e;
  w->f = *f;
  w->f.tail = -1;  // per-line rules only: the server applies --tail to the backlog
  const int rc = klf_reset(e);
  if (rc) { delete w; return rc; }
  *out = w;
  return KLF_OK;
}

extern "C" int klf_follow_feed(klf_follow* w, uint32_t id, const uint8_t* p, size_t n) {
  if (!w || (n && !p)) return KLF_EINVAL;
  std::string* c;
  try {
    c = follow_carry(w, id);
  } catch (...) {
    return KLF_ENOMEM;
  }
  if (!n) return KLF_OK;
  const uint8_t* nl = static_cast<const uint8_t*>(memrchr(p, '\n', n));
  if (!nl) {  // still inside the open line
    c->append(reinterpret_cast<const char*>(p), n);
    return KLF_OK;
  }
  const size_t cut = (size_t)(nl - p) + 1;
  if (!c->empty()) {
    const int rc = klf_stage(w->e, id, reinterpret_cast<const uint8_t*>(c->data()), c->size());
    if (rc) return rc;
    c->clear();  // staged: a retried feed must not stage it again
  }
  const int rc = klf_stage(w->e, id, p, cut);
  if (rc) return rc;
  c->assign(reinterpret_cast<const char*>(p + cut), n - cut);
  return KLF_OK;
}

extern "C" int klf_follow_flush(klf_follow* w, int final, klf_result** out) {
  if (!w || !out) return KLF_EINVAL;
  *out = nullptr;
  const uint32_t n = (uint32_t)w->carry.size();
  if (final)
    for (uint32_t i = 0; i < n; ++i) {
      std::string& c = *w->carry[i];
      if (c.empty()) continue;
      const int rc = klf_stage(w->e, i, reinterpret_cast<const uint8_t*>(c.data()), c.size());
      if (rc) return rc;
      c.clear();
    }
  int rc = klf_set_streams(w->e, n);
  if (!rc) rc = klf_run(w->e, &w->f, out);
  const int rr = klf_reset(w->e);  // the result keeps its outputs; the staging is released
  return rc ? rc : rr;
}

extern "C" uint64_t klf_follow_open_bytes(const klf_follow* w, uint32_t id) {
  return (w && id < w->carry.size()) ? w->carry[id]->size() : 0;
}

extern "C" void klf_follow_close(klf_follow* w) { delete w; }

// ---------------------------------------------------------------- host helpers ---

extern "C" int klf_parse_rfc3339nano(const uint8_t* s, size_t n, klf_time* out) {
  if (!s || !out) return KLF_EINVAL;
  klf::TsResult r;
  auto get = [&](uint32_t i) -> int { return i < n ? s[i] : -1; };
  if (!klf::parse_rfc3339nano(get, r) || r.len != n) return KLF_EINVAL;
  out->sec = r.sec;
  out->nsec = r.nsec;
  out->_reserved = 0;
  return KLF_OK;
}

extern "C" int klf_debug_match(const klf_pattern* pats, uint32_t n, const uint8_t* content, size_t len, int* match) {
  if ((n && !pats) || (len && !content) || !match) return KLF_EINVAL;
  std::vector<std::vector<uint8_t>> ps;
  std::vector<uint32_t> kinds;
  for (uint32_t i = 0; i < n; ++i) {
    ps.emplace_back(pats[i].bytes, pats[i].bytes + pats[i].len);
    kinds.push_back(pats[i].kind);
  }
  klf::CompiledSet cs;
  std::string err;
  int code = KLF_OK;
  if (!klf::compile_set(ps, kinds, cs, err, code)) return code;
  bool hit = false;
  switch (cs.mode) {
    case klf::CompiledSet::kNone: case klf::CompiledSet::kAll: hit = true; break;
    case klf::CompiledSet::kNever: hit = false; break;
    case klf::CompiledSet::kLiteral1:
      hit = std::search(content, content + len, cs.literal.begin(), cs.literal.end()) != content + len;
      break;
    case klf::CompiledSet::kGeneral: {
      hit = cs.also_all;
      if (cs.ac_states) {  // run the same DFA tables the GPU runs
        uint32_t st = 0;
        for (size_t i = 0; i < len && !hit; ++i) {
          st = cs.ac_next[(size_t)st * cs.ac_classes + cs.ac_class[content[i]]];
          hit = cs.ac_accept[st] != 0;
        }
      }
      for (uint32_t r = 0; r < cs.rx_count && !hit; ++r) {  // the GPU recurrence on host
        const uint32_t fl = cs.rx_flags[r];
        if (len == 0) { hit = fl & 2u; continue; }
        if (fl & 1u) { hit = true; continue; }
        uint64_t d = cs.rx_init0[r];
        for (size_t i = 0; i < len && !hit; ++i) {
          const uint64_t c = d & cs.rx_b[(size_t)r * cs.rx_classes + cs.rx_class[content[i]]];
          if (c & cs.rx_last[r]) { hit = true; break; }
          uint64_t nd = cs.rx_first[r];
          for (int p = 0; p < 64; ++p)
            if (c >> p & 1) nd |= cs.rx_follow[(size_t)r * 64 + p];
          d = nd;
        }
        if (!hit) hit = (d & cs.rx_end[r]) != 0;
      }
      break;
    }
  }
  *match = hit ? 1 : 0;
  return KLF_OK;
}

extern "C" int klf_debug_clock(int device, uint32_t iters, uint32_t reps, double* mhz) {
  if (!mhz || !iters || !reps) return KLF_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return KLF_EHIP;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
    return KLF_EHIP;
  const size_t nb = (size_t)ncu * 4;
  uint64_t* d = nullptr;
  if (hipMalloc(&d, (2 * nb + 1) * 8) != hipSuccess) return KLF_ENOMEM;
  hipStream_t st = nullptr;
  hipError_t h = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (h == hipSuccess) h = klf::clock_probe(ncu, iters, reps, d, st);
  std::vector<uint64_t> v(2 * nb + 1, 0);
  if (h == hipSuccess) h = hipMemcpyAsync(v.data(), d, v.size() * 8, hipMemcpyDeviceToHost, st);
  if (h == hipSuccess) h = hipStreamSynchronize(st);
  if (st) (void)hipStreamDestroy(st);
  (void)hipFree(d);
  if (h != hipSuccess) return KLF_EHIP;
  std::vector<double> f;
  for (size_t b = 0; b < nb; ++b)
    if (v[2 * b + 1]) f.push_back(100.0 * (double)v[2 * b] / (double)v[2 * b + 1]);  // 100 MHz real time
  if (f.empty()) return KLF_EHIP;
  std::sort(f.begin(), f.end());
  mhz[0] = f[f.size() / 2];
  mhz[1] = f.front();
  mhz[2] = f.back();
  return KLF_OK;
}

extern "C" int klf_debug_since_digits(int64_t sec, int32_t nsec, uint32_t* out) {
  if (!out) return KLF_EINVAL;
  since_digits(sec, nsec, out);
  return KLF_OK;
}

extern "C" int klf_debug_prefilter(const klf_pattern* pats, uint32_t n, const uint8_t* content, size_t len,
                                   uint32_t phase, int* match, uint32_t* info) {
  if ((n && !pats) || (len && !content) || !match) return KLF_EINVAL;
  std::vector<std::vector<uint8_t>> ps;
  std::vector<uint32_t> kinds;
  for (uint32_t i = 0; i < n; ++i) {
    ps.emplace_back(pats[i].bytes, pats[i].bytes + pats[i].len);
    kinds.push_back(pats[i].kind);
  }
  klf::CompiledSet cs;
  std::string err;
  int code = KLF_OK;
  if (!klf::compile_set(ps, kinds, cs, err, code)) return code;
  if (info) {
    info[0] = cs.qf_on ? 1u : 0u;
    info[1] = cs.qf_q;
    info[2] = cs.qf_stride;
    info[3] = cs.qf_needles;
    info[4] = cs.qf_anc_on ? 0x100u | cs.qf_anc_byte : 0u;
  }
  if (cs.mode != klf::CompiledSet::kGeneral || !cs.qf_on) return klf_debug_match(pats, n, content, len, match);
  *match = klf::prefilter_match(cs, content, len, phase) ? 1 : 0;
  return KLF_OK;
}

extern "C" int klf_debug_prefilter_hits(const klf_pattern* pats, uint32_t n, const uint8_t* sample, size_t slen,
                                        const uint8_t* data, size_t dlen, uint64_t* out, char* layout, size_t cap) {
  if ((n && !pats) || (slen && !sample) || (dlen && !data) || !out) return KLF_EINVAL;
  std::vector<std::vector<uint8_t>> ps;
  std::vector<uint32_t> kinds;
  for (uint32_t i = 0; i < n; ++i) {
    ps.emplace_back(pats[i].bytes, pats[i].bytes + pats[i].len);
    kinds.push_back(pats[i].kind);
  }
  klf::CompiledSet cs;
  std::string err;
  int code = KLF_OK;
  if (!klf::compile_set(ps, kinds, cs, err, code)) return code;
  if (cs.mode != klf::CompiledSet::kGeneral || !cs.qf_on) return KLF_EINVAL;
  if (slen) {
    klf::DataStats st;
    klf::data_stats(sample, slen, cs.qf_fold, st);
    klf::place_needles(cs, &st);
  }
  const klf::PrefilterHits h = klf::prefilter_hits(cs, data, dlen);
  out[0] = cs.qf_stride;
  out[1] = cs.qf_q;
  out[2] = cs.qf_k;
  out[3] = cs.qf_anc_on ? 0x100u | cs.qf_anc_byte : 0u;
  out[4] = h.probes;
  out[5] = h.bitmap_hits;
  out[6] = h.anchor_hits;
  out[7] = h.verified;
  out[8] = h.pair_pass;
  if (layout && cap) { strncpy(layout, cs.qf_layout.c_str(), cap - 1); layout[cap - 1] = 0; }
  return KLF_OK;
}

extern "C" int klf_debug_compile(const klf_pattern* pats, uint32_t n, uint32_t* mode, char* err, size_t err_cap) {
  if ((n && !pats) || !mode) return KLF_EINVAL;
  std::vector<std::vector<uint8_t>> ps;
  std::vector<uint32_t> kinds;
  for (uint32_t i = 0; i < n; ++i) {
    ps.emplace_back(pats[i].bytes, pats[i].bytes + pats[i].len);
    kinds.push_back(pats[i].kind);
  }
  klf::CompiledSet cs;
  std::string e;
  int code = KLF_OK;
  bool ok = klf::compile_set(ps, kinds, cs, e, code);
  if (err && err_cap) { strncpy(err, e.c_str(), err_cap - 1); err[err_cap - 1] = 0; }
  *mode = (uint32_t)cs.mode;
  return ok ? KLF_OK : code;
}

extern "C" int klf_debug_factors(const uint8_t* pat, size_t len, uint32_t want, char* buf, size_t cap, uint32_t* n,
                                 uint32_t* pre, uint32_t* loose) {
  if ((len && !pat) || (cap && !buf) || !n || !pre || !loose) return KLF_EINVAL;
  std::vector<std::string> alts;
  bool l = false;
  uint32_t p = 0;
  if (!klf::regex_factors(pat, len, alts, l, &p, want ? want : SIZE_MAX)) return KLF_EINVAL;
  size_t o = 0;
  for (auto& a : alts) {
    if (o + a.size() + 1 > cap) return KLF_ETOOBIG;
    memcpy(buf + o, a.data(), a.size());
    o += a.size();
    buf[o++] = 0;
  }
  *n = (uint32_t)alts.size();
  *pre = p;
  *loose = l ? 1u : 0u;
  return KLF_OK;
}
