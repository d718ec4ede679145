/*
 * klf.h — C ABI of the MI355X log-filter engine (libklf.so).
 *
 * This is the seam klogs' Go host binds through cgo.  It replaces
 * the byte sink `writeLogToDisk(logs io.ReadCloser, logFile *os.File)`
 * (/root/reference/cmd/root.go:359-374, called from streamLog at :337) for streams the
 * host now fetches with Timestamps=true and without SinceSeconds/TailLines
 * (getLopOpts, cmd/root.go:201-221).  The filtering kubelet used to do server-side
 * (k8s v1.30.3 logs.go ReadLogs / tail.go FindTailLineStartIndex) runs here, on the GPU,
 * with the exact semantics of SPEC.md.
 *
 * Conventions: every function returns 0 (KLF_OK) or a negative KLF_E* code; no C++
 * types, no HIP types (streams are passed as void*).  Pointers handed in are not
 * retained after return unless stated (cgo pointer rules).  Views handed out stay valid
 * until the owning object is freed.
 *
 * Threading: klf_stage may be called concurrently for DIFFERENT stream ids (one
 * goroutine per container stream, cmd/root.go:249/:261), with no other precondition (the
 * stream table grows as needed); calls for one id are in order.  Everything else is
 * single-caller per engine, and klf_run starts after every klf_stage has returned
 * (wg.Wait(), cmd/root.go:470).
 */
#ifndef KLF_H
#define KLF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------- */
#define KLF_OK 0
#define KLF_EINVAL -1      /* bad argument (null pointer, bad id, tail < -1, ...)      */
#define KLF_ENOMEM -2      /* host or device allocation failed                          */
#define KLF_EHIP -3        /* a HIP runtime call failed (no device, launch error, ...)  */
#define KLF_EPATTERN -4    /* a --match pattern is outside the supported RE2 subset     */
#define KLF_ETOOBIG -5     /* pattern set exceeds engine limits                         */
#define KLF_ESTATE -6      /* call out of order (e.g. stage after run without reset)    */
#define KLF_EIO -7         /* write(2) to a stream's file failed (klf_result_write)       */

/* ---- instants ------------------------------------------------------------------- */
/* An absolute UTC instant: seconds since the Unix epoch + nanoseconds in [0, 1e9).
 * Comparisons are lexicographic (Go time.Time.Before). */
typedef struct klf_time {
  int64_t sec;
  int32_t nsec;
  int32_t _reserved;
} klf_time;

/* Go's zero time.Time, 0001-01-01T00:00:00Z: kubelet's `since` when SinceSeconds is
 * unset (logs.go NewLogOptions); pass it for "no --since". */
#define KLF_GO_ZERO_TIME_SEC (-62135596800LL)

/* ---- patterns ------------------------------------------------------------------- */
#define KLF_PAT_LITERAL 0 /* --grep: Go bytes.Contains(content, p)                      */
#define KLF_PAT_REGEX 1   /* --match: Go regexp.Match(p, content), SPEC.md S5 subset     */

typedef struct klf_pattern {
  const uint8_t* bytes;
  uint32_t len;
  uint32_t kind; /* KLF_PAT_* */
} klf_pattern;

/* ---- engine --------------------------------------------------------------------- */
typedef struct klf_config {
  int32_t device;          /* HIP device ordinal (one process per GPU)                 */
  uint32_t n_patterns;     /* OR'ed; 0 = no grep stage                                 */
  const klf_pattern* patterns;
  void* hip_stream;        /* hipStream_t to launch on; NULL = HIP's null stream        */
  uint64_t staging_hint;   /* expected total staged bytes (pre-reserve), 0 = none       */
} klf_config;

typedef struct klf_engine klf_engine;

/* Compiles the pattern set once (replaces nothing in the reference: --grep/--match are
 * new flags added at cmd/root.go:485-497).  Every pattern error is reported here.  A set
 * with several literals starts one host thread that builds and uploads their Aho-Corasick
 * automaton while the first klf_run samples the data; that run (or klf_close) joins it. */
int klf_open(const klf_config* cfg, klf_engine** out);
void klf_close(klf_engine* e);
/* Human-readable detail of the last error on this engine (e.g. the pattern error). */
const char* klf_last_error(const klf_engine* e);
const char* klf_strerror(int code);

/* ---- host staging path (what the cgo glue calls) -------------------------------- */
/* Appends n bytes of stream `stream_id`'s body (chunks arrive in order).  Replaces the
 * io.Copy in writeLogToDisk (cmd/root.go:366).  Ids are dense, 0-based, caller-chosen
 * (the stream-table order of getPodLogs, cmd/root.go:240-262).  The bytes are copied into
 * pinned host chunks (large pieces striped over a few copy threads; KLF_STAGE_THREADS)
 * and every chunk that fills (64 MiB) is DMA'd to HBM at once, overlapping the capture.
 * KLF_ESTATE after klf_run until klf_reset. */
int klf_stage(klf_engine* e, uint32_t stream_id, const uint8_t* p, size_t n);
/* Declares stream ids [0, n_streams) (streams never staged are empty). */
int klf_set_streams(klf_engine* e, uint32_t n_streams);
/* Drops all staged bytes (engine and compiled patterns stay). */
int klf_reset(klf_engine* e);

typedef struct klf_filter {
  klf_time since;   /* lines with ts.Before(since) are dropped (S3)                    */
  int64_t tail;     /* -1 = all, else >= 0 (S4)                                        */
  uint32_t flags;   /* KLF_FILTER_* bits, 0 = none                                     */
  uint32_t _reserved;
} klf_filter;

/* klf_filter.flags: record the inner stage boundaries (klf_result_timing [0]-[3]).
 * Each boundary costs a few microseconds of idle GPU; off, only [4]-[6] are measured. */
#define KLF_FILTER_STAGE_TIMES 1u
/* klf_filter.flags: count matching lines per pattern (klf_result_pattern_counts). */
#define KLF_FILTER_PATTERN_COUNTS 2u
/* klf_filter.flags: write every line's u64 offset inside the run (KLF_INDEX_FULL), also where
 * the run needs only part of the index (see klf_result_index_mode). */
#define KLF_FILTER_FULL_INDEX 4u
/* klf_filter.flags: record no timing events (klf_result_timing then reports zeros; it
 * overrides KLF_FILTER_STAGE_TIMES).  The k_scan dispatch's own events and the run's
 * bracket cost a few microseconds of device time per run (C1: ~5 of ~75 us), which a
 * caller that never reads the timing need not pay. */
#define KLF_FILTER_NO_TIMING 8u

/* klf_result_index_mode: how much of the u64 line index the run wrote itself. */
#define KLF_INDEX_FULL 0       /* every line of every stream                                  */
#define KLF_INDEX_WINDOWS 1    /* the lines of each stream's --tail window (prefiltered sets)  */
#define KLF_INDEX_ON_DEMAND 2  /* none (no patterns, --tail -1, the dense copy path)          */

typedef struct klf_counts {
  uint64_t lines;      /* all lines (a trailing fragment counts)                       */
  uint64_t parsed;     /* lines with a valid RFC3339Nano prefix                       */
  uint64_t since_ok;   /* parsed lines with ts >= since                               */
  uint64_t matched;    /* |G|: matching parsed lines (all lines without patterns)     */
  uint64_t selected;   /* emitted lines                                               */
  uint64_t out_bytes;  /* emitted bytes                                               */
} klf_counts;

typedef struct klf_result klf_result;

/* Runs the whole filter over the staged streams (H2D, kernels, counts D2H).  Called
 * once after wg.Wait() (cmd/root.go:470). */
int klf_run(klf_engine* e, const klf_filter* f, klf_result** out);

/* ---- device-resident path (bench / callers that already hold bytes in HBM) ------- */
/* Device layout helper: segment base offsets (256-B aligned, in stream order) and the
 * total device bytes to allocate (includes tail slack the kernels may over-read). */
int klf_layout(uint32_t n_streams, const uint64_t* lens, uint64_t* seg_base,
               uint64_t* total_alloc);
/* Runs over streams already laid out in device memory at d_bytes + seg_base[i]
 * (d_bytes must be a 16-B aligned device allocation of >= total_alloc bytes from klf_layout;
 * KLF_EINVAL otherwise). */
int klf_run_device(klf_engine* e, const uint8_t* d_bytes, uint32_t n_streams,
                   const uint64_t* seg_base, const uint64_t* lens, const klf_filter* f,
                   klf_result** out);

/* Re-applies the tail rule with a different N to the latest run (prev must be the
 * engine's latest result): re-runs only matched counts, the tail window and the
 * compaction on the line index, parse/since bits and match bitmap the run left in HBM.
 * The byte-range shards of one stream need it: a rank's share of the
 * global --tail is known only after the count exchange.  prev becomes stale
 * (KLF_ESTATE on access) because the output buffer is rewritten.  Replaces nothing in
 * the reference (kubelet applies --tail once, server-side: logs.go / tail.go). */
int klf_retail(klf_engine* e, klf_result* prev, int64_t tail, klf_result** out);

/* ---- results -------------------------------------------------------------------- */
/* Selected bytes of one stream (host view, D2H on first access; bytes == NULL: len and
 * counts only, no D2H). */
int klf_result_stream(klf_result* r, uint32_t stream_id, const uint8_t** bytes,
                      uint64_t* len, klf_counts* counts);
/* Line-start offsets of one stream: n_lines+1 u64 (last = stream length).  Runs that did
 * not need the whole line index (no patterns with --tail -1, or literal patterns: only the
 * tail windows' lines were indexed) build it here on first use, on the device. */
int klf_result_lines(klf_result* r, uint32_t stream_id, const uint64_t** off,
                     uint64_t* n_lines);
/* Match bitmap of one stream (bit l LSB-first in byte l>>3); *nbytes = ceil(lines/8).
 * Returns KLF_EINVAL when the engine has no patterns. */
int klf_result_match_bits(klf_result* r, uint32_t stream_id, const uint8_t** bits,
                          uint64_t* nbytes);
/* Per-pattern match counts of one stream (SURVEY.md §8a K4/K5 `count[stream][pattern]`, the
 * per-stream record the ranks gather, §8e): counts[p] = parsed lines whose content matches
 * pattern p (klf_config order; a line matching several patterns counts for each), for
 * p < min(cap, n_patterns); *n = n_patterns.  Independent of --since / --tail, like
 * klf_counts.matched.  The run must set KLF_FILTER_PATTERN_COUNTS (KLF_ESTATE otherwise).
 * A pattern that matches every content (an empty --grep, a regex such as `x*`) counts every
 * parsed line, also beside other patterns, whose counts are then evaluated as usual (their
 * tables are compiled on the first run that asks for counts).  Extends the size report of printLogSize
 * (cmd/root.go:279-309) with the new --grep / --match flags (:485-497). */
int klf_result_pattern_counts(klf_result* r, uint32_t stream_id, uint64_t* counts, uint32_t cap, uint32_t* n);
/* Position of the stream's last unparseable newline-terminated line, counted from the end
 * over the newline-terminated lines (1 = the last one; 0 = every terminated line parses).
 * The byte-range shards of one stream need it: kubelet emits the trailing
 * fragment when the --tail window holds an unparseable line (SPEC.md S4), and that line
 * may sit in an earlier shard.  Reads the latest run's line meta (KLF_ESTATE otherwise). */
int klf_result_last_unparsed(klf_result* r, uint32_t stream_id, uint64_t* rank);
/* Device views: the concatenated output and the stream's [off, len) in it.  No copy, except
 * for a one-pass result (KLF_COMPACT_ONEPASS), whose per-range extents the first call joins
 * into a second engine-owned device buffer the size of the output; that buffer is freed when
 * the engine's next run starts (the view is stale by then anyway) or at klf_close. */
int klf_result_device_out(klf_result* r, uint32_t stream_id, const uint8_t** d_out,
                          uint64_t* off, uint64_t* len);
/* Output write path: appends every stream's selected bytes to its open
 * file, fds[i] for stream i (fds[i] < 0 skips the stream), at the descriptor's current
 * offset with write(2), as io.Copy(logFile, logs) does in writeLogToDisk
 * (cmd/root.go:359-374).  The device output is copied D2H through 64 MiB pinned chunks,
 * double-buffered (DMA of the next 32 MiB while the current one is written).  With 8 MiB
 * or more of output and distinct descriptors, up to 8 worker threads (KLF_WRITE_THREADS
 * overrides) each own whole streams, so files are written in parallel and each file still
 * sees one in-order write(2) sequence; a descriptor shared by several streams gets them in
 * stream order from one thread.  EINTR and short writes are retried.  n_fds must equal
 * the stream count.  *written (optional) = bytes written over all streams.  KLF_EIO
 * (klf_last_error names the stream and errno text) reports the first failing write. */
int klf_result_write(klf_result* r, const int* fds, uint32_t n_fds, uint64_t* written);
/* Per-stage device time of the run in ms, HIP events on the launch stream:
 * [0] scan stage (newline + line index + timestamp + since + fused grep prefilter),
 * [1] pattern verification / matchers, [2] counts + tail + window prefix, [3] compaction
 * (these four only with KLF_FILTER_STAGE_TIMES, else 0), [4] total device time,
 * [5] workspace memsets (KLF_FILTER_STAGE_TIMES, else 0), [6] the k_scan kernel alone
 * (part of [0]): the start / end timestamps of its own dispatch (hipExtLaunchKernel
 * events, no event record beside it), [7] the dense copy kernel k_tcopy alone, the same way
 * (part of [3]; it exits at once when the run takes the sparse gather path).  With
 * KLF_GRAPH=1 a batch of at most KLF_GRAPH_MAX_MB (default 256) MiB whose run repeats the
 * previous run's arguments replays its launch sequence as a HIP graph: such a run reports
 * [4] only, a graph's replays recording no per-kernel events.  n = entries written. */
int klf_result_timing(const klf_result* r, double* ms, uint32_t cap, uint32_t* n);
/* Totals across streams. */
int klf_result_totals(const klf_result* r, klf_counts* totals);
/* KLF_INDEX_* of the run (klf_result_lines builds the rest on demand, after the run). */
int klf_result_index_mode(const klf_result* r);
/* klf_result_compaction: how the run put the selected bytes together in HBM. */
#define KLF_COMPACT_GATHER 0   /* line gather of the selected lines (--tail windows, sparse)   */
#define KLF_COMPACT_TILES 1    /* tile copy after the scan (most lines selected)               */
#define KLF_COMPACT_ONEPASS 2  /* in the scan itself, each tile range in place (no patterns,   */
                               /* --tail -1): a stream's output is a few extents in HBM, the   */
                               /* host views / klf_result_write join them, klf_result_device_out */
                               /* makes one contiguous copy on demand                          */
int klf_result_compaction(const klf_result* r);
void klf_result_free(klf_result* r);

/* ---- follow mode (-f) -------------------------------------------- */
/* The reference streams each container until EOF with Follow set (cmd/root.go:217-218,
 * streamLog :312-339, the "ended prematurely" warning :314-318) while the main goroutine
 * waits for 'q' (pressKeyToExit :399-421).  In follow mode the server keeps applying
 * SinceSeconds / TailLines to the backlog, so the engine applies what is per line: since
 * and the grep set (tail is -1; the filter's tail is ignored).  A session carries every
 * stream's open (unterminated) line across the chunks fed to it; each flush runs ONE engine
 * batch over the complete lines all streams received since the previous flush. */
typedef struct klf_follow klf_follow;
int klf_follow_open(klf_engine* e, const klf_filter* f, klf_follow** out);
/* Appends bytes read from stream `stream_id` (any split; concurrent calls for different
 * ids are safe, as klf_stage).  Complete lines are staged on the engine at once. */
int klf_follow_feed(klf_follow* fw, uint32_t stream_id, const uint8_t* p, size_t n);
/* Filters what is complete; final != 0 also flushes every stream's open line (the streams'
 * EOF: kubelet emits the last unterminated line).  *out covers stream ids [0, max id fed];
 * a stream fed nothing since the last flush has 0 lines.  The previous flush's result
 * stays valid until this call (results of the session share the engine's workspace). */
int klf_follow_flush(klf_follow* fw, int final, klf_result** out);
/* Bytes of the stream's open line (received, not yet filtered). */
uint64_t klf_follow_open_bytes(const klf_follow* fw, uint32_t stream_id);
void klf_follow_close(klf_follow* fw);

/* ---- host-side helpers mirroring cmd/root.go (no GPU needed) ---------------------- */
/* Go time.Parse(time.RFC3339Nano, s) restated (SPEC.md S2); 0 = ok. */
int klf_parse_rfc3339nano(const uint8_t* s, size_t n, klf_time* out);

#ifdef __cplusplus
}
#endif
#endif /* KLF_H */
