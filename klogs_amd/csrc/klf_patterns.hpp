// klf_patterns.hpp — host-side compilation of --grep / --match pattern sets into the
// tables the GPU matchers read.
//
//   * literals (Go bytes.Contains) -> one fused literal scan (single literal) or an
//     Aho-Corasick DFA over byte classes (several literals);
//   * regexes (Go regexp.Match, SPEC.md S5 RE2 subset) -> one Glushkov position
//     automaton per regex, simulated bit-parallel (one 64-bit state word per regex).
//
// Zero-width assertions (^ $ \A \z) are Glushkov positions evaluated at text
// boundaries; content never contains '\n', so only the two ends of the content can
// satisfy them (SPEC.md S5).
#pragma once
#include <stdint.h>
#include <stddef.h>

#include <array>
#include <string>
#include <vector>

namespace klf {

constexpr int kMaxRegexPositions = 64;  // one u64 state word per regex
constexpr int kMaxRegexes = 1024;

struct GlushkovTables {
  // per-position tables (bit p = position p)
  std::vector<uint64_t> follow;  // [npos]
  uint64_t first = 0;            // entered at every boundary (unanchored search)
  uint64_t last = 0;             // a completed position in `last` = match
  uint64_t init0 = 0;            // entered set at boundary 0 (BOT closure of first)
  uint64_t end_accept = 0;       // entered at the end boundary -> match via EOT closure
  bool accept_at_start = false;  // matches at boundary 0 of a non-empty content
  bool accept_empty = false;     // matches the empty content
  std::vector<std::vector<uint8_t>> pos_bytes;  // byte set (256 flags) per position
  std::vector<std::array<uint64_t, 4>> pos_bits;  // the same sets as 256-bit masks
  int npos = 0;
};

// Aho-Corasick DFA over a literal set (byte classes; a state's missing edges are its fail
// state's, so every byte is one table step).
struct AcTables {
  uint32_t states = 0, classes = 0;
  std::vector<uint8_t> cls;       // [256] byte -> class
  std::vector<uint32_t> next;     // [states * classes]
  std::vector<uint8_t> accept;    // [states] 1 if a literal ends here (via fail links)
  std::vector<int32_t> out;       // [states] id of the literal ending exactly here, -1 none
  std::vector<uint32_t> dict;     // [states] nearest fail-chain state with out >= 0 (0 none)
};
// The literals' byte classes need at most 255 (class 0 = bytes in no literal): checked
// before the build, so a deferred build cannot fail.
bool ac_alphabet_ok(const std::vector<std::vector<uint8_t>>& lits);
// lits: sorted, deduplicated (ids = positions), no empty literal.
void build_ac(const std::vector<std::vector<uint8_t>>& lits, AcTables& t);

struct CompiledSet {
  enum Mode : uint32_t {
    kNone = 0,      // no patterns: G = every line
    kNever = 1,     // patterns given but none can ever match content
    kAll = 2,       // some pattern matches every content: G = parsed lines
    kLiteral1 = 3,  // exactly one effective pattern, a literal of length 1..256
    kGeneral = 4,   // AC over literals and/or Glushkov regexes
  };
  Mode mode = kNone;
  // kGeneral only: the set also holds a pattern that matches every content (an empty
  // --grep, or a regex such as `x*`).  The filter is then kAll's (every parsed line); the
  // other patterns are compiled so that a run with per-pattern counts can evaluate them.
  bool also_all = false;
  // compile_set(defer_also_all): such a set comes back as kAll with also_all_pending set and
  // no matcher tables; the engine compiles it in full on the first run that asks for
  // per-pattern counts (a run without them never reads the tables)
  bool also_all_pending = false;
  std::vector<uint8_t> literal;  // kLiteral1
  uint32_t literal_anchor = 0;   // kLiteral1: index of its rarest byte in log text

  // kGeneral: Aho-Corasick over the literals (empty when no literal).  compile_set(defer_ac)
  // leaves it unbuilt (ac_states 0) and the literals in ac_lits: the engine builds and
  // uploads it on a host thread while its first run samples the data and places the needles
  // (the automaton serves only deferred lines and the fallback matcher).
  std::vector<std::vector<uint8_t>> ac_lits;
  uint32_t ac_states = 0;
  uint32_t ac_classes = 0;
  std::vector<uint8_t> ac_class;    // [256] byte -> class
  std::vector<uint32_t> ac_next;    // [states * classes]
  std::vector<uint8_t> ac_accept;   // [states] 1 if a literal ends here (via fail links)
  std::vector<int32_t> ac_out;      // [states] id of the literal ending exactly here, -1 none
  std::vector<uint32_t> ac_dict;    // [states] nearest fail-chain state with ac_out >= 0 (0 none)

  // per-pattern counts: compiled ids = literals (sorted, deduplicated) then regexes
  static constexpr int32_t kCidNever = -1, kCidAlways = -2;
  uint32_t n_cids = 0, n_lits = 0;
  std::vector<int32_t> user_map;    // [patterns] compiled id, or kCid* for the special cases

  // kGeneral: regexes.  Byte classes shared by all regexes (partition refinement).
  uint32_t rx_count = 0;
  uint32_t rx_classes = 0;
  std::vector<uint8_t> rx_class;      // [256]
  std::vector<uint64_t> rx_b;         // [rx_count * rx_classes] positions accepting class
  std::vector<uint64_t> rx_follow;    // [rx_count * 64]
  std::vector<uint64_t> rx_first, rx_last, rx_init0, rx_end;  // [rx_count]
  std::vector<uint32_t> rx_flags;     // bit0 accept_at_start, bit1 accept_empty
  std::vector<uint32_t> rx_pre;       // bound on match start -> first factor occurrence (prefilter on)
  uint32_t rx_maxpos = 0;             // most Glushkov positions of any regex

  // kGeneral: q-gram prefilter fused into the scan (qf_on).  Needles = the literals
  // (final: a verified hit is a match) and one required factor set per regex (a verified
  // hit makes the line a candidate the Glushkov NFA then decides).  Sampled positions
  // p (qf_sampled: 0 mod qf_stride, or the 3-per-16-B grid for 6) of every 8 KiB tile probe
  // a hashed bitmap of the needles' q-grams at window offsets 0..stride-1; bitmap hits are
  // verified against the needles of the bucket.
  bool qf_on = false;
  uint32_t qf_q = 4;         // gram length (bytes)
  uint32_t qf_stride = 1;    // 1, 2, 4, 6 (grid) or 8
  uint32_t qf_fold = 0;      // 0x20202020 when some needle compares case-insensitively
  uint32_t qf_mask = ~0u;    // gram bytes (q < 4: low q bytes)
  uint32_t qf_k = 3;         // bitmap bits per gram (qf_bits)
  std::vector<uint32_t> qf_bitmap;   // [kQfWords]: qf_k bits of word qf_word(qf_hash) per gram
  std::vector<uint32_t> qf_head;     // [kQfWords + 1] bucket (= bitmap word) -> first entry
  std::vector<uint32_t> qf_ent;      // 16-B entries {needle dword offset, len | k << 16 | flags,
                                     //  regex, first needle dword}; k = offset of the gram
  std::vector<uint32_t> qf_nbytes;   // needle bytes, each padded to whole dwords
  uint32_t qf_needles = 0;
  std::vector<std::string> qf_needle;  // literal / factor bytes (loose: OR 0x20)
  std::vector<uint32_t> qf_nflags, qf_nrx;
  bool qf_tuned = false;               // windows placed from the data's gram histogram
  std::string qf_why;                // why the prefilter is off (diagnostics)
  // Short needles: a needle shorter than the window q + S - 1 of the stride the others
  // allow (S = 8 needs 10 bytes at q = 3) is not sampled by the probes.  When every short
  // needle holds one byte that is rare in the data (the anchor), the scan tests each 16-B
  // chunk for that byte (one SWAR any-test, like the newline test), pre-checks the dword at
  // each anchor against the short needles' bytes there, and records the passing anchors as
  // hits; their bucket entries (k = the anchor's offset in the needle) sit beside the
  // probed ones, so k_verify walks both alike.  Off: every needle is probed (stride by the
  // shortest needle).
  bool qf_anc_on = false;
  uint32_t qf_anc_byte = 0;          // the anchor byte (loose short needles: compared OR 0x20)
  uint32_t qf_anc_fold = 0;          // 0x20202020 when a short needle is loose
  double qf_anc_share = 0;           // the anchor's estimated share of data bytes
  std::vector<uint32_t> qf_anc_pre;  // {want, mask} pairs: (dword at the anchor | qf_fold) & mask == want
  std::vector<uint8_t> qf_nshort;    // [needles] 1: anchored (not probed)
  std::vector<uint32_t> qf_nanc;     // [needles] offset of the anchor byte in a short needle
  std::string qf_layout;             // diagnostics: the chosen layout
  // The needle sets the layout picks from (one per factor choice of the regexes: [0] the
  // shortest needle's stride kept, [1] factors of >= 10 bytes preferred); the chosen one
  // is copied into qf_needle / qf_nflags / qf_nrx and its bounds into rx_pre.
  struct NeedleSet {
    std::vector<std::string> s;
    std::vector<uint32_t> flags, rx, rx_pre;
  };
  std::vector<NeedleSet> qf_variants;
  uint32_t qf_variant = 0;
};

// Statistics of a data sample (k_gramhist, first batch): the exact 2-gram counts (fold
// applied, at even positions, scaled to every position) and the byte histogram.
struct DataStats {
  std::vector<uint32_t> pair;   // [65536] 2-gram b0 | b1 << 8
  std::vector<uint64_t> bytes;  // [256]
  uint64_t nbytes = 0;          // positions counted in `bytes`
  // derived by stats_finish: 2-gram marginals and their total, and the reciprocals
  // gram_share multiplies by (it runs ~20 K times per layout candidate of a large set)
  std::vector<double> marg;
  double pair_tot = 0;
  double inv_tot = 0;
  std::vector<double> inv_marg;  // [256] tot / (marg + 128)
};
// The derived fields, once the counts are in.
void stats_finish(DataStats& st);
// Estimated share of the data's positions that hold gram g (q bytes, folded): a
// first-order Markov chain over the exact 2-gram counts, which resolves shares far below
// one occurrence per sample (round 3's count-min sketches of the 3- and 4-grams saw only
// their collision noise there).
double gram_share(const DataStats& st, uint32_t g, uint32_t q);
constexpr uint32_t kQfAncPreMax = 8;  // distinct short-needle pre-check dwords

// Required literal factors of one regex (Go syntax, SPEC.md S5): every match contains
// one of `alts`; `loose` when some byte is an ASCII case pair ((?i)), then every byte is
// stored OR 0x20 and compared that way.  *pre (nullable): bound on the distance from a
// match's start to its first factor occurrence (kRxPreUnbounded: none).  want: sets
// whose shortest string has at least `want` bytes are preferred (then a bounded pre,
// then length).  False when the regex has no factor.
constexpr uint32_t kRxPreUnbounded = 0xFFFFFFFFu;
bool regex_factors(const uint8_t* pat, size_t n, std::vector<std::string>& alts, bool& loose,
                   uint32_t* pre = nullptr, size_t want = SIZE_MAX);

// Host twin of k_gramhist over one sample (tests / diagnostics): the 2-grams (OR fold) at
// even positions, every byte into the histogram.
void data_stats(const uint8_t* p, size_t n, uint32_t fold, DataStats& st);

// Diagnostics of the prefiltered scan over `data` with the current layout: sampled
// positions, bitmap hits, anchor hits (pre-check passed), verified needle occurrences.
struct PrefilterHits {
  uint64_t probes = 0, bitmap_hits = 0, anchor_hits = 0, verified = 0;
  uint64_t pair_pass = 0;  // two-level probe: samples past the exact 2-gram stage
};
PrefilterHits prefilter_hits(const CompiledSet& cs, const uint8_t* data, size_t n);

// (Re)chooses the prefilter layout (stride, gram length, short-needle anchor) and places
// every needle's sampling window, rebuilding the bitmap and buckets; st = statistics of a
// data sample (the first batch) or null for the byte-class estimates.
void place_needles(CompiledSet& cs, const DataStats* st);

// Regex r over content s[0, n) restricted to matches holding the factor occurrence that
// starts at x: starts in [x - rx_pre[r], x], then no new start (the GPU's k_nfa).
bool nfa_window(const CompiledSet& cs, uint32_t r, const uint8_t* s, size_t n, size_t x);

// Host emulation of the prefiltered matcher on one content (tests): sampled positions
// p = phase mod stride, bitmap probe, bucket verification, NFA over each factor
// occurrence's window.
bool prefilter_match(const CompiledSet& cs, const uint8_t* s, size_t n, uint32_t phase);

// Parses one Go-syntax regex (SPEC.md S5) and builds its Glushkov tables.
// Returns false with `err` set for syntax outside the subset or > 64 positions.
bool compile_regex(const uint8_t* pat, size_t n, GlushkovTables& out, std::string& err,
                   int& err_code);

// Compiles a whole OR'ed pattern set.  kinds[i]: 0 literal, 1 regex.  place = false leaves
// the prefilter layout (qf_stride, windows, bitmap, buckets) to a later place_needles call
// with the first batch's statistics (the engine's first run): placing without them first
// is wasted work on the klf_open path.
bool compile_set(const std::vector<std::vector<uint8_t>>& pats, const std::vector<uint32_t>& kinds,
                 CompiledSet& out, std::string& err, int& err_code, bool place = true,
                 bool defer_also_all = false, bool defer_ac = false);

// Expected-frequency class of a byte in log text (lower = rarer); picks scan anchors.
int log_byte_class(uint8_t c);

// Host reference simulation of one compiled regex on a content (used by unit tests of
// the compiler through klf_debug_regex_match; the GPU kernel runs the same recurrence).
bool glushkov_match(const GlushkovTables& g, const uint8_t* s, size_t n);

}  // namespace klf
