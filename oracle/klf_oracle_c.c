/* klf_oracle_c.c — C restatement of the klogs filter path.  TEST INFRASTRUCTURE ONLY:
 * linked by tests/ (the checker of the HIP engine at sizes Python cannot reach) and by
 * bench.py's cpu_baseline leg (kind "port").  The product never loads it.
 *
 * Written independently of the engine (no shared source with klogs_amd/csrc):
 *   - ko_parse_ts:   Go 1.22 time.Parse(RFC3339Nano) restated chunk by chunk the way
 *                    src/time/format.go's parse loop walks the layout (getnum, skip,
 *                    stdFracSecond9 / parseNanoseconds, stdISO8601ColonTZ, daysIn);
 *   - tail:          kubelet pkg/util/tail/tail.go FindTailLineStartIndex restated with
 *                    its 1024-byte backward block scan;
 *   - read loop:     kubelet pkg/kubelet/kuberuntime/logs/logs.go ReadLogs (limitedNum
 *                    decremented per parsed line, unparseable lines skipped uncounted)
 *                    + logWriter.write (drop ts.Before(since));
 *   - grep:          Go bytes.Contains via memmem over the content without its '\n'
 *                    (sets of more than 8 literals: an Aho-Corasick DFA, same answer);
 *   - match:         Go regexp.Match, in klf_oracle_rx.c (ko_filter_rx: its own parser of the
 *                    SPEC.md S5 subset, Thompson NFA, lazy DFA), through ko_filter_impl below.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t lines, parsed, since_ok, matched, selected, out_bytes;
} ko_counts;

/* ---- time.Parse("2006-01-02T15:04:05.999999999Z07:00", v) ------------------------ */
static int isdig(const uint8_t* v, size_t n, size_t i) { return i < n && v[i] >= '0' && v[i] <= '9'; }

/* getnum(s, fixed): 1 or 2 digits (2 when fixed) starting at *i */
static int getnum(const uint8_t* v, size_t n, size_t* i, int fixed, int* out) {
  if (!isdig(v, n, *i)) return 0;
  if (!isdig(v, n, *i + 1)) {
    if (fixed) return 0;
    *out = v[*i] - '0';
    *i += 1;
    return 1;
  }
  *out = (v[*i] - '0') * 10 + (v[*i + 1] - '0');
  *i += 2;
  return 1;
}
static int skip(const uint8_t* v, size_t n, size_t* i, char c) {
  if (*i >= n || v[*i] != (uint8_t)c) return 0;
  *i += 1;
  return 1;
}
static int leap(int64_t y) { return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0); }
static int days_in(int m, int64_t y) {
  static const int d[13] = {0, 31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return m == 2 && leap(y) ? 29 : d[m];
}
/* days from 0000-03-01-based count (different formulation from the engine's) */
static int64_t days_since_epoch(int64_t y, int m, int d) {
  /* count days from 0000-01-01 then shift: the proleptic Gregorian calendar */
  int64_t days = y * 365 + (y + 3) / 4 - (y + 99) / 100 + (y + 399) / 400; /* days before Jan 1 of year y */
  static const int cum[13] = {0, 0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
  days += cum[m] + (m > 2 && leap(y) ? 1 : 0) + (d - 1);
  return days - 719528; /* 1970-01-01 */
}

/* Parses v[0..n) entirely; returns 1 on success. */
int ko_parse_ts(const uint8_t* v, size_t n, int64_t* sec_out, int32_t* nsec_out) {
  size_t i = 0;
  int64_t year;
  int month, day, hour, min, sec;
  /* stdLongYear */
  if (n < 4 || !isdig(v, n, 0)) return 0;
  for (int k = 0; k < 4; ++k)
    if (!isdig(v, n, (size_t)k)) return 0;
  year = (v[0] - '0') * 1000 + (v[1] - '0') * 100 + (v[2] - '0') * 10 + (v[3] - '0');
  i = 4;
  if (!skip(v, n, &i, '-') || !getnum(v, n, &i, 1, &month) || month < 1 || month > 12) return 0;
  if (!skip(v, n, &i, '-') || !getnum(v, n, &i, 1, &day)) return 0;
  if (!skip(v, n, &i, 'T') || !getnum(v, n, &i, 0, &hour) || hour >= 24) return 0;
  if (!skip(v, n, &i, ':') || !getnum(v, n, &i, 1, &min) || min >= 60) return 0;
  if (!skip(v, n, &i, ':') || !getnum(v, n, &i, 1, &sec) || sec >= 60) return 0;
  int64_t nsec = 0;
  if (n - i >= 2 && (v[i] == '.' || v[i] == ',') && isdig(v, n, i + 1)) {
    size_t j = 0;
    while (i + j + 1 < n && isdig(v, n, i + j + 1)) ++j;
    size_t nbytes = 1 + j; /* parseNanoseconds(value, 1+j) */
    size_t take = nbytes > 10 ? 10 : nbytes;
    for (size_t k = 1; k < take; ++k) nsec = nsec * 10 + (v[i + k] - '0');
    for (size_t k = take; k < 10; ++k) nsec *= 10;
    i += nbytes;
  }
  int64_t off = 0;
  if (i < n && v[i] == 'Z') {
    i += 1;
  } else {
    if (n - i < 6 || v[i + 3] != ':') return 0;
    int hh, mm;
    size_t a = i + 1, b = i + 4;
    if (!getnum(v, i + 3, &a, 1, &hh) || !getnum(v, i + 6, &b, 1, &mm)) return 0;
    if (hh > 24 || mm > 60) return 0;
    off = (int64_t)(hh * 60 + mm) * 60;
    if (v[i] == '-') off = -off;
    else if (v[i] != '+') return 0;
    i += 6;
  }
  if (i != n) return 0; /* extra text */
  if (day < 1 || day > days_in(month, year)) return 0;
  *sec_out = days_since_epoch(year, month, day) * 86400 + hour * 3600 + min * 60 + sec - off;
  *nsec_out = (int32_t)nsec;
  return 1;
}

/* parseCRILog-style: ts = line[:first ' '] */
static int parse_line(const uint8_t* l, size_t n, int64_t* s, int32_t* ns, size_t* plen) {
  const uint8_t* sp = memchr(l, ' ', n);
  if (!sp) return 0;
  size_t idx = (size_t)(sp - l);
  if (!ko_parse_ts(l, idx, s, ns)) return 0;
  *plen = idx + 1;
  return 1;
}

static int before(int64_t s1, int32_t n1, int64_t s2, int32_t n2) { return s1 < s2 || (s1 == s2 && n1 < n2); }

/* FindTailLineStartIndex over buf[0..size) */
static uint64_t find_tail_start(const uint8_t* buf, uint64_t size, int64_t n) {
  if (n < 0) return 0;
  const uint64_t bs = 1024;
  uint64_t left = 0, right = size, blen = 0;
  int64_t cnt = 0;
  const uint8_t* blk = buf;
  while (right > 0 && cnt <= n) {
    left = right >= bs ? right - bs : 0;
    blk = buf + left;
    blen = right - left;
    for (uint64_t k = 0; k < blen; ++k) cnt += blk[k] == '\n';
    right = right >= bs ? right - bs : 0;
  }
  while (cnt > n) {
    const uint8_t* p = memchr(blk, '\n', blen);
    uint64_t idx = (uint64_t)(p - blk) + 1;
    blk += idx;
    blen -= idx;
    left += idx;
    --cnt;
  }
  return left;
}

/* Large literal sets (C4: 1,024 literals): OR of bytes.Contains through a textbook
 * Aho-Corasick automaton (goto trie, BFS failure links, completed into a 256-way DFA; a
 * state accepts when some literal ends there or on its failure chain), one table step per
 * content byte instead of one memmem per literal.  Small sets keep memmem. */
typedef struct {
  int32_t* next;  /* [states * nc]: byte classes (the literals' bytes, one class each; the rest 0) */
  uint8_t* acc;   /* [states] */
  int32_t n, nc;
  uint16_t cls[256];  /* class per byte: 0 = in no literal, else 1..256 */
  int32_t* wide;      /* small automata: [states * 256] by raw byte, bit 30 = the target accepts
                         (one dependent load per byte instead of two) */
} ko_ac;

static void ac_free(ko_ac* a) {
  free(a->next);
  free(a->acc);
  free(a->wide);
  a->next = NULL;
  a->acc = NULL;
  a->wide = NULL;
}

/* fold: ASCII letters compare case-insensitively (an upper-case byte takes its lower-case
 * byte's class; the literals are given lower-cased). */
static int ac_build_fold(ko_ac* a, uint32_t n_lit, const uint8_t* const* lits, const uint64_t* lens, int fold) {
  uint64_t cap = 1;
  for (uint32_t k = 0; k < n_lit; ++k) cap += lens[k];
  memset(a->cls, 0, sizeof a->cls);
  a->nc = 1;
  for (uint32_t k = 0; k < n_lit; ++k)
    for (uint64_t j = 0; j < lens[k]; ++j)
      if (!a->cls[lits[k][j]]) a->cls[lits[k][j]] = (uint16_t)a->nc++;
  if (fold)
    for (int c = 'A'; c <= 'Z'; ++c) a->cls[c] = a->cls[c | 0x20];
  const int NC = a->nc;  /* <= 257: class 0 = bytes in no literal */
  a->next = (int32_t*)malloc(cap * NC * sizeof(int32_t));
  a->acc = (uint8_t*)calloc(cap, 1);
  int32_t* fail = (int32_t*)malloc(cap * sizeof(int32_t));
  int32_t* queue = (int32_t*)malloc(cap * sizeof(int32_t));
  if (!a->next || !a->acc || !fail || !queue) { free(fail); free(queue); ac_free(a); return -1; }
  for (uint64_t i = 0; i < cap * NC; ++i) a->next[i] = -1;
  a->n = 1;
  for (uint32_t k = 0; k < n_lit; ++k) {  /* goto trie */
    int32_t st = 0;
    for (uint64_t j = 0; j < lens[k]; ++j) {
      int32_t* t = &a->next[(uint64_t)st * NC + a->cls[lits[k][j]]];
      if (*t < 0) *t = a->n++;
      st = *t;
    }
    a->acc[st] = 1;
  }
  uint64_t qh = 0, qt = 0;  /* BFS: root's missing edges loop to the root */
  for (int c = 0; c < NC; ++c) {
    int32_t* t = &a->next[c];
    if (*t < 0 || c == 0) { *t = 0; continue; }
    fail[*t] = 0;
    queue[qt++] = *t;
  }
  while (qh < qt) {
    const int32_t u = queue[qh++];
    a->acc[u] |= a->acc[fail[u]];
    for (int c = 0; c < NC; ++c) {
      int32_t* t = &a->next[(uint64_t)u * NC + c];
      const int32_t via_fail = a->next[(uint64_t)fail[u] * NC + c];
      if (*t < 0) { *t = via_fail; continue; }
      fail[*t] = via_fail;
      queue[qt++] = *t;
    }
  }
  free(fail);
  free(queue);
  a->wide = NULL;
  if ((uint64_t)a->n * 256 <= (1u << 19) && (a->wide = (int32_t*)malloc((size_t)a->n * 256 * sizeof(int32_t))))
    for (int32_t st = 0; st < a->n; ++st)
      for (int c = 0; c < 256; ++c) {
        const int32_t t = a->next[(uint64_t)st * NC + a->cls[c]];
        a->wide[(size_t)st * 256 + c] = t | (a->acc[t] ? (1 << 30) : 0);
      }
  return 0;
}
/* 1 when some literal occurs in c[0, cn) */
static int ac_scan(const ko_ac* a, const uint8_t* c, size_t cn) {
  int32_t st = 0;
  if (a->wide) {
    for (size_t i = 0; i < cn; ++i) {
      st = a->wide[(size_t)st * 256 + c[i]];
      if (st & (1 << 30)) return 1;
    }
    return 0;
  }
  for (size_t i = 0; i < cn; ++i) {
    st = a->next[(uint64_t)st * a->nc + a->cls[c[i]]];
    if (a->acc[st]) return 1;
  }
  return 0;
}
static int ac_build(ko_ac* a, uint32_t n_lit, const uint8_t* const* lits, const uint64_t* lens) {
  return ac_build_fold(a, n_lit, lits, lens, 0);
}

static int content_matches(const uint8_t* c, size_t cn, uint32_t n_lit, const uint8_t* const* lits,
                           const uint64_t* lens, const ko_ac* ac) {
  if (cn && c[cn - 1] == '\n') --cn;
  for (uint32_t k = 0; k < n_lit; ++k)
    if (lens[k] == 0) return 1;
  if (ac && ac->next) return ac_scan(ac, c, cn);
  for (uint32_t k = 0; k < n_lit; ++k)
    if (lens[k] <= cn && memmem(c, cn, lits[k], lens[k])) return 1;
  return 0;
}

/* The line matcher of one filter call: content (its '\n' included or not) -> match.
 * ko_filter_impl is the kubelet read loop every matcher shares (exported for
 * klf_oracle_rx.c). */
typedef int (*ko_match_fn)(void* ctx, const uint8_t* c, size_t cn);

int64_t ko_filter_impl(const uint8_t* data, uint64_t n, int64_t since_sec, int32_t since_nsec, int64_t tail,
                           int grep_active, ko_match_fn match, void* mctx, uint8_t* out, uint64_t* line_off,
                           uint64_t line_cap, uint8_t* match_bits, ko_counts* cnt) {
  ko_counts c;
  memset(&c, 0, sizeof(c));
  /* pass 1: lines, counts, G */
  uint8_t* gfile = NULL;
  uint64_t glen = 0, gcap = 0;
  const uint8_t* gbuf = data;
  uint64_t gsize = n;
  uint64_t pos = 0, li = 0;
  while (pos < n) {
    const uint8_t* nl = memchr(data + pos, '\n', n - pos);
    const uint64_t end = nl ? (uint64_t)(nl - data) + 1 : n;
    if (line_off && li < line_cap) line_off[li] = pos;
    int64_t s;
    int32_t ns;
    size_t plen;
    const int ok = parse_line(data + pos, end - pos, &s, &ns, &plen);
    if (ok) {
      c.parsed++;
      if (!before(s, ns, since_sec, since_nsec)) c.since_ok++;
    }
    if (grep_active) {
      const int hit = ok && match(mctx, data + pos + plen, end - pos - plen);
      if (hit) {
        if (match_bits) match_bits[li >> 3] |= (uint8_t)(1u << (li & 7));
        c.matched++;
        if (glen + (end - pos) > gcap) {
          gcap = (gcap + (end - pos)) * 2;
          uint8_t* g2 = (uint8_t*)realloc(gfile, gcap);
          if (!g2) { free(gfile); return -1; }
          gfile = g2;
        }
        memcpy(gfile + glen, data + pos, end - pos);
        glen += end - pos;
      }
    } else {
      c.matched++;
    }
    pos = end;
    ++li;
  }
  c.lines = li;
  if (line_off && li < line_cap) line_off[li] = n;
  if (grep_active) { gbuf = gfile; gsize = glen; }
  /* pass 2: kubelet ReadLogs over G */
  uint64_t p = find_tail_start(gbuf, gsize, tail);
  const int limited = tail >= 0;
  int64_t left = tail;
  uint64_t o = 0;
  int stop = 0;
  for (;;) {
    if (stop || (limited && left == 0)) break;
    if (p >= gsize) { stop = 1; continue; }
    const uint8_t* nl = memchr(gbuf + p, '\n', gsize - p);
    uint64_t end = nl ? (uint64_t)(nl - gbuf) + 1 : gsize;
    if (!nl) stop = 1;
    int64_t s;
    int32_t ns;
    size_t plen;
    if (parse_line(gbuf + p, end - p, &s, &ns, &plen)) {
      if (!before(s, ns, since_sec, since_nsec)) {
        memcpy(out + o, gbuf + p + plen, end - p - plen);
        o += end - p - plen;
        c.selected++;
      }
      if (limited) --left;
    }
    p = end;
  }
  free(gfile);
  c.out_bytes = o;
  if (cnt) *cnt = c;
  return (int64_t)o;
}

typedef struct {
  uint32_t n_lit;
  const uint8_t* const* lits;
  const uint64_t* lens;
  const ko_ac* ac;
} lit_ctx;
static int lit_match(void* ctx, const uint8_t* c, size_t cn) {
  const lit_ctx* x = (const lit_ctx*)ctx;
  return content_matches(c, cn, x->n_lit, x->lits, x->lens, x->ac);
}

/* Filters one stream.  out: capacity >= n.  line_off (nullable): capacity line_cap, gets
 * lines+1 entries when they fit.  match_bits (nullable, only with literals): capacity
 * ceil(lines/8) bytes, zeroed by the caller.  Returns the output length, or -1 on error. */
int64_t ko_filter(const uint8_t* data, uint64_t n, int64_t since_sec, int32_t since_nsec, int64_t tail,
                  int grep_active, uint32_t n_lit, const uint8_t* const* lits, const uint64_t* lit_lens, uint8_t* out,
                  uint64_t* line_off, uint64_t line_cap, uint8_t* match_bits, ko_counts* cnt) {
  ko_ac ac;
  memset(&ac, 0, sizeof ac);
  if (grep_active && n_lit > 8 && ac_build(&ac, n_lit, lits, lit_lens) != 0) return -1;
  lit_ctx x = {n_lit, lits, lit_lens, &ac};
  const int64_t r = ko_filter_impl(data, n, since_sec, since_nsec, tail, grep_active, lit_match, &x, out, line_off,
                                line_cap, match_bits, cnt);
  ac_free(&ac);
  return r;
}
