/* klf_synth.c — seeded synthetic kubelet log streams (Timestamps=true format) for the
 * tests and bench.py.  Test/bench infrastructure, not part of the filter path.
 *
 * Every line is a pure function of (seed, stream, line index): line i of stream s uses
 * key k_i = mix(mix(seed ^ 0x5851F42D4C957F2D * (s + 1)) + i), so generation is
 * parallel (lengths first, exclusive prefix, then per-thread fills) and reproducible.
 *
 * Kinds:
 *   KS_TEXT  (C1/C3): content length from a lognormal(median 96, sigma 0.7) quantile
 *            table clamped to [16, 1024]; words from a fixed vocabulary.
 *   KS_JSON  (C2/C4): {"ts":...,"level":...,"msg":...,"trace":...}, 200..599 bytes;
 *            `needle_permille` of the lines carry `needle` inside msg.
 *   KS_ADVERSARIAL: valid and invalid RFC3339Nano prefixes (fraction digits 0..12, ','
 *            separator, +-hh:mm offsets, one-digit hours, out-of-range fields), missing
 *            delimiters, empty lines, CRLF, non-monotonic timestamps, long lines, NUL and
 *            high bytes, needle hits; sequential (small sizes only).
 * Timestamps of TEXT/JSON are monotonic: t0 + i * step, step = span / estimated lines,
 * fixed-width "YYYY-MM-DDTHH:MM:SS.nnnnnnnnnZ ".
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define KS_TEXT 0
#define KS_JSON 1
#define KS_ADVERSARIAL 2
#define KS_MIXED 3    /* C4: mixed-length word lines, 16 B..8 KiB (lognormal), literal hits   */
#define KS_LONGJSON 4 /* C5: long JSON lines, 1..32 KiB (log-uniform), regex events + misses */
#define KS_C4_LITS 1024

static inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static const uint16_t kLogn[256] = {
    16,  16,  19,  20,  22,  23,  24,  26,  27,  28,  28,  29,  30,  31,  32,  32,  33,  34,  35,  35,  36,  37,
    37,  38,  38,  39,  40,  40,  41,  41,  42,  43,  43,  44,  44,  45,  45,  46,  47,  47,  48,  48,  49,  49,
    50,  50,  51,  51,  52,  52,  53,  53,  54,  54,  55,  55,  56,  57,  57,  58,  58,  59,  59,  60,  60,  61,
    61,  62,  62,  63,  63,  64,  64,  65,  65,  66,  66,  67,  67,  68,  68,  69,  70,  70,  71,  71,  72,  72,
    73,  73,  74,  74,  75,  75,  76,  77,  77,  78,  78,  79,  79,  80,  80,  81,  82,  82,  83,  83,  84,  85,
    85,  86,  86,  87,  87,  88,  89,  89,  90,  91,  91,  92,  92,  93,  94,  94,  95,  96,  96,  97,  98,  98,
    99,  100, 100, 101, 102, 102, 103, 104, 105, 105, 106, 107, 108, 108, 109, 110, 111, 111, 112, 113, 114, 115,
    115, 116, 117, 118, 119, 120, 120, 121, 122, 123, 124, 125, 126, 127, 128, 129, 130, 131, 132, 133, 134, 135,
    136, 137, 138, 139, 140, 141, 142, 143, 145, 146, 147, 148, 149, 151, 152, 153, 155, 156, 157, 159, 160, 162,
    163, 165, 166, 168, 169, 171, 173, 174, 176, 178, 180, 181, 183, 185, 187, 189, 191, 194, 196, 198, 200, 203,
    205, 208, 211, 213, 216, 219, 222, 225, 229, 232, 236, 240, 244, 248, 252, 257, 261, 267, 272, 278, 284, 291,
    298, 306, 315, 324, 335, 347, 361, 377, 396, 419, 450, 492, 560, 724};

static const char* const kWords[32] = {
    "request", "handled", "user",  "session", "cache",  "miss",  "hit",     "db",     "query",   "took",    "ms",
    "status",  "ok",      "retry", "backoff", "pod",    "ready", "volume",  "mount",  "sync",    "config",  "reload",
    "worker",  "queue",   "depth", "latency", "bytes",  "sent",  "receive", "client", "upstream", "timeout"};
static const char* const kLevels[4] = {"INFO", "WARN", "DEBUG", "ERROR"};

static void civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  *d = (int)(doy - (153 * mp + 2) / 5 + 1);
  *m = (int)(mp < 10 ? mp + 3 : mp - 9);
  *y = yoe + era * 400 + (*m <= 2);
}

static void put_dig(uint8_t* p, uint64_t v, int n) {
  for (int i = n - 1; i >= 0; --i) { p[i] = (uint8_t)('0' + v % 10); v /= 10; }
}

/* "YYYY-MM-DDTHH:MM:SS.nnnnnnnnnZ" (30 bytes) for unix ns (>= 0) */
static void fmt_ts(uint8_t* p, int64_t ns) {
  int64_t sec = ns / 1000000000, nsec = ns % 1000000000;
  int64_t days = sec / 86400, sod = sec % 86400;
  int64_t y; int m, d;
  civil_from_days(days, &y, &m, &d);
  put_dig(p, (uint64_t)y, 4); p[4] = '-'; put_dig(p + 5, (uint64_t)m, 2); p[7] = '-'; put_dig(p + 8, (uint64_t)d, 2);
  p[10] = 'T'; put_dig(p + 11, (uint64_t)(sod / 3600), 2); p[13] = ':'; put_dig(p + 14, (uint64_t)(sod / 60 % 60), 2);
  p[16] = ':'; put_dig(p + 17, (uint64_t)(sod % 60), 2); p[19] = '.'; put_dig(p + 20, (uint64_t)nsec, 9); p[29] = 'Z';
}

typedef struct {
  uint32_t kind;
  uint64_t seed;
  uint32_t stream;
  int64_t t0_ns, step_ns;
  const uint8_t* needle;
  uint32_t needle_len, needle_permille;
} gen_cfg;

static inline uint64_t line_key(const gen_cfg* g, uint64_t i) {
  return mix(mix(g->seed ^ (0x5851F42D4C957F2Dull * (g->stream + 1ull))) + i);
}

/* ---- C4 literal vocabulary / C5 regex set ----------------------------------------- */
static const char* const kLitPrefix[8] = {"ERR_", "E", "TX-", "REQ", "ORA-", "HTTP_", "SIG", "KEY"};

/* Literal i of the C4 vocabulary: 6..24 bytes of [A-Z0-9_-] (log text is lower case). */
uint32_t ks_c4_literal(uint32_t i, uint8_t* out) {
  static const char al[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
  uint64_t r = mix(0xC4C4C4C4ull ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull));
  const uint32_t len = 6 + (uint32_t)(r % 19);
  const char* pre = kLitPrefix[(r >> 8) & 7];
  uint32_t o = 0;
  for (; pre[o] && o < len; ++o) out[o] = (uint8_t)pre[o];
  while (o < len) { r = mix(r); out[o++] = (uint8_t)al[r % 36]; }
  return len;
}

/* C5: 8 families x 8 variants (regex index = family * 8 + variant): the regex, a snippet
 * it matches, and a near miss that holds the regex's required factor but no match. */
static const char* const kC5[8][3] = {
    {"(?i)panic: \\w+ error in mod%u", "PANIC: runtime error in mod%u", "retry error in mod%u"},
    {"user%u_id=u\\d{4,6} (login|logout)", "user%u_id=u12345 logout", "user%u_id=u12 login"},
    {"status=5\\d\\d path=/api/v%u/\\w+", "status=503 path=/api/v%u/orders", "status=200 path=/api/v%u/orders"},
    {"tx-[0-9a-f]{8}-commit%u", "tx-0a1b2c3d-commit%u", "tx-0a1b-commit%u"},
    {"(?i)oom(killed|_score_adj) for pid%u=\\d+", "OOMKilled for pid%u=42", "oomfoo for pid%u=42"},
    {"shard%u deadline exceeded after \\d+\\.\\d+s", "shard%u deadline exceeded after 1.25s",
     "shard%u deadline exceeded after xs"},
    {"GET /v%u/items/\\d+ (4\\d\\d|5\\d\\d)", "GET /v%u/items/77 404", "GET /v%u/items/77 200"},
    {"(?i)conn(ection)? reset by peer%u", "Connection reset by peer%u", "pipe reset by peer%u"},
};

/* which: 0 regex, 1 matching snippet, 2 near miss.  Returns the length (no NUL). */
uint32_t ks_c5_pattern(uint32_t r, int which, char* out, uint32_t cap) {
  const int n = snprintf(out, cap, kC5[(r >> 3) & 7][which % 3], r & 7u);
  return n < 0 ? 0 : (uint32_t)n;
}

/* content length (without prefix and '\n') */
static uint32_t content_len(const gen_cfg* g, uint64_t k) {
  if (g->kind == KS_TEXT) return kLogn[k & 255];
  if (g->kind == KS_MIXED) {  /* lognormal-ish: median 180 B, clamped to 16 B .. 8 KiB */
    const uint64_t m = mix(k ^ 0x4D49ull);
    const double u = ((m & 0xFFFF) + ((m >> 16) & 0xFFFF) + ((m >> 32) & 0xFFFF) + ((m >> 48) & 0xFFFF)) / 65536.0;
    const double z = (u - 2.0) * 1.7320508075688772;
    double l = 180.0 * exp(1.1 * z);
    l = l < 16 ? 16 : (l > 8192 ? 8192 : l);
    return (uint32_t)l;
  }
  if (g->kind == KS_LONGJSON) /* log-uniform 1 KiB .. 32 KiB */
    return (uint32_t)(1024.0 * exp2(5.0 * (double)(mix(k ^ 0x10C6ull) >> 11) / 9007199254740992.0));
  return 200 + (uint32_t)((k >> 8) % 400); /* JSON */
}

static void fill_words(uint8_t* p, uint32_t n, uint64_t k) {
  uint32_t o = 0;
  uint64_t r = k;
  while (o < n) {
    r = mix(r);
    const char* w = kWords[r & 31];
    size_t wl = strlen(w);
    for (size_t j = 0; j < wl && o < n; ++j) p[o++] = (uint8_t)w[j];
    if (o < n) p[o++] = ((r >> 8) & 7) == 0 ? '=' : ' ';
    if (o < n && ((r >> 11) & 3) == 0) { p[o++] = (uint8_t)('0' + ((r >> 13) % 10)); }
  }
}

/* writes line i (prefix + content + '\n') at p; len must be 31 + content_len + 1 */
static void write_line(const gen_cfg* g, uint64_t i, uint64_t k, uint8_t* p, uint32_t clen) {
  const int64_t ns = g->t0_ns + (int64_t)i * g->step_ns;
  fmt_ts(p, ns);
  p[30] = ' ';
  uint8_t* c = p + 31;
  if (g->kind == KS_TEXT) {
    fill_words(c, clen, k);
  } else if (g->kind == KS_MIXED) {
    fill_words(c, clen, k);
    if (((k >> 32) % 1000) < g->needle_permille) {
      uint8_t lit[32];
      const uint32_t ll = ks_c4_literal((uint32_t)((k >> 42) % KS_C4_LITS), lit);
      if (ll + 2 <= clen) memcpy(c + 1 + (uint32_t)((k >> 20) % (clen - ll - 1)), lit, ll);
    }
  } else {
    /* {"ts":"<24>","level":"<L>","msg":"<...>","trace":"<32 hex>"} */
    static const char hex[] = "0123456789abcdef";
    uint32_t o = 0;
    const char* lv = kLevels[(k >> 20) & 3];
    char head[96];
    uint8_t tsb[30];
    fmt_ts(tsb, ns);
    memcpy(head, "{\"ts\":\"", 7);
    memcpy(head + 7, tsb, 23); /* millisecond resolution */
    memcpy(head + 30, "Z\",\"level\":\"", 12);
    size_t hl = 42;
    size_t ll = strlen(lv);
    memcpy(head + hl, lv, ll); hl += ll;
    memcpy(head + hl, "\",\"msg\":\"", 9); hl += 9;
    memcpy(c, head, hl); o = (uint32_t)hl;
    const uint32_t tail_len = 11 + 32 + 2; /* ","trace":" + 32 hex + "} */
    const uint32_t msg_len = clen - o - tail_len;
    fill_words(c + o, msg_len, k ^ 0xABCDEFull);
    if (g->kind == KS_LONGJSON) {  /* regex events (permille) and near misses (2 x permille) */
      const uint32_t ev = (uint32_t)((k >> 32) % 1000);
      if (ev < 3 * g->needle_permille) {
        char snip[96];
        const uint32_t sl = ks_c5_pattern((uint32_t)((k >> 42) % 64), ev < g->needle_permille ? 1 : 2, snip, sizeof snip);
        if (sl + 4 <= msg_len) {
          const uint32_t at = 1 + (uint32_t)((k >> 50) % (msg_len - sl - 2));
          c[o + at - 1] = ' ';
          memcpy(c + o + at, snip, sl);
          c[o + at + sl] = ' ';
        }
      }
    } else if (g->needle_len && g->needle_len + 2 <= msg_len && ((k >> 32) % 1000) < g->needle_permille) {
      const uint32_t at = (uint32_t)((k >> 42) % (msg_len - g->needle_len - 1)) + 1;
      memcpy(c + o + at, g->needle, g->needle_len);
    }
    o += msg_len;
    memcpy(c + o, "\",\"trace\":\"", 11); o += 11;
    uint64_t r = mix(k ^ 0x1234ull);
    for (int j = 0; j < 32; ++j) { if ((j & 15) == 0) r = mix(r); c[o++] = (uint8_t)hex[(r >> (4 * (j & 15))) & 15]; }
    c[o++] = '"'; c[o++] = '}';
  }
  p[31 + clen] = '\n';
}

typedef struct {
  const gen_cfg* g;
  uint8_t* buf;
  const uint64_t* offs; /* per line start offsets */
  uint64_t lo, hi;
} fill_job;

static void* fill_thread(void* arg) {
  fill_job* j = (fill_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    const uint64_t k = line_key(j->g, i);
    const uint32_t clen = (uint32_t)(j->offs[i + 1] - j->offs[i]) - 32;
    write_line(j->g, i, k, j->buf + j->offs[i], clen);
  }
  return NULL;
}

/* ---- adversarial (sequential) ---------------------------------------------------- */
typedef struct {
  uint8_t* buf;
  uint64_t cap, n;
} sink;
static void put(sink* s, const void* p, size_t n) {
  if (s->buf && s->n + n <= s->cap) memcpy(s->buf + s->n, p, n);
  s->n += n;
}
static void putc_(sink* s, uint8_t c) { put(s, &c, 1); }

static void adv_line(const gen_cfg* g, uint64_t i, sink* s) {
  const uint64_t k = line_key(g, i), k2 = mix(k ^ 0x77ull);
  const uint32_t v = (uint32_t)(k % 100);
  int64_t ns = g->t0_ns + (int64_t)i * g->step_ns;
  if ((k2 & 15) == 0) ns += (int64_t)((k2 >> 8) % 7200) * 1000000000ll - 3600ll * 1000000000ll; /* out of order */
  uint8_t ts[40];
  fmt_ts(ts, ns);
  size_t tl = 30;
  if (v < 55) {
    /* canonical */
  } else if (v < 63) { /* fraction digits 0..12 */
    const int nd = (int)((k2 >> 20) % 13);
    uint8_t frac[13];
    for (int j = 0; j < 12; ++j) frac[j] = (uint8_t)('0' + ((k2 >> (24 + j)) % 10));
    if (nd == 0) { tl = 19; } else { tl = 20; memcpy(ts + 20, frac, (size_t)nd); tl = 20 + (size_t)nd; }
    ts[tl++] = 'Z';
  } else if (v < 66) { /* comma separator */
    ts[19] = ',';
  } else if (v < 72) { /* +-hh:mm */
    static const char* offs[] = {"+01:30", "-07:00", "+24:00", "-00:00", "+05:45", "+24:60", "+25:00", "+01:61", "+1:00", "-12:3x"};
    const char* o = offs[(k2 >> 30) % 10];
    tl = 29;
    memcpy(ts + tl, o, strlen(o));
    tl += strlen(o);
  } else if (v < 74) { /* one-digit hour */
    memmove(ts + 11, ts + 12, 18);
    tl = 29;
  } else if (v < 80) { /* invalid fields */
    static const char* bad[] = {"2024-13-01T00:00:00Z", "2023-02-29T00:00:00Z", "2024-02-29T23:59:59.5Z",
                                "2024-10-22T24:00:00Z", "2024-10-22T23:60:00Z", "2024-10-22T23:59:60Z",
                                "2024-10-22 23:59:59Z", "2024-10-22T23:59:59", "0000-01-01T00:00:00Z",
                                "0001-01-01T00:00:00Z", "9999-12-31T23:59:59.999999999Z", "2024-1-22T00:00:00Z",
                                "abc", "", "2024-10-22T10:00:00.Z", "2024-10-22T10:00:00Zx"};
    const char* b = bad[(k2 >> 30) % 16];
    tl = strlen(b);
    memcpy(ts, b, tl);
  }
  const int no_space = (v >= 80 && v < 82);
  const int empty = (v >= 82 && v < 84);
  if (empty) { if (((k2 >> 40) & 1) == 0) putc_(s, '\r'); putc_(s, '\n'); return; }
  put(s, ts, tl);
  if (!no_space) putc_(s, ' ');
  /* content */
  const uint32_t shape = (uint32_t)((k2 >> 44) % 100);
  uint32_t clen = 8 + (uint32_t)((k2 >> 50) % 120);
  if (shape < 3) clen = 2000 + (uint32_t)((k2 >> 52) % 30000); /* long line, crosses tiles */
  if (shape >= 3 && shape < 6) clen = 0;
  uint8_t tmp[40000];
  fill_words(tmp, clen, k);
  if (shape >= 6 && shape < 10 && clen) tmp[(k2 >> 3) % clen] = (uint8_t)(0x80 + ((k2 >> 9) & 0x7f));
  if (shape >= 10 && shape < 12 && clen) tmp[(k2 >> 5) % clen] = 0;
  if (shape >= 12 && shape < 14 && clen) tmp[0] = ' '; /* double space after prefix */
  if (g->needle_len && clen > g->needle_len && ((k >> 32) % 1000) < g->needle_permille)
    memcpy(tmp + (k2 >> 7) % (clen - g->needle_len + 1), g->needle, g->needle_len);
  put(s, tmp, clen);
  if (((k2 >> 60) & 7) == 0) putc_(s, '\r');
  putc_(s, '\n');
}

/* Generates one stream.  buf == NULL: returns the size only.  Returns bytes written.
 * TEXT/JSON: lines are added until the size reaches target_bytes (the last line ends the
 * stream, so the size can exceed the target by one line).  ADVERSARIAL: n_lines lines
 * of the target (target_bytes is read as a line count).  `drop_final_nl` removes the
 * last '\n' (an unterminated fragment). */
uint64_t ks_generate(uint32_t kind, uint64_t seed, uint32_t stream, uint64_t target, int64_t t0_sec,
                     int64_t span_sec, const uint8_t* needle, uint32_t needle_len, uint32_t needle_permille,
                     int drop_final_nl, uint8_t* buf, uint64_t cap, int threads) {
  gen_cfg g;
  g.kind = kind;
  g.seed = seed;
  g.stream = stream;
  g.t0_ns = t0_sec * 1000000000ll;
  g.needle = needle;
  g.needle_len = needle_len;
  g.needle_permille = needle_permille;
  if (kind == KS_ADVERSARIAL) {
    g.step_ns = target ? (span_sec * 1000000000ll) / (int64_t)target : 1;
    sink s = {buf, cap, 0};
    for (uint64_t i = 0; i < target; ++i) adv_line(&g, i, &s);
    if (drop_final_nl && s.n && (!buf || s.n <= cap) && (!buf || buf[s.n - 1] == '\n')) s.n -= 1;
    return s.n;
  }
  const uint64_t avg = kind == KS_TEXT ? 154 : kind == KS_MIXED ? 350 : kind == KS_LONGJSON ? 9500 : 432;
  const uint64_t est = target / avg + 1;
  g.step_ns = (span_sec * 1000000000ll) / (int64_t)est;
  /* pass 1: line lengths until the target is reached */
  uint64_t n = 0, total = 0, capl = 1024;
  uint64_t* offs = buf ? (uint64_t*)malloc(capl * sizeof(uint64_t)) : NULL;
  if (buf && !offs) return 0;
  while (total < target) {
    const uint32_t clen = content_len(&g, line_key(&g, n));
    if (offs) {
      if (n + 2 > capl) {
        capl *= 2;
        uint64_t* o2 = (uint64_t*)realloc(offs, capl * sizeof(uint64_t));
        if (!o2) { free(offs); return 0; }
        offs = o2;
      }
      offs[n] = total;
    }
    total += 32 + clen;
    ++n;
  }
  if (!buf) return drop_final_nl && total ? total - 1 : total;
  offs[n] = total;
  if (total > cap) { free(offs); return 0; }
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if ((uint64_t)threads > n) threads = (int)(n ? n : 1);
  pthread_t th[64];
  fill_job jobs[64];
  for (int t = 0; t < threads; ++t) {
    jobs[t].g = &g;
    jobs[t].buf = buf;
    jobs[t].offs = offs;
    jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
  }
  for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, fill_thread, &jobs[t]);
  fill_thread(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
  free(offs);
  return drop_final_nl && total ? total - 1 : total;
}
