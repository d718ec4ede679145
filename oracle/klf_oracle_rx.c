/* klf_oracle_rx.c — Go regexp.Match over the RE2 subset of SPEC.md S5, restated in C.
 * TEST INFRASTRUCTURE ONLY: the C oracle's regex leg (ko_filter_rx), linked into
 * oracle/_build/libklf_oracle.so beside klf_oracle_c.c.  The product never loads it.
 *
 * Written from Go's regexp/syntax and regexp packages (Go 1.22), sharing no code with the
 * Python oracle (oracle/klf_oracle.py, which translates the same subset into Python `re`)
 * or with the engine (klogs_amd/csrc/klf_patterns.cpp, Glushkov tables):
 *   - parser:   regexp/syntax/parse.go restated as a recursive descent over the pattern
 *               bytes: parse()'s main loop (repetition applies to the item before it, a
 *               repetition right after one is ErrInvalidRepeatOp, none before it is
 *               ErrMissingRepeatArgument), parseRepeat/parseInt (no leading zeros, counts
 *               <= 1000, else '{' is a literal), parsePerlFlags ((?flags) for the rest of
 *               the group, (?flags:re), named groups), parseEscape (octal, \x, \x{..},
 *               control and punctuation escapes), parseClass (']' first is literal, ranges,
 *               [:name:] and [:^name:], \d \w \s and negations, fold before negation as in
 *               appendGroup / appendFoldedRange).  ASCII only: a pattern byte >= 0x80, an
 *               escape to a value >= 0x80, \b \B \p \P \C and backreferences are rejected.
 *   - compiler: Thompson construction (regexp/syntax/compile.go's shape): byte-set,
 *               split, empty-width begin / end of text, match.  x{m,n} expands to m copies
 *               and n - m nested optional ones, as simplify.go does.
 *   - matcher:  regexp.Match is an unanchored search for any match: a lazily built DFA
 *               over sets of NFA states (the state set after each byte, the start state's
 *               closure added at every position), end-of-text assertions decided at the
 *               content's end.  Content never holds '\n' (S5), so ^ / $ are \A / \z with or
 *               without (?m).
 *   - prefilter: each pattern's required literal (the longest run of single bytes or ASCII
 *               case pairs that every match contains, taken from the parse tree's top-level
 *               concatenation), searched lower-cased with one Aho-Corasick pass per line;
 *               only the patterns whose literal occurs run their DFA.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t lines, parsed, since_ok, matched, selected, out_bytes;
} ko_counts;
typedef int (*ko_match_fn)(void* ctx, const uint8_t* c, size_t cn);
/* klf_oracle_c.c: the kubelet read loop shared by every matcher */
int64_t ko_filter_impl(const uint8_t* data, uint64_t n, int64_t since_sec, int32_t since_nsec, int64_t tail,
                       int grep_active, ko_match_fn match, void* mctx, uint8_t* out, uint64_t* line_off,
                       uint64_t line_cap, uint8_t* match_bits, ko_counts* cnt);

/* ---- byte sets ------------------------------------------------------------------- */
typedef struct { uint32_t w[8]; } bset;
static void bs_add(bset* s, int c) { s->w[c >> 5] |= 1u << (c & 31); }
static int bs_has(const bset* s, int c) { return (s->w[c >> 5] >> (c & 31)) & 1; }
static void bs_range(bset* s, int lo, int hi) { for (int c = lo; c <= hi; ++c) bs_add(s, c); }
static void bs_or(bset* d, const bset* s) { for (int k = 0; k < 8; ++k) d->w[k] |= s->w[k]; }
static void bs_not(bset* s) { for (int k = 0; k < 8; ++k) s->w[k] = ~s->w[k]; }
static int bs_count(const bset* s) { int n = 0; for (int k = 0; k < 8; ++k) n += __builtin_popcount(s->w[k]); return n; }
static void bs_fold(bset* s) {  /* ASCII simple folds: A-Z <-> a-z */
  for (int c = 'A'; c <= 'Z'; ++c)
    if (bs_has(s, c) || bs_has(s, c + 32)) { bs_add(s, c); bs_add(s, c + 32); }
}
/* Perl classes (regexp/syntax/perl_groups.go): \d [0-9], \s [\t\n\f\r ], \w [0-9A-Za-z_] */
static bset perl_class(int c) {
  bset s;
  memset(&s, 0, sizeof s);
  switch (c | 0x20) {
    case 'd': bs_range(&s, '0', '9'); break;
    case 's': bs_add(&s, '\t'); bs_add(&s, '\n'); bs_add(&s, '\f'); bs_add(&s, '\r'); bs_add(&s, ' '); break;
    default: bs_range(&s, '0', '9'); bs_range(&s, 'A', 'Z'); bs_range(&s, 'a', 'z'); bs_add(&s, '_'); break;
  }
  return s;
}
/* POSIX classes (perl_groups.go posixGroup), ASCII */
static int posix_class(const uint8_t* name, size_t len, bset* s) {
  static const struct { const char* n; const char* r; } tab[] = {
      {"alnum", "09AZaz"}, {"alpha", "AZaz"}, {"ascii", "\x01\x7f"}, {"blank", "\t\t  "},
      {"cntrl", "\x01\x1f\x7f\x7f"}, {"digit", "09"}, {"graph", "!~"}, {"lower", "az"},
      {"print", " ~"}, {"punct", "!/:@[`{~"}, {"space", "\t\r  "}, {"upper", "AZ"},
      {"word", "09AZaz__"}, {"xdigit", "09AFaf"}};
  memset(s, 0, sizeof *s);
  for (size_t k = 0; k < sizeof tab / sizeof tab[0]; ++k) {
    if (strlen(tab[k].n) != len || memcmp(tab[k].n, name, len) != 0) continue;
    for (const char* r = tab[k].r; *r; r += 2) bs_range(s, (uint8_t)r[0], (uint8_t)r[1]);
    if (!strcmp(tab[k].n, "ascii") || !strcmp(tab[k].n, "cntrl")) bs_add(s, 0);  /* (NUL: not in a C string) */
    return 1;
  }
  return 0;
}

/* ---- parse tree -------------------------------------------------------------------- */
enum { N_SET, N_EMPTY, N_CAT, N_ALT, N_REP, N_BOL, N_EOL };
typedef struct {
  int op, min, max;  /* N_REP: max -1 = unbounded */
  int kid, next;     /* first child, next sibling (-1: none) */
  bset set;
} rnode;
typedef struct { int fold, dotnl; } rflags;
typedef struct {
  const uint8_t* p;
  size_t n, i;
  rnode* nd;
  int nn, cap;
  const char* err;
  int quoting;       /* inside \Q...\E */
  size_t q_end;      /* index of the closing \E (n: none) */
} rparser;

#define NONE (-2)  /* a flag group: nothing pushed */

static int new_node(rparser* P, int op) {
  if (P->nn == P->cap) {
    int c = P->cap ? P->cap * 2 : 64;
    rnode* q = (rnode*)realloc(P->nd, (size_t)c * sizeof(rnode));
    if (!q) { P->err = "out of memory"; return -1; }
    P->nd = q;
    P->cap = c;
  }
  rnode* r = &P->nd[P->nn];
  memset(r, 0, sizeof *r);
  r->op = op;
  r->kid = r->next = -1;
  return P->nn++;
}
static int set_node(rparser* P, const bset* s) {
  const int k = new_node(P, N_SET);
  if (k >= 0) P->nd[k].set = *s;
  return k;
}
static int lit_node(rparser* P, int c, const rflags* f) {
  bset s;
  memset(&s, 0, sizeof s);
  bs_add(&s, c);
  if (f->fold) bs_fold(&s);
  return set_node(P, &s);
}
static int peek(const rparser* P, size_t k) { return P->i + k < P->n ? P->p[P->i + k] : -1; }
static int isalnum_a(int c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
static int unhex(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

/* parseEscape: the byte an escape stands for (P->i at the backslash), or -1 with P->err */
static int parse_escape(rparser* P) {
  P->i++;
  if (P->i >= P->n) { P->err = "trailing backslash at end of expression"; return -1; }
  const int c = P->p[P->i++];
  int v = -1;
  if (c >= '1' && c <= '7' && !(P->i < P->n && P->p[P->i] >= '0' && P->p[P->i] <= '7')) {
    P->err = "invalid escape sequence";  /* \1 alone: a backreference */
    return -1;
  }
  if (c >= '0' && c <= '7') {
    v = c - '0';
    for (int k = 0; k < 2 && P->i < P->n && P->p[P->i] >= '0' && P->p[P->i] <= '7'; ++k) v = v * 8 + P->p[P->i++] - '0';
  } else if (c == 'x') {
    if (P->i < P->n && P->p[P->i] == '{') {
      P->i++;
      int nhex = 0;
      v = 0;
      for (;;) {
        if (P->i >= P->n) { P->err = "invalid escape sequence"; return -1; }
        const int d = P->p[P->i++];
        if (d == '}') break;
        const int h = unhex(d);
        if (h < 0) { P->err = "invalid escape sequence"; return -1; }
        v = v * 16 + h;
        if (v > 0x10FFFF) { P->err = "invalid escape sequence"; return -1; }
        ++nhex;
      }
      if (!nhex) { P->err = "invalid escape sequence"; return -1; }
    } else {
      const int h1 = peek(P, 0) >= 0 ? unhex(peek(P, 0)) : -1, h2 = peek(P, 1) >= 0 ? unhex(peek(P, 1)) : -1;
      if (h1 < 0 || h2 < 0) { P->err = "invalid escape sequence"; return -1; }
      v = h1 * 16 + h2;
      P->i += 2;
    }
  } else if (c == 'a') v = 7;
  else if (c == 'f') v = 12;
  else if (c == 'n') v = 10;
  else if (c == 'r') v = 13;
  else if (c == 't') v = 9;
  else if (c == 'v') v = 11;
  else if (c < 0x80 && !isalnum_a(c)) v = c;  /* punctuation (and '_') stands for itself */
  else { P->err = "invalid escape sequence"; return -1; }
  if (v >= 0x80) { P->err = "non-ASCII escapes are outside the supported subset"; return -1; }
  return v;
}

static int parse_alt(rparser* P, rflags* f);

/* parseClass (P->i at '[') */
static int parse_class(rparser* P, const rflags* f) {
  P->i++;
  int neg = 0;
  if (peek(P, 0) == '^') { neg = 1; P->i++; }
  bset s;
  memset(&s, 0, sizeof s);
  int first = 1;
  for (;;) {
    const int c = peek(P, 0);
    if (c < 0) { P->err = "missing closing ]"; return -1; }
    if (c == ']' && !first) { P->i++; break; }
    first = 0;
    if (c == '[' && peek(P, 1) == ':') {  /* [:name:] / [:^name:] */
      size_t k = P->i + 2;
      while (k + 1 < P->n && !(P->p[k] == ':' && P->p[k + 1] == ']')) ++k;
      if (k + 1 < P->n) {
        const uint8_t* name = P->p + P->i + 2;
        size_t len = k - (P->i + 2);
        const int gneg = len && name[0] == '^';
        bset g;
        if (!posix_class(name + gneg, len - gneg, &g)) { P->err = "invalid character class range"; return -1; }
        if (f->fold) bs_fold(&g);
        if (gneg) bs_not(&g);
        bs_or(&s, &g);
        P->i = k + 2;
        continue;
      }
    }
    if (c == '\\' && peek(P, 1) >= 0 && strchr("dDsSwW", peek(P, 1))) {
      bset g = perl_class(peek(P, 1));
      if (peek(P, 1) < 'a') bs_not(&g);  /* \D \S \W (fold-closed sets) */
      bs_or(&s, &g);
      P->i += 2;
      continue;
    }
    if (c == '\\' && (peek(P, 1) == 'p' || peek(P, 1) == 'P')) { P->err = "unicode classes are outside the supported subset"; return -1; }
    int lo, hi;
    if (c == '\\') { if ((lo = parse_escape(P)) < 0) return -1; }
    else lo = P->p[P->i++];
    hi = lo;
    if (peek(P, 0) == '-' && peek(P, 1) >= 0 && peek(P, 1) != ']') {
      P->i++;
      if (peek(P, 0) == '\\') { if ((hi = parse_escape(P)) < 0) return -1; }
      else hi = P->p[P->i++];
      if (hi < lo) { P->err = "invalid character class range"; return -1; }
    }
    bset r;
    memset(&r, 0, sizeof r);
    bs_range(&r, lo, hi);
    if (f->fold) bs_fold(&r);
    bs_or(&s, &r);
  }
  if (neg) bs_not(&s);
  return set_node(P, &s);
}

/* parsePerlFlags / capture groups (P->i at '(') */
static int parse_group(rparser* P, rflags* f) {
  P->i++;
  rflags nf = *f;
  if (peek(P, 0) == '?') {
    size_t j = P->i + 1;
    if ((j < P->n && P->p[j] == '<') || (j + 1 < P->n && P->p[j] == 'P' && P->p[j + 1] == '<')) {
      j += P->p[j] == 'P' ? 2 : 1;
      const size_t name0 = j;
      while (j < P->n && (isalnum_a(P->p[j]) || P->p[j] == '_')) ++j;
      if (j == name0 || j >= P->n || P->p[j] != '>') { P->err = "invalid named capture"; return -1; }
      P->i = j + 1;
    } else {
      int sign = 1, saw = 0;
      for (;; ++j) {
        if (j >= P->n) { P->err = "missing closing )"; return -1; }
        const int c = P->p[j];
        if (c == 'i' || c == 'm' || c == 's' || c == 'U') {
          if (c == 'i') nf.fold = sign > 0;
          if (c == 's') nf.dotnl = sign > 0;
          saw = 1;
        } else if (c == '-') {
          if (sign < 0) { P->err = "invalid or unsupported Perl syntax"; return -1; }
          sign = -1;
          saw = 0;
        } else if (c == ':' || c == ')') {
          if (sign < 0 && !saw) { P->err = "invalid or unsupported Perl syntax"; return -1; }
          P->i = j + 1;
          if (c == ')') { *f = nf; return NONE; }  /* the rest of the current group */
          break;
        } else {
          P->err = "invalid or unsupported Perl syntax";
          return -1;
        }
      }
    }
  }
  const int inner = parse_alt(P, &nf);
  if (inner < 0) return -1;
  if (peek(P, 0) != ')') { P->err = "missing closing )"; return -1; }
  P->i++;
  return inner;
}

/* one item of a concatenation, P->i not at a repetition operator */
static int parse_atom(rparser* P, rflags* f) {
  const int c = P->p[P->i];
  if (c == '(') return parse_group(P, f);
  if (c == '[') return parse_class(P, f);
  if (c == '.') {
    P->i++;
    bset s;
    memset(&s, 0xFF, sizeof s);
    if (!f->dotnl) s.w['\n' >> 5] &= ~(1u << ('\n' & 31));
    return set_node(P, &s);
  }
  if (c == '^') { P->i++; return new_node(P, N_BOL); }
  if (c == '$') { P->i++; return new_node(P, N_EOL); }
  if (c == '\\') {
    const int e = peek(P, 1);
    if (e == 'A') { P->i += 2; return new_node(P, N_BOL); }
    if (e == 'z') { P->i += 2; return new_node(P, N_EOL); }
    if (e == 'b' || e == 'B') { P->err = "word boundaries are outside the supported subset"; return -1; }
    if (e == 'p' || e == 'P') { P->err = "unicode classes are outside the supported subset"; return -1; }
    if (e == 'C') { P->err = "invalid escape sequence"; return -1; }
    if (e == 'Q') {
      P->i += 2;
      size_t k = P->i;
      while (k + 1 < P->n && !(P->p[k] == '\\' && P->p[k + 1] == 'E')) ++k;
      P->q_end = k + 1 < P->n ? k : P->n;
      P->quoting = 1;
      return NONE;
    }
    if (e >= 0 && strchr("dDsSwW", e)) {
      bset g = perl_class(e);
      if (e < 'a') bs_not(&g);
      P->i += 2;
      return set_node(P, &g);
    }
    const int v = parse_escape(P);
    return v < 0 ? -1 : lit_node(P, v, f);
  }
  P->i++;
  return lit_node(P, c, f);
}

/* parseRepeat + parseInt: {m} {m,} {m,n}; 0 = not a repetition ('{' is then a literal) */
static int parse_int(const rparser* P, size_t* j, int* v) {
  size_t k = *j;
  if (k >= P->n || P->p[k] < '0' || P->p[k] > '9') return 0;
  if (k + 1 < P->n && P->p[k] == '0' && P->p[k + 1] >= '0' && P->p[k + 1] <= '9') return 0;  /* leading zero */
  long x = 0;
  while (k < P->n && P->p[k] >= '0' && P->p[k] <= '9') {
    if (x >= 100000000) x = -1;
    else if (x >= 0) x = x * 10 + (P->p[k] - '0');
    ++k;
  }
  *v = x < 0 || x > 100000000 ? 1000000000 : (int)x;
  *j = k;
  return 1;
}
static int try_braces(rparser* P, int* mn, int* mx) {
  size_t j = P->i + 1;
  if (!parse_int(P, &j, mn)) return 0;
  *mx = *mn;
  if (j < P->n && P->p[j] == ',') {
    ++j;
    if (j < P->n && P->p[j] == '}') *mx = -1;
    else if (!parse_int(P, &j, mx)) return 0;
  }
  if (j >= P->n || P->p[j] != '}') return 0;
  if (*mn > 1000 || *mx > 1000 || (*mx >= 0 && *mn > *mx)) { P->err = "invalid repeat count"; return -1; }
  P->i = j + 1;
  return 1;
}

static int parse_concat(rparser* P, rflags* f) {
  int head = -1, tail = -1, prev = -1, last_rep = 0;
  for (;;) {
    if (P->err) return -1;
    int item;
    if (P->quoting) {
      if (P->i >= P->q_end) {
        P->i = P->q_end < P->n ? P->q_end + 2 : P->n;
        P->quoting = 0;
        last_rep = 0;
        continue;
      }
      item = lit_node(P, P->p[P->i++], f);
    } else {
      if (P->i >= P->n || P->p[P->i] == '|' || P->p[P->i] == ')') break;
      const int c = P->p[P->i];
      int mn = 0, mx = 0, rep = 0;
      if (c == '*' || c == '+' || c == '?') {
        rep = 1;
        mn = c == '+';
        mx = c == '?' ? 1 : -1;
      } else if (c == '{') {
        const int r = try_braces(P, &mn, &mx);
        if (r < 0) return -1;
        if (r) rep = 2;
      }
      if (rep) {
        if (prev < 0) { P->err = "missing argument to repetition operator"; return -1; }
        if (last_rep) { P->err = "invalid nested repetition operator"; return -1; }
        if (rep == 1) P->i++;
        if (peek(P, 0) == '?') P->i++;  /* non-greedy: the same boolean match */
        const int r = new_node(P, N_REP);
        if (r < 0) return -1;
        rnode* R = &P->nd[r];
        R->min = mn;
        R->max = mx;
        R->kid = prev;
        R->next = -1;
        /* the repetition takes the place of the item it repeats */
        if (head == prev) head = r;
        else {
          int k = head;
          while (P->nd[k].next != prev) k = P->nd[k].next;
          P->nd[k].next = r;
        }
        P->nd[prev].next = -1;
        if (tail == prev) tail = r;
        prev = r;
        last_rep = 1;
        continue;
      }
      item = parse_atom(P, f);
      if (item == NONE) { last_rep = 0; continue; }
    }
    if (item < 0) return -1;
    if (head < 0) head = item;
    else P->nd[tail].next = item;
    tail = item;
    prev = item;
    last_rep = 0;
  }
  if (head < 0) return new_node(P, N_EMPTY);
  if (P->nd[head].next < 0) return head;
  const int k = new_node(P, N_CAT);
  if (k >= 0) P->nd[k].kid = head;
  return k;
}

static int parse_alt(rparser* P, rflags* f) {
  int first = parse_concat(P, f);
  if (first < 0 || peek(P, 0) != '|' || P->quoting) return first;
  const int k = new_node(P, N_ALT);
  if (k < 0) return -1;
  P->nd[k].kid = first;
  int tail = first;
  while (!P->quoting && peek(P, 0) == '|') {
    P->i++;
    const int b = parse_concat(P, f);
    if (b < 0) return -1;
    P->nd[tail].next = b;
    tail = b;
  }
  return k;
}

/* ---- NFA program --------------------------------------------------------------------- */
enum { I_SET, I_SPLIT, I_BOL, I_EOL, I_MATCH, I_NOP };
typedef struct { int op, x, y, set; } rinst;
typedef struct {
  rinst* in;
  int n, cap;
  bset* sets;
  int ns, scap;
  int start;
  int err;
} rprog;

#define KO_RX_MAX_INST 400000

static int emit(rprog* G, int op, int x, int y) {
  if (G->n >= KO_RX_MAX_INST) { G->err = 1; return 0; }
  if (G->n == G->cap) {
    int c = G->cap ? G->cap * 2 : 256;
    rinst* q = (rinst*)realloc(G->in, (size_t)c * sizeof(rinst));
    if (!q) { G->err = 1; return 0; }
    G->in = q;
    G->cap = c;
  }
  G->in[G->n] = (rinst){op, x, y, -1};
  return G->n++;
}
static int add_set(rprog* G, const bset* s) {
  if (G->ns == G->scap) {
    int c = G->scap ? G->scap * 2 : 64;
    bset* q = (bset*)realloc(G->sets, (size_t)c * sizeof(bset));
    if (!q) { G->err = 1; return 0; }
    G->sets = q;
    G->scap = c;
  }
  G->sets[G->ns] = *s;
  return G->ns++;
}

static int compile(rprog* G, const rnode* nd, int k, int next);
/* a concatenation's items from k on, then `next` */
static int compile_list(rprog* G, const rnode* nd, int k, int next) {
  return k < 0 ? next : compile(G, nd, k, compile_list(G, nd, nd[k].next, next));
}
static int compile_alt_rest(rprog* G, const rnode* nd, const rnode* r, int next) {
  const int b = compile(G, nd, r->kid, next);
  if (nd[r->kid].next < 0) return b;
  rnode rest = *r;
  rest.kid = nd[r->kid].next;
  return emit(G, I_SPLIT, b, compile_alt_rest(G, nd, &rest, next));
}

/* compiles node k so that it continues at `next`; returns its entry */
static int compile(rprog* G, const rnode* nd, int k, int next) {
  if (G->err) return next;
  const rnode* r = &nd[k];
  switch (r->op) {
    case N_SET: {
      const int pc = emit(G, I_SET, next, 0);
      if (!G->err) G->in[pc].set = add_set(G, &r->set);
      return pc;
    }
    case N_EMPTY: return next;
    case N_BOL: return emit(G, I_BOL, next, 0);
    case N_EOL: return emit(G, I_EOL, next, 0);
    case N_CAT: return compile_list(G, nd, r->kid, next);
    case N_ALT: {
      const int b = compile(G, nd, r->kid, next);
      if (nd[r->kid].next < 0) return b;
      rnode rest = *r;  /* the alternation of the remaining branches */
      rest.kid = nd[r->kid].next;
      return emit(G, I_SPLIT, b, compile_alt_rest(G, nd, &rest, next));
    }
    default: {  /* N_REP */
      int s = next;
      if (r->max < 0) {  /* L: split(body -> L, next) */
        const int L = emit(G, I_SPLIT, 0, next);
        const int b = compile(G, nd, r->kid, L);
        if (!G->err) G->in[L].x = b;
        s = L;
      } else {
        for (int j = 0; j < r->max - r->min; ++j) {  /* nested optionals */
          const int b = compile(G, nd, r->kid, s);
          s = emit(G, I_SPLIT, b, next);
        }
      }
      for (int j = 0; j < r->min; ++j) s = compile(G, nd, r->kid, s);
      return s;
    }
  }
}

/* ---- required literal ------------------------------------------------------------------ */
typedef struct { uint8_t best[256], run[256]; int nbest, nrun; } rlit;
static void lit_flush(rlit* L) {
  if (L->nrun > L->nbest) { memcpy(L->best, L->run, (size_t)L->nrun); L->nbest = L->nrun; }
  L->nrun = 0;
}
/* the byte a set stands for when it is one byte or one ASCII case pair (lower case), else -1 */
static int lit_byte(const bset* s) {
  const int n = bs_count(s);
  if (n == 1) for (int c = 0; c < 256; ++c) if (bs_has(s, c)) return (c >= 'A' && c <= 'Z') ? c | 0x20 : c;
  if (n == 2) for (int c = 'a'; c <= 'z'; ++c) if (bs_has(s, c) && bs_has(s, c - 32)) return c;
  return -1;
}
static void lit_walk(const rnode* nd, int k, rlit* L) {
  const rnode* r = &nd[k];
  if (r->op == N_CAT) {
    for (int c = r->kid; c >= 0; c = nd[c].next) lit_walk(nd, c, L);
    return;
  }
  if (r->op == N_BOL || r->op == N_EOL || r->op == N_EMPTY) return;  /* zero width: the run goes on */
  int b = -1;
  if (r->op == N_SET) b = lit_byte(&r->set);
  else if (r->op == N_REP && r->min >= 1 && nd[r->kid].op == N_SET) b = lit_byte(&nd[r->kid].set);
  if (b < 0 || L->nrun == 255) { lit_flush(L); if (b < 0) return; }
  L->run[L->nrun++] = (uint8_t)b;
  if (r->op == N_REP) lit_flush(L);  /* the byte once, then the repetition */
}

/* ---- lazy DFA over NFA state sets ------------------------------------------------------ */
typedef struct {
  rprog G;
  int32_t* next;    /* [cap * 256], -1 = not built */
  uint8_t* fl;      /* [cap] 1: holds MATCH, 2: end decided, 4: matches at the end */
  int32_t* loff;    /* [cap + 1] leaf list offsets into pool */
  int32_t* pool;
  size_t pool_n, pool_cap;
  int32_t* hash;    /* [hcap] state + 1, 0 empty */
  size_t hcap;
  int ns, cap;
  int s0;           /* state at position 0 (-1: not built) */
  int32_t* restart; /* leaves of the start closure without ^ */
  int nrestart;
  uint32_t* mark;   /* [G.n] closure visit generation */
  uint32_t gen;
  int32_t *stack, *tmp, *tmp2;
  int has_eol;
  uint32_t epoch;   /* flushes so far */
} rdfa;

#define KO_RX_MAX_STATES 4096

static void dfa_free(rdfa* D) {
  free(D->G.in); free(D->G.sets); free(D->next); free(D->fl); free(D->loff); free(D->pool);
  free(D->hash); free(D->restart); free(D->mark); free(D->stack); free(D->tmp); free(D->tmp2);
  memset(D, 0, sizeof *D);
}

/* closure of pc into leaves (SET, MATCH, and EOL while !eol); returns the new count */
static int closure(rdfa* D, int pc, int bol, int eol, int32_t* out, int n) {
  int sp = 0;
  D->stack[sp++] = pc;
  while (sp) {
    const int p = D->stack[--sp];
    if (D->mark[p] == D->gen) continue;
    D->mark[p] = D->gen;
    const rinst* I = &D->G.in[p];
    switch (I->op) {
      case I_SET: case I_MATCH: out[n++] = p; break;
      case I_SPLIT: D->stack[sp++] = I->y; D->stack[sp++] = I->x; break;
      case I_NOP: D->stack[sp++] = I->x; break;
      case I_BOL: if (bol) D->stack[sp++] = I->x; break;
      case I_EOL: if (eol) D->stack[sp++] = I->x; else out[n++] = p; break;
    }
  }
  return n;
}
static void next_gen(rdfa* D) {
  if (++D->gen == 0) { memset(D->mark, 0, (size_t)D->G.n * sizeof(uint32_t)); D->gen = 1; }
}
static int cmp_i32(const void* a, const void* b) { return *(const int32_t*)a - *(const int32_t*)b; }
static uint64_t hash_leaves(const int32_t* v, int n) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
  for (int k = 0; k < n; ++k) h = (h ^ (uint32_t)v[k]) * 1099511628211ull;
  return h ^ (h >> 29);
}
static void dfa_flush(rdfa* D) {
  D->epoch++;
  D->ns = 0;
  D->pool_n = 0;
  D->s0 = -1;
  memset(D->hash, 0, D->hcap * sizeof(int32_t));
}
/* the state of a sorted leaf list; -1 on allocation failure */
static int intern(rdfa* D, const int32_t* v, int n) {
  const uint64_t h = hash_leaves(v, n);
  for (size_t k = h & (D->hcap - 1);; k = (k + 1) & (D->hcap - 1)) {
    const int32_t e = D->hash[k];
    if (!e) break;
    const int s = e - 1;
    if (D->loff[s + 1] - D->loff[s] == n && !memcmp(D->pool + D->loff[s], v, (size_t)n * sizeof(int32_t))) return s;
  }
  if (D->ns == KO_RX_MAX_STATES) dfa_flush(D);
  if (D->ns == D->cap) {
    const int c = D->cap * 2;
    int32_t* nx = (int32_t*)realloc(D->next, (size_t)c * 256 * sizeof(int32_t));
    if (nx) D->next = nx;
    uint8_t* fl = (uint8_t*)realloc(D->fl, (size_t)c);
    if (fl) D->fl = fl;
    int32_t* lo = (int32_t*)realloc(D->loff, (size_t)(c + 1) * sizeof(int32_t));
    if (lo) D->loff = lo;
    if (!nx || !fl || !lo) return -1;
    D->cap = c;
  }
  if (D->pool_n + (size_t)n > D->pool_cap) {
    size_t c = (D->pool_cap + (size_t)n) * 2;
    int32_t* q = (int32_t*)realloc(D->pool, c * sizeof(int32_t));
    if (!q) return -1;
    D->pool = q;
    D->pool_cap = c;
  }
  const int s = D->ns++;
  D->loff[s] = (int32_t)D->pool_n;
  memcpy(D->pool + D->pool_n, v, (size_t)n * sizeof(int32_t));
  D->pool_n += (size_t)n;
  D->loff[s + 1] = (int32_t)D->pool_n;
  memset(D->next + (size_t)s * 256, 0xFF, 256 * sizeof(int32_t));
  uint8_t f = 0;
  for (int k = 0; k < n; ++k) if (D->G.in[v[k]].op == I_MATCH) f = 1;
  D->fl[s] = f;
  for (size_t k = h & (D->hcap - 1);; k = (k + 1) & (D->hcap - 1))
    if (!D->hash[k]) { D->hash[k] = s + 1; break; }
  return s;
}
static int sort_unique(int32_t* v, int n) {
  qsort(v, (size_t)n, sizeof(int32_t), cmp_i32);
  int m = 0;
  for (int k = 0; k < n; ++k) if (!m || v[m - 1] != v[k]) v[m++] = v[k];
  return m;
}
static int start_state(rdfa* D) {
  if (D->s0 < 0) {
    next_gen(D);
    int n = closure(D, D->G.start, 1, 0, D->tmp, 0);
    n = sort_unique(D->tmp, n);
    D->s0 = intern(D, D->tmp, n);
  }
  return D->s0;
}
/* the state after byte c from state s */
static int step(rdfa* D, int s, int c) {
  const int32_t t = D->next[(size_t)s * 256 + c];
  if (t >= 0) return t;
  next_gen(D);
  int n = 0;
  for (int32_t k = D->loff[s]; k < D->loff[s + 1]; ++k) {
    const rinst* I = &D->G.in[D->pool[k]];
    if (I->op == I_SET && bs_has(&D->G.sets[I->set], c)) n = closure(D, I->x, 0, 0, D->tmp, n);
  }
  for (int k = 0; k < D->nrestart; ++k)  /* unanchored: a match may start at every position */
    if (D->mark[D->restart[k]] != D->gen) { D->mark[D->restart[k]] = D->gen; D->tmp[n++] = D->restart[k]; }
  n = sort_unique(D->tmp, n);
  const uint32_t epoch = D->epoch;
  const int r = intern(D, D->tmp, n);
  if (r >= 0 && D->epoch == epoch) D->next[(size_t)s * 256 + c] = r;  /* (s is gone after a flush) */
  return r;
}
/* does a deferred $ of state s's leaves reach MATCH at the content's end? */
static int end_match(rdfa* D, int s, int bol) {
  for (int32_t k = D->loff[s]; k < D->loff[s + 1]; ++k) {
    const rinst* I = &D->G.in[D->pool[k]];
    if (I->op != I_EOL) continue;
    next_gen(D);
    const int n = closure(D, I->x, bol, 1, D->tmp2, 0);
    for (int j = 0; j < n; ++j) if (D->G.in[D->tmp2[j]].op == I_MATCH) return 1;
  }
  return 0;
}

static int dfa_init(rdfa* D, const rnode* nd, int root) {
  memset(D, 0, sizeof *D);
  const int m = emit(&D->G, I_MATCH, 0, 0);
  D->G.start = compile(&D->G, nd, root, m);
  if (D->G.err) return -1;
  for (int k = 0; k < D->G.n; ++k) D->has_eol |= D->G.in[k].op == I_EOL;
  D->cap = 16;
  D->hcap = 2 * KO_RX_MAX_STATES;
  D->next = (int32_t*)malloc((size_t)D->cap * 256 * sizeof(int32_t));
  D->fl = (uint8_t*)malloc((size_t)D->cap);
  D->loff = (int32_t*)malloc((size_t)(D->cap + 1) * sizeof(int32_t));
  D->hash = (int32_t*)calloc(D->hcap, sizeof(int32_t));
  D->mark = (uint32_t*)calloc((size_t)D->G.n, sizeof(uint32_t));
  D->stack = (int32_t*)malloc((size_t)(2 * D->G.n + 2) * sizeof(int32_t));
  D->tmp = (int32_t*)malloc((size_t)(2 * D->G.n + 2) * sizeof(int32_t));
  D->tmp2 = (int32_t*)malloc((size_t)(D->G.n + 1) * sizeof(int32_t));
  D->restart = (int32_t*)malloc((size_t)(D->G.n + 1) * sizeof(int32_t));
  if (!D->next || !D->fl || !D->loff || !D->hash || !D->mark || !D->stack || !D->tmp || !D->tmp2 || !D->restart)
    return -1;
  D->s0 = -1;
  next_gen(D);
  D->nrestart = closure(D, D->G.start, 0, 0, D->restart, 0);
  return 0;
}

/* regexp.Match(re, c[0, n)) */
static int dfa_match(rdfa* D, const uint8_t* c, size_t n) {
  int s = start_state(D);
  if (s < 0) return -1;
  if (D->fl[s] & 1) return 1;
  if (!n) return D->has_eol && end_match(D, s, 1);
  for (size_t i = 0; i < n; ++i) {
    s = step(D, s, c[i]);
    if (s < 0) return -1;
    if (D->fl[s] & 1) return 1;
  }
  if (!D->has_eol) return 0;
  if (!(D->fl[s] & 2)) D->fl[s] |= 2 | (end_match(D, s, 0) ? 4 : 0);
  return (D->fl[s] & 4) != 0;
}

/* ---- one pattern: parse, literal, program --------------------------------------------- */
typedef struct {
  rdfa dfa;
  uint8_t lit[256];
  int nlit;
} rpat;

static const char* compile_pattern(const uint8_t* p, uint64_t n, rpat* out) {
  for (uint64_t k = 0; k < n; ++k)
    if (p[k] >= 0x80) return "non-ASCII pattern bytes are outside the supported subset";
  rparser P;
  memset(&P, 0, sizeof P);
  P.p = p;
  P.n = (size_t)n;
  rflags f = {0, 0};
  int root = parse_alt(&P, &f);
  if (!P.err && root >= 0 && P.i < P.n) P.err = "unexpected )";
  if (!P.err && root < 0) P.err = "out of memory";
  const char* err = P.err;
  if (!err && out) {
    rlit L;
    memset(&L, 0, sizeof L);
    if (P.nd[root].op != N_ALT) lit_walk(P.nd, root, &L);
    lit_flush(&L);
    memcpy(out->lit, L.best, (size_t)L.nbest);
    out->nlit = L.nbest;
    if (dfa_init(&out->dfa, P.nd, root) != 0) err = out->dfa.G.err ? "expression too large" : "out of memory";
  }
  free(P.nd);
  return err;
}

/* ---- Aho-Corasick over the required literals (lower case), with pattern outputs ------- */
typedef struct {
  int nc;
  uint16_t cls[256];
  int32_t* next;   /* [states * nc] */
  int32_t* term;   /* [states] first pattern whose literal ends here, -1 none */
  int32_t* dict;   /* [states] nearest terminal state on the suffix chain, 0 none */
  int32_t* pnext;  /* [patterns] next pattern with the same literal, -1 */
  int32_t* wide;   /* small automata: [states * 256] by raw byte (upper case folded), bit 30 =
                      the target state or its suffix chain ends a literal */
  int ns;
} lac;

static void lac_free(lac* A) {
  free(A->next); free(A->term); free(A->dict); free(A->pnext); free(A->wide);
  memset(A, 0, sizeof *A);
}
static int lac_build(lac* A, const rpat* pats, uint32_t np) {
  memset(A, 0, sizeof *A);
  size_t cap = 1;
  for (uint32_t k = 0; k < np; ++k) cap += (size_t)pats[k].nlit;
  A->nc = 1;
  for (uint32_t k = 0; k < np; ++k)
    for (int j = 0; j < pats[k].nlit; ++j)
      if (!A->cls[pats[k].lit[j]]) A->cls[pats[k].lit[j]] = (uint16_t)A->nc++;
  const int NC = A->nc;
  A->next = (int32_t*)malloc(cap * NC * sizeof(int32_t));
  A->term = (int32_t*)malloc(cap * sizeof(int32_t));
  A->dict = (int32_t*)calloc(cap, sizeof(int32_t));
  A->pnext = (int32_t*)malloc((np ? np : 1) * sizeof(int32_t));
  int32_t* fail = (int32_t*)calloc(cap, sizeof(int32_t));
  int32_t* queue = (int32_t*)malloc(cap * sizeof(int32_t));
  if (!A->next || !A->term || !A->dict || !A->pnext || !fail || !queue) { free(fail); free(queue); return -1; }
  for (size_t k = 0; k < cap * NC; ++k) A->next[k] = -1;
  for (size_t k = 0; k < cap; ++k) A->term[k] = -1;
  A->ns = 1;
  for (uint32_t k = 0; k < np; ++k) {
    A->pnext[k] = -1;
    if (!pats[k].nlit) continue;
    int32_t st = 0;
    for (int j = 0; j < pats[k].nlit; ++j) {
      int32_t* t = &A->next[(size_t)st * NC + A->cls[pats[k].lit[j]]];
      if (*t < 0) *t = A->ns++;
      st = *t;
    }
    A->pnext[k] = A->term[st];
    A->term[st] = (int32_t)k;
  }
  size_t qh = 0, qt = 0;
  for (int c = 0; c < NC; ++c) {
    int32_t* t = &A->next[c];
    if (*t < 0 || c == 0) { *t = 0; continue; }
    queue[qt++] = *t;
  }
  while (qh < qt) {
    const int32_t u = queue[qh++];
    for (int c = 0; c < NC; ++c) {
      int32_t* t = &A->next[(size_t)u * NC + c];
      const int32_t via = A->next[(size_t)fail[u] * NC + c];
      if (*t < 0) { *t = via; continue; }
      fail[*t] = via;
      A->dict[*t] = A->term[via] >= 0 ? via : A->dict[via];
      queue[qt++] = *t;
    }
  }
  free(fail);
  free(queue);
  if ((size_t)A->ns * 256 <= (1u << 20) && (A->wide = (int32_t*)malloc((size_t)A->ns * 256 * sizeof(int32_t))))
    for (int32_t st = 0; st < A->ns; ++st)
      for (int c = 0; c < 256; ++c) {
        const int32_t t = A->next[(size_t)st * NC + A->cls[c >= 'A' && c <= 'Z' ? c | 0x20 : c]];
        A->wide[(size_t)st * 256 + c] = t | ((A->term[t] >= 0 || A->dict[t] > 0) ? (1 << 30) : 0);
      }
  return 0;
}

/* ---- the line matcher and the exports ---------------------------------------------------- */
typedef struct {
  uint32_t n;
  rpat* pats;
  lac ac;
  int32_t* always;   /* patterns without a literal */
  uint32_t nalways;
  uint32_t* seen;    /* [n] generation of the last line that listed the pattern */
  uint32_t gen;
  int32_t* cand;
  int oom;
} rx2_ctx;

static int rx2_match(void* ctx, const uint8_t* c, size_t cn) {
  rx2_ctx* x = (rx2_ctx*)ctx;
  if (cn && c[cn - 1] == '\n') --cn;
  for (uint32_t k = 0; k < x->nalways; ++k) {
    const int m = dfa_match(&x->pats[x->always[k]].dfa, c, cn);
    if (m < 0) { x->oom = 1; return 0; }
    if (m) return 1;
  }
  if (x->nalways == x->n) return 0;
  if (++x->gen == 0) { memset(x->seen, 0, x->n * sizeof(uint32_t)); x->gen = 1; }
  uint32_t nc = 0;
  int32_t st = 0;
  const lac* A = &x->ac;
  if (A->wide) {
    for (size_t i = 0; i < cn; ++i) {
      st = A->wide[(size_t)st * 256 + c[i]];
      if (!(st & (1 << 30))) continue;
      st &= ~(1 << 30);
      for (int32_t t = A->term[st] >= 0 ? st : A->dict[st]; t > 0; t = A->dict[t])
        for (int32_t p = A->term[t]; p >= 0; p = A->pnext[p])
          if (x->seen[p] != x->gen) { x->seen[p] = x->gen; x->cand[nc++] = p; }
    }
  } else for (size_t i = 0; i < cn; ++i) {
    const uint8_t b = (uint8_t)(c[i] >= 'A' && c[i] <= 'Z' ? c[i] | 0x20 : c[i]);
    st = A->next[(size_t)st * A->nc + A->cls[b]];
    for (int32_t t = A->term[st] >= 0 ? st : A->dict[st]; t > 0; t = A->dict[t])
      for (int32_t p = A->term[t]; p >= 0; p = A->pnext[p])
        if (x->seen[p] != x->gen) { x->seen[p] = x->gen; x->cand[nc++] = p; }
  }
  for (uint32_t k = 0; k < nc; ++k) {
    const int m = dfa_match(&x->pats[x->cand[k]].dfa, c, cn);
    if (m < 0) { x->oom = 1; return 0; }
    if (m) return 1;
  }
  return 0;
}

/* NULL when the pattern is in the subset, else Go's error text (or the subset's) */
const char* ko_rx_error(const uint8_t* pat, uint64_t len) { return compile_pattern(pat, len, NULL); }

/* regexp.Match(pat, s): 1 / 0, -1 when the pattern does not compile */
int ko_rx_match(const uint8_t* pat, uint64_t plen, const uint8_t* s, uint64_t n) {
  rpat P;
  memset(&P, 0, sizeof P);
  if (compile_pattern(pat, plen, &P)) { dfa_free(&P.dfa); return -1; }
  const int m = dfa_match(&P.dfa, s, (size_t)n);
  dfa_free(&P.dfa);
  return m;
}

/* The required literal compile_pattern picked (lower case), for tests: its length, -1 on error. */
int ko_rx_literal(const uint8_t* pat, uint64_t plen, uint8_t* out256) {
  rpat P;
  memset(&P, 0, sizeof P);
  if (compile_pattern(pat, plen, &P)) { dfa_free(&P.dfa); return -1; }
  memcpy(out256, P.lit, (size_t)P.nlit);
  dfa_free(&P.dfa);
  return P.nlit;
}

/* As ko_filter with n_rx Go-subset regexes (pattern bytes + lengths) in place of literals.
 * Returns the output length, -1 on allocation failure, -2 - k when pattern k is not in the
 * subset (ko_rx_error names why). */
int64_t ko_filter_rx(const uint8_t* data, uint64_t n, int64_t since_sec, int32_t since_nsec, int64_t tail,
                     uint32_t n_rx, const uint8_t* const* pats, const uint64_t* pat_lens, uint8_t* out,
                     uint64_t* line_off, uint64_t line_cap, uint8_t* match_bits, ko_counts* cnt) {
  rx2_ctx x;
  memset(&x, 0, sizeof x);
  int64_t r = -1;
  uint32_t ok = 0;
  x.n = n_rx;
  x.pats = (rpat*)calloc(n_rx ? n_rx : 1, sizeof(rpat));
  x.always = (int32_t*)malloc((n_rx ? n_rx : 1) * sizeof(int32_t));
  x.seen = (uint32_t*)calloc(n_rx ? n_rx : 1, sizeof(uint32_t));
  x.cand = (int32_t*)malloc((n_rx ? n_rx : 1) * sizeof(int32_t));
  if (!x.pats || !x.always || !x.seen || !x.cand) goto done;
  for (; ok < n_rx; ++ok) {
    if (compile_pattern(pats[ok], pat_lens[ok], &x.pats[ok])) {
      dfa_free(&x.pats[ok].dfa);
      r = -2 - (int64_t)ok;
      goto done;
    }
    if (!x.pats[ok].nlit) x.always[x.nalways++] = (int32_t)ok;
  }
  if (lac_build(&x.ac, x.pats, n_rx) != 0) goto done;
  r = ko_filter_impl(data, n, since_sec, since_nsec, tail, n_rx != 0, rx2_match, &x, out, line_off, line_cap,
                     match_bits, cnt);
  if (x.oom) r = -1;
done:
  for (uint32_t k = 0; k < ok && x.pats; ++k) dfa_free(&x.pats[k].dfa);
  free(x.pats);
  free(x.always);
  free(x.seen);
  free(x.cand);
  lac_free(&x.ac);
  return r;
}
