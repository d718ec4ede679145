// klf_patterns.cpp — Go RE2-subset parser, Glushkov construction, Aho-Corasick build.
// See klf_patterns.hpp and SPEC.md S5 for the accepted syntax and semantics.
#include "klf_patterns.hpp"

#include <algorithm>
#include <chrono>
#include <bitset>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <queue>
#include <thread>

#include "../../include/klf.h"
#include "klf_kernels.hpp"

namespace klf {
namespace {

using ByteSet = std::bitset<256>;

ByteSet range_set(int lo, int hi) {  // bits lo..hi (whole-word shifts, no per-bit loop)
  ByteSet s;
  if (hi < lo) return s;
  s.set();
  s >>= 255 - (hi - lo);
  s <<= lo;
  return s;
}
const ByteSet& perl_d() {
  static const ByteSet d = range_set('0', '9');
  return d;
}
const ByteSet& perl_w() {
  static const ByteSet w = range_set('0', '9') | range_set('A', 'Z') | range_set('a', 'z') | range_set('_', '_');
  return w;
}
const ByteSet& perl_s() {
  static const ByteSet sp = [] {
    ByteSet x;
    for (int c : {'\t', '\n', '\f', '\r', ' '}) x.set(c);  // Go \s has no \v
    return x;
  }();
  return sp;
}
ByteSet fold(const ByteSet& s) {  // ASCII case pairs: 'A'..'Z' <-> 'a'..'z' are 32 bits apart
  static const ByteSet up = range_set('A', 'Z'), lo = range_set('a', 'z');
  return s | ((s & up) << 32) | ((s & lo) >> 32);
}

struct RNode {
  enum Kind { kEmpty, kSet, kCat, kAlt, kStar, kPlus, kQuest, kRepeat, kBot, kEot } k = kEmpty;
  ByteSet set;
  std::vector<int> kids;
  int lo = 0, hi = 0;  // kRepeat; hi = -1 means unbounded
};

struct Flags {
  bool i = false, s = false;
};

class Parser {
 public:
  Parser(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  std::vector<RNode> pool;
  std::string err;

  int parse() {
    for (size_t k = 0; k < n_; ++k)
      if (p_[k] >= 0x80) return fail("non-ASCII pattern bytes are outside the supported subset");
    Flags f;
    int r = alt(f);
    if (r < 0) return r;
    if (i_ < n_) return fail("unexpected )");
    return r;
  }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t i_ = 0;

  int fail(const char* m) {
    if (err.empty()) err = m;
    return -1;
  }
  int peek(size_t k = 0) const { return i_ + k < n_ ? p_[i_ + k] : -1; }
  int mk(RNode::Kind k) {
    RNode n;
    n.k = k;
    pool.push_back(n);
    return (int)pool.size() - 1;
  }
  int mkset(const ByteSet& s) {
    int x = mk(RNode::kSet);
    pool[x].set = s;
    return x;
  }

  int alt(Flags& f) {
    std::vector<int> br;
    int c = concat(f);
    if (c < 0) return c;
    br.push_back(c);
    while (peek() == '|') {
      ++i_;
      c = concat(f);
      if (c < 0) return c;
      br.push_back(c);
    }
    if (br.size() == 1) return br[0];
    int x = mk(RNode::kAlt);
    pool[x].kids = br;
    return x;
  }

  int concat(Flags& f) {
    std::vector<int> items;
    while (i_ < n_ && peek() != '|' && peek() != ')') {
      bool flags_only = false;
      int a = atom(f, flags_only);
      if (a < 0 && !flags_only) return -1;
      if (flags_only) continue;
      a = repeat(a);
      if (a < 0) return -1;
      items.push_back(a);
    }
    if (items.empty()) return mk(RNode::kEmpty);
    if (items.size() == 1) return items[0];
    int x = mk(RNode::kCat);
    pool[x].kids = items;
    return x;
  }

  // {m}, {m,}, {m,n}; returns false (no consumption) when not a valid repeat spec.
  bool braces(int& lo, int& hi, size_t& len) const {
    size_t j = i_;
    if (j >= n_ || p_[j] != '{') return false;
    ++j;
    size_t d0 = j;
    long v = 0;
    while (j < n_ && p_[j] >= '0' && p_[j] <= '9') { v = std::min(v * 10 + (p_[j] - '0'), 100000L); ++j; }
    if (j == d0) return false;
    lo = (int)v;
    if (j < n_ && p_[j] == '}') { hi = lo; len = j + 1 - i_; return true; }
    if (j >= n_ || p_[j] != ',') return false;
    ++j;
    size_t d1 = j;
    v = 0;
    while (j < n_ && p_[j] >= '0' && p_[j] <= '9') { v = std::min(v * 10 + (p_[j] - '0'), 100000L); ++j; }
    if (j >= n_ || p_[j] != '}') return false;
    hi = (j == d1) ? -1 : (int)v;
    len = j + 1 - i_;
    return true;
  }

  int repeat(int a) {
    bool seen = false;
    for (;;) {
      int c = peek();
      int k;
      if (c == '*' || c == '+' || c == '?') {
        if (seen) return fail("invalid nested repetition operator");
        ++i_;
        k = mk(c == '*' ? RNode::kStar : c == '+' ? RNode::kPlus : RNode::kQuest);
        pool[k].kids = {a};
      } else if (c == '{') {
        int lo, hi;
        size_t len;
        if (!braces(lo, hi, len)) return a;  // Go: '{' is then a literal
        if (seen) return fail("invalid nested repetition operator");
        if (lo > 1000 || hi > 1000 || (hi >= 0 && hi < lo)) return fail("invalid repeat count");
        i_ += len;
        k = mk(RNode::kRepeat);
        pool[k].kids = {a};
        pool[k].lo = lo;
        pool[k].hi = hi;
      } else {
        return a;
      }
      a = k;
      seen = true;
      if (peek() == '?') ++i_;  // lazy: same boolean match
    }
  }

  int atom(Flags& f, bool& flags_only) {
    int c = peek();
    if (c == '*' || c == '+' || c == '?') return fail("missing argument to repetition operator");
    if (c == '{') {
      int lo, hi;
      size_t len;
      if (braces(lo, hi, len)) return fail("missing argument to repetition operator");
    }
    if (c == '(') return group(f, flags_only);
    if (c == '[') {
      ByteSet s;
      if (!bracket(f, s)) return -1;
      return mkset(s);
    }
    if (c == '.') {
      ++i_;
      ByteSet s;
      s.set();
      if (!f.s) s.reset('\n');
      return mkset(s);
    }
    if (c == '^') { ++i_; return mk(RNode::kBot); }
    if (c == '$') { ++i_; return mk(RNode::kEot); }
    if (c == '\\') return escape_atom(f);
    ++i_;
    ByteSet s;
    s.set(c);
    return mkset(f.i ? fold(s) : s);
  }

  int group(Flags& f, bool& flags_only) {
    ++i_;  // (
    Flags inner = f;
    if (peek() == '?') {
      // named groups (?P<name>  (?<name>
      size_t j = i_ + 1;
      if (j < n_ && p_[j] == 'P') ++j;
      if (j < n_ && p_[j] == '<') {
        size_t k = j + 1;
        while (k < n_ && (isalnum(p_[k]) || p_[k] == '_')) ++k;
        if (k == j + 1 || k >= n_ || p_[k] != '>') return fail("invalid named capture");
        i_ = k + 1;
      } else {
        // flags: (?imsU-imsU) or (?imsU-imsU:...)
        size_t k = i_ + 1;
        bool neg = false, saw = false, saw_neg_flag = false;
        Flags nf = f;
        for (;; ++k) {
          if (k >= n_) return fail("missing closing )");
          int ch = p_[k];
          if (ch == 'i' || ch == 'm' || ch == 's' || ch == 'U') {
            if (ch == 'i') nf.i = !neg;
            if (ch == 's') nf.s = !neg;
            saw = true;
            if (neg) saw_neg_flag = true;
          } else if (ch == '-') {
            if (neg) return fail("invalid or unsupported Perl syntax");
            neg = true;
          } else if (ch == ':' || ch == ')') {
            if (neg && !saw_neg_flag) return fail("invalid or unsupported Perl syntax");
            if (ch == ')' && !saw) return fail("invalid or unsupported Perl syntax");
            break;
          } else {
            return fail("invalid or unsupported Perl syntax");
          }
        }
        if (p_[k] == ')') {  // flags for the rest of the current group
          f = nf;
          i_ = k + 1;
          flags_only = true;
          return -1;
        }
        inner = nf;
        i_ = k + 1;
      }
    }
    int r = alt(inner);
    if (r < 0) return r;
    if (peek() != ')') return fail("missing closing )");
    ++i_;
    return r;
  }

  // One escape; kind: 0 byte (v), 1 class (s), 2 assertion BOT, 3 assertion EOT.
  bool escape(bool in_class, int& kind, int& v, ByteSet& s) {
    ++i_;  // backslash
    int c = peek();
    if (c < 0) { fail("trailing backslash at end of expression"); return false; }
    ++i_;
    switch (c) {
      case 'd': kind = 1; s = perl_d(); return true;
      case 'w': kind = 1; s = perl_w(); return true;
      case 's': kind = 1; s = perl_s(); return true;
      case 'D': kind = 1; s = ~perl_d(); return true;
      case 'W': kind = 1; s = ~perl_w(); return true;
      case 'S': kind = 1; s = ~perl_s(); return true;
      case 't': kind = 0; v = '\t'; return true;
      case 'n': kind = 0; v = '\n'; return true;
      case 'r': kind = 0; v = '\r'; return true;
      case 'f': kind = 0; v = '\f'; return true;
      case 'v': kind = 0; v = '\v'; return true;
      case 'a': kind = 0; v = 7; return true;
      default: break;
    }
    if (c == 'x') {
      long val = 0;
      if (peek() == '{') {
        size_t j = i_ + 1, d0 = j;
        while (j < n_ && isxdigit(p_[j]) && j - d0 < 8) { val = val * 16 + (isdigit(p_[j]) ? p_[j] - '0' : (tolower(p_[j]) - 'a' + 10)); ++j; }
        if (j == d0 || j >= n_ || p_[j] != '}') { fail("invalid escape sequence"); return false; }
        i_ = j + 1;
      } else {
        if (i_ + 2 > n_ || !isxdigit(p_[i_]) || !isxdigit(p_[i_ + 1])) { fail("invalid escape sequence"); return false; }
        for (int k = 0; k < 2; ++k) val = val * 16 + (isdigit(p_[i_ + k]) ? p_[i_ + k] - '0' : (tolower(p_[i_ + k]) - 'a' + 10));
        i_ += 2;
      }
      if (val >= 0x80) { fail("non-ASCII escapes are outside the supported subset"); return false; }
      kind = 0; v = (int)val; return true;
    }
    if (c >= '0' && c <= '7') {
      // Go parseEscape: a single non-zero digit would be a backreference.
      if (c != '0' && !(peek() >= '0' && peek() <= '7')) { fail("invalid escape sequence"); return false; }
      int val = c - '0';
      for (int k = 0; k < 2 && peek() >= '0' && peek() <= '7'; ++k) { val = val * 8 + (peek() - '0'); ++i_; }
      if (val >= 0x80) { fail("non-ASCII escapes are outside the supported subset"); return false; }
      kind = 0; v = val; return true;
    }
    if (!in_class && c == 'A') { kind = 2; return true; }
    if (!in_class && c == 'z') { kind = 3; return true; }
    if (!isalnum(c)) { kind = 0; v = c; return true; }  // punctuation (and '_') is itself
    fail("invalid or unsupported escape");
    return false;
  }

  int escape_atom(Flags& f) {
    if (peek(1) == 'Q') {  // \Q...\E
      i_ += 2;
      std::vector<int> items;
      while (i_ < n_) {
        if (p_[i_] == '\\' && i_ + 1 < n_ && p_[i_ + 1] == 'E') { i_ += 2; break; }
        ByteSet s;
        s.set(p_[i_]);
        items.push_back(mkset(f.i ? fold(s) : s));
        ++i_;
      }
      if (items.empty()) return mk(RNode::kEmpty);
      if (items.size() == 1) return items[0];
      int x = mk(RNode::kCat);
      pool[x].kids = items;
      return x;
    }
    int kind, v = 0;
    ByteSet s;
    if (!escape(false, kind, v, s)) return -1;
    if (kind == 2) return mk(RNode::kBot);
    if (kind == 3) return mk(RNode::kEot);
    if (kind == 0) { s.reset(); s.set(v); }
    return mkset(f.i ? fold(s) : s);
  }

  bool posix_class(ByteSet& out) {
    // at "[:"; returns false (no consumption) when not a known [:name:]
    size_t j = i_ + 2;
    bool neg = false;
    if (j < n_ && p_[j] == '^') { neg = true; ++j; }
    size_t k = j;
    while (k < n_ && p_[k] >= 'a' && p_[k] <= 'z') ++k;
    if (k + 1 >= n_ || p_[k] != ':' || p_[k + 1] != ']') return false;
    std::string name((const char*)p_ + j, k - j);
    ByteSet s;
    if (name == "alnum") s = range_set('0', '9') | range_set('A', 'Z') | range_set('a', 'z');
    else if (name == "alpha") s = range_set('A', 'Z') | range_set('a', 'z');
    else if (name == "ascii") s = range_set(0, 0x7f);
    else if (name == "blank") { s.set('\t'); s.set(' '); }
    else if (name == "cntrl") { s = range_set(0, 0x1f); s.set(0x7f); }
    else if (name == "digit") s = range_set('0', '9');
    else if (name == "graph") s = range_set(0x21, 0x7e);
    else if (name == "lower") s = range_set('a', 'z');
    else if (name == "print") s = range_set(0x20, 0x7e);
    else if (name == "punct") s = range_set(0x21, 0x2f) | range_set(0x3a, 0x40) | range_set(0x5b, 0x60) | range_set(0x7b, 0x7e);
    else if (name == "space") { for (int c : {9, 10, 11, 12, 13, 32}) s.set(c); }
    else if (name == "upper") s = range_set('A', 'Z');
    else if (name == "word") s = perl_w();
    else if (name == "xdigit") s = range_set('0', '9') | range_set('A', 'F') | range_set('a', 'f');
    else return false;
    out |= neg ? ~s : s;
    i_ = k + 2;
    return true;
  }

  // class char: returns -2 on error, -3 when a set was added to `acc`, else the byte.
  int class_char(ByteSet& acc) {
    int c = peek();
    if (c == '\\') {
      int kind, v = 0;
      ByteSet s;
      if (!escape(true, kind, v, s)) return -2;
      if (kind == 1) { acc |= s; return -3; }
      return v;
    }
    ++i_;
    return c;
  }

  bool bracket(const Flags& f, ByteSet& out) {
    ++i_;  // [
    bool neg = false;
    if (peek() == '^') { neg = true; ++i_; }
    ByteSet s;
    bool first = true;
    for (;;) {
      int c = peek();
      if (c < 0) { fail("missing closing ]"); return false; }
      if (c == ']' && !first) { ++i_; break; }
      first = false;
      if (c == '[' && peek(1) == ':' && posix_class(s)) continue;
      int lo = class_char(s);
      if (lo == -2) return false;
      if (lo == -3) continue;
      if (peek() == '-' && peek(1) != ']' && peek(1) >= 0) {
        ++i_;
        ByteSet dummy;
        int hi = class_char(dummy);
        if (hi == -2) return false;
        if (hi == -3 || hi < lo) { fail("invalid character class range"); return false; }
        s |= range_set(lo, hi);
      } else {
        s.set(lo);
      }
    }
    if (f.i) s = fold(s);
    out = neg ? ~s : s;
    return true;
  }
};

// ---- repetition expansion + Glushkov -------------------------------------------------

struct Builder {
  std::vector<RNode>& pool;
  int npos = 0;
  std::string err;
  explicit Builder(std::vector<RNode>& p) : pool(p) {}

  int clone(int x) {
    RNode n = pool[x];
    for (int& k : n.kids) k = clone(k);
    pool.push_back(n);
    return (int)pool.size() - 1;
  }

  // Counts leaves (positions) after expansion without materialising it.
  long count_pos(int x) const {
    const RNode& n = pool[x];
    switch (n.k) {
      case RNode::kEmpty: return 0;
      case RNode::kSet: case RNode::kBot: case RNode::kEot: return 1;
      case RNode::kRepeat: {
        long c = count_pos(n.kids[0]);
        long reps = n.hi < 0 ? std::max(n.lo, 1) : n.hi;
        return std::min(c * reps, 1L << 30);
      }
      default: {
        long s = 0;
        for (int k : n.kids) s = std::min(s + count_pos(k), 1L << 30);
        return s;
      }
    }
  }

  int expand(int x) {
    RNode n = pool[x];
    if (n.k == RNode::kRepeat) {
      int a = expand(n.kids[0]);
      std::vector<int> items;
      for (int r = 0; r < n.lo; ++r) items.push_back(r == 0 ? a : clone(a));
      int used = n.lo;
      if (n.hi < 0) {
        int st = (int)pool.size();
        RNode s;
        s.k = RNode::kStar;
        s.kids = {used == 0 ? a : clone(a)};
        pool.push_back(s);
        items.push_back(st);
      } else if (n.hi > n.lo) {
        // x{lo,hi} = x^lo (x(x(...)?)?)?  — nested optionals keep it linear
        int tail = -1;
        for (int r = n.hi - n.lo - 1; r >= 0; --r) {
          int xr = (used == 0 && r == 0) ? a : clone(a);
          int body = xr;
          if (tail >= 0) {
            RNode c;
            c.k = RNode::kCat;
            c.kids = {xr, tail};
            pool.push_back(c);
            body = (int)pool.size() - 1;
          }
          RNode q;
          q.k = RNode::kQuest;
          q.kids = {body};
          pool.push_back(q);
          tail = (int)pool.size() - 1;
        }
        items.push_back(tail);
      }
      if (items.empty()) {
        RNode e;
        e.k = RNode::kEmpty;
        pool.push_back(e);
        return (int)pool.size() - 1;
      }
      if (items.size() == 1) return items[0];
      RNode c;
      c.k = RNode::kCat;
      c.kids = items;
      pool.push_back(c);
      return (int)pool.size() - 1;
    }
    for (size_t k = 0; k < n.kids.size(); ++k) {
      int e = expand(n.kids[k]);
      pool[x].kids[k] = e;
    }
    return x;
  }

  struct Info {
    bool nullable;
    uint64_t first, last;
  };
  std::vector<uint64_t> follow;
  std::vector<ByteSet> pos_set;
  uint64_t a_bot = 0, a_eot = 0;

  Info glushkov(int x) {
    const RNode& n = pool[x];
    switch (n.k) {
      case RNode::kEmpty: return {true, 0, 0};
      case RNode::kSet: case RNode::kBot: case RNode::kEot: {
        int p = npos++;
        follow.push_back(0);
        pos_set.push_back(n.k == RNode::kSet ? n.set : ByteSet());
        if (n.k == RNode::kBot) a_bot |= 1ull << p;
        if (n.k == RNode::kEot) a_eot |= 1ull << p;
        return {false, 1ull << p, 1ull << p};
      }
      case RNode::kCat: {
        Info acc{true, 0, 0};
        bool firstk = true;
        for (int k : n.kids) {
          Info b = glushkov(k);
          if (firstk) { acc = b; firstk = false; continue; }
          for (int p = 0; p < 64; ++p)
            if (acc.last >> p & 1) follow[p] |= b.first;
          Info r;
          r.nullable = acc.nullable && b.nullable;
          r.first = acc.first | (acc.nullable ? b.first : 0);
          r.last = b.last | (b.nullable ? acc.last : 0);
          acc = r;
        }
        return acc;
      }
      case RNode::kAlt: {
        Info acc{false, 0, 0};
        for (int k : n.kids) {
          Info b = glushkov(k);
          acc.nullable = acc.nullable || b.nullable;
          acc.first |= b.first;
          acc.last |= b.last;
        }
        return acc;
      }
      case RNode::kStar: case RNode::kPlus: {
        Info a = glushkov(n.kids[0]);
        for (int p = 0; p < 64; ++p)
          if (a.last >> p & 1) follow[p] |= a.first;
        return {n.k == RNode::kStar ? true : a.nullable, a.first, a.last};
      }
      case RNode::kQuest: {
        Info a = glushkov(n.kids[0]);
        return {true, a.first, a.last};
      }
      default: return {true, 0, 0};
    }
  }
};

// Closure of an entered set at one boundary: assertion positions in `holds` pass and
// enter their follow sets.  Returns the entered set; *acc = a passed position is final.
uint64_t closure(uint64_t entered, uint64_t holds, const std::vector<uint64_t>& follow,
                 uint64_t last, bool* acc) {
  uint64_t passed = 0;
  for (;;) {
    uint64_t todo = entered & holds & ~passed;
    if (!todo) break;
    passed |= todo;
    for (int p = 0; p < 64; ++p)
      if (todo >> p & 1) entered |= follow[p];
  }
  if (acc) *acc = (passed & last) != 0;
  return entered;
}

// ---- required factors (prefilter) ------------------------------------------------------
// Per node: `exact` when the node matches exactly one string (a byte set of one byte or
// one ASCII case pair counts as one byte; zero-width assertions are ""), and `req`, an
// OR-set of strings one of which every match contains.  Case pairs make the factor loose
// (stored OR 0x20).  The same analysis as RE2's prefilter, restricted to what the q-gram
// scan can use.
//
// Each set also carries `pre`: an upper bound on the distance from the start of a match
// of the node to the start of the first factor occurrence in it (kUnbounded when a
// repetition precedes it).  The GPU runs the NFA only over a window around each factor
// occurrence the prefilter verified: match starts in [x - pre, x], then on without new
// starts until the automaton dies (every match holds its first factor occurrence, and
// each occurrence is a candidate of its own), instead of over the whole line.
//
// Choice among a node's sets: those with at least `want` bytes in their shortest string
// first (the sampling stride of the whole pattern set needs that many; regex_factors runs
// the analysis once with want = unbounded to find each regex's best length), then a
// bounded `pre`, then the longest shortest string, then fewer strings.
constexpr uint32_t kUnbounded = 0xFFFFFFFFu;
uint32_t sat_add(uint32_t a, uint32_t b) { return (a == kUnbounded || b == kUnbounded) ? kUnbounded : a + b; }

struct FInfo {
  bool has_exact = false;
  std::string exact;
  bool exact_loose = false;
  std::vector<std::string> req;
  bool req_loose = false;
  uint32_t req_pre = kUnbounded;
  uint32_t maxlen = 0;  // longest match of the node (kUnbounded: no bound)
};

size_t req_score(const std::vector<std::string>& r) {
  if (r.empty()) return 0;
  size_t m = SIZE_MAX;
  for (auto& s : r) m = std::min(m, s.size());
  return m;
}

struct FactorCtx {
  size_t want = SIZE_MAX;  // shortest string the stride needs
};

// (the analysis runs ~4 times per regex at klf_open: candidate sets are moved, not copied,
// and a single-string candidate is only materialised when it wins -- allocations were most
// of the compile's time)
bool better(const FactorCtx& cx, const FInfo& f, size_t a, uint32_t pre, size_t n) {
  const size_t b = req_score(f.req);
  if (a == 0) return false;
  auto key = [&](size_t len, uint32_t p, size_t k) {
    return std::make_tuple(len >= cx.want ? 1 : 0, (len >= cx.want && p != kUnbounded) ? 1 : 0, len,
                           -(long)k);
  };
  return b == 0 || key(a, pre, n) > key(b, f.req_pre, f.req.size());
}
void consider(const FactorCtx& cx, FInfo& f, std::vector<std::string>&& r, bool loose, uint32_t pre) {
  if (!better(cx, f, req_score(r), pre, r.size())) return;
  f.req = std::move(r);
  f.req_loose = loose;
  f.req_pre = pre;
}
void consider_one(const FactorCtx& cx, FInfo& f, const std::string& run, bool loose, uint32_t pre) {
  if (!better(cx, f, run.size(), pre, 1)) return;
  f.req.assign(1, run);
  f.req_loose = loose;
  f.req_pre = pre;
}

std::vector<std::string> req_or_exact(const FInfo& f, bool& loose, uint32_t* pre = nullptr) {
  if (f.has_exact) {
    loose = f.exact_loose;
    if (pre) *pre = 0;
    return {f.exact};
  }
  loose = f.req_loose;
  if (pre) *pre = f.req_pre;
  return f.req;
}
// req_or_exact of a node result no longer needed: its strings moved out
std::vector<std::string> take_req_or_exact(FInfo&& f, bool& loose, uint32_t* pre = nullptr) {
  if (f.has_exact) {
    loose = f.exact_loose;
    if (pre) *pre = 0;
    std::vector<std::string> v(1);
    v[0] = std::move(f.exact);
    return v;
  }
  loose = f.req_loose;
  if (pre) *pre = f.req_pre;
  return std::move(f.req);
}

FInfo factor_of(const FactorCtx& cx, const std::vector<RNode>& pool, int x) {
  const RNode& n = pool[x];
  FInfo f;
  switch (n.k) {
    case RNode::kEmpty: case RNode::kBot: case RNode::kEot:
      f.has_exact = true;
      return f;
    case RNode::kSet: {
      f.maxlen = 1;
      const size_t c = n.set.count();
      int b0 = -1, b1 = -1;
      if (c <= 2) {
        b0 = (int)n.set._Find_first();
        if (c == 2) b1 = (int)n.set._Find_next((size_t)b0);
      }
      if (c == 1) {
        f.has_exact = true;
        f.exact.assign(1, (char)b0);
      } else if (c == 2 && b0 >= 'A' && b0 <= 'Z' && b1 == b0 + 32) {
        f.has_exact = true;
        f.exact.assign(1, (char)b1);
        f.exact_loose = true;
      }
      return f;
    }
    case RNode::kCat: {
      std::string run;
      bool run_loose = false, all = true;
      uint32_t off = 0, run_pre = 0;  // offset of the kid (bound), of the current exact run
      for (int k : n.kids) {
        FInfo kf = factor_of(cx, pool, k);
        consider(cx, f, std::move(kf.req), kf.req_loose, sat_add(off, kf.req_pre));
        if (kf.has_exact) {
          if (run.empty()) run_pre = off;
          run += kf.exact;
          run_loose |= kf.exact_loose;
        } else {
          if (!run.empty()) consider_one(cx, f, run, run_loose, run_pre);
          run.clear();
          run_loose = false;
          all = false;
        }
        off = sat_add(off, kf.maxlen);
      }
      if (!run.empty()) consider_one(cx, f, run, run_loose, run_pre);
      if (all) { f.has_exact = true; f.exact = run; f.exact_loose = run_loose; }
      f.maxlen = off;
      return f;
    }
    case RNode::kAlt: {
      std::vector<std::string> u;
      bool loose = false;
      uint32_t pre = 0;
      bool none = false;
      for (int k : n.kids) {
        bool l = false;
        uint32_t p = 0;
        FInfo kf = factor_of(cx, pool, k);
        f.maxlen = std::max(f.maxlen, kf.maxlen);
        const std::vector<std::string> r = take_req_or_exact(std::move(kf), l, &p);
        if (req_score(r) == 0) { none = true; continue; }  // some branch needs no byte at all
        loose |= l;
        pre = std::max(pre, p);
        for (auto& s : r)
          if (std::find(u.begin(), u.end(), s) == u.end()) u.push_back(s);
      }
      if (!none && u.size() <= 16) { f.req = u; f.req_loose = loose; f.req_pre = pre; }
      return f;
    }
    case RNode::kPlus: {
      FInfo kf = factor_of(cx, pool, n.kids[0]);
      f.maxlen = kf.maxlen == 0 ? 0 : kUnbounded;
      f.req = take_req_or_exact(std::move(kf), f.req_loose, &f.req_pre);  // the first repetition holds one
      return f;
    }
    case RNode::kRepeat: {
      FInfo kf = factor_of(cx, pool, n.kids[0]);
      f.maxlen = n.hi < 0 ? (kf.maxlen == 0 ? 0 : kUnbounded)
                          : (kf.maxlen == kUnbounded ? kUnbounded : kf.maxlen * (uint32_t)n.hi);
      if (n.lo == 0) return f;
      if (kf.has_exact) {
        std::string rep;
        for (int r = 0; r < n.lo && rep.size() <= kQfMaxFactor; ++r) rep += kf.exact;
        if (n.hi == n.lo) { f.has_exact = true; f.exact = rep; f.exact_loose = kf.exact_loose; }
        else { f.req = {rep}; f.req_loose = kf.exact_loose; f.req_pre = 0; }
        if (rep.empty()) f.req.clear();
      } else {
        f.req = std::move(kf.req);
        f.req_loose = kf.req_loose;
        f.req_pre = kf.req_pre;
      }
      return f;
    }
    case RNode::kStar: {
      const FInfo kf = factor_of(cx, pool, n.kids[0]);
      f.maxlen = kf.maxlen == 0 ? 0 : kUnbounded;
      return f;
    }
    default: {  // kQuest: a match may skip the node
      f.maxlen = factor_of(cx, pool, n.kids[0]).maxlen;
      return f;
    }
  }
}

}  // namespace

// Required factors of a parsed regex (regex_factors without the parse).
static bool factors_of(const std::vector<RNode>& pool, int root, std::vector<std::string>& alts, bool& loose,
                       uint32_t* pre, size_t want) {
  alts.clear();
  loose = false;
  if (pre) *pre = kUnbounded;
  if (root < 0) return false;
  FactorCtx cx;
  cx.want = want;
  uint32_t p = kUnbounded;
  alts = req_or_exact(factor_of(cx, pool, root), loose, &p);
  if (req_score(alts) == 0) { alts.clear(); return false; }
  for (auto& s : alts) {
    if (s.size() > kQfMaxFactor) s.resize(kQfMaxFactor);  // a substring of a factor is one too (its own start: same pre)
    if (loose)
      for (auto& c : s) c = (char)((uint8_t)c | 0x20);
  }
  std::sort(alts.begin(), alts.end());
  alts.erase(std::unique(alts.begin(), alts.end()), alts.end());
  if (pre) *pre = p;
  return true;
}

bool regex_factors(const uint8_t* pat, size_t n, std::vector<std::string>& alts, bool& loose, uint32_t* pre,
                   size_t want) {
  Parser ps(pat, n);
  const int root = ps.parse();
  return factors_of(ps.pool, root, alts, loose, pre, want);
}

void build_prefilter(const std::vector<std::vector<uint8_t>>& lits,
                     const std::vector<std::vector<std::vector<std::string>>>& fac_v,
                     const std::vector<std::vector<bool>>& loose_v, const std::vector<std::vector<uint32_t>>& pre_v,
                     CompiledSet& out, bool place);

// Glushkov tables of a parsed regex (the pool is rewritten: {m,n} expansion).
static bool build_glushkov(std::vector<RNode>& pool, int root, GlushkovTables& out, std::string& err, int& err_code) {
  Builder b(pool);
  if (b.count_pos(root) > kMaxRegexPositions) {
    err = "regex needs more than 64 Glushkov positions after {m,n} expansion";
    err_code = KLF_ETOOBIG;
    return false;
  }
  root = b.expand(root);
  Builder::Info info = b.glushkov(root);
  out = GlushkovTables();
  out.npos = b.npos;
  out.follow = b.follow;
  out.first = info.first;
  out.last = info.last;
  for (auto& s : b.pos_set) {
    std::vector<uint8_t> v(256);
    std::array<uint64_t, 4> m{0, 0, 0, 0};
    for (size_t c = s._Find_first(); c < 256; c = s._Find_next(c)) {
      v[c] = 1;
      m[c >> 6] |= 1ull << (c & 63);
    }
    out.pos_bytes.push_back(std::move(v));
    out.pos_bits.push_back(m);
  }
  bool acc0 = false;
  out.init0 = closure(info.first, b.a_bot, b.follow, info.last, &acc0);
  out.accept_at_start = info.nullable || acc0;
  bool acce = false;
  closure(info.first, b.a_bot | b.a_eot, b.follow, info.last, &acce);
  out.accept_empty = info.nullable || acce;
  // end_accept: EOT positions from which a chain of EOT passes reaches `last`
  uint64_t ea = 0;
  for (;;) {
    uint64_t nea = ea;
    for (int p = 0; p < out.npos; ++p)
      if ((b.a_eot >> p & 1) && (((info.last >> p) & 1) || (b.follow[p] & ea))) nea |= 1ull << p;
    if (nea == ea) break;
    ea = nea;
  }
  out.end_accept = ea;
  return true;
}

bool compile_regex(const uint8_t* pat, size_t n, GlushkovTables& out, std::string& err,
                   int& err_code) {
  Parser ps(pat, n);
  int root = ps.parse();
  if (root < 0) {
    err = ps.err;
    err_code = KLF_EPATTERN;
    return false;
  }
  return build_glushkov(ps.pool, root, out, err, err_code);
}

bool glushkov_match(const GlushkovTables& g, const uint8_t* s, size_t n) {
  if (n == 0) return g.accept_empty;
  if (g.accept_at_start) return true;
  uint64_t d = g.init0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t c = 0;
    for (int p = 0; p < g.npos; ++p)
      if ((d >> p & 1) && g.pos_bytes[p][s[i]]) c |= 1ull << p;
    if (c & g.last) return true;
    uint64_t nd = g.first;
    for (int p = 0; p < g.npos; ++p)
      if (c >> p & 1) nd |= g.follow[p];
    d = nd;
  }
  return (d & g.end_accept) != 0;
}

int log_byte_class(uint8_t c) {
  if (c >= 0x80 || (c < 0x20 && c != '\t')) return 1;          // control and high bytes
  if (strchr("!#$%&'*+;<>?@[\\]^_`|~", c) && c) return 2;        // rare punctuation
  if (c >= 'A' && c <= 'Z') return strchr("ERONWAIFDBUGT", c) ? 4 : 3;  // log-level letters are common
  if (c >= '0' && c <= '9') return 5;
  return 6;                                                    // lowercase, space, common punctuation
}

bool ac_alphabet_ok(const std::vector<std::vector<uint8_t>>& lits) {
  std::bitset<256> used;
  for (auto& l : lits)
    for (uint8_t c : l) used[c] = true;
  return used.count() <= 255;
}

void build_ac(const std::vector<std::vector<uint8_t>>& lits, AcTables& t) {
  t = AcTables();
  t.cls.assign(256, 0);
  uint32_t ncls = 1;
  {
    std::bitset<256> used;
    for (auto& l : lits)
      for (uint8_t c : l) used[c] = true;
    for (int c = 0; c < 256; ++c)
      if (used[c]) t.cls[c] = (uint8_t)ncls++;
  }
  // goto trie straight into the DFA table (0 = no child: the root is nobody's child),
  // then BFS: a state's missing edges copy its fail state's finished row
  size_t cap = 1;
  for (auto& l : lits) cap += l.size();
  std::vector<uint32_t> nxt(cap * (size_t)ncls, 0u);
  std::vector<uint8_t> term(cap, 0);
  std::vector<int32_t> term_id(cap, -1);  // literal id ending exactly at a state
  size_t ns = 1;
  for (size_t li = 0; li < lits.size(); ++li) {
    uint32_t st = 0;
    for (uint8_t c : lits[li]) {
      uint32_t& x = nxt[(size_t)st * ncls + t.cls[c]];
      if (!x) x = (uint32_t)ns++;
      st = x;
    }
    term[st] = 1;
    term_id[st] = (int32_t)li;
  }
  nxt.resize(ns * (size_t)ncls);
  t.states = (uint32_t)ns;
  t.classes = ncls;
  t.accept.assign(ns, 0);
  t.out.assign(term_id.begin(), term_id.begin() + ns);
  t.dict.assign(ns, 0u);
  std::vector<uint32_t> fail(ns, 0), queue;
  queue.reserve(ns);
  for (uint32_t c = 0; c < ncls; ++c)
    if (const uint32_t x = nxt[c]) queue.push_back(x);
  t.accept[0] = term[0];
  for (size_t qh = 0; qh < queue.size(); ++qh) {
    const uint32_t st = queue[qh];
    const uint32_t fs = fail[st];
    t.accept[st] = term[st] | t.accept[fs];
    // dictionary link: the nearest state on the fail chain where a literal ends
    t.dict[st] = (uint32_t)(term_id[fs] >= 0 ? (int)fs : (int)t.dict[fs]);
    uint32_t* row = &nxt[(size_t)st * ncls];
    const uint32_t* frow = &nxt[(size_t)fs * ncls];
    for (uint32_t c = 0; c < ncls; ++c) {
      if (const uint32_t x = row[c]) {  // a trie child (its row is still pure trie)
        fail[x] = frow[c];
        queue.push_back(x);
      } else {
        row[c] = frow[c];
      }
    }
  }
  t.next = std::move(nxt);
}

bool compile_set(const std::vector<std::vector<uint8_t>>& pats, const std::vector<uint32_t>& kinds,
                 CompiledSet& out, std::string& err, int& err_code, bool place, bool defer_also_all,
                 bool defer_ac) {
  out = CompiledSet();
  if (pats.empty()) {
    out.mode = CompiledSet::kNone;
    return true;
  }
  if (pats.size() > (size_t)kMaxRegexes * 64) {
    err = "too many patterns";
    err_code = KLF_ETOOBIG;
    return false;
  }
  std::vector<std::vector<uint8_t>> lits;
  std::vector<GlushkovTables> rxs;
  std::vector<std::vector<std::string>> rx_fac;  // required factors per regex (prefilter)
  std::vector<bool> rx_loose;
  std::vector<uint32_t> rx_pre;
  std::vector<size_t> rx_src;  // pattern index of each kept regex
  std::vector<std::vector<RNode>> rx_tree;  // parse tree of each kept regex
  std::vector<int> rx_root;
  std::vector<size_t> always_rx;  // regexes that match every content
  bool always = false;
  auto drop_nl = [](std::vector<std::string>& alts) {  // content never holds '\n'
    alts.erase(std::remove_if(alts.begin(), alts.end(),
                              [](const std::string& f) { return f.find('\n') != std::string::npos; }),
               alts.end());
  };
  // Each regex compiled on its own (parse, Glushkov tables, required factors), then gathered
  // in pattern order, the first error by pattern index.  KLF_COMPILE_THREADS=n spreads them
  // over n host threads (measured: slower than one thread for C5's 64 regexes -- thread
  // start-up outweighs ~5 us per regex -- so one by default)
  struct RxOut {
    bool ok = false, always = false, never = false, have_fac = false;
    std::string err;
    int code = 0;
    int root = -1;
    std::vector<RNode> pool;
    GlushkovTables g;
    std::vector<std::string> alts;
    bool loose = false;
    uint32_t pre = kRxPreUnbounded;
  };
  std::vector<RxOut> rxo(pats.size());
  // KLF_DIAG: the compile's phases (klf_open's "pattern compile" mark is their sum)
  static const bool cdiag = getenv("KLF_DIAG") != nullptr;
  const auto ct0 = std::chrono::steady_clock::now();
  auto cmark = [&](const char* what) {
    if (cdiag)
      fprintf(stderr, "[klf] compile: %s at %.1f us\n", what,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - ct0).count());
  };
  auto compile_rx = [&](size_t k) {
    RxOut& o = rxo[k];
    // parsed once: the factor analyses read the tree, the Glushkov build rewrites a copy
    Parser ps(pats[k].data(), pats[k].size());
    o.root = ps.parse();
    if (o.root < 0) {
      o.err = "pattern " + std::to_string(k) + ": " + ps.err;
      o.code = KLF_EPATTERN;
      return;
    }
    {
      std::vector<RNode> work = ps.pool;
      if (!build_glushkov(work, o.root, o.g, o.err, o.code)) {
        o.err = "pattern " + std::to_string(k) + ": " + o.err;
        return;
      }
    }
    o.ok = true;
    if (o.g.accept_at_start && o.g.accept_empty) { o.always = true; return; }
    o.pool = std::move(ps.pool);
    if (factors_of(o.pool, o.root, o.alts, o.loose, &o.pre, SIZE_MAX)) {
      // such alternatives cannot occur; none left = no match ever
      drop_nl(o.alts);
      if (o.alts.empty()) o.never = true;
    }
  };
  {
    std::vector<size_t> rk;
    for (size_t k = 0; k < pats.size(); ++k)
      if (kinds[k] == KLF_PAT_REGEX) rk.push_back(k);
    size_t nthr = 1;
    if (const char* v = getenv("KLF_COMPILE_THREADS")) nthr = std::max<size_t>(1, (size_t)atol(v));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nthr; ++t)
      th.emplace_back([&, t]() { for (size_t i = t; i < rk.size(); i += nthr) compile_rx(rk[i]); });
    for (size_t i = 0; i < rk.size(); i += nthr) compile_rx(rk[i]);
    for (auto& x : th) x.join();
  }
  for (size_t k = 0; k < pats.size(); ++k) {
    if (kinds[k] == KLF_PAT_LITERAL) {
      const auto& l = pats[k];
      if (l.empty()) { always = true; continue; }  // bytes.Contains(x, "") == true
      if (std::find(l.begin(), l.end(), (uint8_t)'\n') != l.end()) continue;  // never in content
      lits.push_back(l);
    } else if (kinds[k] == KLF_PAT_REGEX) {
      RxOut& o = rxo[k];
      if (!o.ok) {
        err = o.err;
        err_code = o.code;
        return false;
      }
      if (o.always) { always_rx.push_back(k); always = true; continue; }
      if (o.never) continue;
      rxs.push_back(std::move(o.g));
      rx_tree.push_back(std::move(o.pool));
      rx_root.push_back(o.root);
      rx_fac.push_back(std::move(o.alts));
      rx_loose.push_back(o.loose);
      rx_pre.push_back(o.pre);
      rx_src.push_back(k);
    } else {
      err = "unknown pattern kind";
      err_code = KLF_EINVAL;
      return false;
    }
  }
  if (rxs.size() > (size_t)kMaxRegexes) {
    err = "more than 1024 regexes";
    err_code = KLF_ETOOBIG;
    return false;
  }
  cmark("regexes parsed");
  // Second pass: two factor choices per regex for the layout to pick from (place_needles,
  // with the data's statistics at the first batch).  [0]: the sampling stride follows the
  // shortest needle of the first pass; keep it, and per regex prefer factor sets with a
  // bounded match-start window (rx_pre).  [1]: prefer sets of >= 10 bytes (stride 8), the
  // shorter needles left then being anchored on a rare byte when they share one.
  std::vector<std::vector<std::vector<std::string>>> fac_v;
  std::vector<std::vector<bool>> loose_v;
  std::vector<std::vector<uint32_t>> pre_v;
  {
    size_t g = SIZE_MAX;
    for (auto& l : lits) g = std::min(g, l.size());
    for (auto& f : rx_fac)
      for (auto& x : f) g = std::min(g, x.size());
    const size_t want0 = g >= 10 ? 10 : g >= 8 ? 8 : g >= 6 ? 6 : g >= 4 ? 4 : 3;  // = the stride rule
    // (8-byte needles allow the stride-6 grid, whose windows then span a whole needle of 8:
    // the 6-byte choice at stride 4 stays a candidate, the layout cost decides)
    std::vector<size_t> wants = {want0};
    if (want0 == 8) wants.push_back(6);
    if (want0 != 10) wants.push_back(10);
    for (size_t want : wants) {
      auto fac = rx_fac;
      auto lo = rx_loose;
      auto pr = rx_pre;
      for (size_t r = 0; r < fac.size(); ++r) {
        if (fac[r].empty()) continue;
        std::vector<std::string> alts;
        bool loose = false;
        uint32_t pre = kRxPreUnbounded;
        if (!factors_of(rx_tree[r], rx_root[r], alts, loose, &pre, want)) continue;
        drop_nl(alts);
        size_t m = SIZE_MAX;
        for (auto& x : alts) m = std::min(m, x.size());
        if (alts.empty() || m < want) continue;
        fac[r] = alts;
        lo[r] = loose;
        pr[r] = pre;
      }
      if (std::find(fac_v.begin(), fac_v.end(), fac) != fac_v.end()) continue;  // the same choice
      fac_v.push_back(fac);
      loose_v.push_back(lo);
      pre_v.push_back(pr);
    }
  }
  out.rx_pre = pre_v[0];
  cmark("factor choices");
  // dedupe literals
  std::sort(lits.begin(), lits.end());
  lits.erase(std::unique(lits.begin(), lits.end()), lits.end());
  {  // per-pattern counts: user pattern -> compiled id (literals, then regexes)
    out.n_cids = (uint32_t)(lits.size() + rxs.size());
    out.n_lits = (uint32_t)lits.size();
    out.user_map.assign(pats.size(), CompiledSet::kCidNever);
    size_t r = 0;
    for (size_t k = 0; k < pats.size(); ++k) {
      if (kinds[k] == KLF_PAT_LITERAL) {
        const auto& l = pats[k];
        if (l.empty()) { out.user_map[k] = CompiledSet::kCidAlways; continue; }
        if (std::find(l.begin(), l.end(), (uint8_t)'\n') != l.end()) continue;
        out.user_map[k] = (int32_t)(std::lower_bound(lits.begin(), lits.end(), l) - lits.begin());
      } else {
        while (r < rx_src.size() && rx_src[r] < k) ++r;
        if (r < rx_src.size() && rx_src[r] == k) out.user_map[k] = (int32_t)(lits.size() + r);
      }
    }
    for (size_t k : always_rx) out.user_map[k] = CompiledSet::kCidAlways;  // regexes that match every content
  }
  if (always && lits.empty() && rxs.empty()) { out.mode = CompiledSet::kAll; return true; }
  if (lits.empty() && rxs.empty()) { out.mode = CompiledSet::kNever; return true; }
  // an always-pattern beside real ones: the general tables (counted per pattern), kAll's
  // filter (also_all); deferred, kAll until a run asks for per-pattern counts
  out.also_all = always;
  if (always && defer_also_all) {
    out.mode = CompiledSet::kAll;
    out.also_all_pending = true;
    return true;
  }
  if (!always && rxs.empty() && lits.size() == 1 && lits[0].size() <= 256) {
    out.mode = CompiledSet::kLiteral1;
    out.literal = lits[0];
    int best = 99;
    for (size_t i = 0; i < out.literal.size(); ++i) {
      const int cl = log_byte_class(out.literal[i]);
      if (cl < best) { best = cl; out.literal_anchor = (uint32_t)i; }
    }
    return true;
  }
  out.mode = CompiledSet::kGeneral;

  // ---- Aho-Corasick over the literals ----
  if (!lits.empty()) {
    if (!ac_alphabet_ok(lits)) { err = "literal alphabet too large"; err_code = KLF_ETOOBIG; return false; }
    if (defer_ac) {
      out.ac_lits = lits;
    } else {
      AcTables t;
      build_ac(lits, t);
      out.ac_states = t.states;
      out.ac_classes = t.classes;
      out.ac_class = std::move(t.cls);
      out.ac_next = std::move(t.next);
      out.ac_accept = std::move(t.accept);
      out.ac_out = std::move(t.out);
      out.ac_dict = std::move(t.dict);
    }
  }

  // ---- regexes: shared byte classes by partition refinement ----
  cmark("automaton");
  out.rx_count = (uint32_t)rxs.size();
  if (!rxs.empty()) {
    // a byte's signature = the positions (per regex) whose set holds it; equal signatures
    // share a class, numbered in order of the first byte that has it
    const size_t words = rxs.size();
    std::vector<uint64_t> sig((size_t)256 * words, 0);
    for (size_t r = 0; r < words; ++r)
      for (int p = 0; p < rxs[r].npos; ++p)
        for (int w = 0; w < 4; ++w)
          for (uint64_t m = rxs[r].pos_bits[p][w]; m; m &= m - 1)
            sig[(size_t)(w * 64 + __builtin_ctzll(m)) * words + r] |= 1ull << p;
    std::unordered_map<std::string, int> sig2cls;
    std::vector<int> rep;  // first byte of each class
    out.rx_class.assign(256, 0);
    for (int c = 0; c < 256; ++c) {
      std::string key(reinterpret_cast<const char*>(&sig[(size_t)c * words]), words * 8);
      auto it = sig2cls.emplace(std::move(key), (int)rep.size());
      if (it.second) rep.push_back(c);
      out.rx_class[c] = (uint8_t)it.first->second;
    }
    out.rx_classes = (uint32_t)rep.size();
    out.rx_b.assign((size_t)rxs.size() * out.rx_classes, 0);
    for (size_t cl = 0; cl < rep.size(); ++cl)
      for (size_t r = 0; r < rxs.size(); ++r) out.rx_b[r * out.rx_classes + cl] = sig[(size_t)rep[cl] * words + r];
    out.rx_follow.assign((size_t)rxs.size() * 64, 0);
    for (size_t r = 0; r < rxs.size(); ++r) {
      for (int p = 0; p < rxs[r].npos; ++p) out.rx_follow[r * 64 + p] = rxs[r].follow[p];
      out.rx_maxpos = std::max<uint32_t>(out.rx_maxpos, (uint32_t)rxs[r].npos);
      out.rx_first.push_back(rxs[r].first);
      out.rx_last.push_back(rxs[r].last);
      out.rx_init0.push_back(rxs[r].init0);
      out.rx_end.push_back(rxs[r].end_accept);
      out.rx_flags.push_back((rxs[r].accept_at_start ? 1u : 0u) | (rxs[r].accept_empty ? 2u : 0u));
    }
  }
  cmark("byte classes");
  build_prefilter(lits, fac_v, loose_v, pre_v, out, place);
  cmark("prefilter");
  return true;
}

// q-gram prefilter tables (CompiledSet::qf_*).  Off (k_match decides every line) when a
// literal or some regex's best factor is shorter than kQfMinNeedle, or a regex can match
// without any factor (e.g. `\d+`): those need a look at every line anyway.
//
// Each needle is sampled through a window of q + S - 1 of its bytes (any substring of a
// literal / factor occurs wherever the needle does); place_needles picks the layout, the
// needle set (one per factor choice, fac_v) and the windows.
void build_prefilter(const std::vector<std::vector<uint8_t>>& lits,
                     const std::vector<std::vector<std::vector<std::string>>>& fac_v,
                     const std::vector<std::vector<bool>>& loose_v, const std::vector<std::vector<uint32_t>>& pre_v,
                     CompiledSet& out, bool place) {
  out.qf_variants.clear();
  bool loose = false;
  for (size_t v = 0; v < fac_v.size(); ++v) {
    CompiledSet::NeedleSet ns;
    for (size_t i = 0; i < lits.size(); ++i) {
      ns.s.push_back(std::string(lits[i].begin(), lits[i].end()));
      ns.flags.push_back(0u);
      ns.rx.push_back((uint32_t)i);
    }
    const auto& rx_fac = fac_v[v];
    for (size_t r = 0; r < rx_fac.size(); ++r) {
      if (rx_fac[r].empty()) { out.qf_why = "regex " + std::to_string(r) + " has no required literal factor"; return; }
      for (auto& f : rx_fac[r]) {
        ns.s.push_back(f);
        ns.flags.push_back(kQfRegex | (loose_v[v][r] ? kQfLoose : 0u));
        ns.rx.push_back((uint32_t)r);
        loose |= loose_v[v][r];
      }
    }
    if (ns.s.empty()) { out.qf_why = "no needles"; return; }
    if (ns.s.size() > (1u << 24)) { out.qf_why = "too many needles"; return; }
    size_t minlen = SIZE_MAX;
    for (auto& x : ns.s) minlen = std::min(minlen, x.size());
    if (minlen < kQfMinNeedle) {
      if (v == 0) { out.qf_why = "a needle is shorter than 3 bytes"; return; }
      break;
    }
    ns.rx_pre = pre_v[v];
    out.qf_variants.push_back(std::move(ns));
  }
  out.qf_fold = loose ? 0x20202020u : 0u;  // grams of every variant fold alike
  out.qf_on = true;
  if (place) place_needles(out, nullptr);
}

namespace {

// The widest sampling stride whose windows (q + S - 1 bytes, grams of q >= 3 bytes) fit
// every needle of length >= minlen (each probe costs ~6-13 VALU in the scan, so S = 8
// halves the probe work of S = 4; S = 6 is the 3-per-16-B grid, qf_sampled), then the
// longest gram that stride allows.
void stride_rule(size_t minlen, uint32_t& S, uint32_t& q) {
  const size_t sw = std::min<size_t>(8, minlen - 2);
  static const bool grid6 = !(getenv("KLF_QF_GRID6") && !strcmp(getenv("KLF_QF_GRID6"), "0"));
  S = sw >= 8 ? 8 : (sw >= 6 && grid6) ? 6 : (sw >= 4 ? 4 : (sw >= 2 ? 2 : 1));
  q = (uint32_t)std::min<size_t>(4, minlen - S + 1);
}

// Estimated share of data positions holding byte c (anchors of short needles): the sample's
// byte histogram, else the byte-class guess of log text.
double byte_share(uint32_t c, uint32_t fold, const DataStats* st) {
  if (st && st->nbytes) {
    uint64_t n = st->bytes[c];
    if (fold && (c & 0x20u)) n += st->bytes[c & ~0x20u];  // loose: both cases
    return (double)n / (double)st->nbytes;
  }
  uint8_t b = (uint8_t)c;
  if (b >= 'a' && b <= 'z') return 1.0 / 20;
  if (b == ' ' || (b >= '0' && b <= '9')) return 1.0 / 20;
  if (b && strchr("\":,=./{}-TZ", b)) return 1.0 / 60;
  return 1.0 / 2000;
}

// Picks the layout: all needles probed at the stride of the shortest, or (when that
// stride is below 8 and the needles shorter than 10 bytes share a rare byte) the long
// needles probed at stride 8 and the short ones anchored.
void choose_layout(CompiledSet& out, const DataStats* st, bool allow_anchor, uint32_t qmax = 4) {
  const auto& nd = out.qf_needle;
  const size_t n = nd.size();
  size_t minlen = SIZE_MAX, minlong = SIZE_MAX;
  for (auto& x : nd) {
    minlen = std::min(minlen, x.size());
    if (x.size() >= 10) minlong = std::min(minlong, x.size());
  }
  uint32_t S, q;
  stride_rule(minlen, S, q);
  q = std::min(q, qmax);
  out.qf_anc_on = false;
  out.qf_anc_pre.clear();
  out.qf_nshort.assign(n, 0);
  out.qf_nanc.assign(n, 0);
  out.qf_layout = "all probed, S=" + std::to_string(S) + " q=" + std::to_string(q);
  const char* env = getenv("KLF_QF_ANCHOR");  // tests / ablation: 0 never anchors
  if (allow_anchor && S < 8 && minlong != SIZE_MAX && !(env && !strcmp(env, "0"))) {
    uint32_t Sl, ql;
    stride_rule(minlong, Sl, ql);
    ql = std::min(ql, qmax);
    uint32_t afold = 0;
    for (size_t i = 0; i < n; ++i)
      if (nd[i].size() < 10 && (out.qf_nflags[i] & kQfLoose)) afold = 0x20202020u;
    // candidate anchors: a byte every short needle holds at an offset <= len - q (the
    // bucket's gram at the anchor lies inside the needle); 3-byte grams when no byte
    // qualifies for 4-byte ones
    // more common than 1 in 256 bytes: not worth it (tests: KLF_QF_ANCHOR=force takes any)
    const double limit = (env && !strcmp(env, "force")) ? 2.0 : 1.0 / 256;
    double best = limit;
    int best_c = -1;
    for (uint32_t qq = ql; qq >= 3 && best_c < 0; --qq) {
      // bytes every short needle holds at an offset <= len - qq: the intersection of the
      // needles' byte sets (first occurrences, as the pre-check records them)
      std::bitset<256> common;
      common.set();
      for (size_t i = 0; i < n && common.any(); ++i) {
        if (nd[i].size() >= 10) continue;
        const size_t lim = nd[i].size() - qq;
        std::bitset<256> has, seen_b;
        for (size_t k = 0; k < nd[i].size(); ++k) {
          const uint8_t b = (uint8_t)nd[i][k];
          if (seen_b.test(b)) continue;  // (its first occurrence decides)
          seen_b.set(b);
          if (k <= lim) has.set(b);
        }
        common &= has;
      }
      for (uint32_t c = 0; c < 256; ++c) {
        if (!common.test(c) || c == '\n') continue;
        if (afold && ((c | 0x20u) != c)) continue;  // stored loose bytes carry bit 5
        const double sh = byte_share(c, afold, st);
        if (sh < best) { best = sh; best_c = (int)c; }
      }
      if (best_c >= 0) ql = qq;
    }
    if (best_c >= 0) {
      std::vector<std::pair<uint32_t, uint32_t>> pre;
      for (size_t i = 0; i < n; ++i) {
        if (nd[i].size() >= 10) continue;
        const uint32_t a = (uint32_t)nd[i].find((char)best_c);
        const uint32_t m = (uint32_t)std::min<size_t>(4, nd[i].size() - a);
        uint32_t w = 0;
        for (uint32_t b = 0; b < m; ++b) w |= (uint32_t)(uint8_t)nd[i][a + b] << (8 * b);
        const uint32_t mask = m == 4 ? ~0u : (1u << (8 * m)) - 1u;
        pre.push_back({(w | out.qf_fold) & mask, mask});
        out.qf_nshort[i] = 1;
        out.qf_nanc[i] = a;
      }
      std::sort(pre.begin(), pre.end());
      pre.erase(std::unique(pre.begin(), pre.end()), pre.end());
      if (pre.size() <= kQfAncPreMax) {
        S = Sl;
        q = ql;
        out.qf_anc_on = true;
        out.qf_anc_share = best;
        out.qf_anc_byte = (uint32_t)best_c;
        out.qf_anc_fold = afold;
        for (auto& x : pre) {
          out.qf_anc_pre.push_back(x.first);
          out.qf_anc_pre.push_back(x.second);
        }
        char buf[160];
        snprintf(buf, sizeof buf, "long needles probed S=%u q=%u; short ones anchored at 0x%02x (share %.2e, %zu pre-checks)",
                 S, q, (unsigned)best_c, best, pre.size());
        out.qf_layout = buf;
      } else {
        out.qf_nshort.assign(n, 0);
      }
    }
  }
  out.qf_q = q;
  out.qf_stride = S;
  out.qf_mask = q == 4 ? ~0u : ((1u << (8 * q)) - 1u);
}

// Estimated scan work per 8 KiB tile of a placed layout on the sample's statistics, in
// VALU-instruction units of one wave: the probes (~11 each, a lane per 128 B), the anchor
// test, and every hit (bitmap or anchor: the exact pass in the scan, the recording, the
// verification) at ~40.  Hits per tile = samples per tile x the summed data share of the
// sampled grams, plus the anchors whose dword passes a pre-check.
double layout_cost(const CompiledSet& c, const DataStats& st) {
  std::vector<uint32_t> grams;
  grams.reserve(c.qf_ent.size() / 4);
  for (size_t e = 0; e + 3 < c.qf_ent.size(); e += 4) {  // the probed grams, read back from the needles
    if (c.qf_ent[e + 1] & kQfAnchored) continue;
    const uint32_t off = c.qf_ent[e], len = c.qf_ent[e + 1] & 0xFFFFu, k = (c.qf_ent[e + 1] >> 16) & 0xFFu;
    const uint8_t* nb8 = reinterpret_cast<const uint8_t*>(c.qf_nbytes.data() + off);
    uint32_t g = 0;
    for (uint32_t b = 0; b < c.qf_q && k + b < len; ++b) g |= (uint32_t)nb8[k + b] << (8 * b);
    grams.push_back((g | c.qf_fold) & c.qf_mask);
  }
  // distinct grams through an open-addressing set (top bits of a product; sorting them was
  // most of the cost's time)
  size_t cap = 64;
  uint32_t shift = 26;
  while (cap < 2 * grams.size()) cap <<= 1, --shift;
  std::vector<uint32_t> seen(cap, ~0u);
  double hit_share = 0;  // probed grams (the anchored ones only reach a bucket through an anchor)
  for (uint32_t g : grams) {
    uint32_t i = (g * 0x9E3779B1u) >> shift;
    while (seen[i] != ~0u && seen[i] != g) i = (i + 1) & (uint32_t)(cap - 1);
    if (seen[i] == g) continue;
    seen[i] = g;
    hit_share += gram_share(st, g, c.qf_q);
  }
  const double samples = qf_samples_per_tile(c.qf_stride);
  double hits = samples * std::min(1.0, hit_share);
  // VALU per probe (the scan's ISA, its unrolled fast pass / 32 probes): 6.9 for a 3-byte
  // gram with two bits (fold, multiply, word offset, two shifts, and / or), 9.9 with the
  // fourth byte, 13.4 for 3 bits (folded gram, two more multiplies, a shift)
  // (two-level: ~5 per sample for the pair stage, the 3-bit probe on the ~5 % survivors)
  const double per_probe = c.qf_k == kQfTwoLevel ? 6.0 + (c.qf_q == 4 ? 1.0 : 0.0)
                                                 : 7.0 + (c.qf_q == 4 ? 3.0 : 0.0) + (c.qf_k == 3 ? 6.5 : 0.0);
  double cost = per_probe * samples / 64.0;
  if (c.qf_anc_on) {
    cost += 60.0;
    double pass = 0;
    for (size_t j = 0; j + 1 < c.qf_anc_pre.size(); j += 2)
      pass += c.qf_anc_pre[j + 1] == ~0u ? gram_share(st, c.qf_anc_pre[j], 4)
                                         : gram_share(st, c.qf_anc_pre[j] & 0xFFFFFFu, 3);
    hits += 8192.0 * std::min(1.0, pass);
  }
  return cost + 40.0 * hits;
}

void place_tables(CompiledSet& out, const DataStats* st);

}  // namespace

// The layout: each needle set (factor choice) with every needle probed, and, where short
// needles can be anchored, with the long ones probed at stride 8.  With the data's
// statistics the cheapest by layout_cost wins; without them (klf_open, before any batch)
// the widest stride, then the rarest anchor.
void place_needles(CompiledSet& out, const DataStats* st) {
  // the matcher tables play no part in the layout: kept aside while the candidates are
  // copied (a 1,024-literal set's AC automaton is megabytes per copy)
  std::vector<uint32_t> ac_next, ac_dict;
  std::vector<uint8_t> ac_accept;
  std::vector<int32_t> ac_out;
  std::vector<uint64_t> rx_b, rx_follow;
  std::vector<CompiledSet::NeedleSet> variants;  // read-only here: not copied per candidate
  std::vector<int32_t> user_map;
  ac_next.swap(out.ac_next);
  ac_dict.swap(out.ac_dict);
  ac_accept.swap(out.ac_accept);
  ac_out.swap(out.ac_out);
  rx_b.swap(out.rx_b);
  rx_follow.swap(out.rx_follow);
  variants.swap(out.qf_variants);
  user_map.swap(out.user_map);
  CompiledSet best;
  double best_cost = 0;
  bool have = false;
  std::vector<std::string> seen;  // layouts already placed (a 3-byte cap can give the 4-byte one's)
  for (uint32_t v = 0; v < variants.size(); ++v)
    for (int cand = 0; cand < 4; ++cand) {
      const int anchored = cand & 1;
      const uint32_t qmax = cand < 2 ? 4u : 3u;  // 3-byte grams: a cheaper probe, more hits
      if (qmax == 3 && !(st && st->nbytes)) continue;  // (only the data can say whether they pay)
      if (const char* qv = getenv("KLF_QF_QMAX"))  // ablation: one gram length at the data's layout
        if (st && st->nbytes && (uint32_t)atoi(qv) != qmax) continue;
      CompiledSet c = out;
      const auto& ns = variants[v];
      c.qf_variant = v;
      c.qf_needle = ns.s;
      c.qf_nflags = ns.flags;
      c.qf_nrx = ns.rx;
      c.qf_needles = (uint32_t)ns.s.size();
      c.rx_pre = ns.rx_pre;
      choose_layout(c, st, anchored != 0, qmax);
      if (anchored && !c.qf_anc_on) continue;  // nothing to anchor: same as the probed layout
      {
        const std::string key = std::to_string(v) + "/" + c.qf_layout;
        if (std::find(seen.begin(), seen.end(), key) != seen.end()) continue;  // placed already
        seen.push_back(key);
      }
      const auto t0 = std::chrono::steady_clock::now();
      place_tables(c, st);
      const auto t1 = std::chrono::steady_clock::now();
      double cost;
      if (st && st->nbytes) {
        cost = layout_cost(c, *st);
      } else {  // no statistics: stride first (8 is ~2x cheaper than 4), then the anchor's share
        cost = 1e6 * qf_samples_per_tile(c.qf_stride) / 8192.0 + (c.qf_anc_on ? c.qf_anc_share * 1e3 : 0.0);
      }
      char buf[64];
      snprintf(buf, sizeof buf, " [est %.0f VALU/tile]", cost);
      c.qf_layout += buf;
      if (getenv("KLF_DIAG"))
        fprintf(stderr, "[klf] layout candidate (variant %u): %s (tables %.0f us, cost %.0f us)\n", v, c.qf_layout.c_str(),
                std::chrono::duration<double, std::micro>(t1 - t0).count(),
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
      if (!have || cost < best_cost) {
        best = std::move(c);
        best_cost = cost;
        have = true;
      }
    }
  if (have) out = std::move(best);  // (every candidate skipped: the layout stays as it was)
  out.qf_variants.swap(variants);
  out.user_map.swap(user_map);
  out.ac_next.swap(ac_next);
  out.ac_dict.swap(ac_dict);
  out.ac_accept.swap(ac_accept);
  out.ac_out.swap(ac_out);
  out.rx_b.swap(rx_b);
  out.rx_follow.swap(rx_follow);
}

namespace {

// Window choice + tables.  Each probed needle is sampled through q + S - 1 of its bytes:
// the window whose S grams are the least frequent -- by gram_share on the data's 2-gram
// statistics when given (k_gramhist over a sample of the first batch), else by a
// byte-class estimate -- with a small penalty for grams other needles already sample
// (bucket length).  Every probed gram sets K bits of one bitmap word (blocked Bloom); an
// anchored needle has one bucket entry, at its anchor's gram, and no bitmap bits.
void place_tables(CompiledSet& out, const DataStats* st) {
  const uint32_t q = out.qf_q, S = out.qf_stride;
  const bool hist = st && st->pair.size() >= 65536 && st->pair_tot > 0;  // data statistics
  const double nsample = st && st->nbytes ? (double)st->nbytes : 1.0;
  // a window's score: the summed shares of its S grams (one of them is sampled per
  // occurrence), plus, under the two-level probe, a twentieth of each gram's leading pair
  // share (the pair stage passes those samples to the hashed Bloom word, whose false
  // positives they then risk)
  static const double pair_w = getenv("KLF_QF_PAIRW") ? atof(getenv("KLF_QF_PAIRW")) : 0.05;
  const bool loose = out.qf_fold != 0;
  out.qf_bitmap.assign(kQfWords, 0u);
  out.qf_head.clear();
  out.qf_ent.clear();
  out.qf_nbytes.clear();
  auto gram_at = [&](const std::string& s, uint32_t k) {
    uint32_t g = 0;
    for (uint32_t b = 0; b < q; ++b) g |= (uint32_t)(uint8_t)s[k + b] << (8 * b);
    return (g | out.qf_fold) & out.qf_mask;
  };
  uint8_t rank[256];  // rough frequency rank of a byte in log text
  for (uint32_t c0 = 0; c0 < 256; ++c0) {
    uint8_t c = (uint8_t)c0;
    if (loose && c >= 'A' && c <= 'Z') c |= 0x20;
    rank[c0] = ((c >= 'a' && c <= 'z') || c == ' ' || (c >= '0' && c <= '9')) ? 4  // words, numbers, timestamps
               : (c && strchr("\":,=./{}-TZ", c)) ? 3                             // JSON / timestamp punctuation
               : 1;  // upper case, '_', other punctuation, control and high bytes
  }
  auto common = [&](uint8_t c) -> int { return rank[c]; };
  // gram -> needles sampling it so far: a flat open-addressing table (grams are < 2^32 - 1)
  struct Used {
    std::vector<uint32_t> key, cnt;
    uint32_t mask, shift;
    explicit Used(size_t n) {
      size_t cap = 64;
      shift = 26;
      while (cap < 2 * n) cap <<= 1, --shift;
      key.assign(cap, ~0u);
      cnt.assign(cap, 0u);
      mask = (uint32_t)cap - 1;
    }
    // the product's top bits (its low bits follow only the gram's low bytes, which needles
    // with a common prefix share: linear probing then walked long clusters)
    uint32_t slot(uint32_t g) const {
      uint32_t i = (g * 0x9E3779B1u) >> shift;
      while (key[i] != ~0u && key[i] != g) i = (i + 1) & mask;
      return i;
    }
    uint32_t get(uint32_t g) const { return cnt[slot(g)]; }
    void add(uint32_t g) {
      const uint32_t i = slot(g);
      key[i] = g;
      ++cnt[i];
    }
  } used(out.qf_needle.size() * S + 1);
  std::vector<uint64_t> gcost;             // a needle's gram costs by offset
  std::vector<std::pair<uint32_t, uint32_t>> bent;  // (bucket, needle << 8 | gram offset), in needle order
  bent.reserve(out.qf_needle.size() * S);
  const size_t n = out.qf_needle.size();
  size_t nprobed = 0;
  for (size_t i = 0; i < n; ++i) nprobed += out.qf_nshort[i] ? 0 : 1;
  // few grams: two bits per gram keep the false hits rare; many at stride 4: the two-level
  // probe (an exact 2-gram stage, then three bits; KLF_QF_TWO=0 keeps the one-level one)
  const char* two = getenv("KLF_QF_TWO");
  const bool two_ok = S == 4 && !out.qf_anc_on && !(two && !strcmp(two, "0"));
  out.qf_k = (two_ok && two && !strcmp(two, "force")) ? kQfTwoLevel
             : nprobed * S <= kQfK2MaxGrams ? 2u : two_ok ? kQfTwoLevel : 3u;
  const uint32_t w24 = q == 4 ? 24u : 0u;
  for (uint32_t i = 0; i < n; ++i) {
    const std::string& s = out.qf_needle[i];
    if (out.qf_nshort[i]) {  // anchored: the bucket of the gram at the anchor
      const uint32_t k = out.qf_nanc[i], g = gram_at(s, k);
      bent.push_back({qf_bucket(g, w24, out.qf_k), i << 8 | k});
      continue;
    }
    const uint32_t amax = (uint32_t)std::min<size_t>(s.size() - (q + S - 1), 255 - (S - 1));
    // each gram's cost once (a gram lies in up to S windows), then the windows
    gcost.resize(amax + S);
    for (uint32_t k = 0; k < amax + S; ++k) {
      const uint32_t g = gram_at(s, k);
      const uint64_t u = used.get(g);
      uint64_t c;
      if (hist) {
        double sh = gram_share(*st, g, q);
        if (pair_w > 0 && out.qf_k == kQfTwoLevel && st->pair_tot > 0)  // the pair stage's survivors
          sh += pair_w * (st->pair[g & 0xFFFFu] + 0.5) / st->pair_tot;
        c = (uint64_t)(sh * nsample * 256.0) + 2 * u;
      } else {
        c = 2 * u;
        for (uint32_t b = 0; b < q; ++b) c += common((uint8_t)s[k + b]);
      }
      gcost[k] = c;
    }
    uint32_t best_a = 0;
    uint64_t best = UINT64_MAX;
    for (uint32_t a = 0; a <= amax; ++a) {
      uint64_t sc = 0;
      for (uint32_t j = 0; j < S; ++j) sc = hist ? sc + gcost[a + j] : std::max(sc, gcost[a + j]);
      if (sc < best) { best = sc; best_a = a; }
    }
    for (uint32_t j = 0; j < S; ++j) {
      const uint32_t k = best_a + j, g = gram_at(s, k);
      used.add(g);
      const uint32_t h = qf_hash(g, w24, out.qf_k);
      const uint32_t bw = qf_bucket(g, w24, out.qf_k);
      out.qf_bitmap[qf_bloom_word(g, w24, out.qf_k)] |= qf_bits(g, h, out.qf_k);
      if (out.qf_k == kQfTwoLevel) {  // the exact pair set, over raw bytes: every case variant
        const uint32_t g16 = g & 0xFFFFu, fv = out.qf_fold & 0xFFFFu & g16;
        for (uint32_t x = fv;; x = (x - 1u) & fv) {  // subsets of the folded bits
          const uint32_t pr = g16 & ~x;
          out.qf_bitmap[qf_pair_word(pr)] |= 1u << (pr & 31u);
          if (!x) break;
        }
      }
      bent.push_back({bw, i << 8 | k});
    }
  }
  // needle bytes (loose needles are already stored OR 0x20), then 16-B entries per bucket
  std::vector<uint32_t> noff;
  for (auto& ns : out.qf_needle) {
    noff.push_back((uint32_t)out.qf_nbytes.size());
    for (size_t b = 0; b < ns.size(); b += 4) {
      uint32_t w = 0;
      for (size_t j = 0; j < 4 && b + j < ns.size(); ++j) w |= (uint32_t)(uint8_t)ns[b + j] << (8 * j);
      out.qf_nbytes.push_back(w);
    }
  }
  // entries grouped by bucket, in needle order within one (a stable counting sort)
  out.qf_head.assign(kQfWords + 1, 0u);
  for (auto& be : bent) out.qf_head[be.first + 1]++;
  for (uint32_t b = 0; b < kQfWords; ++b) out.qf_head[b + 1] += out.qf_head[b];
  out.qf_ent.assign((size_t)bent.size() * 4, 0u);
  std::vector<uint32_t> fill(out.qf_head.begin(), out.qf_head.end() - 1);
  for (auto& be : bent) {
    const uint32_t v = be.second, i = v >> 8;
    uint32_t* en = &out.qf_ent[(size_t)fill[be.first]++ * 4];
    en[0] = noff[i];
    en[1] = (uint32_t)out.qf_needle[i].size() | (v & 0xFFu) << 16 | out.qf_nflags[i] |
            (out.qf_nshort[i] ? kQfAnchored : 0u);
    en[2] = out.qf_nrx[i];
    {  // the pre-check (round 6): the needle's four bytes at its sampled offset k, which k_verify
       // compares with the data's sample dword already in a register (bytes past the needle: 0)
      const auto& nd = out.qf_needle[i];
      const uint32_t k = v & 0xFFu;
      uint32_t w = 0;
      for (uint32_t j = 0; j < 4 && k + j < nd.size(); ++j) w |= (uint32_t)(uint8_t)nd[k + j] << (8 * j);
      en[3] = w;
    }
  }
}

}  // namespace

void stats_finish(DataStats& st) {
  st.marg.assign(256, 0.0);
  st.inv_marg.assign(256, 0.0);
  st.pair_tot = 0;
  st.inv_tot = 0;
  if (st.pair.size() >= 65536) {
    for (uint32_t x = 0; x < 65536; ++x) st.marg[x & 0xFFu] += st.pair[x];
    for (double m : st.marg) st.pair_tot += m;
    if (st.pair_tot > 0) {
      st.inv_tot = 1.0 / st.pair_tot;
      for (int c = 0; c < 256; ++c) st.inv_marg[c] = st.pair_tot / (st.marg[c] + 128.0);
    }
  }
}

double gram_share(const DataStats& st, uint32_t g, uint32_t q) {
  if (st.pair.size() < 65536 || st.inv_marg.size() != 256 || st.pair_tot <= 0) return 1.0;
  // P(b0 b1) * prod P(b_i b_i+1) / P(b_i): pair counts + 1/2, marginals (+ 128) from the pairs
  const double it = st.inv_tot;
  double p = (st.pair[g & 0xFFFFu] + 0.5) * it;
  for (uint32_t i = 1; i + 1 < q; ++i) {
    const uint32_t a = (g >> (8 * i)) & 0xFFu, ab = (g >> (8 * i)) & 0xFFFFu;
    p *= (st.pair[ab] + 0.5) * it * st.inv_marg[a];
  }
  return p;
}

void data_stats(const uint8_t* p, size_t n, uint32_t fold, DataStats& st) {
  st.pair.assign(65536, 0u);
  st.bytes.assign(256, 0u);
  st.nbytes = 0;
  for (size_t i = 0; i + 4 <= n; ++i) {
    st.bytes[p[i]]++;
    st.nbytes++;
    if (i % 4) continue;  // the 2-grams at even positions (k_gramhist: two per dword), counted twice
    uint32_t g = 0;
    for (int b = 0; b < 4; ++b) g |= (uint32_t)p[i + b] << (8 * b);
    g |= fold;
    st.pair[g & 0xFFFFu] += 2;
    st.pair[g >> 16] += 2;
  }
  stats_finish(st);
}

PrefilterHits prefilter_hits(const CompiledSet& cs, const uint8_t* s, size_t n) {
  PrefilterHits r;
  const uint32_t S = cs.qf_stride, w24 = cs.qf_q == 4 ? 24u : 0u;
  for (size_t p = 0; p < n; ++p) {
    uint32_t g = 0;
    for (uint32_t b = 0; b < 4; ++b) g |= (uint32_t)(p + b < n ? s[p + b] : 0) << (8 * b);
    bool hit = false;
    if (qf_sampled(p, S)) {
      ++r.probes;
      const uint32_t gq = (g | cs.qf_fold) & cs.qf_mask;
      hit = qf_pass(cs.qf_bitmap.data(), gq, w24, cs.qf_k);
      r.bitmap_hits += hit;
      if (cs.qf_k == kQfTwoLevel) r.pair_pass += (cs.qf_bitmap[qf_pair_word(gq & 0xFFFFu)] >> (gq & 31u)) & 1u;
    }
    if (!hit && cs.qf_anc_on && ((uint32_t)s[p] | (cs.qf_anc_fold & 0xFFu)) == cs.qf_anc_byte) {
      for (size_t j = 0; j + 1 < cs.qf_anc_pre.size() && !hit; j += 2)
        hit = ((g | cs.qf_fold) & cs.qf_anc_pre[j + 1]) == cs.qf_anc_pre[j];
      r.anchor_hits += hit;
    }
    if (!hit) continue;
    const uint32_t b = qf_bucket((g | cs.qf_fold) & cs.qf_mask, w24, cs.qf_k);
    for (uint32_t e = cs.qf_head[b]; e < cs.qf_head[b + 1]; ++e) {
      const uint32_t* E = cs.qf_ent.data() + 4 * (size_t)e;
      const uint32_t m = E[1] & 0xFFFFu, k = (E[1] >> 16) & 0xFFu;
      const int64_t x = (int64_t)p - (int64_t)k;
      if (x < 0 || (uint64_t)x + m > n) continue;
      const uint8_t* nb = reinterpret_cast<const uint8_t*>(cs.qf_nbytes.data() + E[0]);
      const uint8_t lm = (E[1] & kQfLoose) ? 0x20 : 0;
      bool eq = true;
      for (uint32_t j = 0; j < m && eq; ++j) eq = (uint8_t)(s[x + j] | lm) == nb[j];
      r.verified += eq;
    }
  }
  return r;
}

bool nfa_window(const CompiledSet& cs, uint32_t r, const uint8_t* s, size_t n, size_t x) {
  // matches holding the factor occurrence at x start in [x - pre, x]; past x no new start
  // is entered and the run ends when the automaton dies
  const uint32_t pre = cs.rx_pre.empty() ? kRxPreUnbounded : cs.rx_pre[r];
  const size_t ws = (pre == kRxPreUnbounded || (size_t)pre >= x) ? 0 : x - pre;
  const uint64_t first = cs.rx_first[r];
  uint64_t d = ws == 0 ? cs.rx_init0[r] : first;
  for (size_t i = ws; i < n; ++i) {
    const uint64_t c = d & cs.rx_b[(size_t)r * cs.rx_classes + cs.rx_class[s[i]]];
    if (c & cs.rx_last[r]) return true;
    uint64_t nd = i + 1 <= x ? first : 0;
    for (uint64_t m = c; m; m &= m - 1) nd |= cs.rx_follow[(size_t)r * 64 + __builtin_ctzll(m)];
    d = nd;
    if (!d) return false;
  }
  return (d & cs.rx_end[r]) != 0;
}

bool prefilter_match(const CompiledSet& cs, const uint8_t* s, size_t n, uint32_t phase) {
  // Any window of S consecutive positions holds a sample, and every needle's chosen
  // window is q + S - 1 long, so each occurrence spans one sample with its gram inside
  // the window (the scan's tiles own their samples; the occurrence may start before).
  // Anchored short needles: every position holding the anchor byte whose dword passes a
  // pre-check is a hit too (the scan's anchor test), walked through the same buckets.
  const uint32_t S = cs.qf_stride;
  for (size_t p = 0; p < n; ++p) {
    uint32_t g = 0;
    for (uint32_t b = 0; b < 4; ++b) g |= (uint32_t)(p + b < n ? s[p + b] : 0) << (8 * b);
    bool hit = false;
    if (qf_sampled(p + 16 - phase % 16, S)) {
      const uint32_t gq = (g | cs.qf_fold) & cs.qf_mask;
      hit = qf_pass(cs.qf_bitmap.data(), gq, cs.qf_q == 4 ? 24u : 0u, cs.qf_k);
    }
    if (!hit && cs.qf_anc_on && ((uint32_t)s[p] | (cs.qf_anc_fold & 0xFFu)) == cs.qf_anc_byte)
      for (size_t j = 0; j + 1 < cs.qf_anc_pre.size() && !hit; j += 2)
        hit = ((g | cs.qf_fold) & cs.qf_anc_pre[j + 1]) == cs.qf_anc_pre[j];
    if (!hit) continue;
    g = (g | cs.qf_fold) & cs.qf_mask;
    const uint32_t b = qf_bucket(g, cs.qf_q == 4 ? 24u : 0u, cs.qf_k);
    for (uint32_t e = cs.qf_head[b]; e < cs.qf_head[b + 1]; ++e) {
      const uint32_t* E = cs.qf_ent.data() + 4 * (size_t)e;
      const uint32_t m = E[1] & 0xFFFFu, k = (E[1] >> 16) & 0xFFu;
      const int64_t x = (int64_t)p - (int64_t)k;
      if (x < 0 || (uint64_t)x + m > n) continue;
      const uint8_t* nb = reinterpret_cast<const uint8_t*>(cs.qf_nbytes.data() + E[0]);
      const uint8_t lm = (E[1] & kQfLoose) ? 0x20 : 0;
      bool eq = true;
      for (uint32_t j = 0; j < m && eq; ++j) eq = (uint8_t)(s[x + j] | lm) == nb[j];
      if (!eq) continue;
      if (!(E[1] & kQfRegex)) return true;  // literal: final
      // regex factor occurrence: the NFA over its window (k_nfa on the GPU)
      if ((cs.rx_flags[E[2]] & 1u) || nfa_window(cs, E[2], s, n, (size_t)x)) return true;
    }
  }
  return false;
}

}  // namespace klf
