// klf_ts.hpp — Go time.Parse(time.RFC3339Nano) for the kubelet timestamp prefix,
// shared by the HIP kernels and the host (klf_parse_rfc3339nano).
//
// Restates Go 1.22 src/time/format.go (parse: stdLongYear, stdZeroMonth, stdZeroDay,
// stdHour, stdZeroMinute, stdZeroSecond, stdFracSecond9, stdISO8601ColonTZ; getnum;
// parseNanoseconds; the daysIn validation) for the one layout kubelet uses,
// "2006-01-02T15:04:05.999999999Z07:00" (k8s v1.30.3 logs.go timeFormatIn), as frozen
// in SPEC.md S2.  The line-level rule of parseCRILog (split at the first ' ') is
// klf_parse_line_prefix below.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KLF_HD __host__ __device__ __forceinline__
#else
#define KLF_HD inline
#endif

namespace klf {

KLF_HD bool is_digit(int c) { return c >= '0' && c <= '9'; }

KLF_HD int days_in_month(int m, int64_t y) {
  if (m == 2) return ((y % 4 == 0) && (y % 100 != 0 || y % 400 == 0)) ? 29 : 28;
  return (m == 4 || m == 6 || m == 9 || m == 11) ? 30 : 31;
}

// Days since 1970-01-01 of a proleptic-Gregorian civil date (y in 0..9999 here).
KLF_HD int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t mp = (m + 9) % 12;
  const int64_t doy = (153 * mp + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

struct TsResult {
  int64_t sec;   // Unix seconds of the instant
  int32_t nsec;  // [0, 1e9)
  uint32_t len;  // bytes consumed by the timestamp
};

// Parses a timestamp at the start of a byte source.  `get(i)` returns byte i, or -1
// past the end.  Returns true with r filled when bytes [0, r.len) are a complete
// RFC3339Nano value per Go; the caller decides what must follow (parseCRILog: ' ').
// Go's parse is deterministic and greedy for this layout (getnum takes two digits
// when present; the fraction takes every digit), so "longest valid prefix followed by
// the delimiter" is exactly "time.Parse(line[:first_space]) == nil".
template <class Get>
KLF_HD bool parse_rfc3339nano(Get get, TsResult& r) {
  int c0 = get(0), c1 = get(1), c2 = get(2), c3 = get(3);
  // stdLongYear: 4 bytes, first a digit, atoi of all 4 (no sign possible after that)
  if (!is_digit(c0) || !is_digit(c1) || !is_digit(c2) || !is_digit(c3)) return false;
  const int64_t year = (c0 - '0') * 1000 + (c1 - '0') * 100 + (c2 - '0') * 10 + (c3 - '0');
  if (get(4) != '-') return false;
  // stdZeroMonth: exactly two digits, 1..12
  int a = get(5), b = get(6);
  if (!is_digit(a) || !is_digit(b)) return false;
  const int month = (a - '0') * 10 + (b - '0');
  if (month < 1 || month > 12) return false;
  if (get(7) != '-') return false;
  // stdZeroDay: two digits; range validated after the loop (daysIn)
  a = get(8); b = get(9);
  if (!is_digit(a) || !is_digit(b)) return false;
  const int day = (a - '0') * 10 + (b - '0');
  if (get(10) != 'T') return false;
  // stdHour: getnum(value, false) — ONE or two digits, < 24
  uint32_t i = 11;
  a = get(i);
  if (!is_digit(a)) return false;
  int hour = a - '0';
  ++i;
  b = get(i);
  if (is_digit(b)) { hour = hour * 10 + (b - '0'); ++i; }
  if (hour >= 24) return false;
  if (get(i) != ':') return false;
  ++i;
  // stdZeroMinute: two digits, < 60
  a = get(i); b = get(i + 1);
  if (!is_digit(a) || !is_digit(b)) return false;
  const int minute = (a - '0') * 10 + (b - '0');
  if (minute >= 60) return false;
  i += 2;
  if (get(i) != ':') return false;
  ++i;
  // stdZeroSecond: two digits, < 60
  a = get(i); b = get(i + 1);
  if (!is_digit(a) || !is_digit(b)) return false;
  const int second = (a - '0') * 10 + (b - '0');
  if (second >= 60) return false;
  i += 2;
  // stdFracSecond9: optional; '.' or ',' then >= 1 digit; all digits consumed, first 9 kept
  int32_t nsec = 0;
  a = get(i);
  if ((a == '.' || a == ',') && is_digit(get(i + 1))) {
    ++i;
    int nd = 0;
    for (;;) {
      const int d = get(i);
      if (!is_digit(d)) break;
      if (nd < 9) { nsec = nsec * 10 + (d - '0'); ++nd; }
      ++i;
    }
    for (; nd < 9; ++nd) nsec *= 10;
  }
  // stdISO8601ColonTZ: 'Z' or [+-]hh:mm with hh <= 24, mm <= 60
  int64_t off = 0;
  a = get(i);
  if (a == 'Z') {
    ++i;
  } else {
    const int s = a, h1 = get(i + 1), h2 = get(i + 2), col = get(i + 3), m1 = get(i + 4),
              m2 = get(i + 5);
    if (m2 < 0) return false;  // len(value) < 6
    if (col != ':') return false;
    if (!is_digit(h1) || !is_digit(h2) || !is_digit(m1) || !is_digit(m2)) return false;
    const int hh = (h1 - '0') * 10 + (h2 - '0');
    const int mm = (m1 - '0') * 10 + (m2 - '0');
    if (hh > 24 || mm > 60) return false;
    off = (int64_t)(hh * 60 + mm) * 60;
    if (s == '-') off = -off;
    else if (s != '+') return false;
    i += 6;
  }
  if (day < 1 || day > days_in_month(month, year)) return false;
  r.sec = days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + second - off;
  r.nsec = nsec;
  r.len = i;
  return true;
}

// parseCRILog's split + parse for a line starting at byte 0: true iff the bytes up to
// the line's first ' ' are a valid RFC3339Nano value.  plen = index of that space + 1,
// i.e. where the content starts.
template <class Get>
KLF_HD bool parse_line_prefix(Get get, TsResult& r, uint32_t& plen) {
  if (!parse_rfc3339nano(get, r)) return false;
  if (get(r.len) != ' ') return false;  // extra text before the delimiter, or no delimiter
  plen = r.len + 1;
  return true;
}

KLF_HD bool time_before(int64_t s1, int32_t n1, int64_t s2, int32_t n2) {
  return s1 < s2 || (s1 == s2 && n1 < n2);
}

}  // namespace klf
