// klogs_host.cpp — the host side of klogs' cmd/root.go above libklf, restated in C++
// (include/klogs_host.h).  Pure host code: flags -> engine options, stream table, output
// file layout, size report.  Semantics cite /root/reference/cmd/root.go line by line.
#include "../../include/klogs_host.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <utility>

namespace {

void put_err(char* err, size_t cap, const std::string& m) {
  if (!err || !cap) return;
  std::snprintf(err, cap, "%s", m.c_str());
}

size_t put_str(const std::string& s, char* buf, size_t cap) {
  if (buf && cap) std::snprintf(buf, cap, "%s", s.c_str());
  return s.size();
}

std::string go_quote(const std::string& s) { return "\"" + s + "\""; }

constexpr uint64_t kMaxI64Plus1 = 1ull << 63;

// time.leadingInt: [0-9]* with overflow detection
bool leading_int(const std::string& s, size_t& i, uint64_t& x) {
  x = 0;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') break;
    if (x > kMaxI64Plus1 / 10) return false;
    x = x * 10 + (uint64_t)(c - '0');
    if (x > kMaxI64Plus1) return false;
  }
  return true;
}

// time.leadingFraction: digits after '.', overflow -> stop accumulating (not an error)
void leading_fraction(const std::string& s, size_t& i, uint64_t& x, double& scale) {
  x = 0;
  scale = 1;
  bool overflow = false;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') break;
    if (overflow) continue;
    if (x > (kMaxI64Plus1 - 1) / 10) { overflow = true; continue; }
    const uint64_t y = x * 10 + (uint64_t)(c - '0');
    if (y > kMaxI64Plus1) { overflow = true; continue; }
    x = y;
    scale *= 10;
  }
}

bool unit_ns(const std::string& u, uint64_t& ns) {
  // time.unitMap; "µs" is U+00B5, "μs" is U+03BC (UTF-8 bytes)
  if (u == "ns") ns = 1;
  else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") ns = 1000;
  else if (u == "ms") ns = 1000000;
  else if (u == "s") ns = 1000000000ull;
  else if (u == "m") ns = 60ull * 1000000000ull;
  else if (u == "h") ns = 3600ull * 1000000000ull;
  else return false;
  return true;
}

}  // namespace

extern "C" int klh_parse_duration(const char* cs, int64_t* out, char* err, size_t err_cap) {
  if (!cs || !out) return KLH_EINVAL;
  const std::string orig(cs);
  std::string s = orig;
  const std::string bad = "time: invalid duration " + go_quote(orig);
  uint64_t d = 0;
  bool neg = false;
  size_t i = 0;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    i = 1;
  }
  if (s.substr(i) == "0") { *out = 0; return KLH_OK; }
  if (i == s.size()) { put_err(err, err_cap, bad); return KLH_EPARSE; }
  while (i < s.size()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    if (!(s[i] == '.' || (s[i] >= '0' && s[i] <= '9'))) { put_err(err, err_cap, bad); return KLH_EPARSE; }
    const size_t p0 = i;
    if (!leading_int(s, i, v)) { put_err(err, err_cap, bad); return KLH_EPARSE; }
    const bool pre = i != p0;
    bool post = false;
    if (i < s.size() && s[i] == '.') {
      ++i;
      const size_t p1 = i;
      leading_fraction(s, i, f, scale);
      post = i != p1;
    }
    if (!pre && !post) { put_err(err, err_cap, bad); return KLH_EPARSE; }
    size_t j = i;
    for (; j < s.size(); ++j) {
      const char c = s[j];
      if (c == '.' || (c >= '0' && c <= '9')) break;
    }
    if (j == i) { put_err(err, err_cap, "time: missing unit in duration " + go_quote(orig)); return KLH_EPARSE; }
    const std::string u = s.substr(i, j - i);
    i = j;
    uint64_t unit;
    if (!unit_ns(u, unit)) {
      put_err(err, err_cap, "time: unknown unit " + go_quote(u) + " in duration " + go_quote(orig));
      return KLH_EPARSE;
    }
    if (v > kMaxI64Plus1 / unit) { put_err(err, err_cap, bad); return KLH_EPARSE; }
    v *= unit;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)unit / scale));
      if (v > kMaxI64Plus1) { put_err(err, err_cap, bad); return KLH_EPARSE; }
    }
    d += v;
    if (d > kMaxI64Plus1) { put_err(err, err_cap, bad); return KLH_EPARSE; }
  }
  if (neg) {
    *out = d == kMaxI64Plus1 ? INT64_MIN : -(int64_t)d;
    return KLH_OK;
  }
  if (d > kMaxI64Plus1 - 1) { put_err(err, err_cap, bad); return KLH_EPARSE; }
  *out = (int64_t)d;
  return KLH_OK;
}

extern "C" int klh_lop_opts(const char* since_flag, int64_t tail_flag, klf_time now, klf_filter* f, int* rejected,
                            char* err, size_t err_cap) {
  if (!f || !rejected) return KLH_EINVAL;
  std::memset(f, 0, sizeof(*f));
  *rejected = 0;
  // Since (:204-212): int64(duration.Seconds()); Seconds() = float64(d/1s) + float64(d%1s)/1e9
  f->since.sec = KLF_GO_ZERO_TIME_SEC;  // kubelet's default since (logs.go NewLogOptions)
  f->since.nsec = 0;
  if (since_flag && since_flag[0]) {
    int64_t d;
    const int rc = klh_parse_duration(since_flag, &d, err, err_cap);
    if (rc != KLH_OK) return rc;  // the reference panics here, before any file exists
    const int64_t sec = d / 1000000000LL, nsec = d % 1000000000LL;
    const double secs = (double)sec + (double)nsec / 1e9;
    const int64_t since_s = (int64_t)secs;  // truncation toward zero
    if (since_s < 1) {
      *rejected = 1;  // ValidatePodLogOptions: sinceSeconds must be greater than 0
    } else {
      f->since.sec = now.sec - since_s;
      f->since.nsec = now.nsec;
    }
  }
  // Tail (:214-216): only sent when != -1; the server rejects a negative TailLines
  f->tail = tail_flag;
  if (tail_flag < -1) *rejected = 1;
  return KLH_OK;
}

extern "C" int klh_stream_table(const klh_pod* pods, uint32_t n_pods, int init_flag, klh_stream* out, uint32_t cap,
                                uint32_t* n_out) {
  if ((n_pods && !pods) || !n_out || (cap && !out)) return KLH_EINVAL;
  std::set<std::pair<std::string, std::string>> seen;
  uint32_t n = 0;
  auto add = [&](uint32_t p, uint32_t c, const char* cname, uint32_t is_init) {
    if (!seen.emplace(pods[p].name ? pods[p].name : "", cname ? cname : "").second) return;
    if (n < cap) out[n] = klh_stream{p, c, is_init, 0};
    ++n;
  };
  for (uint32_t p = 0; p < n_pods; ++p) {
    if (init_flag)
      for (uint32_t c = 0; c < pods[p].n_init; ++c) add(p, c, pods[p].init[c], 1);
    for (uint32_t c = 0; c < pods[p].n_containers; ++c) add(p, c, pods[p].containers[c], 0);
  }
  *n_out = n;
  return KLH_OK;
}

extern "C" size_t klh_log_file_name(const char* pod, const char* container, char* buf, size_t cap) {
  const std::string s = std::string(pod ? pod : "") + "__" + (container ? container : "") + ".log";
  return put_str(s, buf, cap);
}

static int mkdir_all(const std::string& path) {
  // os.MkdirAll(path, 0755)
  if (path.empty()) return 0;
  struct stat st;
  if (stat(path.c_str(), &st) == 0) return S_ISDIR(st.st_mode) ? 0 : ENOTDIR;
  const size_t slash = path.find_last_of('/');
  if (slash != std::string::npos && slash > 0) {
    const int rc = mkdir_all(path.substr(0, slash));
    if (rc) return rc;
  }
  if (mkdir(path.c_str(), 0755) != 0 && errno != EEXIST) return errno;
  return 0;
}

extern "C" int klh_create_log_file(const char* logpath, const char* pod, const char* container, char* path_out,
                                   size_t cap) {
  if (!logpath || !pod || !container) return KLH_EINVAL;
  if (mkdir_all(logpath) != 0) return KLH_EIO;
  char name[4096];
  klh_log_file_name(pod, container, name, sizeof(name));
  std::string path = std::string(logpath);
  if (!path.empty() && path.back() != '/') path += '/';
  path += name;  // filepath.Join
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);  // os.Create
  if (fd < 0) return KLH_EIO;
  close(fd);
  put_str(path, path_out, cap);
  return KLH_OK;
}

extern "C" size_t klh_convert_bytes(int64_t bytes, int color, char* buf, size_t cap) {
  char tmp[64];
  if (bytes == 0) return put_str(color ? "\x1b[31m0 B\x1b[0m" : "0 B", buf, cap);  // pterm.Red
  if (bytes < 1024) std::snprintf(tmp, sizeof(tmp), "%lld B", (long long)bytes);
  else if (bytes < 1024 * 1024) std::snprintf(tmp, sizeof(tmp), "%lld KB", (long long)(bytes / 1024));
  else std::snprintf(tmp, sizeof(tmp), "%lld MB", (long long)(bytes / 1024 / 1024));
  return put_str(tmp, buf, cap);
}

extern "C" size_t klh_default_log_path(int64_t unix_sec, char* buf, size_t cap) {
  const time_t t = (time_t)unix_sec;
  struct tm lt;
  localtime_r(&t, &lt);
  char tmp[64];
  strftime(tmp, sizeof(tmp), "logs/%Y-%m-%dT%H-%M", &lt);  // Go layout 2006-01-02T15-04
  return put_str(tmp, buf, cap);
}
