// klogs-filter — the klogs batch path (rootCmd.Run, /root/reference/cmd/root.go:442-474)
// over captured log bodies, with the filter on the GPU through libklf.
//
//   klogs-filter [-p logpath] [-s since] [-t tail] [-i] [--grep LIT]... [--match RE]...
//                [--now UNIX_SEC[.NSEC]] [--device N] [--no-color] MANIFEST
//
// MANIFEST has one line per container of the pod selection, in pod-spec order:
//   <pod> TAB <init|container> TAB <container> TAB <path of the captured body | ->
// A body is what GetLogs(...).Stream() returns for Timestamps=true without
// SinceSeconds/TailLines; "-" or an unreadable path is a failed Stream() call (:326-328:
// error line, the file stays empty).  Cluster discovery (:449-461) is out of scope: the
// manifest stands for its result.
#include <fcntl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/klf.h"
#include "../../include/klogs_host.h"

namespace {

struct PodEnt {
  std::string name;
  std::vector<std::string> init, containers;
  std::vector<std::string> init_body, cont_body;
};

[[noreturn]] void panic_exit(const std::string& m) {
  std::fprintf(stderr, "panic: %s\n", m.c_str());
  std::exit(2);
}

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  out.clear();
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.insert(out.end(), buf, buf + n);
  const bool ok = !std::ferror(f);
  std::fclose(f);
  return ok;
}

void usage() {
  std::fprintf(stderr,
               "usage: klogs-filter [-p logpath] [-s since] [-t tail] [-i] [--grep LIT]... [--match RE]...\n"
               "                    [--now UNIX_SEC[.NSEC]] [--device N] [--no-color] MANIFEST\n");
  std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
  std::string logpath, since, manifest;
  int64_t tail = -1;
  bool init = false, color = true;
  int device = 0;
  klf_time now{(int64_t)time(nullptr), 0, 0};
  std::vector<std::string> greps, matches;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) usage();
      return argv[++i];
    };
    if (a == "-p" || a == "--logpath") logpath = val();
    else if (a == "-s" || a == "--since") since = val();
    else if (a == "-t" || a == "--tail") tail = std::strtoll(val().c_str(), nullptr, 10);
    else if (a == "-i" || a == "--init") init = true;
    else if (a == "--grep") greps.push_back(val());
    else if (a == "--match") matches.push_back(val());
    else if (a == "--device") device = std::atoi(val().c_str());
    else if (a == "--no-color") color = false;
    else if (a == "--now") {
      const std::string v = val();
      const size_t dot = v.find('.');
      now.sec = std::strtoll(v.substr(0, dot).c_str(), nullptr, 10);
      if (dot != std::string::npos) {
        std::string frac = v.substr(dot + 1);
        frac.resize(9, '0');
        now.nsec = (int32_t)std::strtol(frac.c_str(), nullptr, 10);
      }
    } else if (!a.empty() && a[0] == '-') usage();
    else manifest = a;
  }
  if (manifest.empty()) usage();
  if (logpath.empty()) {  // defaultLogPath (:47)
    char buf[128];
    klh_default_log_path(now.sec, buf, sizeof(buf));
    logpath = buf;
  }

  // getLopOpts (:201-221)
  klf_filter filter;
  int rejected = 0;
  char err[512] = {0};
  if (klh_lop_opts(since.c_str(), tail, now, &filter, &rejected, err, sizeof(err)) != KLH_OK) panic_exit(err);
  filter.flags |= KLF_FILTER_NO_TIMING;  // (the CLI reads no device timing)

  // the pod selection, grouped by pod in first-appearance order
  std::vector<PodEnt> pods;
  {
    FILE* f = std::fopen(manifest.c_str(), "r");
    if (!f) panic_exit("open " + manifest + ": no such file");
    char line[8192];
    while (std::fgets(line, sizeof(line), f)) {
      std::string l(line);
      while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
      if (l.empty() || l[0] == '#') continue;
      std::vector<std::string> col;
      size_t p = 0;
      for (;;) {
        const size_t q = l.find('\t', p);
        col.push_back(l.substr(p, q == std::string::npos ? std::string::npos : q - p));
        if (q == std::string::npos) break;
        p = q + 1;
      }
      if (col.size() != 4) panic_exit("manifest line needs 4 tab-separated fields: " + l);
      PodEnt* pe = nullptr;
      for (auto& x : pods)
        if (x.name == col[0]) pe = &x;
      if (!pe) {
        pods.push_back(PodEnt{col[0], {}, {}, {}, {}});
        pe = &pods.back();
      }
      if (col[1] == "init") { pe->init.push_back(col[2]); pe->init_body.push_back(col[3]); }
      else { pe->containers.push_back(col[2]); pe->cont_body.push_back(col[3]); }
    }
    std::fclose(f);
  }
  std::vector<std::vector<const char*>> ip(pods.size()), cp(pods.size());
  std::vector<klh_pod> kp(pods.size());
  for (size_t i = 0; i < pods.size(); ++i) {
    for (auto& s : pods[i].init) ip[i].push_back(s.c_str());
    for (auto& s : pods[i].containers) cp[i].push_back(s.c_str());
    kp[i] = klh_pod{pods[i].name.c_str(), (uint32_t)ip[i].size(), ip[i].data(), (uint32_t)cp[i].size(), cp[i].data()};
  }
  // getPodLogs (:224-277): stream table + createLogFile per stream
  uint32_t n = 0;
  klh_stream_table(kp.data(), (uint32_t)kp.size(), init ? 1 : 0, nullptr, 0, &n);
  std::vector<klh_stream> table(n);
  klh_stream_table(kp.data(), (uint32_t)kp.size(), init ? 1 : 0, table.data(), n, &n);
  std::vector<std::string> files(n), cname(n), body(n);
  for (uint32_t i = 0; i < n; ++i) {
    const PodEnt& pe = pods[table[i].pod];
    cname[i] = table[i].is_init ? pe.init[table[i].container] : pe.containers[table[i].container];
    body[i] = table[i].is_init ? pe.init_body[table[i].container] : pe.cont_body[table[i].container];
    char path[8192];
    if (klh_create_log_file(logpath.c_str(), pe.name.c_str(), cname[i].c_str(), path, sizeof(path)) != KLH_OK)
      panic_exit("create log file for " + pe.name + "/" + cname[i]);
    files[i] = path;
  }
  std::fprintf(stderr, "INFO  Found %zu Pod(s) %u Container(s)\n", pods.size(), n);

  if (n > 0 && rejected) {  // the API server refuses every request: error lines, empty files
    for (uint32_t i = 0; i < n; ++i)
      std::fprintf(stderr, "ERROR Error getting logs for container %s\n%s\n", cname[i].c_str(),
                   "the server rejected our request (invalid PodLogOptions)");
  } else if (n > 0) {
    std::vector<klf_pattern> pats;
    for (auto& g : greps) pats.push_back(klf_pattern{(const uint8_t*)g.data(), (uint32_t)g.size(), KLF_PAT_LITERAL});
    for (auto& m : matches) pats.push_back(klf_pattern{(const uint8_t*)m.data(), (uint32_t)m.size(), KLF_PAT_REGEX});
    klf_config cfg{};
    cfg.device = device;
    cfg.n_patterns = (uint32_t)pats.size();
    cfg.patterns = pats.empty() ? nullptr : pats.data();
    klf_engine* e = nullptr;
    int rc = klf_open(&cfg, &e);
    if (rc != KLF_OK) {
      std::string m = klf_strerror(rc);
      if (e) { m += std::string(": ") + klf_last_error(e); klf_close(e); }
      if (rc == KLF_EPATTERN || rc == KLF_ETOOBIG) {
        std::fprintf(stderr, "ERROR %s\n", m.c_str());
        return 1;
      }
      panic_exit(m);
    }
    if (klf_set_streams(e, n) != KLF_OK) panic_exit("klf_set_streams");
    std::vector<uint8_t> buf;
    for (uint32_t i = 0; i < n; ++i) {  // streamLog (:312-339): one body per stream
      if (body[i] == "-" || !read_file(body[i], buf)) {
        std::fprintf(stderr, "ERROR Error getting logs for container %s\n%s\n", cname[i].c_str(),
                     ("cannot read " + body[i]).c_str());
        continue;
      }
      if (!buf.empty() && klf_stage(e, i, buf.data(), buf.size()) != KLF_OK) panic_exit("klf_stage");
    }
    klf_result* r = nullptr;
    rc = klf_run(e, &filter, &r);
    if (rc != KLF_OK) panic_exit(std::string("klf_run: ") + klf_strerror(rc) + ": " + klf_last_error(e));
    // writeLogToDisk (:359-374): one klf_result_write over every stream's file (chunked,
    // double-buffered D2H from pinned memory), files closed afterwards
    std::vector<int> fds(n, -1);
    for (uint32_t i = 0; i < n; ++i) {
      fds[i] = ::open(files[i].c_str(), O_WRONLY | O_TRUNC);
      if (fds[i] < 0) panic_exit("open " + files[i]);
    }
    rc = klf_result_write(r, fds.data(), n, nullptr);
    if (rc != KLF_OK) panic_exit(std::string("klf_result_write: ") + klf_strerror(rc) + ": " + klf_last_error(e));
    for (uint32_t i = 0; i < n; ++i)
      if (::close(fds[i]) != 0) panic_exit("close " + files[i]);
    klf_result_free(r);
    klf_close(e);
  }

  // printLogSize (:279-309)
  if (n == 0) {
    std::fprintf(stdout, "ERROR No logs saved\n");
    return 0;
  }
  std::fprintf(stdout, "INFO  Logs saved to %s\n", logpath.c_str());
  std::fprintf(stdout, "Pod\tContainer\tSize\n");
  for (uint32_t i = 0; i < n; ++i) {
    struct stat st;
    if (stat(files[i].c_str(), &st) != 0) continue;
    char sz[64];
    klh_convert_bytes((int64_t)st.st_size, color ? 1 : 0, sz, sizeof(sz));
    std::fprintf(stdout, "%s\t%s\t%s\n", pods[table[i].pod].name.c_str(), cname[i].c_str(), sz);
  }
  return 0;
}
