/*
 * klogs_host.h — C ABI of the host mirror of klogs' cmd/root.go (libklogs_host.so).
 *
 * The reference host is Go (/root/reference/cmd/root.go) and this image has no Go
 * toolchain, so the host logic that sits above libklf (include/klf.h) is restated in C++
 * with these entry points.  Each one names the reference code it mirrors; the cgo glue in
 * INTEGRATION.md is the Go-side equivalent.  No GPU is needed for anything here except
 * klh_run (which drives libklf).
 */
#ifndef KLOGS_HOST_H
#define KLOGS_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "klf.h"

#ifdef __cplusplus
extern "C" {
#endif

#define KLH_OK 0
#define KLH_EPARSE -101  /* a flag value does not parse (the reference panics)            */
#define KLH_EIO -102     /* file-system error (the reference panics)                       */
#define KLH_EINVAL -103  /* bad argument                                                   */

/* Go time.ParseDuration(s) (Go 1.22 src/time/format.go), restated: nanoseconds.
 * Returns KLH_EPARSE with the Go error text in err for an invalid duration. */
int klh_parse_duration(const char* s, int64_t* ns, char* err, size_t err_cap);

/* getLopOpts (cmd/root.go:201-221) split into what the engine needs.
 *   since_flag: the -s value, NULL or "" = unset;  tail_flag: the -t value (-1 = all).
 *   now: the instant the request is made (kubelet takes its own now, logs.go NewLogOptions).
 * On success fills *filter (since = now - int64(d.Seconds()) s, or Go's zero time when
 * unset; tail) and *rejected = 1 when the API server would refuse the request
 * (ValidatePodLogOptions: SinceSeconds < 1 or TailLines < 0 once sent), which in klogs
 * leaves every stream's file empty (cmd/root.go:326-328).  KLH_EPARSE when the duration
 * does not parse (cmd/root.go:207-209 panics). */
int klh_lop_opts(const char* since_flag, int64_t tail_flag, klf_time now, klf_filter* filter, int* rejected,
                 char* err, size_t err_cap);

/* One pod of the selection: name plus its init containers and containers, in spec order. */
typedef struct klh_pod {
  const char* name;
  uint32_t n_init;
  const char* const* init;
  uint32_t n_containers;
  const char* const* containers;
} klh_pod;

/* One stream of the table, in getPodLogs order (cmd/root.go:224-277). */
typedef struct klh_stream {
  uint32_t pod;        /* index into the pods array                     */
  uint32_t container;  /* index into pods[pod].init or .containers      */
  uint32_t is_init;    /* 1 = init container (only with -i)             */
  uint32_t _reserved;
} klh_stream;

/* The ordered stream set: for each pod, init containers first when init_flag (-i,
 * :240-251), then containers (:253-262).  A (pod name, container name) pair already in the
 * table is skipped (several -l selectors can return the same pod, :458-460; klogs would
 * race two goroutines on one file).  Writes min(n, cap) entries, *n_out = n. */
int klh_stream_table(const klh_pod* pods, uint32_t n_pods, int init_flag, klh_stream* out, uint32_t cap,
                     uint32_t* n_out);

/* "<pod>__<container>.log" (createLogFile :341-356, fileNameSeparator :52).  Returns the
 * length; writes a NUL-terminated prefix into buf when cap > 0. */
size_t klh_log_file_name(const char* pod, const char* container, char* buf, size_t cap);

/* createLogFile: MkdirAll(logpath, 0755) + os.Create (truncate) of the stream's file.
 * Writes the path into path_out. */
int klh_create_log_file(const char* logpath, const char* pod, const char* container, char* path_out, size_t cap);

/* convertBytes (:423-434): "0 B" (red when color), "%d B", "%d KB", "%d MB", floored. */
size_t klh_convert_bytes(int64_t bytes, int color, char* buf, size_t cap);

/* The default log path "logs/" + now.Format("2006-01-02T15-04") (:47), in local time. */
size_t klh_default_log_path(int64_t unix_sec, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* KLOGS_HOST_H */
