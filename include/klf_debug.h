/*
 * klf_debug.h — test hooks of libklf.so (host only, no GPU).  Not part of the product
 * ABI that the Go host binds (include/klf.h): the CPU tests use them to run the compiled
 * pattern tables on the host against independent oracles.
 */
#ifndef KLF_DEBUG_H
#define KLF_DEBUG_H

#include "klf.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Compiles `pats` and reports the matcher mode: 0 none, 1 never, 2 all, 3 single
 * literal (fused scan), 4 general (AC + Glushkov).  err receives the compile message. */
int klf_debug_compile(const klf_pattern* pats, uint32_t n, uint32_t* mode, char* err, size_t err_cap);
/* Runs the compiled tables (the exact recurrences the GPU matcher runs) on one content. */
int klf_debug_match(const klf_pattern* pats, uint32_t n, const uint8_t* content, size_t len, int* match);
/* The prefiltered path of general sets on one content, as the scan runs it: q-gram
 * samples at positions = phase (mod stride), bitmap + bucket verification, literal hits
 * final, regex factor hits -> Glushkov NFA; anchored short needles at every position
 * holding the anchor byte.  info (nullable, 5 words) = {prefilter on, q, stride, needles,
 * 0x100 | anchor byte (0: no anchor)}; when the prefilter is off *match is the full
 * matcher's answer. */
int klf_debug_prefilter(const klf_pattern* pats, uint32_t n, const uint8_t* content, size_t len,
                        uint32_t phase, int* match, uint32_t* info);

/* The prefilter's layout chosen on the statistics of `sample` (the host twin of the first
 * batch's k_gramhist; slen 0: the compile-time layout), then its work over `data`:
 * out[9] = {stride, q, K, 0x100 | anchor byte (0: none), probes, bitmap hits, anchor hits,
 * verified needle occurrences, samples past the two-level probe's 2-gram stage}; layout
 * (cap bytes) gets the layout's description. */
int klf_debug_prefilter_hits(const klf_pattern* pats, uint32_t n, const uint8_t* sample, size_t slen,
                             const uint8_t* data, size_t dlen, uint64_t* out, char* layout, size_t cap);

/* The required factor set of one regex (SPEC.md S5) as the prefilter uses it: the
 * strings '\0'-separated into buf (cap bytes), *pre = bound on the distance from a match's
 * start to its first factor occurrence (0xFFFFFFFF: none), *loose = compared OR 0x20;
 * want = the shortest string length preferred (0 = the longest set).  *n = strings.
 * KLF_EINVAL when the regex has no factor. */
int klf_debug_factors(const uint8_t* pat, size_t len, uint32_t want, char* buf, size_t cap, uint32_t* n,
                      uint32_t* pre, uint32_t* loose);

/* The since cutoff as the scan's fast timestamp path compares it: out[6] = the 23 digits
 * of its canonical UTC prefix (YYYYMMDDhhmmss + 9 fraction digits) packed big-endian, a
 * '0' pad before the last digit; before 1970 the digits of 1970-01-01T00:00:00Z, from 2100
 * on all '9'. */
int klf_debug_since_digits(int64_t sec, int32_t nsec, uint32_t* out);

/* The clock a VALU-bound loop holds on `device` (needs a GPU): `reps` back-to-back
 * launches of a multiply-add loop over every CU, `iters` iterations each; per workgroup of
 * the last launch the shader-clock delta over the 100 MHz real-time delta.  mhz[3] =
 * {median, min, max} over the workgroups.  A yardstick of the board, not of a kernel. */
int klf_debug_clock(int device, uint32_t iters, uint32_t reps, double* mhz);

#ifdef __cplusplus
}
#endif
#endif /* KLF_DEBUG_H */
