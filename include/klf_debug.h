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
 * final, regex factor hits -> Glushkov NFA.  info (nullable) = {prefilter on, q, stride,
 * needles}; when the prefilter is off *match is the full matcher's answer. */
int klf_debug_prefilter(const klf_pattern* pats, uint32_t n, const uint8_t* content, size_t len,
                        uint32_t phase, int* match, uint32_t* info);

#ifdef __cplusplus
}
#endif
#endif /* KLF_DEBUG_H */
