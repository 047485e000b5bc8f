/*
 * approx_counter_amd_testing.h -- test-only entry point of libapprox_counter_amd.so.
 *
 * Not part of the drop-in boundary (include/approx_counter_amd.h): no product
 * caller sets these hooks, and the reference has no counterpart.  They let the
 * test suite drive failure and diagnostic paths of the early-launch stage
 * (ac_error_count_jobs, the replacement of errorCount, approx_counter.cpp:531-601)
 * that a well-behaved host never reaches.  Hooks are process-wide and apply to
 * calls made after the call that sets them; 0 clears them.
 */
#ifndef APPROX_COUNTER_AMD_TESTING_H
#define APPROX_COUNTER_AMD_TESTING_H

#include <stdint.h>

#include "approx_counter_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The last job of an early-launch call is never flagged complete: the kernel's
 * bounded waits run out (0.5 s without progress), it reports AC_DEVERR_STAGE, and
 * the synchronous call retries through the DMA path (ac_stage_mode() == 0 after). */
#define AC_TESTING_UNFLAG_LAST 1u
/* Every job is sent ahead of the staged launch by the copy kernel, so the staged
 * kernel runs on resident input (a measurement of its own cost). */
#define AC_TESTING_ALL_AHEAD 2u
/* The publishing thread sleeps 60 ms after each of a call's first 12 progress
 * records: a host slower in total than the kernel's 0.5 s timeout, whose every
 * gap is not (the waits restart their clock on progress). */
#define AC_TESTING_SLOW_HOST 4u
/* Device packing (ABI 7) for every eligible job, whatever the call's size: the
 * default policy leaves small calls to the host pool. */
#define AC_TESTING_DEVICE_PACK 8u

/* Sets the hooks (an OR of the flags above); returns the previous value. */
uint32_t ac_testing_stage_hooks(uint32_t flags);


#ifdef __cplusplus
}
#endif
#endif /* APPROX_COUNTER_AMD_TESTING_H */
