/*
 * s3hc_lz4_diag.h — diagnostic entry points of libs3hc_lz4.so (tests, A/B measurements).
 *
 * Not part of the drop-in boundary (include/s3hc_lz4.h): the reference has one codec and no
 * switches. Production callers never need these; the Rust binding in INTEGRATION.md leaves them out.
 * S3HC_DEC_ONEWAVE (the one-wave-per-unit decoder) exists only in diagnostic builds
 * (make diag DIAG=-DS3HC_DIAG_VARIANTS=1); the shipped library refuses the name.
 */
#ifndef S3HC_LZ4_DIAG_H
#define S3HC_LZ4_DIAG_H

#include "s3hc_lz4.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic / A-B switches (no reference counterpart: the reference has one codec). Read from
 * the environment (S3HC_FAST_DISABLE, S3HC_FAST, S3HC_LB_DISABLE, S3HC_LBW_DISABLE, S3HC_LBW_CAP,
 * S3HC_LBW_ROUNDS, S3HC_DEC_ONEWAVE, S3HC_FAST_TRACE, S3HC_LB_TRACE, S3HC_HOST_TRACE,
 * S3HC_READER_SLOTS, S3HC_POISON) once per
 * process at the first s3hc_create; this call changes one afterwards (value NULL = default; a
 * flag knob is on when its value is non-NULL, S3HC_FAST is on unless "0"). Process-wide. The
 * per-call decode path only reads the cached values. S3HC_INVALID_ARG for an unknown name.
 * S3HC_POISON=1 fills every device scratch buffer with 0xFF when it is (re)allocated, so a read
 * of memory no launch wrote fails the same way on every box. */
int s3hc_set_knob(const char* name, const char* value);
/* The knob's current raw value (S3HC_FAST reads S3HC_FAST_DISABLE's slot), and setting that raw
 * value back: tests save and restore knobs exactly (aliases share one slot). */
int s3hc_get_knob(const char* name, long long* value);
int s3hc_set_knob_value(const char* name, long long value);

/* Diagnostics (no reference counterpart): the range reader's check of the frame results a batch
 * decode wrote (lengths, statuses) before they drive any device-to-host copy. Frame f's slot is
 * [dst_off[f], dst_off[f + 1]) (the last one up to slot_total). S3HC_OK with *good = frames before
 * the first failing one and *bytes = their decoded bytes; S3HC_DEVICE when a status is not one a
 * decoder assigns or a good frame's length exceeds its slot. Pure host code (tests forge results). */
int s3hc_diag_check_batch_results(uint32_t n, const uint32_t* olen, const int32_t* status,
                                  const uint64_t* dst_off, uint64_t slot_total, uint32_t* good,
                                  uint64_t* bytes);

#ifdef __cplusplus
}
#endif
#endif
