// s3hc_knobs.hpp — diagnostic / A-B switches of the engine (host side only).
//
// Every knob is read from the environment once per process, at the first s3hc_create(), and
// can be changed later through s3hc_set_knob() (tests flip decoders between calls). The
// per-call decode path only reads these cached values: no getenv on it.
#pragma once
#include <atomic>
#include <stdint.h>

// Comparison variants (the one-wave unit decoder): diagnostic builds only,
// make diag DIAG=-DS3HC_DIAG_VARIANTS=1; the shipped library has neither the kernel nor the knob.
#ifndef S3HC_DIAG_VARIANTS
#define S3HC_DIAG_VARIANTS 0
#endif

namespace s3hc {

enum Knob : int {
    KN_FAST_DISABLE = 0,  // S3HC_FAST_DISABLE=1 or S3HC_FAST=0: every 64 KiB unit on the per-unit decoder
    KN_LB_DISABLE,        // S3HC_LB_DISABLE=1: no large-block path (every block one unit per workgroup)
    KN_LBW_DISABLE,       // S3HC_LBW_DISABLE=1: large blocks on the step loop, never spread
    KN_LBW_CAP,           // S3HC_LBW_CAP=<positions>: spread-execution capacity (-1: the size rule)
    KN_LBW_ROUNDS,        // S3HC_LBW_ROUNDS=<n>: fewer pointer-jumping launches (-1: all)
    KN_DEC_ONEWAVE,       // S3HC_DEC_ONEWAVE=1 (S3HC_DIAG_VARIANTS builds): the one-wave unit decoder
    KN_FAST_TRACE,        // S3HC_FAST_TRACE=1: stderr line per decode launch (serialises the stream)
    KN_LB_TRACE,          // S3HC_LB_TRACE=1: stderr line per large-block launch (serialises the stream)
    KN_HOST_TRACE,        // S3HC_HOST_TRACE=1: host-call stage times on stderr
    KN_READER_SLOTS,      // S3HC_READER_SLOTS=<n>: range-reader batches in flight per HIP queue (1..4)
    KN_POISON,            // S3HC_POISON=1: device scratch filled with 0xFF on (re)allocation
    KN_COUNT
};

extern std::atomic<long long> g_knob[KN_COUNT];

inline long long knob(Knob k) { return g_knob[k].load(std::memory_order_relaxed); }
inline bool knob_on(Knob k) { return knob(k) > 0; }

// reads the environment (first s3hc_create of the process)
void knobs_load_env_once();

}  // namespace s3hc
