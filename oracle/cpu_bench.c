/*
 * cpu_bench.c — TEST INFRASTRUCTURE ONLY: the timing harness of bench.py's cpu_baseline leg.
 *
 * Times the CPU port of the reference path (lz4_oracle.c: the lz4_flex FrameEncoder restatement
 * followed by decompress_data, i.e. compression.rs:530-591 then :463-502) on the host's cores,
 * one std-style thread per core over contiguous block ranges, mirroring the reference's
 * one-request-per-spawn_blocking-thread model (http_proxy.rs:11608-11622).
 * Wall-clock CLOCK_MONOTONIC. The product library never links this file.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lz4_oracle.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    const uint8_t* data;
    size_t nblocks, block, lo, cnt;
    double deadline;
    int fixed;  /* 1: exactly cnt blocks; 0: until the deadline (at least one pass over lo..) */
    int lib;    /* 0: the oracle's lz4_flex frame path; 1: liblz4's raw block API (third-party C) */
    uint64_t done;
    double enc_s, dec_s;
    int rc;
} tjob_t;

/* liblz4 (system library, dlopen'ed: a third-party C LZ4, not the proxy's codec): the raw block
 * API without frames or checksums, the fastest CPU LZ4 this host has as a labelled reference. */
typedef int (*lz4_comp_fn)(const char*, char*, int, int);
typedef int (*lz4_dec_fn)(const char*, char*, int, int);
static lz4_comp_fn g_lz4_comp;
static lz4_dec_fn g_lz4_dec;
static int lz4_load(void) {
    if (g_lz4_comp && g_lz4_dec) return 0;
    void* h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    g_lz4_comp = (lz4_comp_fn)dlsym(h, "LZ4_compress_default");
    g_lz4_dec = (lz4_dec_fn)dlsym(h, "LZ4_decompress_safe");
    return g_lz4_comp && g_lz4_dec ? 0 : -1;
}

static void* tmain(void* arg) {
    tjob_t* J = (tjob_t*)arg;
    const size_t cap = or_frame_bound(J->block);
    uint8_t* fr = (uint8_t*)malloc(cap);
    uint8_t* out = (uint8_t*)malloc(J->block);
    if (!fr || !out) {
        J->rc = -1;
        free(fr);
        free(out);
        return NULL;
    }
    for (size_t k = 0;; ++k) {
        if (J->fixed ? k >= J->cnt : (k > 0 && (k & 7) == 0 && now_s() >= J->deadline)) break;
        const size_t i = (J->lo + k) % J->nblocks;
        size_t n = 0, m = 0;
        const double t0 = now_s();
        int rc;
        if (J->lib) {
            const int c = g_lz4_comp((const char*)(J->data + i * J->block), (char*)fr, (int)J->block, (int)cap);
            rc = c > 0 ? 0 : -4;
            n = c > 0 ? (size_t)c : 0;
        } else {
            rc = or_lz4flex_compress_frame(J->data + i * J->block, J->block, fr, cap, &n);
        }
        const double t1 = now_s();
        if (!rc && J->lib) {
            const int d = g_lz4_dec((const char*)fr, (char*)out, (int)n, (int)J->block);
            rc = d >= 0 ? 0 : -4;
            m = d >= 0 ? (size_t)d : 0;
        } else if (!rc) {
            rc = or_decompress_data(fr, n, out, J->block, &m);
        }
        const double t2 = now_s();
        if (rc || m != J->block || memcmp(out, J->data + i * J->block, J->block) != 0) {
            J->rc = rc ? rc : -2;
            break;
        }
        J->enc_s += t1 - t0;
        J->dec_s += t2 - t1;
        J->done++;
    }
    free(fr);
    free(out);
    return NULL;
}

/* Encode+decode blocks on `threads` threads, thread t starting at block t*nblocks/threads.
 * fixed_per_thread > 0: exactly that many blocks per thread; else run for `seconds` of wall.
 * Outputs: blocks done (all threads), wall seconds, summed per-thread encode/decode seconds.
 * Returns 0, or the first failing thread's status (a round trip that did not reproduce). */
static int bench_blocks(const uint8_t* data, size_t nblocks, size_t block, int threads, double seconds,
                        size_t fixed_per_thread, uint64_t* blocks_done, double* wall, double* enc_s, double* dec_s,
                        int lib) {
    if (!data || !nblocks || !block || threads < 1) return OR_INVALID_ARG;
    if (lib && lz4_load() != 0) return -5;
    tjob_t* J = (tjob_t*)calloc((size_t)threads, sizeof(tjob_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    char* started = (char*)calloc((size_t)threads, 1);
    if (!J || !th || !started) {
        free(J);
        free(th);
        free(started);
        return OR_INVALID_ARG;
    }
    const double t0 = now_s();
    for (int t = 0; t < threads; ++t) {
        J[t].data = data;
        J[t].nblocks = nblocks;
        J[t].block = block;
        J[t].lo = (size_t)t * nblocks / (size_t)threads;
        J[t].cnt = fixed_per_thread;
        J[t].fixed = fixed_per_thread > 0;
        J[t].deadline = t0 + seconds;
        J[t].lib = lib;
        started[t] = pthread_create(&th[t], NULL, tmain, &J[t]) == 0;
    }
    int rc = 0;
    uint64_t done = 0;
    double es = 0, ds = 0;
    for (int t = 0; t < threads; ++t) {
        if (started[t]) pthread_join(th[t], NULL);
        else rc = rc ? rc : -3;
        if (J[t].rc && !rc) rc = J[t].rc;
        done += J[t].done;
        es += J[t].enc_s;
        ds += J[t].dec_s;
    }
    *wall = now_s() - t0;
    *blocks_done = done;
    *enc_s = es;
    *dec_s = ds;
    free(J);
    free(th);
    free(started);
    return rc;
}

int or_bench_blocks(const uint8_t* data, size_t nblocks, size_t block, int threads, double seconds,
                    size_t fixed_per_thread, uint64_t* blocks_done, double* wall, double* enc_s, double* dec_s) {
    return bench_blocks(data, nblocks, block, threads, seconds, fixed_per_thread, blocks_done, wall, enc_s, dec_s, 0);
}
/* The same harness over liblz4's LZ4_compress_default + LZ4_decompress_safe (-5: liblz4 absent). */
int or_bench_blocks_liblz4(const uint8_t* data, size_t nblocks, size_t block, int threads, double seconds,
                           size_t fixed_per_thread, uint64_t* blocks_done, double* wall, double* enc_s,
                           double* dec_s) {
    return bench_blocks(data, nblocks, block, threads, seconds, fixed_per_thread, blocks_done, wall, enc_s, dec_s, 1);
}
