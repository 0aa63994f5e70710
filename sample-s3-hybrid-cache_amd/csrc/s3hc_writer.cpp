// s3hc_writer.cpp — batched incremental range writers over a cross-request batch aggregator.
//
// Mirrors IncrementalRangeWriter (src/disk_cache.rs:262-305) and its life cycle:
//   begin_incremental_range_write  (disk_cache.rs:1716-1778)  -> s3hc_writer_begin
//   write_range_chunk              (disk_cache.rs:1798-1810)  -> s3hc_writer_write
//   flush_batch                    (disk_cache.rs:1820-1870)  -> queued on the aggregator
//   finalize_incremental_range     (disk_cache.rs:1968-2090)  -> s3hc_writer_commit
//   abort_incremental_range        (disk_cache.rs:2093-2116)  -> s3hc_writer_abort
// The reference encodes every batch inline on the writer's own spawn_blocking thread, one
// lz4_flex FrameEncoder per ~1 MiB batch. Here a full batch is queued instead, and the
// aggregator encodes the queued batches of all writers together in one GPU launch (one
// s3hc_plan_encode item per batch). Each batch still becomes exactly
// one frame — compressed (lz4_flex Auto layout) when the writer has compression enabled,
// store-mode otherwise — byte-identical to s3hc_compress_frame / s3hc_store_mode_frame of the
// same bytes, and each writer's frames reach its sink in batch order (the reference's
// file.write_all). Batching semantics are unchanged: a batch is flushed when it reaches
// batch_size (>=), the residual at commit, nothing when empty; bytes_written counts every
// chunk, compressed_bytes_written counts delivered frames, and the shared handler stats get
// record_batch_bytes per frame and record_object per committed range.
//
// Differences forced by aggregation (documented in DESIGN.md): an encode or sink failure of a
// queued batch is reported at the writer's next write/commit call instead of by the write that
// filled the batch; sinks may be called from whichever thread runs the aggregated flush.
//
// This file uses only the public C ABI (include/s3hc_lz4.h), like disk_cache.rs uses
// compression.rs: it is caller-side code, not part of the codec.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "s3hc_guard.hpp"
#include "s3hc_lz4.h"

namespace {

struct Batch {
    s3hc_writer* w;
    std::vector<uint8_t> data;
    uint8_t mode;  // 0 compress, 1 store-mode
};

// Device + pinned host staging reused across flushes (grown on demand).
// Batch mode of S3HC_BLK_LZ4FLEX_COMPAT (not a plan mode: those batches go through
// s3hc_compat_encode_dev, the rest of the flush through one s3hc_encode_dev launch).
constexpr uint8_t kModeCompat = 3;

struct Staging {
    void* h_in = nullptr;
    size_t h_in_cap = 0;
    void* h_out = nullptr;
    size_t h_out_cap = 0;
    void* h_meta = nullptr;
    size_t h_meta_cap = 0;
    void* d_in = nullptr;
    size_t d_in_cap = 0;
    void* d_out = nullptr;
    size_t d_out_cap = 0;
    void* d_meta = nullptr;
    size_t d_meta_cap = 0;
    void* d_cout = nullptr;  // compat frames (slots of s3hc_frame_bound bytes) and lengths
    size_t d_cout_cap = 0;
    void* h_cout = nullptr;
    size_t h_cout_cap = 0;
};

int grow_host(s3hc_ctx* ctx, void** p, size_t* cap, size_t n) {
    if (n <= *cap) return S3HC_OK;
    if (*p) s3hc_host_free(ctx, *p);
    *p = nullptr;
    *cap = 0;
    const size_t want = std::max<size_t>(n, 1 << 20);
    int rc = s3hc_host_alloc(ctx, want, p);
    if (rc == S3HC_OK) *cap = want;
    return rc;
}
int grow_dev(s3hc_ctx* ctx, void** p, size_t* cap, size_t n) {
    if (n <= *cap) return S3HC_OK;
    if (*p) s3hc_dev_free(ctx, *p);
    *p = nullptr;
    *cap = 0;
    const size_t want = std::max<size_t>(n, 1 << 20);
    int rc = s3hc_dev_alloc(ctx, want, p);
    if (rc == S3HC_OK) *cap = want;
    return rc;
}

}  // namespace

// One device of an aggregator: its context, HIP queue and staging (s3hc_aggregator_create_multi
// gives one per device; a flush encodes one contiguous shard of the queued batches on each).
struct Lane {
    s3hc_ctx* ctx = nullptr;
    void* queue = nullptr;   // the lane's HIP queue
    Staging stg;
};

struct s3hc_aggregator {
    std::vector<Lane> lanes;  // lanes[0]: the context of s3hc_aggregator_create
    size_t batch_size;
    size_t flush_bytes;
    uint32_t flush_batches;
    s3hc_handler* stats;     // optional shared counters (the writers' Arc<CompressionStatsAtomic>)
    uint8_t compress_mode = 0;  // compressed batches: 0 lz4_flex Auto, 2 64 KiB frames, kModeCompat
    std::mutex mu;           // guards pending / pending_bytes / counters
    std::mutex flush_mu;     // one aggregated flush at a time (keeps per-writer frame order)
    std::deque<Batch> pending;
    size_t pending_bytes = 0;
    uint64_t launches = 0;
    uint64_t batches_encoded = 0;
};

struct s3hc_writer {
    s3hc_aggregator* agg;
    s3hc_frame_sink sink;
    void* user;
    uint64_t start, end;
    bool compression_enabled;
    std::vector<uint8_t> batch_buf;
    uint64_t bytes_written = 0;             // every chunk (uncompressed)
    uint64_t compressed_bytes_written = 0;  // delivered frames
    uint32_t queued = 0;                    // batches queued and not yet delivered
    std::atomic<int> error{S3HC_OK};        // sticky: first failure of a queued batch (set under agg->mu)
    std::string error_msg;                  // guarded by agg->mu
};

static thread_local std::string g_werr;
extern "C" const char* s3hc_writer_last_error(void) { return g_werr.c_str(); }
static int werr(int code, const std::string& m) {
    g_werr = m;
    return code;
}
// The writer's sticky error as a status + message (a flush on another thread may set it).
static int writer_error(s3hc_writer* w) {
    if (!w->error.load(std::memory_order_acquire)) return S3HC_OK;
    std::lock_guard<std::mutex> g(w->agg->mu);
    return werr(w->error.load(std::memory_order_relaxed), w->error_msg);
}
template <class F>
static int guarded(F&& f) {
    return s3hc::guarded_call(werr, f);
}
static void set_writer_error(s3hc_writer* w, int rc, const std::string& msg) {  // caller holds agg->mu
    if (!w->error.load(std::memory_order_relaxed)) {
        w->error_msg = msg;
        w->error.store(rc, std::memory_order_release);
    }
}

// Contiguous shards by byte midpoint (s3hc_shard_items in s3hc_lz4.h).
extern "C" int s3hc_shard_items(const uint64_t* len, uint32_t n, int ndev, uint32_t* first) {
    if ((!len && n) || !first || ndev < 1) return werr(S3HC_INVALID_ARG, "bad arguments");
    unsigned __int128 total = 0;
    for (uint32_t i = 0; i < n; ++i) total += len[i];
    first[0] = 0;
    first[ndev] = n;
    uint32_t i = 0;
    unsigned __int128 acc = 0;  // bytes of items [0, i)
    for (int d = 1; d < ndev; ++d) {
        // first item whose midpoint lies at or beyond d / ndev of the bytes
        while (i < n && (2 * acc + len[i]) * (unsigned __int128)ndev < 2 * total * (unsigned __int128)d) acc += len[i++];
        uint32_t f = i;
        if (n >= (uint32_t)ndev) {  // every shard non-empty
            f = std::max<uint32_t>(f, first[d - 1] + 1);
            f = std::min<uint32_t>(f, n - (uint32_t)(ndev - d));
        } else {
            f = std::max<uint32_t>(f, first[d - 1]);
        }
        first[d] = f;
    }
    return S3HC_OK;
}

// Encode batches [i0, i1) of `work` on one lane: frame[i] / flen[i] point into the lane's pinned
// staging afterwards. On failure returns the status and sets *msg (the C ABI's message is
// thread-local, so it is read on this thread).
static int encode_shard(const s3hc_aggregator* a, Lane& Ln, const std::deque<Batch>& work, uint32_t i0, uint32_t i1,
                        std::vector<const uint8_t*>& frame, std::vector<uint32_t>& flen, std::string* msg) {
    const uint32_t n = i1 - i0;
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    std::vector<uint8_t> mode(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        off[i] = total;
        len[i] = (uint32_t)work[i0 + i].data.size();
        mode[i] = work[i0 + i].mode;
        total += len[i];
    }
    auto failed = [&](int rc, const char* what) {
        *msg = std::string(what) + ": " + s3hc_last_error();
        return rc;
    };
    s3hc_ctx* ctx = Ln.ctx;
    Staging& S = Ln.stg;
    int rc = grow_host(ctx, &S.h_in, &S.h_in_cap, total + 64);
    if (!rc) rc = grow_dev(ctx, &S.d_in, &S.d_in_cap, total + 64);
    if (rc) return failed(rc, "staging allocation");
    for (uint32_t i = 0; i < n; ++i) memcpy((uint8_t*)S.h_in + off[i], work[i0 + i].data.data(), len[i]);
    // plan-encoded batches (Auto / 64 KiB frames / store-mode) and compat batches
    std::vector<uint32_t> ia, ic;
    for (uint32_t i = 0; i < n; ++i) (mode[i] == kModeCompat ? ic : ia).push_back(i);
    if (total) rc = s3hc_memcpy_async(ctx, S.d_in, S.h_in, total, 1, Ln.queue);
    if (rc) return failed(rc, "staging copy");
    if (!ia.empty()) {
        const uint32_t na = (uint32_t)ia.size();
        std::vector<uint64_t> offa(na);
        std::vector<uint32_t> lena(na);
        std::vector<uint8_t> modea(na);
        for (uint32_t j = 0; j < na; ++j) { offa[j] = off[ia[j]]; lena[j] = len[ia[j]]; modea[j] = mode[ia[j]]; }
        s3hc_plan* plan = nullptr;
        rc = s3hc_plan_encode(ctx, offa.data(), lena.data(), modea.data(), na, &plan);
        if (rc) return failed(rc, "plan");
        const uint64_t bound = s3hc_plan_dst_bound(plan);
        rc = grow_dev(ctx, &S.d_out, &S.d_out_cap, bound + 64);
        if (!rc) rc = grow_host(ctx, &S.h_out, &S.h_out_cap, bound + 64);
        if (!rc) rc = grow_dev(ctx, &S.d_meta, &S.d_meta_cap, 12ull * na + 64);
        if (!rc) rc = grow_host(ctx, &S.h_meta, &S.h_meta_cap, 12ull * na + 64);
        uint64_t* d_ioff = (uint64_t*)S.d_meta;
        uint32_t* d_ilen = (uint32_t*)((uint8_t*)S.d_meta + 8ull * na);
        if (!rc) rc = s3hc_encode_dev(ctx, plan, (const uint8_t*)S.d_in, (uint8_t*)S.d_out, S.d_out_cap, d_ioff, d_ilen, Ln.queue);
        if (!rc) rc = s3hc_memcpy_async(ctx, S.h_meta, S.d_meta, 12ull * na, 2, Ln.queue);
        if (!rc) rc = s3hc_queue_sync(ctx, Ln.queue);
        s3hc_plan_free(plan);
        if (rc) return failed(rc, "encode");
        const uint64_t* io = (const uint64_t*)S.h_meta;
        const uint32_t* il = (const uint32_t*)((const uint8_t*)S.h_meta + 8ull * na);
        const uint64_t bytes = io[na - 1] + il[na - 1];  // frames are packed in item order
        rc = s3hc_memcpy_async(ctx, S.h_out, S.d_out, bytes, 2, Ln.queue);
        if (!rc) rc = s3hc_queue_sync(ctx, Ln.queue);
        if (rc) return failed(rc, "frame copy");
        for (uint32_t j = 0; j < na; ++j) { frame[i0 + ia[j]] = (const uint8_t*)S.h_out + io[j]; flen[i0 + ia[j]] = il[j]; }
    }
    if (!ic.empty()) {
        const uint32_t nc = (uint32_t)ic.size();
        std::vector<uint64_t> offc(nc), dof(nc);
        std::vector<uint32_t> lenc(nc);
        uint64_t slots = 0;
        for (uint32_t j = 0; j < nc; ++j) {
            offc[j] = off[ic[j]];
            lenc[j] = len[ic[j]];
            dof[j] = slots;
            slots += s3hc_frame_bound(lenc[j]);
        }
        const uint64_t lens_at = (slots + 15) & ~15ull;
        rc = grow_dev(ctx, &S.d_cout, &S.d_cout_cap, lens_at + 4ull * nc + 64);
        if (!rc) rc = grow_host(ctx, &S.h_cout, &S.h_cout_cap, lens_at + 4ull * nc + 64);
        uint32_t* d_clen = (uint32_t*)((uint8_t*)S.d_cout + lens_at);
        if (!rc) rc = s3hc_compat_encode_dev(ctx, (const uint8_t*)S.d_in, offc.data(), lenc.data(), nc,
                                             (uint8_t*)S.d_cout, dof.data(), d_clen, Ln.queue);
        // frame lengths first
        if (!rc) rc = s3hc_memcpy_async(ctx, (uint8_t*)S.h_cout + lens_at, d_clen, 4ull * nc, 2, Ln.queue);
        if (!rc) rc = s3hc_queue_sync(ctx, Ln.queue);
        if (rc) return failed(rc, "compat encode");
        const uint32_t* cl = (const uint32_t*)((const uint8_t*)S.h_cout + lens_at);
        for (uint32_t j = 0; j < nc; ++j) { frame[i0 + ic[j]] = (const uint8_t*)S.h_cout + dof[j]; flen[i0 + ic[j]] = cl[j]; }
        // then only each frame's own bytes (not its whole s3hc_frame_bound slot)
        for (uint32_t j = 0; j < nc && !rc; ++j)
            if (cl[j]) rc = s3hc_memcpy_async(ctx, (uint8_t*)S.h_cout + dof[j], (const uint8_t*)S.d_cout + dof[j], cl[j], 2, Ln.queue);
        if (!rc) rc = s3hc_queue_sync(ctx, Ln.queue);
        if (rc) return failed(rc, "compat frame copy");
    }
    (void)a;
    return S3HC_OK;
}

// Encode every queued batch (one launch per device: contiguous shards over the aggregator's
// lanes, run concurrently) and deliver the frames in queue order. Caller holds flush_mu.
static int aggregated_flush(s3hc_aggregator* a) {
    std::deque<Batch> work;
    {
        std::lock_guard<std::mutex> g(a->mu);
        work.swap(a->pending);
        a->pending_bytes = 0;
    }
    if (work.empty()) return S3HC_OK;
    const uint32_t n = (uint32_t)work.size();
    const int nl = (int)std::min<size_t>(a->lanes.size(), n);
    std::vector<uint64_t> blen(n);
    for (uint32_t i = 0; i < n; ++i) blen[i] = work[i].data.size();
    std::vector<uint32_t> first(nl + 1);
    (void)s3hc_shard_items(blen.data(), n, nl, first.data());
    std::vector<const uint8_t*> frame(n, nullptr);
    std::vector<uint32_t> flen(n, 0);
    std::vector<int> rc(nl, S3HC_OK);
    std::vector<std::string> msg(nl);
    auto run = [&](int d) {
        try {
            if (first[d] < first[d + 1]) rc[d] = encode_shard(a, a->lanes[d], work, first[d], first[d + 1], frame, flen, &msg[d]);
        } catch (const std::bad_alloc&) {
            rc[d] = S3HC_NO_MEMORY;
            msg[d] = "out of memory";
        } catch (...) {
            rc[d] = S3HC_DEVICE;
            msg[d] = "internal error";
        }
    };
    // every shard must encode with lane 0's match-finder mode, or the frames would depend on
    // which device a batch landed on (the byte-identical guarantee of the one-device aggregator)
    const int mode0 = s3hc_get_encode_mode(a->lanes[0].ctx);
    bool mixed = false;
    for (int d = 1; d < nl; ++d) mixed |= s3hc_get_encode_mode(a->lanes[d].ctx) != mode0;
    if (mixed)
        for (int d = 0; d < nl; ++d) {
            rc[d] = S3HC_INVALID_ARG;
            msg[d] = "aggregator contexts use different encode modes (s3hc_set_encode_mode)";
        }
    auto run_ok = [&](int d) {
        if (rc[d] == S3HC_OK) run(d);
    };
    if (nl == 1) {
        run_ok(0);
    } else {
        // (a thread that cannot be started leaves its shard to this thread, after the others;
        // every started thread is joined on every path)
        std::vector<std::thread> th;
        std::vector<int> inline_d;
        for (int d = 1; d < nl; ++d) {
            try {
                th.emplace_back(run_ok, d);
            } catch (...) {
                inline_d.push_back(d);
            }
        }
        run_ok(0);
        for (int d : inline_d) run_ok(d);
        for (auto& t : th) t.join();
    }
    int first_rc = S3HC_OK;
    std::string first_msg;
    {
        std::lock_guard<std::mutex> g(a->mu);
        for (int d = 0; d < nl; ++d) {
            if (rc[d] == S3HC_OK) continue;
            if (!first_rc) { first_rc = rc[d]; first_msg = msg[d]; }
            for (uint32_t i = first[d]; i < first[d + 1]; ++i) set_writer_error(work[i].w, rc[d], msg[d]);
        }
        for (int d = 0; d < nl; ++d) a->launches += rc[d] == S3HC_OK && first[d] < first[d + 1];
        a->batches_encoded += n;
    }
    // deliver in queue order: each writer's frames keep their batch order (a writer with a
    // failed batch gets none of its later frames)
    for (uint32_t i = 0; i < n; ++i) {
        s3hc_writer* w = work[i].w;
        const uint8_t* fr = frame[i];
        int src = S3HC_OK;
        if (!w->error.load(std::memory_order_acquire) && fr) {
            if (w->sink && w->sink(w->user, fr, flen[i]) != 0) {
                src = S3HC_INVALID_ARG;
            } else {
                w->compressed_bytes_written += flen[i];
                if (a->stats) s3hc_handler_record_batch_bytes(a->stats, blen[i], flen[i]);
            }
        }
        std::lock_guard<std::mutex> g(a->mu);
        if (src) set_writer_error(w, src, "frame sink failed (write_all)");
        w->queued--;
    }
    return first_rc ? werr(first_rc, first_msg) : S3HC_OK;
}

static int maybe_flush(s3hc_aggregator* a, bool force) {
    bool go = force;
    {
        std::lock_guard<std::mutex> g(a->mu);
        if (a->pending.empty()) return S3HC_OK;
        if (!go) go = (a->flush_bytes && a->pending_bytes >= a->flush_bytes) ||
                      (a->flush_batches && a->pending.size() >= a->flush_batches);
    }
    if (!go) return S3HC_OK;
    std::lock_guard<std::mutex> f(a->flush_mu);
    return aggregated_flush(a);
}

// flush_batch (disk_cache.rs:1820-1870): no-op on an empty buffer; otherwise the batch
// becomes one queued frame.
static void queue_batch(s3hc_writer* w) {
    if (w->batch_buf.empty()) return;
    s3hc_aggregator* a = w->agg;
    Batch b;
    b.w = w;
    b.data.swap(w->batch_buf);
    w->batch_buf.clear();
    w->batch_buf.reserve(a->batch_size);
    std::lock_guard<std::mutex> g(a->mu);
    b.mode = w->compression_enabled ? a->compress_mode : 1;
    a->pending_bytes += b.data.size();
    w->queued++;
    a->pending.push_back(std::move(b));
}

namespace s3hc {
void ctx_retain(s3hc_ctx* ctx);   // s3hc_runtime.cpp: a lane keeps its context alive
void ctx_release(s3hc_ctx* ctx);
}  // namespace s3hc
static void free_lane(Lane& L) {
    s3hc_ctx* ctx = L.ctx;
    Staging& S = L.stg;
    if (S.h_in) s3hc_host_free(ctx, S.h_in);
    if (S.h_out) s3hc_host_free(ctx, S.h_out);
    if (S.h_meta) s3hc_host_free(ctx, S.h_meta);
    if (S.d_in) s3hc_dev_free(ctx, S.d_in);
    if (S.d_out) s3hc_dev_free(ctx, S.d_out);
    if (S.d_meta) s3hc_dev_free(ctx, S.d_meta);
    if (S.h_cout) s3hc_host_free(ctx, S.h_cout);
    if (S.d_cout) s3hc_dev_free(ctx, S.d_cout);
    if (L.queue) s3hc_queue_destroy(ctx, L.queue);
    L = Lane();
    if (ctx) s3hc::ctx_release(ctx);
}

static int aggregator_new(s3hc_ctx* const* ctxs, int nctx, size_t batch_size, size_t flush_bytes,
                          uint32_t flush_batches, s3hc_handler* stats, s3hc_aggregator** out) {
    for (int i = 0; i < nctx; ++i) {
        if (!ctxs[i]) return werr(S3HC_INVALID_ARG, "NULL context");
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return werr(S3HC_INVALID_ARG, "a context is listed twice");
    }
    for (int i = 1; i < nctx; ++i)
        if (s3hc_get_encode_mode(ctxs[i]) != s3hc_get_encode_mode(ctxs[0]))
            return werr(S3HC_INVALID_ARG, "contexts use different encode modes (s3hc_set_encode_mode)");
    std::unique_ptr<s3hc_aggregator> a(new s3hc_aggregator);
    a->batch_size = batch_size;
    a->flush_bytes = flush_bytes;
    a->flush_batches = flush_batches;
    a->stats = stats;
    a->lanes.resize(nctx);
    for (int i = 0; i < nctx; ++i) {
        a->lanes[i].ctx = ctxs[i];
        s3hc::ctx_retain(ctxs[i]);  // released by free_lane
        int rc = s3hc_queue_create(ctxs[i], &a->lanes[i].queue);
        if (rc) {
            const std::string m = std::string("queue: ") + s3hc_last_error();
            for (auto& L : a->lanes) if (L.ctx) free_lane(L);
            return werr(rc, m);
        }
    }
    *out = a.release();
    return S3HC_OK;
}

extern "C" int s3hc_aggregator_create(s3hc_ctx* ctx, size_t batch_size, size_t flush_bytes, uint32_t flush_batches,
                                      s3hc_handler* stats, s3hc_aggregator** out) {
    return guarded([&]() -> int {
        if (!ctx || !out) return werr(S3HC_INVALID_ARG, "bad arguments");
        *out = nullptr;
        // DiskCacheManager takes any batch size (its tests use 4-8 KiB); the 64 KiB..16 MiB bounds
        // belong to Config::validate (config.rs:1617-1627), the caller's configuration layer.
        if (batch_size == 0 || batch_size > 0xFFFFFFFFull / 2) return werr(S3HC_INVALID_ARG, "batch_size out of range");
        return aggregator_new(&ctx, 1, batch_size, flush_bytes, flush_batches, stats, out);
    });
}
extern "C" int s3hc_aggregator_create_multi(s3hc_ctx* const* ctxs, int nctx, size_t batch_size, size_t flush_bytes,
                                            uint32_t flush_batches, s3hc_handler* stats, s3hc_aggregator** out) {
    return guarded([&]() -> int {
        if (!ctxs || nctx < 1 || !out) return werr(S3HC_INVALID_ARG, "bad arguments");
        *out = nullptr;
        if (batch_size == 0 || batch_size > 0xFFFFFFFFull / 2) return werr(S3HC_INVALID_ARG, "batch_size out of range");
        return aggregator_new(ctxs, nctx, batch_size, flush_bytes, flush_batches, stats, out);
    });
}

extern "C" int s3hc_aggregator_set_frame_policy(s3hc_aggregator* a, int policy) {
    return guarded([&]() -> int {
        if (!a || (policy != S3HC_BLK_AUTO_LZ4FLEX && policy != S3HC_BLK_64K_PER_FRAME &&
                   policy != S3HC_BLK_LZ4FLEX_COMPAT))
            return werr(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(a->mu);
        a->compress_mode = policy == S3HC_BLK_64K_PER_FRAME ? 2 : (policy == S3HC_BLK_LZ4FLEX_COMPAT ? kModeCompat : 0);
        return S3HC_OK;
    });
}

extern "C" int s3hc_aggregator_flush(s3hc_aggregator* a) {
    return guarded([&]() -> int {
        if (!a) return werr(S3HC_INVALID_ARG, "bad arguments");
        return maybe_flush(a, true);
    });
}

extern "C" void s3hc_aggregator_counters(const s3hc_aggregator* a, uint64_t* launches, uint64_t* batches) {
    if (!a) return;
    std::lock_guard<std::mutex> g(const_cast<s3hc_aggregator*>(a)->mu);
    if (launches) *launches = a->launches;
    if (batches) *batches = a->batches_encoded;
}

extern "C" void s3hc_aggregator_destroy(s3hc_aggregator* a) {
    if (!a) return;
    {
        std::lock_guard<std::mutex> f(a->flush_mu);
        (void)aggregated_flush(a);
    }
    for (auto& L : a->lanes) free_lane(L);
    delete a;
}

extern "C" int s3hc_writer_begin(s3hc_aggregator* a, uint64_t start, uint64_t end, int compression_enabled,
                                 s3hc_frame_sink sink, void* user, s3hc_writer** out) {
    return guarded([&]() -> int {
        if (!a || !out) return werr(S3HC_INVALID_ARG, "bad arguments");
        *out = nullptr;
        if (start > end) return werr(S3HC_INVALID_ARG, "Invalid range: start > end");  // disk_cache.rs:1723-1728
        s3hc_writer* w = new s3hc_writer;
        w->agg = a;
        w->sink = sink;
        w->user = user;
        w->start = start;
        w->end = end;
        w->compression_enabled = compression_enabled != 0;
        w->batch_buf.reserve(a->batch_size);
        *out = w;
        return S3HC_OK;
    });
}

extern "C" int s3hc_writer_write(s3hc_writer* w, const uint8_t* chunk, size_t n) {
    return guarded([&]() -> int {
        if (!w || (!chunk && n)) return werr(S3HC_INVALID_ARG, "bad arguments");
        if (int e = writer_error(w)) return e;
        if (n == 0) return S3HC_OK;                    // disk_cache.rs:1799-1801
        // one batch is one frame of one plan item (32-bit length): a batch of >= 4 GiB is refused
        if (w->batch_buf.size() + n > 0xFFFFFFFFull) return werr(S3HC_UNSUPPORTED, "a batch of 4 GiB or more");
        w->bytes_written += n;
        w->batch_buf.insert(w->batch_buf.end(), chunk, chunk + n);
        if (w->batch_buf.size() >= w->agg->batch_size) {  // >= flushes (disk_cache.rs:1806)
            queue_batch(w);
            int rc = maybe_flush(w->agg, false);
            if (rc && !w->error.load(std::memory_order_acquire)) return rc;
        }
        return writer_error(w);
    });
}

extern "C" size_t s3hc_writer_batch_buf_len(const s3hc_writer* w) { return w ? w->batch_buf.size() : 0; }
extern "C" uint64_t s3hc_writer_bytes_written(const s3hc_writer* w) { return w ? w->bytes_written : 0; }
extern "C" uint64_t s3hc_writer_compressed_bytes_written(const s3hc_writer* w) {
    return w ? w->compressed_bytes_written : 0;
}

// Wait until every queued batch of w has been delivered (flushes as needed).
static int drain(s3hc_writer* w) {
    for (;;) {
        {
            std::lock_guard<std::mutex> g(w->agg->mu);
            if (w->queued == 0) return S3HC_OK;
        }
        int rc = maybe_flush(w->agg, true);  // serialized by flush_mu: waits for a flush in flight
        if (rc) return rc;
    }
}

// Frees a writer when commit returns, however it returns: commit consumes the writer, so an
// exception out of queue_batch / drain (caught by guarded()) must not leak it. On that path the
// writer's queued batches are drained first (they reference it), as s3hc_writer_abort does.
struct WriterReaper {
    s3hc_writer* w;
    ~WriterReaper() {
        if (!w) return;
        try {
            {
                std::lock_guard<std::mutex> g(w->agg->mu);
                set_writer_error(w, S3HC_INVALID_ARG, "commit failed");
            }
            (void)drain(w);
        } catch (...) {
        }
        delete w;
    }
};

extern "C" int s3hc_writer_commit(s3hc_writer* w, double min_commit_ratio, uint64_t spec_out[4]) {
    if (!w) return werr(S3HC_INVALID_ARG, "bad arguments");
    WriterReaper reaper{w};
    return guarded([&]() -> int {
        // finalize_incremental_range: residual batch first (disk_cache.rs:1981-1986)
        queue_batch(w);
        int rc = drain(w);
        if (!rc) rc = writer_error(w);
        if (rc) {
            reaper.w = nullptr;
            delete w;  // the reference removes the .tmp file; the caller discards what its sink wrote
            return rc;
        }
        uint64_t end = w->end;
        const uint64_t expected = w->end - w->start + 1;
        if (w->bytes_written != expected) {
            // partial-prefix salvage (disk_cache.rs:1988-2023): read path passes a ratio; < 0 = exact only
            const bool salvage = min_commit_ratio >= 0.0 && w->bytes_written > 0 && w->bytes_written < expected &&
                                 (double)w->bytes_written >= min_commit_ratio * (double)expected;
            if (!salvage) {
                char m[160];
                snprintf(m, sizeof m, "Incremental write size mismatch: expected %llu bytes, got %llu",
                         (unsigned long long)expected, (unsigned long long)w->bytes_written);
                reaper.w = nullptr;
                delete w;
                return werr(S3HC_INVALID_ARG, m);
            }
            end = w->start + w->bytes_written - 1;
        }
        if (w->agg->stats) s3hc_handler_record_object(w->agg->stats, w->compression_enabled ? 1 : 0);  // :2053
        if (spec_out) {  // RangeSpec::new(start, end, path, Lz4, compressed, uncompressed) (disk_cache.rs:2080-2087)
            spec_out[0] = w->start;
            spec_out[1] = end;
            spec_out[2] = w->compressed_bytes_written;
            spec_out[3] = w->bytes_written;
        }
        reaper.w = nullptr;
        delete w;
        return S3HC_OK;
    });
}

extern "C" void s3hc_writer_abort(s3hc_writer* w) {
    if (!w) return;
    // queued batches still reference w: let them drain (their frames go to the sink, which the
    // caller is discarding together with the .tmp file) before freeing
    {
        std::lock_guard<std::mutex> g(w->agg->mu);
        set_writer_error(w, S3HC_INVALID_ARG, "aborted");
    }
    (void)drain(w);
    delete w;
}
