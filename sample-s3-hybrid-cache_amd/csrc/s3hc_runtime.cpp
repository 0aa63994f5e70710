// s3hc_runtime.cpp — host side of the MI355X LZ4 frame engine: the C ABI of
// include/s3hc_lz4.h, the batch planner, and the frame walker for host buffers.
//
// Division of labour: the host plans (frame/block/segment layout,
// header bytes, frame-structure walk of host buffers) and moves bytes; every per-byte
// computation of the codec — LZ4 match finding and token emission, LZ4 block decode,
// stored-block copies and every xxh32 content/block checksum — runs in the HIP kernels
// of s3hc_kernels.hip. There is no CPU codec fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "s3hc_lz4.h"
#include "s3hc_lz4_diag.h"
#include "s3hc_plan.hpp"
#include "s3hc_guard.hpp"
#include "s3hc_knobs.hpp"

namespace s3hc {
hipError_t launch_xxh32(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint32_t*, hipStream_t);
hipError_t launch_compat_frames(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint8_t*, const uint64_t*,
                                const uint32_t*, uint32_t*, uint32_t, hipStream_t);
// per-unit launches: units [0, *ucount) when ucount is set (a device-built plan), else [0, nunits);
// `grid` workgroups stride over them
hipError_t launch_decode_units(const uint8_t*, uint8_t*, const DecBlock*, const DecUnit*, uint32_t, const uint64_t*,
                               uint32_t, uint32_t*, int32_t*, const uint8_t*, const uint8_t*, hipStream_t);
hipError_t launch_fast_tok(const uint8_t*, const DecBlock*, const DecUnit*, uint32_t, const uint64_t*, uint32_t,
                           const uint8_t*, const FastArgs&, hipStream_t);
hipError_t launch_fast_exec(const uint8_t*, uint8_t*, const DecBlock*, const DecUnit*, uint32_t, const uint64_t*,
                            uint32_t, uint32_t*, int32_t*, const FastArgs&, hipStream_t);
bool fast_exec_hashes();
hipError_t launch_fast_small(const uint8_t*, uint8_t*, const DecBlock*, const DecUnit*, uint32_t, const uint8_t*,
                             const FastArgs&, uint32_t*, int32_t*, hipStream_t, bool, bool*);
hipError_t launch_lb_parse(const LbArgs&, const uint8_t*, const DecBlock*, const DecUnit*, uint32_t, const uint64_t*,
                           uint32_t*, int32_t*, hipStream_t);
hipError_t launch_lb_exec(const LbArgs&, const uint8_t*, uint8_t*, uint32_t*, int32_t*, hipStream_t);
hipError_t launch_enc_parse(const uint8_t*, const EncBlock*, const uint2*, uint32_t, const uint64_t*, const uint32_t*,
                            uint32_t, uint32_t*, uint2*, SegSummary*, int, hipStream_t);
hipError_t launch_enc_sizes(const EncBlock*, uint32_t, const SegSummary*, SegPlace*, uint32_t*, uint32_t*,
                            uint32_t*, hipStream_t);
hipError_t launch_scan(const uint32_t*, uint32_t, uint64_t*, uint64_t*, hipStream_t);
hipError_t launch_enc_emit(const uint8_t*, const EncBlock*, const uint32_t*, uint32_t, const uint2*,
                           const SegSummary*, const SegPlace*, const uint32_t*, const uint32_t*, const uint64_t*,
                           const uint32_t*, uint8_t*, hipStream_t);
hipError_t launch_enc_groups(const uint32_t*, const uint32_t*, uint32_t, const uint64_t*, const uint32_t*,
                             uint64_t*, uint32_t*, hipStream_t);
hipError_t launch_dframe_count(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, uint32_t,
                               uint32_t*, int32_t*, hipStream_t);
hipError_t launch_dframe_fill(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, const uint64_t*,
                              const uint32_t*, const uint64_t*, const int32_t*, DecBlock*, DecUnit*, uint32_t*,
                              const uint64_t*, hipStream_t);
hipError_t launch_dframe_finish(const uint64_t*, uint32_t, const uint32_t*, const DecBlock*, const uint32_t*,
                                const int32_t*, int32_t*, uint32_t*, hipStream_t);
hipError_t launch_dframe_verify(const uint8_t*, const uint64_t*, uint32_t, const uint32_t*, const uint32_t*,
                                const uint32_t*, int32_t*, hipStream_t);
hipError_t launch_dframe_close(const uint8_t*, const uint64_t*, const uint64_t*, const uint32_t*, const DecBlock*,
                               const uint32_t*, const int32_t*, const uint64_t*, const uint8_t*, const uint64_t*,
                               const uint32_t*, uint32_t, const int32_t*, int32_t*, uint32_t*, uint32_t*, hipStream_t,
                               uint32_t* pend = nullptr);
}  // namespace s3hc

using namespace s3hc;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
template <class F>
static int guarded(F&& f) {
    return s3hc::guarded_call(fail, f);
}
int s3hc::set_error(int code, const std::string& msg) { return fail(code, msg); }
#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(S3HC_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    } while (0)

extern "C" const char* s3hc_last_error(void) { return g_err.c_str(); }
extern "C" const char* s3hc_version(void) { return "s3hc-lz4 0.1.0 (gfx950)"; }

// ------------------------------------------------------ frame-header xxh32
// Only ever applied to frame-descriptor bytes (<= 14 bytes: FLG, BD, content size,
// dictionary id) to form/check the one-byte header checksum (compression.rs:340-342).
static uint32_t hdr_xxh32(const uint8_t* p, size_t n) {
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
    auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
    uint32_t h = P5 + (uint32_t)n;
    size_t t = 0;
    for (; t + 4 <= n; t += 4) {
        uint32_t w = (uint32_t)p[t] | ((uint32_t)p[t + 1] << 8) | ((uint32_t)p[t + 2] << 16) | ((uint32_t)p[t + 3] << 24);
        h += w * P3;
        h = rotl(h, 17) * P4;
    }
    for (; t < n; ++t) {
        h += p[t] * P5;
        h = rotl(h, 11) * P1;
    }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}
static uint8_t header_hc(uint8_t bd) {
    uint8_t fd[2] = {kFlgIndependentChecksum, bd};
    return (uint8_t)(hdr_xxh32(fd, 2) >> 8);
}
static inline uint32_t rd32h(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// ------------------------------------------------------------ device memory
// Size for a buffer of capacity cap that must hold n > cap bytes: a regrowth of a small buffer
// (< 256 MiB) takes 1.5x its old capacity, so batches whose sizes vary do not reallocate (host
// pinned frees cost ~0.6 ms each); first allocations and large buffers are exact.
static inline size_t regrow(size_t n, size_t cap) {
    return cap && n < ((size_t)256 << 20) ? std::max<size_t>(n, cap + cap / 2) : n;
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    void trim(size_t keep) {  // free a buffer grown beyond `keep` bytes (the next ensure reallocates)
        if (p && cap > keep) { (void)hipFree(p); p = nullptr; cap = 0; }
    }
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        // a buffer that grows again (per-batch sizes vary) takes 1.5x: no realloc churn
        size_t want = std::max<size_t>(regrow(n, cap), 256);
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        if (e == hipSuccess && knob_on(KN_POISON)) {  // diagnostics: unwritten bytes read as 0xFF everywhere
            if ((e = hipMemset(p, 0xFF, want)) == hipSuccess) e = hipDeviceSynchronize();
        }
        return e;
    }
    template <class T> T* as() const { return (T*)p; }
};

template <class T> static hipError_t upload(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
    hipError_t e = b.ensure(v.size() * sizeof(T) + 16);
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st);
}

// ------------------------------------------------------------ pinned host memory
struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    void trim(size_t keep) {
        if (p && cap > keep) { (void)hipHostFree(p); p = nullptr; cap = 0; }
    }
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        const size_t want = std::max<size_t>(regrow(n, cap), 1 << 16);
        if (p) { (void)hipHostFree(p); p = nullptr; cap = 0; }
        hipError_t e = hipHostMalloc((void**)&p, want, hipHostMallocPortable);
        if (e == hipSuccess) cap = want;
        return e;
    }
    // grow to n bytes keeping the first `keep` (no copy into the buffer may be in flight)
    hipError_t ensure_keep(size_t n, size_t keep) {
        if (n <= cap) return hipSuccess;
        uint8_t* q = nullptr;
        const size_t want = std::max<size_t>(regrow(n, cap), 1 << 16);
        hipError_t e = hipHostMalloc((void**)&q, want, hipHostMallocPortable);
        if (e != hipSuccess) return e;
        if (p) {
            memcpy(q, p, std::min(keep, cap));
            (void)hipHostFree(p);
        }
        p = q;
        cap = want;
        return hipSuccess;
    }
};

// Host copy of a large staging buffer split over a few threads (one thread copies ~6-10 GB/s;
// the reader's feed/stage/deliver copies are otherwise the bottleneck of the pipeline).
// Host copies of the range reader and the batch paths: split over a small persistent pool of
// copy threads (no thread start-up per call). The calling thread copies too and helps with
// queued pieces while it waits, so concurrent callers never block each other.
namespace {
class CopyPool {
  public:
    struct State {
        std::atomic<int> left{0};
    };
    struct Job {
        uint8_t* d;
        const uint8_t* s;
        size_t n;
        State* st;
    };
    explicit CopyPool(unsigned nt) {
        for (unsigned i = 0; i < nt; ++i) th_.emplace_back([this] { run(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    unsigned threads() const { return (unsigned)th_.size(); }
    void copy(uint8_t* d, const uint8_t* s, size_t n, size_t parts) {
        const size_t per = ((n + parts - 1) / parts + 63) & ~(size_t)63;
        State st;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (size_t o = per; o < n; o += per) {
                q_.push_back(Job{d + o, s + o, std::min(per, n - o), &st});
                st.left.fetch_add(1, std::memory_order_relaxed);
            }
        }
        cv_.notify_all();
        memcpy(d, s, std::min(per, n));
        while (st.left.load(std::memory_order_acquire) > 0) {
            Job j{};
            bool have = false;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!q_.empty()) {
                    j = q_.back();
                    q_.pop_back();
                    have = true;
                }
            }
            if (have) do_job(j);
            else std::this_thread::yield();
        }
    }

  private:
    static void do_job(const Job& j) {
        memcpy(j.d, j.s, j.n);
        j.st->left.fetch_sub(1, std::memory_order_release);
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                j = q_.back();
                q_.pop_back();
            }
            do_job(j);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Job> q_;
    bool stop_ = false;
};
CopyPool& copy_pool() {
    static CopyPool p(std::max(1u, std::min(7u, std::thread::hardware_concurrency() / 2)));
    return p;
}
}  // namespace

static void par_memcpy(void* dst, const void* src, size_t n) {
    constexpr size_t kPiece = 128u << 10;
    CopyPool& P = copy_pool();
    const size_t parts = std::min<size_t>(P.threads() + 1, n / kPiece);
    if (parts < 2) {
        memcpy(dst, src, n);
        return;
    }
    P.copy((uint8_t*)dst, (const uint8_t*)src, n, parts);
}

// Host <-> device copies of the host-buffer calls. A hipMemcpyAsync on pageable memory costs
// ~0.13 ms per call on this platform whatever its size (measured: 16 x 64 KiB D2H = 2.2 ms of a
// 2.6 ms 1 MiB decompress), so pageable caller buffers go through two pinned chunks: the DMA of
// one chunk overlaps the (multi-threaded) host copy of the other. Pinned caller buffers are
// copied directly.
static bool host_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error: clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}
// outputs up to this size come back in the readback round trip (no second synchronisation)
static constexpr uint64_t kSpecBytes = 8u << 20;
struct HostStage {
    static constexpr size_t kChunk = 8u << 20;
    PinnedBuf buf[2];
    PinnedBuf small;  // per-block / per-frame results read back in one copy
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~HostStage() {
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    hipError_t init(size_t n) {
        hipError_t e = hipSuccess;
        for (int b = 0; b < 2; ++b) {
            if (!ev[b] && (e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming)) != hipSuccess) return e;
            if ((e = buf[b].ensure(std::min(n, kChunk))) != hipSuccess) return e;
        }
        return e;
    }
    // host src -> device dst (stream ordered; returns once src may be reused)
    hipError_t h2d(void* dst, const void* src, size_t n, hipStream_t st) {
        if (!n) return hipSuccess;
        if (host_pinned(src)) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
        hipError_t e = init(n);
        if (e != hipSuccess) return e;
        int b = 0;
        for (size_t o = 0; o < n; o += kChunk, b ^= 1) {
            const size_t k = std::min(kChunk, n - o);
            if ((e = hipEventSynchronize(ev[b])) != hipSuccess) return e;  // chunk b's last DMA is done
            par_memcpy(buf[b].p, (const uint8_t*)src + o, k);
            if ((e = hipMemcpyAsync((uint8_t*)dst + o, buf[b].p, k, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
            if ((e = hipEventRecord(ev[b], st)) != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // device runs (in order) -> contiguous host dst; returns when dst holds every byte
    hipError_t d2h(uint8_t* dst, const std::vector<std::pair<const uint8_t*, uint64_t>>& runs, hipStream_t st) {
        uint64_t n = 0;
        for (auto& r : runs) n += r.second;
        if (!n) return hipSuccess;
        hipError_t e;
        if (host_pinned(dst)) {
            uint64_t o = 0;
            for (auto& r : runs) {
                if (r.second && (e = hipMemcpyAsync(dst + o, r.first, r.second, hipMemcpyDeviceToHost, st)) != hipSuccess)
                    return e;
                o += r.second;
            }
            return hipStreamSynchronize(st);
        }
        if ((e = init(n)) != hipSuccess) return e;
        size_t ri = 0, rpos = 0;  // next run byte to stage
        int b = 0, pend = -1;
        uint64_t pend_off = 0, pend_len = 0;
        for (uint64_t o = 0; o < n; o += kChunk, b ^= 1) {
            const uint64_t k = std::min<uint64_t>(kChunk, n - o);
            for (uint64_t f = 0; f < k;) {  // the chunk's pieces of the runs
                while (runs[ri].second == rpos) { ++ri; rpos = 0; }
                const uint64_t take = std::min<uint64_t>(k - f, runs[ri].second - rpos);
                if ((e = hipMemcpyAsync(buf[b].p + f, runs[ri].first + rpos, take, hipMemcpyDeviceToHost, st)) != hipSuccess)
                    return e;
                f += take;
                rpos += take;
            }
            if ((e = hipEventRecord(ev[b], st)) != hipSuccess) return e;
            if (pend >= 0) {
                if ((e = hipEventSynchronize(ev[pend])) != hipSuccess) return e;
                par_memcpy(dst + pend_off, buf[pend].p, pend_len);
            }
            pend = b;
            pend_off = o;
            pend_len = k;
        }
        if ((e = hipEventSynchronize(ev[pend])) != hipSuccess) return e;
        par_memcpy(dst + pend_off, buf[pend].p, pend_len);
        return hipSuccess;
    }
};

// ------------------------------------------------- large-block decode scratch
// Caps of the large-block path (s3hc_lb.hip) for one decode launch. They only size scratch:
// a block beyond any cap is decoded by the one-wave decoder instead.
struct LbCaps {
    uint32_t lb = 0, chunks = 0;
    uint32_t min_limit = kLbMinLimit;
    uint32_t big_csize = 0xFFFFFFFFu;  // (LbArgs::big_csize)
    uint64_t outb = 0;  // decoded bytes of the candidate blocks, at most (sizes the spread execution)
    bool exact = false; // lb is the candidate count itself (host walk), not a bound (device plans)
    uint32_t nbig = 0;  // candidates of frames that allow more than 64 KiB (the spread ones; exact only)
    void add_block(uint32_t csize, uint32_t out_bound, uint32_t limit) {
        ++lb;
        chunks += (csize + kLbChunk - 1) / kLbChunk;
        if (limit > kLbwMinLimit) {
            ++nbig;
            outb += std::min<uint64_t>(out_bound, (uint64_t)kLbMaxSteps * kLbStep);
        }
    }
};
static bool lb_candidate(const DecBlock& D, bool unit_single, uint32_t min_limit, uint32_t big_csize = 0xFFFFFFFFu) {
    return unit_single && !(D.flags & (DB_STORED | DB_LINKED)) && (D.limit >= min_limit || D.csize > big_csize) &&
           D.csize > 0 &&
           D.limit <= kLbMaxSteps * kLbStep;
}

struct LbScratch {
    DevBuf lbt, ctl, unit_lb, chunk_blk, nzg, E, J0, entry, trec, ntok, slsum, badrel, tokbase, outbase, total, seq4,
        seqoff, lb_err, lb_size, lb_stat, lb_tok0, lb_ntok, rfirst, blk_hash, wbase, wtile0, wP, tpend, tinit;
    LbArgs a{};
    // 64 KiB-block fast path (s3hc_fast.hip): per-unit token bitmaps and results
    DevBuf f_bmp, f_fu, f_unit_fast;  // (f_bmp: sequence records)
    DevBuf f_hash;                     // launches without the large-block path: per-block hashes (FastArgs::bh)
    FastArgs fa{};
    bool fast_ready = false;
    // small launch (host-walked, <= kLbFewBlocks blocks): 64 KiB blocks run the fused k_dsmall
    // (token index + executor + content xxh32 in one workgroup per block) instead of the
    // large-block chain; set by small_caps()
    bool small = false;
    // tok_entries: the launch's token-slot entries (DecBlock::tok + tok_slot_entries(csize) of
    // every block stays below it; sized by compressed bytes, not by a per-unit maximum)
    // maxc: the largest compressed block the launch may hand the fast path (sizes k_dtok's LDS)
    // nblocks: the launch's DecBlock count (block hashes are per DecBlock)
    hipError_t prepare_fast(uint32_t nunits, uint32_t nblocks, uint64_t tok_entries, uint64_t maxc) {
        fast_ready = false;
        fa.maxc = (uint32_t)std::min<uint64_t>(maxc, kFastMaxC);
        fa.bh = nullptr;
        if (!nunits || tok_entries > 0xFFFFFFF0ull) return hipSuccess;  // (u32 slots: the fast path sits out)
        hipError_t e;
        if ((e = f_bmp.ensure((size_t)tok_entries * sizeof(uint2) + 256)) != hipSuccess) return e;
        if ((e = f_fu.ensure((size_t)nunits * sizeof(FastUnit) + 64)) != hipSuccess) return e;
        if ((e = f_unit_fast.ensure((size_t)nunits + 64)) != hipSuccess) return e;
        if ((e = f_hash.ensure((size_t)std::max(nunits, nblocks) * 8 + 64)) != hipSuccess) return e;
        fa.rec = f_bmp.as<uint2>();
        fa.fu = f_fu.as<FastUnit>();
        fa.unit_fast = f_unit_fast.as<uint8_t>();
        fast_ready = true;
        return hipSuccess;
    }
    bool active = false;
    bool all_lb = false;  // every unit of the launch is a taken large block (host walks know): no unit decoder launch
    // nunits: units of the launch; nblocks: its DecBlock count (block hashes are per DecBlock)
    hipError_t prepare(uint32_t nunits, uint32_t nblocks, const LbCaps& c) {
        active = c.lb > 0 && c.chunks > 0;
        all_lb = active && c.exact && c.lb == nunits;  // (the caps equal the counts: every candidate is taken)
        if (!active) return hipSuccess;
        const size_t nch = c.chunks, nlb = c.lb;
        const size_t nseq = nch * kLbTokSlot;
        hipError_t e = hipSuccess;
#define LBE(buf, bytes) if ((e = (buf).ensure((size_t)(bytes) + 64)) != hipSuccess) return e;
        LBE(lbt, nlb * sizeof(LbBlock)) LBE(ctl, sizeof(LbCtl)) LBE(unit_lb, nunits) LBE(chunk_blk, nch * 4)
        LBE(nzg, nch * (kLbChunk / 64) * 4) LBE(E, nch * kLbEPerChunk * 4) LBE(J0, nch * kLbJ0PerChunk * 2) LBE(entry, nch * 4)
        LBE(trec, nch * kLbTokSlot * 16) LBE(ntok, nch * 4) LBE(slsum, nch * 4) LBE(badrel, nch * 4)
        LBE(tokbase, nch * 8) LBE(outbase, nch * 8) LBE(total, 32) LBE(seq4, nseq * 16) LBE(seqoff, nseq * 2)
        LBE(lb_err, nlb * 4) LBE(lb_size, nlb * 4) LBE(lb_stat, nlb * 4) LBE(lb_tok0, nlb * 4) LBE(lb_ntok, nlb * 4)
        LBE(rfirst, nlb * kLbMaxSteps * 4) LBE(blk_hash, (size_t)std::max(nunits, nblocks) * 8)
        // spread execution (few blocks, §4b): P holds one u32 per decoded byte of the spread blocks;
        // S3HC_LBW_CAP (positions, 0 = off; tests split a launch with it) replaces the size rule,
        // S3HC_LBW_DISABLE=1 turns it off
        uint64_t wcap = c.outb <= kLbwMaxOut ? c.outb : 0;
        if (knob(KN_LBW_CAP) >= 0) wcap = std::min<uint64_t>(c.outb, (uint64_t)knob(KN_LBW_CAP));
        // (a host walk knows its candidates: no spread launches that would find nothing to do)
        if (knob_on(KN_LBW_DISABLE) || (c.exact && (c.nbig == 0 || c.nbig > kLbwMaxBlocks))) wcap = 0;
        wcap = std::min<uint64_t>(wcap, kLbwCapMax);
        const size_t tcap = wcap ? wcap / kLbStep + nlb + 1 : 0;
        if (wcap) {
            LBE(wbase, nlb * 4) LBE(wtile0, nlb * 4) LBE(wP, wcap * 4) LBE(tpend, tcap) LBE(tinit, tcap)
        }
#undef LBE
        a.lb_cap = c.lb;
        a.chunk_cap = c.chunks;
        a.min_limit = c.min_limit;
        a.big_csize = c.big_csize;
        a.lbt = lbt.as<LbBlock>(); a.ctl = ctl.as<LbCtl>(); a.unit_lb = unit_lb.as<uint8_t>();
        a.chunk_blk = chunk_blk.as<uint32_t>(); a.nzg = nzg.as<uint32_t>(); a.E = E.as<uint32_t>(); a.J0 = J0.as<uint16_t>();
        a.entry = entry.as<uint32_t>(); a.trec = trec.as<uint4>(); a.ntok = ntok.as<uint32_t>();
        a.slsum = slsum.as<uint32_t>(); a.badrel = badrel.as<uint32_t>(); a.tokbase = tokbase.as<uint64_t>();
        a.outbase = outbase.as<uint64_t>(); a.total = total.as<uint64_t>(); a.seq4 = seq4.as<uint4>();
        a.seqoff = seqoff.as<uint16_t>(); a.lb_err = lb_err.as<uint32_t>(); a.lb_size = lb_size.as<uint32_t>();
        a.lb_stat = lb_stat.as<uint32_t>(); a.lb_tok0 = lb_tok0.as<uint32_t>(); a.lb_ntok = lb_ntok.as<uint32_t>();
        a.rfirst = rfirst.as<uint32_t>();
        a.blk_hash = blk_hash.as<uint64_t>();
        a.wcap = (uint32_t)wcap;
        a.tile_cap = (uint32_t)tcap;
        // every taken block spreads when the candidates (an upper bound) are few enough and their
        // decoded bytes (an upper bound) fit P (k_lbw_plan's rule)
        a.all_spread = wcap && c.exact && c.nbig == c.lb && c.nbig <= kLbwMaxBlocks && c.outb <= wcap ? 1u : 0u;
        a.wbase = wcap ? wbase.as<uint32_t>() : nullptr;
        a.wtile0 = wcap ? wtile0.as<uint32_t>() : nullptr;
        a.P = wcap ? wP.as<uint32_t>() : nullptr;
        a.tpend = wcap ? tpend.as<uint8_t>() : nullptr;
        a.tinit = wcap ? tinit.as<uint8_t>() : nullptr;
        return hipSuccess;
    }
};

static uint64_t max_csize(const DecBlock* b, size_t n) {
    uint64_t m = 0;
    for (size_t i = 0; i < n; ++i) m = std::max<uint64_t>(m, b[i].csize);
    return m;
}

// Sequence-record slots of host-built block tables: consecutive per block, sized by compressed
// bytes (s3hc_plan.hpp tok_slot_entries), each starting on a 128-byte line (16 records): k_dsmall
// writes a block's records and reads them back in the same launch, so no two blocks may share a
// cache line. Returns the launch's entries.
static uint64_t assign_tok_slots(DecBlock* b, size_t n) {
    uint64_t t = 0;
    for (size_t i = 0; i < n; ++i) {
        b[i].tok = (uint32_t)std::min<uint64_t>(t, 0xFFFFFFFFull);
        t += (tok_slot_entries(b[i].csize) + 15u) & ~15ull;
    }
    return t;
}

// Scratch and routing of a host-walked decode launch. Small launches (<= kLbFewBlocks blocks):
// with the fast path on, 64 KiB blocks it can take run k_dsmall (one fused launch); every other
// compressed block (frames allowing more than 64 KiB, blocks above kFastMaxC compressed bytes)
// runs the large-block path. Without the fast path every compressed block of a small launch
// takes the large-block path (many workgroups per block). Larger launches: large blocks only.
static hipError_t prepare_host_launch(LbScratch& L, const DecBlock* blocks, size_t nb, const DecUnit* units,
                                      uint32_t nu, uint64_t tok_entries) {
    LbCaps lc;
    lc.exact = true;
    const bool few = nb <= kLbFewBlocks;
    const bool small = few && !knob_on(KN_FAST_DISABLE) && !knob_on(KN_LB_DISABLE);
    if (small) lc.big_csize = kFastMaxC;
    else if (few) lc.min_limit = 1;  // few blocks: all of them on many workgroups
    for (uint32_t k = 0; k < nu; ++k) {
        const DecBlock& D = blocks[units[k].first];
        if (lb_candidate(D, units[k].n == 1, lc.min_limit, lc.big_csize))
            lc.add_block(D.csize, std::min(D.limit, D.cap), D.limit);
    }
    hipError_t e;
    if ((e = L.prepare(nu, (uint32_t)nb, lc)) != hipSuccess) return e;
    if ((e = L.prepare_fast(nu, (uint32_t)nb, tok_entries, max_csize(blocks, nb))) != hipSuccess) return e;
    L.small = small && L.fast_ready;
    return hipSuccess;
}

// The 64 KiB-block fast path (k_dtok + k_dexec) is on by default; the knob
// KN_FAST_DISABLE (S3HC_FAST=0 / S3HC_FAST_DISABLE=1) leaves every unit to the per-unit decoder
// (A/B runs, parity tests).
static bool fast_path_enabled() { return !knob_on(KN_FAST_DISABLE); }

// Block decode of a batch: large blocks by the large-block path (when L is active), the rest
// one wave per unit. *blk_hash: the large-block path's per-block output hashes (single-block
// units: 1 << 32 | xxh32, or 0), nullptr when the path did not run.
// Plans walked on the device pass ucount (the frame walk's block total: the units' count) and
// size the per-unit grids to their frames; host-walked plans know their units exactly.
// The caller closes the frames (k_dframe_close) after it.
static hipError_t decode_launch(LbScratch* L, const uint8_t* src, uint8_t* dst, const DecBlock* blk,
                                const DecUnit* units, uint32_t nunits, uint32_t* blk_out, int32_t* blk_status,
                                hipStream_t st, const uint64_t** blk_hash = nullptr, const uint64_t* ucount = nullptr,
                                uint32_t grid = 0) {
    if (!grid || grid > nunits) grid = nunits;
    // S3HC_LB_DISABLE (tests, comparisons): every block goes to the one-wave decoder
    const bool lb = L && L->active && nunits && !knob_on(KN_LB_DISABLE);
    if (blk_hash) *blk_hash = lb ? L->a.blk_hash : nullptr;
    hipError_t e;
    if (lb && (e = launch_lb_parse(L->a, src, blk, units, nunits, ucount, blk_out, blk_status, st)) != hipSuccess) return e;
    // 64 KiB blocks: token index + executor (S3HC_FAST_DISABLE=1: every block on the per-unit
    // decoder, for comparisons); blocks the fast path leaves go to the per-unit decoder below
    const bool fast = L && L->fast_ready && L->fa.maxc && nunits && !(lb && L->all_lb) && fast_path_enabled();
    if (fast && (L->small || fast_exec_hashes())) {
        // the executors hash their output (the frame close takes those hashes, like the
        // large-block path's: one array, the large-block path zeroes it for every single-block
        // unit, the fast path sets its own and zeroes those it leaves when the other path is off)
        L->fa.bh = lb ? L->a.blk_hash : L->f_hash.as<uint64_t>();
        if (blk_hash) *blk_hash = L->fa.bh;
    } else {
        L->fa.bh = nullptr;
    }
    if (fast && L->small) {
        // small host-walked launch: token index + block decode + content xxh32 in one launch; without
        // large blocks it also runs the per-unit decoder for the blocks it leaves (no second launch)
        bool owned = false;
        if ((e = launch_fast_small(src, dst, blk, units, nunits, lb ? L->a.unit_lb : nullptr, L->fa, blk_out,
                                   blk_status, st, !lb, &owned)) != hipSuccess)
            return e;
        if (owned) return hipSuccess;
    } else if (fast) {
        if ((e = launch_fast_tok(src, blk, units, nunits, ucount, grid, lb ? L->a.unit_lb : nullptr, L->fa, st)) !=
            hipSuccess)
            return e;
        if ((e = launch_fast_exec(src, dst, blk, units, nunits, ucount, grid, blk_out, blk_status, L->fa, st)) !=
            hipSuccess)
            return e;
        if (knob_on(KN_FAST_TRACE)) {  // diagnostics (serialises the stream): units the fast path took
            uint64_t nu = nunits;
            if (ucount && (e = hipMemcpyAsync(&nu, ucount, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            nu = std::min<uint64_t>(nu, nunits);
            std::vector<uint8_t> f(nu + 1);
            std::vector<FastUnit> fu(nu + 1);
            if ((e = hipMemcpyAsync(f.data(), L->fa.unit_fast, nu, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipMemcpyAsync(fu.data(), L->fa.fu, nu * sizeof(FastUnit), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            uint32_t k = 0;
            uint64_t ntok = 0;
            for (uint64_t i = 0; i < nu; ++i)
                if (f[i]) { ++k; ntok += fu[i].ntok; }
            fprintf(stderr, "[s3hc fast] units %llu taken %u tokens %llu grid %u\n", (unsigned long long)nu, k,
                    (unsigned long long)ntok, grid);
        }
    }
    if (!(lb && L->all_lb) &&
        (e = launch_decode_units(src, dst, blk, units, nunits, ucount, grid, blk_out, blk_status,
                                 lb ? L->a.unit_lb : nullptr, fast ? L->fa.unit_fast : nullptr, st)) != hipSuccess)
        return e;
    if (lb && (e = launch_lb_exec(L->a, src, dst, blk_out, blk_status, st)) != hipSuccess) return e;
    if (lb && knob_on(KN_LB_TRACE)) {  // diagnostics (serialises the stream): blocks and chunks taken
        LbCtl c;
        if ((e = hipMemcpyAsync(&c, L->a.ctl, sizeof c, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        fprintf(stderr, "[s3hc lb] blocks %u chunks %u spread tiles %u pending tiles per round", c.nlb, c.nchunks,
                c.ntiles);
        for (uint32_t r = 0; r <= kLbwRounds; ++r) fprintf(stderr, " %u", c.rflag[r]);
        fprintf(stderr, "\n");
    }
    return hipSuccess;
}

// --------------------------------------------------------------- context
struct TimedSpan {
    std::string name;
    hipEvent_t a, b;
    bool shared_a;  // a is the previous span's b (returned to the pool once, with that span)
};
struct s3hc_ctx {
    // references: the creator's (s3hc_destroy drops it) and one per reader / aggregator built on
    // the context, so a context destroyed while they live is freed when the last one closes
    std::atomic<int> refs{1};
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    int timing = 0;  // 0 off, 1 every phase, 2 coarse (enc_parse, dec_all)
    int enc_mode = S3HC_ENC_FAST;  // match-finder mode of this context's encodes
    std::map<std::string, float> kernel_ms;
    std::map<std::string, int> kernel_n;
    std::vector<TimedSpan> pending;
    std::vector<hipEvent_t> event_pool;
    hipEvent_t take_event() {
        if (event_pool.empty()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            return e;
        }
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    // scratch for host-buffer calls
    DevBuf d_in, d_out;
    s3hc_plan* host_plan = nullptr;
    DevBuf d_blocks, d_units, d_blk_out, d_blk_status, d_rng_off, d_rng_len, d_hash;
    DevBuf d_c_soff, d_c_len, d_c_doff, d_c_hash, d_c_flen;  // compat encoder descriptors
    DevBuf d_ftab, d_fstat, d_flen, d_fhash;                  // per-frame tables of decode_walk
    HostStage hs;
    LbScratch lb;
    // range-reader resources kept warm between the readers of this context (s3hc_reader_*): one
    // reader per GET (stream_range_data) would otherwise allocate its pinned and device buffers,
    // HIP queues and events on every open
    std::mutex rpool_mu;
    std::vector<void*> rslot_pool;         // RSlot* (reader section)
    std::vector<hipStream_t> rqueue_pool;  // non-blocking queues of this device
    std::vector<void*> rin_pool;           // PinnedBuf* (readers' input buffers)
    ~s3hc_ctx();
};
static void reader_pool_release(s3hc_ctx* ctx);

// Per-kernel event timing (s3hc_set_timing). Events come from a pool and are only resolved
// by s3hc_timing_collect(), so timing adds no host synchronisation inside a timed region.
// Adjacent phases of one call share their boundary event (a phase that begins right where the
// previous one ended reuses its end event): every event record on the stream is a dispatch
// boundary the command processor waits at, so fewer records perturb the timed region less.
struct KTimer {
    s3hc_ctx* ctx;
    hipStream_t st;
    bool adjacent = false;  // the last call was end(): nothing was enqueued since
    explicit KTimer(s3hc_ctx* c, hipStream_t s) : ctx(c), st(s) {}
    bool fine() const;      // every phase its own span (s3hc_set_timing 1), else the coarse spans (2)
    void begin(const char* name);
    void end();
};
// ------------------------------------------------------------------ plans
struct s3hc_plan {
    bool is_encode = true;
    // ---- encode
    std::vector<EncBlock> blocks;
    std::vector<uint32_t> seg_block;
    std::vector<uint2> groups;           // match-finding workgroups: (block, first segment)
    std::vector<uint32_t> frame_blk0, frame_nblk;
    std::vector<uint64_t> frame_src_off;
    std::vector<uint32_t> frame_src_len;
    std::vector<uint32_t> item_blk0, item_nblk;
    uint64_t dst_bound = 0;
    DevBuf d_groups, d_blocks, d_seg_block, d_frame_src_off, d_frame_src_len, d_item_blk0, d_item_nblk;
    DevBuf d_recs, d_summ, d_place, d_blk_payload, d_blk_size, d_blk_carry, d_blk_off, d_frame_hash, d_total;
    // ---- decode
    uint32_t nframes = 0;
    uint32_t blk_cap = 0;
    uint32_t dec_grid = 1;  // per-unit decode workgroups (one per 64 KiB of frame room, <= blk_cap)
    DevBuf d_frame_off, d_frame_len, d_dst_off, d_dst_cap, d_ftok;
    DevBuf d_nblk, d_fstatus, d_blk_base, d_fwant, d_dblocks, d_units, d_blk_out, d_blk_status, d_got;
    LbScratch lb;                        // large-block path scratch (frames allowing > 64 KiB blocks)
};

bool KTimer::fine() const { return ctx->timing != 2; }
void KTimer::begin(const char* name) {
    if (!ctx->timing) return;
    if (adjacent && !ctx->pending.empty()) {
        // this phase starts where the previous one ended: its start is that end event (a shared
        // event is never handed back to the pool twice: the span marks it as borrowed)
        TimedSpan t{name, ctx->pending.back().b, ctx->take_event(), true};
        ctx->pending.push_back(t);
    } else {
        TimedSpan t{name, ctx->take_event(), ctx->take_event(), false};
        (void)hipEventRecord(t.a, st);
        ctx->pending.push_back(t);
    }
    adjacent = false;
}
void KTimer::end() {
    if (!ctx->timing || ctx->pending.empty()) return;
    (void)hipEventRecord(ctx->pending.back().b, st);
    adjacent = true;
}

s3hc_ctx::~s3hc_ctx() {
    for (auto& t : pending) {
        if (!t.shared_a) (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : event_pool) (void)hipEventDestroy(e);
    delete host_plan;
    if (stream) (void)hipStreamDestroy(stream);
}

// Frame layout of one item (lz4_flex FrameEncoder Auto / 64K-per-frame / store mode).
static void plan_item(s3hc_plan* P, uint64_t off, uint64_t len, int mode, int policy) {
    P->item_blk0.push_back((uint32_t)P->blocks.size());
    auto add_frame = [&](uint64_t foff, uint64_t flen, uint8_t bd, uint64_t bmax, bool store) {
        const uint32_t f = (uint32_t)P->frame_blk0.size();
        P->frame_blk0.push_back((uint32_t)P->blocks.size());
        P->frame_src_off.push_back(foff);
        P->frame_src_len.push_back((uint32_t)flen);
        const uint8_t hc = header_hc(bd);
        uint32_t nb = 0;
        if (flen == 0) {
            EncBlock B{};
            B.src_off = foff;
            B.len = 0;
            B.seg0 = (uint32_t)P->seg_block.size();
            B.nseg = 1;
            B.frame = f;
            B.flags = EB_FIRST | EB_LAST | EB_EMPTY;
            B.bd = bd;
            B.hc = hc;
            P->seg_block.push_back((uint32_t)P->blocks.size());
            P->blocks.push_back(B);
            P->dst_bound += 15;
            nb = 1;
        } else {
            for (uint64_t o = 0; o < flen; o += bmax, ++nb) {
                EncBlock B{};
                B.src_off = foff + o;
                B.len = (uint32_t)std::min<uint64_t>(bmax, flen - o);
                B.seg0 = (uint32_t)P->seg_block.size();
                B.nseg = (B.len + kSeg - 1) / kSeg;
                B.frame = f;
                B.flags = (o == 0 ? EB_FIRST : 0u) | (o + bmax >= flen ? EB_LAST : 0u) | (store ? EB_STORE : 0u);
                B.bd = bd;
                B.hc = hc;
                for (uint32_t s = 0; s < B.nseg; ++s) P->seg_block.push_back((uint32_t)P->blocks.size());
                P->blocks.push_back(B);
                P->dst_bound += 4 + B.len;
            }
            P->dst_bound += 15;
        }
        P->frame_nblk.push_back(nb);
    };
    if (mode == 1) {  // store-mode frame: BD 0x70, stored blocks <= 4 MiB (compression.rs:326-368)
        add_frame(off, len, 0x70, kStoreModeBlock, true);
    } else if (policy == S3HC_BLK_64K_PER_FRAME) {
        if (len == 0) add_frame(off, 0, 0x40, 65536, false);
        for (uint64_t o = 0; o < len; o += 65536) add_frame(off + o, std::min<uint64_t>(65536, len - o), 0x40, 65536, false);
    } else {  // BlockSize::from_buf_length
        const uint8_t bd = len <= 65536 ? 0x40 : (len <= 262144 ? 0x50 : 0x70);
        const uint64_t bmax = len <= 65536 ? 65536 : (len <= 262144 ? 262144 : (4u << 20));
        add_frame(off, len, bd, bmax, false);
    }
    P->item_nblk.push_back((uint32_t)P->blocks.size() - P->item_blk0.back());
}

static int plan_upload_encode(s3hc_plan* P, hipStream_t st) {
    const size_t nseg = P->seg_block.size(), nb = P->blocks.size(), nf = P->frame_blk0.size();
    HIPCHK(upload(P->d_blocks, P->blocks, st));
    HIPCHK(upload(P->d_seg_block, P->seg_block, st));
    P->groups.clear();
    for (uint32_t b = 0; b < (uint32_t)P->blocks.size(); ++b) {
        const EncBlock& B = P->blocks[b];
        if (B.flags & (EB_STORE | EB_EMPTY)) continue;  // nothing to match
        for (uint32_t k = 0; k < B.nseg; k += kGroupSegs) P->groups.push_back(make_uint2(b, k));
    }
    HIPCHK(upload(P->d_groups, P->groups, st));
    HIPCHK(upload(P->d_frame_src_off, P->frame_src_off, st));
    HIPCHK(upload(P->d_frame_src_len, P->frame_src_len, st));
    HIPCHK(upload(P->d_item_blk0, P->item_blk0, st));
    HIPCHK(upload(P->d_item_nblk, P->item_nblk, st));
    HIPCHK(P->d_recs.ensure(nseg * kMaxSeqPerSeg * sizeof(uint2)));
    HIPCHK(P->d_summ.ensure(nseg * sizeof(SegSummary)));
    HIPCHK(P->d_place.ensure(nseg * sizeof(SegPlace)));
    HIPCHK(P->d_blk_payload.ensure(nb * 4));
    HIPCHK(P->d_blk_size.ensure(nb * 4));
    HIPCHK(P->d_blk_carry.ensure(nb * 4));
    HIPCHK(P->d_blk_off.ensure(nb * 8));
    HIPCHK(P->d_frame_hash.ensure(nf * 4));
    HIPCHK(P->d_total.ensure(8));
    return S3HC_OK;
}

static int run_encode(s3hc_ctx* ctx, s3hc_plan* P, const uint8_t* d_src, uint8_t* d_dst, uint64_t* d_item_off,
                      uint32_t* d_item_len, hipStream_t st) {
    const uint32_t nseg = (uint32_t)P->seg_block.size(), nb = (uint32_t)P->blocks.size();
    const uint32_t nf = (uint32_t)P->frame_blk0.size(), ni = (uint32_t)P->item_blk0.size();
    KTimer T(ctx, st);
    // match finding; the grid's first workgroups compute the frames' content xxh32 meanwhile
    // (measured round 6: the same hash as its own launch on a second queue beside the finder
    // slowed the finder as much as the in-grid workgroups do — the cost is issue, not LDS slots)
    T.begin("enc_parse");
    HIPCHK(launch_enc_parse(d_src, P->d_blocks.as<EncBlock>(), P->d_groups.as<uint2>(), (uint32_t)P->groups.size(),
                            P->d_frame_src_off.as<uint64_t>(), P->d_frame_src_len.as<uint32_t>(), nf,
                            P->d_frame_hash.as<uint32_t>(), P->d_recs.as<uint2>(), P->d_summ.as<SegSummary>(), ctx->enc_mode, st));
    T.end();
    const bool fine = T.fine();
    if (fine) T.begin("enc_sizes");
    HIPCHK(launch_enc_sizes(P->d_blocks.as<EncBlock>(), nb, P->d_summ.as<SegSummary>(), P->d_place.as<SegPlace>(),
                            P->d_blk_payload.as<uint32_t>(), P->d_blk_size.as<uint32_t>(),
                            P->d_blk_carry.as<uint32_t>(), st));
    HIPCHK(launch_scan(P->d_blk_size.as<uint32_t>(), nb, P->d_blk_off.as<uint64_t>(), P->d_total.as<uint64_t>(), st));
    if (fine) {
        T.end();
        T.begin("enc_emit");
    }
    HIPCHK(launch_enc_emit(d_src, P->d_blocks.as<EncBlock>(), P->d_seg_block.as<uint32_t>(), nseg,
                           P->d_recs.as<uint2>(), P->d_summ.as<SegSummary>(), P->d_place.as<SegPlace>(),
                           P->d_blk_payload.as<uint32_t>(), P->d_blk_carry.as<uint32_t>(),
                           P->d_blk_off.as<uint64_t>(), P->d_frame_hash.as<uint32_t>(), d_dst, st));
    HIPCHK(launch_enc_groups(P->d_item_blk0.as<uint32_t>(), P->d_item_nblk.as<uint32_t>(), ni,
                             P->d_blk_off.as<uint64_t>(), P->d_blk_size.as<uint32_t>(), d_item_off, d_item_len, st));
    if (fine) T.end();
    return S3HC_OK;
}

// ------------------------------------------------------------ knobs (s3hc_knobs.hpp)
namespace s3hc {
std::atomic<long long> g_knob[KN_COUNT];
namespace {
struct KnobName {
    const char* name;
    Knob k;
    long long dflt;
};
constexpr KnobName kKnobNames[] = {
    {"S3HC_FAST_DISABLE", KN_FAST_DISABLE, 0}, {"S3HC_LB_DISABLE", KN_LB_DISABLE, 0},
    {"S3HC_LBW_DISABLE", KN_LBW_DISABLE, 0},   {"S3HC_LBW_CAP", KN_LBW_CAP, -1},
    {"S3HC_LBW_ROUNDS", KN_LBW_ROUNDS, -1},
#if S3HC_DIAG_VARIANTS
    {"S3HC_DEC_ONEWAVE", KN_DEC_ONEWAVE, 0},
#endif
    {"S3HC_FAST_TRACE", KN_FAST_TRACE, 0},     {"S3HC_LB_TRACE", KN_LB_TRACE, 0},
    {"S3HC_HOST_TRACE", KN_HOST_TRACE, 0},     {"S3HC_READER_SLOTS", KN_READER_SLOTS, 1},
    {"S3HC_POISON", KN_POISON, 0},
};
// the slot a name reads and writes (S3HC_FAST: the other spelling of S3HC_FAST_DISABLE)
int knob_slot(const char* name) {
    if (!strcmp(name, "S3HC_FAST")) return KN_FAST_DISABLE;
    for (const auto& n : kKnobNames)
        if (!strcmp(n.name, name)) return n.k;
    return -1;
}
// a flag knob is on when its variable is set at all (the env convention of earlier rounds);
// the numeric ones take the value
long long knob_value(const KnobName& n, const char* v) {
    if (!v) return n.dflt;
    if (n.k == KN_LBW_CAP || n.k == KN_LBW_ROUNDS || n.k == KN_READER_SLOTS) return strtoll(v, nullptr, 10);
    return 1;
}
int knob_set(const char* name, const char* v) {
    if (!strcmp(name, "S3HC_FAST")) {  // S3HC_FAST=0 is the other spelling of S3HC_FAST_DISABLE=1
        g_knob[KN_FAST_DISABLE].store(v && v[0] == '0' ? 1 : 0, std::memory_order_relaxed);
        return S3HC_OK;
    }
    for (const auto& n : kKnobNames)
        if (!strcmp(n.name, name)) {
            g_knob[n.k].store(knob_value(n, v), std::memory_order_relaxed);
            return S3HC_OK;
        }
    return S3HC_INVALID_ARG;
}
std::once_flag g_knob_once;
}  // namespace
void knobs_load_env_once() {
    std::call_once(g_knob_once, [] {
        for (const auto& n : kKnobNames) g_knob[n.k].store(knob_value(n, getenv(n.name)), std::memory_order_relaxed);
        const char* f = getenv("S3HC_FAST");
        if (f && f[0] == '0') g_knob[KN_FAST_DISABLE].store(1, std::memory_order_relaxed);
    });
}
}  // namespace s3hc

extern "C" int s3hc_set_knob(const char* name, const char* value) {
    if (!name) return fail(S3HC_INVALID_ARG, "name is NULL");
    knobs_load_env_once();  // (a knob set before the first context keeps its value)
    if (knob_set(name, value) != S3HC_OK) return fail(S3HC_INVALID_ARG, "unknown knob");
    return S3HC_OK;
}
extern "C" int s3hc_get_knob(const char* name, long long* value) {
    if (!name || !value) return fail(S3HC_INVALID_ARG, "bad arguments");
    knobs_load_env_once();
    const int k = knob_slot(name);
    if (k < 0) return fail(S3HC_INVALID_ARG, "unknown knob");
    *value = g_knob[k].load(std::memory_order_relaxed);
    return S3HC_OK;
}
extern "C" int s3hc_set_knob_value(const char* name, long long value) {
    if (!name) return fail(S3HC_INVALID_ARG, "name is NULL");
    knobs_load_env_once();
    const int k = knob_slot(name);
    if (k < 0) return fail(S3HC_INVALID_ARG, "unknown knob");
    g_knob[k].store(value, std::memory_order_relaxed);
    return S3HC_OK;
}

// ------------------------------------------------------------ C ABI: ctx
extern "C" int s3hc_create(s3hc_ctx** out, int device) {
    return guarded([&]() -> int {
        if (!out) return fail(S3HC_INVALID_ARG, "out is NULL");
        *out = nullptr;
        knobs_load_env_once();
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess || n == 0) return fail(S3HC_DEVICE, "no HIP device available (the engine has no CPU path)");
        if (device < 0 || device >= n) return fail(S3HC_INVALID_ARG, "device index out of range");
        HIPCHK(hipSetDevice(device));
        std::unique_ptr<s3hc_ctx> c(new s3hc_ctx);
        c->device = device;
        HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        *out = c.release();
        return S3HC_OK;
    });
}
extern "C" int s3hc_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}
namespace s3hc {
void ctx_retain(s3hc_ctx* ctx) { ctx->refs.fetch_add(1, std::memory_order_relaxed); }
void ctx_release(s3hc_ctx* ctx) {
    if (ctx->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    reader_pool_release(ctx);
    delete ctx;
}
}  // namespace s3hc
extern "C" void s3hc_destroy(s3hc_ctx* ctx) {
    if (ctx) ctx_release(ctx);
}
extern "C" int s3hc_set_encode_mode(s3hc_ctx* ctx, int mode) {
    if (!ctx || (mode != S3HC_ENC_FAST && mode != S3HC_ENC_SMALL)) return fail(S3HC_INVALID_ARG, "bad arguments");
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->enc_mode = mode;
    return S3HC_OK;
}
extern "C" int s3hc_get_encode_mode(const s3hc_ctx* ctx) { return ctx ? ctx->enc_mode : -1; }
extern "C" void s3hc_set_timing(s3hc_ctx* ctx, int enabled) {
    if (ctx) ctx->timing = enabled == 2 ? 2 : (enabled != 0 ? 1 : 0);
}
// Resolve recorded spans into per-name totals (ms) and launch counts; clears the spans.
extern "C" int s3hc_timing_collect(s3hc_ctx* ctx) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        for (auto& t : ctx->pending) {
            HIPCHK(hipEventSynchronize(t.b));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, t.a, t.b));
            ctx->kernel_ms[t.name] += ms;
            ctx->kernel_n[t.name] += 1;
            if (!t.shared_a) ctx->event_pool.push_back(t.a);
            ctx->event_pool.push_back(t.b);
        }
        ctx->pending.clear();
        return S3HC_OK;
    });
}
extern "C" void s3hc_timing_reset(s3hc_ctx* ctx) {
    if (!ctx) return;
    s3hc_timing_collect(ctx);
    ctx->kernel_ms.clear();
    ctx->kernel_n.clear();
}
extern "C" float s3hc_last_kernel_ms(const s3hc_ctx* ctx, const char* name) {
    if (!ctx || !name) return -1.f;
    auto it = ctx->kernel_ms.find(name);
    return it == ctx->kernel_ms.end() ? -1.f : it->second;
}
extern "C" int s3hc_kernel_count(const s3hc_ctx* ctx, const char* name) {
    return guarded([&]() -> int {
        if (!ctx || !name) return 0;
        auto it = ctx->kernel_n.find(name);
        return it == ctx->kernel_n.end() ? 0 : it->second;
    });
}

extern "C" size_t s3hc_frame_bound(size_t n) {
    // 64 KiB frames (header 7 + word 4 + trailer 8 per 64 KiB) bound every layout we write.
    return n + 19 * (n / 65536 + 1) + 16;
}

// ------------------------------------------------------ C ABI: batch encode
extern "C" int s3hc_plan_encode(s3hc_ctx* ctx, const uint64_t* src_off, const uint32_t* len, const uint8_t* mode,
                                uint32_t n, s3hc_plan** out) {
    return guarded([&]() -> int {
        if (!ctx || !out || (n && (!src_off || !len))) return fail(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        std::unique_ptr<s3hc_plan> P(new s3hc_plan);
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t m = mode ? mode[i] : 0;
            if (m > 2) return fail(S3HC_INVALID_ARG, "mode must be 0, 1 or 2");
            plan_item(P.get(), src_off[i], len[i], m == 1 ? 1 : 0, m == 2 ? S3HC_BLK_64K_PER_FRAME : S3HC_BLK_AUTO_LZ4FLEX);
        }
        int rc = plan_upload_encode(P.get(), ctx->stream);
        if (rc) return rc;
        HIPCHK(hipStreamSynchronize(ctx->stream));
        *out = P.release();
        return S3HC_OK;
    });
}
extern "C" uint64_t s3hc_plan_dst_bound(const s3hc_plan* P) { return P ? P->dst_bound : 0; }
extern "C" void s3hc_plan_free(s3hc_plan* P) { delete P; }

extern "C" int s3hc_encode_dev(s3hc_ctx* ctx, s3hc_plan* P, const uint8_t* d_src, uint8_t* d_dst, uint64_t dst_cap,
                               uint64_t* d_item_off, uint32_t* d_item_len, void* stream) {
    return guarded([&]() -> int {
        if (!ctx || !P || !P->is_encode || !d_item_off || !d_item_len) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (dst_cap < P->dst_bound) return fail(S3HC_DST_TOO_SMALL, "dst_cap < s3hc_plan_dst_bound(plan)");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
        return run_encode(ctx, P, d_src, d_dst, d_item_off, d_item_len, st);
    });
}

// ------------------------------------------------------ C ABI: batch decode
extern "C" int s3hc_plan_decode(s3hc_ctx* ctx, const uint64_t* frame_off, const uint32_t* frame_len,
                                const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t n, s3hc_plan** out) {
    return guarded([&]() -> int {
        if (!ctx || !out || (n && (!frame_off || !frame_len || !dst_off || !dst_cap)))
            return fail(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        std::unique_ptr<s3hc_plan> P(new s3hc_plan);
        P->is_encode = false;
        P->nframes = n;
        uint64_t cap = 0;
        for (uint32_t i = 0; i < n; ++i) cap += dst_cap[i] / 65536u + 2u;
        if (cap > 0xFFFFFFF0ull) return fail(S3HC_INVALID_ARG, "batch too large");
        P->blk_cap = (uint32_t)cap;
        hipStream_t st = ctx->stream;
        std::vector<uint64_t> fo(frame_off, frame_off + n), d(dst_off, dst_off + n);
        std::vector<uint32_t> fl(frame_len, frame_len + n), dc(dst_cap, dst_cap + n);
        // token-position slots per frame (tok_frame_entries) and the per-unit grid: one workgroup
        // per 64 KiB of each frame's room (frames of several independent blocks keep their
        // parallelism; the grid still strides over any extra units)
        std::vector<uint64_t> ftok(n);
        uint64_t tok_entries = 0, grid = 0, max_frame_len = 0;
        for (uint32_t i = 0; i < n; ++i) {
            ftok[i] = tok_entries;
            max_frame_len = std::max<uint64_t>(max_frame_len, frame_len[i]);  // (a block is shorter than its frame)
            tok_entries += tok_frame_entries(frame_len[i]);
            grid += std::max<uint64_t>(1, (dst_cap[i] + 65535u) / 65536u);
        }
        P->dec_grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(grid, cap));
        HIPCHK(upload(P->d_frame_off, fo, st));
        HIPCHK(upload(P->d_frame_len, fl, st));
        HIPCHK(upload(P->d_ftok, ftok, st));
        HIPCHK(upload(P->d_dst_off, d, st));
        HIPCHK(upload(P->d_dst_cap, dc, st));
        HIPCHK(P->d_nblk.ensure(n * 4 + 16));
        HIPCHK(P->d_fstatus.ensure(n * 4 + 16));
        HIPCHK(P->d_blk_base.ensure(n * 8 + 16));
        HIPCHK(P->d_fwant.ensure(n * 4 + 16));
        HIPCHK(P->d_got.ensure(n * 4 + 16));
        HIPCHK(P->d_total.ensure(16));
        HIPCHK(P->d_dblocks.ensure((size_t)P->blk_cap * sizeof(DecBlock) + 16));
        HIPCHK(P->d_units.ensure((size_t)P->blk_cap * sizeof(DecUnit) + 16));
        HIPCHK(P->d_blk_out.ensure((size_t)P->blk_cap * 4 + 16));
        HIPCHK(P->d_blk_status.ensure((size_t)P->blk_cap * 4 + 16));
        // large blocks: the device walk finds them; frames with room for more than 64 KiB may hold
        // some (well-formed frames fill every block but the last, so <= cap / 256 KiB + 1 of them)
        LbCaps lc;
        if (n <= kLbFewBlocks / 4) {  // few frames: every compressed block takes the path
            lc.min_limit = 1;
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t nl = dst_cap[i] / 65536u + 1u;
                lc.lb += nl;
                lc.chunks += frame_len[i] / kLbChunk + nl;
                lc.outb += dst_cap[i];
            }
        } else {
            for (uint32_t i = 0; i < n; ++i) {
                if (dst_cap[i] <= 65536u) continue;
                const uint32_t nl = dst_cap[i] / 262144u + 1u;
                lc.lb += nl;
                lc.chunks += frame_len[i] / kLbChunk + nl;
                lc.outb += dst_cap[i];
            }
        }
        HIPCHK(P->lb.prepare(P->blk_cap, P->blk_cap, lc));
        HIPCHK(P->lb.prepare_fast(P->blk_cap, P->blk_cap, tok_entries, max_frame_len));
        P->lb.small = false;
        HIPCHK(hipStreamSynchronize(st));
        *out = P.release();
        return S3HC_OK;
    });
}

extern "C" int s3hc_decode_dev(s3hc_ctx* ctx, s3hc_plan* P, const uint8_t* d_src, uint8_t* d_dst, uint32_t* d_out_len,
                               int32_t* d_status, void* stream) {
    return guarded([&]() -> int {
        if (!ctx || !P || P->is_encode || !d_out_len || !d_status) return fail(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
        const uint32_t n = P->nframes;
        if (!n) return S3HC_OK;
        KTimer T(ctx, st);
        const bool fine = T.fine();
        T.begin(fine ? "dec_plan" : "dec_all");  // (coarse timing: the whole decode, one span)
        HIPCHK(launch_dframe_count(d_src, P->d_frame_off.as<uint64_t>(), P->d_frame_len.as<uint32_t>(),
                                   P->d_dst_cap.as<uint32_t>(), n, P->d_nblk.as<uint32_t>(), d_status, st));
        HIPCHK(launch_scan(P->d_nblk.as<uint32_t>(), n, P->d_blk_base.as<uint64_t>(), P->d_total.as<uint64_t>(), st));
        // (no clearing of the unit table: the per-unit kernels stop at the walk's block total)
        HIPCHK(launch_dframe_fill(d_src, P->d_frame_off.as<uint64_t>(), P->d_frame_len.as<uint32_t>(), n,
                                  P->d_dst_off.as<uint64_t>(), P->d_dst_cap.as<uint32_t>(), P->d_blk_base.as<uint64_t>(),
                                  d_status, P->d_dblocks.as<DecBlock>(), P->d_units.as<DecUnit>(),
                                  P->d_fwant.as<uint32_t>(), P->d_ftok.as<uint64_t>(), st));
        if (fine) {
            T.end();
            T.begin("decode");
        }
        const uint64_t* bh = nullptr;
        // one workgroup per frame (the common one block per frame: the exact unit count); frames of
        // several independent blocks have their extra units taken by a stride of the grid
        HIPCHK(decode_launch(&P->lb, d_src, d_dst, P->d_dblocks.as<DecBlock>(), P->d_units.as<DecUnit>(), P->blk_cap,
                             P->d_blk_out.as<uint32_t>(), P->d_blk_status.as<int32_t>(), st, &bh,
                             P->d_total.as<uint64_t>(), P->dec_grid));
        if (fine) {
            T.end();
            // frame results, content xxh32 and EndMark checks (one launch)
            T.begin("dec_close");
        }
        HIPCHK(launch_dframe_close(d_src, P->d_frame_off.as<uint64_t>(), P->d_blk_base.as<uint64_t>(),
                                   P->d_nblk.as<uint32_t>(), P->d_dblocks.as<DecBlock>(), P->d_blk_out.as<uint32_t>(),
                                   P->d_blk_status.as<int32_t>(), bh, d_dst, P->d_dst_off.as<uint64_t>(),
                                   P->d_fwant.as<uint32_t>(), n, d_status, d_status, d_out_len, nullptr, st));
        T.end();
        return S3HC_OK;
    });
}

// ------------------------------------------------- C ABI: host-buffer encode
static int host_encode(s3hc_ctx* ctx, const uint8_t* src, size_t n, int mode, int policy, uint8_t* dst, size_t cap,
                       size_t* out_len) {
    if (!ctx || (!src && n) || !out_len) return fail(S3HC_INVALID_ARG, "bad arguments");
    if (n > 0xFFFFFFFFull * 16) return fail(S3HC_INVALID_ARG, "input too large");
    std::lock_guard<std::mutex> g(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    s3hc_plan* P = new s3hc_plan;
    // items of <= 4 GiB (u32 lengths); each item is one frame (Auto) or 64 KiB frames
    const uint64_t item_max = (mode == 1 || policy == S3HC_BLK_64K_PER_FRAME) ? (1ull << 31) : (uint64_t)n;
    if (n == 0) plan_item(P, 0, 0, mode, policy);
    for (uint64_t o = 0; o < n; o += item_max) plan_item(P, o, std::min<uint64_t>(item_max, n - o), mode, policy);
    if (mode != 1 && policy != S3HC_BLK_64K_PER_FRAME && n > 0xFFFFFFFFull) {
        delete P;
        return fail(S3HC_INVALID_ARG, "single-frame input above 4 GiB");
    }
    std::unique_ptr<s3hc_plan> guard(P);
    if (cap < P->dst_bound) return fail(S3HC_DST_TOO_SMALL, "dst capacity below frame bound");
    int rc = plan_upload_encode(P, st);
    if (rc) return rc;
    HIPCHK(ctx->d_in.ensure(n + 64));
    HIPCHK(ctx->d_out.ensure(P->dst_bound + 64));
    DevBuf d_io, d_il;
    const size_t ni = P->item_blk0.size();
    HIPCHK(d_io.ensure(ni * 8));
    HIPCHK(d_il.ensure(ni * 4));
    HostStage& hs = ctx->hs;
    HIPCHK(hs.h2d(ctx->d_in.p, src, n, st));
    rc = run_encode(ctx, P, ctx->d_in.as<uint8_t>(), ctx->d_out.as<uint8_t>(), d_io.as<uint64_t>(),
                    d_il.as<uint32_t>(), st);
    if (rc) return rc;
    HIPCHK(hs.small.ensure(16));
    HIPCHK(hipMemcpyAsync(hs.small.p, P->d_total.p, 8, hipMemcpyDeviceToHost, st));
    // small outputs come back in the same round trip (bound-sized copy into pinned staging)
    const bool spec = P->dst_bound <= kSpecBytes && !host_pinned(dst);
    if (spec) {
        HIPCHK(hs.init(P->dst_bound));
        HIPCHK(hs.buf[0].ensure(P->dst_bound + 16));
        HIPCHK(hipMemcpyAsync(hs.buf[0].p, ctx->d_out.p, P->dst_bound, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    uint64_t total = 0;
    memcpy(&total, hs.small.p, 8);
    if (total > cap) return fail(S3HC_DST_TOO_SMALL, "dst capacity below encoded size");
    if (spec) par_memcpy(dst, hs.buf[0].p, total);
    else HIPCHK(hs.d2h(dst, {{ctx->d_out.as<uint8_t>(), total}}, st));
    *out_len = total;
    return S3HC_OK;
}

// ------------------------------------- lz4_flex-compatible encoder (§8(f) row 4)
// One frame per input range, laid out as FrameEncoder writes it, block payloads from the
// s3hc_compat.hip kernel (one wave per frame). Descriptors are host arrays; the caller's dst
// offsets must leave s3hc_frame_bound(len[i]) bytes per frame. Caller holds ctx->mu.
static int run_compat(s3hc_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint32_t* len, uint32_t n,
                      uint8_t* d_dst, const uint64_t* dst_off, uint32_t* d_frame_len, hipStream_t st) {
    if (!n) return S3HC_OK;
    std::vector<uint64_t> so(src_off, src_off + n), dof(dst_off, dst_off + n);
    std::vector<uint32_t> ln(len, len + n);
    uint32_t n_small = 0;  // frames of <= 64 KiB (16-bit hash-table kernel)
    for (uint32_t i = 0; i < n; ++i) n_small += ln[i] <= 65536u;
    for (uint32_t i = 0; i + 1 < n; ++i)
        if (dof[i + 1] < dof[i] || dof[i + 1] - dof[i] < s3hc_frame_bound(ln[i]))
            return fail(S3HC_INVALID_ARG, "dst_off leaves less than s3hc_frame_bound(len) per frame");
    HIPCHK(upload(ctx->d_c_soff, so, st));
    HIPCHK(upload(ctx->d_c_len, ln, st));
    HIPCHK(upload(ctx->d_c_doff, dof, st));
    HIPCHK(ctx->d_c_hash.ensure((size_t)n * 4));
    KTimer T(ctx, st);
    T.begin("xxh32");
    HIPCHK(launch_xxh32(d_src, ctx->d_c_soff.as<uint64_t>(), ctx->d_c_len.as<uint32_t>(), n, ctx->d_c_hash.as<uint32_t>(), st));
    T.end();
    T.begin("compat");
    HIPCHK(launch_compat_frames(d_src, ctx->d_c_soff.as<uint64_t>(), ctx->d_c_len.as<uint32_t>(), n, d_dst,
                                ctx->d_c_doff.as<uint64_t>(), ctx->d_c_hash.as<uint32_t>(), d_frame_len, n_small, st));
    T.end();
    // the descriptors live in ctx scratch: the next call may not overwrite them early
    HIPCHK(hipStreamSynchronize(st));
    return S3HC_OK;
}

extern "C" int s3hc_compat_encode_dev(s3hc_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint32_t* len,
                                      uint32_t n, uint8_t* d_dst, const uint64_t* dst_off, uint32_t* d_frame_len,
                                      void* stream) {
    return guarded([&]() -> int {
        if (!ctx || (n && (!d_src || !src_off || !len || !d_dst || !dst_off || !d_frame_len)))
            return fail(S3HC_INVALID_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        return run_compat(ctx, d_src, src_off, len, n, d_dst, dst_off, d_frame_len, stream ? (hipStream_t)stream : ctx->stream);
    });
}

static int host_compat(s3hc_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    if (!ctx || (!src && n) || !out_len) return fail(S3HC_INVALID_ARG, "bad arguments");
    if (n > 0xFFFFFFFFull) return fail(S3HC_INVALID_ARG, "single-frame input above 4 GiB");
    const size_t bound = s3hc_frame_bound(n);
    if (cap < bound) return fail(S3HC_DST_TOO_SMALL, "dst capacity below frame bound");
    std::lock_guard<std::mutex> g(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    HIPCHK(ctx->d_in.ensure(n + 64));
    HIPCHK(ctx->d_out.ensure(bound + 64));
    HIPCHK(ctx->d_c_flen.ensure(16));
    HIPCHK(ctx->hs.h2d(ctx->d_in.p, src, n, st));
    const uint64_t so = 0, dof = 0;
    const uint32_t ln = (uint32_t)n;
    int rc = run_compat(ctx, ctx->d_in.as<uint8_t>(), &so, &ln, 1, ctx->d_out.as<uint8_t>(), &dof,
                        ctx->d_c_flen.as<uint32_t>(), st);
    if (rc) return rc;
    HIPCHK(ctx->hs.small.ensure(16));
    HIPCHK(hipMemcpyAsync(ctx->hs.small.p, ctx->d_c_flen.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint32_t flen = 0;
    memcpy(&flen, ctx->hs.small.p, 4);
    if (flen > bound) return fail(S3HC_DEVICE, "compat frame longer than its bound");
    HIPCHK(ctx->hs.d2h(dst, {{ctx->d_out.as<uint8_t>(), flen}}, st));
    *out_len = flen;
    return S3HC_OK;
}

extern "C" int s3hc_compress_frame(s3hc_ctx* ctx, const uint8_t* src, size_t n, int policy, uint8_t* dst, size_t cap,
                                   size_t* out_len, int* was_compressed) {
    return guarded([&]() -> int {
        if (policy == S3HC_BLK_LZ4FLEX_COMPAT) {
            int rc = host_compat(ctx, src, n, dst, cap, out_len);
            if (was_compressed) *was_compressed = rc == S3HC_OK;
            return rc;
        }
        if (policy != S3HC_BLK_AUTO_LZ4FLEX && policy != S3HC_BLK_64K_PER_FRAME) return fail(S3HC_INVALID_ARG, "policy");
        int rc = host_encode(ctx, src, n, 0, policy, dst, cap, out_len);
        if (was_compressed) *was_compressed = rc == S3HC_OK;
        return rc;
    });
}

extern "C" int s3hc_store_mode_frame(s3hc_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                                     size_t* out_len) {
    return guarded([&]() -> int {
        return host_encode(ctx, src, n, 1, S3HC_BLK_AUTO_LZ4FLEX, dst, cap, out_len);
    });
}

// --------------------------------------------- host-buffer frame walker
// Structure of concatenated frames in a host buffer, in decompress_data order
// (compression.rs:474-494). Mirrors lz4_flex FrameInfo::read / FrameDecoder::read_more.
struct HFrame {
    size_t pos;          // frame start in src
    uint32_t flg, bmax;
    uint32_t blk0, nblk;
    uint64_t out_off;    // slot-layout output offset (device)
    uint64_t content_size;
    uint32_t want;       // content checksum
};
struct HWalk {
    std::vector<HFrame> frames;
    std::vector<DecBlock> blocks;
    std::vector<uint32_t> blk_cs_want;  // block checksums (FLG 0x10)
    std::vector<uint8_t> blk_has_cs;
    int tail_status = S3HC_OK;   // structural error after the last complete frame
    bool last_incomplete = false; // tail_status belongs to the last frame in `frames` (truncated/bad block)
    bool stopped_empty = false;  // a frame with no blocks ended the walk (Ok(0) => break)
    size_t end = 0;              // bytes consumed by complete frames
    uint64_t slot_total = 0;
};

static int parse_header_h(const uint8_t* p, size_t avail, uint32_t* flg, uint32_t* bmax, size_t* hdr, uint64_t* csize) {
    if (avail < 4) return S3HC_CORRUPT;
    uint32_t magic = rd32h(p);
    if (magic == 0x184C2102u || (magic & 0xFFFFFFF0u) == 0x184D2A50u) return S3HC_UNSUPPORTED;
    if (magic != kMagic || avail < 7) return S3HC_CORRUPT;
    uint32_t f = p[4], bd = p[5];
    size_t need = 7 + ((f & 0x08) ? 8 : 0) + ((f & 0x01) ? 4 : 0);
    if (avail < need) return S3HC_CORRUPT;
    if ((f & 0xC0) != 0x40 || (f & 0x02) || (bd & 0x8F)) return S3HC_CORRUPT;
    uint32_t code = (bd >> 4) & 7;
    if (code < 4) return S3HC_CORRUPT;
    if ((uint8_t)(hdr_xxh32(p + 4, need - 5) >> 8) != p[need - 1]) return S3HC_CORRUPT;
    if (f & 0x01) return S3HC_UNSUPPORTED;
    *flg = f;
    *bmax = 1u << (16 + 2 * (code - 4));
    *hdr = need;
    *csize = (f & 0x08) ? ((uint64_t)rd32h(p + 6) | ((uint64_t)rd32h(p + 10) << 32)) : 0;
    return S3HC_OK;
}

// Walk frames from src; `stream_mode` = stream_range_data semantics (an incomplete final
// frame is left for later instead of being an error; an empty frame does not stop).
// stop_after: the walk ends after the first complete frame that ends at or past this byte (a
// range reader batch needs no more; default: walk everything)
static void walk_frames(const uint8_t* src, size_t n, HWalk& W, bool allow_incomplete, bool stop_on_empty,
                        size_t stop_after = ~(size_t)0) {
    const bool stream_mode = allow_incomplete;
    size_t pos = 0;
    while (pos < n) {
        HFrame F{};
        size_t hdr;
        int rc = parse_header_h(src + pos, n - pos, &F.flg, &F.bmax, &hdr, &F.content_size);
        if (rc) {
            if (stream_mode && rc == S3HC_CORRUPT && n - pos < 19) break;  // maybe just incomplete
            W.tail_status = rc;
            return;
        }
        F.pos = pos;
        F.blk0 = (uint32_t)W.blocks.size();
        F.out_off = W.slot_total;
        const bool linked = !(F.flg & 0x20);
        size_t ip = pos + hdr;
        uint64_t slot = 0;
        int st = S3HC_OK;
        bool complete = false;
        // blocks go straight into W (rolled back when the frame turns out incomplete in
        // stream mode): no per-frame allocations on the range reader's per-batch path
        const size_t b0 = W.blocks.size();
        for (;;) {
            if (n - ip < 4) { st = S3HC_CORRUPT; break; }
            uint32_t w = rd32h(src + ip);
            ip += 4;
            if (w == 0) {
                if (F.flg & 0x04) {
                    if (n - ip < 4) { st = S3HC_CORRUPT; break; }
                    F.want = rd32h(src + ip);
                    ip += 4;
                }
                complete = true;
                break;
            }
            uint32_t len = w & 0x7FFFFFFFu;
            if (len > F.bmax) { st = S3HC_CORRUPT; break; }
            size_t need = (size_t)len + ((F.flg & 0x10) ? 4 : 0);
            if (n - ip < need) { st = S3HC_CORRUPT; break; }
            DecBlock D{};
            D.src_off = ip;
            D.dst_off = F.out_off + slot;
            D.csize = len;
            D.limit = (w & kStoredBit) ? len : F.bmax;
            // Output slot: no LZ4 sequence writes more than 255 bytes per compressed byte (a
            // 255-run extension byte adds at most 255 to a length, every other byte costs at
            // least one), so a block of `len` bytes decodes to < 255 * len. Tiny blocks in a
            // BD 4 MiB frame therefore reserve a few hundred bytes, not 4 MiB each.
            D.cap = (uint32_t)std::min<uint64_t>(D.limit, 255ull * len);
            D.flags = ((w & kStoredBit) ? DB_STORED : 0u) | (linked ? DB_LINKED : 0u);
            D.frame = (uint32_t)W.frames.size();
            W.blocks.push_back(D);
            W.blk_has_cs.push_back((F.flg & 0x10) ? 1 : 0);
            W.blk_cs_want.push_back((F.flg & 0x10) ? rd32h(src + ip + len) : 0);
            slot += D.cap;
            ip += need;
        }
        if (!complete) {
            if (stream_mode && st == S3HC_CORRUPT) {  // wait for more bytes
                W.blocks.resize(b0);
                W.blk_has_cs.resize(b0);
                W.blk_cs_want.resize(b0);
                break;
            }
            // Blocks before the failure still decode (their errors come first in order).
            W.tail_status = st;
            W.last_incomplete = true;
        }
        F.nblk = (uint32_t)(W.blocks.size() - b0);
        W.slot_total += slot;
        W.frames.push_back(F);
        if (!complete) return;
        pos = ip;
        W.end = pos;
        if (F.nblk == 0 && stop_on_empty) {  // empty frame: read_to_end == Ok(0) => break
            W.stopped_empty = true;
            return;
        }
        if (pos >= stop_after) return;
    }
}

extern "C" int s3hc_decompressed_bound(const uint8_t* src, size_t n, size_t* bound) {
    return guarded([&]() -> int {
        if ((!src && n) || !bound) return fail(S3HC_INVALID_ARG, "bad arguments");
        HWalk W;
        walk_frames(src, n, W, false, true);
        uint64_t b = 0;
        for (auto& D : W.blocks) b += D.cap;
        *bound = b;
        return S3HC_OK;
    });
}

// Decode the frames of W (already walked) from a host buffer; append decoded bytes to
// `out` (host) in frame order. Applies the decompress_data loop rules unless stream_mode.
// Returns the first error in frame order (or W.tail_status).
//
// One submission and one readback in the common case: decode, block checksums, each frame's
// output length and content xxh32 over its device slots (k_dframe_finish + k_xxh32_ranges),
// and — for outputs up to kSpecBytes — the decoded slots themselves into pinned staging; then
// one synchronisation, the host resolves frames in order and copies the delivered bytes out.
// Frames whose output is not contiguous on the device (a short non-final independent block)
// take the second round trip below (device compaction, checksum, copy).
static double host_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static int decode_walk(s3hc_ctx* ctx, const uint8_t* src, size_t n, HWalk& W, bool stream_mode,
                       std::vector<uint8_t>* vout, uint8_t* dst, size_t cap, size_t* out_len,
                       bool upload_in = true, bool* stopped_out = nullptr) {
    const bool trace = knob_on(KN_HOST_TRACE);  // diagnostics: stage times
    const double t_0 = trace ? host_us() : 0.0;
#define HTRACE(tag) if (trace) fprintf(stderr, "[s3hc host] %-10s %8.1f us\n", tag, host_us() - t_0);
    hipStream_t st = ctx->stream;
    HostStage& hs = ctx->hs;
    const size_t nb = W.blocks.size(), nf = W.frames.size();
    // readback layout (u32 words): bo[nb] bs[nb] cs_got[nb] flen[nf] fhash[nf]
    const uint32_t* bo = nullptr;
    const int32_t* bs = nullptr;
    const uint32_t *cs_got = nullptr, *flen = nullptr, *fhash = nullptr;
    bool spec = false;  // each frame's slot prefix [out_off, out_off + spre[f]) is in hs.buf[0] at spos[f]
    std::vector<uint64_t> spre, spos;
    if (stopped_out) *stopped_out = false;
    if (nb) {
        if (upload_in) {
            HIPCHK(ctx->d_in.ensure(n + 64));
            HIPCHK(hs.h2d(ctx->d_in.p, src, n, st));
        }
        HIPCHK(ctx->d_out.ensure(W.slot_total + 64));
        std::vector<DecUnit> units;
        for (auto& F : W.frames) {
            if (!F.nblk) continue;
            if (!(F.flg & 0x20)) units.push_back(DecUnit{F.blk0, F.nblk});
            else for (uint32_t k = 0; k < F.nblk; ++k) units.push_back(DecUnit{F.blk0 + k, 1});
        }
        const uint64_t tok_entries = assign_tok_slots(W.blocks.data(), W.blocks.size());
        HIPCHK(upload(ctx->d_blocks, W.blocks, st));
        HIPCHK(upload(ctx->d_units, units, st));
        HIPCHK(ctx->d_blk_out.ensure(nb * 4));
        HIPCHK(ctx->d_blk_status.ensure(nb * 4));
        HIPCHK(prepare_host_launch(ctx->lb, W.blocks.data(), nb, units.data(), (uint32_t)units.size(), tok_entries));
        const uint64_t* bh = nullptr;
        HTRACE("launch")
        HIPCHK(decode_launch(&ctx->lb, ctx->d_in.as<uint8_t>(), ctx->d_out.as<uint8_t>(), ctx->d_blocks.as<DecBlock>(),
                             ctx->d_units.as<DecUnit>(), (uint32_t)units.size(), ctx->d_blk_out.as<uint32_t>(),
                             ctx->d_blk_status.as<int32_t>(), st, &bh));
        // block checksums (FLG bit 4) over the compressed payloads
        bool any_cs = false;
        for (auto h : W.blk_has_cs) any_cs |= h != 0;
        if (any_cs) {
            std::vector<uint64_t> ro(nb);
            std::vector<uint32_t> rl(nb);
            for (size_t i = 0; i < nb; ++i) { ro[i] = W.blocks[i].src_off; rl[i] = W.blocks[i].csize; }
            HIPCHK(upload(ctx->d_rng_off, ro, st));
            HIPCHK(upload(ctx->d_rng_len, rl, st));
            HIPCHK(ctx->d_hash.ensure(nb * 4));
            HIPCHK(launch_xxh32(ctx->d_in.as<uint8_t>(), ctx->d_rng_off.as<uint64_t>(), ctx->d_rng_len.as<uint32_t>(),
                                (uint32_t)nb, ctx->d_hash.as<uint32_t>(), st));
        }
        // per-frame output length (blocks in order, contiguous slots) and content checksum
        // (k_dframe_close; its statuses are not used here: the host resolves frames itself)
        {
            std::vector<uint64_t> ft(3 * nf + (nf + 1) / 2 + (nf + 1) / 2);
            uint32_t* fnb = (uint32_t*)(ft.data() + 3 * nf);
            uint32_t* fw = fnb + nf + (nf & 1);
            for (size_t f = 0; f < nf; ++f) {
                ft[f] = W.frames[f].pos;
                ft[nf + f] = W.frames[f].blk0;
                ft[2 * nf + f] = W.frames[f].out_off;
                fnb[f] = W.frames[f].nblk;
                fw[f] = W.frames[f].want;
            }
            HIPCHK(upload(ctx->d_ftab, ft, st));
            HIPCHK(ctx->d_fstat.ensure(nf * 4));
            HIPCHK(ctx->d_flen.ensure(nf * 4));
            HIPCHK(ctx->d_fhash.ensure(nf * 4));
            const uint64_t* d_ft = ctx->d_ftab.as<uint64_t>();
            const uint32_t* d_fnb = (const uint32_t*)(d_ft + 3 * nf);
            HIPCHK(launch_dframe_close(ctx->d_in.as<uint8_t>(), d_ft, d_ft + nf, d_fnb, ctx->d_blocks.as<DecBlock>(),
                                       ctx->d_blk_out.as<uint32_t>(), ctx->d_blk_status.as<int32_t>(), bh,
                                       ctx->d_out.as<uint8_t>(), d_ft + 2 * nf, d_fnb + nf + (nf & 1), (uint32_t)nf,
                                       nullptr, ctx->d_fstat.as<int32_t>(), ctx->d_flen.as<uint32_t>(),
                                       ctx->d_fhash.as<uint32_t>(), st));
        }
        HIPCHK(hs.small.ensure((3 * nb + 2 * nf) * 4 + 16));
        uint32_t* rb = (uint32_t*)hs.small.p;
        HIPCHK(hipMemcpyAsync(rb, ctx->d_blk_out.p, nb * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rb + nb, ctx->d_blk_status.p, nb * 4, hipMemcpyDeviceToHost, st));
        if (any_cs) HIPCHK(hipMemcpyAsync(rb + 2 * nb, ctx->d_hash.p, nb * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rb + 3 * nb, ctx->d_flen.p, nf * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rb + 3 * nb + nf, ctx->d_fhash.p, nf * 4, hipMemcpyDeviceToHost, st));
        // small outputs: their slots come back in the same round trip (pageable destinations).
        // Per frame only a prefix of its slot, min(slot, max(4 x the frame's compressed bytes,
        // 1 MiB)): a BD 0x70 frame's slot is 4 MiB whatever it decodes to (lz4_flex writes no
        // content size). The prefixes are packed in the staging buffer; adjacent ones (whole
        // slots) are copied in one piece. A frame decoding past its prefix (ratios above 4) sends
        // the delivery through the second round trip below.
        {
            spre.assign(nf, 0);
            spos.assign(nf, 0);
            uint64_t stot = 0;
            for (size_t f = 0; f < nf; ++f) {
                const HFrame& F = W.frames[f];
                uint64_t slot = 0;
                for (uint32_t k = 0; k < F.nblk; ++k) slot += W.blocks[F.blk0 + k].cap;
                const uint64_t fc = (f + 1 < nf ? W.frames[f + 1].pos : n) - F.pos;
                spre[f] = std::min<uint64_t>(slot, std::max<uint64_t>(4 * fc, 1u << 20));
                spos[f] = stot;
                stot += spre[f];
            }
            spec = stot <= kSpecBytes && (vout || !host_pinned(dst));
            if (spec && stot) {
                HIPCHK(hs.init(stot));
                HIPCHK(hs.buf[0].ensure(stot + 16));
                size_t f = 0;
                while (f < nf) {  // one copy per run of frames whose device ranges abut
                    size_t g = f + 1;
                    while (g < nf && W.frames[g - 1].out_off + spre[g - 1] == W.frames[g].out_off) ++g;
                    const uint64_t bytes = spos[g - 1] + spre[g - 1] - spos[f];
                    if (bytes)
                        HIPCHK(hipMemcpyAsync(hs.buf[0].p + spos[f], ctx->d_out.as<uint8_t>() + W.frames[f].out_off,
                                              bytes, hipMemcpyDeviceToHost, st));
                    f = g;
                }
            }
        }
        HTRACE("queued")
        HIPCHK(hipStreamSynchronize(st));
        HTRACE("synced")
        bo = rb;
        bs = (const int32_t*)(rb + nb);
        cs_got = rb + 2 * nb;
        flen = rb + 3 * nb;
        fhash = rb + 3 * nb + nf;
    }
    // Resolve frames in order (FrameDecoder reads frames sequentially): the first failure in
    // stream order wins — a block's checksum/decode error, then at its EndMark the frame's
    // content size and content checksum, then the next frame; a frame yielding 0 bytes ends
    // the loop (Ok(0) => break) and nothing after it is looked at.
    int err_status = S3HC_OK;
    size_t use_frames = nf;    // frames whose output is delivered / checksummed
    bool stopped = false;
    std::vector<uint64_t> fout(nf, 0);
    bool need_compact = false;
    for (size_t f = 0; f < nf; ++f) {
        const HFrame& F = W.frames[f];
        uint64_t tot = 0;
        int fs = S3HC_OK;
        for (uint32_t k = 0; k < F.nblk; ++k) {
            const uint32_t b = F.blk0 + k;
            // device-written results drive the copies below: a status no decoder assigns or a block
            // longer than its frame allows is not a decode's result
            if (bs[b] < S3HC_OK || bs[b] > S3HC_INVALID_ARG || (bs[b] == S3HC_OK && bo[b] > W.blocks[b].limit))
                return fail(S3HC_DEVICE, "decode results out of range");
            if (W.blk_has_cs[b] && cs_got[b] != W.blk_cs_want[b]) { fs = S3HC_CHECKSUM; break; }
            if (bs[b] != S3HC_OK) { fs = bs[b]; break; }
            if ((F.flg & 0x20) && k + 1 < F.nblk && bo[b] != W.blocks[b].cap) need_compact = true;
            tot += bo[b];
        }
        if (fs == S3HC_OK && f + 1 == nf && W.last_incomplete) fs = W.tail_status;  // incomplete frame
        if (fs != S3HC_OK) { err_status = fs; use_frames = f; break; }
        fout[f] = tot;
        if (!stream_mode && tot == 0) { use_frames = f + 1; stopped = true; break; }
    }
    if (stopped_out) *stopped_out = stopped;
    if (err_status == S3HC_OK && !stopped && W.tail_status != S3HC_OK && !W.last_incomplete) {
        // a header-level failure after every walked frame (bad magic, truncated header, ...)
        err_status = W.tail_status;
    }
    // Compact independent frames whose non-final blocks were short (rare) so each frame's
    // output is contiguous before its content checksum is computed.
    uint64_t total = 0;
    for (size_t f = 0; f < use_frames; ++f) total += fout[f];
    DevBuf compact;
    const uint8_t* dev_out = ctx->d_out.as<uint8_t>();
    std::vector<uint64_t> fpos(use_frames);
    if (need_compact) {
        spec = false;
        HIPCHK(compact.ensure(total + 64));
        uint64_t o = 0;
        for (size_t f = 0; f < use_frames; ++f) {
            const HFrame& F = W.frames[f];
            fpos[f] = o;
            const bool linked = !(F.flg & 0x20);
            uint64_t lpos = F.out_off;  // linked units decode contiguously from the frame start
            for (uint32_t k = 0; k < F.nblk; ++k) {
                const uint32_t b = F.blk0 + k;
                const uint64_t from = linked ? lpos : W.blocks[b].dst_off;
                if (bo[b]) HIPCHK(hipMemcpyAsync(compact.as<uint8_t>() + o, dev_out + from, bo[b],
                                                 hipMemcpyDeviceToDevice, st));
                o += bo[b];
                lpos += bo[b];
            }
        }
        dev_out = compact.as<uint8_t>();
    } else {
        for (size_t f = 0; f < use_frames; ++f) fpos[f] = W.frames[f].out_off;
    }
    // EndMark checks of every delivered frame, in order: content size, content checksum (GPU
    // xxh32: the one already read back when the device hashed exactly the frame's bytes)
    {
        std::vector<uint64_t> ro;
        std::vector<uint32_t> rl;
        std::vector<size_t> which;
        for (size_t f = 0; f < use_frames; ++f) {
            if (!(W.frames[f].flg & 0x04)) continue;
            if (flen && !need_compact && flen[f] == fout[f]) continue;  // fhash[f] is the frame's checksum
            // the checksum kernel takes 32-bit range lengths
            if (fout[f] > 0xFFFFFFFFull) return fail(S3HC_UNSUPPORTED, "a frame that decodes to 4 GiB or more");
            ro.push_back(fpos[f]);
            rl.push_back((uint32_t)fout[f]);
            which.push_back(f);
        }
        std::vector<uint32_t> got(nf, 0);
        if (!ro.empty()) {
            HIPCHK(upload(ctx->d_rng_off, ro, st));
            HIPCHK(upload(ctx->d_rng_len, rl, st));
            HIPCHK(ctx->d_hash.ensure(ro.size() * 4));
            HIPCHK(launch_xxh32(dev_out, ctx->d_rng_off.as<uint64_t>(), ctx->d_rng_len.as<uint32_t>(),
                                (uint32_t)ro.size(), ctx->d_hash.as<uint32_t>(), st));
            std::vector<uint32_t> g(ro.size());
            HIPCHK(hipMemcpyAsync(g.data(), ctx->d_hash.p, ro.size() * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (size_t i = 0; i < which.size(); ++i) got[which[i]] = g[i];
        }
        std::vector<bool> redo(nf, false);
        for (size_t f : which) redo[f] = true;
        for (size_t f = 0; f < use_frames; ++f) {
            const HFrame& F = W.frames[f];
            if ((F.flg & 0x08) && fout[f] != F.content_size) return fail(S3HC_CORRUPT, "content size mismatch");
            if ((F.flg & 0x04) && (redo[f] ? got[f] : fhash[f]) != F.want)
                return fail(S3HC_CHECKSUM, "content checksum mismatch");
        }
    }
    HTRACE("resolved")
    if (err_status != S3HC_OK) return fail(err_status, "frame decode failed");
    // Deliver
    uint8_t* hdst = dst;
    if (vout) {
        size_t o0 = vout->size();
        vout->resize(o0 + total);
        hdst = vout->data() + o0;
    } else if (total > cap) {
        *out_len = total;
        return fail(S3HC_DST_TOO_SMALL, "dst capacity below decoded size");
    }
    // runs of adjacent frames' bytes (one copy each)
    std::vector<std::pair<const uint8_t*, uint64_t>> runs;
    std::vector<std::pair<uint64_t, uint64_t>> spans;  // (device offset, bytes)
    for (size_t f = 0; f < use_frames; ++f) {
        if (!fout[f]) continue;
        if (!spans.empty() && spans.back().first + spans.back().second == fpos[f]) spans.back().second += fout[f];
        else spans.push_back({fpos[f], fout[f]});
    }
    if (spec)
        for (size_t f = 0; f < use_frames; ++f)
            if (fout[f] > spre[f]) spec = false;  // decoded past the prefix read back early
    if (spec) {
        // frames' bytes from their packed prefixes; adjacent frames whose prefixes are whole
        // slots sit back to back in staging too, so runs stay one copy
        uint64_t o = 0;
        size_t f = 0;
        while (f < use_frames) {
            size_t g = f + 1;
            while (g < use_frames && fout[g - 1] == spre[g - 1] && spos[g - 1] + spre[g - 1] == spos[g]) ++g;
            uint64_t bytes = 0;
            for (size_t k = f; k < g; ++k) bytes += fout[k];
            if (bytes) par_memcpy(hdst + o, hs.buf[0].p + spos[f], bytes);
            o += bytes;
            f = g;
        }
    } else {
        for (auto& sp : spans) runs.push_back({dev_out + sp.first, sp.second});
        HIPCHK(hs.d2h(hdst, runs, st));
    }
    HTRACE("delivered")
#undef HTRACE
    if (out_len) *out_len = total;
    return S3HC_OK;
}

// Decode a walk in passes of whole frames whose output slots total <= kPassSlot (a frame larger
// than that is a pass of its own), so device scratch follows the real output, not the whole
// input's worst case; decoded bytes go to `vout` (grown by what each pass produced) or to
// dst/cap. Frame order, the first-error rule and the empty-frame stop carry across passes.
static constexpr uint64_t kPassSlot = 2ull << 30;
static int decode_walk_passes(s3hc_ctx* ctx, const uint8_t* src, size_t n, HWalk& W, bool stream_mode,
                              std::vector<uint8_t>* vout, uint8_t* dst, size_t cap, size_t* out_len) {
    if (W.slot_total <= kPassSlot) return decode_walk(ctx, src, n, W, stream_mode, vout, dst, cap, out_len);
    const size_t nf = W.frames.size();
    size_t a = 0;
    uint64_t done = 0;
    bool uploaded = false;
    auto frame_slot = [&](size_t f) {
        uint64_t s = 0;
        for (uint32_t k = 0; k < W.frames[f].nblk; ++k) s += W.blocks[W.frames[f].blk0 + k].cap;
        return s;
    };
    while (a < nf) {
        size_t b = a;
        uint64_t slot = 0;
        while (b < nf) {
            const uint64_t fs = frame_slot(b);
            if (b > a && slot + fs > kPassSlot) break;
            slot += fs;
            ++b;
        }
        HWalk P;
        const uint64_t base = W.frames[a].out_off;
        const uint32_t blk_base = W.frames[a].blk0;
        for (size_t f = a; f < b; ++f) {
            HFrame F = W.frames[f];
            F.out_off -= base;
            F.blk0 -= blk_base;
            P.frames.push_back(F);
            for (uint32_t k = 0; k < F.nblk; ++k) {
                DecBlock D = W.blocks[W.frames[f].blk0 + k];
                D.dst_off -= base;
                D.frame = (uint32_t)(f - a);
                P.blocks.push_back(D);
                P.blk_cs_want.push_back(W.blk_cs_want[W.frames[f].blk0 + k]);
                P.blk_has_cs.push_back(W.blk_has_cs[W.frames[f].blk0 + k]);
            }
        }
        P.slot_total = slot;
        if (b == nf) {  // the walk's own tail belongs to its last pass
            P.tail_status = W.tail_status;
            P.last_incomplete = W.last_incomplete;
            P.stopped_empty = W.stopped_empty;
        }
        size_t got = 0;
        bool stopped = false;
        const int rc = decode_walk(ctx, src, n, P, stream_mode, vout, dst ? dst + done : nullptr,
                                   dst ? cap - (size_t)done : 0, &got, !uploaded, &stopped);
        uploaded = true;
        if (rc) {
            if (out_len) *out_len = (size_t)done + got;
            return rc;
        }
        done += got;
        if (stopped) break;  // a frame yielding 0 bytes ended decompress_data's loop
        a = b;
    }
    if (out_len) *out_len = (size_t)done;
    return S3HC_OK;
}

extern "C" int s3hc_decompress_frames(s3hc_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                                      size_t* out_len) {
    if (!ctx || (!src && n) || !out_len) return fail(S3HC_INVALID_ARG, "bad arguments");
    return guarded([&] {
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        *out_len = 0;
        HWalk W;
        walk_frames(src, n, W, false, true);
        return decode_walk_passes(ctx, src, n, W, false, nullptr, dst, cap, out_len);
    });
}

namespace s3hc {
// decompress_data into a vector sized by the decoded bytes (compression.rs:463-502 read_to_end).
int decompress_frames_vec(s3hc_ctx* ctx, const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
    if (!ctx || (!src && n)) return fail(S3HC_INVALID_ARG, "bad arguments");
    return guarded([&] {
        std::lock_guard<std::mutex> g(ctx->mu);
        HIPCHK(hipSetDevice(ctx->device));
        out.clear();
        HWalk W;
        walk_frames(src, n, W, false, true);
        size_t len = 0;
        const int rc = decode_walk_passes(ctx, src, n, W, false, &out, nullptr, 0, &len);
        if (rc) out.clear();
        return rc;
    });
}
}  // namespace s3hc

extern "C" int s3hc_decompress_frames_alloc(s3hc_ctx* ctx, const uint8_t* src, size_t n, uint8_t** out,
                                            size_t* out_len) {
    if (!out || !out_len) return fail(S3HC_INVALID_ARG, "bad arguments");
    *out = nullptr;
    *out_len = 0;
    std::vector<uint8_t> v;
    const int rc = s3hc::decompress_frames_vec(ctx, src, n, v);
    if (rc) return rc;
    return guarded([&] {
        uint8_t* p = (uint8_t*)malloc(v.size() ? v.size() : 1);
        if (!p) return fail(S3HC_NO_MEMORY, "host allocation failed");
        if (!v.empty()) memcpy(p, v.data(), v.size());
        *out = p;
        *out_len = v.size();
        return S3HC_OK;
    });
}
extern "C" void s3hc_buffer_free(uint8_t* p) { free(p); }

// ------------------------------------------------------ streaming decoder
struct s3hc_stream {
    s3hc_ctx* ctx;
    std::vector<uint8_t> in;    // undecoded input (starts at a frame boundary)
    std::vector<uint8_t> out;   // decoded, not yet read
    size_t out_pos = 0;
    bool finished = false;
    int error = S3HC_OK;
    uint64_t total = 0;
};

extern "C" int s3hc_stream_open(s3hc_ctx* ctx, s3hc_stream** out) {
    return guarded([&]() -> int {
        if (!ctx || !out) return fail(S3HC_INVALID_ARG, "bad arguments");
        *out = new s3hc_stream{ctx};
        return S3HC_OK;
    });
}
extern "C" int s3hc_stream_feed(s3hc_stream* s, const uint8_t* src, size_t n) {
    return guarded([&]() -> int {
        if (!s || (!src && n)) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (s->finished) return fail(S3HC_INVALID_ARG, "stream already finished");
        s->in.insert(s->in.end(), src, src + n);
        return S3HC_OK;
    });
}
extern "C" int s3hc_stream_finish(s3hc_stream* s) {
    return guarded([&]() -> int {
        if (!s) return fail(S3HC_INVALID_ARG, "bad arguments");
        s->finished = true;
        return S3HC_OK;
    });
}
// Decode every complete frame buffered so far (stream_range_data: one FrameDecoder per frame).
static int stream_pump(s3hc_stream* s) {
    if (s->error) return s->error;
    if (s->in.empty()) return S3HC_OK;
    std::lock_guard<std::mutex> g(s->ctx->mu);
    HIPCHK(hipSetDevice(s->ctx->device));
    HWalk W;
    walk_frames(s->in.data(), s->in.size(), W, !s->finished, false);
    if (s->finished && W.tail_status == S3HC_OK && W.end != s->in.size() && W.frames.empty())
        W.tail_status = S3HC_CORRUPT;
    if (W.frames.empty() && W.tail_status == S3HC_OK) return S3HC_OK;
    if (s->out_pos == s->out.size()) { s->out.clear(); s->out_pos = 0; }
    size_t before = s->out.size();
    int rc = decode_walk_passes(s->ctx, s->in.data(), s->in.size(), W, true, &s->out, nullptr, 0, nullptr);
    if (rc) {
        s->out.resize(before);
        s->error = rc;
        return rc;
    }
    s->total += s->out.size() - before;
    s->in.erase(s->in.begin(), s->in.begin() + W.end);
    if (s->finished && !s->in.empty()) {  // trailing bytes that never formed a frame
        s->error = S3HC_CORRUPT;
        return fail(S3HC_CORRUPT, "truncated frame at end of stream");
    }
    return S3HC_OK;
}
extern "C" int s3hc_stream_read(s3hc_stream* s, uint8_t* dst, size_t cap, size_t* n) {
    return guarded([&]() -> int {
        if (!s || !n || (!dst && cap)) return fail(S3HC_INVALID_ARG, "bad arguments");
        *n = 0;
        if (s->out_pos == s->out.size()) {
            int rc = stream_pump(s);
            if (rc) return rc;
        }
        size_t k = std::min(cap, s->out.size() - s->out_pos);
        if (k) memcpy(dst, s->out.data() + s->out_pos, k);
        s->out_pos += k;
        *n = k;
        return S3HC_OK;
    });
}
extern "C" uint64_t s3hc_stream_total(const s3hc_stream* s) { return s ? s->total : 0; }
extern "C" void s3hc_stream_close(s3hc_stream* s) { delete s; }

// ----------------------------------------------- device memory plumbing
// Thin helpers so callers (tests, bench) can stage device-resident batches without a
// second HIP runtime in the process.
extern "C" int s3hc_dev_alloc(s3hc_ctx* ctx, size_t n, void** out) {
    return guarded([&]() -> int {
        if (!ctx || !out) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipMalloc(out, n ? n : 16));
        return S3HC_OK;
    });
}
extern "C" int s3hc_dev_free(s3hc_ctx* ctx, void* p) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        if (p) HIPCHK(hipFree(p));
        return S3HC_OK;
    });
}
// kind: 1 host->device, 2 device->host, 3 device->device. Synchronous w.r.t. the host.
extern "C" int s3hc_memcpy(s3hc_ctx* ctx, void* dst, const void* src, size_t n, int kind) {
    return guarded([&]() -> int {
        if (!ctx || kind < 1 || kind > 3) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
        if (n) HIPCHK(hipMemcpyAsync(dst, src, n, k, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        return S3HC_OK;
    });
}
extern "C" int s3hc_memset(s3hc_ctx* ctx, void* dst, int v, size_t n) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        if (n) HIPCHK(hipMemsetAsync(dst, v, n, ctx->stream));
        return S3HC_OK;
    });
}
extern "C" int s3hc_sync(s3hc_ctx* ctx) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        return S3HC_OK;
    });
}
extern "C" int s3hc_host_alloc(s3hc_ctx* ctx, size_t n, void** out) {
    return guarded([&]() -> int {
        if (!ctx || !out) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipHostMalloc(out, n ? n : 16, hipHostMallocPortable));
        return S3HC_OK;
    });
}
extern "C" int s3hc_host_free(s3hc_ctx* ctx, void* p) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (p) HIPCHK(hipHostFree(p));
        return S3HC_OK;
    });
}
extern "C" int s3hc_queue_create(s3hc_ctx* ctx, void** out) {
    return guarded([&]() -> int {
        if (!ctx || !out) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        hipStream_t s;
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *out = (void*)s;
        return S3HC_OK;
    });
}
extern "C" int s3hc_queue_destroy(s3hc_ctx* ctx, void* q) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (q) HIPCHK(hipStreamDestroy((hipStream_t)q));
        return S3HC_OK;
    });
}
extern "C" int s3hc_queue_sync(s3hc_ctx* ctx, void* q) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamSynchronize(q ? (hipStream_t)q : ctx->stream));
        return S3HC_OK;
    });
}
extern "C" int s3hc_queue_mark(s3hc_ctx* ctx, void* q, void** mark) {
    return guarded([&]() -> int {
        if (!ctx || !mark) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const hipError_t r = hipEventRecord(e, q ? (hipStream_t)q : ctx->stream);
        if (r != hipSuccess) (void)hipEventDestroy(e);
        HIPCHK(r);
        *mark = (void*)e;
        return S3HC_OK;
    });
}
extern "C" int s3hc_queue_wait_mark(s3hc_ctx* ctx, void* q, void* mark) {
    return guarded([&]() -> int {
        if (!ctx || !mark) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        HIPCHK(hipStreamWaitEvent(q ? (hipStream_t)q : ctx->stream, (hipEvent_t)mark, 0));
        return S3HC_OK;
    });
}
extern "C" int s3hc_mark_free(s3hc_ctx* ctx, void* mark) {
    return guarded([&]() -> int {
        if (!ctx) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (mark) HIPCHK(hipEventDestroy((hipEvent_t)mark));
        return S3HC_OK;
    });
}
extern "C" int s3hc_memcpy_async(s3hc_ctx* ctx, void* dst, const void* src, size_t n, int kind, void* q) {
    return guarded([&]() -> int {
        if (!ctx || kind < 1 || kind > 3) return fail(S3HC_INVALID_ARG, "bad arguments");
        HIPCHK(hipSetDevice(ctx->device));
        const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
        if (n) HIPCHK(hipMemcpyAsync(dst, src, n, k, q ? (hipStream_t)q : ctx->stream));
        return S3HC_OK;
    });
}

// ------------------------------------------- pipelined range reader (config 4)
// stream_range_data (disk_cache.rs:3850-3935) for throughput. Complete frames are grouped into
// device batches of about batch_bytes compressed bytes; each batch runs on one of `depth` HIP
// queues (pinned H2D, device frame walk + block decode + content-checksum verify, results D2H),
// so copies and kernels of different batches overlap. Decoded bytes come back in stream order.
// Semantics as s3hc_stream / stream_range_data: an empty frame does not end the stream; the
// first failing frame in stream order ends it after every earlier frame's bytes were delivered;
// bytes that never form a complete frame are CORRUPT at finish. The caller keeps the reference's
// final size check (disk_cache.rs:3929-3934) against s3hc_reader_total.
namespace {
struct RSlot {
    s3hc_ctx* ctx = nullptr;   // the device of the slot's queue
    hipStream_t st = nullptr;  // one of the reader's queues (slot i: queue i % queues)
    hipEvent_t ev = nullptr;
    PinnedBuf h_in, h_out;  // h_in: input + tables; h_out: frame results + decoded slots
    DevBuf d_in, d_out, d_blk_out, d_blk_status;
    LbScratch lb;
    uint32_t n = 0;
    std::vector<uint64_t> dst_off;
    hipEvent_t ev2 = nullptr;  // the batch's D2H of decoded bytes
    hipEvent_t ev3 = nullptr;  // the batch's deferred content checksums (second close) read back
    hipEvent_t ev_in = nullptr;  // the batch's input copied out of the reader's (pinned) input buffer
    DevBuf d_v;                // second close: final statuses (i32[n]) and lengths (u32[n])
    PinnedBuf h_v;             // its final statuses
    int state = 0;          // 0 decoding, 1 copying decoded bytes to h_out, 2 ready
    bool ready = false;     // h_out holds the batch's decoded bytes (in stream order)
    bool deferred = false;  // the batch's first close left content checksums to a second close
    bool verdict = false;   // delivered frames still wait for those checksums (before any later byte)
    uint32_t incl = 0;      // frames whose bytes were copied to h_out: [0, incl)
    std::vector<uint32_t> olen;   // first close: lengths
    std::vector<int32_t> st1;     // first close: statuses
    std::vector<uint8_t> pend;    // first close: checksum deferred
    uint64_t out_len = 0;   // bytes of h_out that may be read now
    uint64_t out_pos = 0;   // bytes already read
    uint64_t spec = 0;      // decoded-slot prefix copied to h_out right behind the decode (one round trip)
    bool covered = false;   // the good frames' bytes lie in that prefix: no second copy
    uint64_t R = 0;         // d_out / h_out: frame results (u32 lengths, i32 statuses) in [0, R), slots after
    uint64_t slot = 0;      // decoded-slot bytes of the batch (frame f's slot: [dst_off[f], dst_off[f + 1]))
    int32_t err = 0;        // status of the first failing frame (good < n)
    void reset() {          // (a slot taken from its context's pool: buffers kept, batch state cleared)
        n = 0; state = 0; ready = false; deferred = false; verdict = false; incl = 0; out_len = 0; out_pos = 0;
        spec = 0; covered = false; R = 0; slot = 0; err = 0; dst_off.clear(); st = nullptr;
        olen.clear(); st1.clear(); pend.clear();
    }
    ~RSlot() {
        if (ctx) (void)hipSetDevice(ctx->device);
        if (ev) (void)hipEventDestroy(ev);
        if (ev2) (void)hipEventDestroy(ev2);
        if (ev3) (void)hipEventDestroy(ev3);
        if (ev_in) (void)hipEventDestroy(ev_in);
    }
};
constexpr size_t kReaderPoolMax = 64;  // pooled slots (and queues) per context
// A slot of ctx (its device current): from the context's pool, else new with its two events.
RSlot* rslot_take(s3hc_ctx* c) {
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (!c->rslot_pool.empty()) {
            RSlot* S = (RSlot*)c->rslot_pool.back();
            c->rslot_pool.pop_back();
            S->reset();
            return S;
        }
    }
    std::unique_ptr<RSlot> S(new RSlot);
    S->ctx = c;
    if (hipEventCreateWithFlags(&S->ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&S->ev2, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&S->ev3, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&S->ev_in, hipEventDisableTiming) != hipSuccess) return nullptr;
    return S.release();
}
// A pooled slot keeps buffers up to this size: one GET with large batches or 4 MiB blocks must
// not pin tens of MiB per slot for the life of the process; bigger ones are freed
// when the slot returns to its pool and regrown by the next batch that needs them.
constexpr size_t kReaderPoolKeep = 8u << 20;
void rslot_give(RSlot* S) {  // (nothing of the slot in flight)
    if (!S) return;
    s3hc_ctx* c = S->ctx;
    (void)hipSetDevice(c->device);
    S->h_in.trim(kReaderPoolKeep);
    S->h_out.trim(kReaderPoolKeep);
    S->d_in.trim(kReaderPoolKeep);
    S->d_out.trim(kReaderPoolKeep);
    S->lb.wP.trim(kReaderPoolKeep);
    S->lb.f_bmp.trim(kReaderPoolKeep);
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (c->rslot_pool.size() < kReaderPoolMax) {
            c->rslot_pool.push_back(S);
            return;
        }
    }
    delete S;
}
hipStream_t rqueue_take(s3hc_ctx* c) {  // (device current)
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (!c->rqueue_pool.empty()) {
            hipStream_t q = c->rqueue_pool.back();
            c->rqueue_pool.pop_back();
            return q;
        }
    }
    hipStream_t q = nullptr;
    return hipStreamCreateWithFlags(&q, hipStreamNonBlocking) == hipSuccess ? q : nullptr;
}
void rqueue_give(s3hc_ctx* c, hipStream_t q) {  // (q synchronised)
    if (!q) return;
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (c->rqueue_pool.size() < kReaderPoolMax) {
            c->rqueue_pool.push_back(q);
            return;
        }
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamDestroy(q);
}
}  // namespace
// A reader's pinned input buffer: from its first context's pool (kept up to kReaderPoolKeep).
static PinnedBuf* rin_take(s3hc_ctx* c) {
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (!c->rin_pool.empty()) {
            PinnedBuf* b = (PinnedBuf*)c->rin_pool.back();
            c->rin_pool.pop_back();
            return b;
        }
    }
    return new PinnedBuf;
}
static void rin_give(s3hc_ctx* c, PinnedBuf* b) {  // (no copy out of it in flight)
    if (!b) return;
    b->trim(kReaderPoolKeep);
    {
        std::lock_guard<std::mutex> g(c->rpool_mu);
        if (c->rin_pool.size() < kReaderPoolMax) {
            c->rin_pool.push_back(b);
            return;
        }
    }
    delete b;
}
static void reader_pool_release(s3hc_ctx* c) {
    std::lock_guard<std::mutex> g(c->rpool_mu);
    for (void* p : c->rslot_pool) delete (RSlot*)p;
    c->rslot_pool.clear();
    for (void* p : c->rin_pool) delete (PinnedBuf*)p;
    c->rin_pool.clear();
    (void)hipSetDevice(c->device);
    for (hipStream_t q : c->rqueue_pool) (void)hipStreamDestroy(q);
    c->rqueue_pool.clear();
}

// The frame results a batch's decode wrote (lengths, statuses) decide the copies out of device
// memory, so they are checked before any copy: every status must be one the decoders assign, every
// good frame's length must fit its slot (slot f = [dst_off[f], dst_off[f + 1]), the last one up
// to slot_total), the failing frame's status must be an error. Returns S3HC_OK with *good (frames
// before the first failing one) and *bytes (their decoded bytes), or S3HC_DEVICE: the results are
// not a decode's (the reference's contract turns every problem into an error chunk,
// disk_cache.rs:3873-3934, never a copy of memory no decode wrote).
static int check_batch_results(uint32_t n, const uint32_t* olen, const int32_t* st, const uint64_t* dst_off,
                               uint64_t slot_total, uint32_t* good, uint64_t* bytes) {
    uint32_t g = 0;
    uint64_t b = 0;
    for (; g < n; ++g) {
        const int32_t s = st[g];
        if (s < S3HC_OK || s > S3HC_INVALID_ARG) return fail(S3HC_DEVICE, "decode results: status out of range");
        const uint64_t lo = dst_off[g], hi = g + 1 < n ? dst_off[g + 1] : slot_total;
        // (a frame that failed only its content checksum is delivered before the error: its
        // length must fit its slot as well)
        if ((s == S3HC_OK || s == S3HC_CHECKSUM) && (lo > hi || hi > slot_total || olen[g] > hi - lo))
            return fail(S3HC_DEVICE, "decode results: frame length beyond its slot");
        if (s != S3HC_OK) break;
        b += olen[g];
    }
    *good = g;
    *bytes = b;
    return S3HC_OK;
}
extern "C" int s3hc_diag_check_batch_results(uint32_t n, const uint32_t* olen, const int32_t* status,
                                             const uint64_t* dst_off, uint64_t slot_total, uint32_t* good,
                                             uint64_t* bytes) {
    if ((n && (!olen || !status || !dst_off)) || !good || !bytes) return fail(S3HC_INVALID_ARG, "bad arguments");
    return check_batch_results(n, olen, status, dst_off, slot_total, good, bytes);
}

// Host-time accounting of the reader (S3HC_HOST_TRACE=1, diagnostics: printed at close)
struct ReaderTrace {
    enum { FEED, WALK, STAGE, SUBMIT, ISSUE, WAIT, DELIVER, N };
    bool on = false;
    double t[N] = {};
    uint64_t batches = 0;
};
struct RTimer {
    ReaderTrace& tr;
    int k;
    double t0;
    RTimer(ReaderTrace& r, int kk) : tr(r), k(kk), t0(r.on ? host_us() : 0.0) {}
    ~RTimer() { if (tr.on) tr.t[k] += host_us() - t0; }
};

struct s3hc_reader {
    ~s3hc_reader();
    s3hc_ctx* ctx;                  // ctxs[0]
    std::vector<s3hc_ctx*> ctxs;    // the reader's devices (queue q on ctxs[q % ctxs.size()])
    ReaderTrace tr;
    size_t batch_bytes;
    size_t batch_max;           // batch limit while earlier batches are in flight (>= batch_bytes)
    std::vector<hipStream_t> queues;  // `depth` HIP queues per device
    std::vector<RSlot*> slots;        // S3HC_READER_SLOTS batches per queue (default 1; more queue
                                      // a queue's next batch behind its running one: measured slower)
    std::vector<int> inflight;  // slot indices in stream order (head may be ready / being read)
    // buffered input, pinned (each batch's input is copied to the device straight out of it; the
    // bytes a submitted batch reads are never moved or freed before its ev_in): undecoded bytes
    // start at in_head (a frame boundary)
    struct Input {
        PinnedBuf* b = nullptr;  // (from the first context's pool)
        size_t n = 0;
        uint8_t* data() const { return b->p; }
        size_t size() const { return n; }
        void clear() { n = 0; }
    } in;
    size_t in_head = 0;
    bool finished = false;
    int error = S3HC_OK;        // reported once every byte before it was read
    std::string error_msg;
    uint64_t total = 0;
};

// Queue frames [0, nf) of W (all complete) as one batch on slot s. The host walk already knows
// every frame and block, so its tables go up with the input (one copy) and the device runs the
// block decode and one frame-close launch (lengths, content xxh32, EndMark checks).
static int reader_submit(s3hc_reader* r, RSlot& S, const HWalk& W, size_t nf) {
    const HFrame& F0 = W.frames[0];
    const bool all = nf >= W.frames.size();
    const size_t end = all ? W.end : W.frames[nf].pos;
    const size_t nin = end - F0.pos;
    const uint32_t n = (uint32_t)nf;
    const uint32_t nbk = (all ? (uint32_t)W.blocks.size() : W.frames[nf].blk0) - F0.blk0;
    const uint64_t slot = (all ? W.slot_total : W.frames[nf].out_off) - F0.out_off;
    S.n = n;
    S.slot = slot;
    S.dst_off.resize(n);
    // frames of blocks > 64 KiB with a content checksum (the reference's own cache files: one
    // block of up to 4 MiB per frame) may have no hash from their decode (spread execution): their
    // checksums are verified behind the delivered bytes by a second close (stream_range_data
    // order, disk_cache.rs:3884-3898)
    S.deferred = false;
    for (uint32_t f = 0; f < n; ++f) S.deferred |= W.frames[f].bmax > 65536u && (W.frames[f].flg & 0x04u);
    std::vector<DecUnit> units;
    for (uint32_t f = 0; f < n; ++f) {
        const HFrame& F = W.frames[f];
        const uint64_t fend = f + 1 < W.frames.size() ? W.frames[f + 1].out_off : W.slot_total;
        if (fend - F.out_off > 0xFFFFFFFFull) return fail(S3HC_UNSUPPORTED, "frame too large for one batch");
        S.dst_off[f] = F.out_off - F0.out_off;
        if (!F.nblk) continue;
        if (!(F.flg & 0x20)) units.push_back(DecUnit{F.blk0 - F0.blk0, F.nblk});
        else for (uint32_t k = 0; k < F.nblk; ++k) units.push_back(DecUnit{F.blk0 - F0.blk0 + k, 1});
    }
    const uint32_t nu = (uint32_t)units.size();
    // meta: frame_off u64[n] | blk_base u64[n] | out_off u64[n] | nblk u32[n] | want u32[n] |
    //       blocks DecBlock[nbk] | units DecUnit[nu]   (sections 16-byte aligned)
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_fo = 0, o_bb = al(8ull * n), o_oo = o_bb + al(8ull * n), o_nb = o_oo + al(8ull * n),
                 o_w = o_nb + al(4ull * n), o_blk = o_w + al(4ull * n), o_u = o_blk + al(sizeof(DecBlock) * nbk),
                 nmeta = o_u + al(sizeof(DecUnit) * nu);
    // two host-to-device copies per batch: the input straight out of the reader's pinned input
    // buffer, then (256-byte aligned) the tables from the slot's
    const size_t o_meta = (nin + 255) & ~(size_t)255;
    HIPCHK(S.h_in.ensure(nmeta));
    uint8_t* m = S.h_in.p;
    for (uint32_t f = 0; f < n; ++f) {
        const HFrame& F = W.frames[f];
        ((uint64_t*)(m + o_fo))[f] = F.pos - F0.pos;
        ((uint64_t*)(m + o_bb))[f] = F.blk0 - F0.blk0;
        ((uint64_t*)(m + o_oo))[f] = S.dst_off[f];
        ((uint32_t*)(m + o_nb))[f] = F.nblk;
        ((uint32_t*)(m + o_w))[f] = F.want;
    }
    DecBlock* mb = (DecBlock*)(m + o_blk);
    for (uint32_t k = 0; k < nbk; ++k) {
        DecBlock D = W.blocks[F0.blk0 + k];
        D.src_off -= F0.pos;
        D.dst_off -= F0.out_off;
        D.frame -= (uint32_t)(&F0 - W.frames.data());
        mb[k] = D;
    }
    const uint64_t tok_entries = assign_tok_slots(mb, nbk);
    if (nu) memcpy(m + o_u, units.data(), sizeof(DecUnit) * nu);
    hipStream_t st = S.st;
    HIPCHK(hipSetDevice(S.ctx->device));
    RTimer T_(r->tr, ReaderTrace::SUBMIT);
    ++r->tr.batches;
    HIPCHK(S.d_in.ensure(o_meta + nmeta + 64));
    // one device-to-host copy per batch: the frame results (lengths, statuses and, deferred,
    // the first close's pending flags), then (256-byte aligned) the slots
    S.R = ((S.deferred ? 12ull : 8ull) * n + 255) & ~255ull;
    HIPCHK(S.d_out.ensure(S.R + slot + 64));
    if (S.deferred) {
        HIPCHK(S.d_v.ensure(8ull * n + 16));
        HIPCHK(S.h_v.ensure(4ull * n + 16));
    }
    HIPCHK(S.d_blk_out.ensure(4ull * nbk + 16));
    HIPCHK(S.d_blk_status.ensure(4ull * nbk + 16));
    {
        // large blocks of the batch (the host walk knows every block)
        HIPCHK(prepare_host_launch(S.lb, mb, nbk, units.data(), nu, tok_entries));
    }
    HIPCHK(hipMemcpyAsync(S.d_in.p, r->in.data() + r->in_head + F0.pos, nin, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.d_in.as<uint8_t>() + o_meta, S.h_in.p, nmeta, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(S.ev_in, st));
    const uint8_t* src = S.d_in.as<uint8_t>();
    const uint8_t* dm = S.d_in.as<uint8_t>() + o_meta;
    const DecBlock* d_blk = (const DecBlock*)(dm + o_blk);
    uint32_t* d_olen = S.d_out.as<uint32_t>();
    int32_t* d_st = (int32_t*)(S.d_out.as<uint8_t>() + 4ull * n);
    uint8_t* d_slots = S.d_out.as<uint8_t>() + S.R;
    KTimer T(S.ctx, st);
    T.begin("decode");
    const uint64_t* bh = nullptr;
    HIPCHK(decode_launch(&S.lb, src, d_slots, d_blk, (const DecUnit*)(dm + o_u), nu, S.d_blk_out.as<uint32_t>(),
                         S.d_blk_status.as<int32_t>(), st, &bh, nullptr, 0));
    T.end();
    T.begin("dec_close");
    uint32_t* d_pend = S.deferred ? (uint32_t*)(S.d_out.as<uint8_t>() + 8ull * n) : nullptr;
    HIPCHK(launch_dframe_close(src, (const uint64_t*)(dm + o_fo), (const uint64_t*)(dm + o_bb),
                               (const uint32_t*)(dm + o_nb), d_blk, S.d_blk_out.as<uint32_t>(),
                               S.d_blk_status.as<int32_t>(), bh, d_slots, (const uint64_t*)(dm + o_oo),
                               (const uint32_t*)(dm + o_w), n, nullptr, d_st, d_olen, nullptr, st, d_pend));
    T.end();
    // speculative copy of the decoded slots behind the decode, in the same round trip: frames of
    // 64 KiB blocks fill their slots, so the prefix is the batch's output; a frame whose slot is
    // its block capacity (BD 0x70: 4 MiB) only gets the prefix a 4:1 ratio can fill
    S.spec = std::min<uint64_t>(slot, std::max<uint64_t>(4ull * nin, 1ull << 20));
    HIPCHK(S.h_out.ensure(S.R + S.spec + 16));
    HIPCHK(hipMemcpyAsync(S.h_out.p, S.d_out.p, S.R + S.spec, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(S.ev, st));
    if (S.deferred) {
        // the second close: the same frames with every content checksum, behind the first
        // close's results on the queue (the host delivers the bytes meanwhile)
        T.begin("dec_verify");
        int32_t* d_hst = S.d_v.as<int32_t>();
        HIPCHK(launch_dframe_close(src, (const uint64_t*)(dm + o_fo), (const uint64_t*)(dm + o_bb),
                                   (const uint32_t*)(dm + o_nb), d_blk, S.d_blk_out.as<uint32_t>(),
                                   S.d_blk_status.as<int32_t>(), bh, d_slots, (const uint64_t*)(dm + o_oo),
                                   (const uint32_t*)(dm + o_w), n, nullptr, d_hst, (uint32_t*)(d_hst + n), nullptr,
                                   st));
        T.end();
        HIPCHK(hipMemcpyAsync(S.h_v.p, d_hst, 4ull * n, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(S.ev3, st));
    }
    S.state = 0;
    S.ready = false;
    S.covered = false;
    S.verdict = false;
    r->in_head += end;
    return S3HC_OK;
}

// Form and queue batches while a slot is free and complete frames are buffered.
static int reader_pump(s3hc_reader* r) {
    while (r->inflight.size() < r->slots.size() && r->in_head < r->in.size()) {
        // walk only what one batch can use (a frame cut by the limit counts as incomplete);
        // the whole buffer only when no frame completes within it (frames larger than that)
        const size_t avail = r->in.size() - r->in_head;
        // an idle pipeline starts with batch_bytes (time to first byte); behind running batches
        // a batch may take up to batch_max of the buffered frames
        const size_t want = r->inflight.empty() ? r->batch_bytes : r->batch_max;
        const size_t lim = std::min(avail, want + ((size_t)8 << 20));
        HWalk W;
        size_t nf;
        {
            RTimer T_(r->tr, ReaderTrace::WALK);
            // frames up to `want` bytes and one past it: the batch never takes more
            walk_frames(r->in.data() + r->in_head, lim, W, true, false, want);
            nf = W.frames.size();
            if (nf && W.last_incomplete) nf--;  // (stream mode leaves incomplete frames unwalked)
            if (nf == 0 && lim < avail) {
                W = HWalk();
                walk_frames(r->in.data() + r->in_head, avail, W, true, false, want);
                nf = W.frames.size();
                if (nf && W.last_incomplete) nf--;
            }
        }
        if (nf == 0) {
            if (W.tail_status != S3HC_OK && W.frames.empty() && !r->error) {  // bad header: nothing decodable
                r->error = W.tail_status;
                r->error_msg = "malformed frame header";
                r->in.clear();
                r->in_head = 0;
            }
            return S3HC_OK;
        }
        // batch = frames up to batch_bytes of input (at least one)
        size_t k = 1;
        while (k < nf && W.frames[k].pos - W.frames[0].pos < want) ++k;
        if (k < nf || W.end - W.frames[0].pos >= r->batch_bytes || r->finished) {
            // full batch (or all that will ever come)
        } else if (!r->inflight.empty()) {
            return S3HC_OK;  // wait for more input to fill the batch while others run
        }
        // a free slot on the queue with the fewest batches in flight
        std::vector<bool> used(r->slots.size(), false);
        std::vector<int> busy(r->queues.size(), 0);
        for (int i : r->inflight) {
            used[i] = true;
            ++busy[(size_t)i % r->queues.size()];
        }
        int s = -1;
        for (int i = 0; i < (int)r->slots.size(); ++i)
            if (!used[i] && (s < 0 || busy[(size_t)i % r->queues.size()] < busy[(size_t)s % r->queues.size()])) s = i;
        int rc = reader_submit(r, *r->slots[s], W, k);
        if (rc) return rc;
        r->inflight.push_back(s);
    }
    return S3HC_OK;
}

// Decode of slot S finished: queue the D2H of its good frames' bytes (stream order) into its
// pinned output buffer. A failing frame ends the stream after them (applied when S is the head).
static int reader_issue_copy(RSlot& S, ReaderTrace& tr) {
    RTimer T_(tr, ReaderTrace::ISSUE);
    HIPCHK(hipSetDevice(S.ctx->device));
    // (the results head h_out; they are copied before h_out may be reallocated below)
    const uint32_t n = S.n;
    S.olen.assign((const uint32_t*)S.h_out.p, (const uint32_t*)S.h_out.p + n);
    S.st1.assign((const int32_t*)(S.h_out.p + 4ull * n), (const int32_t*)(S.h_out.p + 4ull * n) + n);
    const std::vector<uint32_t>& olen = S.olen;
    uint32_t good = 0;
    uint64_t bytes = 0;
    if (int rc = check_batch_results(n, olen.data(), S.st1.data(), S.dst_off.data(), S.slot, &good, &bytes)) return rc;
    // a frame that failed only its content checksum is delivered before the error, as lz4_flex's
    // FrameDecoder returns a frame's bytes before it checks the checksum at the EndMark
    // (stream_range_data, disk_cache.rs:3884-3898)
    uint32_t incl = good;
    if (good < n && S.st1[good] == S3HC_CHECKSUM) {
        bytes += olen[good];
        incl = good + 1;
    }
    if (bytes > S.slot) return fail(S3HC_DEVICE, "decode results: batch output beyond its slots");
    S.err = good < n ? S.st1[good] : 0;
    // frames [0, incl) are copied; of them, the bytes up to and including the first frame whose
    // checksum the first close deferred may be read now, the rest once the second close is in
    uint32_t deliver = incl;
    S.pend.assign(n, 0);
    if (S.deferred) {
        const uint32_t* pd = (const uint32_t*)(S.h_out.p + 8ull * n);
        for (uint32_t f = 0; f < n; ++f) {
            if (pd[f] > 1u || (pd[f] && S.st1[f] != S3HC_OK)) return fail(S3HC_DEVICE, "decode results: bad pending flag");
            S.pend[f] = (uint8_t)pd[f];
        }
        for (uint32_t f = 0; f < incl; ++f)
            if (S.pend[f]) {
                deliver = f + 1;
                S.verdict = true;
                break;
            }
    }
    uint64_t now = 0;
    for (uint32_t f = 0; f < deliver; ++f) now += olen[f];
    // frames decode into slots of their block capacity; when every frame but the last filled
    // its slot (the normal case) the good output is already contiguous: one copy, or none when
    // the speculative prefix already holds it
    bool packed = true;
    for (uint32_t f = 0; f + 1 < incl; ++f) packed &= S.dst_off[f] + olen[f] == S.dst_off[f + 1];
    S.incl = incl;
    S.out_len = now;
    S.out_pos = 0;
    S.state = 1;
    if (packed && bytes <= S.spec) {
        S.covered = true;
        return S3HC_OK;
    }
    const uint8_t* d_slots = S.d_out.as<uint8_t>() + S.R;
    if (packed) {  // the rest beyond the prefix (h_out keeps the results and the prefix it holds)
        HIPCHK(S.h_out.ensure_keep(S.R + bytes + 16, S.R + S.spec));
        HIPCHK(hipMemcpyAsync(S.h_out.p + S.R + S.spec, d_slots + S.spec, bytes - S.spec, hipMemcpyDeviceToHost,
                              S.st));
        HIPCHK(hipEventRecord(S.ev2, S.st));
        return S3HC_OK;
    }
    HIPCHK(S.h_out.ensure(S.R + bytes + 16));
    {
        uint64_t o = 0;
        for (uint32_t f = 0; f < incl; ++f) {
            if (olen[f]) HIPCHK(hipMemcpyAsync(S.h_out.p + S.R + o, d_slots + S.dst_off[f], olen[f],
                                               hipMemcpyDeviceToHost, S.st));
            o += olen[f];
        }
    }
    HIPCHK(hipEventRecord(S.ev2, S.st));
    return S3HC_OK;
}
static bool reader_copy_done(RSlot& S) { return S.state == 1 && (S.covered || hipEventQuery(S.ev2) == hipSuccess); }

// Queue the D2H of every batch whose decode has finished (any order: separate queues).
static int reader_advance(s3hc_reader* r) {
    for (int i : r->inflight) {
        RSlot& S = *r->slots[i];
        if (S.state == 0 && hipSetDevice(S.ctx->device) == hipSuccess && hipEventQuery(S.ev) == hipSuccess) {
            int rc = reader_issue_copy(S, r->tr);
            if (rc) return rc;
        }
    }
    return S3HC_OK;
}

// Every context of a reader locked in one global order (ascending context address, whatever
// order the caller listed them in: two readers over [c0, c1] and [c1, c0] cannot deadlock); the
// reader's per-slot scratch and the contexts' timing state are used under them. unlock()/relock()
// bracket host waits on a batch's events, so a wait on one device never holds the other devices'
// contexts (their aggregator lanes and single-context readers keep running).
struct ReaderLock {
    std::vector<std::mutex*> mus;
    bool held = false;
    explicit ReaderLock(s3hc_reader* r) {
        for (auto* c : r->ctxs) mus.push_back(&c->mu);
        std::sort(mus.begin(), mus.end(), std::less<std::mutex*>());
        relock();
    }
    void relock() {
        for (auto* m : mus) m->lock();
        held = true;
    }
    void unlock() {
        if (!held) return;
        for (auto it = mus.rbegin(); it != mus.rend(); ++it) (*it)->unlock();
        held = false;
    }
    ~ReaderLock() { unlock(); }
};
// Wait for a slot's event with the contexts unlocked (the slot and its queue are the reader's own).
static int reader_wait(RSlot& S, hipEvent_t e, ReaderLock& g, ReaderTrace& tr) {
    HIPCHK(hipSetDevice(S.ctx->device));
    if (hipEventQuery(e) == hipSuccess) return S3HC_OK;
    RTimer T_(tr, ReaderTrace::WAIT);
    g.unlock();
    const hipError_t e2 = hipEventSynchronize(e);
    g.relock();
    HIPCHK(e2);
    return S3HC_OK;
}

// The stream ends inside the head batch with status err: every later batch is dropped (its queue
// synchronised first), and so is the buffered input; the head's readable bytes still come first.
static void reader_end_after_head(s3hc_reader* r, int err, const char* msg) {
    r->error = err;
    r->error_msg = msg;
    for (size_t k = 1; k < r->inflight.size(); ++k) {
        RSlot& L = *r->slots[r->inflight[k]];
        (void)hipSetDevice(L.ctx->device);
        (void)hipStreamSynchronize(L.st);
        L.state = 0;
        L.ready = false;
        L.verdict = false;
    }
    r->inflight.resize(1);
    r->in.clear();
    r->in_head = 0;
}

// Wait until the oldest batch's decoded bytes are in its pinned output buffer.
static int reader_complete(s3hc_reader* r, ReaderLock& g) {
    RSlot& S = *r->slots[r->inflight.front()];
    if (S.state == 0) {
        if (int rc = reader_wait(S, S.ev, g, r->tr)) return rc;
        int rc = reader_issue_copy(S, r->tr);
        if (rc) return rc;
    }
    if (!S.covered)
        if (int rc = reader_wait(S, S.ev2, g, r->tr)) return rc;
    S.state = 2;
    S.ready = true;
    // a failing frame of the first close ends the stream inside this batch whatever the deferred
    // checksums say (they can only end it earlier)
    if (S.err) reader_end_after_head(r, S.err, S.err == S3HC_CHECKSUM ? "content checksum mismatch" : "frame decode failed");
    return S3HC_OK;
}

// The head batch's readable bytes are read and some of its frames wait for their deferred
// content checksums: take the second close's statuses. The readable bytes grow to the next
// pending frame (or the batch's end), or the stream ends with S3HC_CHECKSUM after the bytes of
// the first frame whose checksum failed — that frame's own bytes included, as lz4_flex reads them.
static int reader_verdict(s3hc_reader* r, RSlot& S, ReaderLock& g) {
    if (int rc = reader_wait(S, S.ev3, g, r->tr)) return rc;
    const uint32_t n = S.n;
    const int32_t* hv = (const int32_t*)S.h_v.p;
    uint32_t g2 = 0;
    for (; g2 < n; ++g2) {
        const int32_t s = hv[g2];
        if (s < S3HC_OK || s > S3HC_INVALID_ARG) return fail(S3HC_DEVICE, "verify results: status out of range");
        // a frame the first close did not defer keeps its status; a deferred one may only fail its checksum
        if (S.pend[g2] ? (s != S3HC_OK && s != S3HC_CHECKSUM) : s != S.st1[g2])
            return fail(S3HC_DEVICE, "verify results: status differs from the first close");
        if (s != S3HC_OK) break;
    }
    uint32_t incl = g2 < n && hv[g2] == S3HC_CHECKSUM ? g2 + 1 : g2;
    if (incl > S.incl) incl = S.incl;  // (never more than the first close allowed and copied)
    S.verdict = false;  // (every pending frame of the batch is resolved now)
    uint64_t len = 0;
    for (uint32_t f = 0; f < incl; ++f) len += S.olen[f];
    if (len < S.out_pos) return fail(S3HC_DEVICE, "verify results: fewer bytes than already read");
    S.out_len = len;
    uint32_t good1 = 0;  // the first close's first failing frame
    while (good1 < n && S.st1[good1] == S3HC_OK) ++good1;
    if (g2 < good1) {  // a deferred checksum failed before it: the stream ends there instead
        S.err = S3HC_CHECKSUM;
        reader_end_after_head(r, S3HC_CHECKSUM, "content checksum mismatch");
    }
    return S3HC_OK;
}

static int reader_new(s3hc_ctx* const* ctxs, int nctx, size_t batch_bytes, int depth, s3hc_reader** out) {
    if (!ctxs || nctx < 1 || !out || depth < 1 || depth > 16 || batch_bytes == 0) return fail(S3HC_INVALID_ARG, "bad arguments");
    for (int i = 0; i < nctx; ++i) {
        if (!ctxs[i]) return fail(S3HC_INVALID_ARG, "NULL context");
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return fail(S3HC_INVALID_ARG, "a context is listed twice");
    }
    std::unique_ptr<s3hc_reader> r(new s3hc_reader);
    r->ctx = ctxs[0];
    r->ctxs.assign(ctxs, ctxs + nctx);
    for (auto* c : r->ctxs) ctx_retain(c);  // released by ~s3hc_reader
    r->in.b = rin_take(r->ctx);
    ReaderLock lk(r.get());
    r->batch_bytes = batch_bytes;
    r->batch_max = batch_bytes;
    const long long per = std::min<long long>(4, std::max<long long>(1, knob(KN_READER_SLOTS)));
    const size_t nq = (size_t)depth * (size_t)nctx;
    r->queues.assign(nq, nullptr);
    r->slots.assign(nq * (size_t)per, nullptr);
    r->tr.on = knob_on(KN_HOST_TRACE);
    for (size_t q = 0; q < nq; ++q) {
        s3hc_ctx* c = ctxs[q % (size_t)nctx];
        HIPCHK(hipSetDevice(c->device));
        if (!(r->queues[q] = rqueue_take(c))) return fail(S3HC_DEVICE, "reader queue");
    }
    for (size_t i = 0; i < r->slots.size(); ++i) {
        s3hc_ctx* c = ctxs[(i % nq) % (size_t)nctx];
        HIPCHK(hipSetDevice(c->device));
        if (!(r->slots[i] = rslot_take(c))) return fail(S3HC_DEVICE, "reader slot");
        r->slots[i]->st = r->queues[i % nq];
    }
    *out = r.release();
    return S3HC_OK;
}
extern "C" int s3hc_reader_open(s3hc_ctx* ctx, size_t batch_bytes, int depth, s3hc_reader** out) {
    return guarded([&]() -> int { return reader_new(&ctx, 1, batch_bytes, depth, out); });
}
extern "C" int s3hc_reader_open_multi(s3hc_ctx* const* ctxs, int nctx, size_t batch_bytes, int depth, s3hc_reader** out) {
    return guarded([&]() -> int { return reader_new(ctxs, nctx, batch_bytes, depth, out); });
}
extern "C" int s3hc_reader_set_batch_max(s3hc_reader* r, size_t max_bytes) {
    return guarded([&]() -> int {
        if (!r || max_bytes < r->batch_bytes) return fail(S3HC_INVALID_ARG, "bad arguments");
        r->batch_max = max_bytes;
        return S3HC_OK;
    });
}
extern "C" int s3hc_reader_feed(s3hc_reader* r, const uint8_t* src, size_t n) {
    return guarded([&]() -> int {
        if (!r || (!src && n)) return fail(S3HC_INVALID_ARG, "bad arguments");
        if (r->finished) return fail(S3HC_INVALID_ARG, "reader already finished");
        if (r->error) return S3HC_OK;  // the stream has ended with an error; input is ignored
        auto& in = r->in;
        const bool compact = r->in_head && r->in_head >= in.n / 2;  // drop consumed input (amortized)
        const bool grow = (compact ? in.n - r->in_head : in.n) + n > in.b->cap;
        if (compact || grow) {
            // the bytes move (or the buffer is replaced): every submitted batch's input copy first
            RTimer T_(r->tr, ReaderTrace::FEED);
            for (int i : r->inflight) {
                RSlot& S = *r->slots[i];
                HIPCHK(hipSetDevice(S.ctx->device));
                HIPCHK(hipEventSynchronize(S.ev_in));
            }
        }
        if (compact) {
            RTimer T_(r->tr, ReaderTrace::FEED);
            memmove(in.b->p, in.b->p + r->in_head, in.n - r->in_head);
            in.n -= r->in_head;
            r->in_head = 0;
        }
        {
            RTimer T_(r->tr, ReaderTrace::FEED);
            HIPCHK(in.b->ensure_keep(in.n + n, in.n));
            par_memcpy(in.b->p + in.n, src, n);
            in.n += n;
        }
        ReaderLock g(r);
        int rc = reader_advance(r);
        if (rc) return rc;
        return reader_pump(r);
    });
}
extern "C" int s3hc_reader_finish(s3hc_reader* r) {
    return guarded([&]() -> int {
        if (!r) return fail(S3HC_INVALID_ARG, "bad arguments");
        r->finished = true;
        return S3HC_OK;
    });
}
extern "C" int s3hc_reader_read(s3hc_reader* r, uint8_t* dst, size_t cap, size_t* n) {
    return guarded([&]() -> int {
        if (!r || !n || (!dst && cap)) return fail(S3HC_INVALID_ARG, "bad arguments");
        *n = 0;
        if (!cap) return S3HC_OK;
        // a ready head batch is delivered without the context lock (the copy is the caller's
        // Bytes::copy_from_slice; concurrent readers must not serialize on it)
        if (!r->inflight.empty() && r->slots[r->inflight.front()]->ready) {
            RSlot& S = *r->slots[r->inflight.front()];
            if (S.out_pos < S.out_len) {
                RTimer T_(r->tr, ReaderTrace::DELIVER);
                const size_t k = (size_t)std::min<uint64_t>(cap, S.out_len - S.out_pos);
                if (k) par_memcpy(dst, S.h_out.p + S.R + S.out_pos, k);
                S.out_pos += k;
                r->total += k;
                *n = k;
                if (S.out_pos < S.out_len) return S3HC_OK;
            }
        }
        ReaderLock g(r);
        for (;;) {
            if (!r->inflight.empty() && r->slots[r->inflight.front()]->ready) {
                RSlot& S = *r->slots[r->inflight.front()];
                if (*n == 0 && S.out_pos < S.out_len) {
                    RTimer T_(r->tr, ReaderTrace::DELIVER);
                    const size_t k = (size_t)std::min<uint64_t>(cap, S.out_len - S.out_pos);
                    if (k) par_memcpy(dst, S.h_out.p + S.R + S.out_pos, k);
                    S.out_pos += k;
                    r->total += k;
                    *n = k;
                }
                if (S.out_pos == S.out_len && S.verdict) {
                    // read up to a frame whose content checksum is still being verified: nothing
                    // after it before the verdict (returned bytes first; a wait only when asked again)
                    if (*n) return S3HC_OK;
                    int rc = reader_verdict(r, S, g);
                    if (rc) return rc;
                    continue;
                }
                if (S.out_pos == S.out_len) {  // slot free again: queue the next batch
                    S.ready = false;
                    S.state = 0;
                    r->inflight.erase(r->inflight.begin());
                    if (!r->error) {
                        int rc = reader_pump(r);
                        if (rc) return rc;
                    }
                }
                if (*n) return S3HC_OK;
                continue;
            }
            if (!r->error) {
                int rc = reader_advance(r);
                if (rc) return rc;
                rc = reader_pump(r);
                if (rc) return rc;
            }
            if (r->inflight.empty()) {
                if (r->error) return fail(r->error, r->error_msg);
                if (r->finished && r->in_head < r->in.size()) {
                    r->error = S3HC_CORRUPT;
                    r->error_msg = "truncated frame at end of stream";
                    return fail(r->error, r->error_msg);
                }
                return S3HC_OK;  // needs more input, or end of stream
            }
            // the oldest batch is still running: wait for it only when the pipeline is full, the
            // input is finished or it is already done; otherwise ask the caller for more input
            RSlot& H = *r->slots[r->inflight.front()];
            const bool done = reader_copy_done(H);
            if (!done && r->inflight.size() < r->slots.size() && !r->finished && !r->error) return S3HC_OK;
            int rc = reader_complete(r, g);
            if (rc) return rc;
        }
    });
}
extern "C" uint64_t s3hc_reader_total(const s3hc_reader* r) { return r ? r->total : 0; }
// Give the queues (synchronised) and slots back to their contexts' pools.
s3hc_reader::~s3hc_reader() {
    const size_t nc = ctxs.size();
    for (size_t q = 0; q < queues.size(); ++q)
        if (queues[q]) {
            (void)hipSetDevice(ctxs[q % nc]->device);
            (void)hipStreamSynchronize(queues[q]);
        }
    for (RSlot* S : slots) rslot_give(S);
    for (size_t q = 0; q < queues.size(); ++q)
        if (queues[q]) rqueue_give(ctxs[q % nc], queues[q]);
    rin_give(ctx, in.b);  // (every queue synchronised above)
    for (auto* c : ctxs) ctx_release(c);  // (the last reference frees a destroyed context)
}
extern "C" void s3hc_reader_close(s3hc_reader* r) {
    if (!r) return;
    if (r->tr.on) {
        static const char* nm[] = {"feed", "walk", "stage", "submit", "issue", "wait", "deliver"};
        fprintf(stderr, "[s3hc reader] batches %llu us/batch:", (unsigned long long)r->tr.batches);
        for (int k = 0; k < ReaderTrace::N; ++k)
            fprintf(stderr, " %s %.1f", nm[k], r->tr.t[k] / (double)std::max<uint64_t>(1, r->tr.batches));
        fprintf(stderr, "\n");
    }
    delete r;
}
