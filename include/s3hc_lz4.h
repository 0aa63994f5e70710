/*
 * s3hc_lz4.h — C ABI of the MI355X LZ4 frame engine (libs3hc_lz4.so).
 *
 * Drop-in boundary for the LZ4 codec path of aws-samples/sample-s3-hybrid-cache
 * (crate s3-proxy 2.6.0). The reference path is Rust: CompressionHandler in
 * src/compression.rs plus two places where src/disk_cache.rs drives lz4_flex directly.
 * Every entry point below names the reference item (file:line) it replaces; the Rust
 * binding a maintainer would add is in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes, caller-owned buffers, no exceptions across the
 * boundary, int status (S3HC_*), and a thread-local message via s3hc_last_error().
 * Errors follow the reference's contract: any decode failure is an error for the whole
 * call (ProxyError::CompressionError / CacheError, src/error.rs:19-23) and the caller
 * treats it as a cache miss.
 *
 * Every compute entry point runs on the GPU. There is no CPU codec in this library:
 * without a usable HIP device s3hc_create() fails with S3HC_DEVICE.
 */
#ifndef S3HC_LZ4_H
#define S3HC_LZ4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define S3HC_OK 0
#define S3HC_CORRUPT 1        /* bad magic/header/block/offset, truncated frame */
#define S3HC_CHECKSUM 2       /* content or block xxh32 mismatch */
#define S3HC_DST_TOO_SMALL 3  /* caller buffer too small */
#define S3HC_UNSUPPORTED 4    /* dictionary id, legacy/skippable frame, ... */
#define S3HC_DEVICE 5         /* HIP runtime error / no device */
#define S3HC_INVALID_ARG 6
#define S3HC_NO_MEMORY 7      /* a host or device allocation failed (no exception crosses this ABI) */

/* Frame layout policies for s3hc_compress_frame. */
#define S3HC_BLK_AUTO_LZ4FLEX 0  /* lz4_flex FrameEncoder BlockSize::Auto: one frame, BD by input size */
#define S3HC_BLK_64K_PER_FRAME 1 /* one BD=0x40 frame per 64 KiB of input (GPU batch format) */
#define S3HC_BLK_LZ4FLEX_COMPAT 2 /* Auto layout with block payloads byte-identical to lz4_flex's
                                     greedy compressor as restated in oracle/ (slower; see below) */

typedef struct s3hc_ctx s3hc_ctx;
typedef struct s3hc_stream s3hc_stream;
typedef struct s3hc_plan s3hc_plan;

/* ---- context -------------------------------------------------------------- */
/* One context per device; internally locked, safe to share between threads (the
 * reference calls the codec from many spawn_blocking threads, http_proxy.rs:11608). */
int s3hc_create(s3hc_ctx** out, int device);
int s3hc_device_count(void);
void s3hc_destroy(s3hc_ctx* ctx);
const char* s3hc_last_error(void);
const char* s3hc_version(void);

/* Diagnostic switches and checks (no reference counterpart) are declared in s3hc_lz4_diag.h. */

/* Largest framed size any s3hc_compress_* call can produce for n input bytes. */
size_t s3hc_frame_bound(size_t n);

/* ---- whole-buffer codec (host buffers) ------------------------------------ */
/* Replaces compress_with_algorithm(data, Lz4) (compression.rs:530-591) and the
 * FrameEncoder in flush_batch (disk_cache.rs:1826-1846): an LZ4 frame with independent
 * blocks and an xxh32 content checksum. A block whose compressed form is not smaller than
 * its input is written stored, as lz4_flex does. *was_compressed is 1 (the reference tags
 * every such frame "compressed" even when blocks end up stored). */
int s3hc_compress_frame(s3hc_ctx* ctx, const uint8_t* src, size_t n, int policy,
                        uint8_t* dst, size_t cap, size_t* out_len, int* was_compressed);

/* Replaces CompressionHandler::encode_store_mode_frame (compression.rs:326-368):
 * byte-identical output (BD 0x70, stored blocks of <= 4 MiB, xxh32 content checksum). */
int s3hc_store_mode_frame(s3hc_ctx* ctx, const uint8_t* src, size_t n,
                          uint8_t* dst, size_t cap, size_t* out_len);

/* Upper bound of the decoded size of concatenated frames (walks headers only, host). */
int s3hc_decompressed_bound(const uint8_t* src, size_t n, size_t* bound);

/* Replaces CompressionHandler::decompress_data (compression.rs:463-502): decode
 * concatenated frames; a frame that yields no bytes ends the loop (Ok(0) => break).
 * Device scratch follows the decoded size (frames are decoded in passes of <= 2 GiB of
 * output slots; a block reserves min(frame block size, 255 x its compressed size)). */
int s3hc_decompress_frames(s3hc_ctx* ctx, const uint8_t* src, size_t n,
                           uint8_t* dst, size_t cap, size_t* out_len);
/* The same into a library-allocated buffer of exactly the decoded size (the reference returns
 * an owned Vec<u8>, grown by read_to_end); release it with s3hc_buffer_free. */
int s3hc_decompress_frames_alloc(s3hc_ctx* ctx, const uint8_t* src, size_t n,
                                 uint8_t** out, size_t* out_len);
void s3hc_buffer_free(uint8_t* p);

/* ---- streaming decoder (stream_range_data, disk_cache.rs:3850-3935) ------- */
/* Feed compressed bytes in any pieces; read decoded bytes frame by frame.
 * s3hc_stream_read returns 0 bytes when it needs more input; after
 * s3hc_stream_finish it returns 0 bytes at end of stream. */
int s3hc_stream_open(s3hc_ctx* ctx, s3hc_stream** out);
int s3hc_stream_feed(s3hc_stream* s, const uint8_t* src, size_t n);
int s3hc_stream_finish(s3hc_stream* s);
int s3hc_stream_read(s3hc_stream* s, uint8_t* dst, size_t cap, size_t* n);
uint64_t s3hc_stream_total(const s3hc_stream* s);
void s3hc_stream_close(s3hc_stream* s);

/* ---- pipelined range reader (stream_range_data for throughput, config 4) --- */
/* Complete frames are grouped into device batches of about batch_bytes compressed bytes that
 * run on `depth` HIP queues, S3HC_READER_SLOTS (default 1) batches in flight per queue (pinned
 * H2D of input + host-walked frame tables, decode, one
 * frame-close launch = lengths + content xxh32 + EndMark checks, D2H), so batches overlap;
 * decoded bytes come back in stream order. The first failing frame ends the stream after the bytes
 * of every earlier frame; a frame whose only fault is its content checksum is itself delivered
 * first, as lz4_flex's FrameDecoder returns a frame's bytes before the EndMark check
 * (disk_cache.rs:3884-3898). Frames of blocks > 64 KiB (the reference's cache files) have their
 * checksums verified behind the delivered bytes by a second frame close on the batch's queue; no
 * byte of a later frame is delivered before that verdict.
 * s3hc_reader_set_batch_max (optional, default = batch_bytes): while earlier batches are still
 * in flight, a new batch may take buffered frames up to max_bytes (the first batch after an idle
 * pipeline stays at batch_bytes, so time to first byte is unchanged). */
typedef struct s3hc_reader s3hc_reader;
int s3hc_reader_open(s3hc_ctx* ctx, size_t batch_bytes, int depth, s3hc_reader** out);
/* The same reader over nctx devices of one process (no reference counterpart: the proxy runs
 * every range read on the one host, http_proxy.rs:11608-11622): `depth` queues per context,
 * queue q on ctxs[q % nctx]; each batch goes to the least busy queue, so consecutive batches
 * alternate devices. Batches are independent (no collective); the output is the one-device
 * reader's, in stream order. Duplicate context pointers are refused. */
int s3hc_reader_open_multi(s3hc_ctx* const* ctxs, int nctx, size_t batch_bytes, int depth, s3hc_reader** out);
int s3hc_reader_set_batch_max(s3hc_reader* r, size_t max_bytes);
int s3hc_reader_feed(s3hc_reader* r, const uint8_t* src, size_t n);
int s3hc_reader_finish(s3hc_reader* r);
int s3hc_reader_read(s3hc_reader* r, uint8_t* dst, size_t cap, size_t* n);
uint64_t s3hc_reader_total(const s3hc_reader* r);
void s3hc_reader_close(s3hc_reader* r);

/* ---- device-resident batches (benchmark path, configs 2/3/5) -------------- */
/* A batch of n independent items already in HBM. Item i = d_src[src_off[i] ..
 * src_off[i]+len[i]). mode[i]: 0 = compress (lz4_flex Auto layout, as flush_batch),
 * 1 = store-mode frame (as encode_store_mode_frame; the extension denylist path,
 * compression.rs:252-308), 2 = compress as consecutive 64 KiB frames (S3HC_BLK_64K_PER_FRAME:
 * same bytes once decoded by the reference's frame loop, parallel decode on the GPU).
 * Metadata arrays are host arrays; the plan is reusable. */
int s3hc_plan_encode(s3hc_ctx* ctx, const uint64_t* src_off, const uint32_t* len,
                     const uint8_t* mode, uint32_t n, s3hc_plan** out);
/* Frames of item i land contiguously in d_dst at d_item_off[i], d_item_len[i] bytes
 * (device arrays written by the call; the batch's frames are packed in item order).
 * dst_cap must be >= s3hc_plan_dst_bound(plan). stream = hipStream_t (NULL = ctx stream);
 * a plan's scratch belongs to one call in flight at a time. */
int s3hc_encode_dev(s3hc_ctx* ctx, s3hc_plan* plan, const uint8_t* d_src, uint8_t* d_dst,
                    uint64_t dst_cap, uint64_t* d_item_off, uint32_t* d_item_len, void* stream);
uint64_t s3hc_plan_dst_bound(const s3hc_plan* plan);

/* lz4_flex-compatible encoder: the frame FrameEncoder writes in
 * compress_with_algorithm (compression.rs:539-557) and flush_batch (disk_cache.rs:1829-1846),
 * block payloads from lz4_flex's own greedy parse (block/compress.rs compress_internal as
 * restated in oracle/lz4_oracle.c:173-279; compressed-byte parity with the crate itself is
 * unpinned). One frame per item, one wave per frame. src_off/len/dst_off are
 * host arrays; dst_off[i+1] - dst_off[i] >= s3hc_frame_bound(len[i]). d_frame_len (device)
 * receives each frame's length. Returns after the frames are written. */
int s3hc_compat_encode_dev(s3hc_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint32_t* len,
                           uint32_t n, uint8_t* d_dst, const uint64_t* dst_off, uint32_t* d_frame_len,
                           void* stream);

/* Decode n frames in HBM: frame i = d_src[frame_off[i] .. +frame_len[i]) decodes to
 * d_dst[dst_off[i] ..) with room dst_cap[i]. Per-frame decoded length and status
 * (S3HC_*) are written to the device arrays d_out_len / d_status. Host metadata. */
int s3hc_plan_decode(s3hc_ctx* ctx, const uint64_t* frame_off, const uint32_t* frame_len,
                     const uint64_t* dst_off, const uint32_t* dst_cap, uint32_t n, s3hc_plan** out);
int s3hc_decode_dev(s3hc_ctx* ctx, s3hc_plan* plan, const uint8_t* d_src, uint8_t* d_dst,
                    uint32_t* d_out_len, int32_t* d_status, void* stream);
void s3hc_plan_free(s3hc_plan* plan);

/* Match-finder mode of every GPU encode issued on ctx (s3hc_encode_dev, host-buffer encodes, writers
 * and aggregators on ctx). Frames of either mode are valid lz4_flex frames and decode to the same
 * bytes; only the compressed size and the encode time differ. S3HC_ENC_FAST (default): one probe per
 * two positions, every position in the table (config 2: C/U 0.391). S3HC_ENC_SMALL: a probe at every
 * position, odd positions left out of the table, lazy selection (config 2: C/U 0.375, the match
 * finder ~35 % slower). Returns S3HC_INVALID_ARG for other values; get returns -1 for NULL. */
#define S3HC_ENC_FAST 0
#define S3HC_ENC_SMALL 1
int s3hc_set_encode_mode(s3hc_ctx* ctx, int mode);
int s3hc_get_encode_mode(const s3hc_ctx* ctx);

/* Per-kernel timing for roofline accounting: with timing on, the phases of every *_dev launch are
 * bracketed by HIP events on its stream (no host sync; adjacent phases share their boundary
 * event). s3hc_timing_collect resolves them into per-name totals: s3hc_last_kernel_ms = summed
 * ms, s3hc_kernel_count = launches. enabled: 0 off; 1 every phase ("xxh32", "enc_parse",
 * "enc_sizes", "enc_emit", "dec_plan", "decode", "dec_close", ...); 2 coarse: "enc_parse" and one
 * "dec_all" span over the whole device decode (fewest events in a timed region). */
void s3hc_set_timing(s3hc_ctx* ctx, int enabled);
int s3hc_timing_collect(s3hc_ctx* ctx);
void s3hc_timing_reset(s3hc_ctx* ctx);
float s3hc_last_kernel_ms(const s3hc_ctx* ctx, const char* name);
int s3hc_kernel_count(const s3hc_ctx* ctx, const char* name);

/* ---- device memory plumbing (lets callers stage batches in HBM without a second HIP
 * runtime in the process). kind: 1 H2D, 2 D2H, 3 D2D; s3hc_memcpy is host-synchronous. */
int s3hc_dev_alloc(s3hc_ctx* ctx, size_t n, void** out);
int s3hc_dev_free(s3hc_ctx* ctx, void* p);
int s3hc_memcpy(s3hc_ctx* ctx, void* dst, const void* src, size_t n, int kind);
int s3hc_memset(s3hc_ctx* ctx, void* dst, int value, size_t n);
int s3hc_sync(s3hc_ctx* ctx);

/* ---- pipelined host<->device batches: pinned host memory and caller queues. A queue is a
 * hipStream_t on the context's device, usable as the `stream` of s3hc_encode_dev /
 * s3hc_decode_dev; s3hc_memcpy_async orders a copy on it (kind as above). */
int s3hc_host_alloc(s3hc_ctx* ctx, size_t n, void** out);
int s3hc_host_free(s3hc_ctx* ctx, void* p);
int s3hc_queue_create(s3hc_ctx* ctx, void** out);
int s3hc_queue_destroy(s3hc_ctx* ctx, void* q);
int s3hc_queue_sync(s3hc_ctx* ctx, void* q);
int s3hc_memcpy_async(s3hc_ctx* ctx, void* dst, const void* src, size_t n, int kind, void* q);
/* Cross-queue ordering: a mark records the point reached by the work queued on q so far;
 * work queued on another queue after s3hc_queue_wait_mark starts only once that point is
 * passed (q NULL: the context's own queue). Marks are freed with s3hc_mark_free (any time). */
int s3hc_queue_mark(s3hc_ctx* ctx, void* q, void** mark);
int s3hc_queue_wait_mark(s3hc_ctx* ctx, void* q, void* mark);
int s3hc_mark_free(s3hc_ctx* ctx, void* mark);

/* ---- CompressionHandler mirror (compression.rs:169-604) ------------------- */
/* The host-side mirror of the reference's handler: same decision inputs, same six
 * counters (CompressionStatsAtomic, compression.rs:88-140), shared between clones. */
typedef struct s3hc_handler s3hc_handler;
s3hc_handler* s3hc_handler_new(s3hc_ctx* ctx, size_t threshold, int enabled);          /* :192 */
s3hc_handler* s3hc_handler_new_with_shared_stats(size_t threshold, int enabled,
                                                 const s3hc_handler* source);          /* :227 */
s3hc_handler* s3hc_handler_clone(const s3hc_handler* h);                               /* Clone */
void s3hc_handler_free(s3hc_handler* h);
int s3hc_handler_is_compression_enabled(const s3hc_handler* h);                         /* :520 */
/* compress_with_metadata (:376-460). Writes data (cap from s3hc_frame_bound) and metadata. */
int s3hc_handler_compress_with_metadata(s3hc_handler* h, const uint8_t* src, size_t n,
                                        const char* path, int should_compress, uint8_t* dst,
                                        size_t cap, size_t* out_len, int* algorithm,
                                        int* was_compressed);
/* compress_with_algorithm (:530-591); algorithm 0 = Lz4, 1 = None. */
int s3hc_handler_compress_with_algorithm(s3hc_handler* h, const uint8_t* src, size_t n, int algorithm,
                                         uint8_t* dst, size_t cap, size_t* out_len, int* was_compressed);
/* decompress_data (:463-502) / decompress_with_algorithm (:594-604). On error the
 * decompression_failures counter is incremented and the status returned. */
int s3hc_handler_decompress_with_algorithm(s3hc_handler* h, const uint8_t* src, size_t n, int algorithm,
                                           uint8_t* dst, size_t cap, size_t* out_len);
/* get_stats (:506): out = {compressed, uncompressed, bytes_before, bytes_after,
 * compression_failures, decompression_failures}; ratio = after/before (1.0 if before == 0). */
void s3hc_handler_stats(const s3hc_handler* h, uint64_t out[6], float* ratio);
/* record_batch_bytes / record_object (:105-120) for streaming writers. */
void s3hc_handler_record_batch_bytes(s3hc_handler* h, uint64_t before, uint64_t after);
void s3hc_handler_record_object(s3hc_handler* h, int compressed);
/* Tests only (no reference counterpart): make this handler's LZ4 frame encoder (bit 0),
 * store-mode encoder (bit 1) or decoder (bit 2) fail with S3HC_DEVICE, to exercise the
 * fallback branches of compress_with_metadata (:420-457) and the decode error path (:483-492). */
void s3hc_handler_debug_set_faults(s3hc_handler* h, int mask);
/* is_denylisted_extension (:252-308). */
int s3hc_is_denylisted_extension(const char* path);

/* ---- the cache layer's compression decision (the codec's caller) ------------ */
/* strip_known_cache_key_suffixes (cache.rs:226-275): the object path of a cache key — a trailing
 * ":range:<digits>-<digits>" and then ":part:<digits>" are removed, nothing else. Writes the path
 * NUL-terminated into out (truncated to cap - 1 bytes) and returns its full length. */
size_t s3hc_strip_known_cache_key_suffixes(const char* cache_key, char* out, size_t cap);
/* CacheManager::effective_compression (cache.rs:1158-1178): 1 = compress (compress_with_algorithm),
 * 0 = store-mode. compression_enabled / compression_from_rule are ResolvedSettings'
 * (bucket_settings.rs:364): the rule-or-global enable flag and whether a rule set it. Order:
 * disabled -> 0; size < threshold -> 0; set by a rule -> 1; else !denylisted(stripped key). */
int s3hc_effective_compression(int compression_enabled, int compression_from_rule,
                               size_t compression_threshold, const char* cache_key, uint64_t size);
/* The same with the handler's threshold (CompressionHandler::new(threshold, ..), cache.rs:1076-1083). */
int s3hc_handler_effective_compression(const s3hc_handler* h, int compression_enabled,
                                       int compression_from_rule, const char* cache_key, uint64_t size);

/* ---- batched incremental writers + cross-request aggregator ---------------- */
/* IncrementalRangeWriter (disk_cache.rs:262-305) with flush_batch (:1820-1870) routed
 * through an aggregator that encodes the full batches of many writers in one GPU launch
 * (SURVEY.md §8(f) row 2). Every batch is one frame, byte-identical to s3hc_compress_frame
 * (compression enabled) or s3hc_store_mode_frame (disabled) of the same bytes; a writer's
 * frames reach its sink in order (the reference's file.write_all, :1858). */
typedef struct s3hc_aggregator s3hc_aggregator;
typedef struct s3hc_writer s3hc_writer;
/* Receives one frame; nonzero return = write failure (the writer's next call fails). */
typedef int (*s3hc_frame_sink)(void* user, const uint8_t* frame, size_t n);
/* batch_size: cache.compression_batch_size (config.rs:990-995; the config layer bounds it to
 * 64 KiB..16 MiB, config.rs:1617-1627, the writer itself takes any size). flush_batches = 1
 * encodes every batch as soon as it fills (the reference's inline flush_batch). Queued batches are encoded together once flush_bytes bytes or
 * flush_batches batches are queued (0 = only on commit / s3hc_aggregator_flush).
 * stats: optional handler whose shared counters get record_batch_bytes per frame and
 * record_object per committed range (:1865-1867, :2053). */
int s3hc_aggregator_create(s3hc_ctx* ctx, size_t batch_size, size_t flush_bytes, uint32_t flush_batches,
                           s3hc_handler* stats, s3hc_aggregator** out);
/* The same aggregator over nctx devices of one process (the proxy's concurrent writers,
 * http_proxy.rs:11608-11622, spread over a node's GPUs): each flush splits the queued batches
 * into contiguous shards of about equal bytes (s3hc_shard_items), encodes shard d on ctxs[d]
 * (concurrently, no collective), and delivers every frame in queue order, byte-identical to the
 * one-device aggregator. Duplicate context pointers are refused, and so are contexts whose encode
 * modes (s3hc_set_encode_mode) differ — at creation, and at a flush if a mode changed since: the
 * writers of that flush then fail with S3HC_INVALID_ARG rather than get device-dependent frames. */
int s3hc_aggregator_create_multi(s3hc_ctx* const* ctxs, int nctx, size_t batch_size, size_t flush_bytes,
                                 uint32_t flush_batches, s3hc_handler* stats, s3hc_aggregator** out);
/* Contiguous shards of n items of byte sizes len[] over ndev devices: item i goes to the shard
 * holding its byte midpoint (about equal bytes per shard, order kept), and every shard gets at
 * least one item when n >= ndev. first[d] = first item of shard d, first[ndev] = n. Host only. */
int s3hc_shard_items(const uint64_t* len, uint32_t n, int ndev, uint32_t* first);
int s3hc_aggregator_flush(s3hc_aggregator* a);
/* Layout of compressed batches: S3HC_BLK_AUTO_LZ4FLEX (default, one frame per batch as
 * flush_batch writes it) or S3HC_BLK_64K_PER_FRAME (64 KiB frames: a reference reader decodes
 * them the same, the GPU decoder runs one wave per 64 KiB instead of per batch), or
 * S3HC_BLK_LZ4FLEX_COMPAT (flush_batch's frames with lz4_flex's own block bytes, via
 * s3hc_compat_encode_dev; store-mode batches of the same flush still share one launch). */
int s3hc_aggregator_set_frame_policy(s3hc_aggregator* a, int policy);
/* Encode launches and batches encoded so far. */
void s3hc_aggregator_counters(const s3hc_aggregator* a, uint64_t* launches, uint64_t* batches);
void s3hc_aggregator_destroy(s3hc_aggregator* a);
/* begin_incremental_range_write (:1716-1778): start > end -> S3HC_INVALID_ARG. */
int s3hc_writer_begin(s3hc_aggregator* a, uint64_t start, uint64_t end, int compression_enabled,
                      s3hc_frame_sink sink, void* user, s3hc_writer** out);
/* write_range_chunk (:1798-1810): a batch is flushed once it holds >= batch_size bytes.
 * A failure of an earlier queued batch (encode or sink) is reported here. */
int s3hc_writer_write(s3hc_writer* w, const uint8_t* chunk, size_t n);
size_t s3hc_writer_batch_buf_len(const s3hc_writer* w);                 /* batch_buf_len (:300-304) */
uint64_t s3hc_writer_bytes_written(const s3hc_writer* w);
uint64_t s3hc_writer_compressed_bytes_written(const s3hc_writer* w);
/* finalize_incremental_range (:1968-2090): flushes the residual batch, waits for the
 * writer's frames, checks bytes_written == end - start + 1 (min_commit_ratio >= 0 salvages a
 * prefix >= ratio * expected as a clamped range; < 0 = exact only). spec_out = {start, end,
 * compressed_size, uncompressed_size} (RangeSpec, cache_types.rs:472-508). Frees w. */
int s3hc_writer_commit(s3hc_writer* w, double min_commit_ratio, uint64_t spec_out[4]);
/* abort_incremental_range (:2093-2116): queued batches are dropped undelivered. Frees w. */
void s3hc_writer_abort(s3hc_writer* w);
/* Message of the last failing writer/aggregator call on this thread. */
const char* s3hc_writer_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
