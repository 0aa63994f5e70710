/*
 * lz4_oracle.h — CPU restatement of the reference's LZ4 frame-codec path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * (libs3hc_lz4.so) never links, loads or calls it.
 *
 * What it restates (citations are into /root/reference):
 *   - src/compression.rs:326-368  encode_store_mode_frame (byte-exact, pinned by reference code)
 *   - src/compression.rs:530-591  compress_with_algorithm -> lz4_flex 0.11.6 FrameEncoder
 *                                 (FrameInfo{content_checksum=true, Independent}, BlockSize::Auto).
 *                                 lz4_flex is a crates.io dependency (Cargo.toml:37, Cargo.lock:1226-1232)
 *                                 that is absent from the container; its block compressor is restated
 *                                 from its published algorithm.
 *                                 Compressed-byte equality with lz4_flex is therefore "parity unpinned".
 *   - src/compression.rs:463-502  decompress_data: loop FrameDecoder::read_to_end over concatenated
 *                                 frames; Ok(0) (a frame that yields no bytes) stops the loop.
 *   - twox-hash 2.1.2 XxHash32 (Cargo.toml:43): standard XXH32, pinned against python xxhash 3.8.1.
 *
 * Status codes are shared with include/s3hc_lz4.h.
 */
#ifndef S3HC_LZ4_ORACLE_H
#define S3HC_LZ4_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OR_OK = 0,
    OR_CORRUPT = 1,
    OR_CHECKSUM = 2,
    OR_DST_TOO_SMALL = 3,
    OR_UNSUPPORTED = 4,
    OR_INVALID_ARG = 6,
};

/* XXH32 one-shot (twox-hash XxHash32::oneshot). */
uint32_t or_xxh32(const uint8_t* p, size_t n, uint32_t seed);

/* Worst-case framed size of any frame this oracle writes for n input bytes. */
size_t or_frame_bound(size_t n);

/* compression.rs:326-368 — store-mode frame (BD 0x70, stored blocks of <= 4 MiB). */
int or_store_mode_frame(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* compression.rs:530-591 -> lz4_flex FrameEncoder(content_checksum, Independent, Auto).
 * was_compressed always 1 on success (compress_with_algorithm tags every frame compressed). */
int or_lz4flex_compress_frame(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* The same lz4_flex block compressor on one independent block (first block of a fresh
 * FrameEncoder: HashTable4K zero-initialised, stream offset 0). Returns the compressed
 * length; the frame writer stores the block instead when the result is >= n. */
size_t or_lz4flex_compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap);

/* compression.rs:463-502 decompress_data over concatenated frames. */
int or_decompress_data(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* Upper bound of decompress_data output (walks frame/block headers only). 0 on a malformed walk. */
size_t or_decompressed_bound(const uint8_t* src, size_t n);

/* One raw LZ4 block (no frame) with lz4_flex decompress_internal semantics. */
int or_decode_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* cpu_bench.c: bench.py's cpu_baseline harness — encode (or_lz4flex_compress_frame) + decode
 * (or_decompress_data) of 'block'-byte blocks on 'threads' threads over contiguous ranges. */
int or_bench_blocks(const uint8_t* data, size_t nblocks, size_t block, int threads, double seconds,
                    size_t fixed_per_thread, uint64_t* blocks_done, double* wall, double* enc_s, double* dec_s);

#ifdef __cplusplus
}
#endif
#endif
