// compression_handler.hpp — C++ mirror of the reference's CompressionHandler
// (src/compression.rs:143-604) on top of the MI355X engine.
//
// Same names, argument meaning, result metadata, stats semantics and error behaviour as the
// Rust type; the codec underneath is the GPU engine (s3hc_* C ABI). The Rust toolchain is
// absent from this image, so this is the host-side counterpart a C++ caller (or the tests)
// uses; INTEGRATION.md shows the Rust extern shim that binds the same C ABI.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "s3hc_lz4.h"

namespace s3hc {

enum class CompressionAlgorithm { Lz4 = 0, None = 1 };  // compression.rs:143-156

struct CompressionStats {  // compression.rs:53-76
    uint64_t total_objects_compressed = 0;
    uint64_t total_objects_uncompressed = 0;
    uint64_t total_bytes_before = 0;
    uint64_t total_bytes_after = 0;
    uint64_t compression_failures = 0;
    uint64_t decompression_failures = 0;
    float average_compression_ratio = 1.0f;
};

struct CompressionStatsAtomic {  // compression.rs:88-140 (shared by every clone)
    std::atomic<uint64_t> total_objects_compressed{0};
    std::atomic<uint64_t> total_objects_uncompressed{0};
    std::atomic<uint64_t> total_bytes_before{0};
    std::atomic<uint64_t> total_bytes_after{0};
    std::atomic<uint64_t> compression_failures{0};
    std::atomic<uint64_t> decompression_failures{0};
    void record_batch_bytes(uint64_t before, uint64_t after);
    void record_object(bool compressed);
    CompressionStats snapshot() const;
};

struct CompressionResult {  // compression.rs:159-166
    std::vector<uint8_t> data;
    CompressionAlgorithm algorithm = CompressionAlgorithm::Lz4;
    uint64_t original_size = 0;
    uint64_t compressed_size = 0;
    bool was_compressed = false;
};

struct CodecError {  // ProxyError::CompressionError(String) (error.rs:22-23)
    int status;
    std::string message;
};

class CompressionHandler {
public:
    CompressionHandler(s3hc_ctx* ctx, size_t threshold, bool enabled);                   // :192
    CompressionHandler(s3hc_ctx* ctx, size_t threshold, bool enabled, CompressionAlgorithm preferred);  // :210
    static CompressionHandler with_shared_stats(size_t threshold, bool enabled,
                                                const CompressionHandler& source);       // :227

    std::shared_ptr<CompressionStatsAtomic> shared_stats() const { return stats_; }     // :243
    static bool is_denylisted_extension(const std::string& path);                        // :252
    static std::string extract_file_extension(const std::string& path);                  // :258
    static bool is_already_compressed_format(const std::string& ext);                    // :276

    // :326-368. Returns false (and err) only on a device error.
    bool encode_store_mode_frame(const uint8_t* data, size_t n, std::vector<uint8_t>& out, CodecError* err) const;
    CompressionResult compress_with_metadata(const uint8_t* data, size_t n, const std::string& path,
                                             bool should_compress);                      // :376-460
    bool decompress_data(const uint8_t* data, size_t n, std::vector<uint8_t>& out, CodecError* err) const;  // :463
    CompressionStats get_stats() const { return stats_->snapshot(); }                    // :506
    bool is_compression_enabled() const { return enabled_; }                             // :520
    CompressionAlgorithm get_preferred_algorithm() const { return preferred_; }          // :526
    bool compress_with_algorithm(const uint8_t* data, size_t n, CompressionAlgorithm alg,
                                 CompressionResult& out, CodecError* err);               // :530-591
    bool decompress_with_algorithm(const uint8_t* data, size_t n, CompressionAlgorithm alg,
                                   std::vector<uint8_t>& out, CodecError* err) const;    // :594-604

    s3hc_ctx* ctx() const { return ctx_; }
    size_t compression_threshold() const { return threshold_; }
    // Fault injection for tests of the error-fallback branches (:420-457): bit 0 makes the LZ4
    // frame encoder fail, bit 1 the store-mode encoder, bit 2 the decoder; 0 in production.
    void set_debug_faults(int mask) { faults_ = mask; }

private:
    s3hc_ctx* ctx_;
    size_t threshold_;  // compression.rs:176-183 (the codec never reads it; effective_compression does)
    bool enabled_;
    CompressionAlgorithm preferred_;
    std::shared_ptr<CompressionStatsAtomic> stats_;
    int faults_ = 0;
};

// The compression decision of the cache layer (the caller of this codec): which ranges go through
// compress_with_algorithm and which through encode_store_mode_frame.
// cache.rs:226-275: strip the `:range:<digits>-<digits>` suffix (last), then `:part:<digits>`, from
// the end of a cache key; anything else (a colon inside the object key) is left alone.
std::string strip_known_cache_key_suffixes(const std::string& cache_key);
// bucket_settings.rs:364 ResolvedSettings (the two fields the decision reads)
struct ResolvedCompression {
    bool compression_enabled;    // resolved: rule override or global config
    bool compression_from_rule;  // a cache rule set compression_enabled explicitly
};
// cache.rs:1158-1178 CacheManager::effective_compression: disabled -> false; size below the
// threshold -> false; a rule said so -> true (any extension); else the extension denylist on the
// key with its suffixes stripped.
bool effective_compression(const ResolvedCompression& resolved, size_t compression_threshold,
                           const std::string& cache_key, uint64_t size);

}  // namespace s3hc
