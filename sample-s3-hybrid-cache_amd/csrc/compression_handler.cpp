// compression_handler.cpp — see compression_handler.hpp. Control flow and counter updates
// follow src/compression.rs line by line (cited per method); all codec work is the GPU
// engine's (s3hc_compress_frame / s3hc_store_mode_frame / s3hc_decompress_frames).
#include "compression_handler.hpp"
#include "s3hc_guard.hpp"

#include <algorithm>
#include <cctype>
#include <cstring>

namespace s3hc {

void CompressionStatsAtomic::record_batch_bytes(uint64_t before, uint64_t after) {  // :105-110
    total_bytes_before.fetch_add(before, std::memory_order_relaxed);
    total_bytes_after.fetch_add(after, std::memory_order_relaxed);
}
void CompressionStatsAtomic::record_object(bool compressed) {  // :113-120
    (compressed ? total_objects_compressed : total_objects_uncompressed).fetch_add(1, std::memory_order_relaxed);
}
CompressionStats CompressionStatsAtomic::snapshot() const {  // :121-139
    CompressionStats s;
    s.total_objects_compressed = total_objects_compressed.load(std::memory_order_relaxed);
    s.total_objects_uncompressed = total_objects_uncompressed.load(std::memory_order_relaxed);
    s.total_bytes_before = total_bytes_before.load(std::memory_order_relaxed);
    s.total_bytes_after = total_bytes_after.load(std::memory_order_relaxed);
    s.compression_failures = compression_failures.load(std::memory_order_relaxed);
    s.decompression_failures = decompression_failures.load(std::memory_order_relaxed);
    s.average_compression_ratio =
        s.total_bytes_before > 0 ? (float)s.total_bytes_after / (float)s.total_bytes_before : 1.0f;
    return s;
}

CompressionHandler::CompressionHandler(s3hc_ctx* ctx, size_t threshold, bool enabled)
    : CompressionHandler(ctx, threshold, enabled, CompressionAlgorithm::Lz4) {}
CompressionHandler::CompressionHandler(s3hc_ctx* ctx, size_t threshold, bool enabled, CompressionAlgorithm preferred)
    : ctx_(ctx), threshold_(threshold), enabled_(enabled), preferred_(preferred),
      stats_(std::make_shared<CompressionStatsAtomic>()) {}
CompressionHandler CompressionHandler::with_shared_stats(size_t threshold, bool enabled,
                                                         const CompressionHandler& source) {
    CompressionHandler h(source.ctx_, threshold, enabled, source.preferred_);
    h.stats_ = source.stats_;
    return h;
}

std::string CompressionHandler::extract_file_extension(const std::string& path) {  // :258-266
    size_t slash = path.rfind('/');
    std::string last = slash == std::string::npos ? path : path.substr(slash + 1);
    size_t dot = last.rfind('.');
    if (dot == std::string::npos) return std::string();
    std::string ext = last.substr(dot + 1);
    std::transform(ext.begin(), ext.end(), ext.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return ext;
}

bool CompressionHandler::is_already_compressed_format(const std::string& e) {  // :276-308
    static const char* const kList[] = {
        "jpg", "jpeg", "png", "gif", "webp", "avif", "heic", "heif",            // images
        "mp4", "avi", "mkv", "mov", "wmv", "flv", "webm", "m4v",                // video
        "mp3", "aac", "ogg", "flac", "m4a", "wma", "opus",                      // audio
        "zip", "rar", "7z", "gz", "bz2", "xz", "lz4", "zst", "tgz",             // archives
        "pdf", "docx", "xlsx", "pptx", "odt", "ods", "odp",                     // documents
        "apk", "ipa", "jar", "war", "ear",                                      // applications
        "woff", "woff2",                                                        // fonts
        "sqlite", "db",                                                         // databases
        "exe", "msi", "dmg", "pkg",                                             // executables
    };
    for (const char* k : kList)
        if (e == k) return true;
    return false;
}

bool CompressionHandler::is_denylisted_extension(const std::string& path) {  // :252-255
    return is_already_compressed_format(extract_file_extension(path));
}

bool CompressionHandler::encode_store_mode_frame(const uint8_t* data, size_t n, std::vector<uint8_t>& out,
                                                 CodecError* err) const {
    out.resize(s3hc_frame_bound(n) + 4 * (n / (4u << 20) + 1));
    size_t len = 0;
    int rc = (faults_ & 2) ? s3hc::set_error(S3HC_DEVICE, "injected store-mode encoder fault")
                           : s3hc_store_mode_frame(ctx_, data, n, out.data(), out.size(), &len);
    if (rc) {
        if (err) *err = {rc, std::string("Store-mode frame encoding failed: ") + s3hc_last_error()};
        out.clear();
        return false;
    }
    out.resize(len);
    return true;
}

CompressionResult CompressionHandler::compress_with_metadata(const uint8_t* data, size_t n, const std::string& path,
                                                             bool should_compress) {
    (void)path;  // only used for the warn! log lines of the reference (:400-403, :424-427)
    const uint64_t original = n;
    if (!should_compress) {  // :384-417
        CompressionResult r;
        CodecError e;
        if (encode_store_mode_frame(data, n, r.data, &e)) {
            stats_->total_objects_uncompressed.fetch_add(1, std::memory_order_relaxed);
            r.algorithm = CompressionAlgorithm::Lz4;
            r.original_size = original;
            r.compressed_size = r.data.size();
            r.was_compressed = false;
            return r;
        }
        stats_->compression_failures.fetch_add(1, std::memory_order_relaxed);
        stats_->total_objects_uncompressed.fetch_add(1, std::memory_order_relaxed);
        r.data.assign(data, data + n);
        r.algorithm = CompressionAlgorithm::None;
        r.original_size = original;
        r.compressed_size = original;
        r.was_compressed = false;
        return r;
    }
    CompressionResult r;
    CodecError e;
    if (compress_with_algorithm(data, n, CompressionAlgorithm::Lz4, r, &e)) return r;  // :420
    stats_->compression_failures.fetch_add(1, std::memory_order_relaxed);              // :428-430
    CompressionResult f;
    if (encode_store_mode_frame(data, n, f.data, nullptr)) {                              // :433-447
        f.algorithm = CompressionAlgorithm::Lz4;
        f.original_size = original;
        f.compressed_size = f.data.size();
        f.was_compressed = false;
        return f;
    }
    stats_->total_objects_uncompressed.fetch_add(1, std::memory_order_relaxed);          // :448-457
    f.data.assign(data, data + n);
    f.algorithm = CompressionAlgorithm::Lz4;
    f.original_size = original;
    f.compressed_size = original;
    f.was_compressed = false;
    return f;
}

bool CompressionHandler::compress_with_algorithm(const uint8_t* data, size_t n, CompressionAlgorithm alg,
                                                 CompressionResult& out, CodecError* err) {
    const uint64_t original = n;
    if (alg == CompressionAlgorithm::None) {  // :563-571
        out.data.assign(data, data + n);
        out.algorithm = CompressionAlgorithm::None;
        out.original_size = original;
        out.compressed_size = original;
        out.was_compressed = false;
        return true;
    }
    out.data.resize(s3hc_frame_bound(n));
    size_t len = 0;
    int wc = 0;
    int rc = (faults_ & 1) ? s3hc::set_error(S3HC_DEVICE, "injected LZ4 encoder fault")
                           : s3hc_compress_frame(ctx_, data, n, S3HC_BLK_AUTO_LZ4FLEX, out.data.data(), out.data.size(),
                                                 &len, &wc);
    if (rc) {
        if (err) *err = {rc, std::string("Failed to write data to LZ4 frame encoder: ") + s3hc_last_error()};
        return false;
    }
    out.data.resize(len);
    stats_->total_objects_compressed.fetch_add(1, std::memory_order_relaxed);  // :574-582
    stats_->total_bytes_before.fetch_add(original, std::memory_order_relaxed);
    stats_->total_bytes_after.fetch_add(len, std::memory_order_relaxed);
    out.algorithm = CompressionAlgorithm::Lz4;
    out.original_size = original;
    out.compressed_size = len;
    out.was_compressed = true;
    return true;
}

bool CompressionHandler::decompress_data(const uint8_t* data, size_t n, std::vector<uint8_t>& out,
                                         CodecError* err) const {
    // output grows by the decoded bytes (read_to_end), never by a worst-case bound
    int rc = (faults_ & 4) ? s3hc::set_error(S3HC_DEVICE, "injected decoder fault")
                           : decompress_frames_vec(ctx_, data, n, out);
    if (rc) {  // :483-492
        stats_->decompression_failures.fetch_add(1, std::memory_order_relaxed);
        if (err) *err = {rc, std::string("Failed to decompress cached data: ") + s3hc_last_error()};
        out.clear();
        return false;
    }
    return true;
}

bool CompressionHandler::decompress_with_algorithm(const uint8_t* data, size_t n, CompressionAlgorithm alg,
                                                   std::vector<uint8_t>& out, CodecError* err) const {
    if (alg == CompressionAlgorithm::None) {
        out.assign(data, data + n);
        return true;
    }
    return decompress_data(data, n, out, err);
}

static bool all_ascii_digits(const std::string& s, size_t from, size_t to) {
    for (size_t i = from; i < to; ++i)
        if (s[i] < '0' || s[i] > '9') return false;
    return true;
}

std::string strip_known_cache_key_suffixes(const std::string& key) {  // cache.rs:226-258
    static const std::string kRange = ":range:", kPart = ":part:";
    size_t end = key.size();
    const size_t r = key.rfind(kRange);
    if (r != std::string::npos) {
        // is_range_suffix_body (cache.rs:261-271): split at the first '-', both sides non-empty digits
        const size_t b = r + kRange.size();
        const size_t dash = key.find('-', b);
        if (dash != std::string::npos && dash > b && dash + 1 < key.size() && all_ascii_digits(key, b, dash) &&
            all_ascii_digits(key, dash + 1, key.size()))
            end = r;
    }
    const std::string head = key.substr(0, end);
    const size_t p = head.rfind(kPart);
    if (p != std::string::npos) {
        const size_t b = p + kPart.size();
        if (b < head.size() && all_ascii_digits(head, b, head.size())) return head.substr(0, p);
    }
    return head;
}

bool effective_compression(const ResolvedCompression& resolved, size_t threshold, const std::string& cache_key,
                           uint64_t size) {  // cache.rs:1158-1178
    if (!resolved.compression_enabled) return false;
    if ((size_t)size < threshold) return false;
    if (resolved.compression_from_rule) return true;
    return !CompressionHandler::is_denylisted_extension(strip_known_cache_key_suffixes(cache_key));
}

}  // namespace s3hc

// ------------------------------------------------------------ C wrappers
using s3hc::CompressionAlgorithm;
using s3hc::CompressionHandler;

struct s3hc_handler {
    CompressionHandler h;
};

template <class F>
static int guarded(F&& f) {
    return s3hc::guarded_call(s3hc::set_error, f);  // message via s3hc_last_error()
}
template <class F>
static s3hc_handler* make_handler(F&& f) {
    try {
        return new s3hc_handler{f()};
    } catch (...) {
        s3hc::set_error(S3HC_NO_MEMORY, "handler allocation failed");
        return nullptr;
    }
}

extern "C" s3hc_handler* s3hc_handler_new(s3hc_ctx* ctx, size_t threshold, int enabled) {
    return make_handler([&] { return CompressionHandler(ctx, threshold, enabled != 0); });
}
extern "C" s3hc_handler* s3hc_handler_new_with_shared_stats(size_t threshold, int enabled, const s3hc_handler* src) {
    if (!src) return nullptr;
    return make_handler([&] { return CompressionHandler::with_shared_stats(threshold, enabled != 0, src->h); });
}
extern "C" s3hc_handler* s3hc_handler_clone(const s3hc_handler* h) {
    return h ? make_handler([&] { return h->h; }) : nullptr;
}
extern "C" void s3hc_handler_free(s3hc_handler* h) { delete h; }
extern "C" int s3hc_handler_is_compression_enabled(const s3hc_handler* h) { return h && h->h.is_compression_enabled(); }

static int copy_out(const std::vector<uint8_t>& v, uint8_t* dst, size_t cap, size_t* out_len) {
    if (out_len) *out_len = v.size();
    if (v.size() > cap) return S3HC_DST_TOO_SMALL;
    if (!v.empty()) memcpy(dst, v.data(), v.size());
    return S3HC_OK;
}

extern "C" int s3hc_handler_compress_with_metadata(s3hc_handler* h, const uint8_t* src, size_t n, const char* path,
                                                   int should_compress, uint8_t* dst, size_t cap, size_t* out_len,
                                                   int* algorithm, int* was_compressed) {
    return guarded([&]() -> int {
        if (!h) return S3HC_INVALID_ARG;
        auto r = h->h.compress_with_metadata(src, n, path ? path : "", should_compress != 0);
        if (algorithm) *algorithm = (int)r.algorithm;
        if (was_compressed) *was_compressed = r.was_compressed;
        return copy_out(r.data, dst, cap, out_len);
    });
}
extern "C" int s3hc_handler_compress_with_algorithm(s3hc_handler* h, const uint8_t* src, size_t n, int algorithm,
                                                    uint8_t* dst, size_t cap, size_t* out_len, int* was_compressed) {
    return guarded([&]() -> int {
        if (!h) return S3HC_INVALID_ARG;
        s3hc::CompressionResult r;
        s3hc::CodecError e{0, ""};
        if (!h->h.compress_with_algorithm(src, n, (CompressionAlgorithm)algorithm, r, &e)) return e.status;
        if (was_compressed) *was_compressed = r.was_compressed;
        return copy_out(r.data, dst, cap, out_len);
    });
}
extern "C" int s3hc_handler_decompress_with_algorithm(s3hc_handler* h, const uint8_t* src, size_t n, int algorithm,
                                                      uint8_t* dst, size_t cap, size_t* out_len) {
    return guarded([&]() -> int {
        if (!h) return S3HC_INVALID_ARG;
        std::vector<uint8_t> out;
        s3hc::CodecError e{0, ""};
        if (!h->h.decompress_with_algorithm(src, n, (CompressionAlgorithm)algorithm, out, &e)) return e.status;
        return copy_out(out, dst, cap, out_len);
    });
}
extern "C" void s3hc_handler_stats(const s3hc_handler* h, uint64_t out[6], float* ratio) {
    if (!h) return;
    auto s = h->h.get_stats();
    out[0] = s.total_objects_compressed;
    out[1] = s.total_objects_uncompressed;
    out[2] = s.total_bytes_before;
    out[3] = s.total_bytes_after;
    out[4] = s.compression_failures;
    out[5] = s.decompression_failures;
    if (ratio) *ratio = s.average_compression_ratio;
}
extern "C" void s3hc_handler_record_batch_bytes(s3hc_handler* h, uint64_t before, uint64_t after) {
    if (h) h->h.shared_stats()->record_batch_bytes(before, after);
}
extern "C" void s3hc_handler_record_object(s3hc_handler* h, int compressed) {
    if (h) h->h.shared_stats()->record_object(compressed != 0);
}
extern "C" void s3hc_handler_debug_set_faults(s3hc_handler* h, int mask) {
    if (h) h->h.set_debug_faults(mask);
}
extern "C" int s3hc_is_denylisted_extension(const char* path) {
    return guarded([&]() -> int {
        return path && CompressionHandler::is_denylisted_extension(path);
    });
}
extern "C" size_t s3hc_strip_known_cache_key_suffixes(const char* cache_key, char* out, size_t cap) {
    if (!cache_key) return 0;
    const std::string p = s3hc::strip_known_cache_key_suffixes(cache_key);
    if (out && cap) {
        const size_t k = p.size() < cap - 1 ? p.size() : cap - 1;
        memcpy(out, p.data(), k);
        out[k] = 0;
    }
    return p.size();
}
extern "C" int s3hc_effective_compression(int compression_enabled, int compression_from_rule,
                                          size_t compression_threshold, const char* cache_key, uint64_t size) {
    return guarded([&]() -> int {
        return s3hc::effective_compression({compression_enabled != 0, compression_from_rule != 0}, compression_threshold,
                                           cache_key ? cache_key : "", size);
    });
}
extern "C" int s3hc_handler_effective_compression(const s3hc_handler* h, int compression_enabled,
                                                  int compression_from_rule, const char* cache_key, uint64_t size) {
    return guarded([&]() -> int {
        if (!h) return 0;
        return s3hc_effective_compression(compression_enabled, compression_from_rule, h->h.compression_threshold(),
                                          cache_key, size);
    });
}
