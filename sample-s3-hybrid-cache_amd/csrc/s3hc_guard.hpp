// s3hc_guard.hpp — internal helpers shared by the host-side translation units of libs3hc_lz4.so.
#pragma once
#include <cstdint>
#include <exception>
#include <new>
#include <string>
#include <vector>

#include "s3hc_lz4.h"

namespace s3hc {

// Sets the thread-local message read by s3hc_last_error(); returns code.
int set_error(int code, const std::string& msg);

// Runs f() and turns any C++ exception into a status (no exception crosses the C ABI; the
// reference's Rust API returns Result, never unwinds into the caller): allocation failures
// become S3HC_NO_MEMORY, anything else S3HC_DEVICE, with the message set through `fail`.
template <class Fail, class F>
inline int guarded_call(Fail&& fail, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return fail(S3HC_NO_MEMORY, "host memory allocation failed");
    } catch (const std::exception& e) {
        return fail(S3HC_DEVICE, std::string("internal error: ") + e.what());
    } catch (...) {
        return fail(S3HC_DEVICE, "internal error");
    }
}

// decompress_data (compression.rs:463-502) into a vector sized by the decoded bytes.
int decompress_frames_vec(s3hc_ctx* ctx, const uint8_t* src, size_t n, std::vector<uint8_t>& out);

}  // namespace s3hc
