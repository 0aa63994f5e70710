#!/usr/bin/env python3
"""Counterpart of the reference's examples/compression_demo.rs (BASELINE.json configs[0]).

Same walk-through as the Rust demo: the built-in extension denylist decides, per file name,
whether compress_with_metadata runs the LZ4 block compressor or writes a checksummed store-mode
frame; the handler's live statistics are printed at the end. Then the config-1 workload: one
1 MiB log-text buffer round-tripped through the GPU engine (compress_with_algorithm +
decompress_data), with the CPU restatement of the reference path (oracle/, test infrastructure)
timed beside it when --cpu is given.

The engine has no CPU codec: this demo needs an MI355X (the reference demo runs lz4_flex on CPU).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]

import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

THRESHOLD = 100  # compression_demo.rs:18
TEST_FILES = [  # compression_demo.rs:30-57
    ("config.json", "JSON configuration file - should compress"),
    ("style.css", "CSS stylesheet - should compress"),
    ("script.js", "JavaScript file - should compress"),
    ("data.xml", "XML data file - should compress"),
    ("readme.txt", "Text file - should compress"),
    ("photo.jpg", "JPEG image - should NOT compress (built-in denylist)"),
    ("video.mp4", "MP4 video - should NOT compress (built-in denylist)"),
    ("archive.zip", "ZIP archive - should NOT compress (built-in denylist)"),
    ("document.pdf", "PDF document - should NOT compress (built-in denylist)"),
    ("music.mp3", "MP3 audio - should NOT compress (built-in denylist)"),
]
ALG = {S.ALG_LZ4: "Lz4", S.ALG_NONE: "None"}


def demo(eng, out=print):
    handler = S.CompressionHandler(eng, THRESHOLD, True)
    data = (b"This is some sample text data that should compress well with LZ4 because it has repeating "
            b"patterns and is longer than our threshold. ") * 5
    out("Content-Aware Compression Demo")
    out("==============================")
    out(f"Sample data size: {len(data)} bytes")
    out("")
    results = []
    for filename, description in TEST_FILES:
        deny = S.CompressionHandler.is_denylisted_extension(filename)
        should = handler.is_compression_enabled() and len(data) >= THRESHOLD and not deny
        r = handler.compress_with_metadata(data, filename, should)
        ratio = r.compressed_size / r.original_size if r.was_compressed else 1.0
        assert handler.decompress_data(r.data) == data
        out(f"File: {filename}")
        out(f"  Description: {description}")
        out(f"  Denylisted extension: {str(deny).lower()}")
        out(f"  Should compress: {str(should).lower()}")
        out(f"  Was compressed (LZ4 block compressor ran): {str(r.was_compressed).lower()}")
        out(f"  Size: {r.original_size} -> {r.compressed_size} bytes")
        out(f"  Compression ratio: {ratio:.2f}")
        out(f"  Stored algorithm tag: {ALG[r.algorithm]} (store-mode frames are tagged Lz4 too)")
        out("")
        results.append((filename, deny, should, r))
    st = handler.get_stats()
    out("Compression Statistics:")
    out("======================")
    out(f"Objects compressed: {st.total_objects_compressed}")
    out(f"Objects uncompressed (store-mode): {st.total_objects_uncompressed}")
    out(f"Total bytes before: {st.total_bytes_before}")
    out(f"Total bytes after: {st.total_bytes_after}")
    out(f"Average compression ratio: {st.average_compression_ratio:.2f}")
    out(f"Compression failures: {st.compression_failures}")
    out(f"Decompression failures: {st.decompression_failures}")
    return results, st


def config1(eng, cpu: bool, reps: int = 20):
    """1 MiB of log text through compress_with_algorithm(Lz4) + decompress_data (one frame, one
    1 MiB block in a BD 0x70 frame, as lz4_flex's BlockSize::Auto lays it out)."""
    handler = S.CompressionHandler(eng, THRESHOLD, True)
    data = synth.log_text(1 << 20, synth.SEED_BASE + 0)
    handler.decompress_data(handler.compress_with_algorithm(data).data)  # warm-up
    t0 = time.perf_counter()
    for _ in range(reps):
        frame = handler.compress_with_algorithm(data).data
    t1 = time.perf_counter()
    for _ in range(reps):
        back = handler.decompress_data(frame)
    t2 = time.perf_counter()
    assert back == data
    res = {"bytes": len(data), "frame_bytes": len(frame), "bd": hex(frame[5]),
           "gpu_host_call_encode_ms": round((t1 - t0) / reps * 1e3, 3),
           "gpu_host_call_decode_ms": round((t2 - t1) / reps * 1e3, 3)}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU restatement of the reference path (test infrastructure)

        t0 = time.perf_counter()
        for _ in range(reps):
            cf = O.lz4flex_compress_frame(data)
        t1 = time.perf_counter()
        for _ in range(reps):
            assert O.decompress_data(cf) == data
        t2 = time.perf_counter()
        assert O.decompress_data(frame) == data  # the GPU frame decodes with the CPU restatement
        res.update({"cpu_port_frame_bytes": len(cf), "cpu_port_encode_ms": round((t1 - t0) / reps * 1e3, 3),
                    "cpu_port_decode_ms": round((t2 - t1) / reps * 1e3, 3)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true", help="also time the CPU restatement (oracle/) on config 1")
    a = ap.parse_args()
    eng = S.Engine(0)
    demo(eng)
    print()
    print("Config 1 (1 MiB log text round trip):", config1(eng, a.cpu))


if __name__ == "__main__":
    main()
