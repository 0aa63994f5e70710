#!/usr/bin/env python3
"""Range reads of small cached objects, one reader per GET (stream_range_data opens one per
request, disk_cache.rs:3850): N objects of SIZE bytes (64 KiB frames, fixed 256 KiB batches,
depth 3), each fed in 4 MiB reads and drained in 1 MiB chunks. Prints the mean and p50/p90 time
per object and the aggregate GiB/s. Usage: python tools/reader_small.py [N] [SIZE_KIB]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    size = (int(sys.argv[2]) if len(sys.argv) > 2 else 1024) << 10
    eng = S.Engine(0)
    data = synth.log_text(size, 5)
    frames = b"".join(eng.compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536))
    ts = []
    for k in range(n + 5):
        t0 = time.perf_counter()
        r = S.RangeReader(eng, 256 << 10, 3)
        out = bytearray()
        for i in range(0, len(frames), 4 << 20):
            r.feed(frames[i:i + (4 << 20)])
            while True:
                c = r.read(1 << 20)
                if not c:
                    break
                out += c
        r.finish()
        while True:
            c = r.read(1 << 20)
            if not c:
                break
            out += c
        r.close()
        dt = time.perf_counter() - t0
        assert bytes(out) == data
        if k >= 5:
            ts.append(dt)
    ts.sort()
    print(json.dumps({"objects": n, "object_bytes": size, "mean_ms": round(1e3 * sum(ts) / n, 3),
                      "p50_ms": round(1e3 * ts[n // 2], 3), "p90_ms": round(1e3 * ts[int(n * 0.9)], 3),
                      "GiBps": round(n * size / sum(ts) / 2**30, 3)}))


if __name__ == "__main__":
    main()
