#!/usr/bin/env python3
"""Small-work latency probe: where a few-frame decode spends its time.

(a) device decode_dev of n frames (64 KiB GPU-format frames, or reference 1 MiB frames of one
    block) with the large-block path on and off, wall time per call and per-stage kernel times;
(b) host-buffer decompress_frames of one 1 MiB payload in both formats (wall);
(c) the range reader over a 256 MiB object at 256 KiB batches, depth 1 and 3.
Prints one JSON object. Diagnostic tool (not the bench contract).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

GiB = float(1 << 30)


def frames_of(eng, data, item):
    n = len(data) // item
    d_src = eng.upload(data)
    plan = eng.plan_encode([i * item for i in range(n)], [item] * n)
    d_fr = eng.alloc(plan.dst_bound)
    d_io, d_il = eng.alloc(8 * n), eng.alloc(4 * n)
    eng.encode_dev(plan, d_src, d_fr, d_io, d_il)
    eng.sync()
    fo, fl = d_io.u64(n), d_il.u32(n)
    blob = d_fr.read(fo[-1] + fl[-1])
    return blob, fo, fl


def dev_latency(eng, blob, fo, fl, item, n, reps=20):
    base = fo[0]
    end = fo[n - 1] + fl[n - 1]
    d_in = eng.upload(blob[base:end])
    d_out = eng.alloc(n * item)
    d_ol, d_os = eng.alloc(4 * n), eng.alloc(4 * n)
    dp = eng.plan_decode([fo[i] - base for i in range(n)], fl[:n], [i * item for i in range(n)], [item] * n)
    res = {}
    for lb in (True, False):
        if lb:
            S.set_knob("S3HC_LB_DISABLE", None)
        else:
            S.set_knob("S3HC_LB_DISABLE", "1")
        eng.decode_dev(dp, d_in, d_out, d_ol, d_os)
        eng.sync()
        assert d_os.i32(n) == [0] * n
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.decode_dev(dp, d_in, d_out, d_ol, d_os)
            eng.sync()
            ts.append(time.perf_counter() - t0)
        eng.set_timing(True)
        eng.timing_reset()
        eng.decode_dev(dp, d_in, d_out, d_ol, d_os)
        eng.sync()
        kt = eng.timing()
        eng.set_timing(False)
        res["lb" if lb else "nolb"] = {"wall_ms": round(1e3 * float(np.median(ts)), 4),
                                       "stages_ms": {k: round(v[0], 4) for k, v in kt.items()}}
    S.set_knob("S3HC_LB_DISABLE", None)
    return res


def host_call(eng, payload, reps=20):
    eng.decompress_frames(payload)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.decompress_frames(payload)
        ts.append(time.perf_counter() - t0)
    return round(1e3 * float(np.median(ts)), 4)


def reader_rate(eng, blob, total_u, bb, depth):
    h_in = eng.host_alloc(len(blob))
    h_in.view()[:] = np.frombuffer(blob, dtype=np.uint8)
    h_out = eng.host_alloc(total_u)
    rd = S.RangeReader(eng, bb, depth)
    hp, op = h_in.data_ptr(), h_out.data_ptr()
    got = 0
    t0 = time.perf_counter()
    for o in range(0, len(blob), 4 << 20):
        rd.feed_ptr(hp + o, min(4 << 20, len(blob) - o))
        while True:
            k = rd.read_into(op + got, min(1 << 20, total_u - got))
            if not k:
                break
            got += k
    rd.finish()
    while True:
        k = rd.read_into(op + got, min(1 << 20, total_u - got))
        if not k:
            break
        got += k
    dt = time.perf_counter() - t0
    rd.close()
    ok = got == total_u
    h_in.free()
    h_out.free()
    return round(total_u / dt / GiB, 3), ok


def trace_main():
    """Few iterations of each small path (for a rocprofv3 timeline)."""
    eng = S.Engine(0)
    data = synth.log_text(32 << 20, synth.SEED_BASE + 1)
    blob, fo, fl = frames_of(eng, data, 65536)
    dev_latency(eng, blob, fo, fl, 65536, 10, reps=3)
    payload = blob[fo[0]:fo[15] + fl[15]]
    host_call(eng, payload, reps=3)
    print(reader_rate(eng, blob, len(data), 256 << 10, 1))


def main():
    if "--trace" in sys.argv:
        return trace_main()
    eng = S.Engine(0)
    data = synth.log_text(256 << 20, synth.SEED_BASE + 1)
    out = {}
    for fmt, item in (("gpu_64KiB_frames", 65536), ("ref_1MiB_frames", 1 << 20)):
        blob, fo, fl = frames_of(eng, data, item)
        r = {}
        for n in ((1, 4, 10, 40) if item == 65536 else (1, 4)):
            r[f"dev_n{n}"] = dev_latency(eng, blob, fo, fl, item, n)
        k = (1 << 20) // item
        payload = blob[fo[0]:fo[k - 1] + fl[k - 1]]
        r["host_decompress_1MiB_ms"] = host_call(eng, payload)
        for depth in (1, 3):
            r[f"reader_256KiB_depth{depth}_GiBps"] = reader_rate(eng, blob, len(data), 256 << 10, depth)
        out[fmt] = r
        print(json.dumps({fmt: r}), flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
