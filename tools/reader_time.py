#!/usr/bin/env python3
"""Config 4 reader, fixed 256 KiB batches: where the host's time goes (feed = submit side, read =
wait + delivery), for 64 KiB frames and the reference's 1 MiB frames, depth 3 and 4; --slots
sweeps S3HC_READER_SLOTS (batches in flight per queue), --reps alternates the runs.
Usage: python tools/reader_time.py [--mib N] [--depths 3] [--slots 1,2] [--reps 2]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402


def run(eng, frames_h, ctot, total_u, out_h, bb, depth, bmax=None):
    rd = S.RangeReader(eng, bb, depth, bmax)
    hp, op = frames_h.data_ptr(), out_h.data_ptr()
    got, tf, tr = 0, 0.0, 0.0
    t0 = time.perf_counter()
    for o in range(0, ctot, 4 << 20):
        a = time.perf_counter()
        rd.feed_ptr(hp + o, min(4 << 20, ctot - o))
        b = time.perf_counter()
        while True:
            k = rd.read_into(op + got, min(1 << 20, total_u - got))
            if not k:
                break
            got += k
        tf += b - a
        tr += time.perf_counter() - b
    rd.finish()
    a = time.perf_counter()
    while True:
        k = rd.read_into(op + got, min(1 << 20, total_u - got))
        if not k:
            break
        got += k
    tr += time.perf_counter() - a
    dt = time.perf_counter() - t0
    rd.close()
    assert got == total_u
    return {"GiBps": round(total_u / dt / 2**30, 3), "feed_s": round(tf, 4), "read_s": round(tr, 4), "wall_s": round(dt, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--only", default="")
    ap.add_argument("--depths", default="3,4")
    ap.add_argument("--slots", default="")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    eng = S.Engine(0)
    data = synth.log_text(a.mib << 20, 7)
    res = {}
    for name, item, pol in (("64KiB_frames", 65536, 0), ("ref_1MiB_frames", 1 << 20, 0)):
        if a.only and a.only not in name:
            continue
        fr = b"".join(eng.compress_frame(data[i:i + item], pol) for i in range(0, len(data), item))
        h_fr = eng.host_alloc(len(fr))
        h_fr.view()[:] = np.frombuffer(fr, dtype=np.uint8)
        h_out = eng.host_alloc(len(data))
        for rep in range(a.reps):
            for depth in [int(x) for x in a.depths.split(",")]:
                for sl in (a.slots.split(",") if a.slots else [None]):
                    with S.knobs({"S3HC_READER_SLOTS": sl}):
                        r = run(eng, h_fr, len(fr), len(data), h_out, 256 << 10, depth)
                    assert bytes(h_out.view()[-item:]) == data[-item:]
                    key = f"{name}_depth{depth}" + (f"_slots{sl}" if sl else "") + (f"_rep{rep}" if a.reps > 1 else "")
                    res[key] = r
                    print(key, r, flush=True)
        h_fr.free()
        h_out.free()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
