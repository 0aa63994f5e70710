#!/usr/bin/env python3
"""Large-block decode timing (csrc/s3hc_lb.hip) against the one-wave decoder.

Device-resident decode (plan_decode + decode_dev, inputs already in HBM) of N frames in the
reference's own cache-file format: BlockSize::Auto frames of one large block each (1 MiB
batches -> BD 0x70 with one 1 MiB block; also 4 MiB blocks and 256 KiB BD 0x50 blocks). Each
case is timed with the large-block path and with S3HC_LB_DISABLE=1 (every block on one wave).
Prints one JSON object.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]

import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

GiB = 1 << 30
MiB = 1 << 20


def case(eng, data, item, reps=5):
    n = len(data) // item
    d_src = eng.upload(data)
    plan = eng.plan_encode([i * item for i in range(n)], [item] * n)
    d_fr = eng.alloc(plan.dst_bound)
    d_io, d_il = eng.alloc(8 * n), eng.alloc(4 * n)
    eng.encode_dev(plan, d_src, d_fr, d_io, d_il)
    eng.sync()
    fo, fl = d_io.u64(n), d_il.u32(n)
    C = fo[-1] + fl[-1]
    d_out = eng.alloc(n * item + 64)
    d_ol, d_os = eng.alloc(4 * n), eng.alloc(4 * n)
    dp = eng.plan_decode(fo, fl, [i * item for i in range(n)], [item] * n)
    res = {"frames": n, "frame_bytes": item, "ratio": round(C / (n * item), 4)}
    for mode in ("lb", "wave"):
        if mode == "wave":
            S.set_knob("S3HC_LB_DISABLE", "1")
        try:
            d_out.fill(0)
            eng.decode_dev(dp, d_fr, d_out, d_ol, d_os)
            eng.sync()
            ok = d_os.i32(n) == [0] * n and d_out.read(item) == data[:item] and \
                d_out.read(item, (n - 1) * item) == data[(n - 1) * item:n * item]
            eng.set_timing(True)
            eng.timing_reset()
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.decode_dev(dp, d_fr, d_out, d_ol, d_os)
            eng.sync()
            dt = (time.perf_counter() - t0) / reps
            kt = eng.timing()
            eng.set_timing(False)
        finally:
            S.set_knob("S3HC_LB_DISABLE", None)
        res[mode] = {"ms": round(dt * 1e3, 3), "GiBps": round(n * item / dt / GiB, 3),
                     "decode_kernels_ms": round(kt.get("decode", (0, 1))[0] / reps, 3), "check": ok}
    res["speedup"] = round(res["wave"]["ms"] / res["lb"]["ms"], 2)
    return res


def main():
    eng = S.Engine(0)
    text = synth.log_text(256 * MiB, synth.SEED_BASE + 1)
    out = {}
    if len(sys.argv) > 1:  # one case (profiling): tools/lb.py <frames of 1 MiB> [zeros]
        n = int(sys.argv[1])
        data = bytes(n * MiB) if "zeros" in sys.argv else text[:n * MiB]
        print(json.dumps(case(eng, data, MiB, reps=2)))
        if hasattr(S.lib, "s3hc_diag_lbprof"):  # diagnostic build: k_lb_run phase times per step
            import ctypes
            buf = (ctypes.c_ulonglong * 32)()
            S.lib.s3hc_diag_lbprof(buf, 1)
            v = list(buf)
            steps = max(v[7], 1)
            names = ["owners", "classify_loads", "stores", "next_seqs", "jumps", "flush", "-", "steps",
                     "jump_rounds", "loop_top", "jump_top_barrier", "jump_work_t0"]
            print(json.dumps({nm: (round(v[k] / steps, 1) if k not in (7,) else v[k]) for k, nm in enumerate(names)}))
            # k_lb_mark phases (cycles summed over chunks): load/stage, sub-range jumps, walks, tokenize, scans
            print(json.dumps({"mark_phases_Mcycles": [round(x / 1e6, 2) for x in v[12:17]]}))
            ch = max(v[24], 1)  # segment-walk tokenizer (S3HC_LB_TOKV2): per-chunk phase cycles and hop maxima
            print(json.dumps({"walk_phases_per_chunk": [round(x / ch) for x in v[12:16]],
                              "mark_phases_per_chunk": [round(x / ch) for x in v[16:20]],
                              "max_hops_per_chunk_w2_first_entry_remark": [round(x / ch, 1) for x in v[20:24]],
                              "chunks": v[24]}))
        return
    for n in (1, 4, 16, 64, 256):
        out[f"log_1MiB_x{n}"] = case(eng, text[:n * MiB], MiB)
        print(n, out[f"log_1MiB_x{n}"], flush=True, file=sys.stderr)
    out["log_4MiB_x16"] = case(eng, text[:64 * MiB], 4 * MiB)
    out["log_256KiB_x256"] = case(eng, text[:64 * MiB], 256 << 10)
    out["json_1MiB_x64"] = case(eng, synth.json_records(64 * MiB, 7), MiB)
    out["zeros_4MiB_x4"] = case(eng, bytes(16 * MiB), 4 * MiB)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
