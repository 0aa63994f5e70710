#!/usr/bin/env python3
"""Phase timers of a diagnostic build (S3HC_DIAG_LEVEL=10): config-2 batch, encode + decode
`--steps` times, then prints the per-phase s_memtime sums of k_decode_units / k_enc_parse.
Usage: S3HC_LIB_PATH=.../build/diag/lib_prof.so python tools/prof.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

DEC = ["stage", "parse_walk", "window", "seq", "wave_total", "windows", "members", "passes",
       "pend_windows", "stages", "flush", "bytes", "steps", "walk", "pending", "far_passes"]
ENC = {16: "stage", 17: "cand", 18: "long_ext", 19: "walk", 20: "flush", 21: "wave_total", 22: "subblocks",
       23: "hops", 24: "long_matches"}


def main():
    nb, block, steps = int(os.environ.get("PROF_BLOCKS", "4096")), 65536, 3
    eng = S.Engine(0)
    L = ctypes.CDLL(S.LIB_PATH)
    f = L.s3hc_diag_prof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    data = synth.log_text(nb * block, synth.SEED_BASE + 1)
    offs = [i * block for i in range(nb)]
    d_src = eng.upload(data)
    plan = eng.plan_encode(offs, [block] * nb)
    d_frames = eng.alloc(plan.dst_bound)
    d_ioff, d_ilen = eng.alloc(8 * nb), eng.alloc(4 * nb)
    d_out = eng.alloc(nb * block)
    d_olen, d_ost = eng.alloc(4 * nb), eng.alloc(4 * nb)
    eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
    eng.sync()
    fo, fl = d_ioff.u64(nb), d_ilen.u32(nb)
    dplan = eng.plan_decode(fo, fl, offs, [block] * nb)
    eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
    eng.sync()
    f(buf, 32, 1)
    for _ in range(steps):
        eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
    eng.sync()
    f(buf, 32, 0)
    v = list(buf)
    waves = nb * steps
    out = {"decode": {}, "encode": {}}
    for i, n in enumerate(DEC):
        out["decode"][n] = round(v[i] / waves, 1)
    segs = nb * 16 * steps
    for i, n in ENC.items():
        out["encode"][n] = round(v[i] / segs, 1)
    tot = v[4] or 1
    out["decode_frac"] = {n: round(v[i] / tot, 3) for i, n in enumerate(DEC[:4] + ["x", "x", "x", "x", "x", "x", "flush"]) if n != "x"}
    if v[21]:
        out["encode_frac"] = {ENC[i]: round(v[i] / v[21], 3) for i in range(16, 21)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
