#!/usr/bin/env python3
"""Phase timers of the 64 KiB-block fast path in a diagnostic build (S3HC_DIAG_LEVEL=10):
config-2 batch decoded `steps` times; prints per-workgroup / per-wave s_memtime sums of
k_dtok and k_dexec. Usage: S3HC_LIB_PATH=.../build/diag/lib_fprof.so python tools/fprof.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

TOK = {0: "stage", 1: "walk1", 2: "walk2", 3: "chain", 4: "count_alloc", 5: "emit", 6: "total", 10: "max_ovf_per_wave"}
EXE = {16: "decode_next", 17: "literals", 18: "round0", 19: "pending", 20: "flush_or_slow", 21: "total", 22: "windows", 23: "rounds"}


def main():
    nb, block, steps = int(os.environ.get("PROF_BLOCKS", "4096")), 65536, 3
    eng = S.Engine(0)
    L = ctypes.CDLL(S.LIB_PATH)
    f = L.s3hc_diag_fprof
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
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
    eng.sync()
    f(buf, 32, 0)
    v = list(buf)
    assert d_out.read(nb * block) == data
    wg = v[7] or 1  # k_dtok: timers summed over the 4 waves of each workgroup
    out = {"k_dtok_per_wave_cycles": {n: round(v[i] / (4 * wg), 1) for i, n in TOK.items() if i != 10},
           "k_dtok_max_ovf_per_wave": round(v[10] / (4 * wg), 2),
           "k_dexec_per_unit": {n: round(v[i] / (v[24] or 1), 1) for i, n in EXE.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
