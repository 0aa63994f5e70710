#!/usr/bin/env python3
"""Per-unit lives of k_dexec in a build with -DS3HC_UPROF=1 (start/end on the chip-wide 100 MHz
clock, the SIMD / CU / XCD that ran each unit; no phase timers, so the kernel runs at full speed):
config-2 batch decoded `steps` times, the last launch analysed. Usage:
S3HC_LIB_PATH=.../build/diag/lib_uprof.so python tools/uprof.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402


def main():
    nb, block, steps = int(os.environ.get("PROF_BLOCKS", "4096")), 65536, 5
    eng = S.Engine(0)
    L = ctypes.CDLL(S.LIB_PATH)
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
    res = []
    for _ in range(steps):
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
        eng.sync()
        ub = (ctypes.c_ulonglong * (4 * nb))()
        assert L.s3hc_diag_uprof(ub, nb) == 0
        U = np.frombuffer(ub, dtype=np.uint64).reshape(nb, 4).astype(np.int64)
        t0 = U[:, 0].min()
        st, en = (U[:, 0] - t0) / 100.0, (U[:, 1] - t0) / 100.0  # us
        life = en - st
        hw, xcc = U[:, 2], U[:, 3] & 15
        simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
        key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
        ranks = []
        for k in np.unique(key):
            idx = np.where(key == k)[0]
            if len(idx) == 4:
                ranks.append(np.sort(en[idx]))
        res.append({
            "span_us": round(float(en.max()), 1),
            "xcd_last_end_us": [round(float(en[xcc == x].max()), 1) for x in range(8)],
            "xcd_mean_life_us": [round(float(life[xcc == x].mean()), 1) for x in range(8)],
            "end_pct_10_50_90_100_us": [round(float(np.percentile(en, q)), 1) for q in (10, 50, 90, 100)],
            "simd_end_by_rank_mean_us": [round(float(v), 1) for v in np.mean(np.array(ranks), axis=0)] if ranks else None,
            "simd_last_end_pct_10_50_90_us": [round(float(np.percentile(np.array(ranks)[:, -1], q)), 1) for q in (10, 50, 90)] if ranks else None,
        })
    assert d_out.read(nb * block) == data
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
