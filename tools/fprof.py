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
    if v[31]:  # builds with the spread counters: one more launch alone (max / histogram / span of its units)
        f(buf, 32, 1)
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
        eng.sync()
        f(buf, 32, 0)
        w = list(buf)
        out["k_dexec_spread_one_launch"] = {
            "max_unit_total": w[31], "avg_unit_total": round(w[21] / (w[24] or 1), 1), "max_windows": w[9],
            "units_lt600k_lt900k_lt1200k_ge": [w[k] for k in (12, 13, 14, 15)],
            "span_first_start_to_last_end": w[11] - ((~w[8]) & (2**64 - 1))}
        if hasattr(L, "s3hc_diag_uprof"):  # per-unit lives with the SIMD / CU / XCD that ran them
            import numpy as np
            ub = (ctypes.c_ulonglong * (4 * nb))()
            L.s3hc_diag_uprof(ub, nb)
            U = np.frombuffer(ub, dtype=np.uint64).reshape(nb, 4).astype(np.int64)
            life = U[:, 1] - U[:, 0]
            hw, xcc = U[:, 2], U[:, 3] & 15
            simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
            key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
            sp = {}
            # per XCD: its clock's first start and last end (s_memtime is per XCD), mean and max life
            for x in sorted(set(xcc.tolist())):
                m = xcc == x
                sp[f"xcd{x}"] = {"units": int(m.sum()), "span": int(U[m, 1].max() - U[m, 0].min()),
                                 "life_mean": int(life[m].mean()), "life_max": int(life[m].max()),
                                 "start_spread": int(U[m, 0].max() - U[m, 0].min())}
            _, cnt = np.unique(key, return_counts=True)
            order = np.argsort(key, kind="stable")
            # within a SIMD: lives sorted by start, the rank of each wave's end
            ranks = {}
            for k in np.unique(key):
                idx = np.where(key == k)[0]
                ends = np.sort(U[idx, 1] - U[idx, 0].min())
                ranks.setdefault(len(idx), []).append(ends.tolist())
            sweeps, wins = (U[:, 3] >> 8) & 0xFFFFFF, U[:, 3] >> 32
            # what a unit's life follows: its XCD, its sweeps, its windows, its index mod 8
            out["k_dexec_units_corr"] = {
                "life_vs_sweeps": round(float(np.corrcoef(life, sweeps)[0, 1]), 3),
                "life_vs_windows": round(float(np.corrcoef(life, wins)[0, 1]), 3),
                "sweeps_mean_by_xcd": {int(x): round(float(sweeps[xcc == x].mean()), 1) for x in sorted(set(xcc.tolist()))},
                "life_mean_by_unit_mod8": [int(life[np.arange(nb) % 8 == k].mean()) for k in range(8)],
                "life_mean_by_unit_quarter": [int(life[(np.arange(nb) * 4) // nb == k].mean()) for k in range(4)]}
            t0 = U[:, 0].min()
            out["k_dexec_units_realtime_us"] = {  # s_memrealtime: 100 MHz, one clock for the chip
                "launch_span": round((U[:, 1].max() - t0) / 100, 1),
                "per_xcd_first_start_last_end_mean_life": {int(x): [round((U[xcc == x, 0].min() - t0) / 100, 1), round((U[xcc == x, 1].max() - t0) / 100, 1), round(float(life[xcc == x].mean()) / 100, 1)] for x in sorted(set(xcc.tolist()))},
                "start_quartiles": [round(float(np.percentile(U[:, 0] - t0, q)) / 100, 1) for q in (0, 25, 50, 75, 100)],
                "end_quartiles": [round(float(np.percentile(U[:, 1] - t0, q)) / 100, 1) for q in (0, 25, 50, 75, 100)]}
            out["k_dexec_units"] = {"per_xcd": sp, "waves_per_simd_hist": {int(a): int(b) for a, b in zip(*np.unique(cnt, return_counts=True))},
                                    "simd_end_times_mean_by_rank": {n: [int(v) for v in np.mean(np.array(r), axis=0)] for n, r in ranks.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
