#!/usr/bin/env python3
"""Phase timers of k_dsmall (the range reader's fused small-launch decode) in a diagnostic build
(S3HC_DIAG_LEVEL=10): `nb` 64 KiB log-text frames (default 11, one 256 KiB reader batch) decoded
through the host-walked path `steps` times. Prints the token-index phases (per wave, cycles) and
the executor phases (k_dsmall) or the pointer-jumping phases (k_djump) per block, cycles, and the wall time per call.
Usage: S3HC_LIB_PATH=.../build/diag/lib_prof.so python tools/fprof_small.py [nb]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

TOK = {0: "stage", 1: "walk1", 2: "walk2", 3: "chain", 4: "count_alloc", 5: "emit", 6: "total"}
EXE = {16: "decode_next", 17: "literals", 18: "round0", 19: "pending", 20: "flush_or_slow", 21: "total",
       22: "windows", 23: "rounds"}
JMP = {25: "positions_pointers", 26: "jumping", 27: "gather", 28: "hash", 29: "rounds"}


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    block, steps = 65536, 20
    eng = S.Engine(0)
    L = ctypes.CDLL(S.LIB_PATH)
    f = L.s3hc_diag_fprof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    data = synth.log_text(nb * block, synth.SEED_BASE + 3)
    frames = b"".join(eng.compress_frame(data[i * block:(i + 1) * block]) for i in range(nb))
    assert eng.decompress_frames(frames, nb * block) == data
    f(buf, 32, 1)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.decompress_frames(frames, nb * block)
    dt = (time.perf_counter() - t0) / steps
    f(buf, 32, 0)
    v = list(buf)
    wg = v[7] or 1
    units = v[24] or 1
    out = {"frames": nb, "compressed": len(frames), "call_us": round(dt * 1e6, 1),
           "dtok_per_wave_cycles": {n: round(v[i] / (4 * wg), 1) for i, n in TOK.items()},
           "dexec_per_block": {n: round(v[i] / units, 1) for i, n in EXE.items()},
           "djump_per_block": {n: round(v[i] / (v[30] or 1), 1) for i, n in JMP.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
