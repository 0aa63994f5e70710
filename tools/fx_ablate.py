#!/usr/bin/env python3
"""Phase ablation of k_dexec (diagnostic builds with -DS3HC_FXSKIP=mask; their output is wrong):
config-2 decode time per library. Usage: python tools/fx_ablate.py lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time
sys.path[:0] = [os.path.join(%r, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S, synth
nb, block = int(os.environ.get("FX_BLOCKS", "4096")), 65536
eng = S.Engine(0)
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
for _ in range(3):
    eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
eng.sync()
best = 1e9
for _ in range(5):
    t = time.perf_counter()
    for _ in range(10):
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
    eng.sync()
    best = min(best, (time.perf_counter() - t) / 10)
print(round(best * 1e3, 4))
''' % ROOT

if os.environ.get("FX_INPROC"):  # one library, in this process (for rocprofv3 --pmc)
    exec(CHILD)
    sys.exit(0)
res = {}
for lib in sys.argv[1:]:
    env = dict(os.environ, S3HC_LIB_PATH=lib, S3HC_FAST="1")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    res[os.path.basename(lib)] = r.stdout.strip() or r.stderr[-300:]
    print(os.path.basename(lib), res[os.path.basename(lib)], flush=True)
print(json.dumps(res))
