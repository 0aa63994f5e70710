#!/usr/bin/env python3
"""Debug helper: encode config-2 blocks on the GPU, decode them, and dump (compressed frame,
expected bytes, GPU output) of the first frames whose decode differs to gpurun_out/dbg/."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

n, B = int(os.environ.get("DBG_BLOCKS", "4096")), 65536
eng = S.Engine(0)
data = synth.log_text(n * B, synth.SEED_BASE + 1)
d_src = eng.upload(data)
offs = [i * B for i in range(n)]
plan = eng.plan_encode(offs, [B] * n)
dst = eng.alloc(plan.dst_bound)
ioff, ilen = eng.alloc(8 * n), eng.alloc(4 * n)
eng.encode_dev(plan, d_src, dst, ioff, ilen)
eng.sync()
fo, fl = ioff.u64(n), ilen.u32(n)
dplan = eng.plan_decode(fo, fl, offs, [B] * n)
out = eng.alloc(n * B)
olen, ost = eng.alloc(4 * n), eng.alloc(4 * n)
eng.decode_dev(dplan, dst, out, olen, ost)
eng.sync()
st = ost.i32(n)
got = out.read(n * B)
frames = dst.read(fo[-1] + fl[-1])
os.makedirs(os.path.join(ROOT, "gpurun_out", "dbg"), exist_ok=True)
bad = [i for i in range(n) if st[i] != 0 or got[i * B:(i + 1) * B] != data[i * B:(i + 1) * B]]
print("bad frames", len(bad), bad[:20])
for i in bad[:4]:
    with open(os.path.join(ROOT, "gpurun_out", "dbg", f"f{i}.bin"), "wb") as fh:
        fh.write(frames[fo[i]:fo[i] + fl[i]])
    with open(os.path.join(ROOT, "gpurun_out", "dbg", f"g{i}.bin"), "wb") as fh:
        fh.write(got[i * B:(i + 1) * B])
    with open(os.path.join(ROOT, "gpurun_out", "dbg", f"r{i}.bin"), "wb") as fh:
        fh.write(data[i * B:(i + 1) * B])
