#!/usr/bin/env python3
"""Dump GPU-encoded config-2 frames (the bench's first chunk, first N blocks) for offline token
statistics (tools/seqstats.py). Usage: python tools/dump_frames.py [N] -> gpurun_out/frames.bin
(+ frames.json: offsets/lengths)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd"), ROOT]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = 65536
data = synth.log_text(4096 * B, bench.chunk_seed(0, 0))[: n * B]
eng = S.Engine(0)
d_src = eng.upload(data)
offs = [i * B for i in range(n)]
plan = eng.plan_encode(offs, [B] * n)
dst = eng.alloc(plan.dst_bound)
ioff, ilen = eng.alloc(8 * n), eng.alloc(4 * n)
eng.encode_dev(plan, d_src, dst, ioff, ilen)
eng.sync()
fo, fl = ioff.u64(n), ilen.u32(n)
blob = dst.read(fo[-1] + fl[-1])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", "frames.bin"), "wb").write(blob)
json.dump({"fo": fo, "fl": fl, "block": B, "seed": bench.chunk_seed(0, 0)},
          open(os.path.join(ROOT, "gpurun_out", "frames.json"), "w"))
print("frames", n, "bytes", len(blob))
