#!/usr/bin/env python3
"""sha256 of the frames the loaded library encodes for a fixed set of inputs (A/B of encoder
builds: the same digest means byte-identical frames). Usage: [S3HC_LIB_PATH=...] python tools/frames_sha.py"""
import hashlib
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

eng = S.Engine(0)
rng = random.Random(9)
h = hashlib.sha256()
inputs = [synth.log_text(512 * 65536, 3), synth.json_records(64 * 65536, 4), bytes(300000),
          b"".join(bytes([rng.randrange(256)]) * rng.choice([1, 3, 50, 300]) for _ in range(5000)),
          rng.randbytes(200000), synth.log_text(1 << 20, 5)]
for d in inputs:
    for pol in (0, 1):
        h.update(eng.compress_frame(d, pol))
print(h.hexdigest())
