#!/usr/bin/env python3
"""Compressed sizes of a few inputs under two library builds (diagnostic: ratio impact of an
encoder change). Usage: python tools/ratio_cmp.py LIB_A LIB_B"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, os, json
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import numpy as np, s3hc_lz4 as S, synth
eng = S.Engine(0)
inp = {"zeros_64k": bytes(65536), "runs": b"".join(bytes([c]) * (i % 97 + 1) for i, c in enumerate(b"abcdefghij" * 300)),
       "log_1MiB": synth.log_text(1 << 20, 12), "json_1MiB": synth.json_records(1 << 20, 3),
       "log_64k_x16": synth.log_text(16 << 16, 5), "p251_1MiB": bytes(i % 251 for i in range(1 << 20)),
       "spaces_text": (b"key    =    value   " * 4000)}
out = {}
for k, v in inp.items():
    out[k] = [len(v), len(eng.compress_frame(v, 0)), len(eng.compress_frame(v, 1))]
print(json.dumps(out))
'''
res = {}
for lib in sys.argv[1:]:
    env = dict(os.environ, S3HC_LIB_PATH=lib)
    r = subprocess.run([sys.executable, "-c", "ROOT=%r\n" % ROOT + CODE], env=env, capture_output=True, text=True, timeout=300)
    res[os.path.basename(lib)] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-500:]
print(json.dumps(res, indent=1))
