#!/usr/bin/env python3
"""Host-buffer decompress_frames latency (one 1 MiB payload: 16 x 64 KiB frames, or one
reference 1 MiB frame): sorted per-call times; S3HC_HOST_TRACE=1 adds the library's stage times."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

eng = S.Engine(0)
data = synth.log_text(1 << 20, 5)
reps = int(os.environ.get("REPS", "40"))
for name, pol in (("64k", 1), ("1m", 0)):
    fr = eng.compress_frame(data, pol)
    eng.decompress_frames(fr)
    for mode in ("alloc", "cap"):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = eng.decompress_frames(fr) if mode == "alloc" else eng.decompress_frames(fr, len(data))
            ts.append((time.perf_counter() - t0) * 1e3)
        assert out == data
        print(name, mode, [round(x, 3) for x in sorted(ts)[::max(1, reps // 8)]], flush=True)
