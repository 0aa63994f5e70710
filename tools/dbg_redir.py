#!/usr/bin/env python3
"""Debug: decode 64 KiB frames through the fast path (S3HC_LB_DISABLE=1) with the library named by
S3HC_LIB_PATH; print the first mismatching byte of each failing input and the sequence there."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402
import oracle as O  # noqa: E402


def seqs_of(frame):
    bs = int.from_bytes(frame[7:11], "little")
    b = frame[11:11 + (bs & 0x7FFFFFFF)]
    p, out, res = 0, 0, []
    while p < len(b):
        t = b[p]; p += 1
        L = t >> 4
        if L == 15:
            while True:
                e = b[p]; p += 1; L += e
                if e != 255:
                    break
        p += L
        if p >= len(b):
            res.append((out, L, 0, 0)); break
        off = b[p] | (b[p + 1] << 8); p += 2
        M = (t & 15) + 4
        if (t & 15) == 15:
            while True:
                e = b[p]; p += 1; M += e
                if e != 255:
                    break
        res.append((out, L, off, M))
        out += L + M
    return res


eng = S.Engine(0)
ins = {"log": synth.log_text(65536, 51), "json": synth.json_records(65536, 52), "log2": synth.log_text(65536, 7)}
with S.knobs({"S3HC_LB_DISABLE": "1"}):
    for name, data in ins.items():
        for fname, f in (("gpu", eng.compress_frame(data)), ("oracle", O.lz4flex_compress_frame(data))):
            try:
                got = eng.decompress_frames(f)
                print(name, fname, "ok" if got == data else "WRONG")
            except S.CodecError as e:
                print(name, fname, "error", e)
                # decode without checksum verification: strip the content checksum flag
                g = O._without_content_checksum(f)
                got = eng.decompress_frames(g)
                bad = [i for i in range(min(len(got), len(data))) if got[i] != data[i]]
                print("  mismatching bytes:", len(bad), "first", bad[:8])
                if bad:
                    x = bad[0]
                    for s in seqs_of(f):
                        if s[0] <= x < s[0] + s[1] + s[3] + 40 and s[0] + s[1] + s[3] > x - 60:
                            print("   seq out=%d ll=%d off=%d ml=%d  (window %d, window pos %d)" % (s[0], s[1], s[2], s[3], 0, 0))
