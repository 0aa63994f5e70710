#!/usr/bin/env python3
"""Config-2 batch encode repeated, per-phase kernel times by the library's event spans; for A/B runs
of diagnostic libraries (S3HC_LIB_PATH=...), including ablations whose frames are not valid (no
decode check unless --check). Prints one JSON line: tag, enc_parse / enc_sizes / enc_emit ms
(mean over reps), compressed ratio.
usage: python tools/enc_time.py [--reps N] [--check] [--tag T]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("S3HC_LIB_PATH", "base")))
    ap.add_argument("--mode", type=int, default=0, help="encode mode: 0 fast, 1 small")
    a = ap.parse_args()
    nb, block = 4096, 65536
    eng = S.Engine(0)
    eng.set_encode_mode(a.mode)
    data = synth.log_text(nb * block, synth.SEED_BASE + 1)
    offs = [i * block for i in range(nb)]
    d_src = eng.upload(data)
    plan = eng.plan_encode(offs, [block] * nb)
    d_frames = eng.alloc(plan.dst_bound)
    d_ioff, d_ilen = eng.alloc(8 * nb), eng.alloc(4 * nb)
    eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
    eng.sync()
    eng.set_timing(True)
    eng.timing_reset()
    for _ in range(a.reps):
        eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
    eng.sync()
    t = eng.timing()
    eng.set_timing(False)
    ilen = d_ilen.u32(nb)
    out = {"tag": a.tag, "mode": a.mode, "ratio": round(sum(ilen) / (nb * block), 4)}
    out.update({k: round(v[0] / v[1], 4) for k, v in t.items() if k.startswith("enc")})
    if a.check:
        d_out = eng.alloc(nb * block)
        d_olen, d_ost = eng.alloc(4 * nb), eng.alloc(4 * nb)
        dplan = eng.plan_decode(d_ioff.u64(nb), ilen, offs, [block] * nb)
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)
        eng.sync()
        out["check"] = d_out.read(nb * block) == data
    print(json.dumps(out))


if __name__ == "__main__":
    main()
