#!/usr/bin/env python3
"""Config 2 step (encode 4096 x 64 KiB, then decode the frames) run back to back on one queue,
or pipelined over two queues: step k's decode overlaps step k+1's encode (frames double
buffered; marks order enc(k) -> dec(k) and dec(k) -> enc(k+2)). Prints ms per step of each
mode, alternating, and checks the decoded bytes. Diagnostic tool (not the bench contract)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

GiB = float(1 << 30)


def main():
    nb = int(os.environ.get("BLOCKS", "4096"))
    steps = int(os.environ.get("STEPS", "20"))
    block = 65536
    eng = S.Engine(0)
    data = synth.log_text(nb * block, synth.SEED_BASE + 1)
    d_src = eng.upload(data)
    offs = [i * block for i in range(nb)]
    plan = eng.plan_encode(offs, [block] * nb)
    fr = [eng.alloc(plan.dst_bound) for _ in range(2)]
    io = [eng.alloc(8 * nb) for _ in range(2)]
    il = [eng.alloc(4 * nb) for _ in range(2)]
    d_out, d_ol, d_os = eng.alloc(nb * block), eng.alloc(4 * nb), eng.alloc(4 * nb)
    eng.encode_dev(plan, d_src, fr[0], io[0], il[0])
    eng.sync()
    fo, fl = io[0].u64(nb), il[0].u32(nb)
    dplan = eng.plan_decode(fo, fl, offs, [block] * nb)
    qa, qb = eng.queue(), eng.queue()

    def serial(k):
        for _ in range(k):
            eng.encode_dev(plan, d_src, fr[0], io[0], il[0])
            eng.decode_dev(dplan, fr[0], d_out, d_ol, d_os)
        eng.sync()

    def overlap(k):
        after_dec = {}
        for i in range(k):
            b = i & 1
            if i >= 2:
                m = after_dec.pop(i - 2)
                eng.wait_mark(m, qa)
                eng.free_mark(m)
            eng.encode_dev(plan, d_src, fr[b], io[b], il[b], qa)
            m = eng.mark(qa)
            eng.wait_mark(m, qb)
            eng.free_mark(m)
            eng.decode_dev(dplan, fr[b], d_out, d_ol, d_os, qb)
            after_dec[i] = eng.mark(qb)
        qa.sync()
        qb.sync()
        for m in after_dec.values():
            eng.free_mark(m)

    res = {"serial": [], "overlap": []}
    for fn in (serial, overlap):
        fn(3)
    for _ in range(3):
        for name, fn in (("serial", serial), ("overlap", overlap)):
            d_os.fill(0xFF)
            t0 = time.perf_counter()
            fn(steps)
            dt = time.perf_counter() - t0
            assert d_os.i32(nb) == [0] * nb
            assert d_out.read(4 * block) == data[:4 * block] and d_out.read(block, (nb - 1) * block) == data[-block:]
            res[name].append(round(dt / steps * 1e3, 4))
    out = {k: {"ms_per_step": v, "GiBps_best": round(nb * block / (min(v) / 1e3) / GiB, 2)} for k, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
