#!/usr/bin/env python3
"""End-to-end (host buffer -> host buffer, PCIe included) rates, SURVEY.md §8(d).

config 2: 4096 x 64 KiB log text in pinned host memory. Encode: per 32 MiB chunk, H2D input,
  encode, D2H the chunk's frame table, then D2H exactly the framed bytes; decode: H2D frames,
  decode, D2H output. Chunks rotate over 3 queues (HIP streams) so copies overlap kernels.
config 4: one 8 GiB object (the config-2 text tiled) decoded in host batches through 3 queues:
  (i) GPU format, 64 KiB frames; (ii) reference format, 1 MiB frames of one 1 MiB block
  (BD 0x70, what flush_batch writes at the default batch size). Also device-only decode
  rates of both formats, and raw PCIe copy rates.
Prints one JSON object. Diagnostic tool (not the bench contract).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]
import s3hc_lz4 as S  # noqa: E402
import synth  # noqa: E402

GiB = float(1 << 30)
BLK = 65536


def pcie(eng, nbytes=1 << 30):
    h = eng.host_alloc(nbytes)
    d = eng.alloc(nbytes)
    q = eng.queue()
    out = {}
    for name, kind, dst, src in (("h2d_GBps", 1, d, h), ("d2h_GBps", 2, h, d)):
        eng.copy_async(dst, src, nbytes, kind, q)
        q.sync()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.copy_async(dst, src, nbytes, kind, q)
        q.sync()
        out[name] = round(3 * nbytes / (time.perf_counter() - t0) / 1e9, 2)
    q.close()
    d.free()
    h.free()
    return out


class Lane:
    """One queue with its own device buffers and plans (one chunk in flight)."""

    def __init__(self, eng, chunk_blocks, block, comp_cap):
        self.eng, self.q = eng, eng.queue()
        n = chunk_blocks
        self.src = eng.alloc(n * block)
        self.plan = eng.plan_encode([i * block for i in range(n)], [block] * n)
        self.dst = eng.alloc(self.plan.dst_bound)
        self.ioff, self.ilen = eng.alloc(8 * n), eng.alloc(4 * n)
        self.meta = eng.host_alloc(12 * n)
        self.cin = eng.alloc(comp_cap)
        self.out = eng.alloc(n * block)
        self.olen, self.ost = eng.alloc(4 * n), eng.alloc(4 * n)


def config2(eng, nb=4096, chunk=512, nq=3, reps=3):
    block = BLK
    data = synth.log_text(nb * block, synth.SEED_BASE + 1)
    U = nb * block
    h_in = eng.host_alloc(U)
    h_in.view()[:] = np.frombuffer(data, dtype=np.uint8)
    h_fr = eng.host_alloc(U + U // 8 + (1 << 20))
    h_out = eng.host_alloc(U)
    nch = nb // chunk
    lanes = [Lane(eng, chunk, block, chunk * (block + 64)) for _ in range(nq)]
    frame_tab = [None] * nch  # per chunk: (host offset of its frames, item offsets, item lengths)

    def enc_worker(li):
        L = lanes[li]
        for c in range(li, nch, nq):
            eng.copy_async(L.src, h_in, chunk * block, 1, L.q, src_off=c * chunk * block)
            eng.encode_dev(L.plan, L.src, L.dst, L.ioff, L.ilen, L.q)
            eng.copy_async(L.meta, L.ioff, 8 * chunk, 2, L.q)
            eng.copy_async(L.meta, L.ilen, 4 * chunk, 2, L.q, dst_off=8 * chunk)
            L.q.sync()
            mv = L.meta.view()
            offs = mv[: 8 * chunk].view(np.uint64).copy()
            lens = mv[8 * chunk: 12 * chunk].view(np.uint32).copy()
            total = int(offs[-1] + lens[-1])
            hoff = c * chunk * (block + 64)  # host slot of this chunk's frames
            eng.copy_async(h_fr, L.dst, total, 2, L.q, dst_off=hoff)
            L.q.sync()
            frame_tab[c] = (hoff, offs, lens, total)

    def encode_pass():
        ts = [threading.Thread(target=enc_worker, args=(i,)) for i in range(nq)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    encode_pass()  # warm-up (also builds frame_tab)
    t_enc = min(encode_pass() for _ in range(reps))
    comp = sum(ft[3] for ft in frame_tab)

    dplans = []
    for c in range(nch):
        hoff, offs, lens, total = frame_tab[c]
        dplans.append(eng.plan_decode([int(o) for o in offs], [int(x) for x in lens],
                                      [i * block for i in range(chunk)], [block] * chunk))

    def decode_pass():
        t0 = time.perf_counter()
        for c in range(nch):
            L = lanes[c % nq]
            hoff, offs, lens, total = frame_tab[c]
            eng.copy_async(L.cin, h_fr, total, 1, L.q, src_off=hoff)
            eng.decode_dev(dplans[c], L.cin, L.out, L.olen, L.ost, L.q)
            eng.copy_async(h_out, L.out, chunk * block, 2, L.q, dst_off=c * chunk * block)
        for L in lanes:
            L.q.sync()
        return time.perf_counter() - t0

    decode_pass()
    t_dec = min(decode_pass() for _ in range(reps))
    ok = bytes(h_out.view()[: 4 * block]) == data[: 4 * block] and bytes(h_out.view()[-block:]) == data[-block:]
    return {
        "workload": f"config2 e2e: {nb} x 64 KiB log text, pinned host in/out, {chunk}-block chunks on {nq} queues",
        "encode_GiBps": round(U / t_enc / GiB, 3), "decode_GiBps": round(U / t_dec / GiB, 3),
        "encode_plus_decode_GiBps": round(U / (t_enc + t_dec) / GiB, 3),
        "compressed_bytes": comp, "ratio": round(comp / U, 4), "check": ok,
    }, data, frame_tab, h_fr, chunk


def config4(eng, data2, nq=3, total_gib=8, batch_bytes_list=(256 << 10, 64 << 20, 256 << 20)):
    """8 GiB object decode in host batches. GPU format: 64 KiB frames of the config-2 text
    (tiled); reference format: 1 MiB frames (one 1 MiB block, BD 0x70)."""
    out = {}
    U2 = len(data2)
    tiles = int(total_gib * GiB) // U2
    total_u = tiles * U2
    for fmt, item in (("gpu_64KiB_frames", BLK), ("ref_1MiB_frames", 1 << 20)):
        # encode one 256 MiB tile on the device (frames of `item` bytes), copy to host, tile
        n = U2 // item
        d_src = eng.upload(data2)
        plan = eng.plan_encode([i * item for i in range(n)], [item] * n)
        d_fr = eng.alloc(plan.dst_bound)
        d_io, d_il = eng.alloc(8 * n), eng.alloc(4 * n)
        eng.encode_dev(plan, d_src, d_fr, d_io, d_il)
        eng.sync()
        fo, fl = d_io.u64(n), d_il.u32(n)
        C1 = fo[-1] + fl[-1]
        h_fr = eng.host_alloc(C1 * tiles)
        hv = h_fr.view()
        tile_bytes = np.frombuffer(d_fr.read(C1), dtype=np.uint8)
        for t in range(tiles):
            hv[t * C1:(t + 1) * C1] = tile_bytes
        # device-only decode rate of one tile
        d_out = eng.alloc(U2)
        d_ol, d_os = eng.alloc(4 * n), eng.alloc(4 * n)
        dp = eng.plan_decode(fo, fl, [i * item for i in range(n)], [item] * n)
        eng.decode_dev(dp, d_fr, d_out, d_ol, d_os)
        eng.sync()
        assert d_os.i32(n) == [0] * n
        eng.set_timing(True)
        eng.timing_reset()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.decode_dev(dp, d_fr, d_out, d_ol, d_os)
        eng.sync()
        t_dev = (time.perf_counter() - t0) / 3
        kt = eng.timing()
        eng.set_timing(False)
        res = {"frames_per_tile": n, "ratio": round(C1 / U2, 4),
               "device_decode_GiBps": round(U2 / t_dev / GiB, 3),
               "device_decode_kernel_ms": round(kt.get("decode", (0, 1))[0] / 3, 3)}
        # e2e decode of the whole object in host batches
        h_out = eng.host_alloc(total_u)
        for bb in batch_bytes_list:
            fpb = max(1, bb // item)  # frames per batch
            nbat = (tiles * n) // fpb
            lanes = []
            for _ in range(nq):
                q = eng.queue()
                cin = eng.alloc(fpb * (item + 64))
                dout = eng.alloc(fpb * item)
                ol, os_ = eng.alloc(4 * fpb), eng.alloc(4 * fpb)
                lanes.append((q, cin, dout, ol, os_))
            # batches are identical in layout within a tile: one plan per distinct batch and queue
            # (a plan's scratch belongs to one call in flight at a time, include/s3hc_lz4.h)
            plans = {}
            def plan_for(k):
                f0 = (k * fpb) % n
                key = (k % nq, f0)
                if key not in plans:
                    base = fo[f0]
                    plans[key] = eng.plan_decode([fo[f0 + j] - base for j in range(fpb)], fl[f0:f0 + fpb],
                                                 [j * item for j in range(fpb)], [item] * fpb)
                return plans[key]
            for k in range(min(nbat, nq * (n // fpb))):
                plan_for(k)
            t0 = time.perf_counter()
            for k in range(nbat):
                q, cin, dout, ol, os_ = lanes[k % nq]
                t, f0 = divmod(k * fpb, n)
                src = t * C1 + fo[f0]
                clen = fo[f0 + fpb - 1] + fl[f0 + fpb - 1] - fo[f0]
                eng.copy_async(cin, h_fr, clen, 1, q, src_off=src)
                eng.decode_dev(plan_for(k), cin, dout, ol, os_, q)
                eng.copy_async(h_out, dout, fpb * item, 2, q, dst_off=k * fpb * item)
            for L in lanes:
                L[0].sync()
            dt = time.perf_counter() - t0
            res[f"e2e_decode_GiBps_batch_{bb >> 10}KiB"] = round(nbat * fpb * item / dt / GiB, 3)  # Python-driven
            # 32 frames spread over the object, each compared whole
            hv = h_out.view()
            nfr = nbat * fpb
            ok = all(bytes(hv[g * item:(g + 1) * item]) == data2[(g % n) * item:(g % n + 1) * item]
                     for g in sorted({(i * 7919) % nfr for i in range(31)} | {nfr - 1}))
            res[f"check_batch_{bb >> 10}KiB"] = ok
            for L in lanes:
                L[0].close()
        # the C++ pipelined range reader (s3hc_reader): the object's frames fed in 4 MiB file
        # reads, decoded bytes read back in 1 MiB chunks (stream_range_data's chunk size); fixed
        # batches, and 256 KiB batches that may grow to 16 MiB behind running ones (batch_max)
        for bb, bmax in ((256 << 10, None), (256 << 10, 16 << 20), (4 << 20, None), (64 << 20, None)):
            rd = S.RangeReader(eng, bb, nq, bmax)
            hp, op = h_fr.data_ptr(), h_out.data_ptr()
            ctot, got = C1 * tiles, 0
            t0 = time.perf_counter()
            for o in range(0, ctot, 4 << 20):
                rd.feed_ptr(hp + o, min(4 << 20, ctot - o))
                while True:
                    k = rd.read_into(op + got, min(1 << 20, total_u - got))
                    if not k:
                        break
                    got += k
            rd.finish()
            while True:
                k = rd.read_into(op + got, min(1 << 20, total_u - got))
                if not k:
                    break
                got += k
            dt = time.perf_counter() - t0
            assert got == total_u and rd.total == total_u
            tag = f"{bb >> 10}KiB" + (f"_adaptive_max{bmax >> 20}MiB" if bmax else "")
            res[f"reader_decode_GiBps_batch_{tag}"] = round(total_u / dt / GiB, 3)
            res[f"reader_check_batch_{tag}"] = bytes(h_out.view()[-item:]) == data2[-item:]
            rd.close()
        out[fmt] = res
        h_out.free()
        h_fr.free()
    out["object_bytes"] = total_u
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-config4", action="store_true")
    ap.add_argument("--skip-config2", action="store_true")
    ap.add_argument("--gib", type=float, default=8.0)
    a = ap.parse_args()
    eng = S.Engine(0)
    res = {"pcie": pcie(eng)}
    if a.skip_config2:
        data2 = synth.log_text(4096 * BLK, synth.SEED_BASE + 1)
    else:
        c2, data2, *_ = config2(eng)
        res["config2"] = c2
    if not a.skip_config4:
        res["config4"] = config4(eng, data2, total_gib=a.gib)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
