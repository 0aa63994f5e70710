#!/usr/bin/env python3
"""bench.py — LZ4 encode+decode GiB/s (device-resident), 64 KiB blocks, 1/2/4/8 GPUs.

Workload (BASELINE.json configs[1]): 4096 x 64 KiB synthetic
log-text blocks per GPU, resident in HBM before the timed region. One step = one pass of
the hot path over the batch: encode every block into an LZ4 frame (lz4_flex layout:
FLG 0x64, BD 0x40, xxh32 content checksum; frames packed contiguously) then decode every
frame back (frame walk, block decode, xxh32 verify). value = uncompressed bytes of all
ranks / (max over ranks of the timed wall time), i.e. U / (t_enc + t_dec).

Multi-GPU: one process per GPU (torch.distributed.run), blocks sharded across ranks with
no data-path collective (weak scaling: 4096 blocks per GPU); a gloo (CPU) group provides
the barrier and the max-over-ranks reduction of the timed interval.

The roofline object is for the dominant kernel of the step, from HIP events recorded inside
the library on the launch stream over the timed steps. cpu_baseline times the CPU port of
the reference path (oracle/: the lz4_flex FrameEncoder/FrameDecoder restatement) on the
host's cores over a bounded sample of the same workload (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd")]

import s3hc_lz4 as S  # noqa: E402
import shard  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.3 measured)
METRIC = "LZ4 encode+decode GiB/s (device-resident), 64 KiB blocks, 1/2/4/8 GPU"
GiB = float(1 << 30)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=4096, help="64 KiB blocks per GPU (config 2: 4096; weak scaling)")
    ap.add_argument("--total-blocks", type=int, default=0,
                    help="strong scaling instead: split this many blocks over the ranks (config 5: 1048576)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--skip-check", action="store_true", help="diagnostic builds only: skip output checks")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall seconds of the CPU baseline sample")
    return ap.parse_args()


def cpu_baseline(data: bytes, block: int, seconds: float):
    """Oracle (C port of the reference path) on the host cores, encode+decode per block."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg only

    L = O.lib()
    threads = max(1, min(16, os.cpu_count() or 1))
    nb = len(data) // block
    buf = ctypes.create_string_buffer(data, len(data))
    base = ctypes.addressof(buf)
    cap = O.lib().or_frame_bound(block)

    def work(lo, count):
        fr = ctypes.create_string_buffer(cap)
        out = ctypes.create_string_buffer(block)
        n = ctypes.c_size_t()
        te = td = 0.0
        for k in range(count):
            i = (lo + k) % nb
            t0 = time.perf_counter()
            L.or_lz4flex_compress_frame(base + i * block, block, fr, cap, ctypes.byref(n))
            t1 = time.perf_counter()
            m = ctypes.c_size_t()
            rc = L.or_decompress_data(fr, n.value, out, block, ctypes.byref(m))
            t2 = time.perf_counter()
            assert rc == 0 and m.value == block
            te += t1 - t0
            td += t2 - t1
        return te, td, count

    # single thread: seconds per block (encode + decode)
    te, td, k = work(0, min(nb, 64))
    per_blk = (te + td) / k
    # all threads, each on its own contiguous block range (one request per blocking thread),
    # sized to ~`seconds` of wall time
    per_thread = max(1, int(seconds / per_blk))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(work, (t * nb) // threads, per_thread) for t in range(threads)]
        res = [f.result() for f in futs]
    wall = time.perf_counter() - t0
    blocks = sum(r[2] for r in res)
    return {
        "value": round(blocks * block / wall / GiB, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{blocks} x 64 KiB blocks of the same log-text batch (lz4_flex-faithful frame encode + decompress_data "
                  f"per block, oracle/ C port -O3), {threads} threads over contiguous block ranges, {wall:.2f} s wall "
                  f"= {wall * threads:.1f} CPU-s",
        "single_thread_gibps": round(block / per_blk / GiB, 4),
        "single_thread_encode_gibps": round(k * block / te / GiB, 4),
        "single_thread_decode_gibps": round(k * block / td / GiB, 4),
        "host_nproc": os.cpu_count(),
    }


KERNEL_SYMBOL = {"enc_parse": "k_enc_parse", "enc_emit": "k_enc_emit", "decode": "k_decode_units",
                 "xxh32": "k_xxh32_ranges"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/rNN/traffic.json, made by tools_traffic.sh from this same bench command:
    FETCH_SIZE and WRITE_SIZE in separate --pmc passes, per-dispatch averages in KB).
    FETCH_SIZE is doubled: on gfx950 it counts half the bytes of 16-B/lane streaming reads."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    k = d.get(KERNEL_SYMBOL.get(kernel, kernel), {})
    if "FETCH_SIZE" not in k or "WRITE_SIZE" not in k:
        return None, None
    return int((2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024), os.path.relpath(files[-1], ROOT)


def main():
    args = parse_args()
    g = shard.Group()
    world, rank, local = g.world, g.rank, g.local
    block = 65536
    if args.total_blocks:
        lo, hi = shard.shard_range(args.total_blocks, world, rank)
        nb = hi - lo
    else:
        nb = args.blocks
    eng = S.Engine(local % max(1, S.device_count()))  # one process per GPU (shared GPU only in CPU-box rehearsals)

    # ---- synthetic batch, resident in HBM before timing (distinct data per rank)
    data = synth.log_text(nb * block, synth.SEED_BASE + 1 + 1000 * rank)
    offs = [i * block for i in range(nb)]
    d_src = eng.upload(data)
    plan = eng.plan_encode(offs, [block] * nb)
    d_frames = eng.alloc(plan.dst_bound)
    d_ioff, d_ilen = eng.alloc(8 * nb), eng.alloc(4 * nb)
    d_out = eng.alloc(nb * block)
    d_olen, d_ost = eng.alloc(4 * nb), eng.alloc(4 * nb)

    # frame offsets are deterministic for a given input: learn them once for the decode plan
    eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
    eng.sync()
    fo, fl = d_ioff.u64(nb), d_ilen.u32(nb)
    dplan = eng.plan_decode(fo, fl, offs, [block] * nb)
    comp_bytes = fo[-1] + fl[-1]

    def step():
        eng.encode_dev(plan, d_src, d_frames, d_ioff, d_ilen)
        eng.decode_dev(dplan, d_frames, d_out, d_olen, d_ost)

    for _ in range(args.warmup):
        step()
    eng.sync()
    # correctness gate on the warmed-up state (outside the timed region)
    if not args.skip_check:
        st = d_ost.i32(nb)
        assert st == [0] * nb, f"decode status {set(st)}"
        assert d_out.read(2 * block) == data[: 2 * block]

    eng.timing_reset()
    eng.set_timing(True)
    g.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    t1 = time.perf_counter()
    g.barrier()
    eng.set_timing(False)
    elapsed = g.max(t1 - t0)
    kt = eng.timing()

    # full-output check after the timed steps
    if not args.skip_check:
        assert d_ost.i32(nb) == [0] * nb
        assert d_out.read() == data, "decoded batch differs from the input"

    total_u = g.sum(float(nb * block)) * args.steps
    value = total_u / elapsed / GiB

    # ---- roofline for the dominant kernel
    # side-stream spans overlap the match finder, so they never count as the dominant kernel
    excl = {k: v for k, v in kt.items() if not k.endswith("_side")}
    dom = max(excl, key=lambda k: excl[k][0]) if excl else None
    roof = None
    if dom:
        ms, n = kt[dom]
        per_launch_s = ms / n / 1e3
        # algorithmic bytes per launch: each kernel's own reads + writes
        alg = {
            "enc_parse": nb * block,                  # U read once (match finding)
            "enc_emit": nb * block + comp_bytes,      # U literals read + C framed bytes written
            "decode": comp_bytes + nb * block,        # C read + U written
            "xxh32": nb * block,                      # U read (decode-side verify; encode side runs on the side stream)
        }.get(dom, nb * block)
        achieved = alg / per_launch_s / 1e9
        traffic, tsrc = pmc_traffic(dom)
        roof = {
            "bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ms / n, 4),
        }
        if tsrc:
            roof["traffic_source"] = tsrc + " (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, same bench command)"
    per_kernel = {k: round(v[0] / args.steps, 4) for k, v in kt.items()}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(data, block, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.total_blocks else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic S3 access-log text (SURVEY.md §8d config 2), seeded, distinct per rank",
            "config": {
                "workload": (f"config5: {args.total_blocks} x 64 KiB log-text blocks split over {world} GPUs" if args.total_blocks
                             else f"config2: {nb} x 64 KiB log-text blocks per GPU") + ", LZ4 frame encode + decode, device-resident",
                "blocks_per_gpu": nb, "block_bytes": block, "frame": "FLG 0x64 BD 0x40 (lz4_flex Auto), xxh32 content checksum",
                "compression_ratio": round(comp_bytes / (nb * block), 4), "parallelism": f"shard{world}",
            },
            "kernel_ms_per_step": per_kernel,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    g.close()


if __name__ == "__main__":
    main()
