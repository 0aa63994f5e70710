"""BASELINE.json configs at their stated sizes, on the GPU, every byte checked.

config 2: 4096 x 64 KiB distinct log-text blocks — every GPU frame decodes with the oracle
          (the CPU restatement of decompress_data, compression.rs:463-502), and the GPU batch
          decode returns the input.
config 3: 65,536 x 64 KiB (4 GiB), JSON / JPEG-like alternating; every block's mode comes from
          effective_compression (cache.rs:1158-1178) on a ':range:'-suffixed cache key, so the
          JPEG half becomes store-mode frames (compression.rs:326-368, byte-exact vs the oracle)
          and the JSON half LZ4 frames; the whole batch decodes back bit-exactly.
config 4: one 8 GiB object of 64 KiB frames, and a 2 GiB object of the reference's own 1 MiB
          frames (what flush_batch writes, disk_cache.rs:1820-1870), through the range reader
          (stream_range_data, disk_cache.rs:3850-3935) in 256 KiB batches on 3 queues, 4 MiB
          file reads, 1 MiB chunks out; output equal to the input, total checked.
config 5: one GPU's 131,072-block slice of the 1 M x 64 KiB batch (8 GiB), encode + decode,
          every byte checked, a spread sample of frames through the oracle.
"""
import numpy as np
import pytest

import s3hc_lz4 as S
import synth

pytestmark = pytest.mark.gpu
MiB = 1 << 20
BLOCK = 65536


def _encode_items(engine, d_src, n_items, item, modes=None):
    offs = [i * item for i in range(n_items)]
    plan = engine.plan_encode(offs, [item] * n_items, modes)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n_items), engine.alloc(4 * n_items)
    engine.encode_dev(plan, d_src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(n_items), ilen.u32(n_items)
    return dst, fo, fl


def _decode_all(engine, dst, fo, fl, n, item):
    offs = [i * item for i in range(n)]
    dplan = engine.plan_decode(fo, fl, offs, [item] * n)
    out = engine.alloc(n * item)
    olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
    ost.fill(0xFF)
    engine.decode_dev(dplan, dst, out, olen, ost)
    engine.sync()
    assert ost.i32(n) == [0] * n
    assert olen.u32(n) == [item] * n
    return out


@pytest.mark.timeout(900)
def test_config2_full_batch_every_frame_oracle(engine, oracle):
    n = 4096
    data = synth.log_text(n * BLOCK, synth.SEED_BASE + 1)
    d_src = engine.upload(data)
    dst, fo, fl = _encode_items(engine, d_src, n, BLOCK)
    frames = dst.read(fo[-1] + fl[-1])
    mv = memoryview(data)
    for i in range(n):
        f = frames[fo[i]:fo[i] + fl[i]]
        assert f[:7] == b"\x04\x22\x4d\x18\x64\x40\xa7"
        assert oracle.decompress_data(f) == mv[i * BLOCK:(i + 1) * BLOCK], f"frame {i}"
    out = _decode_all(engine, dst, fo, fl, n, BLOCK)
    assert out.read() == data
    assert (fo[-1] + fl[-1]) / len(data) < 0.45


@pytest.mark.timeout(900)
def test_config3_full_size_routed_by_cache_key(engine, oracle):
    n = 65536
    data, kinds = synth.mixed_blocks(n, BLOCK)
    keys = [f"media-assets/obj-{i:05d}{'.json' if k == 0 else '.jpg'}:range:{i * BLOCK}-{i * BLOCK + BLOCK - 1}"
            for i, k in enumerate(kinds)]
    modes = [0 if S.effective_compression(S.ResolvedSettings(), 1024, key, BLOCK) else 1 for key in keys]
    assert modes == kinds
    d_src = engine.upload(data)
    dst, fo, fl = _encode_items(engine, d_src, n, BLOCK, modes)
    mv = memoryview(data)
    # a spread sample of frames against the oracle: store-mode byte-exact, LZ4 frames decode
    for i in list(range(0, n, 509)) + [n - 2, n - 1]:
        f = dst.read(fl[i], fo[i])
        blk = mv[i * BLOCK:(i + 1) * BLOCK]
        if modes[i]:
            assert f == oracle.store_mode_frame(blk), f"store-mode frame {i}"
        else:
            assert oracle.decompress_data(f) == blk, f"frame {i}"
    sizes = np.array(fl, dtype=np.int64)
    assert (sizes[1::2] == BLOCK + 19).all()      # every JPEG block: one stored block + 19 B of frame
    assert sizes[0::2].mean() < 0.45 * BLOCK
    out = _decode_all(engine, dst, fo, fl, n, BLOCK)
    for c in range(0, n * BLOCK, 256 * MiB):
        assert out.read(256 * MiB, c) == mv[c:c + 256 * MiB], f"decoded bytes differ in [{c}, +256 MiB)"


def _reader_roundtrip(engine, frames, data, batch, depth=3, piece=4 * MiB):
    r = S.RangeReader(engine, batch, depth)
    mv = memoryview(data)
    got = 0

    def drain():
        nonlocal got
        while True:
            c = r.read(MiB)
            if not c:
                return
            assert c == mv[got:got + len(c)], f"reader output differs at {got}"
            got += len(c)

    fmv = memoryview(frames)
    for i in range(0, len(frames), piece):
        r.feed(fmv[i:i + piece])
        drain()
    r.finish()
    drain()
    assert got == len(data) and r.total == len(data)
    r.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("item,size", [(BLOCK, 8 << 30), (MiB, 2 << 30)], ids=["64KiB_frames_8GiB", "ref_1MiB_frames_2GiB"])
def test_config4_object_through_reader_256k_batches(engine, item, size):
    n = size // item
    d_src = engine.alloc(size)
    for c in range(0, size, 256 * MiB):
        d_src.write(synth.log_text(256 * MiB, 4000 + c // (256 * MiB)), c)
    data = d_src.read()
    dst, fo, fl = _encode_items(engine, d_src, n, item)
    del d_src
    frames = dst.read(fo[-1] + fl[-1])
    del dst
    if item == MiB:
        assert frames[4:7] == b"\x64\x70\xb9"  # BD 0x70: lz4_flex Auto for a 1 MiB batch
    _reader_roundtrip(engine, frames, data, 256 << 10)


@pytest.mark.timeout(900)
def test_config5_per_gpu_slice_131072_blocks(engine, oracle):
    # config 5 (1 M x 64 KiB over 8 GPUs, no RCCL) gives each GPU a contiguous 131,072-block
    # slice (8 GiB); this is one GPU's slice at full size: encode + decode in one batch each,
    # every status and length checked, every decoded byte compared chunk by chunk, and a spread
    # sample of frames decoded by the oracle (decompress_data, compression.rs:463-502).
    n = 131072
    chunk_blocks = 4096  # 256 MiB of distinct log text per chunk, regenerated for the checks
    seeds = [synth.SEED_BASE + 5 + 7919 * c for c in range(n // chunk_blocks)]
    d_src = engine.alloc(n * BLOCK)
    for c, sd in enumerate(seeds):
        d_src.write(synth.log_text(chunk_blocks * BLOCK, sd), c * chunk_blocks * BLOCK)
    dst, fo, fl = _encode_items(engine, d_src, n, BLOCK)
    del d_src
    assert (fo[-1] + fl[-1]) / (n * BLOCK) < 0.45
    out = _decode_all(engine, dst, fo, fl, n, BLOCK)
    sample = set(list(range(0, n, 997)) + [n - 1])
    for c, sd in enumerate(seeds):
        want = synth.log_text(chunk_blocks * BLOCK, sd)
        got = out.read(chunk_blocks * BLOCK, c * chunk_blocks * BLOCK)
        assert got == want, f"decoded bytes differ in chunk {c}"
        mv = memoryview(want)
        for i in range(c * chunk_blocks, (c + 1) * chunk_blocks):
            if i in sample:
                k = i - c * chunk_blocks
                f = dst.read(fl[i], fo[i])
                assert f[:7] == b"\x04\x22\x4d\x18\x64\x40\xa7"
                assert oracle.decompress_data(f) == mv[k * BLOCK:(k + 1) * BLOCK], f"frame {i}"
