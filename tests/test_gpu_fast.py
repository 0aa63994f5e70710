"""64 KiB-block decode fast path (csrc/s3hc_fast.hip).

k_dtok indexes each block's tokens (speculative segment walks merged by pointer doubling) and
validates every lz4_flex bound; k_dexec executes 64 sequences at a time. Blocks it does not take
(stored, > 32 KiB compressed, multi-block units, malformed or out of bounds) go to the per-unit
decoder. Bar: decoded bytes and statuses identical to the oracle (decompress_data,
compression.rs:463-502) and to the per-unit decoder alone (S3HC_FAST_DISABLE=1) on every input,
and the path actually taken on well-formed 64 KiB frames (S3HC_FAST_TRACE counts).
"""
import os
import random
import re

import numpy as np
import pytest

import lz4ref
import synth

pytestmark = pytest.mark.gpu
BLOCK = 65536


def _with_env(env, fn):
    # library knobs (s3hc_set_knob): the library reads the environment only once per process
    import s3hc_lz4 as S

    with S.knobs(env):
        return fn()


def _slow(fn):  # the per-unit decoder alone
    return _with_env({"S3HC_FAST_DISABLE": "1", "S3HC_LB_DISABLE": "1"}, fn)


def _fast(fn):  # host calls of few blocks otherwise take the large-block path
    return _with_env({"S3HC_LB_DISABLE": "1"}, fn)


@pytest.fixture(autouse=True)
def _fast_path_on():
    # every test here runs with the fast path enabled (the library default; a stray S3HC_FAST=0
    # in the environment must not turn these tests into per-unit-decoder tests)
    import s3hc_lz4 as S

    with S.knobs({"S3HC_FAST": "1", "S3HC_FAST_DISABLE": None}):
        yield


def _period(k, n):
    base = bytes((i * 37 + 11) & 0xFF for i in range(k))
    return (base * (n // k + 1))[:n]


def _text_with_random_runs(n, seed, run):
    # literal runs far longer than a 2 KiB executor batch
    rng = np.random.default_rng(seed)
    t = bytearray(synth.log_text(n, seed))
    for p in range(1000, n - run, 7 * run):
        t[p:p + run] = rng.integers(0, 256, run, dtype=np.uint8).tobytes()
    return bytes(t)


def _inputs():
    rng = random.Random(777)
    runs = b"".join(bytes([rng.randrange(256)]) * rng.choice([1, 2, 5, 17, 40, 300, 3000]) for _ in range(3000))
    d = {
        "log": synth.log_text(BLOCK, 51),
        "json": synth.json_records(BLOCK, 52),
        "zeros": bytes(BLOCK),
        "runs": runs[:BLOCK],
        "small_1000": synth.log_text(1000, 53),
        "lit_runs_2500": _text_with_random_runs(BLOCK, 54, 2500),
        "lit_runs_300": _text_with_random_runs(BLOCK, 55, 300),
        "half_random": synth.log_text(BLOCK // 2, 56) + rng.randbytes(BLOCK // 2),  # C near 32 KiB
        "p251": bytes(i % 251 for i in range(BLOCK)),
    }
    for k in (1, 2, 3, 4, 5, 7, 8, 12, 15, 16, 17, 31, 64, 1000):
        d[f"period_{k}"] = _period(k, BLOCK - k)
        d[f"period_{k}_full"] = _period(k, BLOCK)
    d["abc"] = (b"abc" * 30000)[:BLOCK]
    d["zeros_then_text"] = bytes(40000) + synth.log_text(BLOCK - 40000, 80)
    for n in (1, 2, 3, 4, 5, 11, 12, 13, 14, 15, 16, 17, 20, 31, 64, 100):
        d[f"tiny_{n}"] = synth.log_text(n, 60 + n)
    return d


def test_fast_path_decodes_every_input(engine, oracle):
    for name, data in _inputs().items():
        for f in (engine.compress_frame(data), oracle.lz4flex_compress_frame(data),
                  lz4ref.compress_frame(data, block_size_id=4, linked=False),
                  lz4ref.compress_frame(data, block_size_id=4, linked=True)):
            assert oracle.decompress_data(f) == data, name
            assert _fast(lambda: engine.decompress_frames(f)) == data, name
            assert _slow(lambda: engine.decompress_frames(f)) == data, name
            assert engine.decompress_frames(f) == data, name


def _encode_batch(engine, data, n, item):
    d_src = engine.upload(data)
    offs = [i * item for i in range(n)]
    plan = engine.plan_encode(offs, [item] * n)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n), engine.alloc(4 * n)
    engine.encode_dev(plan, d_src, dst, ioff, ilen)
    engine.sync()
    return dst, ioff.u64(n), ilen.u32(n)


def _decode_batch(engine, dst, fo, fl, offs, caps):
    n = len(fo)
    dplan = engine.plan_decode(fo, fl, offs, caps)
    out = engine.alloc(max(1, offs[-1] + caps[-1]))
    olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
    ost.fill(0xFF)
    engine.decode_dev(dplan, dst, out, olen, ost)
    engine.sync()
    return out, olen.u32(n), ost.i32(n)


def test_fast_path_taken_on_a_batch(engine, capfd):
    n = 512
    data = synth.log_text(n * BLOCK, 57)
    dst, fo, fl = _encode_batch(engine, data, n, BLOCK)
    offs = [i * BLOCK for i in range(n)]
    capfd.readouterr()
    out, olen, ost = _with_env({"S3HC_FAST_TRACE": "1"},
                               lambda: _decode_batch(engine, dst, fo, fl, offs, [BLOCK] * n))
    err = capfd.readouterr().err
    m = re.search(r"\[s3hc fast\] units (\d+) taken (\d+) tokens (\d+)", err)
    assert m, err
    assert int(m.group(2)) == n  # every frame's block
    assert ost == [0] * n and olen == [BLOCK] * n
    assert out.read(n * BLOCK) == data
    out2, olen2, ost2 = _slow(lambda: _decode_batch(engine, dst, fo, fl, offs, [BLOCK] * n))
    assert ost2 == ost and olen2 == olen and out2.read(n * BLOCK) == data


def test_fast_path_mixed_batch(engine, oracle):
    # one launch: fast blocks beside stored blocks, linked multi-block frames, large blocks,
    # blocks above 32 KiB compressed, tiny blocks and empty frames; unequal caps and offsets
    rng = random.Random(58)
    items = []
    for k in range(200):
        kind = k % 8
        if kind == 0:
            d = synth.log_text(BLOCK, 100 + k)
            f = engine.compress_frame(d)
        elif kind == 1:
            d = rng.randbytes(BLOCK)
            f = engine.compress_frame(d)  # stored block
        elif kind == 2:
            d = synth.log_text(3 * BLOCK + 17, 100 + k)
            f = lz4ref.compress_frame(d, block_size_id=4, linked=True)
        elif kind == 3:
            d = synth.log_text(300_000, 100 + k)
            f = oracle.lz4flex_compress_frame(d)  # BD 0x70 block
        elif kind == 4:
            d = synth.log_text(BLOCK // 2, 100 + k) + rng.randbytes(BLOCK // 2)
            f = oracle.lz4flex_compress_frame(d)
        elif kind == 5:
            d = synth.log_text(rng.randrange(1, 200), 100 + k)
            f = oracle.lz4flex_compress_frame(d)
        elif kind == 6:
            d = b""
            f = oracle.lz4flex_compress_frame(d)
        else:
            d = _period(rng.randrange(1, 40), rng.randrange(1000, BLOCK))
            f = engine.compress_frame(d)
        items.append((f, d))
    blob = b"".join(f for f, _ in items)
    fo, fl, offs, caps = [], [], [], []
    p = o = 0
    for f, d in items:
        fo.append(p)
        fl.append(len(f))
        offs.append(o)
        caps.append(max(len(d), 1) + 13)
        p += len(f)
        o += caps[-1] + 5
    d_blob = engine.upload(blob)
    out, olen, ost = _decode_batch(engine, d_blob, fo, fl, offs, caps)
    out2, olen2, ost2 = _slow(lambda: _decode_batch(engine, d_blob, fo, fl, offs, caps))
    assert ost == ost2 and olen == olen2
    for i, (f, d) in enumerate(items):
        assert ost[i] == 0 and olen[i] == len(d), i
        assert out.read(len(d), offs[i]) == d, i
        assert out2.read(len(d), offs[i]) == d, i


def test_fast_path_dst_too_small_on_device_plans(engine, oracle):
    n = 64
    data = synth.log_text(n * BLOCK, 59)
    dst, fo, fl = _encode_batch(engine, data, n, BLOCK)
    caps = [BLOCK - (i % 5) * 1000 for i in range(n)]  # every fifth frame fits
    offs = [i * BLOCK for i in range(n)]
    out, olen, ost = _fast(lambda: _decode_batch(engine, dst, fo, fl, offs, caps))  # (64 frames: LB otherwise)
    out2, olen2, ost2 = _slow(lambda: _decode_batch(engine, dst, fo, fl, offs, caps))
    assert ost == ost2 and olen == olen2
    for i in range(n):
        if caps[i] == BLOCK:
            assert ost[i] == 0 and out.read(BLOCK, i * BLOCK) == data[i * BLOCK:(i + 1) * BLOCK]
        else:
            assert ost[i] != 0


def test_fast_path_corruption_matches_oracle(engine, oracle):
    import s3hc_lz4 as S

    rng = random.Random(61)
    base = [engine.compress_frame(synth.log_text(BLOCK, 70 + k)) for k in range(3)]
    base += [oracle.lz4flex_compress_frame(synth.json_records(BLOCK, 75))]
    base += [engine.compress_frame(_period(3, BLOCK - 3))]
    for trial in range(200):
        f = bytearray(rng.choice(base))
        mode = trial % 4
        if mode == 0:  # bit flips in the block payload
            for _ in range(rng.randrange(1, 4)):
                q = rng.randrange(11, len(f) - 8)
                f[q] ^= 1 << rng.randrange(8)
        elif mode == 1:  # a zeroed offset somewhere
            q = rng.randrange(11, len(f) - 10)
            f[q:q + 2] = b"\x00\x00"
        elif mode == 2:  # a random byte run
            q = rng.randrange(11, len(f) - 40)
            f[q:q + 16] = rng.randbytes(16)
        else:  # block shortened (its size word kept: the walk sees a truncated frame)
            f = f[:rng.randrange(12, len(f))]
        f = bytes(f)
        want_st, want = oracle.decompress_status(f)

        def dec():
            try:
                return 0, engine.decompress_frames(f)
            except S.CodecError as e:
                return e.status, b""

        st, out = _fast(dec)
        st2, out2 = _slow(dec)
        assert st == st2 == want_st, (trial, mode)
        if want_st == 0:
            assert out == out2 == want


def test_fast_path_device_batch_corruption(engine, oracle):
    # corrupted frames inside a device batch: each frame's status equals the oracle's
    rng = random.Random(62)
    frames, datas = [], []
    for k in range(128):
        d = synth.log_text(BLOCK, 200 + k)
        f = bytearray(engine.compress_frame(d))
        if k % 3 == 0:
            q = rng.randrange(11, len(f) - 8)
            f[q] ^= 1 << rng.randrange(8)
        frames.append(bytes(f))
        datas.append(d)
    blob = b"".join(frames)
    fo, p = [], 0
    for f in frames:
        fo.append(p)
        p += len(f)
    fl = [len(f) for f in frames]
    offs = [i * BLOCK for i in range(len(frames))]
    d_blob = engine.upload(blob)
    out, olen, ost = _decode_batch(engine, d_blob, fo, fl, offs, [BLOCK] * len(frames))
    out2, olen2, ost2 = _slow(lambda: _decode_batch(engine, d_blob, fo, fl, offs, [BLOCK] * len(frames)))
    assert ost == ost2 and olen == olen2
    for i, f in enumerate(frames):
        want_st, want = oracle.decompress_status(f)
        assert ost[i] == want_st, i
        if want_st == 0:
            assert out.read(BLOCK, i * BLOCK) == want


def _raw_frame(block: bytes, out: bytes) -> bytes:
    # one independent BD 0x40 block, content checksum (lz4_flex's frame layout, compression.rs:539-557)
    import xxhash

    hdr = bytes([0x64, 0x40])
    hc = (xxhash.xxh32(hdr, seed=0).intdigest() >> 8) & 0xFF
    return (b"\x04\x22\x4d\x18" + hdr + bytes([hc]) + len(block).to_bytes(4, "little") + block +
            b"\x00\x00\x00\x00" + xxhash.xxh32(out, seed=0).intdigest().to_bytes(4, "little"))


def _densest_block(c_target: int, lit: int = 5):
    # as many sequences as a block of c_target bytes can hold: after one literal, every sequence is
    # a bare token + offset 1 (3 bytes, 4 output bytes), then a literal-only last sequence
    n = (c_target - 2 - 1 - (1 + lit)) // 3
    blk = bytearray(b"\x10a")  # token: 1 literal, match 4; literal 'a'
    blk += b"\x01\x00"         # offset 1
    blk += b"\x00\x01\x00" * n
    blk += bytes([lit << 4]) + b"b" * lit
    out = b"a" * (1 + 4 * (n + 1)) + b"b" * lit
    return bytes(blk), out, n + 2


def test_fast_path_densest_token_blocks(engine, oracle):
    # the token-position list at its bound (kFastMaxTok: N <= (C - 1) / 3 + 1 for C <= 32 KiB),
    # through the fast path and the per-unit decoder, single calls and one batch
    items = []
    for c in (32768, 32767, 32766, 32000, 4096, 100, 12):
        blk, out, ntok = _densest_block(c)
        assert len(blk) <= 32768 and ntok <= (len(blk) - 1) // 3 + 1
        f = _raw_frame(blk, out)
        assert oracle.decompress_data(f) == out
        assert _fast(lambda: engine.decompress_frames(f)) == out
        assert _slow(lambda: engine.decompress_frames(f)) == out
        items.append((f, out))
    blob = b"".join(f for f, _ in items)
    fo, fl, offs, caps = [], [], [], []
    p = o = 0
    for f, d in items:
        fo.append(p)
        fl.append(len(f))
        offs.append(o)
        caps.append(BLOCK)
        p += len(f)
        o += BLOCK
    d_blob = engine.upload(blob)
    out, olen, ost = _decode_batch(engine, d_blob, fo, fl, offs, caps)
    for i, (f, d) in enumerate(items):
        assert ost[i] == 0 and olen[i] == len(d), i
        assert out.read(len(d), offs[i]) == d, i


def test_device_plan_multiblock_frames_keep_their_parallelism(engine, capfd):
    # more than 64 frames (past the all-blocks-to-LB threshold) made of independent
    # 64 KiB blocks (liblz4 BD 0x40, 16 blocks per 1 MiB frame). The device plan's grid is one
    # workgroup per 64 KiB of frame room (1280 here, not one per frame), every block takes the
    # fast path, and the token slots (per frame, sized by compressed bytes) stay disjoint even
    # when two plan entries name the same frame.
    if not lz4ref.available:
        pytest.skip("liblz4 absent")
    n, MiB = 80, 1 << 20
    data = synth.log_text(n * MiB, 91)
    frames = [lz4ref.compress_frame(data[i * MiB:(i + 1) * MiB], block_size_id=4, linked=False) for i in range(n)]
    blob = b"".join(frames)
    fo = [sum(len(f) for f in frames[:i]) for i in range(n)]
    fl = [len(f) for f in frames]
    fo.append(fo[3])  # a duplicate entry: frame 3 decoded a second time into its own slot
    fl.append(fl[3])
    offs = [i * MiB for i in range(n + 1)]
    src = engine.upload(blob)
    capfd.readouterr()
    out, olen, ost = _with_env({"S3HC_FAST_TRACE": "1"},
                               lambda: _decode_batch(engine, src, fo, fl, offs, [MiB] * (n + 1)))
    err = capfd.readouterr().err
    m = re.search(r"\[s3hc fast\] units (\d+) taken (\d+) tokens (\d+) grid (\d+)", err)
    assert m, err
    assert int(m.group(2)) == 16 * (n + 1) and int(m.group(4)) == 16 * (n + 1), err
    assert ost == [0] * (n + 1) and olen == [MiB] * (n + 1)
    got = out.read((n + 1) * MiB)
    assert got[:n * MiB] == data and got[n * MiB:] == data[3 * MiB:4 * MiB]


def _chained_copies(n, seed):
    # text made of copies of recent copies (chains of in-window matches whose sources lie inside
    # earlier matches: k_dexec's sequence-level source redirection, round 6), copies from far
    # back (sources older than the 8 KiB ring, read from HBM) and short literal runs
    rng = random.Random(seed)
    out = bytearray(rng.randbytes(64))
    while len(out) < n:
        r = rng.random()
        if r < 0.55:
            L = rng.randint(4, 14)
            d = rng.randint(L, min(len(out), 300))
            s = len(out) - d
            out += out[s:s + L]
        elif r < 0.75 and len(out) > 9000:
            L = rng.randint(5, 40)
            s = rng.randint(0, len(out) - 8500 - L)
            out += out[s:s + L]
        else:
            out += rng.randbytes(rng.randint(1, 6))
    return bytes(out[:n])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fast_path_chained_in_window_copies(engine, oracle, seed):
    # every frame writer, one block and a 64-block device batch: the output must be the input
    import s3hc_lz4 as S

    data = _chained_copies(BLOCK, seed)
    for f in (engine.compress_frame(data), oracle.lz4flex_compress_frame(data),
              lz4ref.compress_frame(data, block_size_id=4, linked=False)):
        assert oracle.decompress_data(f) == data
        assert _fast(lambda: engine.decompress_frames(f)) == data
    big = b"".join(_chained_copies(BLOCK, 100 * seed + k) for k in range(300))
    fr = [oracle.lz4flex_compress_frame(big[i:i + BLOCK]) for i in range(0, len(big), BLOCK)]
    offs, lens, pos = [], [], 0
    for f in fr:
        offs.append(pos)
        lens.append(len(f))
        pos += len(f)
    src = engine.upload(b"".join(fr))
    n = len(fr)
    plan = engine.plan_decode(offs, lens, [i * BLOCK for i in range(n)], [BLOCK] * n)
    out = engine.alloc(n * BLOCK)
    olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
    engine.decode_dev(plan, src, out, olen, ost)
    engine.sync()
    assert ost.i32(n) == [0] * n
    assert out.read(len(big)) == big
