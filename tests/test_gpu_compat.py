"""GPU tests of the lz4_flex-compatible encoder (S3HC_BLK_LZ4FLEX_COMPAT).

Bar: frames byte-identical to the oracle's restatement of lz4_flex's FrameEncoder + greedy
block compressor (oracle/lz4_oracle.c:173-279, or_lz4flex_compress_frame) on the same input,
and decodable by the GPU decoder and the oracle decoder back to the input. The restatement is
recalled, not checked against lz4_flex source: compressed-byte parity with the
crate itself is "parity unpinned"; parity with the restatement is bit-exact here.
Edge cases: empty, below LZ4_MIN_LENGTH, the reference's i % 251 fixtures
(tests/lz4_roundtrip_preservation_test.rs:192-196), incompressible blocks (stored), zero runs
(overlapping offset-1 matches, 255-run length bytes), hash-colliding text, every BlockSize::Auto
layout (BD 0x40 / 0x50 / 0x70) and a multi-block 4 MiB frame (table carried across blocks).
"""
import numpy as np
import pytest

import s3hc_lz4 as S
import synth

pytestmark = pytest.mark.gpu

KiB, MiB = 1 << 10, 1 << 20


def pattern251(n):
    return bytes(i % 251 for i in range(n))


def rnd(n, seed=7):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def small_alphabet(n, seed=3):  # dense in-batch hash collisions, short matches
    return np.random.default_rng(seed).integers(97, 101, n, dtype=np.uint8).tobytes()


CASES = {
    "empty": lambda: b"",
    "1": lambda: b"x",
    "12": lambda: b"0123456789ab",
    "13": lambda: b"0123456789abc",
    "p251_63": lambda: pattern251(63),
    "p251_64": lambda: pattern251(64),
    "p251_1024": lambda: pattern251(1024),
    "p251_64k": lambda: pattern251(65536),
    "log_64k": lambda: synth.log_text(65536),
    "json_64k": lambda: synth.json_records(65536),
    "jpeg_64k": lambda: synth.jpeg_like(65536),
    "random_64k": lambda: rnd(65536),
    "zeros_64k": lambda: bytes(65536),
    "alpha4_64k": lambda: small_alphabet(65536),
    "log_64k+1": lambda: synth.log_text(65537, 11),
    "log_256k": lambda: synth.log_text(256 * KiB, 12),
    "log_1MiB": lambda: synth.log_text(MiB, 13),
    "random_small_then_text": lambda: rnd(3000, 9) + synth.log_text(20000, 14),
}


@pytest.mark.parametrize("name", list(CASES))
def test_compat_frame_matches_oracle(engine, oracle, name):
    data = CASES[name]()
    want = oracle.lz4flex_compress_frame(data)
    got = engine.compress_frame(data, S.BLK_LZ4FLEX_COMPAT)
    assert got == want, f"{name}: {len(got)} vs {len(want)} bytes, first diff at " + str(
        next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), min(len(got), len(want))))
    assert engine.decompress_frames(got) == data
    assert oracle.decompress_data(got) == data


def test_compat_multiblock_frame(engine, oracle):
    # 4 MiB + 100 KiB: BD 0x70, two blocks, the second compressed with stream_off = 4 MiB
    data = synth.log_text(4 * MiB + 100 * KiB, 21)
    got = engine.compress_frame(data, S.BLK_LZ4FLEX_COMPAT)
    assert got == oracle.lz4flex_compress_frame(data)
    assert engine.decompress_frames(got) == data


def test_compat_batch_dev(engine, oracle):
    # a config-3-like mixed batch of 64 KiB items plus ragged ones, through the device API
    parts = [synth.log_text(65536, 30 + i) if i % 3 == 0 else
             synth.json_records(65536, 40 + i) if i % 3 == 1 else synth.jpeg_like(65536, 50 + i)
             for i in range(48)]
    parts += [pattern251(1000), b"", rnd(70000, 5), bytes(5000), synth.log_text(300 * KiB, 60)]
    data = b"".join(parts)
    src_off, o = [], 0
    for p in parts:
        src_off.append(o)
        o += len(p)
    lens = [len(p) for p in parts]
    d_src = engine.upload(data)
    slots = engine.compat_dst_offsets(lens)
    d_dst = engine.alloc(slots[-1])
    d_len = engine.alloc(4 * len(parts))
    dst_off = engine.compat_encode_dev(src_off, lens, d_src, d_dst, d_len)
    engine.sync()
    flen = d_len.u32(len(parts))
    raw = d_dst.read()
    for i, p in enumerate(parts):
        frame = raw[dst_off[i]: dst_off[i] + flen[i]]
        assert frame == oracle.lz4flex_compress_frame(p), f"item {i}"
    # the batch decodes on the GPU decoder too
    plan = engine.plan_decode(dst_off, flen, src_off, [max(n, 1) for n in lens])
    out = engine.alloc(len(data) + 16)
    olen, ost = engine.alloc(4 * len(parts)), engine.alloc(4 * len(parts))
    engine.decode_dev(plan, d_dst, out, olen, ost)
    engine.sync()
    assert ost.i32(len(parts)) == [0] * len(parts)
    assert olen.u32(len(parts)) == lens
    assert out.read(len(data)) == data


def test_compat_rejects_short_slots(engine):
    d_src = engine.upload(bytes(1000))
    d_dst = engine.alloc(4096)
    d_len = engine.alloc(8)
    with pytest.raises(S.CodecError) as e:
        engine.compat_encode_dev([0, 500], [500, 500], d_src, d_dst, d_len, dst_off=[0, 100])
    assert e.value.status == 6  # S3HC_INVALID_ARG


@pytest.mark.parametrize("n", [4 * MiB, 4 * MiB + 1, 256 * KiB + 1])
def test_compat_block_boundaries(engine, oracle, n):
    # exactly one Max4MB block, a second block of 1 byte, and the smallest BD 0x70 frame
    data = synth.log_text(n, 23)
    got = engine.compress_frame(data, S.BLK_LZ4FLEX_COMPAT)
    assert got == oracle.lz4flex_compress_frame(data)
    assert engine.decompress_frames(got) == data


def test_compat_random_batch(engine, oracle):
    # 300 seeded items of 0..6000 bytes mixing runs, text, random bytes and repeats (one launch)
    rng = np.random.default_rng(2024)
    parts = []
    for i in range(300):
        n = int(rng.integers(0, 6000))
        kind = i % 5
        if kind == 0:
            b = rnd(n, 100 + i)
        elif kind == 1:
            b = synth.log_text(n, 200 + i) if n else b""
        elif kind == 2:
            b = bytes(rng.integers(0, 3, n, dtype=np.uint8) * 85)
        elif kind == 3:
            unit = rnd(int(rng.integers(1, 40)), 300 + i)
            b = (unit * (n // max(len(unit), 1) + 1))[:n]
        else:
            b = small_alphabet(n, 400 + i)
        parts.append(b)
    data = b"".join(parts)
    src_off, o = [], 0
    for p in parts:
        src_off.append(o)
        o += len(p)
    lens = [len(p) for p in parts]
    d_src = engine.upload(data + b"\0" * 16)
    slots = engine.compat_dst_offsets(lens)
    d_dst, d_len = engine.alloc(slots[-1]), engine.alloc(4 * len(parts))
    dst_off = engine.compat_encode_dev(src_off, lens, d_src, d_dst, d_len)
    engine.sync()
    flen = d_len.u32(len(parts))
    raw = d_dst.read()
    bad = [i for i, p in enumerate(parts) if raw[dst_off[i]: dst_off[i] + flen[i]] != oracle.lz4flex_compress_frame(p)]
    assert not bad, f"items differing from the oracle: {bad[:10]}"
