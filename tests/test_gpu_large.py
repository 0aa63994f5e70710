"""Large-block decode path (csrc/s3hc_lb.hip).

Frames that allow blocks above 64 KiB (BD 0x50 / 0x70) are what the reference writes for its
own cache files (flush_batch compresses ~1 MiB batches with lz4_flex BlockSize::Auto,
disk_cache.rs:1820-1870); their blocks are decoded by many workgroups each. Bar: decoded bytes
bit-exact with the oracle, statuses identical to the oracle's on corrupt inputs, and identical
to the one-wave decoder (S3HC_LB_DISABLE=1) on every input. Few-block launches run the spread
execution (k_lbw_*: all tiles of a block at once, global pointer jumping); S3HC_LBW_DISABLE=1 sends
the same blocks through the step loop (k_lb_run), and S3HC_LBW_CAP splits one launch between both.
"""
import os
import random

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _deep_chain(n, seed):
    # every line is a recent line with one edit: matches of matches of matches (long source chains)
    rng = random.Random(seed)
    lines = [b"GET /bucket/object-%06d status=200 bytes=%d\n" % (i, i * 7) for i in range(8)]
    out = bytearray()
    while len(out) < n:
        base = bytearray(lines[-rng.randrange(1, 8)])
        base[rng.randrange(len(base) - 1)] = 0x41 + rng.randrange(26)
        lines.append(bytes(base))
        out += base
    return bytes(out[:n])


def _runs(n, seed):
    rng = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        out += bytes([rng.randrange(256)]) * rng.choice([1, 3, 17, 300, 5000, 70000])
    return bytes(out[:n])


INPUTS = {
    "log_100k": lambda: synth.log_text(100_000, 1),      # BD 0x50, one 100 KB block
    "log_256k": lambda: synth.log_text(256 * 1024, 2),   # BD 0x50, exactly one full block
    "log_1MiB": lambda: synth.log_text(MiB, 3),          # BD 0x70, one 1 MiB block (reference cache frame)
    "log_5MiB+3": lambda: synth.log_text(5 * MiB + 3, 4),  # two blocks: 4 MiB + 1 MiB
    "json_1MiB": lambda: synth.json_records(MiB, 5),
    "zeros_4MiB": lambda: bytes(4 * MiB),                # long 255 length runs
    "zeros_1MiB+7": lambda: bytes(MiB + 7),
    "p251_1MiB+1": lambda: bytes(i % 251 for i in range(MiB + 1)),
    "runs_2MiB": lambda: _runs(2 * MiB, 6),
    "deep_1MiB": lambda: _deep_chain(MiB, 7),
    "half_random_1MiB": lambda: synth.log_text(MiB // 2, 8) + _rnd(MiB // 2, 9),
    # text with 3 KiB random stretches: literal runs of ~3 KiB start and end all over the block, so
    # chains enter many 8 KiB tokenizing chunks past the first 64 positions (k_lbt_entry's walk
    # over the stored marks instead of the exit table)
    "mixed_1MiB": lambda: b"".join(synth.log_text(4096, 20 + k) + _rnd(3072, 40 + k) for k in range(150))[:MiB],
    "random_300k": lambda: _rnd(300_000, 10),            # stored block: not on this path
}
_CACHE = {}


def _data(name):
    if name not in _CACHE:
        _CACHE[name] = INPUTS[name]()
    return _CACHE[name]


def _with_env(var, value, fn):
    # library knob (s3hc_set_knob): the library reads the environment only once per process
    import s3hc_lz4 as S

    with S.knobs({var: value}):
        return fn()


def _wave_path(fn):
    return _with_env("S3HC_LB_DISABLE", "1", fn)


def _step_path(fn):  # large blocks through k_lb_run instead of the spread execution
    return _with_env("S3HC_LBW_DISABLE", "1", fn)


@pytest.mark.parametrize("name", sorted(INPUTS))
def test_lb_decodes_oracle_frames(engine, oracle, name):
    data = _data(name)
    frame = oracle.lz4flex_compress_frame(data)
    assert engine.decompress_frames(frame) == data
    assert _step_path(lambda: engine.decompress_frames(frame)) == data


@pytest.mark.parametrize("name", sorted(INPUTS))
def test_lb_decodes_gpu_frames(engine, oracle, name):
    data = _data(name)
    frame = engine.compress_frame(data)
    assert frame[5] in (0x50, 0x70)
    assert engine.decompress_frames(frame) == data
    assert _wave_path(lambda: engine.decompress_frames(frame)) == data


def test_lb_liblz4_large_blocks(engine):
    import lz4ref

    data = synth.log_text(3 * MiB + 5, 12)
    for bsid in (5, 6, 7):
        frame = lz4ref.compress_frame(data, block_size_id=bsid, linked=False)
        assert engine.decompress_frames(frame) == data


def test_lb_mixed_batch(engine, oracle):
    parts = [synth.log_text(65536, 20), _data("log_1MiB"), bytes(4 * MiB), synth.json_records(65536, 21),
             _data("deep_1MiB"), b"tail bytes" * 100]
    blob = b"".join(
        engine.store_mode_frame(p) if i == 5 else (oracle.lz4flex_compress_frame(p) if i % 2 else engine.compress_frame(p))
        for i, p in enumerate(parts))
    assert engine.decompress_frames(blob) == b"".join(parts)


def test_lb_random_corruption_matches_oracle_and_wave_path(engine, oracle):
    rng = random.Random(11)
    bases = [
        oracle.lz4flex_compress_frame(synth.log_text(300_000, 30)),
        engine.compress_frame(synth.json_records(200_000, 31)),
        oracle.lz4flex_compress_frame(_deep_chain(150_000, 32)),
        oracle.lz4flex_compress_frame(bytes(700_000)),
    ]
    n_err = 0
    for t in range(96):
        b = bytearray(bases[t % len(bases)])
        kind = t % 4
        if kind == 0:  # bit flip in the block payload
            i = rng.randrange(11, len(b))
            b[i] ^= 1 << rng.randrange(8)
        elif kind == 1:  # truncation
            del b[rng.randrange(11, len(b)):]
        elif kind == 2:  # random byte
            i = rng.randrange(11, len(b))
            b[i] = rng.randrange(256)
        else:  # random dword
            i = rng.randrange(11, len(b) - 4)
            b[i:i + 4] = bytes(rng.randrange(256) for _ in range(4))
        blob = bytes(b)
        st_o, out_o = oracle.decompress_status(blob)
        st_g, out_g = engine.decompress_status(blob)
        st_w, out_w = _wave_path(lambda: engine.decompress_status(blob))
        st_s, out_s = _step_path(lambda: engine.decompress_status(blob))
        assert st_g == st_o == st_w == st_s, (t, kind)
        assert out_g == out_o == out_w == out_s
        n_err += st_o != 0
    assert n_err > 50


def test_lb_block_size_errors(engine, oracle):
    # a block that decodes to more than the frame's max block size is corrupt (lz4_flex bounds
    # its output by the block size): BD 0x50 frame whose block expands past 256 KiB
    data = bytes(300_000)
    frame = bytearray(oracle.lz4flex_compress_frame(data))
    assert frame[5] == 0x70
    frame[5] = 0x50
    frame[6] = _hc(frame[4:6])
    st_o, _ = oracle.decompress_status(bytes(frame))
    st_g, _ = engine.decompress_status(bytes(frame))
    assert st_o != 0 and st_g == st_o


def _hc(desc):
    import oracle as O

    return (O.xxh32(bytes(desc)) >> 8) & 0xFF


def test_lb_device_plan(engine, oracle):
    parts = [_data("log_1MiB"), _data("zeros_1MiB+7"), synth.log_text(65536, 40), _data("json_1MiB")]
    frames = [oracle.lz4flex_compress_frame(p) for p in parts]
    blob = b"".join(frames)
    fo, o = [], 0
    for f in frames:
        fo.append(o)
        o += len(f)
    caps = [len(p) for p in parts]
    do = [sum(caps[:i]) for i in range(len(parts))]
    plan = engine.plan_decode(fo, [len(f) for f in frames], do, caps)
    src = engine.upload(blob)
    dst = engine.alloc(sum(caps) + 64)
    olen, st = engine.alloc(4 * len(parts)), engine.alloc(4 * len(parts))
    engine.decode_dev(plan, src, dst, olen, st)
    engine.sync()
    assert st.i32(len(parts)) == [0] * len(parts)
    assert olen.u32(len(parts)) == caps
    assert dst.read(sum(caps)) == b"".join(parts)


def test_lb_reader_reference_frames(engine):
    import s3hc_lz4 as S

    data = _deep_chain(3 * MiB, 50) + synth.log_text(2 * MiB, 51)
    import oracle as O

    blob = b"".join(O.lz4flex_compress_frame(data[i:i + MiB]) for i in range(0, len(data), MiB))
    r = S.RangeReader(engine, batch_bytes=2 * MiB)
    out = bytearray()
    for i in range(0, len(blob), 700_000):
        r.feed(blob[i:i + 700_000])
        while True:
            b = r.read(1 << 20)
            if not b:
                break
            out += b
    r.finish()
    while True:
        b = r.read(1 << 20)
        if not b:
            break
        out += b
    assert bytes(out) == data and r.total == len(data)
    r.close()


def _decode_dev(engine, frames, caps):
    blob = b"".join(frames)
    fo = [sum(len(f) for f in frames[:i]) for i in range(len(frames))]
    do = [sum(caps[:i]) for i in range(len(frames))]
    plan = engine.plan_decode(fo, [len(f) for f in frames], do, caps)
    src = engine.upload(blob)
    dst = engine.alloc(sum(caps) + 64)
    olen, st = engine.alloc(4 * len(frames)), engine.alloc(4 * len(frames))
    engine.decode_dev(plan, src, dst, olen, st)
    engine.sync()
    return st.i32(len(frames)), olen.u32(len(frames))


@pytest.mark.parametrize("short", [1, 1000, 300_000])
def test_lb_dst_too_small_matches_wave_path(engine, oracle, short):
    parts = [_data("log_1MiB"), _data("deep_1MiB"), _data("zeros_1MiB+7")]
    frames = [oracle.lz4flex_compress_frame(p) for p in parts]
    caps = [len(parts[0]) - short, len(parts[1]), len(parts[2]) - short]
    got = _decode_dev(engine, frames, caps)
    want = _wave_path(lambda: _decode_dev(engine, frames, caps))
    assert got == want == _step_path(lambda: _decode_dev(engine, frames, caps))
    assert got[0][0] == 3 and got[0][1] == 0 and got[0][2] == 3  # S3HC_DST_TOO_SMALL


def test_lb_randomized_structures_match_wave_path(engine, oracle):
    # seeded mixtures of text, byte runs, random bytes and match-of-match chains, frame sizes from
    # just above 64 KiB to 4 MiB + 1: both paths and the oracle agree byte for byte
    rng = random.Random(2024)
    for case in range(20):
        size = rng.choice([65_537, 100_000, 262_144, 700_001, MiB, 3 * MiB + 1, 4 * MiB + 1])
        parts, n = [], 0
        while n < size:
            kind = rng.randrange(4)
            k = rng.randrange(1, 200_000)
            if kind == 0:
                p = synth.log_text(k, rng.randrange(1 << 30))
            elif kind == 1:
                p = _runs(k, rng.randrange(1 << 30))
            elif kind == 2:
                p = _rnd(k, rng.randrange(1 << 30))
            else:
                p = _deep_chain(k, rng.randrange(1 << 30))
            parts.append(p)
            n += len(p)
        data = b"".join(parts)[:size]
        for frame in (oracle.lz4flex_compress_frame(data), engine.compress_frame(data)):
            got = engine.decompress_frames(frame)
            assert got == data, case
            assert _wave_path(lambda: engine.decompress_frames(frame)) == data, case
            assert _step_path(lambda: engine.decompress_frames(frame)) == data, case


@pytest.mark.parametrize("rounds", ["0", "1", "2"])
def test_lb_spread_gather_walks_unfinished_chains(engine, oracle, rounds):
    # with fewer pointer-jumping launches than the chains need, k_lbw_gather walks the rest
    for name in ("deep_1MiB", "log_1MiB", "runs_2MiB", "p251_1MiB+1"):
        data = _data(name)
        frame = oracle.lz4flex_compress_frame(data)
        assert _with_env("S3HC_LBW_ROUNDS", rounds, lambda: engine.decompress_frames(frame)) == data, name


@pytest.mark.parametrize("cap", [0, 1, 1_500_000, 3 * MiB])
def test_lb_spread_cap_splits_launch(engine, oracle, cap):
    # P capacity below the launch's output: the first blocks run spread, the rest the step loop
    # (cap 0 = spread execution off), all in one decode launch
    parts = [_data("log_1MiB"), _data("deep_1MiB"), _data("zeros_1MiB+7"), _data("json_1MiB"), _data("runs_2MiB")]
    frames = [oracle.lz4flex_compress_frame(p) for p in parts]
    blob = b"".join(frames)
    assert _with_env("S3HC_LBW_CAP", str(cap), lambda: engine.decompress_frames(blob)) == b"".join(parts)


@pytest.mark.parametrize("nframes", [16, 32])
def test_lb_spread_many_frames_device_plan(engine, nframes):
    # reference-format 1 MiB frames in one device launch: 16 spread (every tile of every block at
    # once), 32 run the step loop (more than kLbwMaxBlocks); both against the step loop
    data = (synth.log_text(16 * MiB, 60) + _deep_chain(8 * MiB, 61) + bytes(4 * MiB) +
            synth.json_records(4 * MiB, 62))[:nframes * MiB]
    import oracle as O

    frames = [O.lz4flex_compress_frame(data[i:i + MiB]) for i in range(0, len(data), MiB)]
    n = len(frames)
    fo = [sum(len(f) for f in frames[:i]) for i in range(n)]

    def run():
        plan = engine.plan_decode(fo, [len(f) for f in frames], [i * MiB for i in range(n)], [MiB] * n)
        src = engine.upload(b"".join(frames))
        dst = engine.alloc(n * MiB + 64)
        olen, st = engine.alloc(4 * n), engine.alloc(4 * n)
        engine.decode_dev(plan, src, dst, olen, st)
        engine.sync()
        return st.i32(n), olen.u32(n), dst.read(n * MiB)

    assert run() == ([0] * n, [MiB] * n, data)
    assert _step_path(run) == ([0] * n, [MiB] * n, data)


def test_lb_spread_execution_is_taken(engine, oracle, capfd):
    # the trace (S3HC_LB_TRACE) shows which execution ran: a lone 1 MiB reference frame spreads
    # over 137 tiles; with S3HC_LBW_DISABLE=1 it has none (step loop)
    frame = oracle.lz4flex_compress_frame(_data("log_1MiB"))
    capfd.readouterr()
    assert _with_env("S3HC_LB_TRACE", "1", lambda: engine.decompress_frames(frame)) == _data("log_1MiB")
    err = capfd.readouterr().err
    assert "blocks 1 " in err and "spread tiles 137 " in err, err
    assert _with_env("S3HC_LB_TRACE", "1", lambda: _step_path(lambda: engine.decompress_frames(frame))) == _data("log_1MiB")
    err = capfd.readouterr().err
    assert "spread tiles 0 " in err, err


def test_lb_spread_and_step_in_one_launch_randomized(engine, oracle):
    # one host call holding frames of both kinds (BD 0x40 blocks run the step loop, larger frames
    # spread), random sizes and contents, compared with the oracle and with the step loop alone
    rng = random.Random(77)
    for case in range(6):
        parts = []
        for _ in range(rng.randrange(2, 9)):
            size = rng.choice([1000, 65_536, 70_000, 300_000, MiB, 2 * MiB + 5])
            kind = rng.randrange(3)
            seed = rng.randrange(1 << 30)
            p = synth.log_text(size, seed) if kind == 0 else (_deep_chain(size, seed) if kind == 1 else _runs(size, seed))
            parts.append(p)
        blob = b"".join(oracle.lz4flex_compress_frame(p) for p in parts)
        want = b"".join(parts)
        assert engine.decompress_frames(blob) == want, case
        assert _step_path(lambda: engine.decompress_frames(blob)) == want, case


# Host-buffer calls read back each frame's slot prefix, min(slot, max(4 x compressed, 1 MiB)),
# in their first round trip: output past a frame's prefix must take the second trip.
def test_hostcall_single_frame_past_its_prefix(engine, oracle):
    # one BD 0x70 frame (4 MiB slot) of very compressible data: ~2.5 MiB decoded from a frame far
    # below 1/4 of that, so the decoded bytes run past the early prefix
    data = (b"abcdefgh" * 7 + b"\n") * (2_500_000 // 57)
    frame = engine.compress_frame(data)
    assert frame[5] == 0x70 and len(frame) * 4 < len(data) - (1 << 20)
    assert engine.decompress_frames(frame) == data
    assert engine.decompress_frames(oracle.lz4flex_compress_frame(data)) == data


@pytest.mark.parametrize("nframes", [2, 3, 4])
def test_hostcall_reference_multi_frame_files(engine, oracle, nframes):
    # a reference cache file: ~1 MiB frames (BD 0x70, 4 MiB slots) written back to back
    parts = [synth.log_text(MiB - 1000 * k, 40 + k) for k in range(nframes)]
    blob = b"".join(oracle.lz4flex_compress_frame(p) for p in parts)
    want = b"".join(parts)
    assert oracle.decompress_data(blob) == want
    assert engine.decompress_frames(blob) == want
    # a compressible frame after a text frame: the second one decodes past its own prefix
    big = bytes(3 * MiB)
    blob2 = oracle.lz4flex_compress_frame(parts[0]) + oracle.lz4flex_compress_frame(big)
    assert engine.decompress_frames(blob2) == parts[0] + big
