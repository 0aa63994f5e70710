"""The per-unit decoder agrees with the oracle, and with the one-wave variant when
the library is a diagnostic build that has it.

k_decode_pe (parser wave + executor wave per unit, the shipped one) and k_decode_units (one wave
per unit, S3HC_DEC_ONEWAVE=1, compiled only with S3HC_DIAG_VARIANTS=1: run these tests with
S3HC_LIB_PATH pointing at such a build) run the same lz4_flex FrameDecoder semantics (compression.rs:463-502):
every output byte and every status must match the oracle, on GPU-encoded, oracle-encoded
(lz4_flex layout) and liblz4 frames, multi-block and linked units, stored blocks, and corrupted
frames. S3HC_LB_DISABLE=1 keeps every block on these decoders.
"""
import os
import random

import pytest

import lz4ref
import synth

pytestmark = pytest.mark.gpu


def _with_env(env, fn):
    # library knobs (s3hc_set_knob): the library reads the environment only once per process
    import s3hc_lz4 as S

    with S.knobs(env):
        return fn()


def _onewave_built():
    import s3hc_lz4 as S

    try:
        S.get_knob("S3HC_DEC_ONEWAVE")
        return True
    except S.CodecError:
        return False


def _both(fn):
    pe = _with_env({"S3HC_LB_DISABLE": "1"}, fn)
    if not _onewave_built():  # (the shipped library: the per-unit decoder alone, against the oracle)
        return pe, pe
    one = _with_env({"S3HC_LB_DISABLE": "1", "S3HC_DEC_ONEWAVE": "1"}, fn)
    return pe, one


def _inputs():
    rng = random.Random(4242)
    runs = b"".join(bytes([rng.randrange(256)]) * rng.choice([1, 2, 5, 40, 300]) for _ in range(4000))
    per3 = b"abc" * 30000
    return {
        "log": synth.log_text(65536, 31),
        "json": synth.json_records(65536, 32),
        "runs": runs[:65536],
        "period3": per3[:65536],
        "small": synth.log_text(1000, 33),
        "rnd": rng.randbytes(65536),
        "log_300k": synth.log_text(300_000, 34),
    }


def test_decoders_agree_on_frames(engine, oracle):
    frames = []
    for name, data in _inputs().items():
        frames.append((engine.compress_frame(data), data))
        frames.append((oracle.lz4flex_compress_frame(data), data))
        frames.append((lz4ref.compress_frame(data, block_size_id=4, linked=True), data))   # 64 KiB linked
        frames.append((lz4ref.compress_frame(data, block_size_id=4, linked=False), data))  # 64 KiB independent
    for f, data in frames:
        pe, one = _both(lambda: engine.decompress_frames(f))
        assert pe == data and one == data


def test_decoders_agree_on_batches(engine):
    import s3hc_lz4 as S

    n, item = 512, 65536
    data = synth.log_text(n * item, 35)
    d_src = engine.upload(data)
    offs = [i * item for i in range(n)]
    plan = engine.plan_encode(offs, [item] * n)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n), engine.alloc(4 * n)
    engine.encode_dev(plan, d_src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(n), ilen.u32(n)

    def run():
        dplan = engine.plan_decode(fo, fl, offs, [item] * n)
        out = engine.alloc(n * item)
        olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
        engine.decode_dev(dplan, dst, out, olen, ost)
        engine.sync()
        return out.read(n * item), olen.u32(n), ost.i32(n)

    pe, one = _both(run)
    assert pe[2] == [0] * n and one[2] == [0] * n
    assert pe[1] == [item] * n and one[1] == [item] * n
    assert pe[0] == data and one[0] == data


def test_decoders_agree_on_corruption(engine, oracle):
    import s3hc_lz4 as S

    rng = random.Random(99)
    base = [engine.compress_frame(synth.log_text(65536, 40 + k)) for k in range(4)]
    for trial in range(60):
        f = bytearray(rng.choice(base))
        for _ in range(rng.randrange(1, 4)):
            p = rng.randrange(7, len(f))
            f[p] ^= 1 << rng.randrange(8)
        f = bytes(f)
        want_st, want = oracle.decompress_status(f)

        def dec():
            try:
                return 0, engine.decompress_frames(f)
            except S.CodecError as e:
                return e.status, b""

        (st_pe, out_pe), (st_one, out_one) = _both(dec)
        assert st_pe == st_one == want_st, trial
        if want_st == 0:
            assert out_pe == out_one == want
