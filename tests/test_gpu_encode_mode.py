"""Encoder modes (s3hc_set_encode_mode, include/s3hc_lz4.h): the fast default and the small mode
are two instantiations of the match finder (csrc/s3hc_kernels.hip k_enc_parse<kPS, kIns>). Both
write lz4_flex frames (compression.rs:539-557 decodes them): every frame must decode to its input
with the oracle's decompress_data (the restated FrameDecoder, compression.rs:479-480) and with the
GPU decoder; the small mode must be smaller on the bench's log text. Inputs: the synthetic families
the other encoder tests use plus short-period and byte-run blocks (the distance-1..4 candidate),
incompressible blocks (stored) and ragged sizes (a 4 KiB segment tail, a 12-byte block)."""
import random

import pytest

import s3hc_lz4 as S
import synth

pytestmark = pytest.mark.gpu
BLOCK = 65536


def _inputs():
    rng = random.Random(7)
    return {
        "log": synth.log_text(64 * BLOCK, synth.SEED_BASE + 11),
        "json": synth.json_records(32 * BLOCK, synth.SEED_BASE + 12),
        "runs": b"".join(bytes([rng.randrange(4)]) * rng.randrange(1, 300) for _ in range(3000))[: 16 * BLOCK],
        "period3": b"ab:" * (8 * BLOCK // 3),
        "random": rng.randbytes(4 * BLOCK),
        "ragged": synth.log_text(5 * BLOCK + 4097, synth.SEED_BASE + 13),
        "tiny": b"0123456789ab",
    }


INPUTS = _inputs()


@pytest.fixture
def mode_engine(engine):
    yield engine
    engine.set_encode_mode(S.ENC_FAST)


def _encode(engine, data, item):
    n = max(1, -(-len(data) // item))
    offs = [i * item for i in range(n)]
    lens = [min(item, len(data) - o) for o in offs]
    d_src = engine.upload(data)
    plan = engine.plan_encode(offs, lens)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n), engine.alloc(4 * n)
    engine.encode_dev(plan, d_src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(n), ilen.u32(n)
    return dst.read(fo[-1] + fl[-1]), fo, fl, offs, lens


@pytest.mark.parametrize("name", sorted(INPUTS))
@pytest.mark.parametrize("mode", [S.ENC_FAST, S.ENC_SMALL])
def test_mode_frames_decode(mode_engine, oracle, name, mode):
    data = INPUTS[name]
    mode_engine.set_encode_mode(mode)
    assert mode_engine.encode_mode == mode
    frames, fo, fl, offs, lens = _encode(mode_engine, data, BLOCK)
    mv = memoryview(data)
    for i in range(len(fo)):
        f = frames[fo[i]:fo[i] + fl[i]]
        assert oracle.decompress_data(f) == mv[offs[i]:offs[i] + lens[i]], f"{name} frame {i}"
    assert mode_engine.decompress_frames(frames, len(data)) == data


def test_small_mode_is_smaller_on_log_text(mode_engine):
    data = INPUTS["log"]
    sizes = {}
    for mode in (S.ENC_FAST, S.ENC_SMALL):
        mode_engine.set_encode_mode(mode)
        frames, *_ = _encode(mode_engine, data, BLOCK)
        sizes[mode] = len(frames)
    assert sizes[S.ENC_SMALL] < sizes[S.ENC_FAST]
    assert sizes[S.ENC_SMALL] / len(data) < 0.385


def test_mode_applies_to_host_calls_and_rejects_unknown(mode_engine, oracle):
    data = INPUTS["json"][: 3 * BLOCK]
    for mode in (S.ENC_FAST, S.ENC_SMALL):
        mode_engine.set_encode_mode(mode)
        assert oracle.decompress_data(mode_engine.compress_frame(data)) == data
    with pytest.raises(S.CodecError):
        mode_engine.set_encode_mode(2)
    assert mode_engine.encode_mode == S.ENC_SMALL
