"""Pipelined range reader (s3hc_reader_*): stream_range_data semantics over batched device
decodes on several queues. Output must equal the oracle's
decompress of the same frames, in order, for any feed piece size and batch size; errors end the
stream after every earlier frame's bytes (tests/streaming_decompression_property_test.rs). A frame
whose only fault is its content checksum is delivered before S3HC_CHECKSUM, as lz4_flex's
FrameDecoder returns a frame's bytes before it checks the checksum at the EndMark
(disk_cache.rs:3884-3898; oracle.stream_range_data)."""
import pytest

import synth

pytestmark = pytest.mark.gpu
MiB = 1 << 20


def _drain(r, out, cap=MiB):
    while True:
        c = r.read(cap)
        if not c:
            return
        out += c


def _run(engine, frames, piece, batch, depth=3, cap=MiB, batch_max=None):
    import s3hc_lz4 as S

    r = S.RangeReader(engine, batch, depth, batch_max)
    out = bytearray()
    for i in range(0, len(frames), piece):
        r.feed(frames[i:i + piece])
        _drain(r, out, cap)
    r.finish()
    _drain(r, out, cap)
    return bytes(out), r


@pytest.mark.parametrize("piece,batch,depth,batch_max", [(1000, 256 << 10, 3, None), (65536, 256 << 10, 3, None),
                                                         (3 * MiB, 64 << 10, 2, None), (777_777, 4 * MiB, 4, None),
                                                         (10 * MiB, 1, 1, None), (3 * MiB, 64 << 10, 3, 2 * MiB),
                                                         (10 * MiB, 256 << 10, 2, 8 * MiB)])
def test_reader_matches_oracle(engine, oracle, piece, batch, depth, batch_max):
    data = synth.log_text(5 * MiB + 321, 41)
    # mixed layouts: 64 KiB frames, a reference-style 1 MiB frame, a store-mode frame, an empty frame
    frames = (engine.compress_frame(data[:2 * MiB], 1) + engine.compress_frame(data[2 * MiB:3 * MiB]) +
              engine.compress_frame(b"") + oracle.store_mode_frame(data[3 * MiB:3 * MiB + 70_000]) +
              engine.compress_frame(data[3 * MiB + 70_000:], 1))
    out, r = _run(engine, frames, piece, batch, depth, batch_max=batch_max)
    assert out == data
    assert r.total == len(data)


@pytest.mark.parametrize("batch_max", [None, 8 * MiB])
def test_reader_corrupt_frame_stops_after_earlier_frames(engine, oracle, batch_max):
    import s3hc_lz4 as S

    data = synth.log_text(16 * 65536, 42)
    fr = [engine.compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536)]
    bad = bytearray(fr[9])
    bad[-1] ^= 0x5A  # content checksum of frame 9
    frames = b"".join(fr[:9]) + bytes(bad) + b"".join(fr[10:])
    r = S.RangeReader(engine, 3 * 65536, 3, batch_max)
    r.feed(frames)
    r.finish()
    out = bytearray()
    with pytest.raises(S.CodecError) as e:
        _drain(r, out)
    assert e.value.status == S.S3HC_CHECKSUM
    # frame 9's bytes come before the error (the reference's order), nothing after it
    assert bytes(out) == data[:10 * 65536]
    assert oracle.stream_range_data(fr[:9] + [bytes(bad)] + fr[10:]) == (S.S3HC_CHECKSUM, bytes(out))


def test_reader_truncated_tail(engine):
    import s3hc_lz4 as S

    data = synth.log_text(300_000, 43)
    frames = engine.compress_frame(data[:200_000], 1) + engine.compress_frame(data[200_000:], 1)
    r = S.RangeReader(engine, 128 << 10, 3)
    r.feed(frames[:-7])
    r.finish()
    out = bytearray()
    with pytest.raises(S.CodecError) as e:
        _drain(r, out)
    assert e.value.status == S.S3HC_CORRUPT
    assert bytes(out) == data[:len(out)] and len(out) >= 196_608  # the complete 64 KiB frames came first


def test_reader_garbage_after_frames(engine):
    import s3hc_lz4 as S

    data = synth.log_text(100_000, 44)
    frames = engine.compress_frame(data, 1) + b"\xde\xad\xbe\xef" * 8
    r = S.RangeReader(engine, 1 << 20, 2)
    r.feed(frames)
    r.finish()
    out = bytearray()
    with pytest.raises(S.CodecError):
        _drain(r, out)
    assert bytes(out) == data


@pytest.mark.parametrize("policy", [1, 0])
@pytest.mark.parametrize("batch,batch_max", [(256 << 10, None), (4 << 20, None), (64 << 20, None),
                                             (256 << 10, 16 << 20)])
def test_reader_large_object_4mib_feeds(engine, policy, batch, batch_max):
    # config-4 shape at 1/64 scale: 128 MiB object, 4 MiB file reads, 1 MiB chunk reads
    data = synth.log_text(128 * MiB, 45)
    item = 65536 if policy == 1 else MiB
    frames = b"".join(engine.compress_frame(data[i:i + item], 0) for i in range(0, len(data), item)) if policy == 0 \
        else engine.compress_frame(data, 1)
    out, r = _run(engine, frames, 4 * MiB, batch, 3, batch_max=batch_max)
    assert len(out) == len(data) and out == data


@pytest.mark.parametrize("item", [65536, MiB])
def test_reader_output_beyond_speculative_prefix(engine, oracle, item):
    # zeros and byte runs compress far below 4:1, so a batch decodes to more than the prefix the
    # reader copies back right behind the decode (max(4 x input, 1 MiB)): the rest takes a second
    # copy; 64 KiB blocks of zeros also run k_dsmall's longest overlapping matches
    data = bytes(6 * MiB) + synth.log_text(MiB, 46) + b"\x07" * (3 * MiB + 5)
    frames = b"".join(oracle.lz4flex_compress_frame(data[i:i + item]) for i in range(0, len(data), item))
    for batch, depth in ((256 << 10, 3), (4 << 20, 2), (1, 1)):
        out, r = _run(engine, frames, 4 * MiB, batch, depth)
        assert out == data, (batch, depth)
        assert r.total == len(data)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_reader_corrupt_block_payloads_one_launch_batches(engine, oracle, seed):
    # batches of 64 KiB frames only: k_djump decodes them and runs the per-unit decoder itself for
    # the blocks its token index leaves (waves 2-15 leave first), k_dframe_close closes the frames.
    # Payload bytes of a few frames are flipped: the reader must deliver exactly the frames before
    # the first failing one (the oracle decodes frame by frame) and then report that frame's status.
    import random

    import s3hc_lz4 as S

    rng = random.Random(900 + seed)
    data = synth.log_text(24 * 65536, 47 + seed)
    fr = [bytearray(engine.compress_frame(data[i:i + 65536])) for i in range(0, len(data), 65536)]
    for k in rng.sample(range(4, 24), 3):
        f = fr[k]
        for _ in range(rng.randint(1, 6)):
            p = rng.randrange(11, len(f) - 8)  # inside the block payload (after header and block size)
            f[p] ^= 1 << rng.randrange(8)
    # (stream_range_data order: a frame that fails only its content checksum is delivered first)
    want_st, good = oracle.stream_range_data([bytes(f) for f in fr])
    first_bad = None if want_st == 0 else True
    r = S.RangeReader(engine, 256 << 10, 3)
    r.feed(b"".join(bytes(f) for f in fr))
    r.finish()
    out = bytearray()
    if first_bad is None:
        _drain(r, out)
        assert bytes(out) == data
        return
    with pytest.raises(S.CodecError) as e:
        _drain(r, out)
    assert e.value.status == want_st, (first_bad, want_st, e.value.status)
    assert bytes(out) == bytes(good)


@pytest.mark.parametrize("slots", ["1", "3", "4"])
def test_reader_batches_per_queue(engine, oracle, slots):
    # S3HC_READER_SLOTS batches in flight per queue (default 1): small batches so that every slot
    # holds one, a depth of 1..3 queues, and a corrupt frame late in the stream (the batches
    # queued behind it are dropped, every earlier byte delivered)
    import s3hc_lz4 as S

    data = synth.log_text(3 * MiB + 4321, 43)
    fr = [engine.compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536)]
    with S.knobs({"S3HC_READER_SLOTS": slots}):
        for depth in (1, 2, 3):
            out, r = _run(engine, b"".join(fr), 200_000, 100_000, depth)
            assert out == data, depth
            assert r.total == len(data)
        bad = bytearray(fr[40])
        bad[-2] ^= 0x21  # content checksum of frame 40
        r = S.RangeReader(engine, 70_000, 3)
        r.feed(b"".join(fr[:40]) + bytes(bad) + b"".join(fr[41:]))
        r.finish()
        out = bytearray()
        with pytest.raises(S.CodecError) as e:
            _drain(r, out)
        assert e.value.status == S.S3HC_CHECKSUM
        assert bytes(out) == data[:41 * 65536]


@pytest.mark.parametrize("poison", [None, "1"])
@pytest.mark.parametrize("corrupt_at", [None, 150, 187])
def test_reader_many_small_frames_stored_and_corrupt(engine, oracle, poison, corrupt_at):
    # batches of far more than 32 small frames, with stored (incompressible)
    # frames the token index leaves to the per-unit decoder, and a corrupt frame late in a batch.
    # Every delivered byte and the status must be the oracle's, frame by frame. S3HC_POISON=1 fills
    # every device scratch buffer with 0xFF when allocated: a read of anything no launch wrote
    # would fail the same way on every box (the GPUTEST_r04 fault: results of the fused close).
    import random

    import s3hc_lz4 as S

    rng = random.Random(77 if corrupt_at is None else corrupt_at)
    items = []
    for k in range(192):
        n = rng.choice((4096, 6000, 1500, 13, 5, 65536 // 8))
        if k % 17 == 5:
            items.append(rng.randbytes(n))             # stored block
        elif k % 11 == 3:
            items.append(bytes([k & 0xFF]) * n)        # one long overlapping match
        else:
            items.append(synth.log_text(n, 300 + k))
    fr = [bytearray(oracle.lz4flex_compress_frame(x)) for x in items]
    if corrupt_at is not None:
        fr[corrupt_at][-1] ^= 0x44  # content checksum
    want_st, good = oracle.stream_range_data([bytes(f) for f in fr])
    with S.knobs({"S3HC_POISON": poison}):
        for batch, depth in ((256 << 10, 3), (64 << 10, 2)):
            r = S.RangeReader(engine, batch, depth)
            r.feed(b"".join(bytes(f) for f in fr))
            r.finish()
            out = bytearray()
            if want_st == 0:
                _drain(r, out)
                assert bytes(out) == b"".join(items), (batch, depth)
            else:
                with pytest.raises(S.CodecError) as e:
                    _drain(r, out)
                assert e.value.status == want_st
                assert bytes(out) == bytes(good), (batch, depth)


def test_reader_slots_pooled_across_readers(engine, oracle):
    # Readers of one context reuse each other's slots and queues (a GET opens one reader): a slot
    # that served 64 KiB frames, reference 1 MiB frames or a failing stream must serve the next
    # reader exactly (its batch state is cleared, its buffers regrow as needed)
    import s3hc_lz4 as S

    small = synth.log_text(3 * MiB + 77, 71)
    big = synth.log_text(5 * MiB + 5, 72)
    f_small = b"".join(engine.compress_frame(small[i:i + 65536]) for i in range(0, len(small), 65536))
    f_big = b"".join(oracle.lz4flex_compress_frame(big[i:i + MiB]) for i in range(0, len(big), MiB))
    bad = bytearray(f_small)
    bad[-3] ^= 0x40  # content checksum of the last frame
    for k in range(12):
        kind = k % 3
        depth = 1 + k % 4
        if kind == 0:
            out, r = _run(engine, f_small, 1 << 20, 256 << 10, depth)
            assert out == small and r.total == len(small)
        elif kind == 1:
            out, r = _run(engine, f_big, 3 << 20, 256 << 10, depth)
            assert out == big and r.total == len(big)
        else:
            r = S.RangeReader(engine, 256 << 10, depth)
            r.feed(bytes(bad))
            r.finish()
            got = bytearray()
            with pytest.raises(S.CodecError) as e:
                _drain(r, got)
            assert e.value.status == S.S3HC_CHECKSUM
            assert bytes(got) == small  # the last frame's bytes, then its checksum error
        r.close()


def _ref_frames(oracle, data, item=MiB):
    return [bytearray(oracle.lz4flex_compress_frame(data[i:i + item])) for i in range(0, len(data), item)]


@pytest.mark.parametrize("batch,depth,batch_max", [(256 << 10, 3, None), (256 << 10, 1, None), (64 << 10, 2, None),
                                                   (256 << 10, 3, 8 * MiB), (16 * MiB, 2, None)])
@pytest.mark.parametrize("fault", ["checksum", "payload"])
def test_reader_reference_frames_checksum_after_bytes(engine, oracle, batch, depth, batch_max, fault):
    # the reference's cache files are chains of ~1 MiB frames of one block
    # (disk_cache.rs:1826-1847); their content checksums are verified behind the delivered bytes
    # (the second close), and a mismatch ends the stream with S3HC_CHECKSUM after that frame's
    # bytes and before any byte of a later frame (stream_range_data, disk_cache.rs:3884-3898).
    import s3hc_lz4 as S

    data = synth.log_text(7 * MiB + 4321, 91)
    fr = _ref_frames(oracle, data)
    k = 4
    if fault == "checksum":
        fr[k][-2] ^= 0x08                      # the stored checksum itself
    else:
        fr[k][len(fr[k]) // 2] ^= 0x01         # a payload byte: decodes (or not), checksum differs
    want_st, want = oracle.stream_range_data([bytes(f) for f in fr])
    assert want_st != 0
    if fault == "checksum":
        assert want_st == S.S3HC_CHECKSUM and want == data[:(k + 1) * MiB]
    for piece in (3 * MiB, 700_001):
        r = S.RangeReader(engine, batch, depth, batch_max)
        out = bytearray()
        with pytest.raises(S.CodecError) as e:
            for i in range(0, sum(map(len, fr)), piece):
                r.feed(b"".join(bytes(f) for f in fr)[i:i + piece])
                _drain(r, out)
            r.finish()
            _drain(r, out)
        assert e.value.status == want_st, (piece, batch, depth)
        assert bytes(out) == want, (piece, batch, depth, len(out), len(want))
        r.close()


@pytest.mark.parametrize("order", ["checksum_first", "corrupt_first", "clean_checksum_then_corrupt"])
def test_reader_deferred_checksum_and_decode_error_in_one_batch(engine, oracle, order):
    # one batch (batch_max) holding several reference frames: a deferred checksum failure and a
    # decode failure of a later frame — the first in stream order decides, with the bytes before it
    import s3hc_lz4 as S

    data = synth.log_text(6 * MiB, 92)
    fr = _ref_frames(oracle, data)
    if order == "checksum_first":
        fr[1][-1] ^= 0x80
        fr[3][9] ^= 0xFF                        # the first block word: a decode/structure error
    elif order == "corrupt_first":
        fr[1][9] ^= 0xFF
        fr[3][-1] ^= 0x80
    else:
        fr[3][9] ^= 0xFF
    want_st, want = oracle.stream_range_data([bytes(f) for f in fr])
    for depth in (1, 3):
        r = S.RangeReader(engine, 64 << 20, depth)
        r.feed(b"".join(bytes(f) for f in fr))
        r.finish()
        out = bytearray()
        with pytest.raises(S.CodecError) as e:
            _drain(r, out)
        assert e.value.status == want_st
        assert bytes(out) == want
        r.close()


def test_reader_reference_frames_clean_many_depths(engine, oracle):
    # the deferred-checksum path on clean reference frames: every byte, in order, every depth
    import s3hc_lz4 as S

    data = synth.log_text(12 * MiB + 99, 93)
    frames = b"".join(bytes(f) for f in _ref_frames(oracle, data))
    for depth in (1, 2, 3, 4):
        for cap in (MiB, 100_000):
            out, r = _run(engine, frames, 2 * MiB, 256 << 10, depth, cap=cap)
            assert out == data, (depth, cap)
            assert r.total == len(data)
