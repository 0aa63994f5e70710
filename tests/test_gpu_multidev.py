"""Multi-device fan-out inside one process (the proxy's concurrent writers and
range reads, /root/reference/src/http_proxy.rs:11608-11622): an aggregator and a range reader over
several contexts. On a one-GPU box the contexts share device 0 (the --share-gpu rehearsal): the
shard / dispatch logic and every copy between devices' queues run as on a multi-GPU node, and
the output must be byte-identical to the one-context path. No collective is involved."""
import threading

import pytest

import synth

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def engines():
    import s3hc_lz4 as S

    n = max(2, min(S.device_count(), 4))
    return [S.Engine(i % S.device_count()) for i in range(n)]


def _write_all(agg, datas, comp, chunk=16_384):
    files, errs = [None] * len(datas), []

    def run(k):
        try:
            d = datas[k]
            w = agg.begin(0, len(d) - 1, comp[k])
            for i in range(0, len(d), chunk):
                w.write(d[i:i + chunk])
            files[k] = w.file
            w.commit()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(datas))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return [bytes(f) for f in files]


@pytest.mark.parametrize("policy", [0, 1, 2])
def test_multi_device_aggregator_byte_identical(engine, engines, oracle, policy):
    import s3hc_lz4 as S

    nw = 20
    datas = [synth.log_text(65536 * 3 + 999 * k, 500 + k) if k % 4 else synth.json_records(65536 * 2 + 17 * k, k)
             for k in range(nw)]
    comp = [k % 6 != 2 for k in range(nw)]
    one = S.BatchAggregator(engine, 65536, flush_batches=12, frame_policy=policy)
    many = S.BatchAggregator(engines, 65536, flush_batches=12, frame_policy=policy)
    f1 = _write_all(one, datas, comp)
    fm = _write_all(many, datas, comp)
    assert fm == f1
    for k in range(nw):
        assert oracle.decompress_data(fm[k]) == datas[k]
    assert one.counters()[1] == many.counters()[1]
    one.close()
    many.close()


def test_multi_device_aggregator_splits_each_flush(engines, oracle):
    # one writer, 8 full batches, one flush of all 8: one launch per device, frames in order
    import s3hc_lz4 as S

    data = synth.log_text(8 * 65536, 77)
    agg = S.BatchAggregator(engines, 65536, flush_batches=8)
    w = agg.begin(0, len(data) - 1, True)
    for i in range(0, len(data), 65536):
        w.write(data[i:i + 65536])
    f = bytes(w.file)
    w.commit()
    launches, batches = agg.counters()
    assert batches == 8 and launches == len(engines)
    assert f == b"".join(engines[0].compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536))
    assert oracle.decompress_data(f) == data
    agg.close()


def test_multi_device_aggregator_refuses_duplicate_context(engine):
    import s3hc_lz4 as S

    with pytest.raises(S.CodecError):
        S.BatchAggregator([engine, engine], 65536)


@pytest.mark.parametrize("batch,depth", [(256 << 10, 2), (4 * MiB, 1), (64 << 10, 3)])
def test_multi_device_reader_matches(engines, oracle, batch, depth):
    import s3hc_lz4 as S

    data = synth.log_text(9 * MiB + 4321, 61)
    frames = b"".join(oracle.lz4flex_compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536))
    frames += oracle.lz4flex_compress_frame(data[:MiB])  # a reference-style 1 MiB frame
    r = S.RangeReader(engines, batch, depth)
    out = bytearray()
    for i in range(0, len(frames), 3 * MiB):
        r.feed(frames[i:i + 3 * MiB])
        while True:
            c = r.read(MiB)
            if not c:
                break
            out += c
    r.finish()
    while True:
        c = r.read(MiB)
        if not c:
            break
        out += c
    assert bytes(out) == data + data[:MiB]


def test_multi_device_reader_corrupt_frame(engines, oracle):
    import s3hc_lz4 as S

    data = synth.log_text(40 * 65536, 62)
    fr = [bytearray(oracle.lz4flex_compress_frame(data[i:i + 65536])) for i in range(0, len(data), 65536)]
    fr[29][-1] ^= 0x10
    r = S.RangeReader(engines, 100_000, 2)
    r.feed(b"".join(bytes(f) for f in fr))
    r.finish()
    out = bytearray()
    with pytest.raises(S.CodecError) as e:
        while True:
            c = r.read(MiB)
            if not c:
                break
            out += c
    assert e.value.status == S.S3HC_CHECKSUM
    assert bytes(out) == data[:30 * 65536]  # frame 29's bytes before its checksum error


def test_context_destroyed_before_reader_and_aggregator(oracle):
    """s3hc_destroy with a reader and an aggregator still open: they keep the context (reference
    counted) and work to the end; the last of them frees it (no use of freed memory at close)."""
    import s3hc_lz4 as S

    e = S.Engine(0)
    data = synth.log_text(3 * 65536 + 123, 77)
    frames = b"".join(e.compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536))
    rd = S.RangeReader(e, 256 << 10, 3)
    agg = S.BatchAggregator(e, 65536, flush_batches=4)
    e.close()
    rd.feed(frames)
    rd.finish()
    out = b""
    while True:
        k = rd.read()
        if not k:
            break
        out += k
    assert out == data
    w = agg.begin(0, len(data) - 1, True)
    for i in range(0, len(data), 16_384):
        w.write(data[i:i + 16_384])
    f = w.file
    w.commit()
    assert oracle.decompress_data(bytes(f)) == data
    rd.close()
    agg.close()


def test_multi_device_aggregator_refuses_mixed_encode_modes(engines):
    # frames must not depend on the device a batch lands on — contexts whose
    # match-finder modes differ are refused at creation, and a flush after a mode change fails
    # every writer of that flush instead of writing device-dependent frames
    import s3hc_lz4 as S

    a, b = engines[0], engines[1]
    try:
        b.set_encode_mode(S.ENC_SMALL)
        with pytest.raises(S.CodecError) as e:
            S.BatchAggregator([a, b], 65536)
        assert e.value.status == S.S3HC_INVALID_ARG
        b.set_encode_mode(S.ENC_FAST)
        agg = S.BatchAggregator([a, b], 65536, flush_batches=0)
        data = [synth.log_text(200_000, 70 + k) for k in range(4)]
        ws = [agg.begin(0, len(d) - 1, True) for d in data]
        for w, d in zip(ws, data):
            w.write(d)
        b.set_encode_mode(S.ENC_SMALL)
        with pytest.raises(S.CodecError) as e:
            agg.flush()
        assert e.value.status == S.S3HC_INVALID_ARG
        for w in ws:  # every writer of the flush failed (a later call reports it)
            with pytest.raises(S.CodecError):
                w.commit()
        agg.close()
    finally:
        b.set_encode_mode(S.ENC_FAST)


def test_multi_device_readers_in_opposite_context_order(engines, oracle):
    # readers over [c0, c1] and [c1, c0] used from two threads at once take the
    # contexts' locks in one global order (no deadlock), and neither holds them while it waits
    import s3hc_lz4 as S

    data = synth.log_text(6 * MiB + 11, 63)
    frames = b"".join(oracle.lz4flex_compress_frame(data[i:i + 65536]) for i in range(0, len(data), 65536))
    frames += b"".join(oracle.lz4flex_compress_frame(data[i:i + MiB]) for i in range(0, 2 * MiB, MiB))
    want = data + data[:2 * MiB]
    outs, errs = [None, None], []

    def run(k):
        try:
            order = engines[:2] if k == 0 else engines[1::-1]
            for _ in range(4):
                r = S.RangeReader(order, 256 << 10, 2)
                out = bytearray()
                for i in range(0, len(frames), MiB):
                    r.feed(frames[i:i + MiB])
                    while True:
                        c = r.read(MiB)
                        if not c:
                            break
                        out += c
                r.finish()
                while True:
                    c = r.read(MiB)
                    if not c:
                        break
                    out += c
                r.close()
                assert bytes(out) == want
            outs[k] = True
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    ts = [threading.Thread(target=run, args=(k,), daemon=True) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    assert not any(t.is_alive() for t in ts), "readers in opposite context order deadlocked"
    assert not errs, errs
    assert outs == [True, True]
