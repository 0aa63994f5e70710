"""Batched incremental writers over the cross-request aggregator.

Ports of the reference's IncrementalRangeWriter tests (src/disk_cache.rs:14352-14633,
tests/batched_incremental_write_property_test.rs) plus aggregation checks: the frames a
writer emits are byte-identical to per-batch s3hc_compress_frame / s3hc_store_mode_frame,
decode back to the input with the oracle, and many writers' batches share GPU launches.
"""
import threading

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _agg(engine, batch_size, **kw):
    import s3hc_lz4 as S

    return S.BatchAggregator(engine, batch_size, **kw)


def _frames(blob):
    """Split concatenated frames at their boundaries (header walk of GPU-written frames:
    FLG 0x64, no block checksums, content checksum)."""
    out, p = [], 0
    while p < len(blob):
        assert blob[p:p + 4] == b"\x04\x22\x4d\x18"
        q = p + 7
        while True:
            w = int.from_bytes(blob[q:q + 4], "little")
            q += 4
            if w == 0:
                q += 4
                break
            q += w & 0x7FFFFFFF
        out.append(blob[p:q])
        p = q
    return out


def test_below_batch_size_does_not_flush(engine):
    # disk_cache.rs:14352-14392
    agg = _agg(engine, 8192, flush_batches=1)
    w = agg.begin(0, 3999, True)
    w.write(b"\x11" * 1500)
    w.write(b"\x22" * 2500)
    assert w.bytes_written == 4000 and w.compressed_bytes_written == 0
    assert w.batch_buf_len() == 4000 and len(w.file) == 0
    w.abort()
    assert agg.counters() == (0, 0)


def test_exactly_batch_size_flushes(engine, oracle):
    # disk_cache.rs:14395-14440
    agg = _agg(engine, 4096, flush_batches=1)
    w = agg.begin(0, 4095, True)
    w.write(b"\x7e" * 4096)
    assert w.bytes_written == 4096 and w.compressed_bytes_written > 0
    assert w.batch_buf_len() == 0 and len(w.file) == w.compressed_bytes_written
    assert oracle.decompress_data(bytes(w.file)) == b"\x7e" * 4096
    w.abort()


def test_commit_flushes_residual(engine, oracle):
    # disk_cache.rs:14460-14568: 2.5 batches -> 3 frames, the last one the residual
    agg = _agg(engine, 8192, flush_batches=1)
    data = synth.log_text(20480, 7)
    w = agg.begin(100, 100 + len(data) - 1, True)
    for i in range(0, len(data), 3000):
        w.write(data[i:i + 3000])
    before = w.compressed_bytes_written
    file = w.file
    spec = w.commit()
    assert spec.start == 100 and spec.end == 100 + len(data) - 1
    assert spec.uncompressed_size == len(data) and spec.compressed_size == len(file) > before
    fr = _frames(bytes(file))
    assert len(fr) == 3  # 9000, 9000, 2480 bytes (a chunk may overshoot batch_size, :1805-1807)
    assert oracle.decompress_data(bytes(file)) == data


def test_compression_disabled_writes_store_mode(engine, oracle):
    # disk_cache.rs:14576-14633: store-mode frames on disk, byte-identical to encode_store_mode_frame
    agg = _agg(engine, 65536, flush_batches=1)
    data = synth.log_text(150_000, 3)
    w = agg.begin(0, len(data) - 1, False)
    for i in range(0, len(data), 10_000):
        w.write(data[i:i + 10_000])
    file = w.file
    w.commit()
    fr = _frames(bytes(file))
    assert [f[5] for f in fr] == [0x70] * len(fr)  # store-mode BD
    sizes = [70_000, 70_000, 10_000]
    assert len(fr) == 3
    o = 0
    for f, n in zip(fr, sizes):
        assert f == oracle.store_mode_frame(data[o:o + n])
        o += n


@pytest.mark.parametrize("batch_size,total", [(65536, 100_000), (MiB, 3 * MiB + 1), (256 * 1024, 1)])
def test_byte_identity_and_frame_equivalence(engine, oracle, batch_size, total):
    # batched_incremental_write_property_test.rs:141-247, :582, :676; every frame equals the
    # single-shot encoder's frame of the same batch bytes
    agg = _agg(engine, batch_size, flush_batches=1)
    data = synth.log_text(total, 21)
    w = agg.begin(0, total - 1, True)
    rng = np.random.default_rng(5)
    i = 0
    while i < total:
        n = int(rng.integers(1, 70_000))
        w.write(data[i:i + n])
        i += n
    sink = w.file
    w.commit()  # flushes the residual batch into the sink
    file = bytes(sink)
    assert oracle.decompress_data(file) == data
    o = 0
    for f in _frames(file):
        u = len(oracle.decompress_data(f))
        assert f == engine.compress_frame(data[o:o + u])
        o += u
    assert o == total


def test_size_mismatch_and_salvage(engine, oracle):
    # finalize_incremental_range: exact-only errors; a prefix >= ratio is committed clamped
    import s3hc_lz4 as S

    agg = _agg(engine, 65536, flush_batches=1)
    data = synth.log_text(90_000, 2)
    w = agg.begin(1000, 1000 + 99_999, True)
    w.write(data)
    with pytest.raises(S.CodecError) as e:
        w.commit()
    assert "size mismatch" in str(e.value)
    w = agg.begin(1000, 1000 + 99_999, True)
    w.write(data)
    file = w.file
    spec = w.commit(min_commit_ratio=0.8)
    assert (spec.start, spec.end, spec.uncompressed_size) == (1000, 1000 + 90_000 - 1, 90_000)
    assert oracle.decompress_data(bytes(file)) == data
    with pytest.raises(S.CodecError):
        agg.begin(10, 9, True)  # start > end


def test_stats_shared_with_handler(engine):
    import s3hc_lz4 as S

    h = S.CompressionHandler(engine, 1024, True)
    agg = _agg(engine, 65536, flush_batches=1, stats=h)
    data = synth.log_text(200_000, 9)
    w = agg.begin(0, len(data) - 1, True)
    w.write(data)
    file = w.file
    w.commit()
    w2 = agg.begin(0, 99, False)
    w2.write(b"z" * 100)
    file2 = w2.file
    w2.commit()
    s = h.get_stats()
    assert s.total_bytes_before == len(data) + 100
    assert s.total_bytes_after == len(file) + len(file2)
    assert s.total_objects_compressed == 1 and s.total_objects_uncompressed == 1


def test_many_writers_share_launches(engine, oracle):
    # 24 concurrent writers (threads, like spawn_blocking writers): their full batches are
    # encoded together; every writer's file decodes to its own input and equals the
    # frame-by-frame single-shot encoding
    agg = _agg(engine, 65536, flush_batches=16)
    nw = 24
    datas = [synth.log_text(65536 * 5 + 777 * k, 100 + k) if k % 5 else synth.json_records(65536 * 4 + 13, k)
             for k in range(nw)]
    comp = [k % 7 != 3 for k in range(nw)]
    files = [None] * nw
    errs = []

    def run(k):
        try:
            d = datas[k]
            w = agg.begin(0, len(d) - 1, comp[k])
            for i in range(0, len(d), 16_384):
                w.write(d[i:i + 16_384])
            files[k] = w.file
            w.commit()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(nw)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    launches, batches = agg.counters()
    assert batches == sum(-(-len(d) // 65536) for d in datas)
    assert launches < batches  # batches of different writers shared launches
    for k in range(nw):
        f = bytes(files[k])
        assert oracle.decompress_data(f) == datas[k]
        o = 0
        for fr in _frames(f):
            u = len(oracle.decompress_data(fr))
            want = engine.compress_frame(datas[k][o:o + u]) if comp[k] else oracle.store_mode_frame(datas[k][o:o + u])
            assert fr == want
            o += u


def test_sink_failure_reported(engine):
    import s3hc_lz4 as S

    agg = _agg(engine, 65536, flush_batches=1)

    def bad(_frame):
        raise OSError("disk full")

    w = agg.begin(0, 2 * 65536 - 1, True, sink=bad)
    with pytest.raises(S.CodecError):
        w.write(synth.log_text(65536, 1))
        w.write(synth.log_text(65536, 2))
    w.abort()


def test_abort_drops_queued_batches(engine):
    agg = _agg(engine, 65536)  # flush only on commit / explicit flush
    got = []
    w = agg.begin(0, 10 * 65536 - 1, True, sink=got.append)
    w.write(synth.log_text(3 * 65536, 4))
    assert w.batch_buf_len() == 0 and not got  # queued, not delivered
    w.abort()
    agg.flush()
    assert not got


def test_64k_frame_policy(engine, oracle):
    # GPU-friendly layout: each batch becomes consecutive 64 KiB frames, identical to
    # s3hc_compress_frame(policy=64K) of the batch; the reference's frame loop decodes it the same
    import s3hc_lz4 as S

    agg = _agg(engine, MiB, flush_batches=4, frame_policy=S.BLK_64K_PER_FRAME)
    data = synth.log_text(2 * MiB + 12_345, 31)
    w = agg.begin(0, len(data) - 1, True)
    for i in range(0, len(data), 100_000):
        w.write(data[i:i + 100_000])
    sink = w.file
    w.commit()
    file = bytes(sink)
    assert oracle.decompress_data(file) == data
    fr = _frames(file)
    sizes = [1_100_000, len(data) - 1_100_000]  # one full batch (11 chunks) + the residual at commit
    assert all(f[5] == 0x40 for f in fr) and len(fr) == sum(-(-n // 65536) for n in sizes)
    o, k = 0, 0
    for n in sizes:
        want = engine.compress_frame(data[o:o + n], S.BLK_64K_PER_FRAME)
        got = b"".join(fr[k:k + len(_frames(want))])
        assert got == want
        k += len(_frames(want))
        o += n


def test_compat_frame_policy(engine, oracle):
    # S3HC_BLK_LZ4FLEX_COMPAT: each batch becomes the frame lz4_flex's FrameEncoder writes in
    # flush_batch (disk_cache.rs:1829-1846), byte for byte as the oracle restates it; a
    # compression-disabled writer in the same flush still gets store-mode frames
    import s3hc_lz4 as S

    agg = _agg(engine, 256 * 1024, flush_batches=8, frame_policy=S.BLK_LZ4FLEX_COMPAT)
    data = synth.log_text(3 * 256 * 1024 + 54_321, 41)
    raw = synth.jpeg_like(300_000, 42)
    w = agg.begin(0, len(data) - 1, True)
    w2 = agg.begin(0, len(raw) - 1, False)
    for i in range(0, len(data), 70_000):
        w.write(data[i:i + 70_000])
    for i in range(0, len(raw), 70_000):
        w2.write(raw[i:i + 70_000])
    f1, f2 = w.file, w2.file
    w.commit()
    w2.commit()
    file, file2 = bytes(f1), bytes(f2)
    assert oracle.decompress_data(file) == data and oracle.decompress_data(file2) == raw
    assert engine.decompress_frames(file) == data
    o = 0
    for fr in _frames(file):
        u = len(oracle.decompress_data(fr))
        assert fr == oracle.lz4flex_compress_frame(data[o:o + u])
        o += u
    assert o == len(data)
    o = 0
    for fr in _frames(file2):
        u = len(oracle.decompress_data(fr))
        assert fr == oracle.store_mode_frame(raw[o:o + u])
        o += u
