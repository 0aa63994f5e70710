"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Bar: decoded bytes bit-exact with the oracle (restatement of the
reference path) on the same inputs; status codes equal on corrupt inputs; store-mode frames
byte-identical (pinned by compression.rs:326-368). Compressed bytes differ from lz4_flex's
by design (parallel match finder; "parity unpinned" for compressed bytes), so encoder output
is checked by decoding it with the oracle and with liblz4.
"""
import os
import random

import numpy as np
import pytest

import lz4ref
import synth
import s3hc_lz4 as S

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def pattern251(n):  # tests/lz4_roundtrip_preservation_test.rs:192-196 fixture data
    return bytes(i % 251 for i in range(n))


def rnd(n, seed=1):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


INPUTS = {
    "empty": b"",
    "1": b"x",
    "13": b"0123456789abc",
    "p251_63": pattern251(63),
    "p251_64": pattern251(64),
    "p251_1024": pattern251(1024),
    "p251_64k": pattern251(65536),
    "p251_64k+1": pattern251(65537),
    "p251_1MiB+1": pattern251(MiB + 1),
    "zeros_64k": bytes(65536),
    "zeros_300k": bytes(300_000),
    "runs": b"".join(bytes([c]) * (i % 97 + 1) for i, c in enumerate(b"abcdefghij" * 300)),
    "random_64k": rnd(65536),
    "random_100": rnd(100, 3),
    "log_64k": synth.log_text(65536),
    "log_200k": synth.log_text(200_000, 11),
    "log_1MiB": synth.log_text(MiB, 12),
    "json_64k": synth.json_records(65536),
    "half_random": synth.log_text(40_000) + rnd(30_000, 5),
    "text_repeat": b"This is some test data that should be compressed because it's longer than the threshold" * 40,
}


@pytest.mark.parametrize("name", sorted(INPUTS))
def test_store_mode_frame_byte_exact(engine, oracle, name):
    data = INPUTS[name]
    assert engine.store_mode_frame(data) == oracle.store_mode_frame(data)


@pytest.mark.parametrize("n", [4 * MiB, 4 * MiB + 1, 9 * MiB + 7])
def test_store_mode_frame_multi_block(engine, oracle, n):
    data = synth.jpeg_like(n)
    assert engine.store_mode_frame(data) == oracle.store_mode_frame(data)


@pytest.mark.parametrize("policy", [0, 1])
@pytest.mark.parametrize("name", sorted(INPUTS))
def test_compress_frame_roundtrip(engine, oracle, name, policy):
    data = INPUTS[name]
    frame = engine.compress_frame(data, policy)
    assert oracle.decompress_data(frame) == data
    assert engine.decompress_frames(frame) == data
    if lz4ref.available:
        assert lz4ref.decompress(frame, len(data)) == data
    if policy == 0:
        ref = oracle.lz4flex_compress_frame(data)
        assert frame[:7] == ref[:7]  # same FLG/BD/HC as lz4_flex BlockSize::Auto
        # lz4_flex stores a block iff it does not shrink; ours must agree on incompressible input
        if name.startswith("random"):
            assert frame == ref


@pytest.mark.parametrize("name", sorted(INPUTS))
def test_decode_oracle_frames(engine, oracle, name):
    data = INPUTS[name]
    frame = oracle.lz4flex_compress_frame(data)
    assert engine.decompress_frames(frame) == data


@pytest.mark.skipif(not lz4ref.available, reason="liblz4 not present")
@pytest.mark.parametrize("bsid", [4, 5, 6, 7])
@pytest.mark.parametrize("linked", [False, True])
@pytest.mark.parametrize("flags", [(True, False, False), (True, True, False), (False, False, True), (True, True, True)])
def test_decode_liblz4_frames(engine, oracle, bsid, linked, flags):
    cc, bc, cs = flags
    data = synth.log_text(700_000, 21) + pattern251(100_000) + bytes(70_000)
    frame = lz4ref.compress_frame(data, bsid, linked, cc, bc, cs)
    assert oracle.decompress_data(frame) == data
    assert engine.decompress_frames(frame) == data


@pytest.mark.skipif(not lz4ref.available, reason="liblz4 not present")
@pytest.mark.parametrize("level", [1, 9])
def test_decode_liblz4_hc(engine, level):
    data = synth.json_records(300_000, 9)
    frame = lz4ref.compress_frame(data, 4, False, True, False, False, level)
    assert engine.decompress_frames(frame) == data


def _statuses(engine, oracle, blob):
    st_o, out_o = oracle.decompress_status(blob)
    st_g, out_g = engine.decompress_status(blob)
    return st_o, out_o, st_g, out_g


@pytest.mark.parametrize(
    "blob",
    [
        bytes([0x04, 0x22, 0x4D, 0x18, 0xFF, 0xFF, 0xFF, 0xFF, 0x00, 0x01, 0x02]),  # compression.rs:740-741
        bytes([0xDE, 0xAD, 0xBE, 0xEF, 0x01, 0x02, 0x03, 0x04]),  # disk_cache.rs:13740
        b"\x04\x22\x4d",
        b"\x04\x22\x4d\x18\x64\x40\xa7",  # header only, truncated
        bytes.fromhex("04224d186440a700000000055dcc02") + b"garbage",  # empty frame then garbage: stops
        bytes.fromhex("04224d186440a700000000055dcc03"),  # bad checksum of empty frame
        bytes.fromhex("02214c18") + bytes(8),  # legacy magic
        bytes.fromhex("502a4d18") + bytes(8),  # skippable frame
    ],
)
def test_corrupt_vectors_match_oracle(engine, oracle, blob):
    st_o, out_o, st_g, out_g = _statuses(engine, oracle, blob)
    assert st_g == st_o
    assert out_g == out_o


def test_random_corruption_matches_oracle(engine, oracle):
    rng = random.Random(7)
    bases = [
        oracle.lz4flex_compress_frame(INPUTS["log_64k"]),
        engine.compress_frame(INPUTS["json_64k"]),
        oracle.store_mode_frame(INPUTS["p251_1024"]),
        oracle.lz4flex_compress_frame(INPUTS["text_repeat"]),
    ]
    n_ok = n_err = 0
    for t in range(160):
        b = bytearray(bases[t % len(bases)])
        kind = t % 4
        if kind == 0:
            i = rng.randrange(len(b))
            b[i] ^= 1 << rng.randrange(8)
        elif kind == 1:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            i = rng.randrange(11, len(b))
            b[i] = rng.randrange(256)
        else:
            i = rng.randrange(len(b))
            b[i:i + 4] = bytes(rng.randrange(256) for _ in range(4))
        st_o, out_o, st_g, out_g = _statuses(engine, oracle, bytes(b))
        assert st_g == st_o, (t, kind, bytes(b).hex() if len(b) < 400 else len(b))
        assert out_g == out_o
        n_ok += st_o == 0
        n_err += st_o != 0
    assert n_err > 100


def test_concatenated_mixed_frames(engine, oracle):
    # compression.rs:684-700 — compressed + store-mode frames concatenated
    comp = engine.compress_frame(b"AAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA" * 5)
    stored = engine.store_mode_frame(b"incompressible-ish chunk")
    assert engine.decompress_frames(comp + stored) == b"A" * 200 + b"incompressible-ish chunk"
    # tests/lz4_roundtrip_preservation_test.rs:129-180 — alternating store/compressed chunks
    data = pattern251(MiB + 1)
    for n_chunks in (1, 3, 8):
        step = -(-len(data) // n_chunks)
        chunks = [data[i:i + step] for i in range(0, len(data), step)]
        blob = b"".join(engine.store_mode_frame(c) if i % 2 else engine.compress_frame(c) for i, c in enumerate(chunks))
        assert engine.decompress_frames(blob) == data
        assert oracle.decompress_data(blob) == data


def test_empty_frame_stops_loop(engine, oracle):
    a = engine.compress_frame(b"first frame bytes " * 10)
    empty = engine.compress_frame(b"")
    c = engine.compress_frame(b"never reached")
    blob = a + empty + c
    assert engine.decompress_frames(blob) == oracle.decompress_data(blob) == b"first frame bytes " * 10


def test_streaming_decoder_matches_buffered(engine, oracle):
    # tests/streaming_decompression_property_test.rs: streamed output == buffered output
    data = synth.log_text(3 * MiB + 123, 31)
    frames = b"".join(engine.compress_frame(data[i:i + MiB]) for i in range(0, len(data), MiB))
    for piece in (1000, 65536, 2 * MiB):
        s = engine.stream()
        out = bytearray()
        for i in range(0, len(frames), piece):
            s.feed(frames[i:i + piece])
            while True:
                chunk = s.read(MiB)
                if not chunk:
                    break
                out += chunk
        s.finish()
        while True:
            chunk = s.read(MiB)
            if not chunk:
                break
            out += chunk
        assert bytes(out) == data
        assert s.total == len(data)


def _batch_roundtrip(engine, oracle, data, block, modes):
    n = len(data) // block
    src = engine.upload(data)
    offs = [i * block for i in range(n)]
    plan = engine.plan_encode(offs, [block] * n, modes)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n), engine.alloc(4 * n)
    engine.encode_dev(plan, src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(n), ilen.u32(n)
    total = fo[-1] + fl[-1]
    host_frames = dst.read(total)
    # every frame decodes with the oracle (a sample) and all frames concatenated decode back
    for i in range(0, n, max(1, n // 16)):
        assert oracle.decompress_data(host_frames[fo[i]:fo[i] + fl[i]]) == data[i * block:(i + 1) * block]
    assert oracle.decompress_data(host_frames) == data
    dplan = engine.plan_decode(fo, fl, offs, [block] * n)
    out = engine.alloc(len(data))
    olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
    ost.fill(0xFF)
    engine.decode_dev(dplan, dst, out, olen, ost)
    engine.sync()
    assert ost.i32(n) == [0] * n
    assert olen.u32(n) == [block] * n
    assert out.read() == data
    return total


def test_batch_config2_log_blocks(engine, oracle):
    block = 65536
    data = synth.log_text(256 * block, synth.SEED_BASE + 1)
    total = _batch_roundtrip(engine, oracle, data, block, None)
    assert total < 0.6 * len(data)


def test_batch_config3_mixed(engine, oracle):
    data, kinds = synth.mixed_blocks(128)
    # the reference's decision per cache key (cache.rs:1158-1178): JPEG ranges -> store-mode
    keys = [f"b/o{i}{'.jpg' if k else '.json'}:range:{65536 * i}-{65536 * i + 65535}" for i, k in enumerate(kinds)]
    modes = [0 if S.effective_compression(S.ResolvedSettings(), 1024, key, 65536) else 1 for key in keys]
    assert modes == kinds
    _batch_roundtrip(engine, oracle, data, 65536, modes)


def test_batch_unaligned_and_ragged(engine, oracle):
    # items at odd offsets with ragged lengths (empty, tiny, > 64 KiB, 256 KiB+)
    rng = np.random.default_rng(5)
    lens = [0, 1, 12, 13, 100, 65535, 65536, 65537, 300_001, 5000, 262_144, 262_145]
    base = synth.log_text(sum(lens) + 64 * len(lens), 55)
    offs, o = [], 3
    for L in lens:
        offs.append(o)
        o += L + int(rng.integers(0, 9))
    data = base[:o]
    src = engine.upload(data)
    n = len(lens)
    plan = engine.plan_encode(offs, lens, [0] * n)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * n), engine.alloc(4 * n)
    engine.encode_dev(plan, src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(n), ilen.u32(n)
    frames = dst.read(fo[-1] + fl[-1])
    for i in range(n):
        item = data[offs[i]:offs[i] + lens[i]]
        f = frames[fo[i]:fo[i] + fl[i]]
        assert oracle.decompress_data(f) == item
        assert f[:7] == oracle.lz4flex_compress_frame(item)[:7]
    # decode into unaligned destinations
    doffs = [sum(lens[:i]) + 5 * i + 1 for i in range(n)]
    dplan = engine.plan_decode(fo, fl, doffs, lens)
    out = engine.alloc(doffs[-1] + lens[-1] + 8)
    olen, ost = engine.alloc(4 * n), engine.alloc(4 * n)
    engine.decode_dev(dplan, dst, out, olen, ost)
    engine.sync()
    assert ost.i32(n) == [0] * n and olen.u32(n) == lens
    got = out.read()
    for i in range(n):
        assert got[doffs[i]:doffs[i] + lens[i]] == data[offs[i]:offs[i] + lens[i]]


def test_batch_decode_reports_corruption(engine, oracle):
    block = 65536
    data = synth.log_text(8 * block, 77)
    frames = [engine.compress_frame(data[i * block:(i + 1) * block]) for i in range(8)]
    frames[3] = frames[3][:-1] + bytes([frames[3][-1] ^ 0x40])  # content checksum
    b = bytearray(frames[5])
    b[200] ^= 0xFF
    frames[5] = bytes(b)
    blob = b"".join(frames)
    fo = np.cumsum([0] + [len(f) for f in frames[:-1]]).tolist()
    plan = engine.plan_decode(fo, [len(f) for f in frames], [i * block for i in range(8)], [block] * 8)
    src = engine.upload(blob)
    out = engine.alloc(8 * block)
    olen, ost = engine.alloc(32), engine.alloc(32)
    engine.decode_dev(plan, src, out, olen, ost)
    engine.sync()
    want = [oracle.decompress_status(f)[0] for f in frames]
    assert ost.i32(8) == want
    assert want[3] == 2 and want[5] != 0


def test_pipelined_queues_pinned_host(engine, oracle):
    """Chunks of a batch rotate over 3 queues with pinned host buffers (the end-to-end path):
    H2D, encode, D2H of the frame table and frames; then H2D, decode, D2H. Same bytes as the
    synchronous path, every frame decodes with the oracle."""
    block, n, chunk, nq = 65536, 48, 8, 3
    data = synth.log_text(n * block, 91)
    h_in = engine.host_alloc(len(data))
    h_in.view()[:] = np.frombuffer(data, dtype=np.uint8)
    h_out = engine.host_alloc(len(data))
    qs = [engine.queue() for _ in range(nq)]
    nch = n // chunk
    lanes = []
    for _ in range(nq):
        plan = engine.plan_encode([i * block for i in range(chunk)], [block] * chunk)
        lanes.append(dict(plan=plan, src=engine.alloc(chunk * block), dst=engine.alloc(plan.dst_bound),
                          ioff=engine.alloc(8 * chunk), ilen=engine.alloc(4 * chunk),
                          meta=engine.host_alloc(12 * chunk), out=engine.alloc(chunk * block),
                          olen=engine.alloc(4 * chunk), ost=engine.alloc(4 * chunk)))
    frames = []
    for c in range(nch):
        L, q = lanes[c % nq], qs[c % nq]
        engine.copy_async(L["src"], h_in, chunk * block, 1, q, src_off=c * chunk * block)
        engine.encode_dev(L["plan"], L["src"], L["dst"], L["ioff"], L["ilen"], q)
        engine.copy_async(L["meta"], L["ioff"], 8 * chunk, 2, q)
        engine.copy_async(L["meta"], L["ilen"], 4 * chunk, 2, q, dst_off=8 * chunk)
        q.sync()
        mv = L["meta"].view()
        fo = mv[:8 * chunk].view(np.uint64).tolist()
        fl = mv[8 * chunk:12 * chunk].view(np.uint32).tolist()
        blob = L["dst"].read(fo[-1] + fl[-1])
        for i in range(chunk):
            f = blob[fo[i]:fo[i] + fl[i]]
            assert oracle.decompress_data(f) == data[(c * chunk + i) * block:(c * chunk + i + 1) * block]
        frames.append((blob, fo, fl))
    h_fr = engine.host_alloc(sum(len(b) for b, _, _ in frames))
    hv, pos, dplans, cins = h_fr.view(), 0, [], []
    for blob, fo, fl in frames:
        hv[pos:pos + len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        dplans.append((engine.plan_decode(fo, fl, [i * block for i in range(chunk)], [block] * chunk), pos, len(blob)))
        pos += len(blob)
    for L in lanes:
        cins.append(engine.alloc(chunk * (block + 64)))
    for c in range(nch):
        L, q, cin = lanes[c % nq], qs[c % nq], cins[c % nq]
        dp, hoff, clen = dplans[c]
        engine.copy_async(cin, h_fr, clen, 1, q, src_off=hoff)
        engine.decode_dev(dp, cin, L["out"], L["olen"], L["ost"], q)
        engine.copy_async(h_out, L["out"], chunk * block, 2, q, dst_off=c * chunk * block)
    for q in qs:
        q.sync()
    assert bytes(h_out.view()) == data
    for q in qs:
        q.close()


# ---- CompressionHandler mirror: ports of src/compression.rs unit tests (:607-992)
def _handler(engine, threshold=10, enabled=True):
    import s3hc_lz4 as S

    return S.CompressionHandler(engine, threshold, enabled)


def test_handler_round_trip(engine):
    h = _handler(engine)
    data = b"This is some test data that should be compressed because it's longer than the threshold"
    c = h.compress_with_algorithm(data)
    assert h.decompress_data(c.data) == data


def test_handler_stats_live_across_clones(engine):
    h = _handler(engine)
    clone = h.clone()
    assert clone.get_stats().total_objects_compressed == 0
    h.compress_with_algorithm(b"A" * 100)
    s = clone.get_stats()
    assert s.total_objects_compressed == 1 and s.total_bytes_before == 100
    assert s.total_bytes_after < 100 and s.average_compression_ratio < 1.0


def test_handler_shared_stats(engine):
    import s3hc_lz4 as S

    src = _handler(engine)
    shared = S.CompressionHandler.new_with_shared_stats(20, False, src)
    assert not shared.is_compression_enabled()
    src.compress_with_algorithm(b"A" * 100)
    assert shared.get_stats().total_objects_compressed == 1


def test_handler_decompression_failure_counts(engine):
    import s3hc_lz4 as S

    h = _handler(engine)
    bad = bytes([0x04, 0x22, 0x4D, 0x18, 0xFF, 0xFF, 0xFF, 0xFF, 0x00, 0x01, 0x02])
    assert h.get_stats().decompression_failures == 0
    with pytest.raises(S.CodecError):
        h.decompress_data(bad)
    assert h.get_stats().decompression_failures == 1


def test_handler_compress_with_metadata(engine):
    h = _handler(engine)
    text = b"This is some test data for compression with metadata. " * 10
    r = h.compress_with_metadata(text, "file.txt", True)
    assert r.was_compressed and r.algorithm == 0 and r.original_size == len(text)
    assert r.compressed_size < r.original_size and r.data != text
    jpg = b"This is fake JPEG data that should not be compressed"
    r = h.compress_with_metadata(jpg, "image.jpg", False)
    assert not r.was_compressed and r.algorithm == 0 and r.data != jpg
    assert _handler(engine).decompress_data(r.data) == jpg
    s = h.get_stats()
    assert s.total_objects_compressed == 1 and s.total_objects_uncompressed == 1


def test_handler_corrupt_cache_entry(engine):
    import s3hc_lz4 as S

    h = _handler(engine)
    c = bytearray(h.compress_with_algorithm(b"Some data to compress and then corrupt").data)
    if len(c) > 15:
        c[15] ^= 0xFF
    with pytest.raises(S.CodecError):
        h.decompress_data(bytes(c))


def test_store_mode_corruption_detected(engine, oracle):
    # compression.rs:666-681 (the flipped byte lands in the EndMark word: any error will do)
    import s3hc_lz4 as S

    f = bytearray(engine.store_mode_frame(b"Data that will be corrupted after store-mode encoding"))
    f[len(f) - 6] ^= 0xFF
    with pytest.raises(S.CodecError) as ei:
        _handler(engine).decompress_data(bytes(f))
    assert ei.value.status == oracle.decompress_status(bytes(f))[0]
    g = bytearray(engine.store_mode_frame(b"Data that will be corrupted after store-mode encoding"))
    g[20] ^= 0xFF  # inside the stored payload: content checksum catches it
    with pytest.raises(S.CodecError) as ei:
        _handler(engine).decompress_data(bytes(g))
    assert ei.value.status == S.S3HC_CHECKSUM


def test_tiny_blocks_in_4mib_frame_decode_to_nothing(engine, oracle):
    """13,000 one-byte blocks in a BD 4 MiB frame decode to b"" (an empty frame ends
    decompress_data's loop, so the frame after it is ignored) without reserving 4 MiB per block."""
    import struct
    f = bytes.fromhex("04224d186470b9") + (struct.pack("<I", 1) + b"\x00") * 13_000 + bytes(4) + \
        struct.pack("<I", 0x02CC5D05)
    tail = oracle.lz4flex_compress_frame(b"after the empty frame")
    for blob in (f, f + tail):
        assert oracle.decompress_status(blob) == (0, b"")
        assert engine.decompress_frames(blob) == b""
    h = S.CompressionHandler(engine, 1024, True)
    assert h.decompress_data(f + tail) == b""
    s = engine.stream()  # stream_range_data does not stop at an empty frame
    s.feed(f + tail)
    s.finish()
    got = b""
    while True:
        c = s.read(1 << 20)
        if not c:
            break
        got += c
    assert got == b"after the empty frame"


# ---- compress_with_metadata's error-fallback branches (compression.rs:384-457), reached through
# the handler's test-only fault hook (s3hc_handler_debug_set_faults)
def test_metadata_lz4_failure_falls_back_to_store_mode(engine, oracle):
    h = _handler(engine)
    data = b"log line 42 status=200 bytes=1234\n" * 50
    h.debug_set_faults(h.FAULT_LZ4)
    r = h.compress_with_metadata(data, "file.txt", True)
    # :420-447: compression_failures += 1, a store-mode frame tagged Lz4, was_compressed false
    assert r.algorithm == S.ALG_LZ4 and not r.was_compressed
    assert r.data == oracle.store_mode_frame(data)
    assert r.original_size == len(data) and r.compressed_size == len(r.data)
    s = h.get_stats()
    assert s.compression_failures == 1 and s.total_objects_uncompressed == 0 and s.total_objects_compressed == 0
    h.debug_set_faults(0)
    assert h.decompress_data(r.data) == data


def test_metadata_both_encoders_failing_returns_raw_tagged_lz4(engine):
    h = _handler(engine)
    data = b"abcdefghij" * 30
    h.debug_set_faults(h.FAULT_LZ4 | h.FAULT_STORE)
    r = h.compress_with_metadata(data, "file.txt", True)
    # :448-457 (last resort): raw bytes, still tagged Lz4, uncompressed counter += 1
    assert r.data == data and r.algorithm == S.ALG_LZ4 and not r.was_compressed
    assert r.compressed_size == r.original_size == len(data)
    s = h.get_stats()
    assert s.compression_failures == 1 and s.total_objects_uncompressed == 1


def test_metadata_store_mode_failure_returns_raw_tagged_none(engine):
    h = _handler(engine)
    data = b"\xff\xd8\xff\xe0fake jpeg bytes"
    h.debug_set_faults(h.FAULT_STORE)
    r = h.compress_with_metadata(data, "image.jpg", False)
    # :399-416: raw bytes tagged None, compression_failures and total_objects_uncompressed += 1
    assert r.data == data and r.algorithm == S.ALG_NONE and not r.was_compressed
    assert r.compressed_size == len(data)
    s = h.get_stats()
    assert s.compression_failures == 1 and s.total_objects_uncompressed == 1


def test_decompress_with_algorithm_none_and_decoder_fault(engine):
    h = _handler(engine)
    raw = b"legacy uncompressed cache entry"
    # :594-604: None -> the bytes as stored (to_vec), no decoder involved, no counter touched
    assert h.decompress_with_algorithm(raw, S.ALG_NONE) == raw
    assert h.get_stats().decompression_failures == 0
    frame = h.compress_with_algorithm(raw).data
    h.debug_set_faults(h.FAULT_DECODE)
    with pytest.raises(S.CodecError):
        h.decompress_with_algorithm(frame, S.ALG_LZ4)
    assert h.get_stats().decompression_failures == 1
    assert h.decompress_with_algorithm(raw, S.ALG_NONE) == raw  # the None arm never decodes
    h.debug_set_faults(0)
    assert h.decompress_with_algorithm(frame, S.ALG_LZ4) == raw


def _short_block_frame(oracle, parts, checksum=True):
    """An independent-block BD 64 KiB frame whose non-final blocks are SHORT (valid for
    lz4_flex's FrameDecoder, never written by its encoder): each part is one compressed block."""
    import struct
    flg = 0x64 if checksum else 0x60
    hdr = bytes([0x04, 0x22, 0x4D, 0x18, flg, 0x40])
    hdr += bytes([(oracle.xxh32(hdr[4:6]) >> 8) & 0xFF])
    body = b""
    for p in parts:
        blk = oracle.lz4flex_compress_block(p)
        body += struct.pack("<I", len(blk)) + blk
    tail = struct.pack("<I", 0) + (struct.pack("<I", oracle.xxh32(b"".join(parts))) if checksum else b"")
    return hdr + body + tail


@pytest.mark.parametrize("checksum", [True, False])
def test_short_nonfinal_independent_blocks(engine, oracle, checksum):
    """Host-buffer decode of short non-final independent blocks: the output slots are not
    contiguous on the device, so decode_walk compacts them before the content checksum."""
    parts = [synth.log_text(5000, 61), synth.log_text(65536, 62), synth.log_text(123, 63), synth.log_text(40_000, 64)]
    f = _short_block_frame(oracle, parts, checksum)
    want = b"".join(parts)
    assert oracle.decompress_data(f) == want
    assert engine.decompress_frames(f) == want
    # the same frame between two ordinary frames (delivery order across compaction)
    a, b = synth.log_text(70_000, 65), synth.log_text(3_000, 66)
    blob = engine.compress_frame(a) + f + engine.compress_frame(b)
    assert engine.decompress_frames(blob) == a + want + b
    bad = bytearray(f)
    if checksum:
        bad[-1] ^= 1
        assert engine.decompress_status(bytes(bad))[0] == oracle.decompress_status(bytes(bad))[0]


# ---- host-buffer staging (pinned chunks / direct DMA for pinned caller buffers, one readback)
@pytest.mark.parametrize("mib,policy", [(20, 1), (20, 0), (3, 1)])
def test_host_calls_large_and_pinned_buffers(engine, oracle, mib, policy):
    """Outputs above the 8 MiB readback size go through the chunked pinned staging; pinned
    caller buffers (hipHostMalloc) are copied directly. Same bytes either way."""
    import ctypes

    data = synth.log_text(mib * MiB + 77, 70 + mib)
    frame = engine.compress_frame(data, policy)
    assert oracle.decompress_data(frame) == data
    assert engine.decompress_frames(frame) == data                # pageable output (library-owned)
    assert engine.decompress_frames(frame, len(data) + 5) == data  # pageable caller buffer
    # pinned source and pinned destination through the raw C ABI
    h_in, h_out = engine.host_alloc(len(frame)), engine.host_alloc(len(data) + 64)
    h_in.view()[:] = np.frombuffer(frame, dtype=np.uint8)
    n = ctypes.c_size_t()
    rc = S.lib.s3hc_decompress_frames(engine.h, ctypes.c_void_p(h_in.data_ptr()), len(frame),
                                      ctypes.c_void_p(h_out.data_ptr()), len(data) + 64, ctypes.byref(n))
    assert rc == 0 and n.value == len(data)
    assert bytes(h_out.view()[:len(data)]) == data
    # encode from a pinned source into a pinned destination: the same frame bytes
    h_src = engine.host_alloc(len(data))
    h_src.view()[:] = np.frombuffer(data, dtype=np.uint8)
    cap = S.frame_bound(len(data))
    h_dst = engine.host_alloc(cap)
    wc = ctypes.c_int()
    rc = S.lib.s3hc_compress_frame(engine.h, ctypes.c_void_p(h_src.data_ptr()), len(data), policy,
                                   ctypes.c_void_p(h_dst.data_ptr()), cap, ctypes.byref(n), ctypes.byref(wc))
    assert rc == 0 and bytes(h_dst.view()[:n.value]) == frame
    for h in (h_in, h_out, h_src, h_dst):
        h.free()


def test_encoder_literal_runs_of_every_length(engine, oracle):
    # the emitter copies literal runs of <= 48 bytes as 16-byte chunks (last chunk and last byte
    # first, the record bytes stored after them) and longer runs wave-wide: runs of every length
    # 1..200 between repeated phrases, at every alignment, in single frames and one device batch,
    # decoded by the oracle (decompress_data, compression.rs:463-502)
    import random

    rng = random.Random(2024)
    phrase = b"GET /bucket/key-000042 HTTP/1.1 200 "
    parts = []
    for n in list(range(1, 201)) * 2:
        parts.append(phrase[: 8 + (n % 29)])
        parts.append(rng.randbytes(n))
    data = b"".join(parts)
    for off in (0, 1, 5, 15, 16, 17, 47, 48, 49):
        d = data[off:]
        f = engine.compress_frame(d)
        assert oracle.decompress_data(f) == d, off
        assert engine.decompress_frames(f) == d, off
    blocks = [data[i:i + 65536] for i in range(0, len(data), 65536)]
    blob = b"".join(blocks)
    d_src = engine.upload(blob)
    offs = [i * 65536 for i in range(len(blocks))]
    lens = [len(b) for b in blocks]
    plan = engine.plan_encode(offs, lens)
    dst = engine.alloc(plan.dst_bound)
    ioff, ilen = engine.alloc(8 * len(lens)), engine.alloc(4 * len(lens))
    engine.encode_dev(plan, d_src, dst, ioff, ilen)
    engine.sync()
    fo, fl = ioff.u64(len(lens)), ilen.u32(len(lens))
    raw = dst.read(fo[-1] + fl[-1])
    for k, b in enumerate(blocks):
        assert oracle.decompress_data(raw[fo[k]:fo[k] + fl[k]]) == b, k
