"""CPU tests of the parity oracle (oracle/lz4_oracle.c), the restatement of the reference path.

The oracle is pinned by: python xxhash (XXH32 known answers), the reference's byte layout of
store-mode frames (golden fixtures), liblz4 decoding every frame the oracle writes and the
oracle decoding liblz4's frames, and ports of the reference's own tests
(src/compression.rs:607-992, tests/lz4_roundtrip_preservation_test.rs)."""
import os
import random

import numpy as np
import pytest
import xxhash
from hypothesis import given, settings, strategies as st

import lz4ref


def test_xxh32_known_answers(oracle):
    assert oracle.xxh32(b"") == 0x02CC5D05
    rng = random.Random(3)
    for n in list(range(0, 70)) + [255, 256, 1000, 4096, 65535, 65536, 65537, 100_003]:
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.xxh32(d) == xxhash.xxh32(d).intdigest(), n


def test_header_checksums(oracle):
    # HC for FLG 0x64 with BD 0x40/0x50/0x70 = 0xA7/0x08/0xB9
    for bd, hc in ((0x40, 0xA7), (0x50, 0x08), (0x70, 0xB9)):
        assert (oracle.xxh32(bytes([0x64, bd])) >> 8) & 0xFF == hc


def test_empty_store_mode_frame(oracle):
    # empty input -> 15 bytes 04224d186470b900000000055dcc02
    assert oracle.store_mode_frame(b"").hex() == "04224d186470b900000000055dcc02"


@pytest.mark.parametrize("n,bd", [(0, 0x40), (1, 0x40), (65536, 0x40), (65537, 0x50), (262144, 0x50),
                                  (262145, 0x70), (1 << 20, 0x70)])
def test_lz4flex_auto_block_size(oracle, n, bd):
    # lz4_flex BlockSize::from_buf_length
    f = oracle.lz4flex_compress_frame(bytes(i % 251 for i in range(n)))
    assert f[:5] == bytes([0x04, 0x22, 0x4D, 0x18, 0x64]) and f[5] == bd


def test_incompressible_block_is_stored(oracle):
    data = os.urandom(65536)
    f = oracle.lz4flex_compress_frame(data)
    assert int.from_bytes(f[7:11], "little") == (65536 | 0x80000000)
    assert oracle.decompress_data(f) == data


@pytest.mark.skipif(not lz4ref.available, reason="liblz4 not present")
@pytest.mark.parametrize("n", [0, 1, 13, 63, 64, 1024, 65536, 65537, 300_000, (1 << 20) + 1, 5 << 20])
def test_liblz4_decodes_oracle_frames(oracle, n):
    data = bytes(i % 251 for i in range(n))
    assert lz4ref.decompress(oracle.lz4flex_compress_frame(data), max(n, 1)) == data
    assert lz4ref.decompress(oracle.store_mode_frame(data), max(n, 1)) == data


@pytest.mark.skipif(not lz4ref.available, reason="liblz4 not present")
@pytest.mark.parametrize("bsid", [4, 5, 6, 7])
@pytest.mark.parametrize("linked", [False, True])
def test_oracle_decodes_liblz4_frames(oracle, bsid, linked):
    rng = np.random.default_rng(bsid)
    words = [b"alpha", b"beta", b"gamma", b"delta", b"status=200 ", b"GET /bucket/key "]
    data = b"".join(words[i] for i in rng.integers(0, len(words), 60_000))
    for cc, bc, cs in ((True, False, False), (True, True, True), (False, False, True)):
        f = lz4ref.compress_frame(data, bsid, linked, cc, bc, cs)
        assert oracle.decompress_data(f) == data


@settings(max_examples=150, deadline=None)
@given(st.binary(min_size=0, max_size=3000))
def test_roundtrip_property(oracle, data):
    # tests/lz4_roundtrip_preservation_test.rs:48-82: decompress(compress(x)) == x
    assert oracle.decompress_data(oracle.lz4flex_compress_frame(data)) == data
    assert oracle.decompress_data(oracle.store_mode_frame(data)) == data


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.binary(min_size=0, max_size=400), st.booleans()), min_size=1, max_size=8))
def test_concatenated_frames_property(oracle, chunks):
    # tests/lz4_roundtrip_preservation_test.rs:129-180: alternating store/compressed frames
    blob = b"".join(oracle.store_mode_frame(c) if s else oracle.lz4flex_compress_frame(c) for c, s in chunks)
    want = b""
    for c, _ in chunks:
        if not c:  # a frame that yields no bytes ends the decompress_data loop (compression.rs:481)
            break
        want += c
    assert oracle.decompress_data(blob) == want


def test_corrupt_inputs(oracle):
    # compression.rs:738-747 and :911-957
    assert oracle.decompress_status(bytes([0x04, 0x22, 0x4D, 0x18, 0xFF, 0xFF, 0xFF, 0xFF, 0, 1, 2]))[0] != 0
    f = bytearray(oracle.lz4flex_compress_frame(b"Some data to compress and then corrupt"))
    f[15] ^= 0xFF
    assert oracle.decompress_status(bytes(f))[0] != 0
    g = bytearray(oracle.store_mode_frame(b"Data that will be corrupted after store-mode encoding"))
    g[len(g) - 6] ^= 0xFF
    assert oracle.decompress_status(bytes(g))[0] != 0


def test_mixed_frames(oracle):
    # compression.rs:684-700
    a = oracle.lz4flex_compress_frame(b"A" * 200)
    b = oracle.store_mode_frame(b"incompressible-ish chunk")
    assert oracle.decompress_data(a + b) == b"A" * 200 + b"incompressible-ish chunk"
    assert len(oracle.lz4flex_compress_frame(b"A" * 200)) < len(oracle.store_mode_frame(b"A" * 200))


def test_stream_range_data_delivers_frame_before_checksum_error(oracle):
    # disk_cache.rs:3884-3898: FrameDecoder::read returns a frame's bytes before the EndMark's
    # content checksum is compared, so stream_range_data sends them, then the error chunk
    data = bytes(range(256)) * 1000
    fr = [bytearray(oracle.lz4flex_compress_frame(data[i:i + 65536])) for i in range(0, len(data), 65536)]
    assert oracle.stream_range_data([bytes(f) for f in fr]) == (0, data)
    bad = [bytearray(f) for f in fr]
    bad[2][-1] ^= 0x01
    assert oracle.stream_range_data([bytes(f) for f in bad]) == (oracle.CHECKSUM, data[:3 * 65536])
    # the same frame without its content checksum (header checksum recomputed) decodes on liblz4
    g = oracle._without_content_checksum(bytes(bad[2]))
    assert g[4] & 0x04 == 0 and len(g) == len(bad[2]) - 4
    if lz4ref.available:
        assert lz4ref.decompress(g, 65536) == data[2 * 65536:3 * 65536]
    # a structural fault (block size word) delivers nothing of its frame
    bad = [bytearray(f) for f in fr]
    bad[1][9] ^= 0xFF
    st, out = oracle.stream_range_data([bytes(f) for f in bad])
    assert st != 0 and out == data[:65536]
    # an empty frame does not end the stream (Ok(0) ends only the inner loop)
    e = oracle.lz4flex_compress_frame(b"")
    assert oracle.stream_range_data([bytes(fr[0]), e, bytes(fr[1])]) == (0, data[:2 * 65536])
