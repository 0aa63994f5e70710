"""CPU-side checks of the product library: it builds, loads, exports every symbol the C
header declares, and fails loudly (S3HC_DEVICE) without a GPU instead of falling back."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("s3hc_lz4.h", "s3hc_lz4_diag.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(s3hc_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_header_symbols():
    import s3hc_lz4 as S

    lib = ctypes.CDLL(S.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_no_oracle_in_product():
    import s3hc_lz4 as S

    data = open(S.LIB_PATH, "rb").read()
    assert b"or_decompress_data" not in data and b"lz4_oracle" not in data


def test_create_without_gpu_fails_loudly():
    import s3hc_lz4 as S

    h = ctypes.c_void_p()
    rc = S.lib.s3hc_create(ctypes.byref(h), 0)
    if rc == S.S3HC_OK:
        S.lib.s3hc_destroy(h)
        pytest.skip("a GPU is present")
    assert rc == S.S3HC_DEVICE
    assert b"no HIP device" in S.lib.s3hc_last_error()


@pytest.mark.parametrize("path,want", [
    ("file.txt", False), ("path/to/file.json", False), ("bucket/folder/image.jpg", True), ("file.tar.gz", True),
    ("noextension", False), ("", False), ("bucket/images/photo.JPG", True), ("deep/nested/path/archive.zip", True),
    ("clip.mp4", True), ("doc.pdf", True), ("index.html", False), ("x.woff2", True), ("a.db", True),
])
def test_denylist(path, want):
    # compression.rs:750-846 (extension extraction + denylist)
    import s3hc_lz4 as S

    assert S.is_denylisted_extension(path) is want


def test_decompressed_bound_host_walk(oracle):
    import s3hc_lz4 as S

    for data in (b"", b"x" * 10, bytes(i % 251 for i in range(300_000))):
        f = oracle.lz4flex_compress_frame(data) + oracle.store_mode_frame(data)
        b = ctypes.c_size_t()
        assert S.lib.s3hc_decompressed_bound(f, len(f), ctypes.byref(b)) == 0
        assert b.value >= 2 * len(data)
        assert b.value <= oracle.decompressed_bound(f)  # slots: min(block max, 255 x compressed size)


def _tiny_block_frame(nblocks):
    """BD 0x70 (4 MiB blocks) frame of nblocks 1-byte compressed blocks that decode to nothing
    (token 0x00: an empty last sequence), EndMark, xxh32("")."""
    import struct
    return bytes.fromhex("04224d186470b9") + (struct.pack("<I", 1) + b"\x00") * nblocks + bytes(4) + \
        struct.pack("<I", 0x02CC5D05)


def test_decompressed_bound_tiny_blocks_not_block_max(oracle):
    """a 4 MiB-BD frame of tiny blocks must not reserve 4 MiB per block."""
    import s3hc_lz4 as S

    f = _tiny_block_frame(13_000)
    assert oracle.decompress_data(f) == b""
    b = ctypes.c_size_t()
    assert S.lib.s3hc_decompressed_bound(f, len(f), ctypes.byref(b)) == 0
    assert b.value <= 255 * len(f)
    assert oracle.decompressed_bound(f) >= 13_000 * (4 << 20)  # what per-block-max sizing would reserve


def test_frame_bound():
    import s3hc_lz4 as S

    for n in (0, 1, 65535, 65536, 65537, 1 << 20, 5 << 20):
        assert S.frame_bound(n) >= n + 4 * (n // 65536 + 1) + 15


def test_knobs_set_and_reject_unknown():
    # diagnostic switches are read from the environment once per process and changed only
    # through s3hc_set_knob; unknown names are rejected (no GPU needed)
    import s3hc_lz4 as S

    for name, value in (("S3HC_FAST_DISABLE", "1"), ("S3HC_FAST", "0"), ("S3HC_LBW_CAP", "4096"),
                        ("S3HC_LBW_ROUNDS", "2"), ("S3HC_HOST_TRACE", None), ("S3HC_READER_SLOTS", "1")):
        S.set_knob(name, value)
        S.set_knob(name, None)
    with pytest.raises(S.CodecError):
        S.set_knob("S3HC_NO_SUCH_KNOB", "1")
    with S.knobs({"S3HC_LB_DISABLE": "1", "S3HC_FAST": "1"}):
        pass


def test_knobs_restore_exact_values_with_aliases():
    # S3HC_FAST and S3HC_FAST_DISABLE share one slot; the context manager restores the
    # values on entry, whatever the order and the environment
    import s3hc_lz4 as S

    S.set_knob("S3HC_FAST", "0")  # fast path off (S3HC_FAST_DISABLE's slot = 1)
    try:
        assert S.get_knob("S3HC_FAST_DISABLE") == 1 and S.get_knob("S3HC_FAST") == 1
        with S.knobs({"S3HC_FAST": "1", "S3HC_FAST_DISABLE": None, "S3HC_POISON": "1"}):
            assert S.get_knob("S3HC_FAST_DISABLE") == 0
            assert S.get_knob("S3HC_POISON") == 1
        assert S.get_knob("S3HC_FAST_DISABLE") == 1
        assert S.get_knob("S3HC_POISON") == 0
    finally:
        S.set_knob("S3HC_FAST_DISABLE", None)
    assert S.get_knob("S3HC_FAST_DISABLE") == 0
    with pytest.raises(S.CodecError):
        S.get_knob("S3HC_NO_SUCH_KNOB")


def test_reader_result_check_rejects_forged_results():
    # device-written frame lengths and statuses are checked on the host before
    # they drive a device-to-host copy (the reader's s3hc_reader_* path; pure host code)
    import s3hc_lz4 as S

    off = [0, 65536, 131072, 196608]
    slot = 262144
    assert S.check_batch_results([65536, 65536, 65536, 100], [0, 0, 0, 0], off, slot) == (4, 196708)
    assert S.check_batch_results([65536, 7, 0, 0], [0, 2, 0, 0], off, slot) == (1, 65536)  # CHECKSUM at frame 1
    assert S.check_batch_results([], [], [], 0) == (0, 0)
    assert S.check_batch_results([65536, 65536, 65536, 65536], [0] * 4, off, slot) == (4, slot)
    for olen, st in (([65537, 0, 0, 0], [0] * 4),              # longer than its slot
                     ([0, 0, 0, 65537], [0] * 4),              # the last frame past the batch's slots
                     ([0xFFFFFFFF, 0, 0, 0], [0] * 4),         # poison-filled length
                     ([0, 0, 0, 0], [0, -1, 0, 0]),            # poison-filled status (0xFFFFFFFF)
                     ([0, 0, 0, 0], [0, 0, 7, 0])):            # a status no decoder assigns
        with pytest.raises(S.CodecError) as e:
            S.check_batch_results(olen, st, off, slot)
        assert e.value.status == S.S3HC_DEVICE
    # lengths after the first failing frame are not the decode's business: never read
    assert S.check_batch_results([10, 0xFFFFFFFF, 0xFFFFFFFF, 0], [0, 1, -1, 9], off, slot) == (1, 10)


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_shard_items_contiguous_balanced(ndev):
    # the multi-device aggregator's shards (host logic, no GPU)
    import random

    import s3hc_lz4 as S

    rng = random.Random(ndev)
    for n in (0, 1, ndev - 1, ndev, ndev + 1, 17, 300):
        if n < 0:
            continue
        lens = [rng.choice((0, 1, 65536, 1 << 20, rng.randrange(1, 3 << 20))) for _ in range(n)]
        f = S.shard_items(lens, ndev)
        assert len(f) == ndev + 1 and f[0] == 0 and f[-1] == n
        assert all(a <= b for a, b in zip(f, f[1:]))  # contiguous, in order
        if n >= ndev:
            assert all(a < b for a, b in zip(f, f[1:]))  # every device gets work
        total = sum(lens)
        if n >= ndev and total:
            big = max(lens)
            for d in range(ndev):
                assert sum(lens[f[d]:f[d + 1]]) <= total / ndev + 2 * big  # about equal bytes
    # equal items split evenly
    assert S.shard_items([10] * 8, 4) == [0, 2, 4, 6, 8]
    f = S.shard_items([10] * 3, 4)  # fewer items than devices: one item per used device
    assert sum(b - a for a, b in zip(f, f[1:])) == 3 and all(b - a <= 1 for a, b in zip(f, f[1:]))
    with pytest.raises(S.CodecError):
        S.shard_items([1, 2], 0)
