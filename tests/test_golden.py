"""Committed golden fixtures (tests/golden/, made by make_golden.py) against the oracle (CPU)
and against the GPU engine (gpu). Store-mode frames are pinned to the reference's byte layout
(compression.rs:326-368); liblz4-written frames are cross-implementation decode vectors."""
import hashlib
import json
import os

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(HERE, "manifest.json")))["cases"]


def _input(case):
    i = case["input"]
    if i["kind"] == "p251":
        return bytes(k % 251 for k in range(i["value"]))
    return bytes.fromhex(i["value"])


def _blob(case):
    for key in ("frame_hex", "blob_hex"):
        if key in case:
            return bytes.fromhex(case[key])
    with open(os.path.join(HERE, case["file"]), "rb") as fh:
        return fh.read()


def _sha(b):
    return hashlib.sha256(b).hexdigest()


IDS = [c["name"] for c in MANIFEST]


@pytest.mark.parametrize("case", MANIFEST, ids=IDS)
def test_oracle_matches_golden(oracle, case):
    kind = case["kind"]
    if kind == "store_mode":
        f = oracle.store_mode_frame(_input(case))
        assert len(f) == case["frame_len"] and _sha(f) == case["frame_sha256"]
        assert _sha(oracle.decompress_data(f)) == case["plain_sha256"]
    elif kind == "lz4flex_frame":
        assert oracle.lz4flex_compress_frame(_input(case)) == _blob(case)
    elif kind in ("decode", "corrupt"):
        st, out = oracle.decompress_status(_blob(case))
        assert st == case["expect_status"]
        if st == 0:
            assert len(out) == case["plain_len"] and _sha(out) == case["plain_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST, ids=IDS)
def test_gpu_matches_golden(engine, case):
    kind = case["kind"]
    if kind == "store_mode":
        f = engine.store_mode_frame(_input(case))
        assert len(f) == case["frame_len"] and _sha(f) == case["frame_sha256"]
        assert _sha(engine.decompress_frames(f)) == case["plain_sha256"]
    elif kind == "lz4flex_frame":
        assert engine.compress_frame(_input(case)) == _blob(case)
    elif kind in ("decode", "corrupt"):
        st, out = engine.decompress_status(_blob(case))
        assert st == case["expect_status"]
        if st == 0:
            assert len(out) == case["plain_len"] and _sha(out) == case["plain_sha256"]
