"""Deterministic synthetic corpora for the BASELINE.json configs.

No datasets are fetchable here; these generators produce data of the stated shape:
  log_text  — S3-proxy access-log lines (timestamp, level, request id, method, key, status,
              bytes, latency), fields from fixed vocabularies with Zipf-ish weights.
  json      — JSON records {"id","user","tags","ts","score"}.
  jpeg_like — JFIF header + high-entropy bytes with FF 00 stuffing (ratio ~1.0).

log_text and json come from csrc/s3hc_synth.c (libs3hc_synth.so, host C, multi-threaded):
every line draws its own fields, so no content repeats at any length — a config-5 corpus of
1 M blocks is 1 M distinct blocks. Output depends only on (n, seed).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

SEED_BASE = 0x5EED0001

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libs3hc_synth.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} not built (run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        for fn in (L.s3hc_synth_log_text, L.s3hc_synth_json):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int]
        _LIB = L
    return _LIB


def _gen(fn, n: int, seed: int, threads: int) -> bytes:
    buf = ctypes.create_string_buffer(max(n, 1))
    if fn(buf, n, seed & 0xFFFFFFFFFFFFFFFF, threads) != 0:
        raise RuntimeError("synthetic generator failed")
    return buf.raw[:n]


def log_text(n: int, seed: int = SEED_BASE + 1, threads: int = 0) -> bytes:
    return _gen(_lib().s3hc_synth_log_text, n, seed, threads)


def log_text_into(ptr: int, n: int, seed: int = SEED_BASE + 1, threads: int = 0):
    """Same bytes as log_text(n, seed), written to host memory at ptr (e.g. pinned staging)."""
    if _lib().s3hc_synth_log_text(ctypes.c_void_p(ptr), n, seed & 0xFFFFFFFFFFFFFFFF, threads) != 0:
        raise RuntimeError("synthetic generator failed")


def json_records(n: int, seed: int = SEED_BASE + 2, threads: int = 0) -> bytes:
    return _gen(_lib().s3hc_synth_json, n, seed, threads)


def jpeg_like(n: int, seed: int = SEED_BASE + 3) -> bytes:
    rng = np.random.default_rng(seed)
    body = rng.integers(0, 256, n, dtype=np.uint8)
    # FF 00 byte stuffing as in JPEG entropy-coded segments
    ff = np.flatnonzero(body[:-1] == 0xFF)
    body[ff + 1] = 0
    hdr = bytes([0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10]) + b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    out = bytearray(body.tobytes())
    out[: min(len(hdr), n)] = hdr[: min(len(hdr), n)]
    return bytes(out)


def mixed_blocks(nblocks: int, block: int = 65536, seed: int = SEED_BASE + 3) -> tuple[bytes, list[int]]:
    """Config 3: even blocks JSON (compress), odd blocks JPEG-like (store-mode via denylist)."""
    nj = (nblocks + 1) // 2
    js = np.frombuffer(json_records(nj * block, seed), dtype=np.uint8).reshape(nj, block)
    jp = np.frombuffer(jpeg_like((nblocks // 2) * block, seed + 7), dtype=np.uint8).reshape(nblocks // 2, block)
    out = np.empty((nblocks, block), dtype=np.uint8)
    out[0::2] = js
    out[1::2] = jp
    return out.tobytes(), [i % 2 for i in range(nblocks)]
