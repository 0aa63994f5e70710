"""Deterministic synthetic corpora for the BASELINE.json configs.

No datasets are fetchable here; these generators produce data of the stated shape:
  log_text  — S3-proxy access-log lines (timestamp, level, request id, method, key, status,
              bytes, latency), fields from fixed vocabularies with Zipf-ish weights.
  json      — JSON records {"id","user","tags","ts","score"}.
  jpeg_like — JFIF header + high-entropy bytes with FF 00 stuffing (ratio ~1.0).
Period-tiling beyond 8 MiB is invisible to LZ4 (window 64 KiB, blocks independent).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x5EED0001

_LEVELS = ["INFO"] * 12 + ["DEBUG"] * 5 + ["WARN"] * 2 + ["ERROR"]
_METHODS = ["GET"] * 14 + ["HEAD"] * 3 + ["PUT"] * 2 + ["DELETE"]
_BUCKETS = ["datalake-prod", "ml-training", "logs-archive", "media-assets", "backup-east"]
_PREFIX = ["2024/01/", "2024/02/", "raw/", "curated/parquet/", "images/thumbs/", "models/ckpt/", "events/"]
_EXT = [".parquet", ".json", ".csv", ".jpg", ".bin", ".log", ".gz", ".txt"]
_STATUS = ["200"] * 20 + ["206"] * 6 + ["304"] * 3 + ["404", "403", "500", "503"]
_USERS = ["alice", "bob", "carol", "dave", "erin", "frank", "grace", "heidi", "ivan", "judy"]
_TAGS = ["hot", "cold", "archive", "pii", "public", "ml", "etl", "raw", "gold", "silver"]


def _fill(gen_chunk, n: int, period: int = 8 << 20) -> bytes:
    base = bytearray()
    while len(base) < min(n, period):
        base += gen_chunk()
    base = bytes(base[: min(n, period)])
    if n <= len(base):
        return base[:n]
    reps = -(-n // len(base))
    return (base * reps)[:n]


def log_text(n: int, seed: int = SEED_BASE + 1) -> bytes:
    rng = np.random.default_rng(seed)
    t0 = [1704067200]

    def chunk():
        m = 4096
        lv = rng.integers(0, len(_LEVELS), m)
        me = rng.integers(0, len(_METHODS), m)
        bu = rng.zipf(1.6, m) % len(_BUCKETS)
        pr = rng.zipf(1.4, m) % len(_PREFIX)
        ex = rng.integers(0, len(_EXT), m)
        st = rng.integers(0, len(_STATUS), m)
        rid = rng.integers(0, 1 << 63, m, dtype=np.int64)
        key = rng.zipf(1.3, m) % 5000
        by = rng.integers(0, 1 << 26, m)
        la = rng.gamma(2.0, 12.0, m).astype(np.int64)
        dt = rng.integers(0, 3, m)
        out = []
        for i in range(m):
            t0[0] += int(dt[i])
            t = t0[0]
            ss, mm_, hh = t % 60, (t // 60) % 60, (t // 3600) % 24
            out.append(
                f"2024-01-{1 + (t // 86400) % 28:02d}T{hh:02d}:{mm_:02d}:{ss:02d}Z {_LEVELS[lv[i]]} "
                f"[req-{int(rid[i]) & 0xFFFFFFFFFFFFFFFF:016x}] {_METHODS[me[i]]} /{_BUCKETS[bu[i]]}/"
                f"{_PREFIX[pr[i]]}part-{int(key[i]):05d}{_EXT[ex[i]]} status={_STATUS[st[i]]} "
                f"bytes={int(by[i])} latency_ms={int(la[i])}\n"
            )
        return "".join(out).encode()

    return _fill(chunk, n)


def json_records(n: int, seed: int = SEED_BASE + 2) -> bytes:
    rng = np.random.default_rng(seed)
    nid = [0]

    def chunk():
        m = 4096
        us = rng.zipf(1.5, m) % len(_USERS)
        nt = rng.integers(0, 4, m)
        tg = rng.integers(0, len(_TAGS), (m, 3))
        ts = rng.integers(1704067200, 1735689600, m)
        sc = rng.random(m)
        out = []
        for i in range(m):
            nid[0] += 1
            tags = ",".join(f'"{_TAGS[tg[i, j]]}"' for j in range(int(nt[i])))
            out.append(
                f'{{"id":{nid[0]},"user":"{_USERS[us[i]]}","tags":[{tags}],"ts":{int(ts[i])},'
                f'"score":{sc[i]:.6f}}}\n'
            )
        return "".join(out).encode()

    return _fill(chunk, n)


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
    js = json_records(nj * block, seed)
    jp = jpeg_like((nblocks // 2) * block, seed + 7)
    parts, modes = [], []
    for i in range(nblocks):
        k = i // 2
        if i % 2 == 0:
            parts.append(js[k * block:(k + 1) * block])
            modes.append(0)
        else:
            parts.append(jp[k * block:(k + 1) * block])
            modes.append(1)
    return b"".join(parts), modes
