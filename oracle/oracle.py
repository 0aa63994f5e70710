"""ctypes wrapper for the CPU parity oracle (oracle/lz4_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liblz4_oracle.so")
_lib = None

OK, CORRUPT, CHECKSUM, DST_TOO_SMALL, UNSUPPORTED, INVALID_ARG = 0, 1, 2, 3, 4, 6


class OracleError(Exception):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: status {status}")
        self.status = status


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p, sz, szp = ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)
        L.or_xxh32.argtypes = [u8p, sz, ctypes.c_uint32]
        L.or_xxh32.restype = ctypes.c_uint32
        L.or_frame_bound.argtypes = [sz]
        L.or_frame_bound.restype = sz
        for f in ("or_store_mode_frame", "or_lz4flex_compress_frame", "or_decompress_data", "or_decode_block"):
            getattr(L, f).argtypes = [u8p, sz, u8p, sz, szp]
            getattr(L, f).restype = ctypes.c_int
        L.or_lz4flex_compress_block.argtypes = [u8p, sz, u8p, sz]
        L.or_lz4flex_compress_block.restype = sz
        L.or_decompressed_bound.argtypes = [u8p, sz]
        L.or_decompressed_bound.restype = sz
        _lib = L
    return _lib


def _buf(data):
    b = bytes(data)
    return b, ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)


def xxh32(data, seed: int = 0) -> int:
    b, p = _buf(data)
    return lib().or_xxh32(p, len(b), seed)


def _frame_call(fn, data, cap):
    b, p = _buf(data)
    out = ctypes.create_string_buffer(max(cap, 1))
    n = ctypes.c_size_t(0)
    rc = fn(p, len(b), out, cap, ctypes.byref(n))
    if rc != OK:
        raise OracleError(rc, fn.__name__)
    return out.raw[: n.value]


def store_mode_frame(data) -> bytes:
    """compression.rs:326-368 encode_store_mode_frame."""
    return _frame_call(lib().or_store_mode_frame, data, lib().or_frame_bound(len(data)))


def lz4flex_compress_frame(data) -> bytes:
    """compression.rs:530-591 compress_with_algorithm(Lz4) -> lz4_flex FrameEncoder."""
    return _frame_call(lib().or_lz4flex_compress_frame, data, lib().or_frame_bound(len(data)))


def lz4flex_compress_block(data) -> bytes:
    b, p = _buf(data)
    cap = len(b) + len(b) // 2 + 64
    out = ctypes.create_string_buffer(cap)
    n = lib().or_lz4flex_compress_block(p, len(b), out, cap)
    return out.raw[:n]


def decompressed_bound(data) -> int:
    b, p = _buf(data)
    return lib().or_decompressed_bound(p, len(b))


def decompress_data(data, cap: int | None = None) -> bytes:
    """compression.rs:463-502 decompress_data (concatenated frames)."""
    if cap is None:
        # no LZ4 block decodes to more than 255 bytes per compressed byte
        cap = min(decompressed_bound(data), 255 * len(data) + 64)
    return _frame_call(lib().or_decompress_data, data, cap)


def decompress_status(data, cap: int | None = None) -> tuple[int, bytes]:
    try:
        return OK, decompress_data(data, cap)
    except OracleError as e:
        return e.status, b""


def _without_content_checksum(frame: bytes) -> bytes | None:
    """The frame with its content-checksum flag cleared (the FLG bit, the header checksum byte
    recomputed, the trailing 4 checksum bytes dropped), or None when it has no such checksum."""
    b = bytes(frame)
    if len(b) < 7 + 4 or b[:4] != b"\x04\x22\x4d\x18" or not b[4] & 0x04:
        return None
    flg = b[4] & ~0x04
    desc = 2 + (8 if flg & 0x08 else 0) + (4 if flg & 0x01 else 0)
    d = bytes([flg]) + b[5:4 + desc]
    return b[:4] + d + bytes([(xxh32(d) >> 8) & 0xFF]) + b[4 + desc + 1:-4]


def stream_range_data(frames) -> tuple[int, bytes]:
    """disk_cache.rs:3850-3935 stream_range_data over a list of whole frames: one lz4_flex
    FrameDecoder per frame, its bytes sent as they decode, the first error ending the stream
    (:3893-3898); an empty frame does not end it (Ok(0) ends only the inner loop, :3880-3882).
    lz4_flex's FrameDecoder checks the content checksum at the EndMark, after the frame's bytes
    were returned, so a frame whose only fault is its content checksum is delivered whole before
    S3HC_CHECKSUM. Any other fault of a frame delivers none of its bytes (restated frame by frame:
    for a later block of a multi-block frame lz4_flex would have returned the earlier blocks
    first; the test streams use single-block frames for that case). Returns (status, bytes)."""
    out = bytearray()
    for f in frames:
        st, b = decompress_status(f)
        if st == OK:
            out += b
            continue
        if st == CHECKSUM:
            g = _without_content_checksum(f)
            if g is not None:
                st2, b2 = decompress_status(g)
                if st2 == OK and xxh32(b2) != int.from_bytes(bytes(f)[-4:], "little"):
                    out += b2
        return st, bytes(out)
    return OK, bytes(out)


def decode_block(data, cap: int) -> bytes:
    return _frame_call(lib().or_decode_block, data, cap)
