"""liblz4 1.9.3 (system library, third-party C LZ4 — not the reference codec) via ctypes.

Used only as an independent cross-check: frames written by our engine must decode with
LZ4F_decompress, and frames written by LZ4F_compressFrame (a different encoder) must decode
with our engine. Tests skip these checks when the library is absent.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os

_CANDIDATES = ["/usr/lib/x86_64-linux-gnu/liblz4.so.1", "/opt/conda/lib/liblz4.so.1", ctypes.util.find_library("lz4")]
_lib = None
for c in _CANDIDATES:
    if c and os.path.exists(c):
        try:
            _lib = ctypes.CDLL(c)
            break
        except OSError:
            pass

available = _lib is not None


class _FramePrefs(ctypes.Structure):
    _fields_ = [
        ("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int), ("contentChecksumFlag", ctypes.c_int),
        ("frameType", ctypes.c_int), ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
        ("blockChecksumFlag", ctypes.c_int),
    ]


class _Prefs(ctypes.Structure):
    _fields_ = [("frameInfo", _FramePrefs), ("compressionLevel", ctypes.c_int), ("autoFlush", ctypes.c_uint),
                ("favorDecSpeed", ctypes.c_uint), ("reserved", ctypes.c_uint * 3)]


if available:
    _lib.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    _lib.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.c_void_p]
    _lib.LZ4F_compressFrame.restype = ctypes.c_size_t
    _lib.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
    _lib.LZ4F_isError.restype = ctypes.c_uint
    _lib.LZ4F_isError.argtypes = [ctypes.c_size_t]
    _lib.LZ4F_createDecompressionContext.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    _lib.LZ4F_freeDecompressionContext.argtypes = [ctypes.c_void_p]
    _lib.LZ4F_decompress.restype = ctypes.c_size_t
    _lib.LZ4F_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]


def compress_frame(data: bytes, block_size_id: int = 4, linked: bool = False, content_checksum: bool = True,
                   block_checksum: bool = False, content_size: bool = False, level: int = 0) -> bytes:
    p = _Prefs()
    p.frameInfo.blockSizeID = block_size_id
    p.frameInfo.blockMode = 0 if linked else 1
    p.frameInfo.contentChecksumFlag = 1 if content_checksum else 0
    p.frameInfo.blockChecksumFlag = 1 if block_checksum else 0
    p.frameInfo.contentSize = len(data) if content_size else 0
    p.compressionLevel = level
    cap = _lib.LZ4F_compressFrameBound(len(data), ctypes.byref(p)) + 64
    out = ctypes.create_string_buffer(cap)
    n = _lib.LZ4F_compressFrame(out, cap, data, len(data), ctypes.byref(p))
    assert not _lib.LZ4F_isError(n)
    return out.raw[:n]


def decompress(frames: bytes, max_out: int) -> bytes:
    """Decode concatenated frames; raises ValueError on any liblz4 error."""
    ctx = ctypes.c_void_p()
    assert _lib.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100) == 0
    try:
        out = ctypes.create_string_buffer(max(max_out, 1) + 64)
        res = bytearray()
        pos = 0
        while pos < len(frames):
            dsz = ctypes.c_size_t(max(max_out, 1) + 64)
            ssz = ctypes.c_size_t(len(frames) - pos)
            r = _lib.LZ4F_decompress(ctx, out, ctypes.byref(dsz), frames[pos:], ctypes.byref(ssz), None)
            if _lib.LZ4F_isError(r):
                raise ValueError("liblz4 decode error")
            res += out.raw[: dsz.value]
            pos += ssz.value
            if ssz.value == 0 and dsz.value == 0:
                raise ValueError("liblz4 made no progress")
        return bytes(res)
    finally:
        _lib.LZ4F_freeDecompressionContext(ctx)
