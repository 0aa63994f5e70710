"""Python binding of libs3hc_lz4.so (the MI355X LZ4 frame engine) over its C ABI.

Mirrors the reference's codec surface (src/compression.rs): ``CompressionHandler`` with
``compress_with_metadata`` / ``compress_with_algorithm`` / ``decompress_data`` /
``decompress_with_algorithm`` / ``encode_store_mode_frame`` / ``get_stats`` and
``is_denylisted_extension``, plus the device-resident batch API used by bench.py.

There is no CPU fallback: if the shared library is missing this module raises at import
time, and if no HIP device is present ``Engine()`` raises ``CodecError(S3HC_DEVICE)``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("S3HC_LIB_PATH") or os.path.join(_HERE, "libs3hc_lz4.so")  # override: diagnostic builds only

S3HC_OK, S3HC_CORRUPT, S3HC_CHECKSUM, S3HC_DST_TOO_SMALL = 0, 1, 2, 3
S3HC_UNSUPPORTED, S3HC_DEVICE, S3HC_INVALID_ARG = 4, 5, 6
STATUS_NAMES = {0: "OK", 1: "CORRUPT", 2: "CHECKSUM", 3: "DST_TOO_SMALL", 4: "UNSUPPORTED", 5: "DEVICE", 6: "INVALID_ARG"}
BLK_AUTO_LZ4FLEX, BLK_64K_PER_FRAME, BLK_LZ4FLEX_COMPAT = 0, 1, 2
ENC_FAST, ENC_SMALL = 0, 1  # match-finder modes (s3hc_set_encode_mode)
ALG_LZ4, ALG_NONE = 0, 1


class CodecError(Exception):
    """ProxyError::CompressionError equivalent (src/error.rs:22-23)."""

    def __init__(self, status: int, message: str = ""):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE, "-j4"], check=True)
    return LIB_PATH


def _q(stream):
    """Queue, raw hipStream_t pointer value, or None (the context stream)."""
    return getattr(stream, "q", stream)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built (run __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p
    szp, ip = ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)
    u64, u32, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "s3hc_create": (i32, [ctypes.POINTER(vp), i32]),
        "s3hc_destroy": (None, [vp]),
        "s3hc_device_count": (i32, []),
        "s3hc_last_error": (ctypes.c_char_p, []),
        "s3hc_version": (ctypes.c_char_p, []),
        "s3hc_set_knob": (i32, [ctypes.c_char_p, ctypes.c_char_p]),
        "s3hc_get_knob": (i32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)]),
        "s3hc_set_knob_value": (i32, [ctypes.c_char_p, ctypes.c_longlong]),
        "s3hc_diag_check_batch_results": (i32, [u32, vp, vp, vp, u64, ctypes.POINTER(u32), ctypes.POINTER(u64)]),
        "s3hc_frame_bound": (sz, [sz]),
        "s3hc_compat_encode_dev": (i32, [vp, vp, vp, vp, u32, vp, vp, vp, vp]),
        "s3hc_compress_frame": (i32, [vp, u8p, sz, i32, u8p, sz, szp, ip]),
        "s3hc_store_mode_frame": (i32, [vp, u8p, sz, u8p, sz, szp]),
        "s3hc_decompressed_bound": (i32, [u8p, sz, szp]),
        "s3hc_decompress_frames": (i32, [vp, u8p, sz, u8p, sz, szp]),
        "s3hc_decompress_frames_alloc": (i32, [vp, u8p, sz, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), szp]),
        "s3hc_buffer_free": (None, [ctypes.POINTER(ctypes.c_uint8)]),
        "s3hc_stream_open": (i32, [vp, ctypes.POINTER(vp)]),
        "s3hc_stream_feed": (i32, [vp, u8p, sz]),
        "s3hc_stream_finish": (i32, [vp]),
        "s3hc_stream_read": (i32, [vp, u8p, sz, szp]),
        "s3hc_stream_total": (u64, [vp]),
        "s3hc_stream_close": (None, [vp]),
        "s3hc_plan_encode": (i32, [vp, vp, vp, vp, u32, ctypes.POINTER(vp)]),
        "s3hc_encode_dev": (i32, [vp, vp, vp, vp, u64, vp, vp, vp]),
        "s3hc_plan_dst_bound": (u64, [vp]),
        "s3hc_plan_decode": (i32, [vp, vp, vp, vp, vp, u32, ctypes.POINTER(vp)]),
        "s3hc_decode_dev": (i32, [vp, vp, vp, vp, vp, vp, vp]),
        "s3hc_plan_free": (None, [vp]),
        "s3hc_last_kernel_ms": (ctypes.c_float, [vp, ctypes.c_char_p]),
        "s3hc_set_timing": (None, [vp, i32]),
        "s3hc_set_encode_mode": (i32, [vp, i32]),
        "s3hc_get_encode_mode": (i32, [vp]),
        "s3hc_timing_collect": (i32, [vp]),
        "s3hc_timing_reset": (None, [vp]),
        "s3hc_kernel_count": (i32, [vp, ctypes.c_char_p]),
        "s3hc_handler_new": (vp, [vp, sz, i32]),
        "s3hc_handler_new_with_shared_stats": (vp, [sz, i32, vp]),
        "s3hc_handler_clone": (vp, [vp]),
        "s3hc_handler_free": (None, [vp]),
        "s3hc_handler_is_compression_enabled": (i32, [vp]),
        "s3hc_handler_compress_with_metadata": (i32, [vp, u8p, sz, ctypes.c_char_p, i32, u8p, sz, szp, ip, ip]),
        "s3hc_handler_compress_with_algorithm": (i32, [vp, u8p, sz, i32, u8p, sz, szp, ip]),
        "s3hc_handler_decompress_with_algorithm": (i32, [vp, u8p, sz, i32, u8p, sz, szp]),
        "s3hc_handler_stats": (None, [vp, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_float)]),
        "s3hc_handler_record_batch_bytes": (None, [vp, u64, u64]),
        "s3hc_handler_record_object": (None, [vp, i32]),
        "s3hc_handler_debug_set_faults": (None, [vp, i32]),
        "s3hc_is_denylisted_extension": (i32, [ctypes.c_char_p]),
        "s3hc_strip_known_cache_key_suffixes": (sz, [ctypes.c_char_p, ctypes.c_char_p, sz]),
        "s3hc_effective_compression": (i32, [i32, i32, sz, ctypes.c_char_p, u64]),
        "s3hc_handler_effective_compression": (i32, [vp, i32, i32, ctypes.c_char_p, u64]),
        "s3hc_dev_alloc": (i32, [vp, sz, ctypes.POINTER(vp)]),
        "s3hc_dev_free": (i32, [vp, vp]),
        "s3hc_memcpy": (i32, [vp, vp, vp, sz, i32]),
        "s3hc_memset": (i32, [vp, vp, i32, sz]),
        "s3hc_sync": (i32, [vp]),
        "s3hc_host_alloc": (i32, [vp, sz, ctypes.POINTER(vp)]),
        "s3hc_host_free": (i32, [vp, vp]),
        "s3hc_queue_create": (i32, [vp, ctypes.POINTER(vp)]),
        "s3hc_queue_destroy": (i32, [vp, vp]),
        "s3hc_queue_sync": (i32, [vp, vp]),
        "s3hc_memcpy_async": (i32, [vp, vp, vp, sz, i32, vp]),
        "s3hc_queue_mark": (i32, [vp, vp, ctypes.POINTER(vp)]),
        "s3hc_queue_wait_mark": (i32, [vp, vp, vp]),
        "s3hc_mark_free": (i32, [vp, vp]),
        "s3hc_reader_open": (i32, [vp, sz, i32, ctypes.POINTER(vp)]),
        "s3hc_reader_set_batch_max": (i32, [vp, sz]),
        "s3hc_reader_feed": (i32, [vp, u8p, sz]),
        "s3hc_reader_finish": (i32, [vp]),
        "s3hc_reader_read": (i32, [vp, u8p, sz, szp]),
        "s3hc_reader_total": (u64, [vp]),
        "s3hc_reader_close": (None, [vp]),
        "s3hc_aggregator_create": (i32, [vp, sz, sz, u32, vp, ctypes.POINTER(vp)]),
        "s3hc_aggregator_create_multi": (i32, [ctypes.POINTER(vp), i32, sz, sz, u32, vp, ctypes.POINTER(vp)]),
        "s3hc_shard_items": (i32, [ctypes.POINTER(u64), u32, i32, ctypes.POINTER(u32)]),
        "s3hc_reader_open_multi": (i32, [ctypes.POINTER(vp), i32, sz, i32, ctypes.POINTER(vp)]),
        "s3hc_aggregator_flush": (i32, [vp]),
        "s3hc_aggregator_set_frame_policy": (i32, [vp, i32]),
        "s3hc_aggregator_counters": (None, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "s3hc_aggregator_destroy": (None, [vp]),
        "s3hc_writer_begin": (i32, [vp, u64, u64, i32, vp, vp, ctypes.POINTER(vp)]),
        "s3hc_writer_write": (i32, [vp, u8p, sz]),
        "s3hc_writer_batch_buf_len": (sz, [vp]),
        "s3hc_writer_bytes_written": (u64, [vp]),
        "s3hc_writer_compressed_bytes_written": (u64, [vp]),
        "s3hc_writer_commit": (i32, [vp, ctypes.c_double, ctypes.POINTER(u64)]),
        "s3hc_writer_abort": (None, [vp]),
        "s3hc_writer_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


lib = _load()


def _ptr(b) -> ctypes.c_void_p:
    if isinstance(b, (bytes, bytearray, memoryview)):
        b = bytes(b)
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), b
    raise TypeError(type(b))


def _check(rc: int):
    if rc != S3HC_OK:
        raise CodecError(rc, (lib.s3hc_last_error() or b"").decode(errors="replace"))


def is_denylisted_extension(path: str) -> bool:
    """CompressionHandler::is_denylisted_extension (compression.rs:252-255)."""
    return bool(lib.s3hc_is_denylisted_extension(path.encode()))


def strip_known_cache_key_suffixes(cache_key: str) -> str:
    """cache.rs:226-275: the object path of a cache key (":range:a-b" then ":part:n" stripped)."""
    k = cache_key.encode()
    n = lib.s3hc_strip_known_cache_key_suffixes(k, None, 0)
    out = ctypes.create_string_buffer(n + 1)
    lib.s3hc_strip_known_cache_key_suffixes(k, out, n + 1)
    return out.raw[:n].decode()


@dataclass
class ResolvedSettings:  # bucket_settings.rs:364 (the fields effective_compression reads)
    compression_enabled: bool = True
    compression_from_rule: bool = False


def effective_compression(resolved: ResolvedSettings, compression_threshold: int, cache_key: str, size: int) -> bool:
    """CacheManager::effective_compression (cache.rs:1158-1178)."""
    return bool(lib.s3hc_effective_compression(1 if resolved.compression_enabled else 0,
                                               1 if resolved.compression_from_rule else 0,
                                               compression_threshold, cache_key.encode(), size))


def device_count() -> int:
    return lib.s3hc_device_count()


def set_knob(name: str, value=None) -> None:
    """Process-wide diagnostic / A-B switch (s3hc_set_knob): value None = default."""
    _check(lib.s3hc_set_knob(name.encode(), None if value is None else str(value).encode()))


def get_knob(name: str) -> int:
    """The knob's raw value (S3HC_FAST reads S3HC_FAST_DISABLE's slot)."""
    v = ctypes.c_longlong()
    _check(lib.s3hc_get_knob(name.encode(), ctypes.byref(v)))
    return v.value


class knobs:
    """Context manager: set knobs (name -> value) for the block, then restore the values they had
    on entry (raw slot values, so alias names such as S3HC_FAST / S3HC_FAST_DISABLE restore
    exactly). Replaces the environment toggles of earlier rounds (the library reads the
    environment once)."""

    def __init__(self, env: dict):
        self.env = dict(env)
        self.saved = []

    def __enter__(self):
        self.saved = [(k, get_knob(k)) for k in self.env]
        for k, v in self.env.items():
            set_knob(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in reversed(self.saved):
            _check(lib.s3hc_set_knob_value(k.encode(), v))
        return False


def shard_items(lens, ndev: int) -> list[int]:
    """s3hc_shard_items: first item of each of ndev contiguous shards (about equal bytes) + [n]."""
    n = len(lens)
    a = (ctypes.c_uint64 * max(n, 1))(*lens)
    f = (ctypes.c_uint32 * (ndev + 1))()
    _check(lib.s3hc_shard_items(a, n, ndev, f))
    return list(f)


def check_batch_results(olen, status, dst_off, slot_total):
    """s3hc_diag_check_batch_results: (good, bytes) or CodecError(S3HC_DEVICE) (the reader's
    check of device-written frame results before any copy)."""
    n = len(olen)
    a = (ctypes.c_uint32 * max(n, 1))(*olen)
    b = (ctypes.c_int32 * max(n, 1))(*status)
    c = (ctypes.c_uint64 * max(n, 1))(*dst_off)
    g, by = ctypes.c_uint32(), ctypes.c_uint64()
    _check(lib.s3hc_diag_check_batch_results(n, a, b, c, slot_total, ctypes.byref(g), ctypes.byref(by)))
    return g.value, by.value


def frame_bound(n: int) -> int:
    return lib.s3hc_frame_bound(n)


class Engine:
    """One s3hc context on one GPU."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib.s3hc_create(ctypes.byref(h), device))
        self.h = h

    def close(self):
        if self.h:
            lib.s3hc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- whole-buffer codec on host buffers
    def compress_frame(self, data, policy: int = BLK_AUTO_LZ4FLEX) -> bytes:
        p, keep = _ptr(data)
        cap = frame_bound(len(keep))
        out = ctypes.create_string_buffer(cap)
        n, wc = ctypes.c_size_t(), ctypes.c_int()
        _check(lib.s3hc_compress_frame(self.h, p, len(keep), policy, out, cap, ctypes.byref(n), ctypes.byref(wc)))
        return out.raw[: n.value]

    def store_mode_frame(self, data) -> bytes:
        p, keep = _ptr(data)
        cap = frame_bound(len(keep)) + 4 * (len(keep) // (4 << 20) + 1)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        _check(lib.s3hc_store_mode_frame(self.h, p, len(keep), out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    def decompress_frames(self, data, cap: int | None = None) -> bytes:
        p, keep = _ptr(data)
        if cap is None:  # library-owned output of exactly the decoded size
            buf, n = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_size_t()
            _check(lib.s3hc_decompress_frames_alloc(self.h, p, len(keep), ctypes.byref(buf), ctypes.byref(n)))
            try:
                return ctypes.string_at(buf, n.value)
            finally:
                lib.s3hc_buffer_free(buf)
        out = ctypes.create_string_buffer(max(cap, 1))
        n = ctypes.c_size_t()
        _check(lib.s3hc_decompress_frames(self.h, p, len(keep), out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    def decompress_status(self, data) -> tuple[int, bytes]:
        try:
            return S3HC_OK, self.decompress_frames(data)
        except CodecError as e:
            return e.status, b""

    def stream(self) -> "FrameStream":
        return FrameStream(self)

    # ---- match-finder mode of this engine's encodes (frames decode the same either way)
    def set_encode_mode(self, mode: int):
        _check(lib.s3hc_set_encode_mode(self.h, mode))

    @property
    def encode_mode(self) -> int:
        return lib.s3hc_get_encode_mode(self.h)

    # ---- timing of the last *_dev call
    def set_timing(self, on, coarse: bool = False):
        """on: every phase its own span; coarse: only "enc_parse" and "dec_all" (fewest events)."""
        lib.s3hc_set_timing(self.h, (2 if coarse else 1) if on else 0)

    def timing_reset(self):
        lib.s3hc_timing_reset(self.h)

    def timing(self) -> dict:
        """{kernel name: (total ms, launches)} since the last reset."""
        _check(lib.s3hc_timing_collect(self.h))
        out = {}
        for name in ("xxh32_side", "xxh32", "enc_parse", "enc_sizes", "enc_emit", "dec_plan", "decode", "dec_finish", "dec_close",
                     "dec_all", "compat"):
            n = lib.s3hc_kernel_count(self.h, name.encode())
            if n:
                out[name] = (lib.s3hc_last_kernel_ms(self.h, name.encode()), n)
        return out

    def sync(self):
        _check(lib.s3hc_sync(self.h))

    def alloc(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    def upload(self, data) -> "DeviceBuffer":
        b = DeviceBuffer(self, len(data))
        b.write(data)
        return b

    # ---- pipelined host<->device batches
    def host_alloc(self, nbytes: int) -> "HostBuffer":
        return HostBuffer(self, nbytes)

    def queue(self) -> "Queue":
        return Queue(self)

    def mark(self, queue: "Queue" = None) -> int:
        """Record the point reached by the work queued on `queue` so far (None: the context
        queue); pass it to wait_mark, release it with free_mark."""
        m = ctypes.c_void_p()
        _check(lib.s3hc_queue_mark(self.h, _q(queue), ctypes.byref(m)))
        return m.value

    def wait_mark(self, mark: int, queue: "Queue" = None):
        """Later work on `queue` starts only after `mark` is passed."""
        _check(lib.s3hc_queue_wait_mark(self.h, _q(queue), ctypes.c_void_p(mark)))

    def free_mark(self, mark: int):
        _check(lib.s3hc_mark_free(self.h, ctypes.c_void_p(mark)))

    def copy_async(self, dst, src, n: int, kind: int, queue: "Queue" = None, dst_off: int = 0, src_off: int = 0):
        """kind 1 H2D, 2 D2H, 3 D2D; dst/src: DeviceBuffer or HostBuffer (data_ptr())."""
        _check(lib.s3hc_memcpy_async(self.h, ctypes.c_void_p(dst.data_ptr() + dst_off),
                                     ctypes.c_void_p(src.data_ptr() + src_off), n, kind,
                                     queue.q if queue is not None else None))

    # ---- device-resident batches (DeviceBuffer or any object with data_ptr()/numel())
    def plan_encode(self, src_off, lengths, modes=None) -> "Plan":
        n = len(src_off)
        a_off = (ctypes.c_uint64 * n)(*src_off)
        a_len = (ctypes.c_uint32 * n)(*lengths)
        a_mode = (ctypes.c_uint8 * n)(*(modes if modes is not None else [0] * n))
        h = ctypes.c_void_p()
        _check(lib.s3hc_plan_encode(self.h, a_off, a_len, a_mode, n, ctypes.byref(h)))
        return Plan(h, n)

    def encode_dev(self, plan: "Plan", d_src, d_dst, d_item_off, d_item_len, stream=None):
        _check(lib.s3hc_encode_dev(self.h, plan.h, d_src.data_ptr(), d_dst.data_ptr(), d_dst.numel(),
                                   d_item_off.data_ptr(), d_item_len.data_ptr(), _q(stream)))

    def compat_dst_offsets(self, lengths) -> list:
        """Frame slots for compat_encode_dev: s3hc_frame_bound(len) bytes per item."""
        out, o = [], 0
        for n in lengths:
            out.append(o)
            o += frame_bound(n)
        return out + [o]

    def compat_encode_dev(self, src_off, lengths, d_src, d_dst, d_frame_len, dst_off=None, stream=None) -> list:
        """lz4_flex-compatible frames (S3HC_BLK_LZ4FLEX_COMPAT), one per item, into slots of
        frame_bound(len) bytes (dst_off[i]); returns dst_off. Frame lengths land in d_frame_len."""
        n = len(src_off)
        if dst_off is None:
            dst_off = self.compat_dst_offsets(lengths)[:n]
        a_off = (ctypes.c_uint64 * n)(*src_off)
        a_len = (ctypes.c_uint32 * n)(*lengths)
        a_dof = (ctypes.c_uint64 * n)(*dst_off)
        _check(lib.s3hc_compat_encode_dev(self.h, d_src.data_ptr(), a_off, a_len, n, d_dst.data_ptr(), a_dof,
                                          d_frame_len.data_ptr(), _q(stream)))
        return list(dst_off)

    def plan_decode(self, frame_off, frame_len, dst_off, dst_cap) -> "Plan":
        n = len(frame_off)
        h = ctypes.c_void_p()
        _check(lib.s3hc_plan_decode(self.h, (ctypes.c_uint64 * n)(*frame_off), (ctypes.c_uint32 * n)(*frame_len),
                                    (ctypes.c_uint64 * n)(*dst_off), (ctypes.c_uint32 * n)(*dst_cap), n,
                                    ctypes.byref(h)))
        return Plan(h, n)

    def decode_dev(self, plan: "Plan", d_src, d_dst, d_out_len, d_status, stream=None):
        _check(lib.s3hc_decode_dev(self.h, plan.h, d_src.data_ptr(), d_dst.data_ptr(), d_out_len.data_ptr(),
                                   d_status.data_ptr(), _q(stream)))


class HostBuffer:
    """Pinned host memory (hipHostMalloc) for overlapped copies; numpy view via .view()."""

    def __init__(self, eng: Engine, nbytes: int):
        self.eng, self.nbytes = eng, int(nbytes)
        p = ctypes.c_void_p()
        _check(lib.s3hc_host_alloc(eng.h, self.nbytes, ctypes.byref(p)))
        self.ptr = p

    def data_ptr(self) -> int:
        return self.ptr.value

    def numel(self) -> int:
        return self.nbytes

    def view(self):
        import numpy as np
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr.value))

    def free(self):
        if self.ptr:
            lib.s3hc_host_free(self.eng.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.eng.h:
                self.free()
        except Exception:
            pass


class Queue:
    """A HIP stream of the engine's device (the `stream` argument of encode_dev/decode_dev)."""

    def __init__(self, eng: Engine):
        self.eng = eng
        q = ctypes.c_void_p()
        _check(lib.s3hc_queue_create(eng.h, ctypes.byref(q)))
        self.q = q

    def sync(self):
        _check(lib.s3hc_queue_sync(self.eng.h, self.q))

    def close(self):
        if self.q:
            lib.s3hc_queue_destroy(self.eng.h, self.q)
            self.q = None


class DeviceBuffer:
    """HBM buffer owned by the engine's HIP runtime (data_ptr()/numel() like a tensor)."""

    def __init__(self, eng: Engine, nbytes: int):
        self.eng, self.nbytes = eng, int(nbytes)
        p = ctypes.c_void_p()
        _check(lib.s3hc_dev_alloc(eng.h, self.nbytes, ctypes.byref(p)))
        self.ptr = p

    def data_ptr(self) -> int:
        return self.ptr.value

    def numel(self) -> int:
        return self.nbytes

    def write(self, data, offset: int = 0):
        p, keep = _ptr(data)
        assert offset + len(keep) <= self.nbytes
        _check(lib.s3hc_memcpy(self.eng.h, ctypes.c_void_p(self.ptr.value + offset), p, len(keep), 1))

    def read(self, n: int | None = None, offset: int = 0) -> bytes:
        n = self.nbytes - offset if n is None else n
        out = ctypes.create_string_buffer(max(n, 1))
        _check(lib.s3hc_memcpy(self.eng.h, out, ctypes.c_void_p(self.ptr.value + offset), n, 2))
        return out.raw[:n]

    def fill(self, value: int = 0):
        _check(lib.s3hc_memset(self.eng.h, self.ptr, value, self.nbytes))

    def u32(self, n: int) -> list:
        import array
        a = array.array("I")
        a.frombytes(self.read(4 * n))
        return list(a)

    def i32(self, n: int) -> list:
        import array
        a = array.array("i")
        a.frombytes(self.read(4 * n))
        return list(a)

    def u64(self, n: int) -> list:
        import array
        a = array.array("Q")
        a.frombytes(self.read(8 * n))
        return list(a)

    def free(self):
        if self.ptr:
            lib.s3hc_dev_free(self.eng.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.eng.h:
                self.free()
        except Exception:
            pass


class Plan:
    def __init__(self, h, n):
        self.h, self.n = h, n

    @property
    def dst_bound(self) -> int:
        return lib.s3hc_plan_dst_bound(self.h)

    def __del__(self):
        try:
            if self.h:
                lib.s3hc_plan_free(self.h)
                self.h = None
        except Exception:
            pass


class FrameStream:
    """stream_range_data (disk_cache.rs:3850-3935): feed compressed bytes, read decoded chunks."""

    def __init__(self, eng: Engine):
        h = ctypes.c_void_p()
        _check(lib.s3hc_stream_open(eng.h, ctypes.byref(h)))
        self.h = h

    def feed(self, data):
        p, keep = _ptr(data)
        _check(lib.s3hc_stream_feed(self.h, p, len(keep)))

    def finish(self):
        _check(lib.s3hc_stream_finish(self.h))

    def read(self, cap: int = 1 << 20) -> bytes:
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        _check(lib.s3hc_stream_read(self.h, out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    @property
    def total(self) -> int:
        return lib.s3hc_stream_total(self.h)

    def __del__(self):
        try:
            if self.h:
                lib.s3hc_stream_close(self.h)
                self.h = None
        except Exception:
            pass


class RangeReader:
    """Pipelined stream_range_data: feed compressed bytes, read decoded bytes in stream order;
    batches of ~batch_bytes run on `depth` HIP queues. batch_max (optional): batches queued behind
    running ones may take up to batch_max bytes of buffered frames (s3hc_reader_set_batch_max)."""

    def __init__(self, eng, batch_bytes: int = 256 << 10, depth: int = 3, batch_max: int | None = None):
        """eng: an Engine, or a list of Engines (s3hc_reader_open_multi: depth queues per device)."""
        h = ctypes.c_void_p()
        if isinstance(eng, (list, tuple)):
            arr = (ctypes.c_void_p * len(eng))(*[e.h for e in eng])
            _check(lib.s3hc_reader_open_multi(arr, len(eng), batch_bytes, depth, ctypes.byref(h)))
        else:
            _check(lib.s3hc_reader_open(eng.h, batch_bytes, depth, ctypes.byref(h)))
        self.h = h
        if batch_max is not None:
            _check(lib.s3hc_reader_set_batch_max(h, batch_max))

    def feed(self, data):
        p, keep = _ptr(data)
        _check(lib.s3hc_reader_feed(self.h, p, len(keep)))

    def feed_ptr(self, ptr: int, n: int):
        _check(lib.s3hc_reader_feed(self.h, ctypes.c_void_p(ptr), n))

    def finish(self):
        _check(lib.s3hc_reader_finish(self.h))

    def read(self, cap: int = 1 << 20) -> bytes:
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        _check(lib.s3hc_reader_read(self.h, out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    def read_into(self, ptr: int, cap: int) -> int:
        n = ctypes.c_size_t()
        _check(lib.s3hc_reader_read(self.h, ctypes.c_void_p(ptr), cap, ctypes.byref(n)))
        return n.value

    @property
    def total(self) -> int:
        return lib.s3hc_reader_total(self.h)

    def close(self):
        if self.h:
            lib.s3hc_reader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class CompressionResult:  # compression.rs:159-166
    data: bytes
    algorithm: int
    original_size: int
    compressed_size: int
    was_compressed: bool


@dataclass
class CompressionStats:  # compression.rs:53-76
    total_objects_compressed: int
    total_objects_uncompressed: int
    total_bytes_before: int
    total_bytes_after: int
    compression_failures: int
    decompression_failures: int
    average_compression_ratio: float


class CompressionHandler:
    """Mirror of src/compression.rs CompressionHandler over the C++ handler in the library."""

    def __init__(self, engine: Engine, compression_threshold: int, compression_enabled: bool, _h=None):
        self.engine = engine
        self.h = _h if _h is not None else lib.s3hc_handler_new(engine.h, compression_threshold,
                                                                1 if compression_enabled else 0)

    @classmethod
    def new_with_shared_stats(cls, threshold: int, enabled: bool, source: "CompressionHandler"):
        return cls(source.engine, threshold, enabled, lib.s3hc_handler_new_with_shared_stats(
            threshold, 1 if enabled else 0, source.h))

    def clone(self) -> "CompressionHandler":
        return CompressionHandler(self.engine, 0, True, lib.s3hc_handler_clone(self.h))

    def __del__(self):
        try:
            if self.h:
                lib.s3hc_handler_free(self.h)
                self.h = None
        except Exception:
            pass

    def is_compression_enabled(self) -> bool:
        return bool(lib.s3hc_handler_is_compression_enabled(self.h))

    @staticmethod
    def is_denylisted_extension(path: str) -> bool:
        return is_denylisted_extension(path)

    @staticmethod
    def encode_store_mode_frame(engine: Engine, data) -> bytes:
        return engine.store_mode_frame(data)

    def compress_with_metadata(self, data, path: str, should_compress: bool) -> CompressionResult:
        p, keep = _ptr(data)
        cap = frame_bound(len(keep)) + 4 * (len(keep) // (4 << 20) + 1) + 64
        out = ctypes.create_string_buffer(cap)
        n, alg, wc = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int()
        _check(lib.s3hc_handler_compress_with_metadata(self.h, p, len(keep), path.encode(), 1 if should_compress else 0,
                                                       out, cap, ctypes.byref(n), ctypes.byref(alg), ctypes.byref(wc)))
        return CompressionResult(out.raw[: n.value], alg.value, len(keep), n.value, bool(wc.value))

    def compress_with_algorithm(self, data, algorithm: int = ALG_LZ4) -> CompressionResult:
        p, keep = _ptr(data)
        cap = frame_bound(len(keep)) + 64
        out = ctypes.create_string_buffer(cap)
        n, wc = ctypes.c_size_t(), ctypes.c_int()
        _check(lib.s3hc_handler_compress_with_algorithm(self.h, p, len(keep), algorithm, out, cap, ctypes.byref(n),
                                                        ctypes.byref(wc)))
        return CompressionResult(out.raw[: n.value], algorithm, len(keep), n.value, bool(wc.value))

    def decompress_with_algorithm(self, data, algorithm: int = ALG_LZ4) -> bytes:
        p, keep = _ptr(data)
        b = ctypes.c_size_t()
        lib.s3hc_decompressed_bound(p, len(keep), ctypes.byref(b))  # <= 255 x len(data)
        cap = max(b.value, len(keep), 1)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        _check(lib.s3hc_handler_decompress_with_algorithm(self.h, p, len(keep), algorithm, out, cap, ctypes.byref(n)))
        return out.raw[: n.value]

    def decompress_data(self, data) -> bytes:
        return self.decompress_with_algorithm(data, ALG_LZ4)

    def get_stats(self) -> CompressionStats:
        arr = (ctypes.c_uint64 * 6)()
        r = ctypes.c_float()
        lib.s3hc_handler_stats(self.h, arr, ctypes.byref(r))
        return CompressionStats(*list(arr), r.value)

    def record_batch_bytes(self, before: int, after: int):
        lib.s3hc_handler_record_batch_bytes(self.h, before, after)

    def effective_compression(self, resolved: ResolvedSettings, cache_key: str, size: int) -> bool:
        """cache.rs:1158-1178 with this handler's threshold (the CacheManager's compression_threshold)."""
        return bool(lib.s3hc_handler_effective_compression(self.h, 1 if resolved.compression_enabled else 0,
                                                           1 if resolved.compression_from_rule else 0,
                                                           cache_key.encode(), size))

    def record_object(self, compressed: bool):
        lib.s3hc_handler_record_object(self.h, 1 if compressed else 0)

    # tests only: make the LZ4 encoder / store-mode encoder / decoder of this handler fail
    FAULT_LZ4, FAULT_STORE, FAULT_DECODE = 1, 2, 4

    def debug_set_faults(self, mask: int):
        lib.s3hc_handler_debug_set_faults(self.h, mask)


# ---------------------------------------------------------------------------------------------
# Batched incremental writers (IncrementalRangeWriter, disk_cache.rs:262-305, 1716-2116) over the
# cross-request aggregator (one GPU launch for the full batches of many writers).
FRAME_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t)


def _wcheck(rc: int):
    if rc != S3HC_OK:
        raise CodecError(rc, (lib.s3hc_writer_last_error() or b"").decode(errors="replace"))


@dataclass
class RangeSpec:  # cache_types.rs:472-508 (codec fields)
    start: int
    end: int
    compressed_size: int
    uncompressed_size: int


class BatchAggregator:
    """Coalesces the flush_batch calls of many writers into one encode launch."""

    def __init__(self, eng, batch_size: int = 1 << 20, flush_bytes: int = 0, flush_batches: int = 0,
                 stats: "CompressionHandler | None" = None, frame_policy: int = BLK_AUTO_LZ4FLEX):
        """eng: an Engine, or a list of Engines (s3hc_aggregator_create_multi: each flush is
        split into contiguous shards, one per device)."""
        h = ctypes.c_void_p()
        st = stats.h if stats is not None else None
        if isinstance(eng, (list, tuple)):
            arr = (ctypes.c_void_p * len(eng))(*[e.h for e in eng])
            _wcheck(lib.s3hc_aggregator_create_multi(arr, len(eng), batch_size, flush_bytes, flush_batches, st,
                                                     ctypes.byref(h)))
        else:
            _wcheck(lib.s3hc_aggregator_create(eng.h, batch_size, flush_bytes, flush_batches, st, ctypes.byref(h)))
        self.h, self.eng, self.stats = h, eng, stats
        if frame_policy != BLK_AUTO_LZ4FLEX:
            _wcheck(lib.s3hc_aggregator_set_frame_policy(h, frame_policy))

    def flush(self):
        _wcheck(lib.s3hc_aggregator_flush(self.h))

    def counters(self) -> tuple[int, int]:
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        lib.s3hc_aggregator_counters(self.h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def begin(self, start: int, end: int, compression_enabled: bool, sink=None) -> "IncrementalRangeWriter":
        return IncrementalRangeWriter(self, start, end, compression_enabled, sink)

    def close(self):
        if self.h:
            lib.s3hc_aggregator_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class IncrementalRangeWriter:
    """begin_incremental_range_write / write_range_chunk / commit / abort. Frames go to `sink`
    (callable(bytes) -> None, the reference's .tmp file) or, by default, to self.file."""

    def __init__(self, agg: BatchAggregator, start: int, end: int, compression_enabled: bool, sink=None):
        self.agg = agg
        self.file = bytearray()
        self._user_sink = sink

        def _sink(_user, frame, n):
            try:
                b = ctypes.string_at(frame, n)
                if self._user_sink is not None:
                    self._user_sink(b)
                else:
                    self.file += b
                return 0
            except Exception:
                return 1

        self._cb = FRAME_SINK(_sink)  # keep alive while the writer exists
        h = ctypes.c_void_p()
        _wcheck(lib.s3hc_writer_begin(agg.h, start, end, 1 if compression_enabled else 0,
                                      ctypes.cast(self._cb, ctypes.c_void_p), None, ctypes.byref(h)))
        self.h = h

    def write(self, chunk):
        p, keep = _ptr(chunk)
        _wcheck(lib.s3hc_writer_write(self.h, p, len(keep)))

    def batch_buf_len(self) -> int:
        return lib.s3hc_writer_batch_buf_len(self.h)

    @property
    def bytes_written(self) -> int:
        return lib.s3hc_writer_bytes_written(self.h)

    @property
    def compressed_bytes_written(self) -> int:
        return lib.s3hc_writer_compressed_bytes_written(self.h)

    def commit(self, min_commit_ratio: float | None = None) -> RangeSpec:
        spec = (ctypes.c_uint64 * 4)()
        h, self.h = self.h, None
        _wcheck(lib.s3hc_writer_commit(h, -1.0 if min_commit_ratio is None else min_commit_ratio, spec))
        return RangeSpec(*list(spec))

    def abort(self):
        h, self.h = self.h, None
        if h:
            lib.s3hc_writer_abort(h)
