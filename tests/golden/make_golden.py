"""Generates the committed golden fixtures in tests/golden/ (run from the repo root).

Sources, none of which is our own codec:
  * store-mode frames: built here byte by byte from the layout in the reference code
    (src/compression.rs:326-368) with python `xxhash` 3.8.1 for XXH32 — independent of
    both oracle/ and the GPU engine; this pins store-mode parity to the reference.
  * lz4-frames of liblz4 1.9.3 (LZ4F_compressFrame, a different encoder than lz4_flex) over
    the reference's own fixture inputs (tests/lz4_roundtrip_preservation_test.rs:192-283,
    compression.rs unit-test strings): decode vectors with known plaintext sha256.
  * corrupt vectors from the reference's tests (compression.rs:740-741, disk_cache.rs:13740)
    and lz4 frame-format edge cases, with the status lz4_flex semantics give.
  * the empty lz4_flex frame: 15 bytes.
The lz4_flex compressed bytes themselves are NOT pinned (lz4_flex absent; parity unpinned).
"""
import hashlib
import json
import os
import struct
import sys

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/ for lz4ref
import lz4ref  # noqa: E402

MAGIC = struct.pack("<I", 0x184D2204)


def p251(n):  # tests/lz4_roundtrip_preservation_test.rs:192-196
    return bytes(i % 251 for i in range(n))


def store_mode(data: bytes) -> bytes:  # compression.rs:326-368
    flg, bd = 0x64, 0x70
    hc = (xxhash.xxh32(bytes([flg, bd]), seed=0).intdigest() >> 8) & 0xFF
    out = bytearray(MAGIC + bytes([flg, bd, hc]))
    for o in range(0, len(data), 4 << 20):
        chunk = data[o:o + (4 << 20)]
        out += struct.pack("<I", len(chunk) | 0x80000000) + chunk
    out += struct.pack("<I", 0) + struct.pack("<I", xxhash.xxh32(data, seed=0).intdigest())
    return bytes(out)


INPUTS = {
    "empty": ("lit", b""),
    "p251_1": ("p251", 1),
    "p251_63": ("p251", 63),
    "p251_64": ("p251", 64),
    "p251_1024": ("p251", 1024),
    "p251_65536": ("p251", 65536),
    "p251_1MiB+1": ("p251", (1 << 20) + 1),
    "p251_4MiB": ("p251", 4 << 20),
    "p251_4MiB+1": ("p251", (4 << 20) + 1),
    "stored_string": ("lit", b"This data will be stored, not compressed"),  # compression.rs:626
    "small_string": ("lit", b"small"),                                      # compression.rs:772
    "threshold_string": ("lit", b"Below threshold data"),                     # compression.rs:964
    "fake_jpeg": ("lit", b"This is fake JPEG data that should not be compressed"),  # compression.rs:935
    "repeat_A": ("lit", b"A" * 100),                                          # compression.rs:719
}


def materialize(spec):
    kind, v = spec
    return v if kind == "lit" else p251(v)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    cases = []
    for name, spec in INPUTS.items():
        data = materialize(spec)
        f = store_mode(data)
        c = {"name": f"store_mode/{name}", "kind": "store_mode", "input": {"kind": spec[0], "value": spec[1] if spec[0] == "p251" else spec[1].hex()},
             "frame_len": len(f), "frame_sha256": sha(f), "plain_len": len(data), "plain_sha256": sha(data)}
        if len(f) <= 4096:
            c["frame_hex"] = f.hex()
        cases.append(c)
    # liblz4-written frames (third-party encoder) as decode vectors
    lzin = {"p251_1024": p251(1024), "p251_65536": p251(65536), "p251_300000": p251(300_000),
            "repeat_text": b"This is some test data for compression with metadata. " * 200,
            "mixed": b"".join(bytes([i % 7]) * (i % 50 + 1) for i in range(2000)) + p251(5000)}
    variants = [("b64k_ind_cc", 4, False, True, False, False), ("b256k_ind_cc_bc", 5, False, True, True, False),
                ("b64k_linked_cc", 4, True, True, False, False), ("b4m_ind_cs", 7, False, False, False, True),
                ("b1m_ind_cc_cs", 6, False, True, False, True)]
    for iname, data in lzin.items():
        for vname, bsid, linked, cc, bc, cs in variants:
            fr = lz4ref.compress_frame(data, bsid, linked, cc, bc, cs)
            fn = f"lz4f_{iname}_{vname}.lz4"
            with open(os.path.join(HERE, fn), "wb") as fh:
                fh.write(fr)
            cases.append({"name": f"liblz4/{iname}/{vname}", "kind": "decode", "file": fn, "expect_status": 0,
                          "plain_len": len(data), "plain_sha256": sha(data)})
    # empty lz4_flex frame: magic, FLG 0x64, BD 0x40, HC 0xA7, EndMark, xxh32("")
    empty = MAGIC + bytes([0x64, 0x40, 0xA7]) + struct.pack("<I", 0) + struct.pack("<I", xxhash.xxh32(b"").intdigest())
    cases.append({"name": "lz4flex/empty_frame", "kind": "lz4flex_frame", "input": {"kind": "lit", "value": ""},
                  "frame_hex": empty.hex(), "plain_len": 0, "plain_sha256": sha(b"")})
    # corrupt / edge vectors: (name, hex, status, plaintext-or-None)
    good = lz4ref.compress_frame(p251(1024), 4, False, True, False, False)
    sm = store_mode(b"incompressible-ish chunk")
    corrupt = [
        ("ref_bad_flg", "04224d18ffffffff000102", 1),                  # compression.rs:740-741
        ("ref_deadbeef", "deadbeef01020304", 1),                       # disk_cache.rs:13740
        ("truncated_magic", "04224d", 1),
        ("header_only", "04224d186440a7", 1),
        ("bad_header_checksum", "04224d186440a800000000055dcc02", 1),
        ("empty_bad_checksum", "04224d186440a700000000055dcc03", 2),
        ("legacy_magic", "02214c18" + "00" * 8, 4),
        ("skippable_magic", "502a4d18" + "00" * 8, 4),
        ("dict_id", None, 4),
        ("trailing_garbage_after_frame", (good + b"xyz").hex(), 1),
        ("empty_then_garbage_stops", (empty + b"garbage").hex(), 0),
        ("store_flipped_payload", None, 2),
        ("block_too_big", None, 1),
    ]
    for name, hx, st in corrupt:
        if name == "dict_id":
            desc = bytes([0x65, 0x40]) + struct.pack("<I", 7)
            hc = (xxhash.xxh32(desc).intdigest() >> 8) & 0xFF
            blob = MAGIC + desc + bytes([hc]) + struct.pack("<I", 0)
        elif name == "store_flipped_payload":
            b = bytearray(sm)
            b[15] ^= 0x01
            blob = bytes(b)
        elif name == "block_too_big":
            hc = (xxhash.xxh32(bytes([0x64, 0x40])).intdigest() >> 8) & 0xFF
            blob = MAGIC + bytes([0x64, 0x40, hc]) + struct.pack("<I", 65537 | 0x80000000) + bytes(65537) + bytes(8)
        else:
            blob = bytes.fromhex(hx)
        case = {"name": f"corrupt/{name}", "kind": "corrupt", "expect_status": st}
        if len(blob) <= 4096:
            case["blob_hex"] = blob.hex()
        else:
            fn = f"corrupt_{name}.bin"
            with open(os.path.join(HERE, fn), "wb") as fh:
                fh.write(blob)
            case["file"] = fn
        if st == 0:
            case["plain_len"], case["plain_sha256"] = 0, sha(b"")
        cases.append(case)
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py", "xxhash": xxhash.VERSION, "cases": cases}, fh, indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
