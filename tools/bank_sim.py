#!/usr/bin/env python3
"""LDS bank-conflict model (gfx950: ds_read_b32 / ds_write_b8 / ds_mskor_b32 serviced in two
groups of 32 lanes, bank = (byte address / 4) mod 32, identical dwords broadcast, each extra
distinct dword on a busy bank = one extra cycle; MI355X_MICROARCH.md §LDS).

1. k_enc_parse's hash table (2^11 x u16 per wave): a wave's 64 probes or inserts hit
   uniformly random entries. A swizzle is a permutation of entry addresses, so random stays
   random: the expected extra cycles per full-wave table access do not change.
2. k_dexec's first literal chunk: lane i (sequence i of a 64-sequence window) stores byte k of
   its run at ring position d0_i + k, one ds_write_b8 per k. The sequences come from real
   frames (log text through the oracle's lz4_flex restatement); the ring is 8 KiB. Compared:
   the plain ring and an XOR swizzle of the 16-byte granule index by its bits 3..5 (a
   permutation inside each 1 KiB flush piece, so the flush's 16-byte reads stay whole).
Prints one JSON object."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sample-s3-hybrid-cache_amd"), os.path.join(ROOT, "oracle")]


def extra_cycles(dwords, active):
    """extra LDS cycles of one wave instruction: dwords[64] addresses (dword index), active[64]"""
    ex = 0
    for g in range(2):
        d = dwords[32 * g:32 * g + 32][active[32 * g:32 * g + 32]]
        if d.size == 0:
            continue
        u = np.unique(d)
        ex += int(np.bincount(u % 32, minlength=32).max()) - 1
    return ex


def table_model(trials=20000, seed=1):
    rng = np.random.default_rng(seed)
    tot = 0
    act = np.ones(64, bool)
    for _ in range(trials):
        idx = rng.integers(0, 2048, 64)
        tot += extra_cycles(idx >> 1, act)
    return tot / trials


def sequences(data):
    import oracle as O
    seqs = []
    for i in range(0, len(data), 65536):
        fr = O.lz4flex_compress_frame(data[i:i + 65536])
        bs = int.from_bytes(fr[7:11], "little")
        if bs & 0x80000000:
            continue
        b = fr[11:11 + bs]
        p, out = 0, 0
        while p < len(b):
            t = b[p]; p += 1
            L = t >> 4
            if L == 15:
                while True:
                    e = b[p]; p += 1; L += e
                    if e != 255:
                        break
            p += L
            if p >= len(b):
                seqs.append((L, 0))
                break
            p += 2
            M = (t & 15) + 4
            if (t & 15) == 15:
                while True:
                    e = b[p]; p += 1; M += e
                    if e != 255:
                        break
            seqs.append((L, M))
    return seqs


def literal_model(seqs, swz):
    tot, n = 0, 0
    pos = 0
    for w in range(0, len(seqs) - 64, 64):
        win = seqs[w:w + 64]
        d0 = []
        for ll, ml in win:
            d0.append(pos)
            pos += ll + ml
        d0 = np.array(d0)
        ll = np.array([s[0] for s in win])
        for k in range(16):
            act = ll > k
            y = (d0 + k) & 8191
            if swz:
                g = y >> 4
                g = g ^ ((g >> 3) & 7)
                y = (g << 4) | (y & 15)
            tot += extra_cycles(y >> 2, act)
            n += 1
    return tot / n


def main():
    import synth
    data = synth.log_text(64 * 65536, 5)
    seqs = sequences(data)
    out = {"enc_table_extra_cycles_per_full_wave_access": round(table_model(), 3),
           "dexec_literal_byte_store_extra_cycles_plain": round(literal_model(seqs, False), 3),
           "dexec_literal_byte_store_extra_cycles_granule_xor": round(literal_model(seqs, True), 3),
           "sequences": len(seqs), "mean_sequence_bytes": round(float(np.mean([a + b for a, b in seqs])), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
