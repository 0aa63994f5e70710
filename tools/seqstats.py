#!/usr/bin/env python3
"""Token statistics of LZ4 frames (gpurun_out/frames.bin from tools/dump_frames.py): sequence
lengths, offsets, and per 64-sequence window how match sources relate to the window (the
executor's round 0 / in-window cases). CPU only."""
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
blob = open(os.path.join(ROOT, "gpurun_out", "frames.bin"), "rb").read()
meta = json.load(open(os.path.join(ROOT, "gpurun_out", "frames.json")))
W = int(sys.argv[1]) if len(sys.argv) > 1 else 64


def blocks(fr):
    ip = 7
    while True:
        w = int.from_bytes(fr[ip:ip + 4], "little")
        ip += 4
        if w == 0:
            return
        n = w & 0x7FFFFFFF
        yield fr[ip:ip + n], bool(w >> 31)
        ip += n


def seqs(b):
    p, o, out = 0, 0, []
    C = len(b)
    while p < C:
        t = b[p]; p += 1
        ll = t >> 4
        if ll == 15:
            while True:
                e = b[p]; p += 1; ll += e
                if e != 255: break
        lit = p
        p += ll
        if p >= C:
            out.append((o, ll, lit, 0, 0)); break
        off = b[p] | (b[p + 1] << 8); p += 2
        ml = (t & 15) + 4
        if (t & 15) == 15:
            while True:
                e = b[p]; p += 1; ml += e
                if e != 255: break
        out.append((o, ll, lit, off, ml))
        o += ll + ml
    return out


st = Counter()
lls, mls, offs, ntok = [], [], [], []
depths = Counter()
for fo, fl in zip(meta["fo"], meta["fl"]):
    fr = blob[fo:fo + fl]
    for b, stored in blocks(fr):
        if stored:
            st["stored"] += 1; continue
        S = seqs(b)
        ntok.append(len(S))
        for (o, ll, lit, off, ml) in S:
            lls.append(ll); mls.append(ml); offs.append(off)
        for w0 in range(0, len(S), W):
            win = S[w0:w0 + W]
            ws = win[0][0]
            # byte kind map of the window: 0 literal, 1 match (pending until resolved)
            we = win[-1][0] + win[-1][1] + win[-1][4]
            kind = np.zeros(we - ws, np.int8)
            for (o, ll, lit, off, ml) in win:
                kind[o + ll - ws:o + ll + ml - ws] = 1
            # depth per match: 0 if source before window or all-literal; else 1 + max depth of
            # the in-window matches its source touches
            dep = {}
            owner = np.full(we - ws, -1, np.int32)
            for i, (o, ll, lit, off, ml) in enumerate(win):
                owner[o + ll - ws:o + ll + ml - ws] = i
            for i, (o, ll, lit, off, ml) in enumerate(win):
                if ml == 0: continue
                st["matches"] += 1
                md = o + ll; ms = md - off
                if ms + ml <= ws:
                    st["src_before_window"] += 1
                    if ms + 8192 < we: st["far_8k"] += 1
                    dep[i] = 0; continue
                if off < ml: st["overlap_self"] += 1
                lo, hi = max(ms, ws) - ws, min(ms + ml, md) - ws
                touched = set(owner[lo:hi][owner[lo:hi] >= 0].tolist()) - {i}
                if ms < ws: st["straddles_window_start"] += 1
                if not touched and off >= ml:
                    st["src_inwin_literal_only"] += 1; dep[i] = 0
                else:
                    d = 1 + max([dep.get(j, 0) for j in touched] + [0])
                    dep[i] = d
                    st["src_inwin_touches_match"] += 1
            depths[max(dep.values()) if dep else 0] += 1
lls, mls, offs = np.array(lls), np.array(mls), np.array(offs)
print("blocks", len(ntok), "tokens/block", np.mean(ntok), "max", max(ntok))
print("ll mean", lls.mean(), "p50", np.median(lls), "ll>15", (lls >= 15).mean(), "ll>16", (lls > 16).mean(), "ll>32", (lls > 32).mean(), "ll==0", (lls == 0).mean())
m = mls[mls > 0]
print("ml mean", m.mean(), "p50", np.median(m), "ml>=19", (m >= 19).mean(), "ml>16", (m > 16).mean(), "ml>32", (m > 32).mean())
o = offs[mls > 0]
print("off p50", np.median(o), "<64", (o < 64).mean(), "<256", (o < 256).mean(), "<1k", (o < 1024).mean(), "<4k", (o < 4096).mean(), ">8k", (o > 8192).mean())
for k, v in sorted(st.items()):
    print(f"{k:28s} {v:9d} {v / max(1, st['matches']):.3f}")
print("window max depth histogram", sorted(depths.items()))
