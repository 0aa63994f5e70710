#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite result (run_results.db): per-kernel count / total / average µs,
optionally the dispatch timeline between two dispatch indices.

usage: tools/dbstats.py DB [--csv OUT] [--timeline FIRST:LAST]
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    agg = {}
    for n, s, e in rows:
        k = short(n)
        cnt, tot = agg.get(k, (0, 0))
        agg[k] = (cnt + 1, tot + (e - s))
    lines = ["Name,Calls,TotalDurationNs,AverageNs,Percentage"]
    allt = sum(t for _, t in agg.values()) or 1
    for k, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k},{cnt},{tot},{tot / cnt:.1f},{100 * tot / allt:.2f}")
    print("\n".join(lines))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")
    if a.timeline:
        lo, hi = (int(x) for x in a.timeline.split(":"))
        t0 = rows[lo][1]
        prev = t0
        for i in range(lo, min(hi, len(rows))):
            n, s, e = rows[i]
            print(f"{i:5d} {short(n):28s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  gap {(s - prev) / 1e3:7.1f}")
            prev = e


if __name__ == "__main__":
    main()
