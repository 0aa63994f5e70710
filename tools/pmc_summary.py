#!/usr/bin/env python3
"""Per-kernel per-dispatch averages of rocprofv3 --pmc counter CSVs under a directory."""
import csv
import glob
import json
import sys
from collections import defaultdict


def kernel_key(name):
    """Base name of a kernel symbol: no return type, namespace, template arguments or parameters
    ("void s3hc::k_enc_parse<2u, 0u>(...)" -> "k_enc_parse")."""
    k = name.split("(")[0].split("<")[0].strip()
    if k.startswith("void "):
        k = k[5:]
    return k.replace("s3hc::", "")


def summarize(root):
    acc = defaultdict(lambda: defaultdict(list))
    for fn in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row["Kernel_Name"])
                per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"])
        for (d, k, c), v in per.items():
            acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in sorted(acc.items())}


if __name__ == "__main__":
    out = {}
    for r in sys.argv[1:]:
        for k, cs in summarize(r).items():
            out.setdefault(k, {}).update(cs)
    print(json.dumps(out, indent=1))
