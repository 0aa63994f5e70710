"""Per-launch-size table of the large-block kernels from rocprofv3 --kernel-trace databases
(one column per database): kernel, grid size in workgroups, launches, mean duration (us).
usage: python tools/lb_kstats.py A.db [B.db ...]"""
import collections
import sqlite3
import sys


def load(path):
    d = collections.defaultdict(list)
    con = sqlite3.connect(path)
    for name, gx, wx, dur in con.execute("select name, grid_x, workgroup_x, duration from kernels"):
        n = name.split("(")[0].replace("s3hc::", "")
        if "k_lb" in n or "k_lbw" in n or n.startswith("k_scan"):
            d[(gx // max(wx, 1), n)].append(dur)
    return {k: sum(v) / len(v) / 1000 for k, v in d.items()}


def main():
    dbs = [load(p) for p in sys.argv[1:]]
    keys = sorted(set().union(*dbs))
    print("%8s %-14s" % ("wgs", "kernel") + "".join("%12s" % ("db%d us" % i) for i in range(len(dbs))))
    for k in keys:
        print("%8d %-14s" % k + "".join("%12s" % ("%.1f" % d[k] if k in d else "-") for d in dbs))


if __name__ == "__main__":
    main()
