# Same-box A/B of the default bench line: alternates the tree's library with another build
# (S3HC_LIB_PATH), N rounds, and prints value and per-phase kernel times of each run.
# usage: bash tools/ab_bench.sh OTHER_LIB [N] [OUTDIR]
OTHER=$1; N=${2:-2}; O=${3:-gpurun_out/ab}
mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/tree_$i.json 2> $O/tree_$i.err || exit 1
  S3HC_LIB_PATH=$OTHER timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/other_$i.json 2> $O/other_$i.err || exit 1
done
python3 - "$O" "$N" <<'PY'
import json, sys
o, n = sys.argv[1], int(sys.argv[2])
for tag in ("tree", "other"):
    for i in range(1, n + 1):
        d = json.loads(open(f"{o}/{tag}_{i}.json").read().strip().splitlines()[-1])
        print(tag, i, d["value"], d["ms_per_step"], d["config"]["compression_ratio"], d["kernel_ms_per_step"])
PY
