#!/bin/bash
# Decode/encode kernel time vs blocks in flight (occupancy sweep) plus rocprof kernel stats of the
# default bench. Each GPU step has its own timeout; the script stops at the first failure.
# Usage: tools/sweep.sh [tag]   -> gpurun_out/sweep_<tag>/
tag=${1:-x}
out=gpurun_out/sweep_$tag
mkdir -p "$out"
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$out/$name.out" "$out/$name.err"; exit $rc; fi
}
for nb in ${SWEEP_BLOCKS:-256 1024 2048 4096 8192}; do
    step "b$nb" 120 python bench.py --blocks "$nb" --steps 10 --warmup 3 --no-cpu-baseline
    python - "$out/b$nb.out" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
print(f'blocks={d["config"]["blocks_per_gpu"]} value={d["value"]} enc_parse={k["enc_parse"]} decode={k["decode"]} emit={k["enc_emit"]} xxh={k["xxh32"]}')
EOF
done
if [ "${SWEEP_PROF:-1}" = 1 ]; then
    export TMPDIR=/tmp
    step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python bench.py --no-cpu-baseline --steps 10 --warmup 3
    find "$out/prof" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
    head -12 "$out/kernel_stats.csv" | cut -c1-200
fi
echo sweep-ok
