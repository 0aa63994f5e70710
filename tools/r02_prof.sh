#!/bin/bash
# Round-2 profile set at HEAD: bench line with CPU baseline, rocprofv3 kernel stats of the same
# command, PMC traffic (FETCH_SIZE / WRITE_SIZE passes), PMC instruction counters, 2-rank line.
# Each step has its own timeout; the script stops at the first failure.
set -o pipefail
out=gpurun_out/r02prof
mkdir -p $out
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$out/$name.out" 2> "$out/$name.err"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/$name.err"; exit $rc; }; }
step bench 300 python bench.py
tail -1 $out/bench.out | cut -c1-300
export TMPDIR=/tmp
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python bench.py --no-cpu-baseline
find $out/stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
tail -1 $out/stats.out > $out/bench_profiled.json
step traffic 600 bash tools/traffic.sh
cp gpurun_out/traffic/traffic.json $out/traffic.json
step pmc 600 bash tools/pmc.sh r02
python tools/pmc_summary.py gpurun_out/pmc/r02_p1 gpurun_out/pmc/r02_p2 > $out/pmc.json
echo prof-ok
