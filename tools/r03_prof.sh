#!/bin/bash
# Round-3 profile set at HEAD: PMC traffic (FETCH_SIZE / WRITE_SIZE passes; copied into
# profiles/r03/ first so the bench line's roofline.traffic reads it), rocprofv3 kernel stats of the
# bench command, PMC instruction counters, then the bench line with its CPU baseline.
set -o pipefail
out=gpurun_out/r03prof
mkdir -p $out profiles/r03
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$out/$name.out" 2> "$out/$name.err"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/$name.err"; exit $rc; }; }
step traffic 600 bash tools/traffic.sh
cp gpurun_out/traffic/traffic.json $out/traffic.json
cp gpurun_out/traffic/traffic.json profiles/r03/traffic.json
export TMPDIR=/tmp
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python bench.py --no-cpu-baseline
find $out/stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
tail -1 $out/stats.out > $out/bench_profiled.json
step pmc 600 bash tools/pmc.sh r03
python tools/pmc_summary.py gpurun_out/pmc/r03_p1 gpurun_out/pmc/r03_p2 > $out/pmc.json
step bench 400 python bench.py
tail -1 $out/bench.out | cut -c1-400
echo prof-ok
