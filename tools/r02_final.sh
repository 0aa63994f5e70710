#!/bin/bash
# Round-2 closing measurement set at HEAD: GPU suite, smoke, bench (N=1, with CPU baseline),
# --gpus 2 self-spawn, rocprofv3 kernel stats of the bench, large-block table, host calls,
# config-4 e2e (8 GiB). Each step has its own timeout; the script stops at the first failure.
out=gpurun_out/r02f
mkdir -p $out
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$out/$name.out" 2> "$out/$name.err"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/$name.out" "$out/$name.err"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
tail -1 $out/gpu_tests.out
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $out/smoke.out
step bench 300 python bench.py
tail -1 $out/bench.out | cut -c1-200
step bench2 300 python bench.py --gpus 2 --steps 5 --warmup 2
export TMPDIR=/tmp
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python bench.py --no-cpu-baseline
find $out/stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
step lb_table 400 python tools/lb.py
step hostcall 300 python tools/hostcall.py
step e2e 900 python tools/e2e.py --skip-config2
echo final-ok
