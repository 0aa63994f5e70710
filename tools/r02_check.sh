#!/bin/bash
# Round-2 GPU check: GPU test suite, smoke, bench (N=1 with CPU baseline), the --gpus 2 self-spawn
# rehearsal on one GPU, config 5's per-GPU slice (131,072 blocks). Each GPU step has its own
# timeout; the script stops at the first failure.
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.out" "gpurun_out/$name.err"; exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
    tail -2 gpurun_out/gpu_tests.out
    step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
    tail -1 gpurun_out/smoke.out
fi
step bench 300 python bench.py
cut -c1-600 gpurun_out/bench.out
step bench2 300 python bench.py --gpus 2 --steps 5 --warmup 2
cut -c1-400 gpurun_out/bench2.out
if [ "${SKIP_C5:-0}" != 1 ]; then
    step bench_c5slice 600 python bench.py --blocks 131072 --steps 3 --warmup 1 --no-cpu-baseline
    cut -c1-600 gpurun_out/bench_c5slice.out
fi
echo all-ok
