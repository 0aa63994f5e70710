#!/bin/bash
# Round-2 spread-execution measurements: GPU suite, large-block table, reader/e2e (config 4),
# host calls. Each GPU step has its own timeout; stops at the first failure.
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.out" "gpurun_out/$name.err"; exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
tail -2 gpurun_out/gpu_tests.out
step lb_table 400 python tools/lb.py
step hostcall 300 python tools/hostcall.py
tail -5 gpurun_out/hostcall.out
step e2e 600 python tools/e2e.py --skip-config2 --gib 2
echo all-ok
