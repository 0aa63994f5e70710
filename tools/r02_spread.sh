#!/bin/bash
# Round-2 spread-execution measurements at HEAD: GPU suite, large-block table (spread default and
# step loop), rocprofv3 stats of 1 and 256 reference frames, host calls, config-4 e2e (8 GiB).
mkdir -p gpurun_out/r02s
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/r02s/$name.out" 2> "gpurun_out/r02s/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/r02s/$name.out" "gpurun_out/r02s/$name.err"; exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
tail -1 gpurun_out/r02s/gpu_tests.out
step lb_table 400 python tools/lb.py
S3HC_LBW_DISABLE=1 step lb_table_step 400 python tools/lb.py
step hostcall 300 python tools/hostcall.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r02s/p1 gpurun_out/r02s/p256
step prof1 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r02s/p1 -o run -- python3 tools/lb.py 1
step prof256 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r02s/p256 -o run -- python3 tools/lb.py 256
step e2e 900 python tools/e2e.py --skip-config2
echo all-ok
