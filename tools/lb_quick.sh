#!/bin/bash
# Large-block quick check: large-block + reader tests, timings at 1/16/256 frames (spread and
# step loop), rocprofv3 kernel stats of the 256-frame case.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_reader.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tl.log 2>&1
rc=$?; tail -3 gpurun_out/tl.log; [ $rc -eq 0 ] || exit $rc
for n in 1 16 256; do
  timeout -k 10 120 python tools/lb.py $n | cut -c1-150 || exit 1
  S3HC_LBW_DISABLE=1 timeout -k 10 120 python tools/lb.py $n | cut -c1-150 || exit 1
done
rm -rf gpurun_out/p256
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/p256 -o run -- python3 tools/lb.py 256 > gpurun_out/p256.log 2>&1
