#!/bin/bash
# Spread-execution check on one GPU: large-block tests, hash-chain probe, pending tiles per
# round (S3HC_LB_TRACE), large-block timings (spread vs step loop). Stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tl.log 2>&1
rc=$?; tail -5 gpurun_out/tl.log; [ $rc -eq 0 ] || exit $rc
if [ -x tools/probe/xxh_chain ]; then timeout -k 10 60 ./tools/probe/xxh_chain || exit $?; fi
for n in 1 16 256; do
  S3HC_LB_TRACE=1 timeout -k 10 120 python tools/lb.py $n > gpurun_out/lbw_$n.out 2> gpurun_out/lbw_$n.err || exit $?
  head -c 400 gpurun_out/lbw_$n.out; echo; grep -m2 "s3hc lb" gpurun_out/lbw_$n.err
done
for n in 1 16 64 256; do
  timeout -k 10 120 python tools/lb.py $n | cut -c1-200 || exit $?
  S3HC_LBW_DISABLE=1 timeout -k 10 120 python tools/lb.py $n | cut -c1-200 || exit $?
done
