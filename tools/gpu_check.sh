#!/bin/bash
# One GPU round trip: parity tests + bench (used from gpurun). Each step has its own timeout.
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -q --timeout 200 --maxfail 40 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/t1.log
tail -4 gpurun_out/t1.log | grep -E "^E |passed|failed|exit"
# 0 = pass, 1 = test failures; anything else (timeout, abort, segfault) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "bench exit $?" >> gpurun_out/bench.err
python -c "
import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'ratio', d['config']['compression_ratio']); print(d['kernel_ms_per_step']); print(d['roofline'])" || tail -5 gpurun_out/bench.err
