#!/bin/bash
# Kernel-time ablations with diagnostic library builds (never shipped). Args: tags.
mkdir -p gpurun_out/abl
for t in "$@"; do
  S3HC_LIB_PATH=$PWD/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --skip-check > gpurun_out/abl/$t.log 2>&1 || { echo "$t failed"; tail -3 gpurun_out/abl/$t.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abl/$t.log').read().strip().splitlines()[-1]);print('$t', d['kernel_ms_per_step'])"
done
