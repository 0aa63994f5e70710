#!/bin/bash
# Kernel-time / ratio comparisons of diagnostic library builds (never shipped). Args: tags of
# sample-s3-hybrid-cache_amd/build/diag/lib_<tag>.so ("base" = the shipped library).
mkdir -p gpurun_out/abl
for t in "$@"; do
  lib=$PWD/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so
  [ "$t" = base ] && lib=$PWD/sample-s3-hybrid-cache_amd/libs3hc_lz4.so
  S3HC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/abl/$t.log 2>&1 || { echo "$t failed"; tail -3 gpurun_out/abl/$t.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abl/$t.log').read().strip().splitlines()[-1]);print('$t', d['value'], d['config']['compression_ratio'], d['kernel_ms_per_step'])"
done
