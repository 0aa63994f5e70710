#!/bin/bash
# A/B of AMDGPU scheduler options on the bench kernels (diag builds lib_<tag>.so vs the in-tree
# library), bench at 4096 blocks, two alternations.
mkdir -p gpurun_out/sab
D=sample-s3-hybrid-cache_amd
for r in 1 2; do
  for tag in head $1; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = head ] && lib=$D/libs3hc_lz4.so
    S3HC_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sab/$tag.$r.out 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print(sys.argv[2], 'decode', k['decode'], 'enc_parse', k['enc_parse'], 'enc_emit', k['enc_emit'], 'value', d['value'])" gpurun_out/sab/$tag.$r.out $tag
  done
done
