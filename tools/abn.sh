#!/bin/bash
# A/B/n of libraries on one box (enc/dec kernel ms at 4096 blocks, 2 rounds, plus the ratio).
# usage: tools/abn.sh LIB...
mkdir -p gpurun_out/abn
for r in 1 2; do
  for lib in "$@"; do
    t=$(basename $lib .so)
    S3HC_LIB_PATH=$lib timeout -k 10 120 python bench.py --blocks 4096 --steps 10 --warmup 3 --no-cpu-baseline --skip-check > gpurun_out/abn/$t.$r.out 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print(sys.argv[2], 'enc_parse', k['enc_parse'], 'emit', k['enc_emit'], 'decode', k['decode'], 'ratio', d['config']['compression_ratio'], 'value', d['value'])" gpurun_out/abn/$t.$r.out $t
  done
done
