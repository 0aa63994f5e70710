#!/bin/bash
# A/B of two libraries on the same box: decode/encode kernel ms at the given block counts,
# alternating A and B three times. usage: tools/ab.sh LIB_A LIB_B "1024 4096"
A=$1; B=$2; NB=${3:-4096}
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    for nb in $NB; do
      S3HC_LIB_PATH=$lib timeout -k 10 120 python bench.py --blocks $nb --steps 10 --warmup 3 --no-cpu-baseline --skip-check > gpurun_out/ab/$tag.$nb.$r.out 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print(sys.argv[2], sys.argv[3], 'decode', k['decode'], 'enc_parse', k['enc_parse'], 'enc_emit', k['enc_emit'], 'value', d['value'])" gpurun_out/ab/$tag.$nb.$r.out $tag $nb
    done
  done
done
