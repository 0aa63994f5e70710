#!/bin/bash
# A/B of diag builds (build/diag/lib_<tag>.so; tag "head" = the in-tree library) on the
# large-block path: tools/lb.py at 1 frame on the step loop (S3HC_LBW_DISABLE=1) and 256 frames,
# two alternations. usage: tools/libs_ab.sh "head tagA tagB"
mkdir -p gpurun_out
D=sample-s3-hybrid-cache_amd
for r in 1 2; do
  for tag in $1; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = head ] && lib=$D/libs3hc_lz4.so
    for n in 1 256; do
      S3HC_LBW_DISABLE=1 S3HC_LIB_PATH=$lib timeout -k 10 120 python tools/lb.py $n > gpurun_out/lab.out 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[0]); print(sys.argv[2], sys.argv[3], d['lb']['ms'], d['lb']['decode_kernels_ms'], d['lb']['check'])" gpurun_out/lab.out $tag $n
    done
  done
done
