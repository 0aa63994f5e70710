#!/bin/bash
# A/B of hops per doubling level in k_lb_exit / k_lb_mark (diag builds): large-block tests on
# x2 and x3, then tools/lb.py 1 / 256 per library, two alternations.
mkdir -p gpurun_out
D=sample-s3-hybrid-cache_amd
for tag in x2 x3; do
  S3HC_LIB_PATH=$D/build/diag/lib_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tx.log 2>&1
  rc=$?; echo "$tag $(tail -1 gpurun_out/tx.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for tag in x1 x2 x3; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = x1 ] && lib=$D/libs3hc_lz4.so
    for n in 1 256; do
      S3HC_LIB_PATH=$lib timeout -k 10 120 python tools/lb.py $n > gpurun_out/xab.out 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[0]); print(sys.argv[2], sys.argv[3], d['lb']['ms'], d['lb']['decode_kernels_ms'], d['lb']['check'])" gpurun_out/xab.out $tag $n
    done
  done
done
