#!/bin/bash
# A/B of k_lb_run's hops per jumping round (diag builds), step loop forced (S3HC_LBW_DISABLE=1):
# large-block tests on the h3 build, then tools/lb.py 1 / 256 per library, two alternations.
mkdir -p gpurun_out
D=sample-s3-hybrid-cache_amd
S3HC_LBW_DISABLE=1 S3HC_LIB_PATH=$D/build/diag/lib_h3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/th.log 2>&1
rc=$?; tail -1 gpurun_out/th.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for tag in h1 h2 h3 h4 h3r160; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = h1 ] && lib=$D/libs3hc_lz4.so
    for n in 1 256; do
      S3HC_LBW_DISABLE=1 S3HC_LIB_PATH=$lib timeout -k 10 120 python tools/lb.py $n > gpurun_out/hab.out 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[0]); print(sys.argv[2], sys.argv[3], d['lb']['ms'], d['lb']['decode_kernels_ms'], d['lb']['check'])" gpurun_out/hab.out $tag $n
    done
  done
done
