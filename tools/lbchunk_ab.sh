#!/bin/bash
# A/B of the large-block tokenizing chunk size (diag builds): large-block tests on each library,
# then tools/lb.py at 1 / 16 / 256 frames, alternating libraries twice.
mkdir -p gpurun_out
for lib in sample-s3-hybrid-cache_amd/build/diag/lib_c8k.so sample-s3-hybrid-cache_amd/build/diag/lib_c4k.so; do
  S3HC_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tl_ab.log 2>&1
  rc=$?; echo "$lib tests rc=$rc"; tail -2 gpurun_out/tl_ab.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for lib in sample-s3-hybrid-cache_amd/libs3hc_lz4.so sample-s3-hybrid-cache_amd/build/diag/lib_c8k.so sample-s3-hybrid-cache_amd/build/diag/lib_c4k.so; do
    for n in 1 16 256; do
      S3HC_LIB_PATH=$lib timeout -k 10 120 python tools/lb.py $n > gpurun_out/ab_lb.out 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[0]); print(sys.argv[2].split('/')[-1], sys.argv[3], d['lb']['ms'], d['lb']['decode_kernels_ms'], d['lb']['check'])" gpurun_out/ab_lb.out $lib $n
    done
  done
done
