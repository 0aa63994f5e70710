#!/bin/bash
# A/B: spread execution also for 64 KiB blocks (diag build ml0) vs HEAD: small-work probe and the
# config-4 reader / e2e, alternating twice; large-block tests on ml0 first.
mkdir -p gpurun_out/mab
D=sample-s3-hybrid-cache_amd
for lib in $D/libs3hc_lz4.so $D/build/diag/lib_ml0.so; do
  S3HC_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_reader.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mab/t.log 2>&1
  rc=$?; tail -1 gpurun_out/mab/t.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python tools/lb.py 1 | cut -c1-160 || exit 1
timeout -k 10 120 python tools/lb.py 16 | cut -c1-160 || exit 1
for r in 1 2; do
  for tag in head ml0; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = head ] && lib=$D/libs3hc_lz4.so
    S3HC_LIB_PATH=$lib timeout -k 10 200 python tools/small.py > gpurun_out/mab/s.$tag.$r.json 2>&1 || exit 1
    S3HC_LIB_PATH=$lib timeout -k 10 300 python tools/e2e.py --skip-config2 > gpurun_out/mab/e.$tag.$r.json 2>&1 || exit 1
    python -c "
import json,sys
s=json.load(open(sys.argv[1]))['gpu_64KiB_frames']; e=json.load(open(sys.argv[2]))['config4']['gpu_64KiB_frames']
print(sys.argv[3], 'dev_n1', s['dev_n1']['lb']['wall_ms'], 'dev_n4', s['dev_n4']['lb']['wall_ms'], 'dev_n10', s['dev_n10']['lb']['wall_ms'], 'host1MiB', s['host_decompress_1MiB_ms'],
      {k.replace('reader_decode_GiBps_batch_','r_').replace('e2e_decode_GiBps_batch_','e_'): v for k, v in e.items() if 'GiBps' in k and 'device' not in k})" gpurun_out/mab/s.$tag.$r.json gpurun_out/mab/e.$tag.$r.json $tag
  done
done
