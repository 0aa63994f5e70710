#!/bin/bash
# A/B on one box: config-4 reader/e2e rates with the pre-spread library (build/diag/lib_old.so)
# and HEAD, alternating; large-block tests and timings at HEAD first.
mkdir -p gpurun_out/rab
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_reader.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rab/tl.log 2>&1
rc=$?; tail -2 gpurun_out/rab/tl.log; [ $rc -eq 0 ] || exit $rc
for n in 1 16 256; do timeout -k 10 120 python tools/lb.py $n | cut -c1-140 || exit 1; done
for r in 1 2; do
  for tag in old new; do
    lib=sample-s3-hybrid-cache_amd/libs3hc_lz4.so; [ $tag = old ] && lib=sample-s3-hybrid-cache_amd/build/diag/lib_old.so
    S3HC_LIB_PATH=$lib timeout -k 10 300 python tools/e2e.py --skip-config2 > gpurun_out/rab/$tag.$r.json 2> gpurun_out/rab/$tag.$r.err || exit 1
    python -c "
import json,sys; d=json.load(open(sys.argv[1]))['config4']
print(sys.argv[2], {f: {k.replace('reader_decode_GiBps_batch_','r_').replace('e2e_decode_GiBps_batch_','e_'): v for k, v in d[f].items() if 'GiBps' in k and 'device' not in k} for f in d if isinstance(d[f], dict)})" gpurun_out/rab/$tag.$r.json $tag
  done
done
