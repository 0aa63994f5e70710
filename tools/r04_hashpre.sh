# k_djump block checksum: stripe products by the whole workgroup into LDS (S3HC_HASH_PRE=1, h2) vs
# the four lanes multiplying their own words (h0); phase timers (diagnostic builds) per block, two
# alternations; then the reader / fast-path tests on the h2 build
L=sample-s3-hybrid-cache_amd/build/diag
mkdir -p gpurun_out/hpre
for k in 1 2; do for v in h0 h2; do
  S3HC_LIB_PATH=$L/lib_$v.so timeout -k 10 120 python -u tools/fprof_small.py 11 > gpurun_out/hpre/$v.$k.json 2> gpurun_out/hpre/$v.$k.err || { tail -5 gpurun_out/hpre/$v.$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hpre/$v.$k.json')); print('$v', d['call_us'], d['djump_per_block'])"
done; done
S3HC_LIB_PATH=$L/lib_h2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hpre/tests.log 2>&1 || { tail -30 gpurun_out/hpre/tests.log; exit 1; }
tail -1 gpurun_out/hpre/tests.log
