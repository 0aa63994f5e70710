# k_djump block checksum: loads double-buffered against the rounds (S3HC_HASH_DB=1) vs one batch of
# 32 loads then 32 rounds; phase timers (diagnostic builds) per block, two alternations
L=sample-s3-hybrid-cache_amd/build/diag
mkdir -p gpurun_out/hdb
for k in 1 2; do for v in h0 h1; do
  S3HC_LIB_PATH=$L/lib_$v.so timeout -k 10 120 python -u tools/fprof_small.py 11 > gpurun_out/hdb/$v.$k.json 2> gpurun_out/hdb/$v.$k.err || { tail -5 gpurun_out/hdb/$v.$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hdb/$v.$k.json')); print('$v', d['call_us'], d['djump_per_block'])"
done; done
