# encoder probe-stride A/B: bench line (ratio, enc_parse ms) of the shipped library and diag variants
mkdir -p gpurun_out/psab
for t in main "$@"; do
  lib=sample-s3-hybrid-cache_amd/build/diag/lib_$t.so
  [ "$t" = main ] && lib=sample-s3-hybrid-cache_amd/libs3hc_lz4.so
  S3HC_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/psab/$t.json 2> gpurun_out/psab/$t.err || { tail -5 gpurun_out/psab/$t.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/psab/$t.json').read().strip().splitlines()[-1])
print('$t', d['value'], 'ratio', d['config']['compression_ratio'], d['kernel_ms_per_step'])"
done
