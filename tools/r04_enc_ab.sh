# Encoder A/B: bench line (value, enc_parse, ratio) for the shipped library and variants, alternated
# (summary lines in gpurun_out/encab_summary.txt); then the config-2 every-frame oracle check and
# the parity tests on each variant, and compressed sizes of a few inputs per library
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
: > gpurun_out/encab_summary.txt
for rep in 1 2; do
for lib in $L/libs3hc_lz4.so "$@"; do
  S3HC_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/encab.json 2>gpurun_out/encab.err || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/encab.json').read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], d['value'], 'parse', d['kernel_ms_per_step']['enc_parse'], 'emit', d['kernel_ms_per_step']['enc_emit'], 'dec', d['kernel_ms_per_step']['decode'], 'ratio', d['config']['compression_ratio'])" $lib | tee -a gpurun_out/encab_summary.txt
done
done
for lib in "$@"; do
  S3HC_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py::test_config2_full_batch_every_frame_oracle tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/encab_tests.log 2>&1
  echo "$lib: $(tail -1 gpurun_out/encab_tests.log)" | tee -a gpurun_out/encab_summary.txt
done
timeout -k 10 300 python -u tools/ratio_cmp.py $L/libs3hc_lz4.so "$@" > gpurun_out/ratio_cmp.json 2>&1 || exit $?
