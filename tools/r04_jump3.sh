# fused k_djump (1024-thread token index + pointer jumping): reader/fast/large tests, phase timers,
# reader A/B against k_dsmall and the large-block path
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out/rab
timeout -k 10 400 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py tests/test_gpu_large.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/j3_tests.log 2>&1 || { tail -30 gpurun_out/j3_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/j3_tests.log)"
S3HC_LIB_PATH=$L/build/diag/lib_fprof.so timeout -k 10 200 python -u tools/fprof_small.py 11 > gpurun_out/fj.json 2>&1 || { cat gpurun_out/fj.json; exit 1; }
python3 -c "import json; a=json.load(open('gpurun_out/fj.json')); print('jump', a['call_us'], a['djump_per_block'], a['dtok_per_wave_cycles'])"
for i in 1 2; do
  timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/jump$i.json || exit 1
  S3HC_LIB_PATH=$L/build/diag/lib_dsmall.so timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/dsmall$i.json || exit 1
  S3HC_FAST=0 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/lb$i.json || exit 1
done
python3 - <<'PY'
import json
for v in ("jump", "dsmall", "lb"):
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/rab/{v}{i}.json"))
        print(v, i, {k.split("_")[-1]: d[k]["GiBps"] for k in d})
PY
