# k_djump phase timers (diag build) vs k_dsmall's, the reader with both, reader tests
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
S3HC_LIB_PATH=$L/build/diag/lib_fprof.so timeout -k 10 200 python -u tools/fprof_small.py 11 > gpurun_out/fj.json 2>&1 || { cat gpurun_out/fj.json; exit 1; }
S3HC_LIB_PATH=$L/build/diag/lib_fprofs.so timeout -k 10 200 python -u tools/fprof_small.py 11 > gpurun_out/fs.json 2>&1 || exit 1
python3 -c "import json; a=json.load(open('gpurun_out/fj.json')); b=json.load(open('gpurun_out/fs.json')); print('jump', a['call_us'], a['djump_per_block'], a['dtok_per_wave_cycles']['total']); print('small', b['call_us'], b['dexec_per_block']['total'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/j2_tests.log 2>&1 || { tail -30 gpurun_out/j2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/j2_tests.log)"
timeout -k 10 300 python -u tools/reader_time.py --mib 256 --only 64KiB > gpurun_out/rt_jump.json 2>&1 || exit 1
S3HC_LIB_PATH=$L/build/diag/lib_dsmall.so timeout -k 10 300 python -u tools/reader_time.py --mib 256 --only 64KiB > gpurun_out/rt_dsmall.json 2>&1 || exit 1
python3 -c "import json; a=json.load(open('gpurun_out/rt_jump.json')); b=json.load(open('gpurun_out/rt_dsmall.json')); print({k: (a[k]['GiBps'], b[k]['GiBps']) for k in a})"
