# pointer-jumping small launches (k_djump) + row-parallel frame close: GPU tests, then the reader
# (k_djump vs k_dsmall) and the batch decode A/B (default vs by-rank records vs five-wave k_dexec)
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoders.py tests/test_gpu_large.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/jump_tests.log 2>&1 || { tail -40 gpurun_out/jump_tests.log; exit 1; }
echo "jump: $(tail -1 gpurun_out/jump_tests.log)"
timeout -k 10 300 python -u tools/reader_time.py --mib 256 > gpurun_out/rt_jump.json 2>&1 || exit 1
S3HC_LIB_PATH=$L/build/diag/lib_dsmall.so timeout -k 10 300 python -u tools/reader_time.py --mib 256 > gpurun_out/rt_dsmall.json 2>&1 || exit 1
python3 -c "import json; a=json.load(open('gpurun_out/rt_jump.json')); b=json.load(open('gpurun_out/rt_dsmall.json')); print({k: (a[k]['GiBps'], b[k]['GiBps']) for k in a})"
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_bal1.so $L/build/diag/lib_dxh.so $L/libs3hc_lz4.so $L/build/diag/lib_bal1.so $L/build/diag/lib_dxh.so > gpurun_out/ab4.txt 2> gpurun_out/ab4.err || exit $?
cat gpurun_out/ab4.txt
