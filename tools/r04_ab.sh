# A/B of decode variants (tools/fx_ablate.py: config-2 decode time per library, alternated),
# the LDS store probe, phase timers of the fast path, and the fast-path tests on the variants
mkdir -p gpurun_out
timeout -k 10 60 tools/probe/ual_lds_w || exit $?
L=sample-s3-hybrid-cache_amd
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_hop1.so $L/build/diag/lib_lit32.so $L/build/diag/lib_bal.so $L/libs3hc_lz4.so $L/build/diag/lib_hop1.so $L/build/diag/lib_lit32.so $L/build/diag/lib_bal.so > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
tail -1 gpurun_out/ab.json
S3HC_LIB_PATH=$L/build/diag/lib_fprof.so timeout -k 10 200 python -u tools/fprof.py > gpurun_out/fprof.json 2>&1 || exit $?
cat gpurun_out/fprof.json
for v in lit32 bal; do
S3HC_LIB_PATH=$L/build/diag/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${v}_tests.log 2>&1
echo "$v: $(tail -1 gpurun_out/${v}_tests.log)"
done
