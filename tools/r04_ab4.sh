# default (interleaved record pass, row-parallel close) vs by-rank records vs the five-wave k_dexec with a hashing wave
# tests first (the interleaved pass is new), then two alternations of the decode A/B
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoders.py tests/test_gpu_fullsize.py::test_config2_full_batch_every_frame_oracle -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t4_tests.log 2>&1 || { tail -30 gpurun_out/t4_tests.log; exit 1; }
echo "t4: $(tail -1 gpurun_out/t4_tests.log)"
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_bal1.so $L/build/diag/lib_dxh.so $L/libs3hc_lz4.so $L/build/diag/lib_bal1.so $L/build/diag/lib_dxh.so > gpurun_out/ab4.txt 2> gpurun_out/ab4.err || exit $?
cat gpurun_out/ab4.txt
