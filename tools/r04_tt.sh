# k_dtok workgroup size A/B: 256 (default) vs 512 vs 1024 speculative segments; fast-path tests on 1024
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
S3HC_LIB_PATH=$L/build/diag/lib_tt1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_fullsize.py::test_config2_full_batch_every_frame_oracle -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tt_tests.log 2>&1 || { tail -30 gpurun_out/tt_tests.log; exit 1; }
echo "tt1024 tests: $(tail -1 gpurun_out/tt_tests.log)"
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_tt512.so $L/build/diag/lib_tt1024.so $L/libs3hc_lz4.so $L/build/diag/lib_tt512.so $L/build/diag/lib_tt1024.so > gpurun_out/tt.txt 2> gpurun_out/tt.err || exit 1
cat gpurun_out/tt.txt
