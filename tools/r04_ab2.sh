# decode variants A/B (two alternations) + tests of the interleaved record pass; encoder variants;
# reader timeline
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_bal.so $L/build/diag/lib_bal2.so $L/libs3hc_lz4.so $L/build/diag/lib_bal.so $L/build/diag/lib_bal2.so > gpurun_out/ab2.txt 2> gpurun_out/ab2.err || exit $?
cat gpurun_out/ab2.txt
S3HC_LIB_PATH=$L/build/diag/lib_bal2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoders.py tests/test_gpu_fullsize.py::test_config2_full_batch_every_frame_oracle -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bal2_tests.log 2>&1
echo "bal2: $(tail -1 gpurun_out/bal2_tests.log)"
bash tools/r04_enc_ab.sh $L/build/diag/lib_sgate.so $L/build/diag/lib_lazy.so $L/build/diag/lib_sgl.so || exit $?
bash tools/reader_trace.sh || exit $?
