# batch decode A/B (default: by-rank records, 16-lane frame close) vs 4-lane close vs interleaved
# records; then kernel stats of the 64 KiB-frame reader with k_djump (default) and k_dsmall
L=sample-s3-hybrid-cache_amd
R=$PWD
mkdir -p gpurun_out/rk
timeout -k 10 500 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_close4.so $L/build/diag/lib_bal2.so $L/libs3hc_lz4.so $L/build/diag/lib_close4.so $L/build/diag/lib_bal2.so > gpurun_out/ab5.txt 2> gpurun_out/ab5.err || exit $?
cat gpurun_out/ab5.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rk/jump -o rk -- python3 $R/tools/reader_time.py --mib 64 --only 64KiB > $R/gpurun_out/rk/jump.log 2>&1 || exit 1
S3HC_LIB_PATH=$R/$L/build/diag/lib_dsmall.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rk/dsmall -o rk -- python3 $R/tools/reader_time.py --mib 64 --only 64KiB > $R/gpurun_out/rk/dsmall.log 2>&1 || exit 1
echo rk-ok
