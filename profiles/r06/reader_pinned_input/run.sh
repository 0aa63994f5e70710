# Round 6 A/B: reader input buffer pinned (batches copied to the device straight out of it, no
# staging copy) vs round 6's earlier library (c2: pageable input + staging copy).
# Counter: host us/batch (stage 12 us -> 0) and fixed-256 KiB GiB/s, 64 KiB and reference frames.
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_multidev.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_large.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/pin_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/pin_suite.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for t in head c2; do
    case $t in head) unset S3HC_LIB_PATH;; c2) export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/ab/lib_c2.so;; esac
    S3HC_HOST_TRACE=1 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --depths 3 > gpurun_out/r06/pin_${t}_${rep}.txt 2>&1 || exit $?
    echo "== $t $rep"; grep -v "^ \|^{\|^}" gpurun_out/r06/pin_${t}_${rep}.txt
  done
done
