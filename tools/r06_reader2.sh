# Round 6: reader tests with batched verify launches (issued when the head batch needs its
# verdict), then the fixed-256 KiB reader against the round-6 library with one verify close per
# batch queue (build/ab/lib_c2.so), 1 and 2 batches per queue, alternated.
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_multidev.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/reader2_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/reader2_suite.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in head c2; do
    if [ $lib = c2 ]; then export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/ab/lib_c2.so; else unset S3HC_LIB_PATH; fi
    timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only ref --depths 3 --slots 1,2 --reps 2 > gpurun_out/r06/reader3_${lib}_${rep}.txt 2>&1 || exit $?
    echo "== $lib rep $rep"; grep "_depth" gpurun_out/r06/reader3_${lib}_${rep}.txt | grep -v '":'
  done
done
