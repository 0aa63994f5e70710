# Round 6: GPU suite at HEAD, then the fixed-256 KiB reader (64 KiB frames and the reference's
# 1 MiB frames) for round 5's library and HEAD, alternated on one box.
mkdir -p gpurun_out/r06
bash tools/gpu_suite.sh || exit $?
for rep in 1 2; do
  for lib in r05 head; do
    if [ $lib = r05 ]; then export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/ab/lib_r05.so; else unset S3HC_LIB_PATH; fi
    timeout -k 10 200 python -u tools/reader_time.py --mib 256 --depths 3,4 > gpurun_out/r06/reader_${lib}_${rep}.txt 2>&1 || exit $?
    echo "== $lib rep $rep"; tail -6 gpurun_out/r06/reader_${lib}_${rep}.txt
  done
done
# phase timers of the 64 KiB-block decoder (diagnostic build, S3HC_DIAG_LEVEL=10)
S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_fprof.so timeout -k 10 120 python -u tools/fprof.py > gpurun_out/r06/fprof_head.json 2>&1 || exit $?
cat gpurun_out/r06/fprof_head.json
