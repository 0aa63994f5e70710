# fast-path phase timers (diag build)
mkdir -p gpurun_out
S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_fprof.so timeout -k 10 120 python -u tools/fprof.py > gpurun_out/fprof.json 2>&1; rc=$?; cat gpurun_out/fprof.json; exit $rc
