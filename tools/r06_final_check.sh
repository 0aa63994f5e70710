# Round 6: whole GPU suite at HEAD (one level of source redirection), the default bench line,
# and the phase timers of the shipped decode kernels.
mkdir -p gpurun_out/r06
bash tools/gpu_suite.sh || exit $?
S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_fprof1.so timeout -k 10 120 python -u tools/fprof.py > gpurun_out/r06/fprof_redirect1.json 2>&1 || exit $?
cat gpurun_out/r06/fprof_redirect1.json
