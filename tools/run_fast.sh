# GPU round trip for the fast decode path: its tests, the decoder suites, then the phase timers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_fast.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_fast.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # a crash or a timeout: nothing more on the GPU
S3HC_FAST=1 S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_fprof.so timeout -k 10 120 python3 tools/fprof.py > gpurun_out/fprof.json 2>&1 || { cat gpurun_out/fprof.json; exit 1; }
cat gpurun_out/fprof.json
exit $rc
