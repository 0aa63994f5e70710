# one call: focused parity + A/B of the working tree against build/diag/lib_old.so, then the full
# GPU suite and the round's profile set
timeout -k 10 500 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_decoders.py tests/test_gpu_parity.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/sc2.log 2>&1; rc=$?; tail -3 gpurun_out/sc2.log; [ $rc -ne 0 ] && exit $rc
LIBS="old" AB_REPS="1 2 3" bash tools/lib_ab.sh || exit $?
bash tools/r03_suite.sh && bash tools/r03_prof.sh
