# Round 6 A/B in one GPU call (same box), bench lines alternated 3x:
#   head    content hash on a second queue beside the match finder + k_dexec source redirection (3 levels)
#   red1    the same with 1 redirection level, red2 with 2
#   redir0  the same without redirection
#   r05     round 5's library (in-grid content hash, no redirection)
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_encode_mode.py tests/test_gpu_fullsize.py tests/test_gpu_writer.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/ab_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r06/ab_suite.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for t in head red1 red2 redir0 r05; do
    case $t in head) unset S3HC_LIB_PATH;; r05) export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/ab/lib_r05.so;; *) export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$t.so;; esac
    timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06/ab_bench_${t}_${rep}.json 2>gpurun_out/r06/ab_bench_${t}_${rep}.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06/ab_bench_${t}_${rep}.json').read().strip().splitlines()[-1]); print('$t', $rep, d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
  done
done
