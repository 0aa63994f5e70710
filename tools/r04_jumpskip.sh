# k_djump jumping rounds that skip final pairs (S3HC_JUMP_SKIP=1, the default build) vs every pair
# every round: phase timers (diagnostic builds j0 / j1, two alternations), then smoke, the whole -m gpu
# suite and the bench line on the default build
L=sample-s3-hybrid-cache_amd/build/diag
mkdir -p gpurun_out/jsk
for k in 1 2; do for v in j0 j1; do
  S3HC_LIB_PATH=$L/lib_$v.so timeout -k 10 120 python -u tools/fprof_small.py 11 > gpurun_out/jsk/$v.$k.json 2> gpurun_out/jsk/$v.$k.err || { tail -5 gpurun_out/jsk/$v.$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/jsk/$v.$k.json')); print('$v', d['call_us'], d['djump_per_block'])"
done; done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/jsk/smoke.log 2>&1 || { tail -20 gpurun_out/jsk/smoke.log; exit 1; }
tail -1 gpurun_out/jsk/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 900 --timeout-method thread --durations=8 -p no:cacheprovider > gpurun_out/jsk/suite.log 2>&1 || { tail -30 gpurun_out/jsk/suite.log; exit 1; }
tail -1 gpurun_out/jsk/suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/jsk/bench.json 2> gpurun_out/jsk/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/jsk/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['kernel_ms_per_step'], d['roofline_decode']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u tools/reader_time.py --mib 256 --depths 3 --reps 2 > gpurun_out/jsk/reader.txt 2> gpurun_out/jsk/reader.err || exit 1
grep -v "^ \|^{\|^}" gpurun_out/jsk/reader.txt
