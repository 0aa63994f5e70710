# Round evidence in one GPU call: smoke, the default bench line (with the CPU baseline), rocprofv3
# kernel stats + two PMC passes + the FETCH/WRITE traffic passes of the same bench command, config 3,
# config 5's per-GPU slice, the large-block table, the range reader and per-GET latency.
# usage: bash tools/evidence.sh TAG   -> gpurun_out/evidence/...
T=${1:-rNN}
O=gpurun_out/evidence
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
tail -1 $O/bench_default.json
bash tools/prof_bench.sh $T || exit 1
cp gpurun_out/prof/ks/ks_kernel_stats.csv $O/kernel_stats_bench.csv 2>/dev/null || find gpurun_out/prof/ks -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bench.csv \;
cp gpurun_out/pmc/$T.json $O/pmc_bench.json
bash tools/traffic.sh || exit 1
cp gpurun_out/traffic/traffic.json $O/traffic.json
timeout -k 10 300 python -u tools/config3.py > $O/config3.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --blocks 131072 --steps 3 --warmup 1 > $O/bench_config5_slice_131072.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/lb.py > $O/lb_decode.json 2> $O/lb_decode.err || exit 1
timeout -k 10 300 python -u tools/reader_time.py --mib 256 --depths 3,4 --reps 3 > $O/reader_fixed256k.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/reader_small.py 200 1024 > $O/reader_small_1MiB.json 2>&1 || exit 1
timeout -k 10 200 python -u tools/reader_small.py 50 8192 > $O/reader_small_8MiB.json 2>&1 || exit 1
timeout -k 10 400 python -u tools/e2e.py --gib 8 > $O/e2e.json 2> $O/e2e.err || exit 1
echo evidence-ok
