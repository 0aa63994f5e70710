# round-4 evidence: default bench line (with the CPU baseline), rocprofv3 kernel stats of the same
# command, two PMC passes and the FETCH/WRITE traffic passes
mkdir -p gpurun_out/final
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
tail -1 gpurun_out/final/bench.json
bash tools/r04_prof.sh r04 || exit 1
bash tools/traffic.sh || exit 1
echo final-ok
