# kernel stats + two PMC passes of the default bench (kernel-trace only, no other traces)
mkdir -p gpurun_out/prof
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/ks -o ks -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 > $R/gpurun_out/prof/ks.log 2>&1 || exit 1
cd $R && bash tools/pmc.sh ${1:-rNN} && python3 tools/pmc_summary.py gpurun_out/pmc/${1:-rNN}_p1 gpurun_out/pmc/${1:-rNN}_p2 > gpurun_out/pmc/${1:-rNN}.json && echo prof-ok
