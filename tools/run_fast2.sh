# bench A/B of the fast decode path (S3HC_FAST=1) against the per-unit decoder, rocprof stats of the fast one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_slow.json 2> gpurun_out/bench_slow.err || exit $?
S3HC_FAST=1 timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fast.json 2> gpurun_out/bench_fast.err || exit $?
python3 -c "
import json
for n in ('slow','fast'):
    d=json.loads(open('gpurun_out/bench_%s.json'%n).read().strip().splitlines()[-1]); print(n, d['value'], d['kernel_ms_per_step'])"
S3HC_FAST=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fast -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_fast.log 2>&1 || exit $?
python3 tools/dbstats.py gpurun_out/prof_fast/run_results.db 2>/dev/null | head -12 || find gpurun_out/prof_fast -name "*stats*"
