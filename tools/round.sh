#!/bin/bash
# Full GPU check: parity + golden (gpu), bench with CPU baseline, 2-rank torchrun rehearsal on one GPU,
# rocprofv3 kernel stats. Each GPU step has its own timeout; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -5 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err || { tail -5 gpurun_out/bench_2rank.err; exit 1; }
tail -1 gpurun_out/bench_2rank.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o rstats -- python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { tail -5 gpurun_out/prof_bench.err; exit 1; }

timeout -k 10 600 python tools/e2e.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -5 gpurun_out/e2e.err; exit 1; }
echo e2e-ok
timeout -k 10 300 python tools/compat.py > gpurun_out/compat.json 2> gpurun_out/compat.err || { tail -5 gpurun_out/compat.err; exit 1; }
echo round-ok
