#!/bin/bash
# kernel stats of the large-block path at 1 and 16 reference frames, new tokenizer vs lib_oldtok
mkdir -p gpurun_out/lbs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 1 16; do
  rm -rf gpurun_out/lbs/new$n gpurun_out/lbs/old$n
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/lbs/new$n -o run -- python3 tools/lb.py $n > gpurun_out/lbs/new$n.log 2>&1 || exit $?
  S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_oldtok.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/lbs/old$n -o run -- python3 tools/lb.py $n > gpurun_out/lbs/old$n.log 2>&1 || exit $?
done
for n in 1 16; do python3 tools/lb_kstats.py gpurun_out/lbs/new$n/run_results.db gpurun_out/lbs/old$n/run_results.db; done
