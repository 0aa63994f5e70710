mkdir -p gpurun_out/p1 gpurun_out/p16 gpurun_out/p256
timeout -k 10 60 ./tools/probe/xxh_chain > gpurun_out/xxh_chain.out 2>&1; cat gpurun_out/xxh_chain.out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/p1 -o run -- python3 tools/lb.py 1 > gpurun_out/p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/p256 -o run -- python3 tools/lb.py 256 > gpurun_out/p256.log 2>&1
echo rc=$?
