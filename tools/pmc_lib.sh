#!/bin/bash
# PMC instruction counters of the bench's kernels for a (diagnostic) library: tools/pmc_lib.sh TAG LIB
TAG=$1; LIB=$2
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export S3HC_LIB_PATH=$R/$LIB
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc/${TAG} -o p1 -- python3 $R/bench.py --no-cpu-baseline --skip-check --steps 2 --warmup 1 > $R/gpurun_out/pmc/${TAG}.log 2>&1 || exit 1
echo pmc-lib-done
