#!/bin/bash
# PMC passes over a short bench run (kernel-trace + counters only, no other traces).
# usage: tools/pmc.sh TAG  -> gpurun_out/pmc/TAG_{p1,p2}/...
TAG=${1:-pmc}
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc/${TAG}_p1 -o p1 -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/pmc/${TAG}_p1.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc/${TAG}_p2 -o p2 -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/pmc/${TAG}_p2.log 2>&1 || exit 1
echo pmc-done
