#!/bin/bash
# PMC passes over a short bench run (kernel-trace only + counters, no other traces).
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S3HC_LIB_PATH=$PWD/sample-s3-hybrid-cache_amd/build/diag/libs3hc_lz4_diag.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --skip-check > gpurun_out/pmc/ablate_nowalk.log 2>&1 || echo "ablate failed" >> gpurun_out/pmc/ablate_nowalk.log
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc -o p1 -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o p2 -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc/p2.log 2>&1 || exit 1
echo pmc-done
