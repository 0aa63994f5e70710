# Large-block path at 256 x 1 MiB: phase timers of the diagnostic build (lib_prof, S3HC_DIAG_LEVEL=10),
# two SQ PMC passes and the FETCH_SIZE / WRITE_SIZE passes over the tree's library (kernel-trace +
# counters only).
# usage: bash tools/lb_pmc.sh -> gpurun_out/lbpmc/
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lbpmc
mkdir -p $O
S3HC_LIB_PATH=$R/sample-s3-hybrid-cache_amd/build/diag/lib_prof.so timeout -k 10 200 python3 $R/tools/lb.py 256 > $O/phases.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/lb.py 256 > $O/p1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU --output-format csv -d $O/p2 -o p2 -- python3 $R/tools/lb.py 256 > $O/p2.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- python3 $R/tools/lb.py 256 > $O/f.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python3 $R/tools/lb.py 256 > $O/w.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $O/p1 $O/p2 > $O/pmc.json
python3 $R/tools/pmc_summary.py $O/f $O/w > $O/traffic.json
echo lbpmc-done
