# instruction counters of k_enc_parse: run-end pass vs every-position pass (shipped library)
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in sparse dense; do
  if [ $v = dense ]; then export S3HC_ENC_DENSE=1; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc/enc_$v -o p1 -- python3 $R/bench.py --no-cpu-baseline --skip-check --steps 2 --warmup 1 > $R/gpurun_out/pmc/enc_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc/enc2_$v -o p2 -- python3 $R/bench.py --no-cpu-baseline --skip-check --steps 2 --warmup 1 > $R/gpurun_out/pmc/enc2_$v.log 2>&1 || exit 1
done
cd $R
for v in sparse dense; do python3 tools/pmc_summary.py gpurun_out/pmc/enc_$v gpurun_out/pmc/enc2_$v > gpurun_out/pmc/enc_$v.json; python3 -c "
import json; d=json.load(open('gpurun_out/pmc/enc_$v.json')); d=[c for k,c in d.items() if 'enc_parse' in k][0]; print('$v', {k: round(v/4096) for k,v in d.items()})"; done
