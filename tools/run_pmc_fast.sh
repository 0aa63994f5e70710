# PMC passes of the fast decode path (S3HC_FAST=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export S3HC_FAST=1
bash tools/pmc.sh fast > gpurun_out/pmc_fast.log 2>&1 || { tail -5 gpurun_out/pmc_fast.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc/fast_p1 gpurun_out/pmc/fast_p2 > gpurun_out/pmc_fast.json
python3 -c "
import json
d=json.load(open('gpurun_out/pmc_fast.json'))
for k in ('k_dtok','k_dexec'):
    print(k, {c: round(v) for c,v in d[k].items()})"
