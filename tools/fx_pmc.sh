# VALU / SALU / LDS instruction counts of k_dtok and k_dexec per diagnostic library (phase ablation)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fxpmc
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  lib=$R/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so
  [ "$t" = main ] && lib=$R/sample-s3-hybrid-cache_amd/libs3hc_lz4.so
  FX_INPROC=1 S3HC_FAST=1 S3HC_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/fxpmc/$t -o p -- python3 $R/tools/fx_ablate.py > $R/gpurun_out/fxpmc/$t.log 2>&1 || exit 1
  python3 - $R/gpurun_out/fxpmc/$t $t <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_dexec" in k or "k_dtok" in k:
        acc[k.split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    w = d["SQ_WAVES"] or 1
    print(sys.argv[2], k, {c: round(v / w) for c, v in d.items() if c != "SQ_WAVES"}, "waves", int(w))
PY
done
