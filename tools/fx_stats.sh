# per-kernel average durations (rocprofv3 --kernel-trace --stats) of the config-2 decode, per library
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fxstats
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  lib=$R/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so
  [ "$t" = main ] && lib=$R/sample-s3-hybrid-cache_amd/libs3hc_lz4.so
  FX_INPROC=1 S3HC_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fxstats/$t -o s -- python3 $R/tools/fx_ablate.py > $R/gpurun_out/fxstats/$t.log 2>&1 || exit 1
  python3 - $R/gpurun_out/fxstats/$t $t <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
out = {}
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("s3hc::", "")
    if n.startswith("k_d"):
        out[n] = round(float(r["AverageNs"]) / 1e3, 1)
print(sys.argv[2], out)
PY
done
