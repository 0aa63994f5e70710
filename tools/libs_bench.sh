# Default bench line (no CPU leg) for the tree's library and each named diagnostic build, in turn.
# usage: bash tools/libs_bench.sh OUTDIR TAG... (TAG: build/diag/lib_TAG.so; "tree" = the tree's)
O=$1; shift
mkdir -p $O
for t in "$@"; do
  if [ "$t" = tree ]; then lib=""; else lib=$GRAFT_REPO_ROOT/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so; fi
  S3HC_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/$t.json 2> $O/$t.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open('$O/$t.json').read().strip().splitlines()[-1])
print('$t', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
