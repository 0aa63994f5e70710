# tools/lb.py N (one case: N frames of 1 MiB) for the tree's library and named diagnostic builds,
# alternated R times; prints device ms per decode of each run.
# usage: bash tools/lb_libs.sh N R TAG... ("tree" = the tree's library)
N=$1; R=$2; shift 2
O=gpurun_out/lblibs; mkdir -p $O
for r in $(seq 1 $R); do
  for t in "$@"; do
    if [ "$t" = tree ]; then lib=""; else lib=$GRAFT_REPO_ROOT/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so; fi
    S3HC_LIB_PATH=$lib timeout -k 10 120 python3 tools/lb.py $N > $O/${t}_$r.txt 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$O/${t}_$r.txt').readline()); print('$t', $r, d['lb']['ms'], d['lb']['decode_kernels_ms'], d['lb']['check'])"
  done
done
