# Bench A/B of the shipped library against diagnostic builds, same box, alternating:
#   LIBS="tagA tagB" bash tools/lib_ab.sh   (build/diag/lib_<tag>.so)
mkdir -p gpurun_out
run() {  # name [lib]
    local name=$1 lib=$2
    if [ -n "$lib" ]; then export S3HC_LIB_PATH=$lib; else unset S3HC_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${AB_STEPS:-20} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || return $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1])
k=d['kernel_ms_per_step']; print('%-10s value %.1f ratio %.4f ' % ('$name', d['value'], d['config']['compression_ratio']) + ' '.join('%s %.4f' % (a, b) for a, b in k.items()))"
}
for rep in ${AB_REPS:-1 2}; do
  run shipped || exit $?
  for v in $LIBS; do run $v sample-s3-hybrid-cache_amd/build/diag/lib_$v.so || exit $?; done
done
