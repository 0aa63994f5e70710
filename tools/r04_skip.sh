# k_dtok record-pass ablation (diagnostic builds; the per-unit decoder decodes every block so the
# output stays right): kernel stats of k_dtok with no record stores / no token parse / neither
L=sample-s3-hybrid-cache_amd
R=$PWD
mkdir -p gpurun_out/skip
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  S3HC_LIB_PATH=$R/$L/build/diag/lib_skip$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/skip/s$v -o s -- python3 $R/tools/dec_repeat.py 10 > $R/gpurun_out/skip/s$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/skip/s$v/s_kernel_stats.csv')):
    if 'k_dtok' in r['Name']: print('skip$v k_dtok', round(float(r['AverageNs'])/1e3, 1), 'us')
"
done
