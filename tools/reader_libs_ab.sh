# range-reader A/B over diagnostic builds, alternating, same box: LIBS="a b" bash tools/reader_libs_ab.sh
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in shipped $LIBS; do
    if [ $v = shipped ]; then unset S3HC_LIB_PATH; else export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$v.so; fi
    timeout -k 10 200 python -u tools/reader_time.py --mib ${RT_MIB:-1024} > gpurun_out/rtab_$v.json 2>&1 || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/rtab_$v.json')); print('%-8s' % '$v', ' '.join('%s %.2f' % (k, x['GiBps']) for k,x in d.items()))"
  done
done
