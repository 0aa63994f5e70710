mkdir -p gpurun_out/r05
for t in ${TAGS:-base abl1 abl2 abl3 walk2 base}; do
  lib=$PWD/sample-s3-hybrid-cache_amd/build/diag/lib_$t.so
  [ "$t" = base ] && lib=$PWD/sample-s3-hybrid-cache_amd/libs3hc_lz4.so
  S3HC_LIB_PATH=$lib timeout -k 10 120 python -u tools/enc_time.py --tag $t $ARGS >> gpurun_out/r05/abl.txt 2>&1 || exit 1
done
cat gpurun_out/r05/abl.txt
