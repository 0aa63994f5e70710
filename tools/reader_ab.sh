# Range reader A/B, alternating: shipped library vs build/diag/lib_$ALT.so, 256 MiB objects,
# fixed 256 KiB batches, depths $DEPTHS, both frame layouts (tools/reader_time.py)
mkdir -p gpurun_out/rab
for rep in 1 2; do
  for v in shipped $ALT; do
    if [ $v = shipped ]; then unset S3HC_LIB_PATH; else export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$v.so; fi
    timeout -k 10 300 python -u tools/reader_time.py --mib 256 --depths ${DEPTHS:-3,6} > gpurun_out/rab/${v}_$rep.txt 2>&1 || exit 1
    echo "== $v $rep"; grep GiBps gpurun_out/rab/${v}_$rep.txt | grep -v "^ "
  done
done
