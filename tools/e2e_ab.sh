#!/bin/bash
# A/B on one box of the config-4 e2e / reader rates of reference 1 MiB frames across library
# builds (build/diag/lib_<tag>.so; "new" = the in-tree library), spread execution off in all.
mkdir -p gpurun_out/eab
D=sample-s3-hybrid-cache_amd
for r in 1 2; do
  for tag in old 585a69d new; do
    lib=$D/build/diag/lib_$tag.so; [ $tag = new ] && lib=$D/libs3hc_lz4.so
    S3HC_LBW_DISABLE=1 S3HC_LIB_PATH=$lib timeout -k 10 300 python tools/e2e.py --skip-config2 > gpurun_out/eab/$tag.$r.json 2> gpurun_out/eab/$tag.$r.err || exit 1
    python -c "
import json,sys; d=json.load(open(sys.argv[1]))['config4']['ref_1MiB_frames']
print(sys.argv[2], {k.replace('reader_decode_GiBps_batch_','r_').replace('e2e_decode_GiBps_batch_','e_'): v for k, v in d.items() if 'GiBps' in k or 'check_batch' in k})" gpurun_out/eab/$tag.$r.json $tag
  done
done
