#!/bin/bash
# phase timers of the segment-walk tokenizer (diag builds lib_<tag>.so with S3HC_DIAG_LEVEL=10) at 1 and 256 frames
for t in $PLIBS; do for n in 1 256; do
  echo "== $t $n"; S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$t.so timeout -k 10 100 python tools/lb.py $n | grep -E "walk_phases|frames" | cut -c1-300 || exit 1
done; done
