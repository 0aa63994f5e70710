for t in head pipe0 redir0; do
  if [ $t = head ]; then unset S3HC_LIB_PATH; else export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$t.so; fi
  echo "== $t"; timeout -k 10 120 python -u tools/dbg_redir.py 2>&1 | head -60 || exit 1
done
