# Encoder A/B: frames byte-identical (sha of tools/frames_sha.py inputs) and bench lines,
# shipped library against build/diag/lib_<tag>.so, alternating. usage: LIBS="tag" bash tools/enc_ab.sh
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/frames_sha.py > gpurun_out/sha_shipped.txt || exit 1
for v in $LIBS; do
  S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$v.so timeout -k 10 120 python -u tools/frames_sha.py > gpurun_out/sha_$v.txt || exit 1
done
head -1 gpurun_out/sha_*.txt
bash tools/lib_ab.sh
