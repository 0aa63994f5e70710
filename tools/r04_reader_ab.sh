# range reader, fixed 256 KiB batches, 64 KiB frames: k_djump (default) vs k_dsmall vs the
# large-block path (S3HC_FAST=0), depth 3/4/6, two alternations
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out/rab
for i in 1 2; do
  timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/jump$i.json || exit 1
  S3HC_LIB_PATH=$L/build/diag/lib_dsmall.so timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/dsmall$i.json || exit 1
  S3HC_FAST=0 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only 64KiB --depths 3,4,6 > gpurun_out/rab/lb$i.json || exit 1
done
python3 - <<'PY'
import json
for v in ("jump", "dsmall", "lb"):
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/rab/{v}{i}.json"))
        print(v, i, {k.split("_")[-1]: d[k]["GiBps"] for k in d})
PY
