# xxh32 chain forms, shipped library vs build/diag/lib_$ALT.so, alternating: one 1 MiB reference
# frame and 16 of them (device decode, tools/lb.py), the default bench line, the range reader on
# reference 1 MiB frames (fixed 256 KiB batches, depth 3, 256 MiB object).
mkdir -p gpurun_out/hab
for rep in 1 2; do
  for v in shipped $ALT; do
    if [ $v = shipped ]; then unset S3HC_LIB_PATH; else export S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$v.so; fi
    timeout -k 10 120 python -u tools/lb.py 1 > gpurun_out/hab/lb1_${v}_$rep.json || exit 1
    timeout -k 10 120 python -u tools/lb.py 16 > gpurun_out/hab/lb16_${v}_$rep.json || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/hab/bench_${v}_$rep.json || exit 1
    timeout -k 10 200 python -u tools/reader_time.py --mib 256 --only ref --depths 3 > gpurun_out/hab/reader_${v}_$rep.json 2>&1 || exit 1
  done
done
unset S3HC_LIB_PATH
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/hab/*.json")):
    t = open(f).read().strip().splitlines()
    if "bench" in f:
        d = json.loads(t[-1]); print(f.split("/")[-1], d["value"], d["kernel_ms_per_step"].get("dec_close"))
    elif "reader" in f:
        print(f.split("/")[-1], t[0])
    else:
        d = json.loads(t[0]); print(f.split("/")[-1], d["lb"])
PY
