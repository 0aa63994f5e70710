# Cost of the bench's HIP events: shipped library (adjacent phases share events), a build with one
# event pair per phase (build/diag/lib_ev12.so), and no events in the timed steps; alternating.
mkdir -p gpurun_out/tab
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/tab/ev8_$rep.json || exit 1
  S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_ev12.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/tab/ev12_$rep.json || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --no-kernel-timing > gpurun_out/tab/none_$rep.json || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["kernel_ms_per_step"])
PY
