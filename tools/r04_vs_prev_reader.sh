# range reader at fixed 256 KiB batches: HEAD against the round-3 build (r03ref) and the previous
# round-4 commit (r04prev: k_djump with separate per-unit and close launches), same box, 2 alternations
mkdir -p gpurun_out/rr2
for i in 1 2; do
  (cd r03ref && timeout -k 10 200 python -u tools/reader_time.py --mib 256) > gpurun_out/rr2/r03_$i.json || exit 1
  (cd r04prev && timeout -k 10 200 python -u tools/reader_time.py --mib 256) > gpurun_out/rr2/prev_$i.json || exit 1
  timeout -k 10 200 python -u tools/reader_time.py --mib 256 > gpurun_out/rr2/head_$i.json || exit 1
done
python3 - <<'PY'
import json
for v in ("r03", "prev", "head"):
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/rr2/{v}_{i}.json"))
        print(v, i, {k: d[k]["GiBps"] for k in d})
PY
