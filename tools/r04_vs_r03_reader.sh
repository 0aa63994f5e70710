# range reader at fixed 256 KiB batches: round-3 library + tools (git worktree r03ref at b998bdf,
# built in place) against HEAD on the same box, two alternations
mkdir -p gpurun_out/rr
for i in 1 2; do
  (cd r03ref && timeout -k 10 200 python -u tools/reader_time.py --mib 256) > gpurun_out/rr/r03_$i.json || exit 1
  timeout -k 10 200 python -u tools/reader_time.py --mib 256 > gpurun_out/rr/r04_$i.json || exit 1
done
python3 - <<'PY'
import json
for v in ("r03", "r04"):
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/rr/{v}_{i}.json"))
        print(v, i, {k: d[k]["GiBps"] for k in d})
PY
