# round-4 evidence for the other configs: config 5's per-GPU slice, config 3, the large-block
# table, the reader at fixed 256 KiB batches
mkdir -p gpurun_out/cfg
timeout -k 10 300 python -u bench.py --blocks 131072 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/bench_c5.json 2> gpurun_out/cfg/bench_c5.err || exit 1
tail -1 gpurun_out/cfg/bench_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['kernel_ms_per_step'], d['roofline_decode']['frac'])"
timeout -k 10 300 python -u tools/config3.py > gpurun_out/cfg/config3.json 2> gpurun_out/cfg/config3.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/cfg/config3.json')); print('c3', {k: d[k] for k in list(d)[:8]})"
timeout -k 10 300 python -u tools/lb.py > gpurun_out/cfg/lb_decode.json 2> gpurun_out/cfg/lb.err || exit 1
head -c 1500 gpurun_out/cfg/lb_decode.json; echo
timeout -k 10 300 python -u tools/reader_time.py --mib 256 --depths 3,4 > gpurun_out/cfg/reader.json 2> gpurun_out/cfg/reader.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/cfg/reader.json')); print('reader', {k: v['GiBps'] for k, v in d.items()})"
