# round-4 closing run with the workgroup-precomputed checksum products in k_djump: smoke, the whole
# -m gpu suite, the default bench line, the config-4 reader (256 KiB batches, depth 3, 256 MiB)
mkdir -p gpurun_out/fin3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin3/smoke.log 2>&1 || { tail -20 gpurun_out/fin3/smoke.log; exit 1; }
tail -1 gpurun_out/fin3/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 900 --timeout-method thread --durations=8 -p no:cacheprovider > gpurun_out/fin3/suite.log 2>&1 || { tail -30 gpurun_out/fin3/suite.log; exit 1; }
tail -1 gpurun_out/fin3/suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/fin3/bench.json 2> gpurun_out/fin3/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/fin3/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['kernel_ms_per_step'], d['roofline_decode']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u tools/reader_time.py --mib 256 --depths 3 --reps 2 > gpurun_out/fin3/reader.txt 2> gpurun_out/fin3/reader.err || exit 1
grep -v "^ \|^{\|^}" gpurun_out/fin3/reader.txt
