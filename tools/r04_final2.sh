# round-4 closing run (after the done-counter clear fix): the reader tests twice (the slot-sweep test
# found the race), smoke, the whole -m gpu suite, the default bench line
mkdir -p gpurun_out/fin
for k in 1 2; do timeout -k 10 300 python -u -m pytest tests/test_gpu_reader.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fin/reader$k.log 2>&1 || { tail -30 gpurun_out/fin/reader$k.log; exit 1; }; tail -1 gpurun_out/fin/reader$k.log; done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin/smoke.log 2>&1 || { tail -20 gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 900 --timeout-method thread --durations=8 -p no:cacheprovider > gpurun_out/fin/suite.log 2>&1 || { tail -30 gpurun_out/fin/suite.log; exit 1; }
tail -1 gpurun_out/fin/suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/fin/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['kernel_ms_per_step'], d['roofline_decode']['frac'], d['cpu_baseline']['value'])"
