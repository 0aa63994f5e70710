# after cleanup: decoder/reader tests, bench line, reader host-time accounting, reader kernel stats
R=$PWD
mkdir -p gpurun_out/chk
timeout -k 10 500 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoders.py tests/test_gpu_reader.py tests/test_gpu_large.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/chk/tests.log 2>&1 || { tail -30 gpurun_out/chk/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/chk/tests.log)"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/chk/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['kernel_ms_per_step'])"
S3HC_HOST_TRACE=1 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --depths 3,4 > gpurun_out/chk/rt.json 2> gpurun_out/chk/rt.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/chk/rt.json')); print({k: v['GiBps'] for k, v in d.items()})"
grep "s3hc reader" gpurun_out/chk/rt.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/chk/rk -o rk -- python3 $R/tools/reader_time.py --mib 64 --only 64KiB > $R/gpurun_out/chk/rk.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/chk/rk/rk_kernel_stats.csv')):
    if 'enc' in r['Name'] or 'scan' in r['Name'] or 'copyBuffer' in r['Name']: continue
    print(r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
"
