# one-launch small batches (k_djump + per-unit decoder + frame close): tests, reader rates, host
# accounting, kernel stats
R=$PWD
mkdir -p gpurun_out/fu
timeout -k 10 600 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoders.py tests/test_gpu_large.py tests/test_gpu_fullsize.py -k "not config5 and not config3" -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fu/tests.log 2>&1 || { tail -40 gpurun_out/fu/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/fu/tests.log)"
S3HC_HOST_TRACE=1 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --depths 3,4 > gpurun_out/fu/rt.json 2> gpurun_out/fu/rt.err || { tail -5 gpurun_out/fu/rt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/fu/rt.json')); print({k: v['GiBps'] for k, v in d.items()})"
grep "s3hc reader" gpurun_out/fu/rt.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fu/rk -o rk -- python3 $R/tools/reader_time.py --mib 64 --only 64KiB --depths 3 > $R/gpurun_out/fu/rk.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/fu/rk/rk_kernel_stats.csv')):
    if 'enc' in r['Name'] or 'scan' in r['Name'] or 'copyBuffer' in r['Name']: continue
    print(r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
"
