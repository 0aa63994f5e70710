# Quick GPU check: the given test files (one process, per-test timeouts), then the bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quick.log 2>&1
rc=$?
tail -6 gpurun_out/quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'ratio', d['config']['compression_ratio']); print(d['kernel_ms_per_step']); print('whole decode frac', d['roofline_decode']['frac'], d['roofline_decode']['avg_launch_ms'])"
