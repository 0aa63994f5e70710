# Whole GPU suite (one process, per-test timeouts), then the default bench line without the CPU leg.
# usage: bash tools/gpu_suite.sh [extra pytest args]
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --durations=12 -p no:cacheprovider "$@" > gpurun_out/suite.log 2>&1
rc=$?
tail -18 gpurun_out/suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'ratio', d['config']['compression_ratio']); print(d['kernel_ms_per_step']); print(d['roofline_decode'])"
