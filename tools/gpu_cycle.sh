bash tools/run_fast.sh && bash tools/run_pmc_fast.sh && S3HC_FAST=1 timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fast.json 2> gpurun_out/bench_fast.err && python3 -c "
import json
d=json.loads(open('gpurun_out/bench_fast.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms_per_step'])"
