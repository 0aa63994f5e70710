#!/bin/bash
# HBM traffic per kernel dispatch (rocprofv3 PMC FETCH_SIZE / WRITE_SIZE, one counter per pass,
# kernel-trace only) over the default bench workload; summary -> gpurun_out/traffic/traffic.json.
# gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads (MI355X_MICROARCH.md, HBM).
mkdir -p gpurun_out/traffic
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/traffic/f -o f -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/traffic/f.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/traffic/w -o w -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/traffic/w.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/traffic/f gpurun_out/traffic/w > gpurun_out/traffic/traffic.json && echo traffic-ok
