#!/bin/bash
# Round-2 secondary measurements at HEAD: end-to-end / config 4, large-block decode, config 3,
# compat encoder. Each step has its own timeout; stops at the first failure.
out=gpurun_out/r02sec
mkdir -p $out
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$out/$name.json" 2> "$out/$name.err"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$name.err"; exit $rc; }; }
step lb 300 python tools/lb.py
step config3 400 python tools/config3.py
step compat 300 python tools/compat.py
step e2e 600 python tools/e2e.py
step small 300 python tools/small.py
echo sec-ok
