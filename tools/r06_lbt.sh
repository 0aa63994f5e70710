#!/bin/bash
# Round 6: large-block tokenizer by segment walks (S3HC_LB_TOKV2=1, shipped) against diag builds
# (LIBS tags: build/diag/lib_<tag>.so, e.g. oldtok = the rounds 1-5 tokenizer): large-block +
# reader tests on the shipped library, then lb.py timings (same box, alternated), then rocprofv3
# kernel stats at 1 and 256 reference frames for the shipped library.
mkdir -p gpurun_out/lbt
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_reader.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/lbt/tests.log 2>&1
rc=$?; tail -3 gpurun_out/lbt/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u tools/lb.py > gpurun_out/lbt/lb_new_$rep.json 2> gpurun_out/lbt/lb_new_$rep.err || exit $?
  for t in $LIBS; do
    S3HC_LIB_PATH=sample-s3-hybrid-cache_amd/build/diag/lib_$t.so timeout -k 10 200 python -u tools/lb.py > gpurun_out/lbt/lb_${t}_$rep.json 2> gpurun_out/lbt/lb_${t}_$rep.err || exit $?
  done
done
python3 - $LIBS <<'PY'
import json, sys
for rep in (1, 2):
    for t in ["new"] + sys.argv[1:]:
        d = json.load(open(f"gpurun_out/lbt/lb_{t}_{rep}.json"))
        print("%-7s %d " % (t, rep) + " ".join("%s %.3f" % (k.replace("log_", ""), v["lb"]["ms"]) for k, v in d.items()))
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 1 256; do
  rm -rf gpurun_out/lbt/p$n
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lbt/p$n -o run -- python3 tools/lb.py $n > gpurun_out/lbt/p$n.log 2>&1 || exit $?
  python3 tools/lb_kstats.py gpurun_out/lbt/p$n/run_results.db | grep -E "lbt|lb_seq|lb_gran|lb_run"
done
