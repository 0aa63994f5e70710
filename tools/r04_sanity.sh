# sanity at HEAD after rebuilding the verified source: smoke and the decoder test files
mkdir -p gpurun_out/san
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/san/smoke.log 2>&1 || { tail -20 gpurun_out/san/smoke.log; exit 1; }
tail -1 gpurun_out/san/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_reader.py tests/test_gpu_fast.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/san/tests.log 2>&1 || { tail -30 gpurun_out/san/tests.log; exit 1; }
tail -1 gpurun_out/san/tests.log
