# range-reader tests (one-launch batches with corrupt payloads included)
timeout -k 10 400 python -u -m pytest tests/test_gpu_reader.py -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/rtest.log 2>&1
rc=$?
tail -12 gpurun_out/rtest.log
exit $rc
