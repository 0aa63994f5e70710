# Range reader: batches in flight per queue (S3HC_READER_SLOTS) A/B at depth 3, fixed 256 KiB
# batches, 512 MiB object, both frame sizes; then the reader tests (the new test sweeps the knob)
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/reader_time.py --mib 512 --depths 3 --slots 1,2,3 --reps 2 > gpurun_out/slots.txt 2> gpurun_out/slots.err || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reader.py > gpurun_out/slots_tests.log 2>&1 || { tail -30 gpurun_out/slots_tests.log; exit 1; }
tail -2 gpurun_out/slots_tests.log
grep -v "^ \|^{\|^}" gpurun_out/slots.txt
