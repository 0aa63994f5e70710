# reader host-time accounting (S3HC_HOST_TRACE=1): per-batch host microseconds by stage
mkdir -p gpurun_out/rh
S3HC_HOST_TRACE=1 timeout -k 10 200 python -u tools/reader_time.py --mib 256 --depths 3,4 > gpurun_out/rh/rt.json 2> gpurun_out/rh/rt.err || exit 1
cat gpurun_out/rh/rt.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: v['GiBps'] for k, v in d.items()})"
grep "s3hc reader" gpurun_out/rh/rt.err
