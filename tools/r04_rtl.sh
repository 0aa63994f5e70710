# kernel + copy timeline of the reader (64 KiB frames, depth 4), no API trace
mkdir -p gpurun_out/rtl
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/rtl -o rt -- python3 $R/tools/reader_time.py --mib 64 --only 64KiB --depths 4 > $R/gpurun_out/rtl/run.log 2>&1 || exit 1
echo done
