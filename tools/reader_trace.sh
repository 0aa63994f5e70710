# Timeline of the fixed-256 KiB range reader (kernel + copy + HIP API traces, no counters)
# usage: tools/reader_trace.sh [DIR] [reader_time.py args...]
D=${1:-rtrace}
shift
mkdir -p gpurun_out/$D
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/$D -o rt -- python3 $R/tools/reader_time.py --mib 64 "$@" > $R/gpurun_out/$D/run.log 2>&1 || exit 1
ls -R $R/gpurun_out/$D | head
