# Round-4 check: full GPU suite, bench line, config-4 reader timing, kernel stats + PMC of the bench
bash tools/r04_suite.sh || exit $?
timeout -k 10 300 python -u tools/reader_time.py --mib 512 > gpurun_out/reader_time.json 2> gpurun_out/reader_time.err || exit $?
cat gpurun_out/reader_time.json
bash tools/r04_prof.sh ${1:-r04} || exit $?
