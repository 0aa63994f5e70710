# Round-4 combined GPU call: suite + bench, decode variant A/B + phase timers, config-4 reader, profiles
bash tools/r04_suite.sh || exit $?
bash tools/r04_ab.sh || exit $?
bash tools/r04_enc_ab.sh sample-s3-hybrid-cache_amd/build/diag/lib_lazy.so sample-s3-hybrid-cache_amd/build/diag/lib_sgate.so sample-s3-hybrid-cache_amd/build/diag/lib_sgl.so || exit $?
timeout -k 10 400 python -u tools/reader_time.py --mib 512 > gpurun_out/reader_time.json 2> gpurun_out/reader_time.err || exit $?
cat gpurun_out/reader_time.json
bash tools/r04_prof.sh ${1:-r04} || exit $?
