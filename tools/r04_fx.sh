# k_dexec phase ablation (diagnostic builds with S3HC_FXSKIP: output wrong, timing only): decode
# time without the in-window gathers (1), literals (2), round 0 (4), flushes (16), two alternations
L=sample-s3-hybrid-cache_amd
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/fx_ablate.py $L/libs3hc_lz4.so $L/build/diag/lib_fx1.so $L/build/diag/lib_fx2.so $L/build/diag/lib_fx4.so $L/build/diag/lib_fx16.so $L/libs3hc_lz4.so $L/build/diag/lib_fx1.so $L/build/diag/lib_fx2.so $L/build/diag/lib_fx4.so $L/build/diag/lib_fx16.so > gpurun_out/fx.txt 2> gpurun_out/fx.err || exit 1
cat gpurun_out/fx.txt
