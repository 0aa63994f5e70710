# reader tests (one-launch batches with corrupt payloads), then the k_dtok record-pass ablation
bash tools/r04_rtest.sh || exit 1
bash tools/r04_skip.sh || exit 1
