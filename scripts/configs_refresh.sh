# Final-tree refresh of the north-star configs on one box (bench.configs, one process each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_configs; mkdir -p $O
for args in "--config 0 --batch 128" "--config 0 --batch 1024" "--config 0 --impl module --batch 1024" \
            "--config 2 --batch 32768" "--config 3 --batch 16384" \
            "--config 4 --batch 8192" "--config 4 --impl module --batch 8192" \
            "--config 5 --precision bf16 --batch 32768" "--config 5 --precision fp8 --batch 32768"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args >> $O/configs.jsonl 2>> $O/configs.err || { echo "FAIL $args"; tail -20 $O/configs.err; exit 1; }
  tail -1 $O/configs.jsonl | cut -c1-300
done
