# kernel trace of the config-5 step, fp8 and bf16 (graph off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/f8prof; mkdir -p $O
for pr in fp8 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$pr -o run --output-format csv -- \
    python3 -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch 32768 --graph off --steps 4 --warmup 3 > $O/$pr.json 2> $O/$pr.err || { tail -20 $O/$pr.err; exit 1; }
done
