# kernel trace of one north-star config (graph off): args CONFIG BATCH [extra configs.py args]
set -o pipefail
export TMPDIR=/tmp
c=$1; b=$2; shift 2
O=gpurun_out/cfgprof_$c; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- \
  python3 -m vi_normflows_amd.bench.configs --config $c --batch $b --graph off --steps 5 --warmup 3 "$@" > $O/r.json 2> $O/r.err || { tail -20 $O/r.err; exit 1; }
cat $O/r.json
