# headline-step A/B of the default library vs a variant .so (arg: variant name), alternating
set -o pipefail
v=$1; L=vi_normflows_amd/_native/libvinf_hip_$v.so
O=gpurun_out/libab_$v; mkdir -p $O
for r in 1 2 3; do
  for lib in default $v; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$L; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
unset VINF_NATIVE_LIB
cat $O/ab.jsonl
