# forward product: ReLU bitmask stored (default) vs computed-not-stored (variant) vs no mask
set -o pipefail
O=gpurun_out/maskdiag; mkdir -p $O
L=vi_normflows_amd/_native/libvinf_hip_masknostore.so
for r in 1 2; do
  for lib in default masknostore; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$L; fi
    VINF_BENCH_TAG=$lib timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --iters 20 --only fwd_l1,fwd_l2,fwd_l2_nomask,dgrad_l2 >> $O/sg.jsonl || exit 1
  done
done
unset VINF_NATIVE_LIB
cat $O/sg.jsonl
