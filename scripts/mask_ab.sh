# forward product: branch-free ReLU-bitmask bits (default) vs the compare/select form (maskold)
set -o pipefail
O=gpurun_out/maskab; mkdir -p $O
L=vi_normflows_amd/_native/libvinf_hip_maskold.so
for r in 1 2; do
  for lib in default maskold; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$L; fi
    VINF_BENCH_TAG=$lib timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --iters 20 --only fwd_l1,fwd_l2,fwd_l2_nomask,dgrad_l2 >> $O/sg.jsonl || exit 1
  done
done
unset VINF_NATIVE_LIB
cat $O/sg.jsonl
