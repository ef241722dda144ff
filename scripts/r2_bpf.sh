set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bpf
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_persistent_gpu.py tests/test_masked_gpu.py tests/test_fp8_gpu.py tests/test_maf_engine.py tests/test_realnvp_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bpf/pytest.log 2>&1 || { tail -30 gpurun_out/bpf/pytest.log; exit 1; }
tail -1 gpurun_out/bpf/pytest.log
bash scripts/ab_lib.sh bpf_ab nobpf fwd_l2,wgrad_l2,wgrad_group,sq4096
