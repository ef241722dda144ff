// TORCH_LIBRARY fragment for the fused planar / radial stacks.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include "launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), n,
              " must be a contiguous fp32 GPU tensor");
}

void planar_stack_fwd(const at::Tensor& z, const at::Tensor& W, const at::Tensor& U,
                      const at::Tensor& B, bool per_sample, bool broadcast, const at::Tensor& zK,
                      const at::Tensor& ldj, const at::Tensor& saved) {
  for (auto* p : {&z, &W, &U, &B, &zK, &ldj, &saved}) chk(*p, "planar arg");
  const int N = z.size(0), D = z.size(1), K = W.size(0);
  TORCH_CHECK(D <= 1024, "planar kernel supports D <= 1024");
  TORCH_CHECK(per_sample ? (W.dim() == 3 && W.size(1) == N && W.size(2) == D && B.numel() == (long)K * N)
                         : (W.dim() == 2 && W.size(1) == D && B.numel() == K),
              "planar parameter shapes");
  TORCH_CHECK(U.sizes() == W.sizes(), "U/W shape");
  // saved may be empty: the shared-parameter recompute backward needs no stored states
  TORCH_CHECK(saved.numel() == (long)K * N * D || saved.numel() == 0, "saved shape");
  nf_launch_planar_fwd(z.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                       B.data_ptr<float>(), zK.data_ptr<float>(), ldj.data_ptr<float>(),
                       saved.numel() ? saved.data_ptr<float>() : nullptr, N, D, K, per_sample,
                       broadcast, cur_stream());
}

int64_t planar_shared_workspace(int64_t N, int64_t D, int64_t K) {
  const int per = nf_planar_shared_per((int)D);
  if (per == 0 || K * per > 256) return -1;   // not eligible: generic saved-state path
  return (int64_t)nf_planar_shared_blocks((int)N) * K * (2 * per + 1);
}

void planar_stack_bwd_shared(const at::Tensor& z0, const at::Tensor& W, const at::Tensor& U,
                             const at::Tensor& B, bool broadcast, const at::Tensor& gz,
                             const at::Tensor& gl, const at::Tensor& dz, const at::Tensor& dW,
                             const at::Tensor& dU, const at::Tensor& dB, const at::Tensor& part) {
  for (auto* p : {&z0, &W, &U, &B, &gz, &gl, &dz, &dW, &dU, &dB, &part}) chk(*p, "planar arg");
  const int N = z0.size(0), D = z0.size(1), K = W.size(0);
  TORCH_CHECK(W.dim() == 2 && W.size(1) == D && U.sizes() == W.sizes() && B.numel() == K,
              "shared planar parameter shapes");
  TORCH_CHECK(gz.sizes() == z0.sizes() && dz.sizes() == z0.sizes() && gl.numel() == N,
              "planar gradient shapes");
  TORCH_CHECK(dW.numel() == (long)K * D && dU.numel() == (long)K * D && dB.numel() == K,
              "shared planar gradient shapes");
  const int64_t need = planar_shared_workspace(N, D, K);
  TORCH_CHECK(need > 0, "shared planar backward needs D <= 16 and K * per(D) <= 256");
  TORCH_CHECK(part.numel() >= need, "planar partial workspace too small");
  nf_launch_planar_bwd_shared(z0.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                              B.data_ptr<float>(), gz.data_ptr<float>(), gl.data_ptr<float>(),
                              dz.data_ptr<float>(), dW.data_ptr<float>(), dU.data_ptr<float>(),
                              dB.data_ptr<float>(), part.data_ptr<float>(),
                              nf_planar_shared_blocks(N), N, D, K, broadcast, cur_stream());
}

void planar_stack_bwd(const at::Tensor& saved, const at::Tensor& W, const at::Tensor& U,
                      const at::Tensor& B, bool per_sample, bool broadcast, const at::Tensor& gz,
                      const at::Tensor& gl, const at::Tensor& dz, const at::Tensor& dW,
                      const at::Tensor& dU, const at::Tensor& dB) {
  for (auto* p : {&saved, &W, &U, &B, &gz, &gl, &dz, &dW, &dU, &dB}) chk(*p, "planar arg");
  const int K = saved.size(0), N = saved.size(1), D = saved.size(2);
  TORCH_CHECK(dW.numel() == (long)K * N * D && dU.numel() == dW.numel() && dB.numel() == (long)K * N,
              "gradient buffer shapes");
  nf_launch_planar_bwd(saved.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                       B.data_ptr<float>(), gz.data_ptr<float>(), gl.data_ptr<float>(),
                       dz.data_ptr<float>(), dW.data_ptr<float>(), dU.data_ptr<float>(),
                       dB.data_ptr<float>(), N, D, K, per_sample, broadcast, cur_stream());
}

void radial_stack_fwd(const at::Tensor& z, const at::Tensor& Z0, const at::Tensor& A,
                      const at::Tensor& Bt, bool per_sample, const at::Tensor& zK,
                      const at::Tensor& ldj, const at::Tensor& saved) {
  for (auto* p : {&z, &Z0, &A, &Bt, &zK, &ldj, &saved}) chk(*p, "radial arg");
  const int N = z.size(0), D = z.size(1), K = Z0.size(0);
  TORCH_CHECK(D <= 1024, "radial kernel supports D <= 1024");
  TORCH_CHECK(per_sample ? (Z0.dim() == 3 && A.numel() == (long)K * N) : (Z0.dim() == 2 && A.numel() == K),
              "radial parameter shapes");
  TORCH_CHECK(A.numel() == Bt.numel(), "alpha/beta shapes");
  nf_launch_radial_fwd(z.data_ptr<float>(), Z0.data_ptr<float>(), A.data_ptr<float>(),
                       Bt.data_ptr<float>(), zK.data_ptr<float>(), ldj.data_ptr<float>(),
                       saved.data_ptr<float>(), N, D, K, per_sample, cur_stream());
}

void radial_stack_bwd(const at::Tensor& saved, const at::Tensor& Z0, const at::Tensor& A,
                      const at::Tensor& Bt, bool per_sample, const at::Tensor& gz,
                      const at::Tensor& gl, const at::Tensor& dz, const at::Tensor& dZ0,
                      const at::Tensor& dA, const at::Tensor& dBt) {
  for (auto* p : {&saved, &Z0, &A, &Bt, &gz, &gl, &dz, &dZ0, &dA, &dBt}) chk(*p, "radial arg");
  const int K = saved.size(0), N = saved.size(1), D = saved.size(2);
  nf_launch_radial_bwd(saved.data_ptr<float>(), Z0.data_ptr<float>(), A.data_ptr<float>(),
                       Bt.data_ptr<float>(), gz.data_ptr<float>(), gl.data_ptr<float>(),
                       dz.data_ptr<float>(), dZ0.data_ptr<float>(), dA.data_ptr<float>(),
                       dBt.data_ptr<float>(), N, D, K, per_sample, cur_stream());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(vinf, m) {
  m.def("planar_stack_fwd(Tensor z, Tensor W, Tensor U, Tensor B, bool per_sample, bool broadcast, "
        "Tensor(a!) zK, Tensor(b!) ldj, Tensor(c!) saved) -> ()");
  m.def("planar_stack_bwd(Tensor saved, Tensor W, Tensor U, Tensor B, bool per_sample, "
        "bool broadcast, Tensor gz, Tensor gl, Tensor(a!) dz, Tensor(b!) dW, Tensor(c!) dU, "
        "Tensor(d!) dB) -> ()");
  m.def("radial_stack_fwd(Tensor z, Tensor Z0, Tensor A, Tensor B, bool per_sample, "
        "Tensor(a!) zK, Tensor(b!) ldj, Tensor(c!) saved) -> ()");
  m.def("radial_stack_bwd(Tensor saved, Tensor Z0, Tensor A, Tensor B, bool per_sample, "
        "Tensor gz, Tensor gl, Tensor(a!) dz, Tensor(b!) dZ0, Tensor(c!) dA, Tensor(d!) dB) -> ()");
  m.def("planar_shared_workspace(int N, int D, int K) -> int", &planar_shared_workspace);
  m.def("planar_stack_bwd_shared(Tensor z0, Tensor W, Tensor U, Tensor B, bool broadcast, "
        "Tensor gz, Tensor gl, Tensor(a!) dz, Tensor(b!) dW, Tensor(c!) dU, Tensor(d!) dB, "
        "Tensor(e!) part) -> ()");
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) {
  m.impl("planar_stack_fwd", &planar_stack_fwd);
  m.impl("planar_stack_bwd", &planar_stack_bwd);
  m.impl("planar_stack_bwd_shared", &planar_stack_bwd_shared);
  m.impl("radial_stack_fwd", &radial_stack_fwd);
  m.impl("radial_stack_bwd", &radial_stack_bwd);
}
