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
  TORCH_CHECK(saved.numel() == (long)K * N * D, "saved shape");
  nf_launch_planar_fwd(z.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                       B.data_ptr<float>(), zK.data_ptr<float>(), ldj.data_ptr<float>(),
                       saved.data_ptr<float>(), N, D, K, per_sample, broadcast, cur_stream());
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
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) {
  m.impl("planar_stack_fwd", &planar_stack_fwd);
  m.impl("planar_stack_bwd", &planar_stack_bwd);
  m.impl("radial_stack_fwd", &radial_stack_fwd);
  m.impl("radial_stack_bwd", &radial_stack_bwd);
}
