// TORCH_LIBRARY fragment for the planar-flow VAE step (csrc/kernels/vae.hip).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include "launchers.h"

namespace {

constexpr int kH = 64;
constexpr long kMaxLds = 163840;   // what nf_launch_vae_step grants the rows kernel

// LDS bytes the rows kernel needs for (Din, dz, K): the engine gate (train.py, PlanarVAEEngine)
// and vae_step's own check use the same number
int64_t vae_rows_lds_bytes(int64_t Din, int64_t dz, int64_t K) {
  const long De = 2 * dz + 2 * dz * K + K;
  return (int64_t)nf_vae_rows_lds_bytes((int)Din, (int)dz, (int)K, (int)De);
}

void f32(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), n,
              " must be a contiguous fp32 GPU tensor");
}

// master / grad: flat fp32 buffers sharing one layout; offs: element offsets of
// [enc W_0..W_{L-1}, enc b_0..b_{L-1}, enc Wo, enc bo, dec W.., dec b.., dec Wo, dec bo]
void vae_step(const at::Tensor& master, const at::Tensor& grad, at::IntArrayRef offs,
              const at::Tensor& x, const c10::optional<at::Tensor>& eps, int64_t seed,
              const at::Tensor& offset, const at::Tensor& beta, int64_t B, int64_t Din,
              int64_t dz, int64_t K, int64_t L, const at::Tensor& ws, const at::Tensor& frow,
              const at::Tensor& loss, const c10::optional<at::Tensor>& zk_out,
              const c10::optional<at::Tensor>& ldj_out) {
  f32(master, "master"); f32(grad, "grad"); f32(x, "x"); f32(ws, "ws"); f32(frow, "frow");
  f32(loss, "loss"); f32(beta, "beta");
  TORCH_CHECK(offset.is_cuda() && offset.scalar_type() == at::kLong, "offset: int64 GPU scalar");
  TORCH_CHECK(L >= 1 && L <= 4 && dz >= 1 && dz <= 64 && K >= 0 && K <= 8 && Din % 4 == 0 &&
                  Din >= 4 && Din <= 1024 && dz % 4 == 0,
              "vae_step: 1 <= L <= 4, dz <= 64 (multiple of 4), K <= 8, Din % 4 == 0, Din <= 1024");
  TORCH_CHECK((long)offs.size() == 4 * L + 4, "vae_step: 4 L + 4 parameter offsets");
  TORCH_CHECK(master.numel() == grad.numel(), "master / grad layouts differ");
  const long De = 2 * dz + 2 * dz * K + K;
  const long ldg = (De + 3) & ~3L;   // gphi rows padded to 16 B (float4 loads of the wgrad phase)
  TORCH_CHECK(nf_vae_rows_lds_bytes((int)Din, (int)dz, (int)K, (int)De) <= kMaxLds,
              "vae_step: Din / dz / K need more than 160 KiB of LDS per row block "
              "(vinf::vae_rows_lds_bytes); use the module path");
  TORCH_CHECK(x.dim() == 2 && x.size(0) == B && x.size(1) == Din, "x must be [B, Din]");
  // parameter extents (out x in + out) for a bounds check of every offset
  std::vector<long> numel;
  for (int l = 0; l < L; ++l) numel.push_back((long)kH * (l == 0 ? Din : kH));
  for (int l = 0; l < L; ++l) numel.push_back(kH);
  numel.push_back(De * kH); numel.push_back(De);
  for (int l = 0; l < L; ++l) numel.push_back((long)kH * (l == 0 ? dz : kH));
  for (int l = 0; l < L; ++l) numel.push_back(kH);
  numel.push_back(Din * kH); numel.push_back(Din);
  for (size_t i = 0; i < numel.size(); ++i)
    TORCH_CHECK(offs[i] >= 0 && offs[i] % 4 == 0 && offs[i] + numel[i] <= master.numel(),
                "vae_step: parameter offset out of range / not 16-B aligned");
  const long need = 4L * L * B * kH + B * ldg + B * dz + B * Din;
  TORCH_CHECK(ws.numel() >= need, "vae_step: workspace too small");
  TORCH_CHECK(frow.numel() >= B && loss.numel() >= 1, "frow / loss");
  const float* eps_p = nullptr;
  if (eps && eps->defined()) {
    f32(*eps, "eps");
    TORCH_CHECK(eps->dim() == 2 && eps->size(0) == B && eps->size(1) == dz, "eps [B, dz]");
    eps_p = eps->data_ptr<float>();
  }
  float* zk_p = nullptr;
  float* ldj_p = nullptr;
  if (zk_out && zk_out->defined()) {
    f32(*zk_out, "zk_out");
    TORCH_CHECK(zk_out->numel() == B * dz, "zk_out [B, dz]");
    zk_p = zk_out->data_ptr<float>();
  }
  if (ldj_out && ldj_out->defined()) {
    f32(*ldj_out, "ldj_out");
    TORCH_CHECK(ldj_out->numel() == B, "ldj_out [B]");
    ldj_p = ldj_out->data_ptr<float>();
  }
  const float* P = master.data_ptr<float>();
  float* G = grad.data_ptr<float>();
  NfVaeParams prm{};
  NfVaeGrads grd{};
  int q = 0;
  for (int l = 0; l < L; ++l) { prm.enc_W[l] = P + offs[q]; grd.enc_W[l] = G + offs[q]; ++q; }
  for (int l = 0; l < L; ++l) { prm.enc_b[l] = P + offs[q]; grd.enc_b[l] = G + offs[q]; ++q; }
  prm.enc_Wo = P + offs[q]; grd.enc_Wo = G + offs[q]; ++q;
  prm.enc_bo = P + offs[q]; grd.enc_bo = G + offs[q]; ++q;
  for (int l = 0; l < L; ++l) { prm.dec_W[l] = P + offs[q]; grd.dec_W[l] = G + offs[q]; ++q; }
  for (int l = 0; l < L; ++l) { prm.dec_b[l] = P + offs[q]; grd.dec_b[l] = G + offs[q]; ++q; }
  prm.dec_Wo = P + offs[q]; grd.dec_Wo = G + offs[q]; ++q;
  prm.dec_bo = P + offs[q]; grd.dec_bo = G + offs[q]; ++q;
  float* w = ws.data_ptr<float>();
  const long BH = B * kH;
  float* eact = w;            w += L * BH;
  float* egrad = w;           w += L * BH;
  float* dact = w;            w += L * BH;
  float* dgrad = w;           w += L * BH;
  float* gphi = w;            w += B * ldg;
  float* zk = w;              w += B * dz;
  float* dl = w;
  nf_launch_vae_step(prm, x.data_ptr<float>(), eps_p, (unsigned)seed, offset.data_ptr<int64_t>(),
                     beta.data_ptr<float>(), (int)B, (int)Din, (int)dz, (int)K, (int)L, eact,
                     egrad, gphi, zk, dact, dgrad, dl, frow.data_ptr<float>(),
                     loss.data_ptr<float>(), zk_p, ldj_p, grd,
                     c10::hip::getCurrentHIPStream().stream());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(vinf, m) {
  m.def("vae_rows_lds_bytes(int Din, int dz, int K) -> int", &vae_rows_lds_bytes);
  m.def("vae_step(Tensor master, Tensor(a!) grad, int[] offs, Tensor x, Tensor? eps, int seed, "
        "Tensor offset, Tensor beta, int B, int Din, int dz, int K, int L, Tensor(b!) ws, "
        "Tensor(c!) frow, Tensor(d!) loss, Tensor(e!)? zk_out, Tensor(f!)? ldj_out) -> ()");
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) { m.impl("vae_step", &vae_step); }
