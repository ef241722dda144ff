// TORCH_LIBRARY registration for the vi_normflows_amd HIP kernels.
//
// Every op is a mutating, allocation-free launcher on the current HIP stream,
// so whole training steps built from them can be captured into a hipGraph.
// Tensors are row-major 2-D views whose leading dimension is stride(0);
// inner stride must be 1. Kernels live in csrc/kernels/*.hip and are exposed
// as plain C launchers declared in launchers.h.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <sstream>
#include <vector>
#include <stdexcept>

#include "launchers.h"

void nf_throw_hip_error(hipError_t e, const char* expr, const char* file, int line) {
  std::ostringstream os;
  os << "HIP error " << hipGetErrorString(e) << " at " << file << ":" << line << " (" << expr << ")";
  throw std::runtime_error(os.str());
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

void check_2d(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, name, " must have unit inner stride");
}

void check_dtype(const at::Tensor& t, at::ScalarType s, const char* name) {
  TORCH_CHECK(t.scalar_type() == s, name, " has dtype ", t.scalar_type(), ", expected ", s);
}

template <typename T>
T* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

long ld_of(const at::Tensor& t) { return t.size(0) <= 1 && t.dim() == 2 ? t.size(1) : t.stride(0); }

// ---------------------------------------------------------------- coupling
void coupling_fwd(const at::Tensor& st, const at::Tensor& x, const at::Tensor& y,
                  const c10::optional<at::Tensor>& ybf, const c10::optional<at::Tensor>& ssav,
                  const at::Tensor& ldj, double scale, bool inverse, bool ldj_init) {
  check_2d(st, "st");
  check_2d(x, "x");
  check_2d(y, "y");
  check_dtype(x, at::kFloat, "x");
  check_dtype(y, at::kFloat, "y");
  check_dtype(ldj, at::kFloat, "ldj");
  const int B = x.size(0), Dh = x.size(1);
  TORCH_CHECK(st.size(0) == B && st.size(1) >= 2 * Dh, "st shape mismatch");
  TORCH_CHECK(y.size(0) == B && y.size(1) == Dh, "y shape mismatch");
  TORCH_CHECK(ldj.numel() == B && ldj.is_contiguous(), "ldj must be contiguous [B]");
  TORCH_CHECK(st.scalar_type() == at::kBFloat16 || st.scalar_type() == at::kFloat, "st dtype");
  long ld_yb = 0, ld_s = 0;
  if (ybf && ybf->defined()) {
    check_2d(*ybf, "ybf");
    TORCH_CHECK(ybf->scalar_type() == at::kBFloat16 || ybf->scalar_type() == at::kFloat, "ybf dtype");
    TORCH_CHECK(ybf->size(0) == B && ybf->size(1) >= Dh, "ybf shape");
    ld_yb = ld_of(*ybf);
  }
  if (ssav && ssav->defined()) {
    check_2d(*ssav, "ssav");
    check_dtype(*ssav, at::kFloat, "ssav");
    TORCH_CHECK(ssav->size(0) == B && ssav->size(1) == Dh, "ssav shape");
    ld_s = ld_of(*ssav);
  }
  const int yb_cols = (ybf && ybf->defined()) ? ybf->size(1) : 0;
  // the kernel pads ybf up to its logical width, not its stride
  nf_launch_coupling_fwd(st.data_ptr(), st.scalar_type() == at::kBFloat16, ld_of(st),
                         x.data_ptr<float>(), ld_of(x), y.data_ptr<float>(), ld_of(y),
                         opt_ptr<void>(ybf),
                         ybf && ybf->defined() && ybf->scalar_type() == at::kBFloat16, ld_yb,
                         opt_ptr<float>(ssav), ld_s,
                         ldj.data_ptr<float>(), B, Dh, (float)scale, inverse, ldj_init, yb_cols,
                         cur_stream());
}

void coupling_bwd(const at::Tensor& gy, const at::Tensor& s, const at::Tensor& x, double c,
                  const c10::optional<at::Tensor>& c_row, const at::Tensor& dst,
                  const at::Tensor& gx, double scale, bool gx_accumulate) {
  check_2d(gy, "gy");
  check_2d(s, "s");
  check_2d(x, "x");
  check_2d(dst, "dst");
  check_2d(gx, "gx");
  check_dtype(gy, at::kFloat, "gy");
  const bool shat = s.scalar_type() == at::kBFloat16;   // s_hat (bf16 conditioner output)
  TORCH_CHECK(shat || s.scalar_type() == at::kFloat, "s: fp32 s or bf16 s_hat");
  check_dtype(x, at::kFloat, "x");
  check_dtype(gx, at::kFloat, "gx");
  TORCH_CHECK(dst.scalar_type() == at::kBFloat16 || dst.scalar_type() == at::kFloat, "dst dtype");
  const int B = x.size(0), Dh = x.size(1);
  TORCH_CHECK(gy.size(0) == B && gy.size(1) == Dh && s.size(0) == B && s.size(1) == Dh, "shape");
  TORCH_CHECK(gx.size(0) == B && gx.size(1) == Dh, "gx shape");
  TORCH_CHECK(dst.size(0) == B && dst.size(1) >= 2 * Dh, "dst shape");
  if (c_row && c_row->defined()) {
    check_dtype(*c_row, at::kFloat, "c_row");
    TORCH_CHECK(c_row->numel() == B && c_row->is_contiguous(), "c_row");
  }
  TORCH_CHECK(!shat || (Dh % 4 == 0 && ld_of(s) % 4 == 0 &&
                        reinterpret_cast<uintptr_t>(s.data_ptr()) % 8 == 0),
              "s_hat input needs Dh % 4 == 0 and 8-B aligned rows");
  nf_launch_coupling_bwd(s.data_ptr(), shat, ld_of(s), gy.data_ptr<float>(), ld_of(gy),
                         x.data_ptr<float>(), ld_of(x), (float)c, opt_ptr<float>(c_row),
                         dst.data_ptr(), dst.scalar_type() == at::kBFloat16, ld_of(dst),
                         gx.data_ptr<float>(), ld_of(gx), B, Dh,
                         (float)scale, gx_accumulate, (int)dst.size(1), cur_stream());
}

// ---------------------------------------------------------------- ELBO
void target_logp_grad(int64_t kind, const at::Tensor& A, const at::Tensor& Bh,
                      const c10::optional<at::Tensor>& gA, const c10::optional<at::Tensor>& gB,
                      bool grad_accumulate, const c10::optional<at::Tensor>& params, double p0,
                      double p1, double p2, double cst, const c10::optional<at::Tensor>& beta,
                      double beta_host, double row_weight, const c10::optional<at::Tensor>& logq0,
                      const c10::optional<at::Tensor>& ldj, const c10::optional<at::Tensor>& logp_out,
                      const c10::optional<at::Tensor>& frow_out) {
  check_2d(A, "A");
  check_2d(Bh, "B");
  check_dtype(A, at::kFloat, "A");
  check_dtype(Bh, at::kFloat, "B");
  const int B = A.size(0), Dh = A.size(1);
  TORCH_CHECK(Bh.size(0) == B && Bh.size(1) == Dh, "halves must match");
  TORCH_CHECK(kind >= 0 && kind <= 2, "unknown target kind");
  if (kind == 0) {
    TORCH_CHECK(params && params->defined() && params->numel() == 4 * Dh, "gaussian params [2D]");
  }
  long ldga = 0, ldgb = 0;
  if (gA && gA->defined()) {
    TORCH_CHECK(gB && gB->defined(), "gA and gB go together");
    check_2d(*gA, "gA");
    check_2d(*gB, "gB");
    ldga = ld_of(*gA);
    ldgb = ld_of(*gB);
  }
  nf_launch_target_logp_grad((int)kind, A.data_ptr<float>(), ld_of(A), Bh.data_ptr<float>(),
                             ld_of(Bh), opt_ptr<float>(gA), ldga, opt_ptr<float>(gB), ldgb,
                             grad_accumulate, opt_ptr<float>(params), (float)p0, (float)p1,
                             (float)p2, (float)cst, opt_ptr<float>(beta), (float)beta_host,
                             (float)row_weight, opt_ptr<float>(logq0), opt_ptr<float>(ldj),
                             opt_ptr<float>(logp_out), opt_ptr<float>(frow_out), B, Dh,
                             cur_stream());
}

void bernoulli_logits(const at::Tensor& logits, const at::Tensor& x,
                      const c10::optional<at::Tensor>& dlogits, const c10::optional<at::Tensor>& coef,
                      double coef_host, const c10::optional<at::Tensor>& logpx) {
  check_2d(logits, "logits");
  check_2d(x, "x");
  check_dtype(x, at::kFloat, "x");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "logits dtype");
  const int B = logits.size(0), P = logits.size(1);
  TORCH_CHECK(x.size(0) == B && x.size(1) == P, "x shape");
  long ldd = 0;
  if (dlogits && dlogits->defined()) {
    check_2d(*dlogits, "dlogits");
    TORCH_CHECK(dlogits->scalar_type() == logits.scalar_type(), "dlogits dtype");
    ldd = ld_of(*dlogits);
  }
  nf_launch_bernoulli_logits(logits.data_ptr(), bf, ld_of(logits), x.data_ptr<float>(), ld_of(x),
                             opt_ptr<void>(dlogits), ldd, opt_ptr<float>(coef), (float)coef_host,
                             opt_ptr<float>(logpx), B, P, cur_stream());
}

void energy2d(int64_t kind, const at::Tensor& z, const c10::optional<at::Tensor>& logp,
              const c10::optional<at::Tensor>& grad, double gscale,
              const c10::optional<at::Tensor>& logq0, const c10::optional<at::Tensor>& ldj,
              const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& frow) {
  check_2d(z, "z");
  check_dtype(z, at::kFloat, "z");
  TORCH_CHECK(kind >= 0 && kind <= 6, "unknown 2-D target kind");
  TORCH_CHECK(z.size(1) == 2 && z.stride(1) == 1, "z must be [B, 2] with unit column stride");
  const int B = z.size(0);
  // float2 row loads / stores: 8-B aligned rows
  auto al8 = [](const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 8 == 0; };
  TORCH_CHECK(ld_of(z) % 2 == 0 && al8(z), "z rows must be 8-B aligned");
  long ldg = 0;
  if (grad && grad->defined()) {
    check_2d(*grad, "grad");
    check_dtype(*grad, at::kFloat, "grad");
    TORCH_CHECK(grad->size(0) == B && grad->size(1) == 2 && grad->stride(1) == 1, "grad shape");
    ldg = ld_of(*grad);
    TORCH_CHECK(ldg % 2 == 0 && al8(*grad), "grad rows must be 8-B aligned");
  }
  auto vec = [&](const c10::optional<at::Tensor>& t, const char* nm) {
    if (t && t->defined()) {
      check_dtype(*t, at::kFloat, nm);
      TORCH_CHECK(t->is_contiguous() && t->numel() == B, nm, " must be a contiguous (B,) vector");
    }
  };
  vec(logp, "logp");
  vec(logq0, "logq0");
  vec(ldj, "ldj");
  vec(frow, "frow");
  if (beta && beta->defined()) {
    check_dtype(*beta, at::kFloat, "beta");
    TORCH_CHECK(beta->numel() >= 1, "beta");
  }
  nf_launch_energy2d((int)kind, z.data_ptr<float>(), ld_of(z), opt_ptr<float>(logp),
                     opt_ptr<float>(grad), ldg, (float)gscale, opt_ptr<float>(logq0),
                     opt_ptr<float>(ldj), opt_ptr<float>(beta), opt_ptr<float>(frow), B,
                     cur_stream());
}

// ---------------------------------------------------------------- sampling
void reparam_sample(const c10::optional<at::Tensor>& mu, const c10::optional<at::Tensor>& logvar,
                    int64_t seed, const c10::optional<at::Tensor>& offset, int64_t offset_host,
                    int64_t stream_id, const at::Tensor& z, const c10::optional<at::Tensor>& eps,
                    const c10::optional<at::Tensor>& zbf, int64_t nbf,
                    const c10::optional<at::Tensor>& logq0) {
  check_2d(z, "z");
  check_dtype(z, at::kFloat, "z");
  const int B = z.size(0), D = z.size(1);
  long lde = 0, ldzb = 0;
  if (eps && eps->defined()) {
    check_2d(*eps, "eps");
    TORCH_CHECK(eps->size(0) == B && eps->size(1) == D, "eps shape");
    lde = ld_of(*eps);
  }
  if (zbf && zbf->defined()) {
    check_2d(*zbf, "zbf");
    TORCH_CHECK(zbf->scalar_type() == at::kBFloat16 || zbf->scalar_type() == at::kFloat, "zbf dtype");
    TORCH_CHECK(zbf->size(0) == B && zbf->size(1) >= nbf && nbf <= D, "zbf shape");
    ldzb = ld_of(*zbf);
  }
  if (offset && offset->defined()) check_dtype(*offset, at::kLong, "offset");
  if (mu && mu->defined()) TORCH_CHECK(mu->numel() == D && mu->is_contiguous(), "mu");
  if (logvar && logvar->defined()) TORCH_CHECK(logvar->numel() == D && logvar->is_contiguous(), "logvar");
  // zbf pad runs to the logical width, so pass it via ldzb = width when contiguous
  long zb_width = (zbf && zbf->defined()) ? zbf->size(1) : 0;
  TORCH_CHECK(!(zbf && zbf->defined()) || zb_width == ldzb, "zbf must be contiguous");
  nf_launch_reparam_sample(opt_ptr<float>(mu), opt_ptr<float>(logvar), (uint64_t)seed,
                           opt_ptr<int64_t>(offset), offset_host, (uint32_t)stream_id,
                           z.data_ptr<float>(), ld_of(z), opt_ptr<float>(eps), lde,
                           opt_ptr<void>(zbf),
                           zbf && zbf->defined() && zbf->scalar_type() == at::kBFloat16, ldzb,
                           (int)nbf, opt_ptr<float>(logq0), B, D,
                           cur_stream());
}

// Diagonal-base reparameterisation backward; dL/dz0 = [g_lo | g_hi] (two strided views).
void reparam_grad(const at::Tensor& g_lo, const at::Tensor& g_hi, const at::Tensor& eps,
                  const at::Tensor& logvar, const at::Tensor& partial, const at::Tensor& gmu,
                  const at::Tensor& glv) {
  check_2d(g_lo, "g_lo");
  check_2d(g_hi, "g_hi");
  check_2d(eps, "eps");
  for (const at::Tensor* t : {&g_lo, &g_hi, &eps, &logvar, &partial, &gmu, &glv})
    check_dtype(*t, at::kFloat, "reparam_grad operand");
  const int B = eps.size(0), D = eps.size(1), Dl = g_lo.size(1);
  TORCH_CHECK(g_lo.size(0) == B && g_hi.size(0) == B && Dl + g_hi.size(1) == D, "reparam_grad shapes");
  TORCH_CHECK(g_lo.stride(1) == 1 && g_hi.stride(1) == 1 && eps.stride(1) == 1, "reparam_grad: unit column stride");
  // one float4 column group per thread of a 256-thread block
  TORCH_CHECK(D % 4 == 0 && Dl % 4 == 0 && D <= 1024, "reparam_grad: D, Dl multiples of 4, D <= 1024");
  const long ldlo = ld_of(g_lo), ldhi = ld_of(g_hi), lde = ld_of(eps);
  TORCH_CHECK(ldlo % 4 == 0 && ldhi % 4 == 0 && lde % 4 == 0, "reparam_grad: 16-B aligned rows");
  for (const at::Tensor* t : {&g_lo, &g_hi, &eps, &partial})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "reparam_grad: 16-B aligned base");
  TORCH_CHECK(logvar.numel() == D && gmu.numel() == D && glv.numel() == D && logvar.is_contiguous() &&
              gmu.is_contiguous() && glv.is_contiguous(), "reparam_grad: (D,) vectors");
  TORCH_CHECK(partial.is_contiguous() && partial.numel() >= 2L * D, "reparam_grad: partial");
  const int npartial = (int)std::min<long>(partial.numel() / (2L * D), (long)B);
  nf_launch_reparam_grad(g_lo.data_ptr<float>(), ldlo, g_hi.data_ptr<float>(), ldhi,
                         eps.data_ptr<float>(), lde, logvar.data_ptr<float>(),
                         partial.data_ptr<float>(), std::max(npartial, 1), gmu.data_ptr<float>(),
                         glv.data_ptr<float>(), B, D, Dl, cur_stream());
}

void normal_fill(const at::Tensor& out, int64_t seed, const c10::optional<at::Tensor>& offset,
                 int64_t offset_host, int64_t stream_id) {
  check_cuda(out, "out");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(out.is_contiguous(), "out must be contiguous");
  nf_launch_normal_fill(out.data_ptr<float>(), out.numel(), (uint64_t)seed, opt_ptr<int64_t>(offset),
                        offset_host, (uint32_t)stream_id, cur_stream());
}

// ---------------------------------------------------------------- optimizer
void flat_optimizer(int64_t kind, const at::Tensor& p, const at::Tensor& g,
                    const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
                    const c10::optional<at::Tensor>& pbf, double lr, double b1, double b2,
                    double eps, double wd, const c10::optional<at::Tensor>& step, double step_host,
                    const c10::optional<at::Tensor>& gscale, double gscale_host,
                    const c10::optional<at::Tensor>& skip, double warmup) {
  check_cuda(p, "p");
  check_dtype(p, at::kFloat, "p");
  check_dtype(g, at::kFloat, "g");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && p.numel() == g.numel(), "p/g flat");
  const long n = p.numel();
  auto chk = [&](const c10::optional<at::Tensor>& t, const char* nm) {
    if (t && t->defined()) TORCH_CHECK(t->is_contiguous() && t->numel() == n, nm, " flat");
  };
  chk(m, "m");
  chk(v, "v");
  chk(pbf, "pbf");
  if (pbf && pbf->defined()) check_dtype(*pbf, at::kBFloat16, "pbf");
  // the kernel moves 16 B per lane on p, g, m, v and 8 B on the bf16 copy
  auto aligned = [](const void* q, uintptr_t a) { return reinterpret_cast<uintptr_t>(q) % a == 0; };
  TORCH_CHECK(aligned(p.data_ptr(), 16), "p must be 16-B aligned");
  TORCH_CHECK(aligned(g.data_ptr(), 16), "g must be 16-B aligned");
  if (m && m->defined()) TORCH_CHECK(aligned(m->data_ptr(), 16), "m must be 16-B aligned");
  if (v && v->defined()) TORCH_CHECK(aligned(v->data_ptr(), 16), "v must be 16-B aligned");
  if (pbf && pbf->defined()) TORCH_CHECK(aligned(pbf->data_ptr(), 8), "pbf must be 8-B aligned");
  nf_launch_flat_optimizer((int)kind, p.data_ptr<float>(), g.data_ptr<float>(), opt_ptr<float>(m),
                           opt_ptr<float>(v), opt_ptr<void>(pbf), n, (float)lr, (float)b1,
                           (float)b2, (float)eps, (float)wd, opt_ptr<float>(step), (float)step_host,
                           opt_ptr<float>(gscale), (float)gscale_host, opt_ptr<float>(skip),
                           (float)warmup, cur_stream());
}

void sumsq_guard(const at::Tensor& x, const at::Tensor& partial,
                 const c10::optional<at::Tensor>& out_sumsq, const c10::optional<at::Tensor>& skip,
                 const c10::optional<at::Tensor>& scale, double max_norm, double base_scale) {
  check_cuda(x, "x");
  check_dtype(x, at::kFloat, "x");
  check_dtype(partial, at::kFloat, "partial");
  TORCH_CHECK(x.is_contiguous() && partial.is_contiguous(), "contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "x must be 16-B aligned");
  TORCH_CHECK(partial.numel() >= 1, "partial needs at least one slot (one block per slot)");
  nf_launch_sumsq_guard(x.data_ptr<float>(), x.numel(), partial.data_ptr<float>(),
                        (int)partial.numel(), opt_ptr<float>(out_sumsq), opt_ptr<float>(skip),
                        opt_ptr<float>(scale), (float)max_norm, (float)base_scale, cur_stream());
}

}  // namespace

void cu_hold(int64_t blocks, double usec) { nf_launch_cu_hold((int)blocks, (float)usec, cur_stream()); }

TORCH_LIBRARY(vinf, m) {
  m.def("coupling_fwd(Tensor st, Tensor x, Tensor(a!) y, Tensor(b!)? ybf, Tensor(c!)? ssav, "
        "Tensor(d!) ldj, float scale, bool inverse, bool ldj_init) -> ()");
  m.def("coupling_bwd(Tensor gy, Tensor s, Tensor x, float c, Tensor? c_row, Tensor(a!) dst, "
        "Tensor(b!) gx, float scale, bool gx_accumulate) -> ()");
  m.def("target_logp_grad(int kind, Tensor A, Tensor B, Tensor(a!)? gA, Tensor(b!)? gB, "
        "bool grad_accumulate, Tensor? params, float p0, float p1, float p2, float cst, "
        "Tensor? beta, float beta_host, float row_weight, Tensor? logq0, Tensor? ldj, "
        "Tensor(c!)? logp_out, Tensor(d!)? frow_out) -> ()");
  m.def("bernoulli_logits(Tensor logits, Tensor x, Tensor(a!)? dlogits, Tensor? coef, "
        "float coef_host, Tensor(b!)? logpx) -> ()");
  m.def("energy2d(int kind, Tensor z, Tensor(a!)? logp, Tensor(b!)? grad, float gscale, "
        "Tensor? logq0, Tensor? ldj, Tensor? beta, Tensor(c!)? frow) -> ()");
  m.def("reparam_sample(Tensor? mu, Tensor? logvar, int seed, Tensor? offset, int offset_host, "
        "int stream_id, Tensor(a!) z, Tensor(b!)? eps, Tensor(c!)? zbf, int nbf, "
        "Tensor(d!)? logq0) -> ()");
  m.def("normal_fill(Tensor(a!) out, int seed, Tensor? offset, int offset_host, int stream_id) -> ()");
  m.def("reparam_grad(Tensor g_lo, Tensor g_hi, Tensor eps, Tensor logvar, Tensor(a!) partial, "
        "Tensor(b!) gmu, Tensor(c!) glv) -> ()");
  m.def("flat_optimizer(int kind, Tensor(a!) p, Tensor g, Tensor(b!)? m, Tensor(c!)? v, "
        "Tensor(d!)? pbf, float lr, float b1, float b2, float eps, float wd, Tensor? step, "
        "float step_host, Tensor? gscale, float gscale_host, Tensor? skip, float warmup=0.0) -> ()");
  m.def("cu_hold(int blocks, float usec) -> ()", &cu_hold);
  m.def("sumsq_guard(Tensor x, Tensor(a!) partial, Tensor(b!)? out_sumsq, Tensor(c!)? skip, "
        "Tensor(d!)? scale, float max_norm, float base_scale) -> ()");
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) {
  m.impl("coupling_fwd", &coupling_fwd);
  m.impl("coupling_bwd", &coupling_bwd);
  m.impl("target_logp_grad", &target_logp_grad);
  m.impl("bernoulli_logits", &bernoulli_logits);
  m.impl("energy2d", &energy2d);
  m.impl("reparam_sample", &reparam_sample);
  m.impl("normal_fill", &normal_fill);
  m.impl("reparam_grad", &reparam_grad);
  m.impl("flat_optimizer", &flat_optimizer);
  m.impl("sumsq_guard", &sumsq_guard);
}
