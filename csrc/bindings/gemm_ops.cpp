// TORCH_LIBRARY fragment for the MFMA GEMM family (csrc/kernels/gemm.hip).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <cstdlib>

#include "launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

long ld2(const at::Tensor& t) { return t.size(0) <= 1 ? t.size(1) : t.stride(0); }

void chk_mat(const at::Tensor& t, const char* n, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), n, " must be on the GPU");
  TORCH_CHECK(t.dim() == 2, n, " must be 2-D");
  TORCH_CHECK(t.scalar_type() == dt, n, " dtype ", t.scalar_type(), " expected ", dt);
  TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, n, " needs unit inner stride");
  TORCH_CHECK(ld2(t) % 8 == 0, n, " leading dimension must be a multiple of 8 (16-B rows)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, " must be 16-B aligned");
}

// y = act(x W^T + b): x [M,K], W [N,K], b [N] (bf16), y [M,N] bf16
void gemm_nt(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
             const at::Tensor& y, int64_t relu) {
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  chk_mat(y, "y", at::kBFloat16);
  const int M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "W inner dim");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N, "y shape");
  TORCH_CHECK(K % 32 == 0, "K must be a multiple of 32 (pad the operands)");
  TORCH_CHECK(N % 8 == 0, "N must be a multiple of 8");
  const void* bp = nullptr;
  if (b && b->defined()) {
    TORCH_CHECK(b->scalar_type() == at::kBFloat16 && b->numel() == N && b->is_contiguous(), "bias");
    bp = b->data_ptr();
  }
  nf_launch_gemm_nt(x.data_ptr(), ld2(x), W.data_ptr(), ld2(W), bp, y.data_ptr(), ld2(y), M, N, K,
                    (int)relu, cur_stream());
}

// dx = dy W  [* 1(h > 0)]: dy [M,K], W [K,N] bf16; dx bf16 (mask) or fp32 (+= when accumulate)
void gemm_nn(const at::Tensor& dy, const at::Tensor& W, const c10::optional<at::Tensor>& h,
             const at::Tensor& dx, bool accumulate) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  const bool f32 = dx.scalar_type() == at::kFloat;
  chk_mat(dx, "dx", f32 ? at::kFloat : at::kBFloat16);
  const int M = dy.size(0), K = dy.size(1), N = W.size(1);
  TORCH_CHECK(W.size(0) == K, "W rows must equal dy cols");
  TORCH_CHECK(dx.size(0) == M && dx.size(1) == N, "dx shape");
  TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "K % 32 and N % 8 required");
  const void* hp = nullptr;
  long ldh = 0;
  if (h && h->defined()) {
    TORCH_CHECK(!f32, "ReLU-mask epilogue writes bf16");
    chk_mat(*h, "h", at::kBFloat16);
    TORCH_CHECK(h->size(0) == M && h->size(1) == N, "h shape");
    hp = h->data_ptr();
    ldh = ld2(*h);
  }
  TORCH_CHECK(!accumulate || f32, "accumulate needs an fp32 output");
  nf_launch_gemm_nn(dy.data_ptr(), ld2(dy), W.data_ptr(), ld2(W), hp, ldh, dx.data_ptr(), ld2(dx),
                    f32, accumulate, M, N, K, cur_stream());
}

// dW = dy^T x (fp32), db = colsum(dy) (fp32): dy [K,M], x [K,N] bf16
void gemm_tn(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& dW,
             const c10::optional<at::Tensor>& db) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(dW, "dW", at::kFloat);
  const int K = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(x.size(0) == K, "batch mismatch");
  TORCH_CHECK(dW.size(0) == M && dW.size(1) == N, "dW shape");
  TORCH_CHECK(K % 32 == 0 && M % 8 == 0 && N % 8 == 0, "K % 32, M % 8, N % 8 required");
  float* dbp = nullptr;
  if (db && db->defined()) {
    TORCH_CHECK(db->scalar_type() == at::kFloat && db->numel() == M && db->is_contiguous(), "db");
    dbp = db->data_ptr<float>();
  }
  const int splits = nf_gemm_tn_splits(M, N, K);
  at::Tensor work;
  float* wp = nullptr;
  const long ws = nf_gemm_tn_workspace(M, N, splits);
  if (ws > 0) {
    work = at::empty({ws}, dW.options());
    wp = work.data_ptr<float>();
  }
  nf_launch_gemm_tn(dy.data_ptr(), ld2(dy), x.data_ptr(), ld2(x), dW.data_ptr<float>(), ld2(dW), dbp,
                    M, N, K, splits, wp, cur_stream());
}

// Grouped weight gradients: dW[p] = dy[p]^T x[p], db[p] = colsum(dy[p]) in one launch (+ reduce).
void gemm_tn_group(at::TensorList dy, at::TensorList x, at::TensorList dW,
                   const c10::List<c10::optional<at::Tensor>>& db) {
  const size_t n = dy.size();
  TORCH_CHECK(n >= 1 && n <= 4 && x.size() == n && dW.size() == n && db.size() == n,
              "gemm_tn_group: 1..4 problems with matching lists");
  NfTnProblem pr[4];
  for (size_t p = 0; p < n; ++p) {
    chk_mat(dy[p], "dy", at::kBFloat16);
    chk_mat(x[p], "x", at::kBFloat16);
    chk_mat(dW[p], "dW", at::kFloat);
    const int K = dy[p].size(0), M = dy[p].size(1), N = x[p].size(1);
    TORCH_CHECK(x[p].size(0) == K, "batch mismatch");
    TORCH_CHECK(dW[p].size(0) == M && dW[p].size(1) == N, "dW shape");
    TORCH_CHECK(K % 32 == 0 && M % 8 == 0 && N % 8 == 0, "K % 32, M % 8, N % 8 required");
    float* dbp = nullptr;
    const c10::optional<at::Tensor> b = db.get(p);
    if (b && b->defined()) {
      TORCH_CHECK(b->scalar_type() == at::kFloat && b->numel() == M && b->is_contiguous(), "db");
      dbp = b->data_ptr<float>();
    }
    pr[p] = NfTnProblem{dy[p].data_ptr(), ld2(dy[p]), x[p].data_ptr(), ld2(x[p]),
                        dW[p].data_ptr<float>(), ld2(dW[p]), dbp, M, N, K};
  }
  at::Tensor work;
  float* wp = nullptr;
  const long ws = nf_gemm_tn_group_workspace((int)n, pr);
  if (ws > 0) {
    work = at::empty({ws}, dW[0].options());
    wp = work.data_ptr<float>();
  }
  nf_launch_gemm_tn_group((int)n, pr, wp, cur_stream());
}

// ----------------------------------------------------------------- masked (MADE) variants
void chk_ranges(const at::Tensor& r, long ntiles, const char* n) {
  TORCH_CHECK(r.is_cuda() && r.scalar_type() == at::kInt && r.is_contiguous() && r.numel() == 2 * ntiles,
              n, " must be an int32 GPU tensor [n_tiles, 2]");
}

void masked_gemm_nt(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                    const at::Tensor& y, int64_t relu, const at::Tensor& krange) {
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  chk_mat(y, "y", at::kBFloat16);
  const int M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && y.size(0) == M && y.size(1) == N, "shapes");
  TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "K % 32 and N % 8 required");
  chk_ranges(krange, (N + 127) / 128, "krange");
  const void* bp = (b && b->defined()) ? b->data_ptr() : nullptr;
  nf_launch_gemm_nt_masked(x.data_ptr(), ld2(x), W.data_ptr(), ld2(W), bp, y.data_ptr(), ld2(y), M,
                           N, K, (int)relu, krange.data_ptr<int>(), cur_stream());
}

void masked_gemm_nn(const at::Tensor& dy, const at::Tensor& W, const c10::optional<at::Tensor>& h,
                    const at::Tensor& dx, const at::Tensor& krange) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  const bool f32 = dx.scalar_type() == at::kFloat;
  chk_mat(dx, "dx", f32 ? at::kFloat : at::kBFloat16);
  const int M = dy.size(0), K = dy.size(1), N = W.size(1);
  TORCH_CHECK(W.size(0) == K && dx.size(0) == M && dx.size(1) == N, "shapes");
  TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "K % 32 and N % 8 required");
  chk_ranges(krange, (N + 127) / 128, "krange");
  const void* hp = nullptr;
  long ldh = 0;
  if (h && h->defined()) {
    chk_mat(*h, "h", at::kBFloat16);
    hp = h->data_ptr();
    ldh = ld2(*h);
  }
  nf_launch_gemm_nn_masked(dy.data_ptr(), ld2(dy), W.data_ptr(), ld2(W), hp, ldh, dx.data_ptr(),
                           ld2(dx), f32, M, N, K, krange.data_ptr<int>(), cur_stream());
}

void masked_gemm_tn(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& dW,
                    const c10::optional<at::Tensor>& db, const at::Tensor& skip) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(dW, "dW", at::kFloat);
  const int K = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(x.size(0) == K && dW.size(0) == M && dW.size(1) == N, "shapes");
  TORCH_CHECK(K % 32 == 0 && M % 8 == 0 && N % 8 == 0, "K % 32, M % 8, N % 8 required");
  TORCH_CHECK(skip.is_cuda() && skip.scalar_type() == at::kByte && skip.is_contiguous() &&
                  skip.numel() == (long)((M + 127) / 128) * ((N + 127) / 128),
              "skip must be a uint8 GPU tensor [tiles]");
  float* dbp = (db && db->defined()) ? db->data_ptr<float>() : nullptr;
  const int splits = nf_gemm_tn_splits(M, N, K);
  at::Tensor work;
  float* wp = nullptr;
  const long ws = nf_gemm_tn_workspace(M, N, splits);
  if (ws > 0) {
    work = at::empty({ws}, dW.options());
    wp = work.data_ptr<float>();
  }
  nf_launch_gemm_tn_masked(dy.data_ptr(), ld2(dy), x.data_ptr(), ld2(x), dW.data_ptr<float>(),
                           ld2(dW), dbp, M, N, K, splits, wp, skip.data_ptr<unsigned char>(),
                           cur_stream());
}

}  // namespace

void gemm_set_mode(int64_t mode, int64_t depth) { nf_gemm_set_mode((int)mode, (int)depth); }

TORCH_LIBRARY_FRAGMENT(vinf, m) {
  m.def("gemm_set_mode(int mode, int depth) -> ()", &gemm_set_mode);
  m.def("masked_gemm_nt(Tensor x, Tensor W, Tensor? b, Tensor(a!) y, int relu, Tensor krange) -> ()");
  m.def("masked_gemm_nn(Tensor dy, Tensor W, Tensor? h, Tensor(a!) dx, Tensor krange) -> ()");
  m.def("masked_gemm_tn(Tensor dy, Tensor x, Tensor(a!) dW, Tensor(b!)? db, Tensor skip) -> ()");
  m.def("gemm_nt(Tensor x, Tensor W, Tensor? b, Tensor(a!) y, int relu) -> ()");
  m.def("gemm_nn(Tensor dy, Tensor W, Tensor? h, Tensor(a!) dx, bool accumulate) -> ()");
  m.def("gemm_tn(Tensor dy, Tensor x, Tensor(a!) dW, Tensor(b!)? db) -> ()");
  m.def("gemm_tn_group(Tensor[] dy, Tensor[] x, Tensor(a!)[] dW, Tensor(b!)?[] db) -> ()");
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) {
  m.impl("masked_gemm_nt", &masked_gemm_nt);
  m.impl("masked_gemm_nn", &masked_gemm_nn);
  m.impl("masked_gemm_tn", &masked_gemm_tn);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("gemm_nn", &gemm_nn);
  m.impl("gemm_tn", &gemm_tn);
  m.impl("gemm_tn_group", &gemm_tn_group);
}
