// TORCH_LIBRARY fragment for the MFMA GEMM family (csrc/kernels/gemm.hip).
#include <vector>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <cstdlib>

#include "launchers.h"
#include "nf_common.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

long ld2(const at::Tensor& t) { return t.size(0) <= 1 ? t.size(1) : t.stride(0); }

// delayed-scale running amax: NF_AMAX_SLOTS contiguous fp32 partial maxima
void chk_amax_slots(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                  t.numel() >= NF_AMAX_SLOTS,
              "amax_cur must hold ", NF_AMAX_SLOTS, " contiguous fp32 slots (ops.fp8.DelayedScale)");
}

void chk_mat(const at::Tensor& t, const char* n, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), n, " must be on the GPU");
  TORCH_CHECK(t.dim() == 2, n, " must be 2-D");
  TORCH_CHECK(t.scalar_type() == dt, n, " dtype ", t.scalar_type(), " expected ", dt);
  TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, n, " needs unit inner stride");
  TORCH_CHECK(ld2(t) % 8 == 0, n, " leading dimension must be a multiple of 8 (16-B rows)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, " must be 16-B aligned");
}

void chk_q(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2, n, " must be a 2-D GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kByte || t.scalar_type() == at::kFloat8_e4m3fn, n,
              " must be uint8 / float8_e4m3fn");
  TORCH_CHECK(t.stride(1) == 1 && ld2(t) % 16 == 0, n, " rows must be 16-B aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, " must be 16-B aligned");
}

void chk_ranges(const at::Tensor& r, long ntiles, const char* n);

// y = act(x W^T + b): x [M,K], W [N,K], b [N] (bf16), y [M,N] bf16
void gemm_nt(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
             const at::Tensor& y, int64_t relu, const c10::optional<at::Tensor>& mask) {
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
  void* mp = nullptr;
  long ldm = 0;
  if (mask && mask->defined()) {  // ReLU bitmask [M][N/8] uint8 for the input-gradient epilogue
    TORCH_CHECK(mask->is_cuda() && mask->dim() == 2 && mask->scalar_type() == at::kByte &&
                    mask->stride(1) == 1, "mask must be a 2-D uint8 GPU tensor with unit inner stride");
    TORCH_CHECK(relu, "the bitmask records 1(y > 0) of a ReLU layer");
    TORCH_CHECK(mask->size(0) == M && mask->size(1) * 8 == N, "mask shape [M, N/8]");
    TORCH_CHECK(ld2(y) % 8 == 0 && ((uintptr_t)y.data_ptr() & 15) == 0,
                "bitmask output needs 16-B aligned y rows");
    mp = mask->data_ptr();
    ldm = ld2(*mask);
  }
  nf_launch_gemm_nt(x.data_ptr(), ld2(x), W.data_ptr(), ld2(W), bp, y.data_ptr(), ld2(y), M, N, K,
                    (int)relu, cur_stream(), mp, ldm);
}

// y = x W^T: x [M,K], W [N,K] bf16, y [M,N] fp32 (the accumulator, unrounded)
void gemm_nt_f32out(const at::Tensor& x, const at::Tensor& W, const at::Tensor& y) {
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  chk_mat(y, "y", at::kFloat);
  const int M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "W inner dim");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N, "y shape");
  TORCH_CHECK(K % 32 == 0 && K > 0, "K must be a positive multiple of 32 (pad the operands)");
  TORCH_CHECK(N % 8 == 0, "N must be a multiple of 8");
  nf_launch_gemm_nt_f32out(x.data_ptr(), ld2(x), W.data_ptr(), ld2(W), y.data_ptr<float>(), ld2(y),
                           M, N, K, cur_stream());
}

// Exact fp32 / fp64 product C (+)= Aop Bop^T (+ bias), dbias = row sums of Aop (gemm_fp.hip).
// A: [M,K] (a_kmajor) or [K,M]; B: [N,K] (b_kmajor) or [K,N]; C [M,N]; bias [N]; dbias [M]; one
// dtype (fp32 or fp64) throughout, unit inner strides, any shape.
void gemm_fp(const at::Tensor& A, bool a_kmajor, const at::Tensor& B, bool b_kmajor,
             const c10::optional<at::Tensor>& bias, const at::Tensor& C, bool accumulate,
             const c10::optional<at::Tensor>& dbias) {
  const auto dt = C.scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kDouble, "gemm_fp: fp32 or fp64 output");
  auto chk = [&](const at::Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.scalar_type() == dt, n,
                " must be a 2-D GPU tensor of the output's dtype");
    TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, n, " needs unit inner stride");
  };
  chk(A, "A"); chk(B, "B"); chk(C, "C");
  const int M = C.size(0), N = C.size(1);
  const int K = a_kmajor ? A.size(1) : A.size(0);
  TORCH_CHECK((a_kmajor ? A.size(0) : A.size(1)) == M, "A rows must match C rows");
  TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == N, "B rows must match C cols");
  TORCH_CHECK((b_kmajor ? B.size(1) : B.size(0)) == K, "A / B inner dims differ");
  const void* bp = nullptr;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == dt && bias->is_contiguous() &&
                    bias->numel() == N, "bias: contiguous [N] of the output's dtype");
    bp = bias->data_ptr();
  }
  void* dbp = nullptr;
  if (dbias && dbias->defined()) {
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == dt && dbias->is_contiguous() &&
                    dbias->numel() == M, "dbias: contiguous [M] of the output's dtype");
    dbp = dbias->data_ptr();
  }
  auto ld = [](const at::Tensor& t) { return t.size(0) <= 1 ? t.size(1) : t.stride(0); };
  // split-K workspace for few-tile, long-K products (caching allocator: graph-capture safe)
  const int S = nf_gemm_fp_splits(M, N, K);
  at::Tensor work;
  if (S > 1) work = at::empty({(long)S * ((long)M * N + M)}, C.options());
  nf_launch_gemm_fp(dt == at::kDouble, A.data_ptr(), ld(A), a_kmajor, B.data_ptr(), ld(B),
                    b_kmajor, bp, C.data_ptr(), ld(C), dbp, M, N, K, accumulate, cur_stream(),
                    S > 1 ? work.data_ptr() : nullptr, S);
}

// dx = dy W  [* 1(h > 0)]: dy [M,K], W [K,N] bf16; dx bf16 (mask) or fp32 (+= when accumulate)
void gemm_nn(const at::Tensor& dy, const at::Tensor& W, const c10::optional<at::Tensor>& h,
             const at::Tensor& dx, bool accumulate, const c10::optional<at::Tensor>& hbits,
             const c10::optional<at::Tensor>& Wt) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  const bool f32 = dx.scalar_type() == at::kFloat;
  chk_mat(dx, "dx", f32 ? at::kFloat : at::kBFloat16);
  const int M = dy.size(0), K = dy.size(1), N = W.size(1);
  TORCH_CHECK(W.size(0) == K, "W rows must equal dy cols");
  const bool use_wt = Wt && Wt->defined();
  if (use_wt) {   // the transposed copy replaces W as the B operand (NT instantiation)
    chk_mat(*Wt, "Wt", at::kBFloat16);
    TORCH_CHECK(Wt->size(0) == N && Wt->size(1) == K, "Wt must be W^T [N, K]");
    TORCH_CHECK(!f32 && !accumulate, "the transposed-weight path writes bf16");
    TORCH_CHECK(ld2(*Wt) % 8 == 0 && ((uintptr_t)Wt->data_ptr() & 15) == 0, "Wt rows 16-B");
  }
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
  int bits = 0;
  if (hbits && hbits->defined()) {  // ReLU bitmask written by gemm_nt(mask=...)
    TORCH_CHECK(!hp, "pass either h or hbits");
    TORCH_CHECK(!f32, "ReLU-mask epilogue writes bf16");
    TORCH_CHECK(hbits->is_cuda() && hbits->dim() == 2 && hbits->scalar_type() == at::kByte &&
                    hbits->stride(1) == 1, "hbits must be a 2-D uint8 GPU tensor with unit inner stride");
    TORCH_CHECK(hbits->size(0) == M && hbits->size(1) * 8 == N, "hbits shape [M, N/8]");
    hp = hbits->data_ptr();
    ldh = ld2(*hbits);
    bits = 1;
  }
  TORCH_CHECK(!accumulate || f32, "accumulate needs an fp32 output");
  if (use_wt) {
    nf_launch_gemm256_nt_dgrad(dy.data_ptr(), ld2(dy), Wt->data_ptr(), ld2(*Wt), hp, ldh, bits,
                               dx.data_ptr(), ld2(dx), M, N, K, cur_stream());
    return;
  }
  nf_launch_gemm_nn(dy.data_ptr(), ld2(dy), W.data_ptr(), ld2(W), hp, ldh, dx.data_ptr(), ld2(dx),
                    f32, accumulate, M, N, K, cur_stream(), bits);
}

// batched bf16 transposes: desc = int64 [n, 5] device table of (src, dst, rows | cols << 32,
// lds | ldd << 32, tile0) as written by ops.layout.TransposePlan
void transpose_bf16_batched(const at::Tensor& desc, int64_t n, int64_t tiles) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.is_contiguous() &&
                  desc.numel() >= 5 * n, "desc: int64 GPU [n, 5]");
  nf_launch_transpose_bf16_batched(desc.data_ptr(), (int)n, (int)tiles, cur_stream());
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
                   const c10::List<c10::optional<at::Tensor>>& db,
                   const c10::List<c10::optional<at::Tensor>>& skip,
                   const c10::List<c10::optional<at::Tensor>>& cmask) {
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
    if (skip.size() == n) {
      const c10::optional<at::Tensor> sk = skip.get(p);
      if (sk && sk->defined()) {
        TORCH_CHECK(sk->is_cuda() && sk->scalar_type() == at::kByte && sk->is_contiguous() &&
                        sk->numel() == (long)((M + 127) / 128) * ((N + 127) / 128), "skip flags");
        pr[p].skip = sk->data_ptr<uint8_t>();
      }
    }
    if (cmask.size() == n) {
      const c10::optional<at::Tensor> cm = cmask.get(p);
      if (cm && cm->defined()) {
        TORCH_CHECK(cm->is_cuda() && cm->scalar_type() == at::kByte && cm->is_contiguous() &&
                        cm->numel() == (long)M * N && N % 4 == 0, "cmask [M,N] uint8");
        TORCH_CHECK(ld2(dW[p]) == N, "cmask needs a dense dW");
        pr[p].cmask = cm->data_ptr<uint8_t>();
      }
    }
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

// Many dense weight gradients, one whole 256x256 tile per block, no split-K: computes the
// tiles [tile0, tile0 + ntiles) of the problem list (tiles numbered problem after problem).
// f8_scales (e4m3 operands): one fp32 pool, dy / x of problem p dequantised by
// f8_scales[sa_idx[p]] / f8_scales[sb_idx[p]]
static void gemm_tn_multi_impl(at::TensorList dy, at::TensorList x, at::TensorList dW,
                               const c10::List<c10::optional<at::Tensor>>& db, int64_t tile0,
                               int64_t ntiles, const c10::List<c10::optional<at::Tensor>>& tiles,
                               const c10::List<c10::optional<at::Tensor>>& cmask,
                               const at::Tensor* f8_scales, at::IntArrayRef sa_idx,
                               at::IntArrayRef sb_idx, int layout = 0) {
  const size_t n = dy.size();
  TORCH_CHECK(layout >= 0 && layout <= 4 && (layout == 0 || !f8_scales), "layout 0..4, bf16");
  const bool f8 = f8_scales != nullptr;
  const auto odt = f8 ? at::kFloat8_e4m3fn : at::kBFloat16;
  if (f8) {
    TORCH_CHECK(f8_scales->is_cuda() && f8_scales->scalar_type() == at::kFloat &&
                    f8_scales->is_contiguous() && sa_idx.size() == n && sb_idx.size() == n,
                "gemm_tn_multi_f8: fp32 scale pool and one (sa, sb) index pair per problem");
    for (size_t p = 0; p < n; ++p)
      TORCH_CHECK(sa_idx[p] >= 0 && sb_idx[p] >= 0 && sa_idx[p] < f8_scales->numel() &&
                      sb_idx[p] < f8_scales->numel() && sa_idx[p] <= 0xffff &&
                      sb_idx[p] <= 0x7fff,
                  "gemm_tn_multi_f8: scale index outside the pool");
  }
  TORCH_CHECK(n >= 1 && n <= 40 && x.size() == n && dW.size() == n && db.size() == n,
              "gemm_tn_multi: 1..40 problems with matching lists");
  TORCH_CHECK((tiles.size() == 0 || tiles.size() == n) && (cmask.size() == 0 || cmask.size() == n),
              "gemm_tn_multi: tiles / cmask lists must be empty or one entry per problem");
  std::vector<NfTnProblem> pr(n);
  long total = 0;
  for (size_t p = 0; p < n; ++p) {
    chk_mat(dy[p], "dy", odt);
    chk_mat(x[p], "x", odt);
    chk_mat(dW[p], "dW", at::kFloat);
    // layout 1: x given as [N][K]; layout 2: dy given as [M][K]
    const int K = layout == 2 ? dy[p].size(1) : dy[p].size(0);
    const int M = layout == 2 ? dy[p].size(0) : dy[p].size(1);
    const int N = layout == 1 ? x[p].size(0) : x[p].size(1);
    TORCH_CHECK((layout == 1 ? x[p].size(1) : x[p].size(0)) == K, "batch mismatch");
    TORCH_CHECK(dW[p].size(0) == M && dW[p].size(1) == N, "dW shape");
    TORCH_CHECK(K % 32 == 0 && M % 8 == 0 && N % 8 == 0, "K % 32, M % 8, N % 8 required");
    TORCH_CHECK(!f8 || (K % 128 == 0 && M % 16 == 0 && N % 16 == 0 && ld2(dy[p]) % 16 == 0 &&
                        ld2(x[p]) % 16 == 0 && ld2(dW[p]) % 4 == 0 &&
                        ((uintptr_t)dW[p].data_ptr() & 15) == 0),
                "gemm_tn_multi_f8: K % 128, M / N / ld % 16, 16-B aligned dW");
    TORCH_CHECK(ld2(dy[p]) < (1L << 31) && ld2(x[p]) < (1L << 31) && ld2(dW[p]) < (1L << 31),
                "leading dimensions must fit in int32");
    float* dbp = nullptr;
    const c10::optional<at::Tensor> b = db.get(p);
    if (b && b->defined()) {
      TORCH_CHECK(b->scalar_type() == at::kFloat && b->numel() == M && b->is_contiguous(), "db");
      dbp = b->data_ptr<float>();
    }
    pr[p] = NfTnProblem{dy[p].data_ptr(), ld2(dy[p]), x[p].data_ptr(), ld2(x[p]),
                        dW[p].data_ptr<float>(), ld2(dW[p]), dbp, M, N, K};
    if (f8) {
      pr[p].sa_idx = (int)sa_idx[p];
      pr[p].sb_idx = (int)sb_idx[p];
    }
    int nt = nf_gemm256_tiles(M, N);
    if (tiles.size() == n) {
      const c10::optional<at::Tensor> tl = tiles.get(p);
      if (tl && tl->defined()) {
        TORCH_CHECK(tl->is_cuda() && tl->scalar_type() == at::kShort && tl->is_contiguous() &&
                        tl->numel() >= 1 && tl->numel() <= nt,
                    "tiles: int16 GPU list of active 256x256 tile ids");
        pr[p].tiles = reinterpret_cast<const unsigned short*>(tl->data_ptr<int16_t>());
        pr[p].ntiles_active = nt = (int)tl->numel();
      }
    }
    if (cmask.size() == n) {
      const c10::optional<at::Tensor> cm = cmask.get(p);
      if (cm && cm->defined()) {
        TORCH_CHECK(cm->is_cuda() && cm->scalar_type() == at::kByte && cm->is_contiguous() &&
                        cm->numel() == (long)M * N && ld2(dW[p]) == N, "cmask [M,N] uint8, dense dW");
        pr[p].cmask = cm->data_ptr<uint8_t>();
      }
    }
    total += nt;
  }
  TORCH_CHECK(tile0 >= 0 && ntiles >= 1 && tile0 + ntiles <= total, "tile range outside the ",
              total, " tiles of the problem list");
  nf_launch_gemm256_tn_multi((int)n, pr.data(), (int)tile0, (int)ntiles, cur_stream(),
                             f8 ? f8_scales->data_ptr<float>() : nullptr, layout);
}

// operand-layout A/B of the bf16 weight-gradient launch (bench/wgrad_bench.py --probe)
void gemm_tn_multi_layout(at::TensorList dy, at::TensorList x, at::TensorList dW,
                          const c10::List<c10::optional<at::Tensor>>& db, int64_t tile0,
                          int64_t ntiles, int64_t layout) {
  const c10::List<c10::optional<at::Tensor>> none;
  gemm_tn_multi_impl(dy, x, dW, db, tile0, ntiles, none, none, nullptr, {}, {}, (int)layout);
}

void gemm_tn_multi(at::TensorList dy, at::TensorList x, at::TensorList dW,
                   const c10::List<c10::optional<at::Tensor>>& db, int64_t tile0, int64_t ntiles,
                   const c10::List<c10::optional<at::Tensor>>& tiles,
                   const c10::List<c10::optional<at::Tensor>>& cmask) {
  gemm_tn_multi_impl(dy, x, dW, db, tile0, ntiles, tiles, cmask, nullptr, {}, {});
}

// e4m3 weight gradients (dy, x: float8_e4m3fn [K = batch][M / N], per-tensor delayed scales)
void gemm_tn_multi_f8(at::TensorList dy, at::TensorList x, at::TensorList dW,
                      const c10::List<c10::optional<at::Tensor>>& db, int64_t tile0,
                      int64_t ntiles, const c10::List<c10::optional<at::Tensor>>& tiles,
                      const c10::List<c10::optional<at::Tensor>>& cmask, const at::Tensor& scales,
                      at::IntArrayRef sa_idx, at::IntArrayRef sb_idx) {
  gemm_tn_multi_impl(dy, x, dW, db, tile0, ntiles, tiles, cmask, &scales, sa_idx, sb_idx);
}

// s * column sums of e4m3 [K][N] tensors (bias gradients of the e4m3 weight gradients)
void fp8_colsum(at::TensorList q, at::TensorList out, const at::Tensor& scales,
                at::IntArrayRef sidx, const at::Tensor& part) {
  const size_t n = q.size();
  TORCH_CHECK(n >= 1 && n <= 40 && out.size() == n && sidx.size() == n,
              "fp8_colsum: 1..40 tensors with matching lists");
  TORCH_CHECK(scales.is_cuda() && scales.scalar_type() == at::kFloat && scales.is_contiguous(),
              "fp8_colsum: fp32 scale pool");
  std::vector<const void*> qp(n);
  std::vector<long> ld(n);
  std::vector<int> K(n), N(n), si(n);
  std::vector<float*> op(n);
  for (size_t i = 0; i < n; ++i) {
    chk_mat(q[i], "q", at::kFloat8_e4m3fn);
    K[i] = (int)q[i].size(0);
    N[i] = (int)q[i].size(1);
    TORCH_CHECK(out[i].is_cuda() && out[i].scalar_type() == at::kFloat && out[i].is_contiguous() &&
                    out[i].numel() == N[i], "fp8_colsum: out[i] fp32 [N]");
    TORCH_CHECK(sidx[i] >= 0 && sidx[i] < scales.numel(), "fp8_colsum: scale index");
    qp[i] = q[i].data_ptr();
    ld[i] = ld2(q[i]);
    op[i] = out[i].data_ptr<float>();
    si[i] = (int)sidx[i];
  }
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= nf_fp8_colsum_workspace((int)n, N.data()),
              "fp8_colsum: part workspace too small");
  nf_launch_fp8_colsum((int)n, qp.data(), ld.data(), K.data(), N.data(), op.data(), si.data(),
                       scales.data_ptr<float>(), part.data_ptr<float>(), cur_stream());
}

// Last conditioner product of coupling layer l with the layer's coupling forward in the epilogue:
// st[:, :Dh] = s_hat (bf16), y = x e^s + t, yb = bf16(y) (0-padded), ldjp[tn] (+)= partial sum s.
// inverse: x = (y - t) e^-s from the layer output (passed as x) into y / yb, ldj share -sum s;
// st may then be None (s_hat not stored)
void gemm_nt_cpl(const at::Tensor& h, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                 const c10::optional<at::Tensor>& st_opt, const at::Tensor& x, const at::Tensor& y,
                 const c10::optional<at::Tensor>& yb, const at::Tensor& ldjp, bool ldj_init,
                 double scale, bool inverse) {
  chk_mat(h, "h", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  const int M = h.size(0), K = h.size(1), Dh = x.size(1);
  const bool has_st = st_opt && st_opt->defined();
  TORCH_CHECK(has_st || inverse, "st (s_hat output) is required in the forward");
  if (has_st) {
    chk_mat(*st_opt, "st", at::kBFloat16);
    TORCH_CHECK(st_opt->size(0) == M && st_opt->size(1) >= Dh, "st shape");
  }
  TORCH_CHECK(W.size(1) == K && W.size(0) >= 2 * Dh, "W: [>= 2 Dh, K]");
  TORCH_CHECK(K % 32 == 0 && Dh % 8 == 0, "K % 32 and Dh % 8 required");
  for (const at::Tensor* t : {&x, &y})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 2 &&
                    t->stride(1) == 1 && t->size(0) == M && t->size(1) == Dh &&
                    ld2(*t) % 4 == 0 && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "x, y: fp32 [M, Dh], 16-B aligned rows");
  const int ntn = (Dh + 127) / 128;
  TORCH_CHECK(ldjp.is_cuda() && ldjp.scalar_type() == at::kFloat && ldjp.dim() == 2 &&
                  ldjp.size(0) >= ntn && ldjp.size(1) == M && ldjp.stride(1) == 1,
              "ldjp: fp32 [ceil(Dh/128), M]");
  const void* bp = nullptr;
  if (b && b->defined()) {
    TORCH_CHECK(b->scalar_type() == at::kBFloat16 && b->numel() == W.size(0) && b->is_contiguous(),
                "bias");
    bp = b->data_ptr();
  }
  void* ybp = nullptr;
  long ldyb = 0;
  int ybw = 0;
  if (yb && yb->defined()) {
    chk_mat(*yb, "yb", at::kBFloat16);
    TORCH_CHECK(yb->size(0) == M && yb->size(1) >= Dh && yb->size(1) % 8 == 0, "yb shape");
    ybp = yb->data_ptr();
    ldyb = ld2(*yb);
    ybw = (int)yb->size(1);
  }
  nf_launch_gemm256_nt_cpl(h.data_ptr(), ld2(h), W.data_ptr(), ld2(W), (int)W.size(0), bp,
                           has_st ? st_opt->data_ptr() : nullptr, has_st ? ld2(*st_opt) : 0, M,
                           K, Dh, x.data_ptr<float>(), ld2(x), y.data_ptr<float>(), ld2(y), ybp,
                           ldyb, ybw, ldjp.data_ptr<float>(), ldjp.stride(0), ldj_init,
                           (float)scale, cur_stream(), inverse ? 1 : 0);
}

// Conditioner input gradient of coupling layer l (gy = G + dy W, fp32, not stored) fused with the
// backward of coupling layer l-1: dst = [dS_hat | dT | 0] (bf16), gx = gy e^s (fp32).
void gemm_nn_cpl(const at::Tensor& dy, const at::Tensor& W, const at::Tensor& G,
                 const at::Tensor& s_hat, const at::Tensor& x, const at::Tensor& dst,
                 const at::Tensor& gx, double scale, double c, const c10::optional<at::Tensor>& Wt) {
  chk_mat(dy, "dy", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  const int M = dy.size(0), K = dy.size(1), N = W.size(1);
  TORCH_CHECK(W.size(0) == K, "W rows must equal dy cols");
  const bool use_wt = Wt && Wt->defined();
  if (use_wt) {
    chk_mat(*Wt, "Wt", at::kBFloat16);
    TORCH_CHECK(Wt->size(0) == N && Wt->size(1) == K, "Wt must be W^T [N, K]");
    TORCH_CHECK(ld2(*Wt) % 8 == 0 && ((uintptr_t)Wt->data_ptr() & 15) == 0, "Wt rows 16-B");
  }
  TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "K % 32 and N % 8 required");
  for (const at::Tensor* t : {&G, &s_hat, &x, &dst, &gx})
    TORCH_CHECK(t->is_cuda() && t->dim() == 2 && t->stride(1) == 1 && t->size(0) == M,
                "gemm_nn_cpl: 2-D GPU operands with unit inner stride and M rows");
  const int Dh = x.size(1);
  const bool x_bf16 = x.scalar_type() == at::kBFloat16;
  // the G chain may be bf16 (G in, gx out) on the bf16-x form
  const bool g_bf16 = G.scalar_type() == at::kBFloat16, gx_bf16 = gx.scalar_type() == at::kBFloat16;
  TORCH_CHECK((G.scalar_type() == at::kFloat || (g_bf16 && x_bf16)) && G.size(1) == N,
              "G: fp32 (or bf16 with bf16 x) [M, N]");
  TORCH_CHECK((x.scalar_type() == at::kFloat || (x_bf16 && use_wt)) &&
                  (gx.scalar_type() == at::kFloat || (gx_bf16 && x_bf16)) && gx.size(1) == Dh,
              "x: fp32 (or bf16 with Wt) [M, Dh], gx: fp32 (or bf16 with bf16 x) [M, Dh]");
  TORCH_CHECK(s_hat.scalar_type() == at::kBFloat16 && s_hat.size(1) >= Dh, "s_hat: bf16 [M, >= Dh]");
  TORCH_CHECK(dst.scalar_type() == at::kBFloat16 && dst.size(1) >= 2 * Dh && dst.size(1) <= Dh + N,
              "dst: bf16 [M, 2 Dh .. Dh + N]");
  nf_launch_gemm256_nn_cpl(dy.data_ptr(), ld2(dy), use_wt ? Wt->data_ptr() : W.data_ptr(),
                           use_wt ? ld2(*Wt) : ld2(W), (const float*)G.data_ptr(),
                           ld2(G), M, N, K, s_hat.data_ptr(), ld2(s_hat), (const float*)x.data_ptr(),
                           ld2(x), dst.data_ptr(), ld2(dst), (int)dst.size(1),
                           (float*)gx.data_ptr(), ld2(gx), Dh, (float)scale, (float)c, cur_stream(),
                           use_wt ? 1 : 0, nullptr, 1, 0, nullptr, x_bf16 ? 1 : 0, g_bf16 ? 1 : 0,
                           gx_bf16 ? 1 : 0);
}

// MAF layer l's second MADE product with the layer's transform fused (gemm256.hip
// nf_launch_gemm256_maf_fwd): bf16 operands, or e4m3 (h / W float8 with hs = h's per-tensor
// scale, ws = W's per-row scales, optional e4m3 copy uq of u under a delayed scale).
void maf_gemm_fwd(const at::Tensor& h, const c10::optional<at::Tensor>& hs, const at::Tensor& W,
                  const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& b,
                  const at::Tensor& krange, const at::Tensor& s_out, const at::Tensor& x,
                  const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& ubf,
                  const at::Tensor& ldjp,
                  bool ldj_init, double bound, const c10::optional<at::Tensor>& uq,
                  const c10::optional<at::Tensor>& q_amax_prev,
                  const c10::optional<at::Tensor>& q_scale,
                  const c10::optional<at::Tensor>& q_amax_cur) {
  const bool f8 = h.scalar_type() != at::kBFloat16;
  if (f8) {
    chk_q(h, "h");
    chk_q(W, "W");
    TORCH_CHECK(hs && hs->defined() && ws && ws->defined(), "fp8 operands need hs and ws");
    TORCH_CHECK(hs->is_cuda() && hs->scalar_type() == at::kFloat && hs->numel() >= 1, "hs");
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == at::kFloat && ws->is_contiguous() &&
                    ws->numel() == W.size(0), "ws: fp32 [2D]");
  } else {
    chk_mat(h, "h", at::kBFloat16);
    chk_mat(W, "W", at::kBFloat16);
  }
  chk_mat(s_out, "s_out", at::kBFloat16);
  // x: fp32 or bf16 (a bf16 flow state); u may be None when ubf is given (bf16 state out)
  const bool x_bf16 = x.scalar_type() == at::kBFloat16;
  chk_mat(x, "x", x_bf16 ? at::kBFloat16 : at::kFloat);
  const bool has_u = u && u->defined();
  if (has_u) chk_mat(*u, "u", at::kFloat);
  TORCH_CHECK(has_u || (ubf && ubf->defined()),
              "maf_gemm_fwd: u may be omitted only with a ubf output (a bf16 state)");
  const int M = h.size(0), K = h.size(1), D = x.size(1);
  TORCH_CHECK(W.size(0) == 2 * D && W.size(1) == K, "W must be [2D, K]");
  TORCH_CHECK(D % 128 == 0 && x.size(0) == M && (!has_u || (u->size(0) == M && u->size(1) == D)) &&
                  s_out.size(0) == M && s_out.size(1) == D, "maf_gemm_fwd shapes (D % 128 == 0)");
  chk_ranges(krange, D / 128, "krange");
  TORCH_CHECK(ldjp.is_cuda() && ldjp.scalar_type() == at::kFloat && ldjp.dim() == 2 &&
                  ldjp.size(0) >= D / 128 && ldjp.size(1) == M && ldjp.stride(1) == 1,
              "ldjp: fp32 [D/128, M]");
  const void* bp = nullptr;
  if (b && b->defined()) {
    TORCH_CHECK(b->scalar_type() == at::kBFloat16 && b->numel() == 2 * D && b->is_contiguous(),
                "b: bf16 [2D]");
    bp = b->data_ptr();
  }
  void* ubp = nullptr;
  long ldub = 0;
  if (ubf && ubf->defined()) {
    chk_mat(*ubf, "ubf", at::kBFloat16);
    TORCH_CHECK(ubf->size(0) == M && ubf->size(1) == D, "ubf shape");
    ubp = ubf->data_ptr();
    ldub = ld2(*ubf);
  }
  void* qp = nullptr;
  long ldq = 0;
  const float* qap = nullptr;
  float* qs = nullptr;
  float* qac = nullptr;
  if (uq && uq->defined()) {
    TORCH_CHECK(f8, "the e4m3 copy of u belongs to the fp8 path");
    chk_q(*uq, "uq");
    TORCH_CHECK(uq->size(0) == M && uq->size(1) == D, "uq shape");
    TORCH_CHECK(q_amax_prev && q_scale && q_amax_cur, "uq needs the delayed-scale state");
    chk_amax_slots(*q_amax_cur);
    qp = uq->data_ptr();
    ldq = ld2(*uq);
    qap = q_amax_prev->data_ptr<float>();
    qs = q_scale->data_ptr<float>();
    qac = q_amax_cur->data_ptr<float>();
  }
  nf_launch_gemm256_maf_fwd(h.data_ptr(), ld2(h), f8 ? 1 : 0, f8 ? hs->data_ptr<float>() : nullptr,
                            W.data_ptr(), ld2(W), f8 ? ws->data_ptr<float>() : nullptr, bp,
                            krange.data_ptr<int>(), s_out.data_ptr(), ld2(s_out), M, K, D,
                            (const float*)x.data_ptr(), ld2(x),
                            has_u ? u->data_ptr<float>() : nullptr, has_u ? ld2(*u) : 0, ubp, ldub,
                            ldjp.data_ptr<float>(), ldjp.stride(0), ldj_init, (float)bound, qp, ldq,
                            qap, qs, qac, cur_stream(), x_bf16 ? 1 : 0);
}

// MAF layer l's first MADE product input gradient (gy = G + dy (W1*M1), NT against Wt = (W1*M1)^T,
// never stored) fused with the MAF backward of layer l-1: dst = [dmu | ds_raw] (bf16 [M, 2D]),
// gx = gy e^-alpha (fp32); s_raw / u are layer l-1's (u = the input of layer l).
// fp8: dy / Wt e4m3 with sa (dy's per-tensor scale) and sb (Wt's per-row scales), and
// optionally the e4m3 copy dstq of dst under a delayed scale.
struct F8Out {
  void* q = nullptr;
  long ldq = 0;
  const float* ap = nullptr;
  float* qs = nullptr;
  float* ac = nullptr;
};
F8Out f8_out(const c10::optional<at::Tensor>& q, const c10::optional<at::Tensor>& amax_prev,
             const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& amax_cur,
             long rows, long cols) {
  F8Out o;
  if (!(q && q->defined())) return o;
  chk_q(*q, "q");
  TORCH_CHECK(q->size(0) == rows && q->size(1) == cols, "e4m3 copy shape");
  TORCH_CHECK(amax_prev && scale && amax_cur && amax_prev->defined() && scale->defined() &&
                  amax_cur->defined(), "the e4m3 copy needs the delayed-scale state");
  chk_amax_slots(*amax_cur);
  o.q = q->data_ptr();
  o.ldq = ld2(*q);
  o.ap = amax_prev->data_ptr<float>();
  o.qs = scale->data_ptr<float>();
  o.ac = amax_cur->data_ptr<float>();
  return o;
}

void chk_scales(const c10::optional<at::Tensor>& sa, const c10::optional<at::Tensor>& sb,
                long nb) {
  TORCH_CHECK(sa && sa->defined() && sb && sb->defined(), "fp8 operands need sa and sb");
  TORCH_CHECK(sa->is_cuda() && sa->scalar_type() == at::kFloat && sa->numel() >= 1, "sa");
  TORCH_CHECK(sb->is_cuda() && sb->scalar_type() == at::kFloat && sb->is_contiguous() &&
                  sb->numel() == nb && ((uintptr_t)sb->data_ptr() & 15) == 0,
              "sb: fp32 per-row scales, 16-B aligned");
}

// masked input gradient on e4m3 operands with the ReLU-mask epilogue (gemm256.hip
// nf_launch_gemm256_fp8_dgrad): dx = relu'(h) * (dyq sa)(Wtq sb)^T (bf16) + optional e4m3 dxq
void fp8_dgrad(const at::Tensor& dyq, const at::Tensor& sa, const at::Tensor& Wtq,
               const at::Tensor& sb, const at::Tensor& h, const c10::optional<at::Tensor>& dx_opt,
               const at::Tensor& krange256, const c10::optional<at::Tensor>& dxq,
               const c10::optional<at::Tensor>& q_amax_prev,
               const c10::optional<at::Tensor>& q_scale,
               const c10::optional<at::Tensor>& q_amax_cur) {
  chk_q(dyq, "dyq");
  chk_q(Wtq, "Wtq");
  const int M = dyq.size(0), K = dyq.size(1), N = Wtq.size(0);
  TORCH_CHECK(Wtq.size(1) == K && K % 128 == 0 && N % 8 == 0, "Wtq [N, K], K % 128 == 0");
  // h: the bf16 activation, or its ReLU bitmask (uint8 [M, N/8], bit e of byte n/8 <-> n + e)
  const bool h_bits = h.scalar_type() == at::kByte;
  if (h_bits) {
    TORCH_CHECK(h.is_cuda() && h.dim() == 2 && h.size(0) == M && h.size(1) * 8 >= N &&
                    h.stride(1) == 1, "h bitmask: uint8 [M, N/8]");
  } else {
    chk_mat(h, "h", at::kBFloat16);
  }
  TORCH_CHECK(h.size(0) == M && (h_bits || h.size(1) == N), "h");
  // dx (bf16) may be omitted when only its e4m3 copy dxq is consumed
  const bool has_dx = dx_opt && dx_opt->defined();
  TORCH_CHECK(has_dx || (dxq && dxq->defined()), "fp8_dgrad: dx and / or dxq");
  if (has_dx) {
    chk_mat(*dx_opt, "dx", at::kBFloat16);
    TORCH_CHECK(dx_opt->size(0) == M && dx_opt->size(1) == N, "dx");
  }
  chk_scales(sa, sb, N);
  const long nt = (N + 255) / 256;
  const int segs = krange256.numel() == 4 * nt ? 2 : 1;
  chk_ranges(krange256, segs * nt, "krange256");
  const F8Out o = f8_out(dxq, q_amax_prev, q_scale, q_amax_cur, M, N);
  nf_launch_gemm256_fp8_dgrad(dyq.data_ptr(), ld2(dyq), sa.data_ptr<float>(), Wtq.data_ptr(),
                              ld2(Wtq), sb.data_ptr<float>(), h.data_ptr(), ld2(h), h_bits ? 1 : 0,
                              has_dx ? dx_opt->data_ptr() : nullptr, has_dx ? ld2(*dx_opt) : N,
                              M, N, K, krange256.data_ptr<int>(), segs,
                              o.q, o.ldq, o.ap, o.qs, o.ac, cur_stream());
}

void maf_gemm_bwd(const at::Tensor& dy, const at::Tensor& Wt, const at::Tensor& krange256,
                  const at::Tensor& G, const at::Tensor& s_raw, const at::Tensor& u,
                  const c10::optional<at::Tensor>& dst_opt, const at::Tensor& gx, double bound,
                  double c,
                  const c10::optional<at::Tensor>& sa, const c10::optional<at::Tensor>& sb,
                  const c10::optional<at::Tensor>& dstq,
                  const c10::optional<at::Tensor>& q_amax_prev,
                  const c10::optional<at::Tensor>& q_scale,
                  const c10::optional<at::Tensor>& q_amax_cur) {
  const bool f8 = dy.scalar_type() != at::kBFloat16;
  if (f8) {
    chk_q(dy, "dy");
    chk_q(Wt, "Wt");
    chk_scales(sa, sb, Wt.size(0));
  } else {
    chk_mat(dy, "dy", at::kBFloat16);
    chk_mat(Wt, "Wt", at::kBFloat16);
    TORCH_CHECK(!(dstq && dstq->defined()), "the e4m3 copy of dst belongs to the fp8 path");
  }
  chk_mat(s_raw, "s_raw", at::kBFloat16);
  // dst (bf16) may be omitted on the e4m3 path when only its e4m3 copy dstq is consumed
  const bool has_dst = dst_opt && dst_opt->defined();
  TORCH_CHECK(has_dst || (f8 && dstq && dstq->defined()), "maf_gemm_bwd: dst and / or dstq");
  if (has_dst) chk_mat(*dst_opt, "dst", at::kBFloat16);
  chk_mat(G, "G", at::kFloat);
  const bool u_bf16 = u.scalar_type() == at::kBFloat16;   // a bf16 MAF state (bf16_state)
  chk_mat(u, "u", u_bf16 ? at::kBFloat16 : at::kFloat);
  chk_mat(gx, "gx", at::kFloat);
  const int M = dy.size(0), K = dy.size(1), D = Wt.size(0);
  TORCH_CHECK(Wt.size(1) == K && K % 32 == 0 && D % 8 == 0, "Wt must be [D, K], K % 32 == 0");
  for (const at::Tensor* t : {&G, &s_raw, &u, &gx})
    TORCH_CHECK(t->size(0) == M && t->size(1) == D, "G / s_raw / u / gx: [M, D]");
  TORCH_CHECK(!has_dst || (dst_opt->size(0) == M && dst_opt->size(1) == 2 * D),
              "dst: bf16 [M, 2D]");
  const long nt = (D + 255) / 256;
  const int segs = krange256.numel() == 4 * nt ? 2 : 1;
  chk_ranges(krange256, segs * nt, "krange256");
  NfF8Operands fo{};
  if (f8) {
    const F8Out o = f8_out(dstq, q_amax_prev, q_scale, q_amax_cur, M, 2 * D);
    fo.sa = sa->data_ptr<float>();
    fo.sb = sb->data_ptr<float>();
    fo.q = o.q; fo.ldq = o.ldq;
    fo.q_amax_prev = o.ap; fo.q_scale_out = o.qs; fo.q_amax_cur = o.ac;
  }
  nf_launch_gemm256_nn_cpl(dy.data_ptr(), ld2(dy), Wt.data_ptr(), ld2(Wt), G.data_ptr<float>(),
                           ld2(G), M, D, K, s_raw.data_ptr(), ld2(s_raw),
                           (const float*)u.data_ptr(), ld2(u),
                           has_dst ? dst_opt->data_ptr() : nullptr,
                           has_dst ? ld2(*dst_opt) : 2 * D, 2 * D, gx.data_ptr<float>(), ld2(gx),
                           D, (float)bound, (float)c, cur_stream(), 1, krange256.data_ptr<int>(),
                           segs, 1, f8 ? &fo : nullptr, u_bf16 ? 1 : 0);
}

// all `layers` weights of one kind (rows_per x C each, layer_stride elements apart in the flat
// fp32 buffer starting at x) quantised per row in one launch
void fp8_quant_rows_strided(const at::Tensor& x, int64_t layer_stride, int64_t rows_per,
                            int64_t layers, int64_t C, const at::Tensor& q, const at::Tensor& scale) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16) &&
                  x.is_contiguous(), "x fp32 / bf16 GPU");
  TORCH_CHECK(x.numel() >= (layers - 1) * layer_stride + rows_per * C, "x too small");
  chk_q(q, "q");
  TORCH_CHECK(q.size(0) == rows_per * layers && q.size(1) >= C && q.size(1) % 4 == 0, "q shape");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat &&
                  scale.numel() == rows_per * layers, "scale");
  nf_launch_fp8_quant_rows_strided(x.data_ptr(), x.scalar_type() == at::kBFloat16, C,
                                   layer_stride, (int)rows_per,
                                   (int)(rows_per * layers), (int)C, q.data_ptr(), ld2(q), q.size(1),
                                   scale.data_ptr<float>(), cur_stream());
}

// ----------------------------------------------------------------- MAF transform (maf.hip)
void maf_fwd(const at::Tensor& x, const at::Tensor& o, double bound, const at::Tensor& u,
             const c10::optional<at::Tensor>& ubf, const c10::optional<at::Tensor>& uq,
             const c10::optional<at::Tensor>& amax_prev, const c10::optional<at::Tensor>& scale,
             const c10::optional<at::Tensor>& amax_cur, const at::Tensor& ldj, bool ldj_init) {
  chk_mat(x, "x", at::kFloat);
  chk_mat(o, "o", at::kBFloat16);
  chk_mat(u, "u", at::kFloat);
  const int B = x.size(0), D = x.size(1);
  TORCH_CHECK(D % 4 == 0 && o.size(0) == B && o.size(1) == 2 * D && u.size(0) == B && u.size(1) == D,
              "maf_fwd shapes");
  TORCH_CHECK(ldj.is_cuda() && ldj.scalar_type() == at::kFloat && ldj.numel() == B, "ldj");
  void* ub = nullptr;
  long ldub = 0;
  if (ubf && ubf->defined()) {
    chk_mat(*ubf, "ubf", at::kBFloat16);
    ub = ubf->data_ptr();
    ldub = ld2(*ubf);
  }
  void* q = nullptr;
  long ldq = 0;
  const float* ap = nullptr;
  float* sc = nullptr;
  float* ac = nullptr;
  if (uq && uq->defined()) {
    chk_q(*uq, "uq");
    TORCH_CHECK(amax_prev && scale && amax_cur, "fp8 output needs the delayed-scale state");
    q = uq->data_ptr();
    ldq = ld2(*uq);
    ap = amax_prev->data_ptr<float>();
    sc = scale->data_ptr<float>();
    ac = amax_cur->data_ptr<float>();
    chk_amax_slots(*amax_cur);
  }
  nf_launch_maf_fwd(x.data_ptr<float>(), ld2(x), o.data_ptr(), ld2(o), B, D, (float)bound,
                    u.data_ptr<float>(), ld2(u), ub, ldub, q, ldq, ap, sc, ac,
                    ldj.data_ptr<float>(), ldj_init, cur_stream());
}

void maf_bwd(const at::Tensor& gu, const at::Tensor& u, const at::Tensor& o, double bound,
             double c_ldj, const at::Tensor& dout, const at::Tensor& gx,
             const c10::optional<at::Tensor>& c_row) {
  chk_mat(gu, "gu", at::kFloat);
  chk_mat(u, "u", at::kFloat);
  chk_mat(o, "o", at::kBFloat16);
  chk_mat(dout, "dout", at::kBFloat16);
  chk_mat(gx, "gx", at::kFloat);
  const int B = gu.size(0), D = gu.size(1);
  // o = [mu | s_raw] [B, 2D], or the s_raw half alone [B, D] (the fused engine keeps only s)
  TORCH_CHECK(D % 4 == 0 && u.size(0) == B && u.size(1) == D && o.size(0) == B &&
                  (o.size(1) == 2 * D || o.size(1) == D) && dout.size(1) == 2 * D &&
                  gx.size(1) == D, "maf_bwd shapes");
  const void* sp = static_cast<const at::BFloat16*>(o.data_ptr()) + (o.size(1) == 2 * D ? D : 0);
  const float* cr = nullptr;
  if (c_row && c_row->defined()) {
    TORCH_CHECK(c_row->is_cuda() && c_row->scalar_type() == at::kFloat &&
                    c_row->is_contiguous() && c_row->numel() == B, "c_row: fp32 [B]");
    cr = c_row->data_ptr<float>();
  }
  nf_launch_maf_bwd(gu.data_ptr<float>(), ld2(gu), u.data_ptr<float>(), ld2(u), sp,
                    ld2(o), B, D, (float)bound, (float)c_ldj, dout.data_ptr(), ld2(dout),
                    gx.data_ptr<float>(), ld2(gx), cur_stream(), cr);
}

// gated IAF update: y = m + sigmoid(s + gb) (z - m), ldj = sum log sigmoid(s + gb)
void iaf_gate_fwd(const at::Tensor& o, const at::Tensor& z, double gate_bias, const at::Tensor& y,
                  const at::Tensor& ldj, const c10::optional<at::Tensor>& ybf) {
  chk_mat(o, "o", at::kBFloat16);
  chk_mat(z, "z", at::kFloat);
  chk_mat(y, "y", at::kFloat);
  const int B = z.size(0), D = z.size(1);
  TORCH_CHECK(D % 4 == 0 && o.size(0) == B && o.size(1) == 2 * D && y.size(0) == B &&
                  y.size(1) == D, "iaf_gate_fwd shapes");
  TORCH_CHECK(ldj.is_cuda() && ldj.scalar_type() == at::kFloat && ldj.is_contiguous() &&
                  ldj.numel() == B, "ldj: fp32 [B]");
  void* yb = nullptr;
  long ldyb = 0;
  if (ybf && ybf->defined()) {   // optional bf16 copy of y (e.g. the next MADE's operand columns)
    chk_mat(*ybf, "ybf", at::kBFloat16);
    TORCH_CHECK(ybf->size(0) == B && ybf->size(1) == D && ld2(*ybf) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(ybf->data_ptr()) % 8 == 0,
                "ybf: bf16 [B, D], 8-B aligned rows");
    yb = ybf->data_ptr();
    ldyb = ld2(*ybf);
  }
  nf_launch_iaf_gate_fwd(o.data_ptr(), ld2(o), z.data_ptr<float>(), ld2(z), B, D, (float)gate_bias,
                         y.data_ptr<float>(), ld2(y), ldj.data_ptr<float>(), cur_stream(), yb,
                         ldyb);
}

void iaf_gate_bwd(const at::Tensor& gy, const c10::optional<at::Tensor>& gl, const at::Tensor& z,
                  const at::Tensor& o, double gate_bias, const at::Tensor& dout,
                  const at::Tensor& gz) {
  chk_mat(gy, "gy", at::kFloat);
  chk_mat(z, "z", at::kFloat);
  chk_mat(o, "o", at::kBFloat16);
  chk_mat(dout, "dout", at::kBFloat16);
  chk_mat(gz, "gz", at::kFloat);
  const int B = z.size(0), D = z.size(1);
  TORCH_CHECK(D % 4 == 0 && gy.size(0) == B && gy.size(1) == D && o.size(0) == B &&
                  o.size(1) == 2 * D && dout.size(0) == B && dout.size(1) == 2 * D &&
                  gz.size(0) == B && gz.size(1) == D, "iaf_gate_bwd shapes");
  const float* glp = nullptr;
  if (gl && gl->defined()) {
    TORCH_CHECK(gl->is_cuda() && gl->scalar_type() == at::kFloat && gl->is_contiguous() &&
                    gl->numel() == B, "gl: fp32 [B]");
    glp = gl->data_ptr<float>();
  }
  nf_launch_iaf_gate_bwd(gy.data_ptr<float>(), ld2(gy), glp, z.data_ptr<float>(), ld2(z),
                         o.data_ptr(), ld2(o), B, D, (float)gate_bias, dout.data_ptr(), ld2(dout),
                         gz.data_ptr<float>(), ld2(gz), cur_stream());
}

// ----------------------------------------------------------------- masked (MADE) variants
void chk_ranges(const at::Tensor& r, long ntiles, const char* n) {
  TORCH_CHECK(r.is_cuda() && r.scalar_type() == at::kInt && r.is_contiguous() && r.numel() == 2 * ntiles,
              n, " must be an int32 GPU tensor [n_tiles, 2]");
}

void masked_gemm_nt(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                    const at::Tensor& y, int64_t relu, const at::Tensor& krange,
                    const c10::optional<at::Tensor>& krange256) {
  chk_mat(x, "x", at::kBFloat16);
  chk_mat(W, "W", at::kBFloat16);
  chk_mat(y, "y", at::kBFloat16);
  const int M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && y.size(0) == M && y.size(1) == N, "shapes");
  TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "K % 32 and N % 8 required");
  chk_ranges(krange, (N + 127) / 128, "krange");
  const void* bp = (b && b->defined()) ? b->data_ptr() : nullptr;
  const int* k256 = nullptr;
  if (krange256 && krange256->defined()) {
    chk_ranges(*krange256, (N + 255) / 256, "krange256");
    k256 = krange256->data_ptr<int>();
  }
  nf_launch_gemm_nt_masked(x.data_ptr(), ld2(x), W.data_ptr(), ld2(W), bp, y.data_ptr(), ld2(y), M,
                           N, K, (int)relu, krange.data_ptr<int>(), cur_stream(), k256);
}

void masked_gemm_nn(const at::Tensor& dy, const at::Tensor& W, const c10::optional<at::Tensor>& h,
                    const at::Tensor& dx, const at::Tensor& krange, bool accumulate,
                    const c10::optional<at::Tensor>& krange256, const c10::optional<at::Tensor>& Wt) {
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
  TORCH_CHECK(!accumulate || f32, "accumulate needs an fp32 dx");
  const int* k256 = nullptr;
  int segs = 1;
  if (krange256 && krange256->defined()) {
    // [tiles, 2] (one K range per 256-column tile) or [tiles, 4] (two ranges)
    const long nt = (N + 255) / 256;
    segs = krange256->numel() == 4 * nt ? 2 : 1;
    chk_ranges(*krange256, segs * nt, "krange256");
    TORCH_CHECK(!hp || (ld2(*h) % 8 == 0 && ((uintptr_t)hp & 15) == 0),
                "ReLU-mask operand rows must be 16-B aligned for the 256x256 kernel");
    k256 = krange256->data_ptr<int>();
  }
  const void* wtp = nullptr;
  long ldwt = 0;
  if (Wt && Wt->defined()) {   // (W*M)^T [N, K], used by the 256x256 path
    chk_mat(*Wt, "Wt", at::kBFloat16);
    TORCH_CHECK(Wt->size(0) == N && Wt->size(1) == K, "Wt must be W^T [N, K]");
    TORCH_CHECK(ld2(*Wt) % 8 == 0 && ((uintptr_t)Wt->data_ptr() & 15) == 0, "Wt rows 16-B");
    wtp = Wt->data_ptr();
    ldwt = ld2(*Wt);
  }
  nf_launch_gemm_nn_masked(dy.data_ptr(), ld2(dy), W.data_ptr(), ld2(W), hp, ldh, dx.data_ptr(),
                           ld2(dx), f32, accumulate, M, N, K, krange.data_ptr<int>(), cur_stream(),
                           k256, segs, wtp, ldwt);
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

// ----------------------------------------------------------------- fp8 (OCP e4m3)

// q = e4m3(x / scale[row]), scale[row] = amax(row) / 448; q may be wider than x (zero pad)
void fp8_quant_rows(const at::Tensor& x, const at::Tensor& q, const at::Tensor& scale) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x: 2-D GPU, unit inner stride");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "x bf16/fp32");
  chk_q(q, "q");
  TORCH_CHECK(q.size(0) == x.size(0) && q.size(1) >= x.size(1) && q.size(1) % 4 == 0, "q shape");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == x.size(0) &&
                  scale.is_contiguous(), "scale [rows] fp32");
  nf_launch_fp8_quant_rows(x.data_ptr(), x.scalar_type() == at::kBFloat16, ld2(x), x.size(0),
                           x.size(1), q.data_ptr(), ld2(q), q.size(1), scale.data_ptr<float>(),
                           cur_stream());
}

// delayed per-tensor scaling: q = e4m3(sat(x / s)), s = amax_prev / 448; amax_cur = max(amax_cur, |x|)
void fp8_quant_tensor(const at::Tensor& x, const at::Tensor& q, const at::Tensor& amax_prev,
                      const at::Tensor& scale, const at::Tensor& amax_cur) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "x: 2-D GPU, unit inner stride");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "x bf16/fp32");
  chk_q(q, "q");
  TORCH_CHECK(q.size(0) == x.size(0) && q.size(1) >= x.size(1) && q.size(1) % 4 == 0, "q shape");
  for (const at::Tensor* t : {&amax_prev, &scale, &amax_cur})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= 1, "scalars fp32");
  chk_amax_slots(amax_cur);
  nf_launch_fp8_quant_tensor(x.data_ptr(), x.scalar_type() == at::kBFloat16, ld2(x), x.size(0),
                             x.size(1), q.data_ptr(), ld2(q), q.size(1), amax_prev.data_ptr<float>(),
                             scale.data_ptr<float>(), amax_cur.data_ptr<float>(), cur_stream());
}

// y = act((xq * sx) (wq * sw)^T + b) -> bf16; K % 128 == 0; optional MADE krange per 128-row tile
// sx: [M] per-row or [1] per-tensor
// y may be omitted (only the e4m3 copy yq and / or the ReLU bitmask mask_out [M][N/8] are
// consumed: the MAF engine's e4m3 weight-gradient steps); those forms run on the 256 kernel
void gemm_fp8_nt(const at::Tensor& xq, const at::Tensor& sx, const at::Tensor& wq,
                 const at::Tensor& sw, const c10::optional<at::Tensor>& b,
                 const c10::optional<at::Tensor>& y_opt, int64_t relu,
                 const c10::optional<at::Tensor>& krange,
                 const c10::optional<at::Tensor>& yq, const c10::optional<at::Tensor>& q_amax_prev,
                 const c10::optional<at::Tensor>& q_scale, const c10::optional<at::Tensor>& q_amax_cur,
                 const c10::optional<at::Tensor>& krange256,
                 const c10::optional<at::Tensor>& mask_out) {
  chk_q(xq, "xq");
  chk_q(wq, "wq");
  const bool has_y = y_opt && y_opt->defined();
  const bool has_mask = mask_out && mask_out->defined();
  const int M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K, "shapes");
  if (has_y) {
    chk_mat(*y_opt, "y", at::kBFloat16);
    TORCH_CHECK(y_opt->size(0) == M && y_opt->size(1) == N, "y shape");
  }
  TORCH_CHECK(has_y || (yq && yq->defined()) || has_mask, "gemm_fp8_nt: no output");
  if (has_mask) {
    TORCH_CHECK(mask_out->is_cuda() && mask_out->scalar_type() == at::kByte && mask_out->dim() == 2 &&
                    mask_out->size(0) == M && mask_out->size(1) * 8 >= N && mask_out->stride(1) == 1 &&
                    relu, "mask_out: uint8 [M, N/8] bitmask of a ReLU product");
  }
  TORCH_CHECK(K % 128 == 0 && N % 8 == 0, "K % 128 and N % 8 required");
  TORCH_CHECK(sx.is_cuda() && sx.scalar_type() == at::kFloat && (sx.numel() == M || sx.numel() == 1) &&
                  sx.is_contiguous(), "sx [M] or [1]");
  TORCH_CHECK(sw.is_cuda() && sw.scalar_type() == at::kFloat && sw.numel() == N && sw.is_contiguous(), "sw");
  const void* bp = nullptr;
  if (b && b->defined()) {
    TORCH_CHECK(b->scalar_type() == at::kBFloat16 && b->numel() == N && b->is_contiguous(), "bias");
    bp = b->data_ptr();
  }
  const int* kr = nullptr;
  if (krange && krange->defined()) {
    chk_ranges(*krange, (N + 127) / 128, "krange");
    kr = krange->data_ptr<int>();
  }
  void* qp = nullptr;
  long ldq = 0;
  const float* qap = nullptr;
  float* qs = nullptr;
  float* qac = nullptr;
  if (yq && yq->defined()) {
    chk_q(*yq, "yq");
    TORCH_CHECK(yq->size(0) == M && yq->size(1) == N, "yq shape");
    TORCH_CHECK(q_amax_prev && q_scale && q_amax_cur, "yq needs the delayed-scale state");
    qp = yq->data_ptr();
    ldq = ld2(*yq);
    qap = q_amax_prev->data_ptr<float>();
    qs = q_scale->data_ptr<float>();
    qac = q_amax_cur->data_ptr<float>();
    chk_amax_slots(*q_amax_cur);
  }
  // the 256x256 kernel when the caller supplies its K ranges (or the weight is dense) and the
  // product has a tile per CU (same rule as the bf16 products)
  const bool dense = !(krange && krange->defined());
  const bool has256 = krange256 && krange256->defined();
  const long ldy = has_y ? ld2(*y_opt) : N;
  const bool lean = !has_y || has_mask;
  if ((dense || has256) && (lean || nf_gemm_prefer_256(M, N, K)) && ld2(xq) % 16 == 0 &&
      ld2(wq) % 16 == 0 && ldy % 8 == 0 && (!qp || ldq % 8 == 0)) {
    const int* k256 = nullptr;
    if (has256) {
      chk_ranges(*krange256, (N + 255) / 256, "krange256");
      k256 = krange256->data_ptr<int>();
    }
    nf_launch_gemm256_fp8_nt(xq.data_ptr(), ld2(xq), sx.data_ptr<float>(),
                             sx.numel() == M && M > 1, wq.data_ptr(), ld2(wq), sw.data_ptr<float>(),
                             bp, has_y ? y_opt->data_ptr() : nullptr, ldy, M, N, K, (int)relu,
                             k256, qp, ldq, qap, qs, qac, cur_stream(),
                             has_mask ? mask_out->data_ptr<uint8_t>() : nullptr,
                             has_mask ? ld2(*mask_out) : 0);
    return;
  }
  TORCH_CHECK(!lean, "gemm_fp8_nt: y-less / bitmask forms need the 256 kernel (krange256, 16-B rows)");
  nf_launch_gemm_fp8_nt(xq.data_ptr(), ld2(xq), sx.data_ptr<float>(), sx.numel() == M && M > 1,
                        wq.data_ptr(), ld2(wq),
                        sw.data_ptr<float>(), bp, y_opt->data_ptr(), ldy, M, N, K, (int)relu, kr,
                        qp, ldq, qap, qs, qac, cur_stream());
}

int64_t gemm_set_mode(int64_t mode) { return nf_gemm_set_mode((int)mode); }   // < 0: query
int64_t gemm_pair(int64_t mode) { return nf_gemm256_set_pair((int)mode); }   // < 0: query
int nf_gemm_cpl4w(int on);
// RealNVP coupling-forward product on the 4-fat-wave kernel (1) or the 8-wave one (0)
int64_t gemm_cpl4w(int64_t on) { return nf_gemm_cpl4w((int)on); }   // < 0: query
int nf_gemm256_xcd_pack(int on);
int64_t gemm_wgrad_xcd_pack(int64_t on) { return nf_gemm256_xcd_pack((int)on); }
int64_t gemm_persist(int64_t on) {   // on < 0: query only; returns the previous setting
  const int prev = nf_gemm256_get_persist();
  if (on >= 0) nf_gemm256_set_persist((int)on);
  return prev;
}
int64_t gemm_grid_reserve(int64_t cus) {   // cus < 0: query only; returns the previous value
  return nf_gemm256_set_reserve((int)cus);
}
#ifdef NF_G256_STAMPS
void nf_g256_set_stamps(void* p);
void g256_set_stamps(const at::Tensor& buf) { nf_g256_set_stamps(buf.numel() ? buf.data_ptr() : nullptr); }
#endif

TORCH_LIBRARY_FRAGMENT(vinf, m) {
#ifdef NF_G256_STAMPS
  m.def("g256_set_stamps(Tensor buf) -> ()", &g256_set_stamps);
#endif
  m.def("gemm_set_mode(int mode) -> int", &gemm_set_mode);
  m.def("gemm_pair(int mode) -> int", &gemm_pair);
  m.def("gemm_cpl4w(int on) -> int", &gemm_cpl4w);
  m.def("gemm_persist(int on) -> int", &gemm_persist);
  m.def("gemm_grid_reserve(int cus) -> int", &gemm_grid_reserve);
  m.def("gemm_wgrad_xcd_pack(int on) -> int", &gemm_wgrad_xcd_pack);
  m.def("fp8_quant_rows(Tensor x, Tensor(a!) q, Tensor(b!) scale) -> ()");
  m.def("fp8_quant_tensor(Tensor x, Tensor(a!) q, Tensor amax_prev, Tensor(b!) scale, Tensor(c!) amax_cur) -> ()");
  m.def("gemm_fp8_nt(Tensor xq, Tensor sx, Tensor wq, Tensor sw, Tensor? b, Tensor(a!)? y, int relu, Tensor? krange, Tensor(b!)? yq=None, Tensor? q_amax_prev=None, Tensor(c!)? q_scale=None, Tensor(d!)? q_amax_cur=None, Tensor? krange256=None, Tensor(e!)? mask_out=None) -> ()");
  m.def("masked_gemm_nt(Tensor x, Tensor W, Tensor? b, Tensor(a!) y, int relu, Tensor krange, Tensor? krange256=None) -> ()");
  m.def("masked_gemm_nn(Tensor dy, Tensor W, Tensor? h, Tensor(a!) dx, Tensor krange, bool accumulate=False, Tensor? krange256=None, Tensor? Wt=None) -> ()");
  m.def("masked_gemm_tn(Tensor dy, Tensor x, Tensor(a!) dW, Tensor(b!)? db, Tensor skip) -> ()");
  m.def("gemm_nt(Tensor x, Tensor W, Tensor? b, Tensor(a!) y, int relu, Tensor(b!)? mask=None) -> ()");
  m.def("gemm_nt_f32out(Tensor x, Tensor W, Tensor(a!) y) -> ()");
  m.def("gemm_fp(Tensor A, bool a_kmajor, Tensor B, bool b_kmajor, Tensor? bias, Tensor(a!) C, bool accumulate, Tensor(b!)? dbias=None) -> ()");
  m.def("gemm_nn(Tensor dy, Tensor W, Tensor? h, Tensor(a!) dx, bool accumulate, Tensor? hbits=None, Tensor? Wt=None) -> ()");
  m.def("transpose_bf16_batched(Tensor desc, int n, int tiles) -> ()");
  m.def("gemm_tn(Tensor dy, Tensor x, Tensor(a!) dW, Tensor(b!)? db) -> ()");
  m.def("gemm_tn_group(Tensor[] dy, Tensor[] x, Tensor(a!)[] dW, Tensor(b!)?[] db, Tensor?[] skip, Tensor?[] cmask) -> ()");
  m.def("gemm_tn_multi(Tensor[] dy, Tensor[] x, Tensor(a!)[] dW, Tensor(b!)?[] db, int tile0, int ntiles, Tensor?[] tiles, Tensor?[] cmask) -> ()");
  m.def("gemm_tn_multi_layout(Tensor[] dy, Tensor[] x, Tensor(a!)[] dW, Tensor(b!)?[] db, int tile0, int ntiles, int layout) -> ()");
  m.def("fp8_colsum(Tensor[] q, Tensor(a!)[] out, Tensor scales, int[] sidx, Tensor(b!) part) -> ()");
  m.def("gemm_tn_multi_f8(Tensor[] dy, Tensor[] x, Tensor(a!)[] dW, Tensor(b!)?[] db, int tile0, int ntiles, Tensor?[] tiles, Tensor?[] cmask, Tensor scales, int[] sa_idx, int[] sb_idx) -> ()");
  m.def("gemm_nt_cpl(Tensor h, Tensor W, Tensor? b, Tensor(a!)? st, Tensor x, Tensor(b!) y, Tensor(c!)? yb, Tensor(d!) ldjp, bool ldj_init, float scale, bool inverse=False) -> ()");
  m.def("gemm_nn_cpl(Tensor dy, Tensor W, Tensor G, Tensor s_hat, Tensor x, Tensor(a!) dst, Tensor(b!) gx, float scale, float c, Tensor? Wt=None) -> ()");
  m.def("maf_gemm_fwd(Tensor h, Tensor? hs, Tensor W, Tensor? ws, Tensor? b, Tensor krange, Tensor(a!) s_out, Tensor x, Tensor(b!)? u, Tensor(c!)? ubf, Tensor(d!) ldjp, bool ldj_init, float bound, Tensor(e!)? uq=None, Tensor? q_amax_prev=None, Tensor(f!)? q_scale=None, Tensor(g!)? q_amax_cur=None) -> ()");
  m.def("maf_gemm_bwd(Tensor dy, Tensor Wt, Tensor krange256, Tensor G, Tensor s_raw, Tensor u, Tensor(a!)? dst, Tensor(b!) gx, float bound, float c, Tensor? sa=None, Tensor? sb=None, Tensor(c!)? dstq=None, Tensor? q_amax_prev=None, Tensor(d!)? q_scale=None, Tensor(e!)? q_amax_cur=None) -> ()");
  m.def("fp8_dgrad(Tensor dyq, Tensor sa, Tensor Wtq, Tensor sb, Tensor h, Tensor(a!)? dx, Tensor krange256, Tensor(b!)? dxq=None, Tensor? q_amax_prev=None, Tensor(c!)? q_scale=None, Tensor(d!)? q_amax_cur=None) -> ()");
  m.def("fp8_quant_rows_strided(Tensor x, int layer_stride, int rows_per, int layers, int C, Tensor(a!) q, Tensor(b!) scale) -> ()");
  m.def("maf_fwd(Tensor x, Tensor o, float bound, Tensor(a!) u, Tensor(b!)? ubf, Tensor(c!)? uq, Tensor? amax_prev, Tensor(d!)? scale, Tensor(e!)? amax_cur, Tensor(f!) ldj, bool ldj_init) -> ()");
  m.def("iaf_gate_fwd(Tensor o, Tensor z, float gate_bias, Tensor(a!) y, Tensor(b!) ldj, "
        "Tensor(c!)? ybf=None) -> ()");
  m.def("iaf_gate_bwd(Tensor gy, Tensor? gl, Tensor z, Tensor o, float gate_bias, Tensor(a!) dout, Tensor(b!) gz) -> ()");
  m.def("maf_bwd(Tensor gu, Tensor u, Tensor o, float bound, float c_ldj, Tensor(a!) dout, Tensor(b!) gx, Tensor? c_row=None) -> ()");
}

TORCH_LIBRARY_IMPL(vinf, CUDA, m) {
  m.impl("masked_gemm_nt", &masked_gemm_nt);
  m.impl("masked_gemm_nn", &masked_gemm_nn);
  m.impl("masked_gemm_tn", &masked_gemm_tn);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("gemm_nt_f32out", &gemm_nt_f32out);
  m.impl("gemm_fp", &gemm_fp);
  m.impl("gemm_nn", &gemm_nn);
  m.impl("transpose_bf16_batched", &transpose_bf16_batched);
  m.impl("gemm_tn", &gemm_tn);
  m.impl("gemm_tn_group", &gemm_tn_group);
  m.impl("gemm_tn_multi", &gemm_tn_multi);
  m.impl("gemm_tn_multi_f8", &gemm_tn_multi_f8);
  m.impl("fp8_colsum", &fp8_colsum);
  m.impl("gemm_tn_multi_layout", &gemm_tn_multi_layout);
  m.impl("gemm_nn_cpl", &gemm_nn_cpl);
  m.impl("gemm_nt_cpl", &gemm_nt_cpl);
  m.impl("fp8_quant_rows", &fp8_quant_rows);
  m.impl("fp8_quant_rows_strided", &fp8_quant_rows_strided);
  m.impl("maf_fwd", &maf_fwd);
  m.impl("maf_gemm_fwd", &maf_gemm_fwd);
  m.impl("maf_gemm_bwd", &maf_gemm_bwd);
  m.impl("fp8_dgrad", &fp8_dgrad);
  m.impl("maf_bwd", &maf_bwd);
  m.impl("iaf_gate_fwd", &iaf_gate_fwd);
  m.impl("iaf_gate_bwd", &iaf_gate_bwd);
  m.impl("fp8_quant_tensor", &fp8_quant_tensor);
  m.impl("gemm_fp8_nt", &gemm_fp8_nt);
}
