// Host-side launcher declarations shared by csrc/kernels/*.hip and csrc/bindings/*.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

void nf_throw_hip_error(hipError_t e, const char* expr, const char* file, int line);

// coupling.hip
void nf_launch_coupling_fwd(const void* st, int st_is_bf16, long ld_st_, const float* x, long ld_x,
                            float* y, long ld_y, void* ybf, int ybf_is_bf16, long ld_yb,
                            float* ssav, long ld_s, float* ldj, int B, int Dh, float scale,
                            int inverse, int ldj_init, int yb_width, hipStream_t stream);
// s: saved fp32 s, or (s_is_shat_bf16) the bf16 conditioner output s_hat (s recomputed)
void nf_launch_coupling_bwd(const void* s, int s_is_shat_bf16, long ld_s, const float* gy,
                            long ld_gy, const float* x, long ld_x, float c_scalar,
                            const float* c_row, void* dst, int dst_is_bf16, long ld_dst, float* gx,
                            long ld_gx, int B, int Dh, float scale, int gx_accumulate,
                            int dst_pad_to, hipStream_t stream);

// elbo.hip
void nf_launch_target_logp_grad(int kind, const float* A, long lda, const float* Bh, long ldb,
                                float* gA, long ldga, float* gB, long ldgb, int grad_accumulate,
                                const float* params, float p0, float p1, float p2, float cst,
                                const float* beta_ptr, float beta_host, float row_weight,
                                const float* logq0, const float* ldj, float* logp_out,
                                float* frow_out, int B, int Dh, hipStream_t stream);
void nf_launch_bernoulli_logits(const void* logits, int is_bf16, long ldl_, const float* x, long ldx,
                                void* dlogits, long ldd, const float* coef_ptr, float coef_host,
                                float* logpx, int B, int P, hipStream_t stream);
// energy2d.hip: the reference's 2-D targets (U1-U4, trial1): log p, gscale * beta * grad log p,
// optional ELBO row logq0 - ldj - beta log p; z [B][2] fp32 rows (ldz, ldg even)
void nf_launch_energy2d(int kind, const float* z, long ldz, float* logp, float* grad, long ldg,
                        float gscale, const float* logq0, const float* ldj, const float* beta,
                        float* frow, int B, hipStream_t stream);

// sampling.hip
void nf_launch_reparam_sample(const float* mu, const float* logvar, uint64_t seed,
                              const int64_t* offset_ptr, int64_t offset_host, uint32_t stream_id,
                              float* z, long ldz, float* eps, long lde, void* zbf, int zbf_is_bf16,
                              long ldzb, int nbf, float* logq0, int B, int D, hipStream_t stream);
void nf_launch_normal_fill(float* out, long n, uint64_t seed, const int64_t* offset_ptr,
                           int64_t offset_host, uint32_t stream_id, hipStream_t stream);
void nf_launch_reparam_grad(const float* g_lo, long ldlo, const float* g_hi, long ldhi,
                            const float* eps, long lde, const float* logvar, float* partial,
                            int npartial, float* gmu, float* glv, int B, int D, int Dl,
                            hipStream_t stream);

// optim.hip
void nf_launch_flat_optimizer(int kind, float* p, const float* g, float* m, float* v, void* pbf,
                              long n, float lr, float b1, float b2, float eps, float wd,
                              const float* step_ptr, float step_host, const float* gscale_ptr,
                              float gscale_host, const float* skip_ptr, float warmup,
                              hipStream_t stream);
// diagnostics: hold `blocks` CU slots for `usec` us (collective-occupancy emulation)
void nf_launch_cu_hold(int blocks, float usec, hipStream_t stream);
void nf_launch_sumsq_guard(const float* x, long n, float* partial, int npartial, float* out_sumsq,
                           float* out_skip, float* out_scale, float max_norm, float base_scale,
                           hipStream_t stream);

// gemm.hip (bf16 MFMA, fp32 accumulate)
// mask_out: optional ReLU bitmask [M][N/8] bytes (bit e of byte n/8 <-> column n+e) written by
// the forward epilogue; aux_is_bits: the dgrad's ReLU mask `aux` is such a bitmask (ld in bytes)
void nf_launch_gemm_nt(const void* x, long ldx, const void* W, long ldw, const void* bias, void* y,
                       long ldy, int M, int N, int K, int relu, hipStream_t stream,
                       void* mask_out = nullptr, long ld_mask = 0);
void nf_launch_gemm_nn(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                       long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                       int N, int K, hipStream_t stream, int aux_is_bits = 0);
// y[M][N] = x W^T with bf16 operands and an fp32 output (no rounding of the accumulator)
void nf_launch_gemm_nt_f32out(const void* x, long ldx, const void* W, long ldw, float* y, long ldy,
                              int M, int N, int K, hipStream_t stream);
// gemm_fp.hip: exact fp32 / fp64 GEMM on the f32 / f64 MFMA, C (+)= Aop Bop^T (+ bias),
// dbias = row sums of Aop (see the kernel header for the operand layouts)
// split-K: `work` holds splits * (M * N + M) elements of the output dtype (nf_gemm_fp_splits
// picks the count: 1 = no split, work unused)
int nf_gemm_fp_splits(int M, int N, int K);
void nf_launch_gemm_fp(int is_f64, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, const void* bias, void* C, long ldc, void* dbias, int M, int N,
                       int K, int accumulate, hipStream_t stream, void* work = nullptr,
                       int splits = 1);
void nf_launch_gemm_tn(const void* dy, long lddy, const void* x, long ldx, float* dW, long lddw,
                       float* db, int M, int N, int K, int splits, float* work,
                       hipStream_t stream);
long nf_gemm_tn_workspace(int M, int N, int splits);
// grouped weight gradients dW_p = dy_p^T x_p, db_p = colsum(dy_p) (p < 4), one GEMM launch +
// one reduce launch
struct NfTnProblem {
  const void* dy; long lddy;
  const void* x; long ldx;
  float* dW; long lddw;
  float* db;
  int M, N, K;
  const unsigned char* skip = nullptr;   // masked (MADE) weights: all-zero 128x128 tiles of dW
  const unsigned char* cmask = nullptr;  // [M][N] 0/1: zero the masked entries of dW
  // gemm256_tn_multi only: the 256x256 tiles to compute (all-masked tiles are left out of the
  // numbering and never written), ntiles_active of them; -1 = every tile
  const unsigned short* tiles = nullptr;
  int ntiles_active = -1;
  // gemm256_tn_multi e4m3 launches: dy / x dequantisation scales = f8_scales[sa_idx / sb_idx]
  int sa_idx = -1, sb_idx = -1;
};
long nf_gemm_tn_group_workspace(int nprob, const NfTnProblem* pr);
void nf_launch_gemm_tn_group(int nprob, const NfTnProblem* pr, float* work, hipStream_t stream);
// gemm256.hip: 256x256 8-phase kernel (forward / input-gradient products)
// krange: optional per-256-column-tile K ranges [lo, hi) of a MADE-masked weight
void nf_launch_gemm256_nt(const void* x, long ldx, const void* W, long ldw, const void* bias,
                          void* y, long ldy, int M, int N, int K, int relu, hipStream_t stream,
                          void* mask_out = nullptr, long ld_mask = 0,
                          const int* krange = nullptr);
void nf_launch_gemm256_nn(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                          long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                          int N, int K, hipStream_t stream, int aux_is_bits = 0,
                          const int* krange = nullptr, int krange_segs = 1, int w_kmajor = 0);
void nf_gemm256_set_persist(int on);
int nf_gemm256_get_persist();
int nf_gemm256_set_reserve(int cus);   // cus < 0: query; returns the previous value
int nf_gemm256_set_pair(int mode);     // MADE tile pairing 0 off / 1 auto / 2 always; < 0: query
// input gradient with W given transposed (Wt [N][K]): NT instantiation, bf16 (ReLU-mask) epilogue
void nf_launch_gemm256_nt_dgrad(const void* dy, long lddy, const void* Wt, long ldwt,
                                const void* aux, long ld_aux, int aux_is_bits, void* dx,
                                long lddx, int M, int N, int K, hipStream_t stream);
// layout.hip: batched bf16 transposes (TrDesc table on the device)
void nf_launch_transpose_bf16_batched(const void* desc, int n, int total_tiles,
                                      hipStream_t stream);
// last conditioner product of coupling layer l with its coupling forward fused (EPI_CPL_FWD)
void nf_launch_gemm256_nt_cpl(const void* h, long ldh, const void* W, long ldw, int w_rows,
                              const void* bias, void* st, long ld_st, int M, int K, int Dh,
                              const float* x, long ld_x, float* y, long ld_y, void* yb, long ld_yb,
                              int yb_width, float* ldjp, long ld_ldjp, int ldj_init, float scale,
                              hipStream_t stream, int inverse = 0);
// input gradient of coupling layer l's conditioner (fp32, + G) fused with coupling layer l-1's
// backward: writes dst (bf16 [dS_hat | dT | 0]) and gx; G itself is not written
// e4m3 operand scales of an fp8 product: sa (A, per-tensor), sb (B, per-row) and the optional
// e4m3 copy q of the output under a delayed per-tensor scale (ops/fp8.py DelayedScale)
struct NfF8Operands {
  const float* sa;
  const float* sb;
  void* q;
  long ldq;
  const float* q_amax_prev;
  float* q_scale_out;
  float* q_amax_cur;
};
void nf_launch_gemm256_nn_cpl(const void* dy, long lddy, const void* W, long ldw, const float* G,
                              long ldg, int M, int N, int K, const void* s_hat, long ld_s,
                              const float* x, long ld_x, void* dst, long ld_dst, int dst_pad,
                              float* gx, long ld_gx, int Dh, float scale, float c,
                              hipStream_t stream, int w_kmajor = 0, const int* krange = nullptr,
                              int krange_segs = 1, int mode = 0, const NfF8Operands* f8 = nullptr,
                              int x_bf16 = 0, int g_in_bf16 = 0, int gx_bf16 = 0);
void nf_launch_gemm256_fp8_dgrad(const void* dyq, long lddy, const float* sa, const void* wtq,
                                 long ldwt, const float* sb, const void* aux, long ld_aux,
                                 int aux_bits, void* dx, long lddx, int M, int N, int K,
                                 const int* krange, int krange_segs, void* dxq, long lddxq,
                                 const float* q_amax_prev, float* q_scale_out, float* q_amax_cur,
                                 hipStream_t stream);
void nf_launch_gemm256_maf_fwd(const void* h, long ldh, int f8, const float* hs, const void* W,
                               long ldw, const float* ws, const void* bias, const int* krange,
                               void* s_out, long ld_s, int M, int K, int D, const float* x,
                               long ld_x, float* u, long ld_u, void* ubf, long ld_ub, float* ldjp,
                               long ld_ldjp, int ldj_init, float bound, void* uq, long lduq,
                               const float* q_amax_prev, float* q_scale_out, float* q_amax_cur,
                               hipStream_t stream, int x_bf16 = 0);
int nf_launch_gemm256_tn_partials(const void* dy, long lddy, const void* x, long ldx, float* C,
                                  long ldc, long slab_stride, float* dbias, int M, int N, int K,
                                  int splits, hipStream_t stream);
// many dense weight gradients (no split-K, one 256x256 tile per block): tiles numbered problem
// after problem, one launch computes [tile0, tile0 + ntiles)
int nf_gemm256_tiles(int M, int N);
void nf_launch_gemm256_tn_multi(int nprob, const NfTnProblem* pr, int tile0, int ntiles,
                                hipStream_t stream, const float* f8_scales = nullptr,
                                int layout = 0);
// layout: 0 = dy [K][M], x [K][N] (batch-major, TN); 1 = x given transposed [N][K] (k-major);
// 2 = dy given transposed [M][K] - the operand-layout A/B (bench/wgrad_bench.py --probe)
// mode: 0 auto, 1 force 128x128, 2 force 256x256; depth: half-tiles in flight (3 or 4)
int nf_gemm_set_mode(int mode);
// fp8.hip (OCP e4m3): per-row quantisation and the MX-scaled K=128 MFMA GEMM
void nf_launch_fp8_quant_rows(const void* x, int x_is_bf16, long ldx, int R, int C, void* q,
                              long ldq, int Cq, float* scale, hipStream_t stream);
// fp8.hip: deterministic column sums s * sum_k q[k][n] of up to 40 e4m3 [K][N] tensors (the
// bias gradients of the e4m3 weight-gradient launches); part = nf_fp8_colsum_workspace floats
long nf_fp8_colsum_workspace(int n, const int* N);
void nf_launch_fp8_colsum(int n, const void* const* q, const long* ld, const int* K, const int* N,
                          float* const* out, const int* sidx, const float* scales, float* part,
                          hipStream_t stream);
void nf_launch_fp8_quant_tensor(const void* x, int x_is_bf16, long ldx, int R, int C, void* q,
                                long ldq, int Cq, const float* amax_prev, float* scale_out,
                                float* amax_cur, hipStream_t stream);
void nf_launch_gemm_fp8_nt(const void* xq, long ldx, const float* sx, int sx_per_row,
                           const void* wq, long ldw, const float* sw, const void* bias, void* y,
                           long ldy, int M, int N, int K, int relu, const int* krange,
                           void* yq, long ldyq, const float* q_amax_prev, float* q_scale_out,
                           float* q_amax_cur, hipStream_t stream);
int nf_gemm_tn_splits(int M, int N, int K);
// the 256x256 kernels' auto rule (a tile per CU, K >= 256; gemm_set_mode)
bool nf_gemm_prefer_256(int M, int N, int K);
// gemm256.hip F8 instantiation: same contract as nf_launch_gemm_fp8_nt on 256x256 tiles
// (krange per 256-column tile)
void nf_launch_gemm256_fp8_nt(const void* xq, long ldx, const float* sx, int sx_per_row,
                              const void* wq, long ldw, const float* sw, const void* bias, void* y,
                              long ldy, int M, int N, int K, int relu, const int* krange,
                              void* yq, long ldyq, const float* q_amax_prev, float* q_scale_out,
                              float* q_amax_cur, hipStream_t stream,
                              unsigned char* mask_out = nullptr, long ld_mask = 0);

// planar.hip / radial.hip (fused K-layer stacks; per-row parameter gradients)
void nf_launch_planar_fwd(const float* z, const float* W, const float* U, const float* B, float* zK,
                          float* ldj, float* saved, int N, int D, int K, int per_sample,
                          int broadcast, hipStream_t stream);
void nf_launch_planar_bwd(const float* saved, const float* W, const float* U, const float* B,
                          const float* gz, const float* gl, float* dz, float* dW, float* dU,
                          float* dB, int N, int D, int K, int per_sample, int broadcast,
                          hipStream_t stream);
// shared parameters, D <= 16, K * per(D) <= 256: recompute-from-z0 backward with in-kernel
// parameter-gradient reduction (part: nblk * K * (2 per + 1) floats)
int nf_planar_shared_per(int D);
int nf_planar_shared_blocks(int N);
void nf_launch_planar_bwd_shared(const float* z0, const float* W, const float* U, const float* B,
                                 const float* gz, const float* gl, float* dz, float* dW, float* dU,
                                 float* dB, float* part, int nblk, int N, int D, int K,
                                 int broadcast, hipStream_t stream);
void nf_launch_radial_fwd(const float* z, const float* Z0, const float* AL, const float* BE,
                          float* zK, float* ldj, float* saved, int N, int D, int K,
                          int per_sample, hipStream_t stream);
void nf_launch_radial_bwd(const float* saved, const float* Z0, const float* AL, const float* BE,
                          const float* gz, const float* gl, float* dz, float* dZ0, float* dA,
                          float* dBe, int N, int D, int K, int per_sample, hipStream_t stream);

// masked (MADE) GEMMs: per-N-tile K ranges [ntn][2] / per-tile skip flags [ntm*ntn] (128x128 tiles)
void nf_launch_gemm_nt_masked(const void* x, long ldx, const void* W, long ldw, const void* bias,
                              void* y, long ldy, int M, int N, int K, int relu, const int* krange,
                              hipStream_t stream, const int* krange256 = nullptr);
void nf_launch_gemm_nn_masked(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                              long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                              int N, int K, const int* krange, hipStream_t stream,
                              const int* krange256 = nullptr, int krange256_segs = 1,
                              const void* Wt = nullptr, long ldwt = 0);
void nf_launch_gemm_tn_masked(const void* dy, long lddy, const void* x, long ldx, float* dW,
                              long lddw, float* db, int M, int N, int K, int splits, float* work,
                              const unsigned char* skip, hipStream_t stream);

// maf.hip: masked autoregressive flow transform (density direction) fwd / bwd
void nf_launch_maf_fwd(const float* x, long ldx, const void* o, long ldo, int B, int D, float bound,
                       float* u, long ldu, void* ubf, long ldub, void* uq, long lduq,
                       const float* amax_prev, float* scale_out, float* amax_cur, float* ldj,
                       int ldj_init, hipStream_t stream);
void nf_launch_maf_bwd(const float* gu, long ldg, const float* u, long ldu, const void* s_raw,
                       long lds, int B, int D, float bound, float c_ldj, void* dout, long lddo,
                       float* gx, long ldgx, hipStream_t stream, const float* c_row = nullptr);
// maf.hip: gated IAF update (o = [m | s] bf16 from the MADE GEMM)
void nf_launch_iaf_gate_fwd(const void* o, long ldo, const float* z, long ldz, int B, int D,
                            float gate_bias, float* y, long ldy, float* ldj, hipStream_t stream,
                            void* ybf = nullptr, long ldyb = 0);
void nf_launch_iaf_gate_bwd(const float* gy, long ldg, const float* gl, const float* z, long ldz,
                            const void* o, long ldo, int B, int D, float gate_bias, void* dout,
                            long lddo, float* gz, long ldgz, hipStream_t stream);
// fp8.hip: layer-strided per-row weight quantisation (rows r -> layer r / rows_per)
void nf_launch_fp8_quant_rows_strided(const void* x, int x_is_bf16, long ldx, long layer_stride,
                                      int rows_per, int R, int C, void* q, long ldq, int Cq,
                                      float* scale, hipStream_t stream);

// vae.hip: whole training step of the amortized planar-flow VAE (reference main workload):
// phase 1 row-parallel forward + input-gradient chain, phase 2 batch-reduction weight gradients
struct NfVaeParams {
  const float* enc_W[4];
  const float* enc_b[4];
  const float* enc_Wo;
  const float* enc_bo;
  const float* dec_W[4];
  const float* dec_b[4];
  const float* dec_Wo;
  const float* dec_bo;
};
struct NfVaeGrads {
  float* enc_W[4];
  float* enc_b[4];
  float* enc_Wo;
  float* enc_bo;
  float* dec_W[4];
  float* dec_b[4];
  float* dec_Wo;
  float* dec_bo;
};
size_t nf_vae_rows_lds_bytes(int Din, int dz, int K, int De);
void nf_launch_vae_step(const NfVaeParams& prm, const float* x, const float* eps_in, unsigned seed,
                        const long* offset, const float* beta, int B, int Din, int dz, int K,
                        int L, float* ws_eact, float* ws_egrad, float* ws_gphi, float* ws_zk,
                        float* ws_dact, float* ws_dgrad, float* ws_dl, float* frow, float* loss,
                        float* zk_out, float* ldj_out, const NfVaeGrads& grd, hipStream_t stream);
