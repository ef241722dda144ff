// Batched ELBO reductions with fused analytic gradients (gfx950).
//
// target_logp_grad: per-row log p(z_K) of a synthetic target and its gradient
//   dL/dz_K = -beta * w_row * grad log p(z_K), written straight into the two
//   fp32 half-buffers that hold z_K (RealNVP keeps the state as two halves).
//   The row free energy F_row = log q0(z0) - ldj - beta * log p(z_K) is
//   emitted in the same pass so the loss needs one tiny mean afterwards.
//   beta lives on the device so a captured hipGraph can follow an annealing
//   schedule without re-capture.
// Targets:
//   kind 0 (diag Gaussian): log N(z; m, diag(v)), params = [m(D), 1/v(D)], cst = -D/2 log 2pi - 1/2 sum log v
//   kind 1 (banana / twisted Gaussian, Haario et al.): pairs (x=z_2i, y=z_2i+1),
//           log N(x; 0, s1^2) + log N(y - b (x^2 - s1^2); 0, s2^2); exactly normalised (log Z = 0).
//   kind 2 (banana, split pairing): the same density with pairs (x=z_i, y=z_{D/2+i}), i.e. each
//           pair straddles the RealNVP coupling split.
//
// bernoulli_logits: per-row sum_j x_j l_j - softplus(l_j) and dL/dl = coef (x - sigmoid(l)).
#include "nf_common.h"

namespace nf {

__device__ __forceinline__ float zval(const float* A, long lda, const float* Bh, long ldb, long row,
                                      int j, int Dh) {
  return j < Dh ? A[row * lda + j] : Bh[row * ldb + (j - Dh)];
}

__global__ void __launch_bounds__(256) target_logp_grad_kernel(
    int kind, const float* __restrict__ A, long lda, const float* __restrict__ Bh, long ldb,
    float* __restrict__ gA, long ldga, float* __restrict__ gB, long ldgb, int grad_accumulate,
    const float* __restrict__ params, float p0, float p1, float p2, float cst,
    const float* __restrict__ beta_ptr, float beta_host, float row_weight,
    const float* __restrict__ logq0, const float* __restrict__ ldj, float* __restrict__ logp_out,
    float* __restrict__ frow_out, int B, int Dh) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float beta = beta_ptr ? *beta_ptr : beta_host;
  const float coef = -beta * row_weight;
  const int D = 2 * Dh;
  float acc = 0.f;
  if (kind == 0) {
    const float* m = params;
    const float* iv = params + D;
    for (int j = lane; j < D; j += 64) {
      const float z = zval(A, lda, Bh, ldb, row, j, Dh);
      const float d = z - m[j];
      acc += d * d * iv[j];
      if (gA) {
        const float g = coef * (-d * iv[j]);
        float* gp = j < Dh ? (gA + row * ldga + j) : (gB + row * ldgb + (j - Dh));
        *gp = grad_accumulate ? (*gp + g) : g;
      }
    }
    acc = -0.5f * wave_sum(acc) + cst;
  } else {
    const float s1 = p0, s2 = p1, bend = p2;
    const float is1 = 1.f / (s1 * s1), is2 = 1.f / (s2 * s2);
    const bool split = kind == 2;
    for (int i = lane; i < Dh; i += 64) {
      // kind 1: pair (2i, 2i+1) - both in one coupling half (straddles only when Dh is odd);
      // kind 2: pair (i, Dh + i) - x in the first half, y in the second
      const int j = split ? i : 2 * i;
      const int j1 = split ? Dh + i : 2 * i + 1;
      const float x = zval(A, lda, Bh, ldb, row, j, Dh);
      const float y = zval(A, lda, Bh, ldb, row, j1, Dh);
      const float r = y - bend * (x * x - s1 * s1);
      acc += x * x * is1 + r * r * is2;
      if (gA) {
        const float dy = -r * is2;
        const float dx = -x * is1 + r * is2 * 2.f * bend * x;
        float* gp0 = j < Dh ? (gA + row * ldga + j) : (gB + row * ldgb + (j - Dh));
        float* gp1 = j1 < Dh ? (gA + row * ldga + j1) : (gB + row * ldgb + (j1 - Dh));
        const float g0 = coef * dx, g1 = coef * dy;
        if (grad_accumulate) {
          *gp0 += g0;
          *gp1 += g1;
        } else {
          *gp0 = g0;
          *gp1 = g1;
        }
      }
    }
    acc = -0.5f * wave_sum(acc) + cst;
  }
  if (lane == 0) {
    if (logp_out) logp_out[row] = acc;
    if (frow_out) {
      const float q = logq0 ? logq0[row] : 0.f;
      const float l = ldj ? ldj[row] : 0.f;
      frow_out[row] = q - l - beta * acc;
    }
  }
}

template <typename TL>
__device__ __forceinline__ float ldl(const TL* p, long i);
template <>
__device__ __forceinline__ float ldl<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldl<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

template <typename TL, typename TG>
__device__ __forceinline__ void stg(TG* p, long i, float v);
template <>
__device__ __forceinline__ void stg<float, float>(float* p, long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void stg<bf16_t, bf16_t>(bf16_t* p, long i, float v) { p[i] = f2bf(v); }

// One wave per row of P pixels. logits and dlogits share a dtype (bf16 or fp32).
template <typename TL>
__global__ void __launch_bounds__(256) bernoulli_logits_kernel(
    const TL* __restrict__ logits, long ldl_, const float* __restrict__ x, long ldx,
    TL* __restrict__ dlogits, long ldd, const float* __restrict__ coef_ptr, float coef_host,
    float* __restrict__ logpx, int B, int P) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float coef = coef_ptr ? *coef_ptr : coef_host;
  float acc = 0.f;
  for (int j = lane; j < P; j += 64) {
    const float l = ldl<TL>(logits, row * ldl_ + j);
    const float xv = x[row * ldx + j];
    acc += xv * l - softplusf(l);
    if (dlogits) {
      const float sg = 1.f / (1.f + __expf(-l));
      stg<TL, TL>(dlogits, row * ldd + j, coef * (xv - sg));
    }
  }
  acc = wave_sum(acc);
  if (lane == 0 && logpx) logpx[row] = acc;
}

}  // namespace nf

using namespace nf;

void nf_launch_target_logp_grad(int kind, const float* A, long lda, const float* Bh, long ldb,
                                float* gA, long ldga, float* gB, long ldgb, int grad_accumulate,
                                const float* params, float p0, float p1, float p2, float cst,
                                const float* beta_ptr, float beta_host, float row_weight,
                                const float* logq0, const float* ldj, float* logp_out,
                                float* frow_out, int B, int Dh, hipStream_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  hipLaunchKernelGGL(target_logp_grad_kernel, grid, block, 0, stream, kind, A, lda, Bh, ldb, gA,
                     ldga, gB, ldgb, grad_accumulate, params, p0, p1, p2, cst, beta_ptr, beta_host,
                     row_weight, logq0, ldj, logp_out, frow_out, B, Dh);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_bernoulli_logits(const void* logits, int is_bf16, long ldl_, const float* x, long ldx,
                                void* dlogits, long ldd, const float* coef_ptr, float coef_host,
                                float* logpx, int B, int P, hipStream_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  if (is_bf16)
    hipLaunchKernelGGL(bernoulli_logits_kernel<bf16_t>, grid, block, 0, stream,
                       (const bf16_t*)logits, ldl_, x, ldx, (bf16_t*)dlogits, ldd, coef_ptr,
                       coef_host, logpx, B, P);
  else
    hipLaunchKernelGGL(bernoulli_logits_kernel<float>, grid, block, 0, stream,
                       (const float*)logits, ldl_, x, ldx, (float*)dlogits, ldd, coef_ptr,
                       coef_host, logpx, B, P);
  NF_HIP_CHECK(hipGetLastError());
}
