// The reference's 2-D target energies with fused analytic gradients (gfx950):
//   log p(z) = -U(z) and grad log p(z), one thread per sample, z [B][2] fp32.
//
// Targets (/root/reference/get_data.py:20-66, /root/reference/theano_implement.py:56-75; the
// module composites are vi_normflows_amd/distributions/energies.py), evaluated in log space
// with a stable log-add-exp (the reference's log(eps + exp(-U)) underflows far from the modes):
//   kind 0 U1:     -1/2 ((|z| - 2) / 0.4)^2 + lse(-1/2 ((z1 - 2) / 0.6)^2, -1/2 ((z1 + 2) / 0.6)^2)
//   kind 1 U2:     -1/2 ((z2 - w1) / 0.4)^2,  w1 = sin(pi z1 / 2)
//   kind 2 U2 gated: as U2 inside |z1| <= 4, -1e7 (zero gradient) outside (get_data.py:37-43)
//   kind 3 U3:     lse(-1/2 ((z2 - w1) / 0.35)^2, -1/2 ((z2 - w1 + w2) / 0.35)^2),
//                  w2 = 3 exp(-1/2 ((z1 - 1) / 0.6)^2)
//   kind 4 U4:     lse(-1/2 ((z2 - w1) / 0.4)^2, -1/2 ((z2 - w1 + w3) / 0.35)^2),
//                  w3 = 3 sigmoid((z1 - 1) / 0.3)
//   kind 5 U4 (theano_implement.py: w3 = 3 sigmoid^4)
//   kind 6 trial1: -1/2 ((|z| - 4) / 0.4)^2 + lse(-1/2 ((z1 - 2) / 0.8)^2, -1/2 ((z1 + 2) / 0.8)^2)
// Optional fused ELBO row: F_row = logq0 - ldj - beta * log p (beta from a device scalar), so a
// planar-flow VI step with millions of MC samples needs one launch for target + gradient.
#include "nf_common.h"

namespace nf {

// lse(a, b) and its weights (softmax of (a, b))
__device__ __forceinline__ float lse2(float a, float b, float& wa, float& wb) {
  const float m = fmaxf(a, b);
  const float ea = __expf(a - m), eb = __expf(b - m);
  const float s = ea + eb;
  wa = ea / s;
  wb = eb / s;
  return m + __logf(s);
}

__device__ __forceinline__ float ring_mix(float z1, float z2, float r0, float rs, float ms,
                                          float& g1, float& g2) {
  // -1/2 ((|z| - r0) / rs)^2 + lse(-1/2 ((z1 - 2) / ms)^2, -1/2 ((z1 + 2) / ms)^2)
  const float r = sqrtf(z1 * z1 + z2 * z2);
  const float ir2 = 1.f / (rs * rs), im2 = 1.f / (ms * ms);
  const float dr = (r - r0) * ir2;
  const float a = -0.5f * (z1 - 2.f) * (z1 - 2.f) * im2, b = -0.5f * (z1 + 2.f) * (z1 + 2.f) * im2;
  float wa, wb;
  const float l = lse2(a, b, wa, wb);
  const float ur = r > 0.f ? 1.f / r : 0.f;
  g1 = -dr * z1 * ur + wa * (-(z1 - 2.f) * im2) + wb * (-(z1 + 2.f) * im2);
  g2 = -dr * z2 * ur;
  return -0.5f * (r - r0) * (r - r0) * ir2 + l;
}

__device__ __forceinline__ float energy2d(int kind, float z1, float z2, float& g1, float& g2) {
  constexpr float kPi = 3.14159265358979323846f;
  if (kind == 0) return ring_mix(z1, z2, 2.f, 0.4f, 0.6f, g1, g2);
  if (kind == 6) return ring_mix(z1, z2, 4.f, 0.4f, 0.8f, g1, g2);
  float sn, cs;
  sincosf(0.5f * kPi * z1, &sn, &cs);
  const float w1 = sn, dw1 = 0.5f * kPi * cs;
  if (kind == 1 || kind == 2) {
    if (kind == 2 && fabsf(z1) > 4.f) {
      g1 = g2 = 0.f;
      return -1e7f;
    }
    const float is = 1.f / (0.4f * 0.4f);
    const float d = z2 - w1;
    g2 = -d * is;
    g1 = d * is * dw1;
    return -0.5f * d * d * is;
  }
  // U3 / U4: lse of two sheared Gaussians, the second offset by w(z1)
  float w, dw, sa, sb;
  if (kind == 3) {
    const float t = (z1 - 1.f) / 0.6f;
    w = 3.f * __expf(-0.5f * t * t);
    dw = -w * t / 0.6f;
    sa = sb = 0.35f;
  } else {
    const float sg = 1.f / (1.f + __expf(-(z1 - 1.f) / 0.3f));
    const float ds = sg * (1.f - sg) / 0.3f;
    if (kind == 5) {
      const float s2 = sg * sg;
      w = 3.f * s2 * s2;
      dw = 12.f * s2 * sg * ds;
    } else {
      w = 3.f * sg;
      dw = 3.f * ds;
    }
    sa = 0.4f;
    sb = 0.35f;
  }
  const float ia = 1.f / (sa * sa), ib = 1.f / (sb * sb);
  const float da = z2 - w1, db = z2 - w1 + w;
  float wa, wb;
  const float l = lse2(-0.5f * da * da * ia, -0.5f * db * db * ib, wa, wb);
  g2 = wa * (-da * ia) + wb * (-db * ib);
  g1 = wa * (da * ia * dw1) + wb * (-db * ib * (dw - dw1));
  return l;
}

__global__ void __launch_bounds__(256) energy2d_kernel(
    int kind, const float* __restrict__ z, long ldz, float* __restrict__ logp,
    float* __restrict__ grad, long ldg, float gscale, const float* __restrict__ logq0,
    const float* __restrict__ ldj, const float* __restrict__ beta_ptr, float* __restrict__ frow,
    int B) {
  const long row = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const float2 v = *reinterpret_cast<const float2*>(z + row * ldz);
  float g1, g2;
  const float lp = energy2d(kind, v.x, v.y, g1, g2);
  if (logp) logp[row] = lp;
  const float beta = beta_ptr ? *beta_ptr : 1.f;
  if (grad)   // gscale * grad log p  (e.g. -beta / B for dF/dz of the mean free energy)
    *reinterpret_cast<float2*>(grad + row * ldg) =
        make_float2(gscale * beta * g1, gscale * beta * g2);
  if (frow) frow[row] = (logq0 ? logq0[row] : 0.f) - (ldj ? ldj[row] : 0.f) - beta * lp;
}

}  // namespace nf

void nf_launch_energy2d(int kind, const float* z, long ldz, float* logp, float* grad, long ldg,
                        float gscale, const float* logq0, const float* ldj, const float* beta,
                        float* frow, int B, hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(nf::energy2d_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, kind, z,
                     ldz, logp, grad, ldg, gscale, logq0, ldj, beta, frow, B);
  NF_HIP_CHECK(hipGetLastError());
}
