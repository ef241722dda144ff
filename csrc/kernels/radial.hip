// Fused K-layer radial flow stack, forward + backward (gfx950).
//
//   f(z) = z + beta h(r) (z - z0),   r = ||z - z0||,   h = 1 / (alpha + r)
//   log|det J| = (D-1) log(1 + beta h) + log(1 + beta alpha h^2)
// (Rezende & Mohamed 2015, Sec. 3.2; named but never implemented in the reference,
//  normflows/normflows/flows.py:1.)  alpha > 0 and beta >= -alpha are enforced by the
// caller's reparameterisation (softplus), so the map is invertible.
// Same row mapping / per-row gradient scheme as planar.hip.
#include "nf_common.h"

namespace nf {

template <bool WROW>
__device__ __forceinline__ float rsum_r(float v) {
  if (WROW) return wave_sum(v);
  return v;
}

struct RadialArgs {
  const float* z;
  const float* Z0;     // [K][D] or [K][N][D]
  const float* AL;     // alpha [K] or [K][N]
  const float* BE;     // beta  [K] or [K][N]
  float* zK;
  float* ldj;
  float* saved;        // [K][N][D]
  const float* gz;
  const float* gl;
  float* dz;
  float* dZ0;          // [K][N][D]
  float* dA;           // [K][N]
  float* dBe;          // [K][N]
  int N, D, K, per_sample;
};

template <bool WROW, int PER>
__global__ void __launch_bounds__(256) radial_fwd_kernel(RadialArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = WROW ? (((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6)
                        : ((long)blockIdx.x * blockDim.x + threadIdx.x);
  if (row >= a.N) return;
  const int D = a.D;
  float z[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = WROW ? lane + 64 * i : i;
    z[i] = j < D ? a.z[row * D + j] : 0.f;
  }
  float ldj = 0.f;
  for (int k = 0; k < a.K; ++k) {
    const long pb = a.per_sample ? ((long)k * a.N + row) * D : (long)k * D;
    const long sb = a.per_sample ? (long)k * a.N + row : k;
    const float al = a.AL[sb], be = a.BE[sb];
    float d[PER];
    float rr = 0.f;
    float* sv = a.saved + ((long)k * a.N + row) * D;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = WROW ? lane + 64 * i : i;
      d[i] = j < D ? z[i] - a.Z0[pb + j] : 0.f;
      if (j < D) sv[j] = z[i];
      rr += d[i] * d[i];
    }
    rr = rsum_r<WROW>(rr);
    const float r = sqrtf(rr);
    const float h = 1.f / (al + r);
    const float bh = be * h;
#pragma unroll
    for (int i = 0; i < PER; ++i) z[i] += bh * d[i];
    ldj += (float)(D - 1) * __logf(fabsf(1.f + bh)) + __logf(fabsf(1.f + be * al * h * h));
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = WROW ? lane + 64 * i : i;
    if (j < D) a.zK[row * D + j] = z[i];
  }
  if (!WROW || lane == 0) a.ldj[row] = ldj;
}

template <bool WROW, int PER>
__global__ void __launch_bounds__(256) radial_bwd_kernel(RadialArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = WROW ? (((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6)
                        : ((long)blockIdx.x * blockDim.x + threadIdx.x);
  if (row >= a.N) return;
  const int D = a.D;
  const float Dm1 = (float)(D - 1);
  float g[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = WROW ? lane + 64 * i : i;
    g[i] = j < D ? a.gz[row * D + j] : 0.f;
  }
  const float c = a.gl[row];
  for (int k = a.K - 1; k >= 0; --k) {
    const long pb = a.per_sample ? ((long)k * a.N + row) * D : (long)k * D;
    const long sb = a.per_sample ? (long)k * a.N + row : k;
    const float al = a.AL[sb], be = a.BE[sb];
    const float* sv = a.saved + ((long)k * a.N + row) * D;
    float d[PER];
    float rr = 0.f, gd = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = WROW ? lane + 64 * i : i;
      d[i] = j < D ? sv[j] - a.Z0[pb + j] : 0.f;
      rr += d[i] * d[i];
      gd += g[i] * d[i];
    }
    rr = rsum_r<WROW>(rr);
    gd = rsum_r<WROW>(gd);
    const float r = sqrtf(rr);
    const float ir = r > 1e-20f ? 1.f / r : 0.f;
    const float h = 1.f / (al + r);
    const float h2 = h * h;
    const float bh = be * h;
    const float q1 = 1.f + bh;            // (D-1) log q1
    const float q2 = 1.f + be * al * h2;  // log q2
    // dldj/dr = -(D-1) beta h^2 / q1 - 2 beta alpha h^3 / q2
    const float dldj_dr = -Dm1 * be * h2 / q1 - 2.f * be * al * h2 * h / q2;
    // coefficient on d in dL/dz beyond (1 + beta h) g
    const float coef_d = -be * h2 * gd * ir + c * dldj_dr * ir;
    const float dbe = gd * h + c * (Dm1 * h / q1 + al * h2 / q2);
    const float dal = -be * h2 * gd + c * (-Dm1 * be * h2 / q1 + be * h2 * (1.f - 2.f * al * h) / q2);
    float* dZr = a.dZ0 + ((long)k * a.N + row) * D;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = WROW ? lane + 64 * i : i;
      const float via_d = bh * g[i] + coef_d * d[i];   // dL/dd (excluding the identity path)
      if (j < D) dZr[j] = -via_d;
      g[i] = g[i] + via_d;
    }
    if (!WROW || lane == 0) {
      a.dA[(long)k * a.N + row] = dal;
      a.dBe[(long)k * a.N + row] = dbe;
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = WROW ? lane + 64 * i : i;
    if (j < D) a.dz[row * D + j] = g[i];
  }
}

template <bool WROW, int PER>
static void launch_radial(const RadialArgs& a, bool bwd, hipStream_t stream) {
  const long threads = WROW ? (long)a.N * 64 : (long)a.N;
  dim3 grid((unsigned)((threads + 255) / 256)), block(256);
  if (bwd)
    hipLaunchKernelGGL((radial_bwd_kernel<WROW, PER>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((radial_fwd_kernel<WROW, PER>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

static void dispatch_radial(const RadialArgs& a, bool bwd, hipStream_t stream) {
  const int D = a.D;
  if (D <= 2) return launch_radial<false, 2>(a, bwd, stream);
  if (D <= 4) return launch_radial<false, 4>(a, bwd, stream);
  if (D <= 8) return launch_radial<false, 8>(a, bwd, stream);
  if (D <= 16) return launch_radial<false, 16>(a, bwd, stream);
  if (D <= 64) return launch_radial<true, 1>(a, bwd, stream);
  if (D <= 128) return launch_radial<true, 2>(a, bwd, stream);
  if (D <= 256) return launch_radial<true, 4>(a, bwd, stream);
  if (D <= 512) return launch_radial<true, 8>(a, bwd, stream);
  return launch_radial<true, 16>(a, bwd, stream);
}

}  // namespace nf

using namespace nf;

void nf_launch_radial_fwd(const float* z, const float* Z0, const float* AL, const float* BE,
                          float* zK, float* ldj, float* saved, int N, int D, int K,
                          int per_sample, hipStream_t stream) {
  if (N <= 0) return;
  RadialArgs a{};
  a.z = z; a.Z0 = Z0; a.AL = AL; a.BE = BE; a.zK = zK; a.ldj = ldj; a.saved = saved;
  a.N = N; a.D = D; a.K = K; a.per_sample = per_sample;
  dispatch_radial(a, false, stream);
}

void nf_launch_radial_bwd(const float* saved, const float* Z0, const float* AL, const float* BE,
                          const float* gz, const float* gl, float* dz, float* dZ0, float* dA,
                          float* dBe, int N, int D, int K, int per_sample, hipStream_t stream) {
  if (N <= 0) return;
  RadialArgs a{};
  a.saved = (float*)saved; a.Z0 = Z0; a.AL = AL; a.BE = BE; a.gz = gz; a.gl = gl; a.dz = dz;
  a.dZ0 = dZ0; a.dA = dA; a.dBe = dBe;
  a.N = N; a.D = D; a.K = K; a.per_sample = per_sample;
  dispatch_radial(a, true, stream);
}
