// Reparameterised base sampling z0 = mu + exp(logvar/2) * eps, eps ~ N(0, I), fused
// with log q0(z0) = -D/2 log(2 pi) - 1/2 sum(logvar) - 1/2 sum(eps^2) (gfx950).
//
// RNG: Philox4x32-10 keyed by a 64-bit seed; the counter is (element group,
// row, offset_lo, offset_hi ^ stream). `stream` separates data-parallel ranks
// (rank-distinct Monte-Carlo noise keeps the DP estimator unbiased); the
// offset is read from device memory so a captured hipGraph draws fresh noise
// each replay once the step counter is bumped on the device.
#include "nf_common.h"

namespace nf {

template <typename TZ>
__global__ void __launch_bounds__(256) reparam_sample_kernel(
    const float* __restrict__ mu, const float* __restrict__ logvar, uint32_t seed_lo,
    uint32_t seed_hi, const int64_t* __restrict__ offset_ptr, int64_t offset_host, uint32_t stream,
    float* __restrict__ z, long ldz, float* __restrict__ eps_out, long lde, TZ* __restrict__ zbf,
    long ldzb, int nbf, float* __restrict__ logq0, int B, int D) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const int64_t off = offset_ptr ? *offset_ptr : offset_host;
  const uint32_t c2 = (uint32_t)(off & 0xffffffffu);
  const uint32_t c3 = (uint32_t)((uint64_t)off >> 32) ^ (stream * 0x9E3779B9u);
  float sq = 0.f, slv = 0.f;
  for (int g = lane; g * 4 < D; g += 64) {
    const Philox4 r = philox4x32_10((uint32_t)g, (uint32_t)row, c2, c3, seed_lo, seed_hi);
    float n[4];
    box_muller(r.x, r.y, n[0], n[1]);
    box_muller(r.z, r.w, n[2], n[3]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 4 * g + q;
      if (j < D) {
        const float e = n[q];
        const float lv = logvar ? logvar[j] : 0.f;
        const float m = mu ? mu[j] : 0.f;
        const float zv = fmaf(__expf(0.5f * lv), e, m);
        z[row * ldz + j] = zv;
        if (eps_out) eps_out[row * lde + j] = e;
        if (zbf && j < nbf) st_cv<TZ>(zbf + row * ldzb + j, zv);
        sq += e * e;
        slv += lv;
      }
    }
  }
  if (zbf) {
    for (int j = nbf + lane; j < ldzb; j += 64) st_cv<TZ>(zbf + row * ldzb + j, 0.f);
  }
  sq = wave_sum(sq);
  slv = wave_sum(slv);
  if (lane == 0 && logq0) logq0[row] = -0.5f * (float)D * 1.8378770664093453f - 0.5f * slv - 0.5f * sq;
}

// Plain N(0,1) fill with the same counter scheme (used by MC estimators and tests).
__global__ void __launch_bounds__(256) normal_fill_kernel(float* __restrict__ out, long n,
                                                           uint32_t seed_lo, uint32_t seed_hi,
                                                           const int64_t* __restrict__ offset_ptr,
                                                           int64_t offset_host, uint32_t stream) {
  const int64_t off = offset_ptr ? *offset_ptr : offset_host;
  const uint32_t c2 = (uint32_t)(off & 0xffffffffu);
  const uint32_t c3 = (uint32_t)((uint64_t)off >> 32) ^ (stream * 0x9E3779B9u);
  const long ngroups = (n + 3) / 4;
  for (long g = (long)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
       g += (long)gridDim.x * blockDim.x) {
    const Philox4 r = philox4x32_10((uint32_t)(g & 0xffffffff), (uint32_t)(g >> 32) ^ 0x5bd1e995u,
                                    c2, c3, seed_lo, seed_hi);
    float v[4];
    box_muller(r.x, r.y, v[0], v[1]);
    box_muller(r.z, r.w, v[2], v[3]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long i = 4 * g + q;
      if (i < n) out[i] = v[q];
    }
  }
}

}  // namespace nf

using namespace nf;

void nf_launch_reparam_sample(const float* mu, const float* logvar, uint64_t seed,
                              const int64_t* offset_ptr, int64_t offset_host, uint32_t stream_id,
                              float* z, long ldz, float* eps, long lde, void* zbf, int zbf_is_bf16,
                              long ldzb, int nbf, float* logq0, int B, int D, hipStream_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  if (zbf_is_bf16 || zbf == nullptr)
    hipLaunchKernelGGL(reparam_sample_kernel<bf16_t>, grid, block, 0, stream, mu, logvar,
                       (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), offset_ptr,
                       offset_host, stream_id, z, ldz, eps, lde, (bf16_t*)zbf, ldzb, nbf, logq0, B,
                       D);
  else
    hipLaunchKernelGGL(reparam_sample_kernel<float>, grid, block, 0, stream, mu, logvar,
                       (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), offset_ptr,
                       offset_host, stream_id, z, ldz, eps, lde, (float*)zbf, ldzb, nbf, logq0, B,
                       D);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_normal_fill(float* out, long n, uint64_t seed, const int64_t* offset_ptr,
                           int64_t offset_host, uint32_t stream_id, hipStream_t stream) {
  if (n <= 0) return;
  long ngroups = (n + 3) / 4;
  long blocks = (ngroups + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(normal_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, out, n,
                     (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), offset_ptr,
                     offset_host, stream_id);
  NF_HIP_CHECK(hipGetLastError());
}
