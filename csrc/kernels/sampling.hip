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
    long ldzb, int nbf, float* __restrict__ logq0, int B, int D, int vec) {
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
    if (vec && 4 * g + 3 < D) {
      // whole float4 group: 16-B stores of z / eps, 8-B store of the bf16 copy
      const int j = 4 * g;
      const float4 lv4 = logvar ? *reinterpret_cast<const float4*>(logvar + j) : make_float4(0, 0, 0, 0);
      const float4 m4 = mu ? *reinterpret_cast<const float4*>(mu + j) : make_float4(0, 0, 0, 0);
      float4 z4;
      z4.x = fmaf(__expf(0.5f * lv4.x), n[0], m4.x);
      z4.y = fmaf(__expf(0.5f * lv4.y), n[1], m4.y);
      z4.z = fmaf(__expf(0.5f * lv4.z), n[2], m4.z);
      z4.w = fmaf(__expf(0.5f * lv4.w), n[3], m4.w);
      *reinterpret_cast<float4*>(z + row * ldz + j) = z4;
      if (eps_out) *reinterpret_cast<float4*>(eps_out + row * lde + j) = make_float4(n[0], n[1], n[2], n[3]);
      if (zbf && j + 3 < nbf) {
        st_cv<TZ>(zbf + row * ldzb + j, z4.x);
        st_cv<TZ>(zbf + row * ldzb + j + 1, z4.y);
        st_cv<TZ>(zbf + row * ldzb + j + 2, z4.z);
        st_cv<TZ>(zbf + row * ldzb + j + 3, z4.w);
      } else if (zbf) {
        const float zz[4] = {z4.x, z4.y, z4.z, z4.w};
        for (int q = 0; q < 4; ++q)
          if (j + q < nbf) st_cv<TZ>(zbf + row * ldzb + j + q, zz[q]);
      }
      sq += (n[0] * n[0] + n[1] * n[1]) + (n[2] * n[2] + n[3] * n[3]);
      slv += (lv4.x + lv4.y) + (lv4.z + lv4.w);
      continue;
    }
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

// Backward of z0 = mu + exp(logvar/2) * eps for the learnable diagonal base:
//   gmu[c] = sum_b g[b,c],  glv[c] = 0.5 exp(lv[c]/2) sum_b g[b,c] eps[b,c] - 0.5
// where dL/dz0 arrives as two strided column blocks (g_lo = columns [0, Dl), g_hi = [Dl, D)),
// so no concatenated copy is materialised. Pass 1: each block owns a row slab and every
// column (one float4 column group per thread) and writes its two column sums to its own
// partial row; pass 2 sums the partial rows in a fixed order (bitwise deterministic).
__global__ void __launch_bounds__(256) reparam_grad_partial_kernel(
    const float* __restrict__ g_lo, long ldlo, const float* __restrict__ g_hi, long ldhi,
    const float* __restrict__ eps, long lde, float* __restrict__ partial, int B, int D, int Dl,
    int rows_per) {
  const int q = threadIdx.x;  // float4 column group
  if (4 * q >= D) return;
  const int c = 4 * q;
  const float* gp = c < Dl ? g_lo + c : g_hi + (c - Dl);
  const long ldg = c < Dl ? ldlo : ldhi;
  const long r0 = (long)blockIdx.x * rows_per;
  const long r1 = min((long)B, r0 + rows_per);
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  long r = r0;
  for (; r + 4 <= r1; r += 4) {
    float4 g[4], e[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      g[u] = *reinterpret_cast<const float4*>(gp + (r + u) * ldg);
      e[u] = *reinterpret_cast<const float4*>(eps + (r + u) * lde + c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s1.x += g[u].x; s1.y += g[u].y; s1.z += g[u].z; s1.w += g[u].w;
      s2.x = fmaf(g[u].x, e[u].x, s2.x); s2.y = fmaf(g[u].y, e[u].y, s2.y);
      s2.z = fmaf(g[u].z, e[u].z, s2.z); s2.w = fmaf(g[u].w, e[u].w, s2.w);
    }
  }
  for (; r < r1; ++r) {
    const float4 g = *reinterpret_cast<const float4*>(gp + r * ldg);
    const float4 e = *reinterpret_cast<const float4*>(eps + r * lde + c);
    s1.x += g.x; s1.y += g.y; s1.z += g.z; s1.w += g.w;
    s2.x = fmaf(g.x, e.x, s2.x); s2.y = fmaf(g.y, e.y, s2.y);
    s2.z = fmaf(g.z, e.z, s2.z); s2.w = fmaf(g.w, e.w, s2.w);
  }
  float* out = partial + (long)blockIdx.x * 2 * D;
  *reinterpret_cast<float4*>(out + c) = s1;
  *reinterpret_cast<float4*>(out + D + c) = s2;
}

// One block per 64 columns: wave w sums partial rows w, w+4, ... for its lane's column (8 rows
// per batch of independent loads), then the 4 wave sums combine in a fixed order via LDS.
__global__ void __launch_bounds__(256) reparam_grad_finalize_kernel(
    const float* __restrict__ partial, int np, const float* __restrict__ logvar,
    float* __restrict__ gmu, float* __restrict__ glv, int D) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s1 = 0.f, s2 = 0.f;
  if (c < D) {
    int p = w;
    for (; p + 28 < np; p += 32) {
      float a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = partial[(long)(p + 4 * u) * 2 * D + c];
        b[u] = partial[(long)(p + 4 * u) * 2 * D + D + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += a[u];
        s2 += b[u];
      }
    }
    for (; p < np; p += 4) {
      s1 += partial[(long)p * 2 * D + c];
      s2 += partial[(long)p * 2 * D + D + c];
    }
  }
  red[0][w][lane] = s1;
  red[1][w][lane] = s2;
  __syncthreads();
  if (w == 0 && c < D) {
    const float t1 = (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]);
    const float t2 = (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]);
    gmu[c] = t1;
    glv[c] = 0.5f * __expf(0.5f * logvar[c]) * t2 - 0.5f;
  }
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
  // float4 groups need 16-B aligned rows of z / eps / mu / logvar
  const auto al16 = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
  const int vec = (D % 4 == 0) && (ldz % 4 == 0) && (eps == nullptr || lde % 4 == 0) && al16(z) &&
                  al16(eps) && al16(mu) && al16(logvar);
  if (zbf_is_bf16 || zbf == nullptr)
    hipLaunchKernelGGL(reparam_sample_kernel<bf16_t>, grid, block, 0, stream, mu, logvar,
                       (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), offset_ptr,
                       offset_host, stream_id, z, ldz, eps, lde, (bf16_t*)zbf, ldzb, nbf, logq0, B,
                       D, vec);
  else
    hipLaunchKernelGGL(reparam_sample_kernel<float>, grid, block, 0, stream, mu, logvar,
                       (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), offset_ptr,
                       offset_host, stream_id, z, ldz, eps, lde, (float*)zbf, ldzb, nbf, logq0, B,
                       D, vec);
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

void nf_launch_reparam_grad(const float* g_lo, long ldlo, const float* g_hi, long ldhi,
                            const float* eps, long lde, const float* logvar, float* partial,
                            int npartial, float* gmu, float* glv, int B, int D, int Dl,
                            hipStream_t stream) {
  if (B <= 0 || D <= 0) return;
  const int rows_per = (B + npartial - 1) / npartial;
  const int np = (B + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(reparam_grad_partial_kernel, dim3(np), dim3(256), 0, stream, g_lo, ldlo,
                     g_hi, ldhi, eps, lde, partial, B, D, Dl, rows_per);
  hipLaunchKernelGGL(reparam_grad_finalize_kernel, dim3((D + 63) / 64), dim3(256), 0, stream,
                     partial, np, logvar, gmu, glv, D);
  NF_HIP_CHECK(hipGetLastError());
}
