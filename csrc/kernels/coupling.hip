// RealNVP affine-coupling epilogues (forward, inverse, backward) for gfx950.
//
// Layout (see vi_normflows_amd/flows/coupling.py for the math):
//   st   [B, ld_st]  conditioner output; s-hat in cols [0, Dh), t in cols [Dh, 2*Dh)
//   x    [B, ld_x]   fp32 half that is transformed (x_b)
//   y    [B, ld_y]   fp32 transformed half, y = x * exp(s) + t,  s = scale * tanh(s_hat)
//   ybf  [B, ld_yb]  bf16 copy of y (next layer's conditioner input); cols [Dh, ld_yb) zeroed
//   ssav [B, ld_s]   fp32 s, saved for backward
//   ldj  [B]         fp32 log|det J| accumulator, ldj += sum_j s_j  (inverse: -=)
//
// One wave64 owns one row; 4 rows per 256-thread block. Memory-bound: each
// lane streams float2/ushort2 pairs so a row of Dh=392 is ~3 iterations.
// The ldj row reduction is a 64-wide shuffle sum, so no LDS is needed.
#include "nf_common.h"

namespace nf {

template <typename TS>
__device__ __forceinline__ float ld_st(const TS* p, long i);
template <>
__device__ __forceinline__ float ld_st<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld_st<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

template <typename TS, bool INVERSE, typename TY>
__global__ void __launch_bounds__(256) coupling_fwd_kernel(
    const TS* __restrict__ st, long ld_st_, const float* __restrict__ x, long ld_x,
    float* __restrict__ y, long ld_y, TY* __restrict__ ybf, long ld_yb,
    float* __restrict__ ssav, long ld_s, float* __restrict__ ldj, int B, int Dh, float scale,
    int ldj_init, int yb_width) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const TS* st_r = st + row * ld_st_;
  const float* x_r = x + row * ld_x;
  float* y_r = y + row * ld_y;
  float acc = 0.f;
  for (int j = lane; j < Dh; j += 64) {
    const float sh = ld_st<TS>(st_r, j);
    const float t = ld_st<TS>(st_r, j + Dh);
    const float s = scale * fast_tanhf(sh);
    const float xv = x_r[j];
    float yv;
    if (INVERSE) {
      yv = (xv - t) * __expf(-s);
    } else {
      yv = fmaf(xv, __expf(s), t);
    }
    y_r[j] = yv;
    if (ybf) st_cv<TY>(ybf + row * ld_yb + j, yv);
    if (ssav) ssav[row * ld_s + j] = s;
    acc += s;
  }
  if (ybf) {
    for (int j = Dh + lane; j < yb_width; j += 64) ybf[row * ld_yb + j] = 0;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float d = INVERSE ? -acc : acc;
    ldj[row] = ldj_init ? d : ldj[row] + d;
  }
}

// Backward of the forward coupling transform.
//   gy  [B, ld_gy]  dL/dy
//   s   [B, ld_s]   saved s
//   x   [B, ld_x]   layer input half
//   c   dL/dldj per row (scalar c_scalar, or per-row array c_row if non-null)
// Outputs:
//   dst [B, ld_dst] bf16: cols [0,Dh) = dL/ds_hat, cols [Dh,2Dh) = dL/dt, pad cols zeroed
//   gx  [B, ld_gx]  dL/dx = gy * exp(s)   (gx_accumulate: +=)
template <typename TD>
__global__ void __launch_bounds__(256) coupling_bwd_kernel(
    const float* __restrict__ gy, long ld_gy, const float* __restrict__ s, long ld_s,
    const float* __restrict__ x, long ld_x, float c_scalar, const float* __restrict__ c_row,
    TD* __restrict__ dst, long ld_dst, float* __restrict__ gx, long ld_gx, int B, int Dh,
    float scale, int gx_accumulate, int dst_pad_to) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float c = c_row ? c_row[row] : c_scalar;
  const float inv_scale = 1.0f / scale;
  for (int j = lane; j < Dh; j += 64) {
    const float g = gy[row * ld_gy + j];
    const float sv = s[row * ld_s + j];
    const float es = __expf(sv);
    const float xv = x[row * ld_x + j];
    const float ds = fmaf(g * xv, es, c);            // dL/ds
    const float dsh = ds * (scale - sv * sv * inv_scale);  // ds/dshat = scale*(1 - tanh^2)
    st_cv<TD>(dst + row * ld_dst + j, dsh);
    st_cv<TD>(dst + row * ld_dst + Dh + j, g);
    const float gxv = g * es;
    float* gp = gx + row * ld_gx + j;
    *gp = gx_accumulate ? (*gp + gxv) : gxv;
  }
  for (int j = 2 * Dh + lane; j < dst_pad_to; j += 64) st_cv<TD>(dst + row * ld_dst + j, 0.f);
}


// ---------------------------------------------------------------------------------------
// Vectorised variants (Dh % 4 == 0, 16-B aligned fp32 rows / 8-B aligned bf16 rows): each
// lane moves 4 columns per step (float4 / ushort4), a Dh = 392 row is 2 steps of a wave.
// The backward can take s_hat (the bf16 conditioner output kept per layer) instead of a saved
// fp32 s: s = scale * tanh(s_hat) is recomputed - the forward computed it from the very same
// bf16 values, so the result is identical while the forward no longer writes (and the
// backward no longer reads) an fp32 [B, Dh] tensor per layer.
__device__ __forceinline__ void ld4(const float* p, float v[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void ld4(const bf16_t* p, float v[4]) {
  const ushort4 t = *reinterpret_cast<const ushort4*>(p);
  v[0] = bf2f(t.x); v[1] = bf2f(t.y); v[2] = bf2f(t.z); v[3] = bf2f(t.w);
}
__device__ __forceinline__ void st4(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st4(bf16_t* p, const float v[4]) {
  ushort4 t;
  t.x = f2bf(v[0]); t.y = f2bf(v[1]); t.z = f2bf(v[2]); t.w = f2bf(v[3]);
  *reinterpret_cast<ushort4*>(p) = t;
}

template <typename TS, bool INVERSE, typename TY>
__global__ void __launch_bounds__(256) coupling_fwd_vec_kernel(
    const TS* __restrict__ st, long ld_st_, const float* __restrict__ x, long ld_x,
    float* __restrict__ y, long ld_y, TY* __restrict__ ybf, long ld_yb,
    float* __restrict__ ssav, long ld_s, float* __restrict__ ldj, int B, int Dh, float scale,
    int ldj_init, int yb_width) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const TS* st_r = st + row * ld_st_;
  float acc = 0.f;
  for (int j = lane * 4; j < Dh; j += 256) {
    float sh[4], t[4], xv[4], yv[4], sv[4];
    ld4(st_r + j, sh);
    ld4(st_r + Dh + j, t);
    ld4(x + row * ld_x + j, xv);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sv[e] = scale * fast_tanhf(sh[e]);
      yv[e] = INVERSE ? (xv[e] - t[e]) * __expf(-sv[e]) : fmaf(xv[e], __expf(sv[e]), t[e]);
      acc += sv[e];
    }
    st4(y + row * ld_y + j, yv);
    if (ybf) st4(ybf + row * ld_yb + j, yv);
    if (ssav) st4(ssav + row * ld_s + j, sv);
  }
  if (ybf) {
    for (int j = Dh + lane; j < yb_width; j += 64) ybf[row * ld_yb + j] = 0;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float d = INVERSE ? -acc : acc;
    ldj[row] = ldj_init ? d : ldj[row] + d;
  }
}

// SH: s given as bf16 s_hat (recomputed) instead of fp32 s
template <typename TD, bool SH>
__global__ void __launch_bounds__(256) coupling_bwd_vec_kernel(
    const float* __restrict__ gy, long ld_gy, const void* __restrict__ s_in, long ld_s,
    const float* __restrict__ x, long ld_x, float c_scalar, const float* __restrict__ c_row,
    TD* __restrict__ dst, long ld_dst, float* __restrict__ gx, long ld_gx, int B, int Dh,
    float scale, int gx_accumulate, int dst_pad_to) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float c = c_row ? c_row[row] : c_scalar;
  const float inv_scale = 1.0f / scale;
  for (int j = lane * 4; j < Dh; j += 256) {
    float g[4], sv[4], xv[4], dsh[4], gxv[4];
    ld4(gy + row * ld_gy + j, g);
    if (SH) {
      ld4(reinterpret_cast<const bf16_t*>(s_in) + row * ld_s + j, sv);
#pragma unroll
      for (int e = 0; e < 4; ++e) sv[e] = scale * fast_tanhf(sv[e]);
    } else {
      ld4(reinterpret_cast<const float*>(s_in) + row * ld_s + j, sv);
    }
    ld4(x + row * ld_x + j, xv);
    if (gx_accumulate) ld4(gx + row * ld_gx + j, gxv);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float es = __expf(sv[e]);
      const float ds = fmaf(g[e] * xv[e], es, c);                 // dL/ds
      dsh[e] = ds * (scale - sv[e] * sv[e] * inv_scale);         // * ds/ds_hat
      gxv[e] = gx_accumulate ? fmaf(g[e], es, gxv[e]) : g[e] * es;
    }
    st4(dst + row * ld_dst + j, dsh);
    st4(dst + row * ld_dst + Dh + j, g);
    st4(gx + row * ld_gx + j, gxv);
  }
  for (int j = 2 * Dh + lane; j < dst_pad_to; j += 64) st_cv<TD>(dst + row * ld_dst + j, 0.f);
}

}  // namespace nf

using namespace nf;

static bool al(const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; }

template <typename TS, bool INV>
static void launch_cf(const void* st, long ld_st_, const float* x, long ld_x, float* y, long ld_y,
                      void* ybf, int ybf_is_bf16, long ld_yb, float* ssav, long ld_s, float* ldj,
                      int B, int Dh, float scale, int ldj_init, int yb_width, hipStream_t stream) {
  dim3 grid((B + 3) / 4), block(256);
  const int es = sizeof(TS);
  const bool vec = Dh % 4 == 0 && ld_st_ % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 &&
                   (!ybf || ld_yb % 4 == 0) && (!ssav || ld_s % 4 == 0) && al(st, 4 * es) &&
                   al(x, 16) && al(y, 16) && (!ybf || al(ybf, ybf_is_bf16 ? 8 : 16)) &&
                   (!ssav || al(ssav, 16));
  if (vec) {
    if (ybf_is_bf16)
      hipLaunchKernelGGL((coupling_fwd_vec_kernel<TS, INV, bf16_t>), grid, block, 0, stream,
                         (const TS*)st, ld_st_, x, ld_x, y, ld_y, (bf16_t*)ybf, ld_yb, ssav, ld_s,
                         ldj, B, Dh, scale, ldj_init, yb_width);
    else
      hipLaunchKernelGGL((coupling_fwd_vec_kernel<TS, INV, float>), grid, block, 0, stream,
                         (const TS*)st, ld_st_, x, ld_x, y, ld_y, (float*)ybf, ld_yb, ssav, ld_s,
                         ldj, B, Dh, scale, ldj_init, yb_width);
    return;
  }
  if (ybf_is_bf16)
    hipLaunchKernelGGL((coupling_fwd_kernel<TS, INV, bf16_t>), grid, block, 0, stream,
                       (const TS*)st, ld_st_, x, ld_x, y, ld_y, (bf16_t*)ybf, ld_yb, ssav, ld_s,
                       ldj, B, Dh, scale, ldj_init, yb_width);
  else
    hipLaunchKernelGGL((coupling_fwd_kernel<TS, INV, float>), grid, block, 0, stream,
                       (const TS*)st, ld_st_, x, ld_x, y, ld_y, (float*)ybf, ld_yb, ssav, ld_s,
                       ldj, B, Dh, scale, ldj_init, yb_width);
}

void nf_launch_coupling_fwd(const void* st, int st_is_bf16, long ld_st_, const float* x, long ld_x,
                            float* y, long ld_y, void* ybf, int ybf_is_bf16, long ld_yb,
                            float* ssav, long ld_s, float* ldj, int B, int Dh, float scale,
                            int inverse, int ldj_init, int yb_width, hipStream_t stream) {
  if (B <= 0) return;
  if (st_is_bf16) {
    if (inverse)
      launch_cf<bf16_t, true>(st, ld_st_, x, ld_x, y, ld_y, ybf, ybf_is_bf16, ld_yb, ssav, ld_s,
                              ldj, B, Dh, scale, ldj_init, yb_width, stream);
    else
      launch_cf<bf16_t, false>(st, ld_st_, x, ld_x, y, ld_y, ybf, ybf_is_bf16, ld_yb, ssav, ld_s,
                               ldj, B, Dh, scale, ldj_init, yb_width, stream);
  } else {
    if (inverse)
      launch_cf<float, true>(st, ld_st_, x, ld_x, y, ld_y, ybf, ybf_is_bf16, ld_yb, ssav, ld_s,
                             ldj, B, Dh, scale, ldj_init, yb_width, stream);
    else
      launch_cf<float, false>(st, ld_st_, x, ld_x, y, ld_y, ybf, ybf_is_bf16, ld_yb, ssav, ld_s,
                              ldj, B, Dh, scale, ldj_init, yb_width, stream);
  }
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_coupling_bwd(const void* s, int s_is_shat_bf16, long ld_s, const float* gy,
                            long ld_gy, const float* x, long ld_x, float c_scalar,
                            const float* c_row, void* dst, int dst_is_bf16, long ld_dst, float* gx,
                            long ld_gx, int B, int Dh, float scale, int gx_accumulate,
                            int dst_pad_to, hipStream_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  const bool vec = Dh % 4 == 0 && ld_gy % 4 == 0 && ld_s % 4 == 0 && ld_x % 4 == 0 &&
                   ld_dst % 4 == 0 && ld_gx % 4 == 0 && al(gy, 16) && al(x, 16) && al(gx, 16) &&
                   al(s, s_is_shat_bf16 ? 8 : 16) && al(dst, dst_is_bf16 ? 8 : 16);
  if (vec) {
#define NF_CB(TD, SH)                                                                          \
  hipLaunchKernelGGL((coupling_bwd_vec_kernel<TD, SH>), grid, block, 0, stream, gy, ld_gy, s,    \
                     ld_s, x, ld_x, c_scalar, c_row, (TD*)dst, ld_dst, gx, ld_gx, B, Dh, scale, \
                     gx_accumulate, dst_pad_to)
    if (dst_is_bf16) {
      if (s_is_shat_bf16) NF_CB(bf16_t, true); else NF_CB(bf16_t, false);
    } else {
      if (s_is_shat_bf16) NF_CB(float, true); else NF_CB(float, false);
    }
#undef NF_CB
    NF_HIP_CHECK(hipGetLastError());
    return;
  }
  if (s_is_shat_bf16) {
    fprintf(stderr, "coupling_bwd: s_hat input needs the vectorised layout (Dh %% 4 == 0)\n");
    abort();
  }
  if (dst_is_bf16)
    hipLaunchKernelGGL(coupling_bwd_kernel<bf16_t>, grid, block, 0, stream, gy, ld_gy, (const float*)s, ld_s, x,
                       ld_x, c_scalar, c_row, (bf16_t*)dst, ld_dst, gx, ld_gx, B, Dh, scale,
                       gx_accumulate, dst_pad_to);
  else
    hipLaunchKernelGGL(coupling_bwd_kernel<float>, grid, block, 0, stream, gy, ld_gy, (const float*)s, ld_s, x,
                       ld_x, c_scalar, c_row, (float*)dst, ld_dst, gx, ld_gx, B, Dh, scale,
                       gx_accumulate, dst_pad_to);
  NF_HIP_CHECK(hipGetLastError());
}
