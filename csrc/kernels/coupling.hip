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
    const float s = scale * tanhf(sh);
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

}  // namespace nf

using namespace nf;

template <typename TS, bool INV>
static void launch_cf(const void* st, long ld_st_, const float* x, long ld_x, float* y, long ld_y,
                      void* ybf, int ybf_is_bf16, long ld_yb, float* ssav, long ld_s, float* ldj,
                      int B, int Dh, float scale, int ldj_init, int yb_width, hipStream_t stream) {
  dim3 grid((B + 3) / 4), block(256);
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

void nf_launch_coupling_bwd(const float* gy, long ld_gy, const float* s, long ld_s, const float* x,
                            long ld_x, float c_scalar, const float* c_row, void* dst,
                            int dst_is_bf16, long ld_dst, float* gx, long ld_gx, int B, int Dh,
                            float scale, int gx_accumulate, int dst_pad_to, hipStream_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  if (dst_is_bf16)
    hipLaunchKernelGGL(coupling_bwd_kernel<bf16_t>, grid, block, 0, stream, gy, ld_gy, s, ld_s, x,
                       ld_x, c_scalar, c_row, (bf16_t*)dst, ld_dst, gx, ld_gx, B, Dh, scale,
                       gx_accumulate, dst_pad_to);
  else
    hipLaunchKernelGGL(coupling_bwd_kernel<float>, grid, block, 0, stream, gy, ld_gy, s, ld_s, x,
                       ld_x, c_scalar, c_row, (float*)dst, ld_dst, gx, ld_gx, B, Dh, scale,
                       gx_accumulate, dst_pad_to);
  NF_HIP_CHECK(hipGetLastError());
}
