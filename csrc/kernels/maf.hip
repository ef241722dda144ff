// Masked autoregressive flow (density direction) elementwise kernels for the MAF engine
// (vi_normflows_amd/models/maf_engine.py; Papamakarios et al. 2017):
//
//   o = MADE(x) = [mu | s_raw]  (bf16 [B, 2D], the second masked GEMM's output)
//   alpha = bound * tanh(s_raw / bound),   u = (x - mu) * exp(-alpha),   ldj -= sum_d alpha
//
// maf_fwd writes u (fp32 master of the next layer's input), its bf16 copy (the next layer's
// first GEMM operand in bf16 mode / weight-gradient operand) and optionally its e4m3 copy
// with a delayed per-tensor scale (amax of this call folded into amax_cur, as fp8.hip's
// quant_tensor) - the fp8 operand of the next layer's first GEMM, produced without another
// pass over u.
// maf_bwd: given g_u = dL/du (reads only s_raw of o: mu drops out of the backward),
// returns d_o = [dL/dmu | dL/ds_raw] (bf16, the masked GEMMs'
// gradient operand) and g_x = g_u * exp(-alpha) (fp32, the direct path; the MADE path is
// accumulated onto it by the input-gradient GEMM). c_ldj = dL/d(sum alpha) per row (e.g. 1/B
// for a batch-mean NLL).
// One wave per row, 4 columns per lane-step (float4 / 8-byte bf16 vectors).
#include "nf_common.h"

namespace nf {

constexpr float MAF_E4M3_MAX = 448.f;

__global__ void __launch_bounds__(256) maf_fwd_kernel(const float* __restrict__ x, long ldx,
                                                      const bf16_t* __restrict__ o, long ldo,
                                                      int B, int D, float bound,
                                                      float* __restrict__ u, long ldu,
                                                      bf16_t* __restrict__ ubf, long ldub,
                                                      unsigned char* __restrict__ uq, long lduq,
                                                      const float* __restrict__ amax_prev,
                                                      float* __restrict__ scale_out,
                                                      float* __restrict__ amax_cur,
                                                      float* __restrict__ ldj, int ldj_init) {
  const int lane = threadIdx.x & 63;
  float inv = 1.f;
  if (uq) {
    const float ap = *amax_prev;
    const float sc = ap > 0.f ? ap / MAF_E4M3_MAX : 1.f;
    inv = 1.f / sc;
    if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = sc;
  }
  float amax = 0.f;
  // grid-stride over rows: one amax atomic (at most) per block, not per row
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < B; row += gridDim.x * 4) {
    float sa = 0.f;
    const float* xr = x + (long)row * ldx;
    const bf16_t* mr = o + (long)row * ldo;
    const bf16_t* sr = mr + D;
    for (int c = lane * 4; c < D; c += 256) {
      const float4 xv = *reinterpret_cast<const float4*>(xr + c);
      const ushort4 mv = *reinterpret_cast<const ushort4*>(mr + c);
      const ushort4 sv = *reinterpret_cast<const ushort4*>(sr + c);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
      const float ms[4] = {bf2f(mv.x), bf2f(mv.y), bf2f(mv.z), bf2f(mv.w)};
      const float ss[4] = {bf2f(sv.x), bf2f(sv.y), bf2f(sv.z), bf2f(sv.w)};
      float us[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float al = bound * tanhf(ss[e] / bound);
        sa += al;
        us[e] = (xs[e] - ms[e]) * __expf(-al);
        amax = fmaxf(amax, fabsf(us[e]));
      }
      *reinterpret_cast<float4*>(u + (long)row * ldu + c) = make_float4(us[0], us[1], us[2], us[3]);
      if (ubf) {
        ushort4 b;
        b.x = f2bf(us[0]); b.y = f2bf(us[1]); b.z = f2bf(us[2]); b.w = f2bf(us[3]);
        *reinterpret_cast<ushort4*>(ubf + (long)row * ldub + c) = b;
      }
      if (uq) {
        int w = 0;
        w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(us[0] * inv, -MAF_E4M3_MAX), MAF_E4M3_MAX),
                                            fminf(fmaxf(us[1] * inv, -MAF_E4M3_MAX), MAF_E4M3_MAX),
                                            w, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(us[2] * inv, -MAF_E4M3_MAX), MAF_E4M3_MAX),
                                            fminf(fmaxf(us[3] * inv, -MAF_E4M3_MAX), MAF_E4M3_MAX),
                                            w, true);
        *reinterpret_cast<int*>(uq + (long)row * lduq + c) = w;
      }
    }
    sa = wave_sum(sa);
    if (lane == 0) ldj[row] = (ldj_init ? 0.f : ldj[row]) - sa;
  }
  if (uq) {
    __shared__ float red[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    if (lane == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0)
      amax_slot_atomic(amax_cur, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

__global__ void __launch_bounds__(256) maf_bwd_kernel(const float* __restrict__ gu, long ldg,
                                                      const float* __restrict__ u, long ldu,
                                                      const bf16_t* __restrict__ s_raw, long lds,
                                                      int B, int D, float bound, float c_ldj,
                                                      const float* __restrict__ c_row,
                                                      bf16_t* __restrict__ dout, long lddo,
                                                      float* __restrict__ gx, long ldgx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  if (c_row) c_ldj = c_row[row];   // per-row dL/d(sum alpha) (autograd callers)
  const float* gr = gu + (long)row * ldg;
  const float* ur = u + (long)row * ldu;
  const bf16_t* sr = s_raw + (long)row * lds;
  bf16_t* dm = dout + (long)row * lddo;
  bf16_t* ds = dm + D;
  for (int c = lane * 4; c < D; c += 256) {
    const float4 gv = *reinterpret_cast<const float4*>(gr + c);
    const float4 uv = *reinterpret_cast<const float4*>(ur + c);
    const ushort4 sv = *reinterpret_cast<const ushort4*>(sr + c);
    const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
    const float us[4] = {uv.x, uv.y, uv.z, uv.w};
    const float ss[4] = {bf2f(sv.x), bf2f(sv.y), bf2f(sv.z), bf2f(sv.w)};
    float dmu[4], dsr[4], gxs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t = tanhf(ss[e] / bound);
      const float al = bound * t;
      const float ea = __expf(-al);
      gxs[e] = gs[e] * ea;          // du/dx
      dmu[e] = -gs[e] * ea;         // du/dmu
      // du/dalpha = -u; ldj term: L += c_ldj * alpha
      dsr[e] = (c_ldj - gs[e] * us[e]) * (1.f - t * t);
    }
    *reinterpret_cast<float4*>(gx + (long)row * ldgx + c) = make_float4(gxs[0], gxs[1], gxs[2], gxs[3]);
    ushort4 a, b;
    a.x = f2bf(dmu[0]); a.y = f2bf(dmu[1]); a.z = f2bf(dmu[2]); a.w = f2bf(dmu[3]);
    b.x = f2bf(dsr[0]); b.y = f2bf(dsr[1]); b.z = f2bf(dsr[2]); b.w = f2bf(dsr[3]);
    *reinterpret_cast<ushort4*>(dm + c) = a;
    *reinterpret_cast<ushort4*>(ds + c) = b;
  }
}

// ---------------------------------------------------------------- gated IAF update
// Kingma et al. 2016 (eq. 11-12), the VI direction of an IAF layer, o = MADE(z, h) = [m | s]:
//   sig = sigmoid(s + gate_bias),  y = sig * z + (1 - sig) * m = m + sig * (z - m),
//   ldj = sum_d log sig
// iaf_gate_bwd, given gy = dL/dy and gl = dL/dldj (per row, optional):
//   gz = gy sig,  dm = gy (1 - sig),  ds = gy sig (1 - sig)(z - m) + gl (1 - sig)
// (d log sig / ds = 1 - sig). d_o = [dm | ds] is written in bf16 (the masked GEMMs' operand).
// One wave per row, 4 columns per lane-step.
__device__ __forceinline__ float sigmoidf_(float t) { return 1.f / (1.f + __expf(-t)); }
__device__ __forceinline__ float log_sigmoidf_(float t) {   // min(t, 0) - log1p(exp(-|t|))
  return fminf(t, 0.f) - log1pf(__expf(-fabsf(t)));
}

__global__ void __launch_bounds__(256) iaf_gate_fwd_kernel(const bf16_t* __restrict__ o, long ldo,
                                                           const float* __restrict__ z, long ldz,
                                                           int B, int D, float gb,
                                                           float* __restrict__ y, long ldy,
                                                           float* __restrict__ ldj,
                                                           bf16_t* __restrict__ ybf, long ldyb) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const bf16_t* mr = o + (long)row * ldo;
  const bf16_t* sr = mr + D;
  const float* zr = z + (long)row * ldz;
  float* yr = y + (long)row * ldy;
  bf16_t* ybr = ybf ? ybf + (long)row * ldyb : nullptr;   // the next MADE's bf16 operand
  float acc = 0.f;
  for (int c = lane * 4; c < D; c += 256) {
    const ushort4 mv = *reinterpret_cast<const ushort4*>(mr + c);
    const ushort4 sv = *reinterpret_cast<const ushort4*>(sr + c);
    const float4 zv = *reinterpret_cast<const float4*>(zr + c);
    const float ms[4] = {bf2f(mv.x), bf2f(mv.y), bf2f(mv.z), bf2f(mv.w)};
    const float ss[4] = {bf2f(sv.x), bf2f(sv.y), bf2f(sv.z), bf2f(sv.w)};
    const float zs[4] = {zv.x, zv.y, zv.z, zv.w};
    float ys[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t = ss[e] + gb;
      ys[e] = fmaf(sigmoidf_(t), zs[e] - ms[e], ms[e]);
      acc += log_sigmoidf_(t);
    }
    *reinterpret_cast<float4*>(yr + c) = make_float4(ys[0], ys[1], ys[2], ys[3]);
    if (ybr) {
      ushort4 b;
      b.x = f2bf(ys[0]); b.y = f2bf(ys[1]); b.z = f2bf(ys[2]); b.w = f2bf(ys[3]);
      *reinterpret_cast<ushort4*>(ybr + c) = b;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) ldj[row] = acc;
}

__global__ void __launch_bounds__(256) iaf_gate_bwd_kernel(const float* __restrict__ gy, long ldg,
                                                           const float* __restrict__ gl,
                                                           const float* __restrict__ z, long ldz,
                                                           const bf16_t* __restrict__ o, long ldo,
                                                           int B, int D, float gb,
                                                           bf16_t* __restrict__ dout, long lddo,
                                                           float* __restrict__ gz, long ldgz) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float g_l = gl ? gl[row] : 0.f;
  const bf16_t* mr = o + (long)row * ldo;
  const bf16_t* sr = mr + D;
  const float* gr = gy + (long)row * ldg;
  const float* zr = z + (long)row * ldz;
  bf16_t* dm = dout + (long)row * lddo;
  bf16_t* ds = dm + D;
  for (int c = lane * 4; c < D; c += 256) {
    const ushort4 mv = *reinterpret_cast<const ushort4*>(mr + c);
    const ushort4 sv = *reinterpret_cast<const ushort4*>(sr + c);
    const float4 zv = *reinterpret_cast<const float4*>(zr + c);
    const float4 gv = *reinterpret_cast<const float4*>(gr + c);
    const float ms[4] = {bf2f(mv.x), bf2f(mv.y), bf2f(mv.z), bf2f(mv.w)};
    const float ss[4] = {bf2f(sv.x), bf2f(sv.y), bf2f(sv.z), bf2f(sv.w)};
    const float zs[4] = {zv.x, zv.y, zv.z, zv.w};
    const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
    float gzs[4], dms[4], dss[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sg = sigmoidf_(ss[e] + gb), om = 1.f - sg;
      gzs[e] = gs[e] * sg;
      dms[e] = gs[e] * om;
      dss[e] = om * fmaf(gs[e] * sg, zs[e] - ms[e], g_l);
    }
    *reinterpret_cast<float4*>(gz + (long)row * ldgz + c) = make_float4(gzs[0], gzs[1], gzs[2], gzs[3]);
    ushort4 a, b;
    a.x = f2bf(dms[0]); a.y = f2bf(dms[1]); a.z = f2bf(dms[2]); a.w = f2bf(dms[3]);
    b.x = f2bf(dss[0]); b.y = f2bf(dss[1]); b.z = f2bf(dss[2]); b.w = f2bf(dss[3]);
    *reinterpret_cast<ushort4*>(dm + c) = a;
    *reinterpret_cast<ushort4*>(ds + c) = b;
  }
}

}  // namespace nf

using namespace nf;

void nf_launch_iaf_gate_fwd(const void* o, long ldo, const float* z, long ldz, int B, int D,
                            float gate_bias, float* y, long ldy, float* ldj, hipStream_t stream,
                            void* ybf, long ldyb) {
  if (B <= 0) return;
  hipLaunchKernelGGL(iaf_gate_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, stream,
                     (const bf16_t*)o, ldo, z, ldz, B, D, gate_bias, y, ldy, ldj, (bf16_t*)ybf,
                     ldyb);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_iaf_gate_bwd(const float* gy, long ldg, const float* gl, const float* z, long ldz,
                            const void* o, long ldo, int B, int D, float gate_bias, void* dout,
                            long lddo, float* gz, long ldgz, hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(iaf_gate_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, gy, ldg, gl, z,
                     ldz, (const bf16_t*)o, ldo, B, D, gate_bias, (bf16_t*)dout, lddo, gz, ldgz);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_maf_fwd(const float* x, long ldx, const void* o, long ldo, int B, int D, float bound,
                       float* u, long ldu, void* ubf, long ldub, void* uq, long lduq,
                       const float* amax_prev, float* scale_out, float* amax_cur, float* ldj,
                       int ldj_init, hipStream_t stream) {
  if (B <= 0) return;
  // a memory-bound pass: one wave per row, full grid; with the e4m3 output each block folds its
  // rows' amax into one atomic that a plain read skips once the running max has settled
  const int nb = (B + 3) / 4;
  const int grid = nb;
  hipLaunchKernelGGL(maf_fwd_kernel, dim3(grid), dim3(256), 0, stream, x, ldx,
                     (const bf16_t*)o, ldo, B, D, bound, u, ldu, (bf16_t*)ubf, ldub,
                     (unsigned char*)uq, lduq, amax_prev, scale_out, amax_cur, ldj, ldj_init);
  NF_HIP_CHECK(hipGetLastError());
}

// s_raw: the s half of o = [mu | s_raw] (row stride lds), or the engine's own s buffer
void nf_launch_maf_bwd(const float* gu, long ldg, const float* u, long ldu, const void* s_raw,
                       long lds, int B, int D, float bound, float c_ldj, void* dout, long lddo,
                       float* gx, long ldgx, hipStream_t stream, const float* c_row) {
  if (B <= 0) return;
  hipLaunchKernelGGL(maf_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, gu, ldg, u, ldu,
                     (const bf16_t*)s_raw, lds, B, D, bound, c_ldj, c_row, (bf16_t*)dout, lddo, gx,
                     ldgx);
  NF_HIP_CHECK(hipGetLastError());
}
