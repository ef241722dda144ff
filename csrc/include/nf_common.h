// Shared device helpers for the vi_normflows_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, reductions use 64-wide shuffles;
//   * bf16 is carried as raw uint16 bits (vector loads as ushort4/ushort8) and
//     converted with the hardware v_cvt_pk_bf16_f32 path (plain __float2bfloat16);
//   * launchers are plain C++ functions taking raw pointers + hipStream_t so that
//     kernel translation units never include torch headers.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define NF_WAVE 64

#define NF_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      nf_throw_hip_error(_e, #expr, __FILE__, __LINE__);                          \
    }                                                                             \
  } while (0)

#include "launchers.h"

namespace nf {

typedef unsigned short bf16_t;  // raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

// Store a float into a bf16 or fp32 "compute copy" buffer.
template <typename T>
__device__ __forceinline__ void st_cv(T* p, float v);
template <>
__device__ __forceinline__ void st_cv<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st_cv<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `scratch` holds >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// tanh for the affine-coupling scale s = c tanh(s_hat): sign(x) (1 - 2 / (1 + e^{2|x|})), one
// v_exp_f32 + one v_rcp_f32 (libm tanhf is a ~25-instruction branchy sequence, and the fused
// coupling epilogues evaluate it for every element of a 256-row tile while no MFMA runs).
// Absolute error ~1e-7 (the s_hat it reads is bf16); e^{2|x|} = inf gives exactly +-1.
// The reciprocal is v_rcp_f32 itself (1 ulp): HIP's __fdividef is an IEEE division here, a
// ~10-instruction v_div_scale / v_div_fmas / v_div_fixup sequence plus its hazard nops, and it
// made up most of the VALU work of every coupling / MAF epilogue (12.7k v_div_scale_f32 in
// gemm256.hip alone before this).
__device__ __forceinline__ float fast_tanhf(float x) {
  const float e = __expf(2.f * fabsf(x));
  return copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e), x);
}

// Numerically stable softplus and log(1+x) helpers used by flow kernels.
__device__ __forceinline__ float softplusf(float x) {
  return x > 20.f ? x : log1pf(__expf(x));
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al. 2011). Each (seed, counter)
// pair yields 4 independent uint32. Streams are distinguished by the 64-bit
// counter's high word (subsequence) and an offset advanced on the device, so a
// captured hipGraph replays fresh randomness each step.
// ---------------------------------------------------------------------------
struct Philox4 { uint32_t x, y, z, w; };

__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n1 = lo1;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    const uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0; k1 += W1;
  }
  return Philox4{c0, c1, c2, c3};
}

__device__ __forceinline__ float u32_to_unit_open(uint32_t x) {
  // (0, 1]: never 0 so log() is finite.
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Box-Muller on two uniforms -> two standard normals.
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
  const float u1 = u32_to_unit_open(a);
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.0f * __logf(u1));
  float s, c;
  __sincosf(6.283185307179586f * u2, &s, &c);
  n0 = r * c;
  n1 = r * s;
}

}  // namespace nf

// Delayed fp8 scaling: the running amax of a tensor is folded into NF_AMAX_SLOTS partial maxima
// (slot = blockIdx.x % NF_AMAX_SLOTS), so thousands of blocks do not serialise on one address;
// the owner reduces the slots when it rolls the state (ops/fp8.py DelayedScale.roll).
#define NF_AMAX_SLOTS 64
namespace nf {
// amax >= 0: integer max on the float bits orders like the floats; a plain read first skips
// the atomic once the slot already holds a larger value
__device__ __forceinline__ void amax_slot_atomic(float* slots, float v) {
  float* dst = slots + (blockIdx.x % NF_AMAX_SLOTS);
  if (v > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(reinterpret_cast<int*>(dst), __float_as_int(v));
}
}  // namespace nf
