// Fused K-layer planar flow stack, forward + backward (gfx950).
//
//   f_k(z) = z + u_hat_k h(a_k),  a_k = w_k.z + b_k,  h = tanh,
//   ldj    = sum_k log|1 + h'(a_k) w_k.u_hat_k|                       (paper form)
//   broadcast variant (reference flows.py:32): z_j += (sum_d u_hat_d) h  for every j,
//   ldj    = sum_k log|1 + h'(a_k) (sum u_hat)(sum w)|
//
// Parameters are shared [K][D] (non-amortized VI) or per-sample [K][N][D] (amortized,
// produced by an encoder). u_hat is precomputed (cheap elementwise, differentiated by
// torch); the kernel owns the K-loop so the state and log-det never leave registers.
//
// Row mapping: D <= 16 -> one lane per row (the 2-D energy-potential regime, N up to
// millions of MC samples); larger D (<= 1024) -> one wave64 per row, lane j holds
// elements j, j+64, ... and dot products are 64-wide shuffle reductions.
// Backward re-reads each layer's saved input, recomputes a/h/psi and emits per-row
// parameter gradients (the caller sums them over rows for shared parameters).
#include "nf_common.h"

namespace nf {

// log|psi| is evaluated as log(|psi| + eps) (the reference's guard, optimization.py:83,
// get_data.py:107): psi = 1 + h' w.u_hat can reach 0 exactly, e.g. in the broadcast variant.
// Its derivative sign(psi) / (|psi| + eps) stays finite there.
constexpr float kPsiEps = 1e-7f;
__device__ __forceinline__ float dlog_guard(float psi) {
  return copysignf(1.f / (fabsf(psi) + kPsiEps), psi);
}

template <bool WROW>
__device__ __forceinline__ float rsum(float v) {
  if (WROW) return wave_sum(v);
  return v;
}

struct PlanarArgs {
  const float* z;
  const float* W;
  const float* U;
  const float* Bv;
  float* zK;
  float* ldj;
  float* saved;   // [K][N][D]
  // backward
  const float* gz;
  const float* gl;
  float* dz;
  float* dW;      // [K][N][D]
  float* dU;      // [K][N][D]
  float* dB;      // [K][N]
  int N, D, K;
  int per_sample;
  int broadcast;
};

template <bool WROW, int PER>
__device__ __forceinline__ bool row_of(const PlanarArgs& a, long& row, int& lane) {
  lane = threadIdx.x & 63;
  if (WROW) {
    row = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  } else {
    row = (long)blockIdx.x * blockDim.x + threadIdx.x;
  }
  return row < a.N;
}

template <bool WROW, int PER>
__device__ __forceinline__ int elem(int i, int lane) {
  return WROW ? lane + 64 * i : i;
}

template <bool WROW, int PER>
__global__ void __launch_bounds__(256) planar_fwd_kernel(PlanarArgs a) {
  long row;
  int lane;
  if (!row_of<WROW, PER>(a, row, lane)) return;
  const int D = a.D;
  float z[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = elem<WROW, PER>(i, lane);
    z[i] = j < D ? a.z[row * D + j] : 0.f;
  }
  float ldj = 0.f;
  for (int k = 0; k < a.K; ++k) {
    const long pbase = a.per_sample ? ((long)k * a.N + row) * D : (long)k * D;
    const float b = a.per_sample ? a.Bv[(long)k * a.N + row] : a.Bv[k];
    float w[PER], u[PER];
    float dot = 0.f, su = 0.f, sw = 0.f, eta = 0.f;
    float* sv = a.saved ? a.saved + ((long)k * a.N + row) * D : nullptr;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = elem<WROW, PER>(i, lane);
      if (j < D) {
        w[i] = a.W[pbase + j];
        u[i] = a.U[pbase + j];
        if (sv) sv[j] = z[i];
      } else {
        w[i] = 0.f;
        u[i] = 0.f;
      }
      dot += z[i] * w[i];
      su += u[i];
      sw += w[i];
      eta += w[i] * u[i];
    }
    dot = rsum<WROW>(dot);
    const float h = tanhf(dot + b);
    const float hp = 1.f - h * h;
    float psi;
    if (a.broadcast) {
      su = rsum<WROW>(su);
      sw = rsum<WROW>(sw);
      psi = 1.f + hp * su * sw;
#pragma unroll
      for (int i = 0; i < PER; ++i) z[i] += su * h;
    } else {
      eta = rsum<WROW>(eta);
      psi = 1.f + hp * eta;
#pragma unroll
      for (int i = 0; i < PER; ++i) z[i] += u[i] * h;
    }
    ldj += __logf(fabsf(psi) + kPsiEps);
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = elem<WROW, PER>(i, lane);
    if (j < D) a.zK[row * D + j] = z[i];
  }
  if (!WROW || lane == 0) a.ldj[row] = ldj;
}

template <bool WROW, int PER>
__global__ void __launch_bounds__(256) planar_bwd_kernel(PlanarArgs a) {
  long row;
  int lane;
  if (!row_of<WROW, PER>(a, row, lane)) return;
  const int D = a.D;
  float g[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = elem<WROW, PER>(i, lane);
    g[i] = j < D ? a.gz[row * D + j] : 0.f;
  }
  const float c = a.gl[row];
  for (int k = a.K - 1; k >= 0; --k) {
    const long pbase = a.per_sample ? ((long)k * a.N + row) * D : (long)k * D;
    const float b = a.per_sample ? a.Bv[(long)k * a.N + row] : a.Bv[k];
    const float* sv = a.saved + ((long)k * a.N + row) * D;
    float w[PER], u[PER], z[PER];
    float dot = 0.f, su = 0.f, sw = 0.f, eta = 0.f, gsum = 0.f, gu = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = elem<WROW, PER>(i, lane);
      if (j < D) {
        w[i] = a.W[pbase + j];
        u[i] = a.U[pbase + j];
        z[i] = sv[j];
      } else {
        w[i] = u[i] = z[i] = 0.f;
      }
      dot += z[i] * w[i];
      su += u[i];
      sw += w[i];
      eta += w[i] * u[i];
      gsum += g[i];
      gu += g[i] * u[i];
    }
    dot = rsum<WROW>(dot);
    const float h = tanhf(dot + b);
    const float hp = 1.f - h * h;
    const float hpp = -2.f * h * hp;
    float da;
    float* dWr = a.dW + ((long)k * a.N + row) * D;
    float* dUr = a.dU + ((long)k * a.N + row) * D;
    if (a.broadcast) {
      su = rsum<WROW>(su);
      sw = rsum<WROW>(sw);
      gsum = rsum<WROW>(gsum);
      const float psi = 1.f + hp * su * sw;
      const float ipsi = dlog_guard(psi);
      da = gsum * su * hp + c * hpp * su * sw * ipsi;
      const float du = gsum * h + c * hp * sw * ipsi;
      const float dwc = c * hp * su * ipsi;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = elem<WROW, PER>(i, lane);
        if (j < D) {
          dUr[j] = du;
          dWr[j] = da * z[i] + dwc;
        }
      }
    } else {
      eta = rsum<WROW>(eta);
      gu = rsum<WROW>(gu);
      const float psi = 1.f + hp * eta;
      const float ipsi = dlog_guard(psi);
      const float r = c * hp * ipsi;
      da = gu * hp + c * hpp * eta * ipsi;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = elem<WROW, PER>(i, lane);
        if (j < D) {
          dUr[j] = g[i] * h + r * w[i];
          dWr[j] = da * z[i] + r * u[i];
        }
      }
    }
    if (!WROW || lane == 0) a.dB[(long)k * a.N + row] = da;
#pragma unroll
    for (int i = 0; i < PER; ++i) g[i] += da * w[i];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = elem<WROW, PER>(i, lane);
    if (j < D) a.dz[row * D + j] = g[i];
  }
}

// Shared (non-amortized) parameters, D <= 16, K * PER <= 256: the backward recomputes every
// layer's input from z0 into LDS (no [K][N][D] saved-state buffer in HBM) and reduces the
// parameter gradients inside the kernel: one wave per block walks rows (grid-stride), each
// layer's dU / dW / db contributions are wave-summed and accumulated in LDS, and every block
// writes ONE partial [K][2 PER + 1] row; a fixed-order finalize sums the partials (bitwise
// reproducible). HBM traffic per row: z0, gz, dz, one ldj-gradient scalar; O(K D) parameter
// gradients instead of the O(K N D) per-row buffers of the generic path.
template <int PER>
__global__ void __launch_bounds__(64) planar_bwd_shared_kernel(PlanarArgs a, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x;
  const int K = a.K, D = a.D;
  constexpr int NV = 2 * PER + 1;
  float* st = lds;                       // [K][PER][64]
  float* acc = lds + K * PER * 64;       // [K][NV]
  for (int i = lane; i < K * NV; i += 64) acc[i] = 0.f;
  __syncthreads();
  for (long row0 = (long)blockIdx.x * 64; row0 < a.N; row0 += (long)gridDim.x * 64) {
    const long row = row0 + lane;
    const bool valid = row < a.N;
    float z[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) z[i] = (valid && i < D) ? a.z[row * D + i] : 0.f;
    for (int k = 0; k < K; ++k) {        // forward recompute, inputs of every layer -> LDS
      float dot = 0.f, su = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        st[(k * PER + i) * 64 + lane] = z[i];
        const float w = i < D ? a.W[k * D + i] : 0.f;
        dot += z[i] * w;
        su += i < D ? a.U[k * D + i] : 0.f;
      }
      const float h = tanhf(dot + a.Bv[k]);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const float u = i < D ? a.U[k * D + i] : 0.f;
        z[i] += (a.broadcast ? su : u) * h;
      }
    }
    float g[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) g[i] = (valid && i < D) ? a.gz[row * D + i] : 0.f;
    const float c = valid ? a.gl[row] : 0.f;
    for (int k = K - 1; k >= 0; --k) {
      float w[PER], u[PER];
      float dot = 0.f, su = 0.f, sw = 0.f, eta = 0.f, gsum = 0.f, gu = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        w[i] = i < D ? a.W[k * D + i] : 0.f;
        u[i] = i < D ? a.U[k * D + i] : 0.f;
        z[i] = st[(k * PER + i) * 64 + lane];
        dot += z[i] * w[i];
        su += u[i];
        sw += w[i];
        eta += w[i] * u[i];
        gsum += g[i];
        gu += g[i] * u[i];
      }
      const float h = tanhf(dot + a.Bv[k]);
      const float hp = 1.f - h * h;
      const float hpp = -2.f * h * hp;
      float da, cu[PER], cw[PER];
      if (a.broadcast) {
        const float ipsi = dlog_guard(1.f + hp * su * sw);
        da = gsum * su * hp + c * hpp * su * sw * ipsi;
        const float du = gsum * h + c * hp * sw * ipsi;
        const float dwc = c * hp * su * ipsi;
#pragma unroll
        for (int i = 0; i < PER; ++i) { cu[i] = du; cw[i] = da * z[i] + dwc; }
      } else {
        const float ipsi = dlog_guard(1.f + hp * eta);
        const float r = c * hp * ipsi;
        da = gu * hp + c * hpp * eta * ipsi;
#pragma unroll
        for (int i = 0; i < PER; ++i) { cu[i] = g[i] * h + r * w[i]; cw[i] = da * z[i] + r * u[i]; }
      }
      if (!valid) {
        da = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) cu[i] = cw[i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        if (i < D) {
          const float su_ = wave_sum(cu[i]);
          const float sw_ = wave_sum(cw[i]);
          if (lane == 0) {
            acc[k * NV + i] += su_;
            acc[k * NV + PER + i] += sw_;
          }
        }
      }
      const float sb = wave_sum(da);
      if (lane == 0) acc[k * NV + 2 * PER] += sb;
#pragma unroll
      for (int i = 0; i < PER; ++i) g[i] += da * w[i];
    }
    if (valid) {
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i < D) a.dz[row * D + i] = g[i];
    }
  }
  __syncthreads();
  for (int i = lane; i < K * NV; i += 64) part[(long)blockIdx.x * K * NV + i] = acc[i];
}

// dU[k][j], dW[k][j], dB[k] = sum over blocks of the partials, in block order (one block per
// output value, strided partial sums + a fixed-shape tree)
__global__ void __launch_bounds__(256) planar_shared_finalize_kernel(
    const float* __restrict__ part, int nblk, int K, int D, int PER, float* dW, float* dU,
    float* dB) {
  __shared__ float scratch[16];
  const int NV = 2 * PER + 1;
  const int kv = blockIdx.x, k = kv / NV, v = kv % NV;
  float acc = 0.f;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) acc += part[(long)b * K * NV + kv];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    if (v < PER) {
      if (v < D) dU[k * D + v] = acc;
    } else if (v < 2 * PER) {
      if (v - PER < D) dW[k * D + (v - PER)] = acc;
    } else {
      dB[k] = acc;
    }
  }
}

template <int PER>
static void launch_planar_shared(const PlanarArgs& a, float* part, int nblk, hipStream_t stream) {
  const size_t lds = ((size_t)a.K * PER * 64 + (size_t)a.K * (2 * PER + 1)) * sizeof(float);
  hipLaunchKernelGGL((planar_bwd_shared_kernel<PER>), dim3(nblk), dim3(64), lds, stream, a, part);
  NF_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(planar_shared_finalize_kernel, dim3(a.K * (2 * PER + 1)), dim3(256), 0, stream,
                     part, nblk, a.K, a.D, PER, a.dW, a.dU, a.dB);
  NF_HIP_CHECK(hipGetLastError());
}

template <bool WROW, int PER>
static void launch_planar(const PlanarArgs& a, bool bwd, hipStream_t stream) {
  const long threads = WROW ? (long)a.N * 64 : (long)a.N;
  dim3 grid((unsigned)((threads + 255) / 256)), block(256);
  if (bwd)
    hipLaunchKernelGGL((planar_bwd_kernel<WROW, PER>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((planar_fwd_kernel<WROW, PER>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

static void dispatch_planar(const PlanarArgs& a, bool bwd, hipStream_t stream) {
  const int D = a.D;
  if (D <= 2) return launch_planar<false, 2>(a, bwd, stream);
  if (D <= 4) return launch_planar<false, 4>(a, bwd, stream);
  if (D <= 8) return launch_planar<false, 8>(a, bwd, stream);
  if (D <= 16) return launch_planar<false, 16>(a, bwd, stream);
  if (D <= 64) return launch_planar<true, 1>(a, bwd, stream);
  if (D <= 128) return launch_planar<true, 2>(a, bwd, stream);
  if (D <= 256) return launch_planar<true, 4>(a, bwd, stream);
  if (D <= 512) return launch_planar<true, 8>(a, bwd, stream);
  return launch_planar<true, 16>(a, bwd, stream);
}

}  // namespace nf

using namespace nf;

void nf_launch_planar_fwd(const float* z, const float* W, const float* U, const float* B, float* zK,
                          float* ldj, float* saved, int N, int D, int K, int per_sample,
                          int broadcast, hipStream_t stream) {
  if (N <= 0) return;
  PlanarArgs a{};
  a.z = z; a.W = W; a.U = U; a.Bv = B; a.zK = zK; a.ldj = ldj; a.saved = saved;
  a.N = N; a.D = D; a.K = K; a.per_sample = per_sample; a.broadcast = broadcast;
  dispatch_planar(a, false, stream);
}

void nf_launch_planar_bwd(const float* saved, const float* W, const float* U, const float* B,
                          const float* gz, const float* gl, float* dz, float* dW, float* dU,
                          float* dB, int N, int D, int K, int per_sample, int broadcast,
                          hipStream_t stream) {
  if (N <= 0) return;
  PlanarArgs a{};
  a.saved = (float*)saved; a.W = W; a.U = U; a.Bv = B; a.gz = gz; a.gl = gl; a.dz = dz;
  a.dW = dW; a.dU = dU; a.dB = dB;
  a.N = N; a.D = D; a.K = K; a.per_sample = per_sample; a.broadcast = broadcast;
  dispatch_planar(a, true, stream);
}

int nf_planar_shared_per(int D) { return D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 16 ? 16 : 0; }

int nf_planar_shared_blocks(int N) {
  const long b = ((long)N + 63) / 64;
  return (int)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

void nf_launch_planar_bwd_shared(const float* z0, const float* W, const float* U, const float* B,
                                 const float* gz, const float* gl, float* dz, float* dW, float* dU,
                                 float* dB, float* part, int nblk, int N, int D, int K,
                                 int broadcast, hipStream_t stream) {
  if (N <= 0) return;
  PlanarArgs a{};
  a.z = z0; a.W = W; a.U = U; a.Bv = B; a.gz = gz; a.gl = gl; a.dz = dz;
  a.dW = dW; a.dU = dU; a.dB = dB;
  a.N = N; a.D = D; a.K = K; a.per_sample = 0; a.broadcast = broadcast;
  switch (nf_planar_shared_per(D)) {
    case 2: return launch_planar_shared<2>(a, part, nblk, stream);
    case 4: return launch_planar_shared<4>(a, part, nblk, stream);
    case 8: return launch_planar_shared<8>(a, part, nblk, stream);
    case 16: return launch_planar_shared<16>(a, part, nblk, stream);
    default: break;
  }
}
