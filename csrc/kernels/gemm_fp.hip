// Exact fp32 / fp64 GEMM on the gfx950 f32- / f64-input matrix cores.
//
//   C[m][n] (+)= sum_k Aop(m,k) Bop(n,k) (+ bias[n]),   optionally dbias[m] = sum_k Aop(m,k)
//
// Aop(m,k) = A[m][k] (A_KM, k-major) or A[k][m]; Bop(n,k) = B[n][k] (B_KM) or B[k][n], so one
// kernel covers the three products of a dense layer in full precision:
//   forward  y = x W^T + b      A = x  (k-major), B = W  (k-major)
//   dgrad    dx = dy W          A = dy (k-major), B = W  (mn-major: B(n,k) = W[k][n])
//   wgrad    dW = dy^T x, db    A = dy (mn-major), B = x (mn-major), dbias = colsum(dy)
//
// This is the precision path of the autograd module layers (ops/linear.py, precision "fp32" /
// "fp64"): fp32 / fp64 models on the GPU keep their own arithmetic instead of being rounded to
// bf16 operands (the reference computes every layer in float64 autograd:
// /root/reference/normflows/normflows/nn_models.py:41-84). v_mfma_f32_16x16x4_f32 is exact f32
// (the same result as an fmaf chain) at 1/16 of the bf16 MFMA rate; v_mfma_f64_16x16x4_f64 is
// the f64 form. These layers are small (the module paths: <= 1024-wide MLPs), so the kernel is
// the simple LDS-tiled one: 64 x 64 block tile, 4 waves of 32 x 32 (2 x 2 MFMA tiles), 16-deep
// K-tiles double-buffered through LDS with a register prefetch of the next tile. Every load and
// store is bounds-checked: no shape constraints and no padded operand copies.
//
// Split-K (nf_gemm_fp_splits): a product with few output tiles and a long K (the module paths'
// weight gradients: one 64 x 64 tile, K = batch; 784-deep layers at M = batch <= 1024) ran
// one to sixteen blocks on the 256 CUs (~50 us each in the config-0 step). blockIdx.z = split s
// then covers K range [s kc, (s + 1) kc), writes its raw tile to the fp32 / fp64 workspace slab
// part[s] (and its row sums to dpart[s]), and gemm_fp_reduce adds the slabs IN SPLIT ORDER
// (deterministic) plus bias / old C, and the bias gradient.
//
// Operand lane maps (cdna_hip_programming.md §3): A[l & 15][k = l >> 4], B[k = l >> 4][l & 15];
// C/D col = l & 15, row = (l >> 4) * 4 + r (f32) or (l >> 4) + 4 r (f64: NOT the f32 map).
// LDS images [k][row + 16 pad]: a 32-lane read group spans two k-rows 80 elements apart, which
// the pad puts on disjoint banks for 4-B (16-bank offset) and 8-B (32-bank offset) elements.
#include "nf_common.h"

namespace nf {
namespace gemmfp {

constexpr int BM = 64, BN = 64, BKT = 16, NTHR = 256, PAD = 16;

template <typename T>
struct Mf;
template <>
struct Mf<float> {
  typedef float v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 op(float a, float b, v4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) * 4 + r; }
};
template <>
struct Mf<double> {
  typedef double v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 op(double a, double b, v4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

template <typename T>
struct FpArgs {
  const T* A;
  long lda;
  const T* B;
  long ldb;
  T* C;
  long ldc;
  const T* bias;
  T* dbias;
  int M, N, K;
  int accumulate;
  int kc;       // split-K: K per split (multiple of BKT), gridDim.z splits; else K
  T* part;      // split-K: [gridDim.z][M][N] raw tiles, or null
  T* dpart;     // split-K: [gridDim.z][M] row sums (with dbias), or null
};

// 4 elements of a 64-row x 16-k operand tile per thread. k-major source (row, k) at
// P[row * ld + k]: thread t -> row t / 4, k 4 (t % 4) + i (4 threads cover 16 contiguous k);
// mn-major source at P[k * ld + row]: thread t -> k t / 16, rows 4 (t % 16) + i (16 threads
// cover 64 contiguous rows).
template <typename T, bool KM>
__device__ __forceinline__ void load_tile(const T* __restrict__ P, long ld, int r0, int R, int k0,
                                          int K, int tid, T (&r)[4]) {
  if constexpr (KM) {
    const int row = r0 + (tid >> 2), kb = k0 + (tid & 3) * 4;
    const bool rok = row < R;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (rok && kb + i < K) ? P[(long)row * ld + kb + i] : T(0);
  } else {
    const int k = k0 + (tid >> 4), rb = r0 + (tid & 15) * 4;
    const bool kok = k < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (kok && rb + i < R) ? P[(long)k * ld + rb + i] : T(0);
  }
}

template <typename T, bool KM>
__device__ __forceinline__ void store_tile(T (*S)[BM + PAD], int tid, const T (&r)[4]) {
  if constexpr (KM) {
    const int row = tid >> 2, kb = (tid & 3) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) S[kb + i][row] = r[i];
  } else {
    const int k = tid >> 4, rb = (tid & 15) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) S[k][rb + i] = r[i];
  }
}

template <typename T, bool A_KM, bool B_KM>
__global__ void __launch_bounds__(NTHR) gemm_fp_kernel(FpArgs<T> a) {
  typedef typename Mf<T>::v4 v4;
  __shared__ T As[2][BKT][BM + PAD];
  __shared__ T Bs[2][BKT][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const bool split = a.part != nullptr;
  const bool do_db = (split ? a.dpart != nullptr : a.dbias != nullptr) && blockIdx.y == 0;
  const int kb = blockIdx.z * a.kc;                       // this split's K range [kb, ke)
  const int ke = kb + a.kc < a.K ? kb + a.kc : a.K;

  v4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v4){T(0), T(0), T(0), T(0)};
  T dsum = T(0);
  T ra[4], rb[4];
  const int nkt = ke > kb ? (ke - kb + BKT - 1) / BKT : 0;
  if (nkt > 0) {
    load_tile<T, A_KM>(a.A, a.lda, m0, a.M, kb, ke, tid, ra);
    load_tile<T, B_KM>(a.B, a.ldb, n0, a.N, kb, ke, tid, rb);
    store_tile<T, A_KM>(As[0], tid, ra);
    store_tile<T, B_KM>(Bs[0], tid, rb);
  }
  __syncthreads();
  for (int t = 0; t < nkt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nkt;
    if (more) {   // next K-tile in flight while this one is multiplied
      load_tile<T, A_KM>(a.A, a.lda, m0, a.M, kb + (t + 1) * BKT, ke, tid, ra);
      load_tile<T, B_KM>(a.B, a.ldb, n0, a.N, kb + (t + 1) * BKT, ke, tid, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BKT / 4; ++kk) {
      const int k = kk * 4 + (lane >> 4);
      T fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[cur][k][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[cur][k][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mf<T>::op(fa[i], fb[j], acc[i][j]);
    }
    if (do_db && tid < BM) {   // bias gradient: row sums of the A tile (zero beyond K)
#pragma unroll
      for (int k = 0; k < BKT; ++k) dsum += As[cur][k][tid];
    }
    if (more) {   // buffer cur ^ 1 was last read before the previous barrier
      store_tile<T, A_KM>(As[cur ^ 1], tid, ra);
      store_tile<T, B_KM>(Bs[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }

  if (split) {   // raw tile into this split's slab; gemm_fp_reduce finishes
    T* slab = a.part + (long)blockIdx.z * a.M * a.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (n >= a.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 32 + i * 16 + Mf<T>::row(lane, r);
          if (m < a.M) slab[(long)m * a.N + n] = acc[i][j][r];
        }
      }
    if (do_db && tid < BM && m0 + tid < a.M) a.dpart[(long)blockIdx.z * a.M + m0 + tid] = dsum;
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
      if (n >= a.N) continue;
      const T bn = a.bias ? a.bias[n] : T(0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + Mf<T>::row(lane, r);
        if (m >= a.M) continue;
        T* cp = a.C + (long)m * a.ldc + n;
        T v = acc[i][j][r] + bn;
        if (a.accumulate) v += *cp;
        *cp = v;
      }
    }
  if (do_db && tid < BM && m0 + tid < a.M) a.dbias[m0 + tid] = dsum;
}

// C[m][n] (+)= sum_s part[s][m][n] + bias[n] (s ascending), dbias[m] = sum_s dpart[s][m]
template <typename T>
__global__ void __launch_bounds__(256) gemm_fp_reduce(FpArgs<T> a, int S) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long MN = (long)a.M * a.N;
  if (i < MN) {
    const int m = (int)(i / a.N), n = (int)(i % a.N);
    T v = T(0);
    for (int s = 0; s < S; ++s) v += a.part[(long)s * MN + i];
    if (a.bias) v += a.bias[n];
    T* cp = a.C + (long)m * a.ldc + n;
    if (a.accumulate) v += *cp;
    *cp = v;
  }
  if (a.dbias && i < a.M) {
    T d = T(0);
    for (int s = 0; s < S; ++s) d += a.dpart[(long)s * a.M + i];
    a.dbias[i] = d;
  }
}

// split count: only products that leave most CUs idle and have a long K
inline int splits_for(int M, int N, int K) {
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles >= 128 || K < 256) return 1;
  int s = (int)((512 + tiles - 1) / tiles);     // ~512 blocks
  const int smax = K / 64;                      // >= 4 K-tiles per split
  s = s < smax ? s : smax;
  s = s < 64 ? s : 64;
  return s > 1 ? s : 1;
}

template <typename T>
void launch(const void* A, long lda, int a_km, const void* B, long ldb, int b_km,
            const void* bias, void* C, long ldc, void* dbias, int M, int N, int K, int accumulate,
            void* work, int S, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  FpArgs<T> a{(const T*)A, lda, (const T*)B, ldb, (T*)C, ldc, (const T*)bias, (T*)dbias,
              M, N, K, accumulate, K, nullptr, nullptr};
  if (S > 1 && work) {
    a.kc = ((K + S - 1) / S + BKT - 1) / BKT * BKT;
    S = (K + a.kc - 1) / a.kc;
    a.part = (T*)work;
    a.dpart = dbias ? (T*)work + (long)S * M * N : nullptr;
  } else {
    S = 1;
  }
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, S), block(NTHR);
  if (a_km && b_km) hipLaunchKernelGGL((gemm_fp_kernel<T, true, true>), grid, block, 0, stream, a);
  else if (a_km) hipLaunchKernelGGL((gemm_fp_kernel<T, true, false>), grid, block, 0, stream, a);
  else if (b_km) hipLaunchKernelGGL((gemm_fp_kernel<T, false, true>), grid, block, 0, stream, a);
  else hipLaunchKernelGGL((gemm_fp_kernel<T, false, false>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
  if (S > 1) {
    const long n = (long)M * N > M ? (long)M * N : M;
    hipLaunchKernelGGL((gemm_fp_reduce<T>), dim3((n + 255) / 256), dim3(256), 0, stream, a, S);
    NF_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace gemmfp
}  // namespace nf

int nf_gemm_fp_splits(int M, int N, int K) { return nf::gemmfp::splits_for(M, N, K); }

void nf_launch_gemm_fp(int is_f64, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, const void* bias, void* C, long ldc, void* dbias, int M, int N,
                       int K, int accumulate, hipStream_t stream, void* work, int splits) {
  if (is_f64)
    nf::gemmfp::launch<double>(A, lda, a_kmajor, B, ldb, b_kmajor, bias, C, ldc, dbias, M, N, K,
                               accumulate, work, splits, stream);
  else
    nf::gemmfp::launch<float>(A, lda, a_kmajor, B, ldb, b_kmajor, bias, C, ldc, dbias, M, N, K,
                              accumulate, work, splits, stream);
}
