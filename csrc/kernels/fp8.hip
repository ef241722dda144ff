// FP8 (OCP e4m3) path for the MAF-64 configuration (gfx950):
//
//  * quant_rows: per-row absmax scaling + conversion to e4m3 (v_cvt_pk_fp8_f32), one wave per
//    row, optional zero padding of the row to a multiple of 128 bytes;
//  * gemm_fp8_nt: y = act((qx * sx) (qw * sw)^T + b) -> bf16, with the MX-scaled
//    v_mfma_scale_f32_16x16x128_f8f6f4 (K = 128 per instruction, 2x the bf16 MFMA rate; block
//    scales fixed at 2^0 - the real scales are per-row of x and per-row of W, applied as a
//    rank-1 factor in the epilogue, exact because the per-block scale is uniform along K).
//
// Tile: 128x128 output, 128-byte K step - byte-for-byte the LDS image of the bf16 kernel
// (128 rows x 128 B, 16-B chunks XOR-swizzled by row, filled by LDS-DMA, conflict-free
// fragment reads by the same argument as gemm.hip's k-major image). Each lane's A/B fragment is 32
// k-bytes (two ds_read_b128 of chunks g, g+4); the MFMA's k order is a permutation applied
// identically to both operands, so the dot products are exact whatever the hardware's
// internal k interleave (the row/column lane maps and C/D layout are the bf16 ones).
// MADE tile skipping: per N-tile K ranges (rounded out to 128; columns outside the mask's
// support hold zero weights, so the extra bytes contribute exactly 0).
#include "gemm_tile.h"

namespace nf {
namespace fp8 {

using gemm::v4f;
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr float E4M3_MAX = 448.f;

template <typename T>
__device__ __forceinline__ float ld_val(const T* p) {
  if constexpr (sizeof(T) == 2) return bf2f(*reinterpret_cast<const unsigned short*>(p));
  else return *p;
}

// q[r][c] = e4m3(x[r][c] / s[r]), s[r] = amax_r / 448 (1 for an all-zero row); c in [C, Cq) -> 0
// rows may come from `layers` equally shaped matrices `layer_stride` elements apart (all MAF
// weights of one kind in one launch): row r -> matrix r / rows_per, row r % rows_per
template <typename T>
__global__ void __launch_bounds__(256) quant_rows_kernel(const T* __restrict__ x, long ldx,
                                                         long layer_stride, int rows_per, int R,
                                                         int C, unsigned char* __restrict__ q,
                                                         long ldq, int Cq, float* __restrict__ s) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* xr = x + (long)(row / rows_per) * layer_stride + (long)(row % rows_per) * ldx;
  float amax = 0.f;
  for (int c = lane; c < C; c += 64) amax = fmaxf(amax, fabsf(ld_val(xr + c)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
  const float sc = amax > 0.f ? amax / E4M3_MAX : 1.f;
  const float inv = 1.f / sc;
  if (lane == 0) s[row] = sc;
  unsigned char* qr = q + (long)row * ldq;
  // 4 consecutive columns per lane-step -> one packed 32-bit store
  for (int c0 = lane * 4; c0 < Cq; c0 += 256) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      v[e] = c < C ? fminf(fmaxf(ld_val(xr + c) * inv, -E4M3_MAX), E4M3_MAX) : 0.f;
    }
    int w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
    *reinterpret_cast<int*>(qr + c0) = w;
  }
}

// Delayed per-tensor scaling (activations): scale = amax_prev / 448 (amax_prev = the previous
// step's amax; 1 when none yet), q = e4m3(sat(x / scale)); the current amax is folded into
// amax_cur with an integer atomicMax on the float bits (|x| >= 0 orders like its bits). A
// constant scale keeps the map x -> q elementwise, so MADE's autoregressive structure is exact.
// amax of a block's 4 waves -> one atomicMax per block into one of NF_AMAX_SLOTS partial maxima
// (a per-wave atomic on one address serialises: 8192 rows cost ~100 us)
__device__ __forceinline__ void block_amax_atomic(float amax, float* dst) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
  if (lane == 0) red[wave] = amax;
  __syncthreads();
  if (threadIdx.x == 0) amax_slot_atomic(dst, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

template <typename T>
__global__ void __launch_bounds__(256) quant_tensor_kernel(const T* __restrict__ x, long ldx, int R,
                                                           int C, unsigned char* __restrict__ q,
                                                           long ldq, int Cq,
                                                           const float* __restrict__ amax_prev,
                                                           float* __restrict__ scale_out,
                                                           float* __restrict__ amax_cur) {
  const int lane = threadIdx.x & 63;
  const float ap = *amax_prev;
  const float sc = ap > 0.f ? ap / E4M3_MAX : 1.f;
  const float inv = 1.f / sc;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = sc;
  float amax = 0.f;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < R; row += gridDim.x * 4) {
    const T* xr = x + (long)row * ldx;
    unsigned char* qr = q + (long)row * ldq;
    for (int c0 = lane * 4; c0 < Cq; c0 += 256) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + e;
        const float xv = c < C ? ld_val(xr + c) : 0.f;
        amax = fmaxf(amax, fabsf(xv));
        v[e] = fminf(fmaxf(xv * inv, -E4M3_MAX), E4M3_MAX);
      }
      int w = 0;
      w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], w, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
      *reinterpret_cast<int*>(qr + c0) = w;
    }
  }
  block_amax_atomic(amax, amax_cur);
}

struct Fp8Args {
  const unsigned char* A;  // [M][lda] e4m3 (x)
  long lda;
  const unsigned char* B;  // [N][ldb] e4m3 (W)
  long ldb;
  const float* sa;         // [M] row scales of A, or [1] (sa_per_row == 0: per-tensor)
  int sa_per_row;
  const float* sb;         // [N] row scales of B
  const bf16_t* bias;      // [N] or null
  bf16_t* C;
  long ldc;
  int M, N, K;             // K in bytes (= elements), multiple of 128
  int relu;
  const int* krange;       // [ntn][2] per 128-wide N tile, or null
  // optional e4m3 copy of the (bf16-rounded) output with a delayed per-tensor scale (the next
  // fp8 GEMM's operand): q = e4m3(sat(y / s)), s = amax_prev / 448; amax_cur = max |y|
  unsigned char* Cq;
  long ldcq;
  const float* q_amax_prev;
  float* q_scale_out;
  float* q_amax_cur;
};

constexpr int BM = 128, BN = 128, BKB = 128, NTHR = 256;
constexpr int TILE_BYTES = 128 * 128;
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int SMEM_BYTES = 2 * STAGE_BYTES;

// 128 rows x 128 bytes via LDS-DMA: chunk c of row r at c ^ (r & 7) (same image as bf16 k-major)
__device__ __forceinline__ void stage(const unsigned char* __restrict__ base, long ld, int row0,
                                      int rows, int k0, char* lds, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int r = piece * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (r & 7);
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const unsigned char* src = base + (long)gr * ld + k0 + lc * 16;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(lds + piece * 1024), 16,
                                     0, 0);
  }
}

// Lane group g = lane >> 4 takes the 16-B chunks g and g + 4 of its row (32 k-bytes). Reading
// chunk pairs (2g, 2g+1) instead costs 4 bank-conflict cycles per LDS cycle (PMC,
// profiles/r1_pmc_gemm256_group_fp8.txt); (g, g+4) is the bf16 kernel's conflict-free pattern.
__device__ __forceinline__ v8i read_frag(const char* tile, int r0, int lane) {
  const int r = r0 + (lane & 15), g = lane >> 4;
  const v4i lo = *(const LDS_AS v4i*)(tile + r * 128 + ((g ^ (r & 7)) << 4));
  const v4i hi = *(const LDS_AS v4i*)(tile + r * 128 + (((g + 4) ^ (r & 7)) << 4));
  return (v8i){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ void __launch_bounds__(NTHR, 2) gemm_fp8_nt_kernel(Fp8Args a) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (a.N + BN - 1) / BN, ntm = (a.M + BM - 1) / BM;
  const int wg = gemm::xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = wg / ntn, tn = wg % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  int kbeg = 0, kend = a.K;
  if (a.krange) {
    const int lo = a.krange[2 * tn], hi = a.krange[2 * tn + 1];
    kbeg = (lo / BKB) * BKB;
    kend = hi > kbeg ? ((hi + BKB - 1) / BKB) * BKB : kbeg;
    kend = kend < a.K ? kend : a.K;
  }
  const int nkt = (kend - kbeg) / BKB;

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  if (nkt > 0) {
    stage(a.A, a.lda, m0, a.M, kbeg, smem, wave, lane);
    stage(a.B, a.ldb, n0, a.N, kbeg, smem + TILE_BYTES, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE_BYTES;
    if (kt + 1 < nkt) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
      const int k0 = kbeg + (kt + 1) * BKB;
      stage(a.A, a.lda, m0, a.M, k0, nxt, wave, lane);
      stage(a.B, a.ldb, n0, a.N, k0, nxt + TILE_BYTES, wave, lane);
    }
    v8i fm[4], fn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fm[j] = read_frag(cur, wm * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fn[i] = read_frag(cur + TILE_BYTES, wn * 64 + i * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fn[i], fm[j], acc[i][j], 0, 0,
                                                                     0, 127, 0, 127);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // acc[i][j]: n = n0 + wn*64 + i*16 + (lane>>4)*4 + r, m = m0 + wm*64 + j*16 + (lane&15)
  const int g = lane >> 4, c = lane & 15;
  float qinv = 1.f, qamax = 0.f;
  if (a.Cq) {
    const float ap = *a.q_amax_prev;
    const float qs = ap > 0.f ? ap / E4M3_MAX : 1.f;
    qinv = 1.f / qs;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.q_scale_out = qs;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + c;
    if (m >= a.M) continue;
    const float sm = a.sa_per_row ? a.sa[m] : a.sa[0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + g * 4;
      if (n >= a.N) continue;
      const float4 sn = *reinterpret_cast<const float4*>(a.sb + n);
      v4f v = acc[i][j];
      v[0] *= sm * sn.x; v[1] *= sm * sn.y; v[2] *= sm * sn.z; v[3] *= sm * sn.w;
      if (a.bias) {
        const ushort4 bb = *reinterpret_cast<const ushort4*>(a.bias + n);
        v[0] += bf2f(bb.x); v[1] += bf2f(bb.y); v[2] += bf2f(bb.z); v[3] += bf2f(bb.w);
      }
      if (a.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      ushort4 o;
      o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
      *reinterpret_cast<ushort4*>(a.C + (long)m * a.ldc + n) = o;
      if (a.Cq) {
        const float r0 = bf2f(o.x), r1 = bf2f(o.y), r2 = bf2f(o.z), r3 = bf2f(o.w);
        qamax = fmaxf(qamax, fmaxf(fmaxf(fabsf(r0), fabsf(r1)), fmaxf(fabsf(r2), fabsf(r3))));
        int w = 0;
        w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(r0 * qinv, -E4M3_MAX), E4M3_MAX),
                                            fminf(fmaxf(r1 * qinv, -E4M3_MAX), E4M3_MAX), w, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(r2 * qinv, -E4M3_MAX), E4M3_MAX),
                                            fminf(fmaxf(r3 * qinv, -E4M3_MAX), E4M3_MAX), w, true);
        *reinterpret_cast<int*>(a.Cq + (long)m * a.ldcq + n) = w;
      }
    }
  }
  if (a.Cq) block_amax_atomic(qamax, a.q_amax_cur);
}

// Column sums of e4m3 [K][N] tensors, s * sum_k q[k][n] (the bias gradients of the e4m3
// weight-gradient launches, ops/gemm.py WgradPlan): deterministic two-pass. Pass 1: block =
// (descriptor, 256-column chunk, K slab); 16 lanes x 16 columns (one 16-B load per row and
// lane), 16 row groups, 4 rows in flight per lane; the groups folded through LDS in a fixed
// order -> part[slab][column]. Pass 2: each column's slabs summed in slab order, times the
// tensor's scale.
constexpr int CS_SLABS = 8;
struct ColsumDesc {
  const unsigned char* q;
  long ld;
  float* out;
  int K, N, sidx, blk0, col0;   // blk0: first pass-1 block, col0: first column of the part rows
};
constexpr int CS_MAX = 40;
struct ColsumArgs {
  ColsumDesc d[CS_MAX];
  int n, ncols;
  const float* scales;
  float* part;   // [CS_SLABS][ncols]
};

__device__ __forceinline__ int cs_desc(const ColsumArgs& a, int b) {
  int p = 0;
  for (int i = 1; i < a.n; ++i)
    if (b >= a.d[i].blk0) p = i;
  return p;
}

__device__ __forceinline__ void cs_add16(float (&s)[16], uint4 w) {
  const int ws[4] = {(int)w.x, (int)w.y, (int)w.z, (int)w.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(ws[e], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(ws[e], true);
    s[4 * e] += lo[0];
    s[4 * e + 1] += lo[1];
    s[4 * e + 2] += hi[0];
    s[4 * e + 3] += hi[1];
  }
}

__global__ void __launch_bounds__(256) colsum_partial_kernel(ColsumArgs a) {
  __shared__ float red[16][257];
  const int p = cs_desc(a, blockIdx.x);
  const ColsumDesc& d = a.d[p];
  const int local = blockIdx.x - d.blk0;
  const int chunk = local / CS_SLABS, slab = local % CS_SLABS;
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int n = chunk * 256 + cl * 16;
  const int rows = (d.K + CS_SLABS - 1) / CS_SLABS;
  const int k0 = slab * rows, k1 = min(d.K, k0 + rows);
  float s[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) s[e] = 0.f;
  if (n < d.N) {
    const unsigned char* col = d.q + n;
    int k = k0 + grp;
    for (; k + 48 < k1; k += 64) {   // 4 rows in flight per lane
      const uint4 w0 = *reinterpret_cast<const uint4*>(col + (long)k * d.ld);
      const uint4 w1 = *reinterpret_cast<const uint4*>(col + (long)(k + 16) * d.ld);
      const uint4 w2 = *reinterpret_cast<const uint4*>(col + (long)(k + 32) * d.ld);
      const uint4 w3 = *reinterpret_cast<const uint4*>(col + (long)(k + 48) * d.ld);
      cs_add16(s, w0);
      cs_add16(s, w1);
      cs_add16(s, w2);
      cs_add16(s, w3);
    }
    for (; k < k1; k += 16) cs_add16(s, *reinterpret_cast<const uint4*>(col + (long)k * d.ld));
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) red[grp][cl * 16 + e] = s[e];
  __syncthreads();
  const int c = threadIdx.x, nc = chunk * 256 + c;
  if (nc < d.N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][c];
    a.part[(long)slab * a.ncols + d.col0 + nc] = t;
  }
}

__global__ void __launch_bounds__(256) colsum_final_kernel(ColsumArgs a) {
  const int gc = blockIdx.x * 256 + threadIdx.x;
  if (gc >= a.ncols) return;
  int p = 0;
  for (int i = 1; i < a.n; ++i)
    if (gc >= a.d[i].col0) p = i;
  const ColsumDesc& d = a.d[p];
  float s = 0.f;
#pragma unroll
  for (int sl = 0; sl < CS_SLABS; ++sl) s += a.part[(long)sl * a.ncols + gc];
  d.out[gc - d.col0] = s * a.scales[d.sidx];
}

}  // namespace fp8
}  // namespace nf

using namespace nf::fp8;

void nf_launch_fp8_quant_rows(const void* x, int x_is_bf16, long ldx, int R, int C, void* q,
                              long ldq, int Cq, float* scale, hipStream_t stream) {
  if (R <= 0) return;
  dim3 grid((R + 3) / 4), block(256);
  if (x_is_bf16)
    hipLaunchKernelGGL(quant_rows_kernel<nf::bf16_t>, grid, block, 0, stream, (const nf::bf16_t*)x,
                       ldx, 0L, R, R, C, (unsigned char*)q, ldq, Cq, scale);
  else
    hipLaunchKernelGGL(quant_rows_kernel<float>, grid, block, 0, stream, (const float*)x, ldx, 0L, R,
                       R, C, (unsigned char*)q, ldq, Cq, scale);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_fp8_quant_rows_strided(const void* x, int x_is_bf16, long ldx, long layer_stride,
                                      int rows_per, int R, int C, void* q, long ldq, int Cq,
                                      float* scale, hipStream_t stream) {
  if (R <= 0) return;
  dim3 grid((R + 3) / 4), block(256);
  if (x_is_bf16)
    hipLaunchKernelGGL(quant_rows_kernel<nf::bf16_t>, grid, block, 0, stream, (const nf::bf16_t*)x,
                       ldx, layer_stride, rows_per, R, C, (unsigned char*)q, ldq, Cq, scale);
  else
    hipLaunchKernelGGL(quant_rows_kernel<float>, grid, block, 0, stream, (const float*)x, ldx,
                       layer_stride, rows_per, R, C, (unsigned char*)q, ldq, Cq, scale);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_fp8_quant_tensor(const void* x, int x_is_bf16, long ldx, int R, int C, void* q,
                                long ldq, int Cq, const float* amax_prev, float* scale_out,
                                float* amax_cur, hipStream_t stream) {
  if (R <= 0) return;
  const int nb = (R + 3) / 4;
  dim3 grid(nb < 256 ? nb : 256), block(256);
  if (x_is_bf16)
    hipLaunchKernelGGL(quant_tensor_kernel<nf::bf16_t>, grid, block, 0, stream, (const nf::bf16_t*)x,
                       ldx, R, C, (unsigned char*)q, ldq, Cq, amax_prev, scale_out, amax_cur);
  else
    hipLaunchKernelGGL(quant_tensor_kernel<float>, grid, block, 0, stream, (const float*)x, ldx, R,
                       C, (unsigned char*)q, ldq, Cq, amax_prev, scale_out, amax_cur);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_gemm_fp8_nt(const void* xq, long ldx, const float* sx, int sx_per_row,
                           const void* wq, long ldw, const float* sw, const void* bias, void* y,
                           long ldy, int M, int N, int K, int relu, const int* krange,
                           void* yq, long ldyq, const float* q_amax_prev, float* q_scale_out,
                           float* q_amax_cur, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  Fp8Args a{};
  a.Cq = (unsigned char*)yq; a.ldcq = ldyq;
  a.q_amax_prev = q_amax_prev; a.q_scale_out = q_scale_out; a.q_amax_cur = q_amax_cur;
  a.A = (const unsigned char*)xq; a.lda = ldx; a.sa = sx; a.sa_per_row = sx_per_row;
  a.B = (const unsigned char*)wq; a.ldb = ldw; a.sb = sw;
  a.bias = (const nf::bf16_t*)bias;
  a.C = (nf::bf16_t*)y; a.ldc = ldy;
  a.M = M; a.N = N; a.K = K; a.relu = relu; a.krange = krange;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  hipLaunchKernelGGL(gemm_fp8_nt_kernel, dim3(ntm * ntn), dim3(NTHR), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

long nf_fp8_colsum_workspace(int n, const int* N) {
  long c = 0;
  for (int i = 0; i < n; ++i) c += N[i];
  return c * nf::fp8::CS_SLABS;
}

void nf_launch_fp8_colsum(int n, const void* const* q, const long* ld, const int* K, const int* N,
                          float* const* out, const int* sidx, const float* scales, float* part,
                          hipStream_t stream) {
  using nf::fp8::ColsumArgs;
  if (n <= 0) return;
  if (n > nf::fp8::CS_MAX) {
    fprintf(stderr, "vinf: fp8_colsum: more than %d tensors\n", nf::fp8::CS_MAX);
    abort();
  }
  ColsumArgs a{};
  int blk = 0, col = 0;
  for (int i = 0; i < n; ++i) {
    if (N[i] % 16 || ld[i] % 16 || ((unsigned long)q[i] & 15)) {
      fprintf(stderr, "vinf: fp8_colsum: N %% 16, ld %% 16, 16-B aligned rows\n");
      abort();
    }
    auto& d = a.d[i];
    d.q = (const unsigned char*)q[i]; d.ld = ld[i]; d.out = out[i];
    d.K = K[i]; d.N = N[i]; d.sidx = sidx[i]; d.blk0 = blk; d.col0 = col;
    blk += ((N[i] + 255) / 256) * nf::fp8::CS_SLABS;
    col += N[i];
  }
  a.n = n; a.ncols = col; a.scales = scales; a.part = part;
  hipLaunchKernelGGL(nf::fp8::colsum_partial_kernel, dim3(blk), dim3(256), 0, stream, a);
  hipLaunchKernelGGL(nf::fp8::colsum_final_kernel, dim3((col + 255) / 256), dim3(256), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}
