// bf16 MFMA GEMM family with fused epilogues for gfx950 (CDNA4).
//
//   C[m][n] = sum_k Aop(m,k) * Bop(n,k)     (fp32 accumulate)
//   Aop(m,k) = A[m*lda + k]  (A_KMAJOR)  or  A[k*lda + m]  (M-major)
//   Bop(n,k) = B[n*ldb + k]  (B_KMAJOR)  or  B[k*ldb + n]  (N-major)
//
// One template covers the three products of a dense layer y = x W^T (W [out,in]):
//   forward  y  = x  W^T : A k-major (x),  B k-major (W)         EPI: +bias, ReLU, bf16
//   dgrad    dx = dy W   : A k-major (dy), B N-major (W)         EPI: *1(h>0) bf16 | fp32 +=
//   wgrad    dW = dy^T x : A M-major (dy), B N-major (x), K=batch EPI: fp32 split-K slabs,
//                          db = sum_k dy computed by an extra MFMA against a ones fragment.
//
// Structure (CDNA4 guide §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves (2x2), block tile 128x128, BK=64, each wave 64x64 =
//     4x4 tiles of v_mfma_f32_16x16x32_bf16;
//   * operands staged HBM->LDS with global_load_lds_dwordx4 (LDS-DMA, 1 KiB per
//     wave-instruction, no VGPR round trip), two LDS stages (64 KiB/block, 2 blocks/CU);
//   * LDS images are XOR-swizzled on the *source* address (LDS-DMA writes lane-linear):
//       k-major [128][64]  : 16-B chunk c stored at c ^ (row & 7)            -> ds_read_b128 conflict-free
//       mn-major [64][128] : 16-B chunk c stored at c ^ 2*((k&3)|((k>>1)&4)) -> ds_read_b64_tr_b16 conflict-free
//     (tools/lds_bank_model.py models the gfx950 bank groups for both);
//   * operand roles are swapped inside the MFMA (A-slot <- N side, B-slot <- M side) so each
//     lane's 4 accumulator registers are 4 consecutive n of one output row: 8-B bf16 / 16-B fp32
//     stores instead of 2-byte scatters;
//   * XCD-aware bijective block remap (guide §5.5 T1) so the 8 column tiles that share an
//     A row-panel run on one XCD's L2.
// Requirements (checked on the host): K % 32 == 0, M % 8 == 0 (M-major A), N % 8 == 0,
// 16-byte aligned rows (ld % 8 == 0).
#include "nf_common.h"

#include <cstdlib>

namespace nf {
namespace gemm {

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;       // one operand, one stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + B
constexpr int SMEM_BYTES = 2 * STAGE_BYTES;    // double buffered

enum Epi : int {
  EPI_BF16 = 0,          // C(bf16) = act(acc + bias)
  EPI_F32 = 1,           // C(fp32) = acc  (split-K slab when gridDim.y > 1)
  EPI_BF16_RELUMASK = 2, // C(bf16) = acc * 1(aux > 0)
  EPI_F32_ACC = 3,       // C(fp32) += acc
};

struct GemmArgs {
  const bf16_t* A;
  long lda;
  const bf16_t* B;
  long ldb;
  void* C;
  long ldc;
  long c_split_stride;   // elements between split-K slabs (EPI_F32)
  const bf16_t* bias;    // [N] bf16 (EPI_BF16), may be null
  const bf16_t* aux;     // [M][ld_aux] (EPI_BF16_RELUMASK)
  long ld_aux;
  float* dbias;          // [splits][M] partial sum_k Aop(m,k), may be null
  int M, N, K;
  int k_per_split;       // multiple of BK
  int relu;
  // Masked (MADE) GEMMs - structural sparsity of the weight mask:
  const int* krange;           // [ntn][2] per output N-tile K range [lo, hi) (multiples of 64), or null
  const unsigned char* skip;   // [ntm*ntn] 1 -> tile entirely masked: write zeros, no MFMA, or null
};

__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

// Stage one 128 x 64 operand tile into LDS (wave-uniform dst per 1 KiB piece).
template <bool KMAJOR>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ base, long ld, int row0,
                                           int rows_total, int k0, int K, char* lds_tile,
                                           int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;  // 0..15, 1 KiB each
    const bf16_t* src;
    if (KMAJOR) {
      // image [128 rows][64 k]: 8 rows per piece, lane -> (row, physical chunk)
      const int r = piece * 8 + (lane >> 3);
      const int pc = lane & 7;
      const int lc = pc ^ (r & 7);
      int gr = row0 + r;
      gr = gr < rows_total ? gr : rows_total - 1;
      int gk = k0 + lc * 8;
      gk = gk < K ? gk : K - 8;
      src = base + (long)gr * ld + gk;
    } else {
      // image [64 k][128 mn]: 4 k-rows per piece
      const int kr = piece * 4 + (lane >> 4);
      const int pc = lane & 15;
      const int lc = pc ^ mn_swz(kr);
      int gk = k0 + kr;
      gk = gk < K ? gk : K - 1;
      int gm = row0 + lc * 8;
      gm = gm < rows_total ? gm : rows_total - 8;
      src = base + (long)gk * ld + gm;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(lds_tile + piece * 1024), 16,
                                     0, 0);
  }
}

// 8 consecutive k (k-step ks in {0,1}) for tile row r0 + (lane & 15).
template <bool KMAJOR>
__device__ __forceinline__ v8s read_frag(const char* lds_tile, int r0, int ks, int lane) {
  if (KMAJOR) {
    const int r = r0 + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *(const LDS_AS v8s*)(lds_tile + r * 128 + ((c ^ (r & 7)) << 4));
  } else {
    const int i = lane & 15, g = lane >> 4;
    const int col = r0 + 4 * (i & 3);
    const int chunk = col >> 3, sub = (col >> 2) & 1;
    v8s out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + (i >> 2);
      const LDS_AS v4s* p =
          (const LDS_AS v4s*)(lds_tile + k * 256 + ((chunk ^ mn_swz(k)) << 4) + sub * 8);
      const v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)p);
      if (h == 0) {
        out[0] = t[0]; out[1] = t[1]; out[2] = t[2]; out[3] = t[3];
      } else {
        out[4] = t[0]; out[5] = t[1]; out[6] = t[2]; out[7] = t[3];
      }
    }
    return out;
  }
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI>
__global__ void __launch_bounds__(NTHR, 2) gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int ntn = (a.N + BN - 1) / BN;
  const int ntm = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = wg / ntn, tn = wg % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.y;
  int kbeg = split * a.k_per_split;
  int kend = kbeg + a.k_per_split;
  kend = kend < a.K ? kend : a.K;
  if (a.krange) {  // skip K-tiles whose weight block is entirely masked
    const int lo = a.krange[2 * tn], hi = a.krange[2 * tn + 1];
    kbeg = kbeg > lo ? kbeg : lo;
    kend = kend < hi ? kend : hi;
    if (kend < kbeg) kend = kbeg;
  }
  int nkt = (kend - kbeg + BK - 1) / BK;
  if (a.skip && a.skip[tm * ntn + tn] && !(a.dbias != nullptr && tn == 0)) nkt = 0;

  const bool do_db = (a.dbias != nullptr) && tn == 0 && wn == 0;
  v4f acc[4][4];
  v4f accb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    accb[i] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  }
  v8s ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3F80;

  if (nkt > 0) {
    stage_tile<A_KMAJOR>(a.A, a.lda, m0, a.M, kbeg, a.K, smem, wave, lane);
    stage_tile<B_KMAJOR>(a.B, a.ldb, n0, a.N, kbeg, a.K, smem + TILE_BYTES, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    if (kt + 1 < nkt) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
      const int k0 = kbeg + (kt + 1) * BK;
      stage_tile<A_KMAJOR>(a.A, a.lda, m0, a.M, k0, a.K, nxt, wave, lane);
      stage_tile<B_KMAJOR>(a.B, a.ldb, n0, a.N, k0, a.K, nxt + TILE_BYTES, wave, lane);
    }
    const int kvalid = kend - (kbeg + kt * BK);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks * 32 < kvalid) {
        v8s fm[4], fn[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) fm[j] = read_frag<A_KMAJOR>(cur, wm * 64 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fn[i] = read_frag<B_KMAJOR>(cur + TILE_BYTES, wn * 64 + i * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fn[i], fm[j], acc[i][j], 0, 0, 0);
        if (do_db) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fm[j], accb[j], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // acc[i][j]: row n = n0 + wn*64 + i*16 + (lane>>4)*4 + r, col m = m0 + wm*64 + j*16 + (lane&15)
  const int g = lane >> 4, c = lane & 15;
  if (do_db && g == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wm * 64 + j * 16 + c;
      if (m < a.M) a.dbias[(long)split * a.M + m] = accb[j][0];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + c;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + g * 4;
      if (n >= a.N) continue;
      v4f v = acc[i][j];
      if (EPI == EPI_BF16) {
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
        *reinterpret_cast<ushort4*>((bf16_t*)a.C + (long)m * a.ldc + n) = o;
      } else if (EPI == EPI_BF16_RELUMASK) {
        const ushort4 h = *reinterpret_cast<const ushort4*>(a.aux + (long)m * a.ld_aux + n);
        // bf16 > 0  <=>  sign bit clear and not +0
        v[0] = (h.x != 0 && !(h.x & 0x8000)) ? v[0] : 0.f;
        v[1] = (h.y != 0 && !(h.y & 0x8000)) ? v[1] : 0.f;
        v[2] = (h.z != 0 && !(h.z & 0x8000)) ? v[2] : 0.f;
        v[3] = (h.w != 0 && !(h.w & 0x8000)) ? v[3] : 0.f;
        ushort4 o;
        o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
        *reinterpret_cast<ushort4*>((bf16_t*)a.C + (long)m * a.ldc + n) = o;
      } else if (EPI == EPI_F32) {
        float* cp = (float*)a.C + (long)split * a.c_split_stride + (long)m * a.ldc + n;
        *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      } else {  // EPI_F32_ACC
        float* cp = (float*)a.C + (long)m * a.ldc + n;
        float4 o = *reinterpret_cast<float4*>(cp);
        o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
        *reinterpret_cast<float4*>(cp) = o;
      }
    }
  }
}

// One launch for the split-K epilogue of a weight-gradient GEMM:
//   items [0, rows*cols/4)          : dW[r][c..c+3] = sum_s slab[s][r][c..c+3]
//   items [rows*cols/4, + rows)     : db[r]         = sum_s part[s][r]
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slabs,
                                                             long slab_stride, int splits,
                                                             float* __restrict__ out, long ld_out,
                                                             int rows, int cols,
                                                             const float* __restrict__ dpart,
                                                             float* __restrict__ db) {
  const int c4 = cols >> 2;
  const long n_w = (long)rows * c4;
  const long total = n_w + (db ? rows : 0);
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    if (idx < n_w) {
      const int r = (int)(idx / c4), q = (int)(idx % c4);
      const float* sp = slabs + (long)r * cols + 4 * q;
      float4 acc = *reinterpret_cast<const float4*>(sp);
      for (int k = 1; k < splits; ++k) {
        const float4 t = *reinterpret_cast<const float4*>(sp + k * slab_stride);
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
      }
      *reinterpret_cast<float4*>(out + (long)r * ld_out + 4 * q) = acc;
    } else {
      const int m = (int)(idx - n_w);
      float acc = 0.f;
      for (int k = 0; k < splits; ++k) acc += dpart[(long)k * rows + m];
      db[m] = acc;
    }
  }
}

template <bool AK, bool BK_, int EPI>
static void launch(const GemmArgs& a, int splits, hipStream_t stream) {
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, splits), block(NTHR);
  hipLaunchKernelGGL((gemm_kernel<AK, BK_, EPI>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

}  // namespace gemm
}  // namespace nf

using namespace nf;
using namespace nf::gemm;

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

// y[M][N] = act(x[M][K] W[N][K]^T + bias)   -> bf16
void nf_launch_gemm_nt(const void* x, long ldx, const void* W, long ldw, const void* bias, void* y,
                       long ldy, int M, int N, int K, int relu, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const bf16_t*)x; a.lda = ldx;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK; a.relu = relu;
  launch<true, true, EPI_BF16>(a, 1, stream);
}

// dx[M][N] = dy[M][K] W[K][N]  (* 1(aux>0) -> bf16)  or  (fp32 dx (+)= ...)
void nf_launch_gemm_nn(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                       long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                       int N, int K, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = dx; a.ldc = lddx;
  a.aux = (const bf16_t*)aux; a.ld_aux = ld_aux;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK;
  if (dx_is_f32) {
    if (accumulate) launch<true, false, EPI_F32_ACC>(a, 1, stream);
    else launch<true, false, EPI_F32>(a, 1, stream);
  } else if (aux) {
    launch<true, false, EPI_BF16_RELUMASK>(a, 1, stream);
  } else {
    launch<true, false, EPI_BF16>(a, 1, stream);
  }
}

long nf_gemm_tn_workspace(int M, int N, int splits) {
  return splits > 1 ? (long)splits * M * N + (long)splits * M : 0;
}

// Split-K count for the weight-gradient GEMM: fill exactly one wave of resident blocks
// (2 per CU); a partial second wave costs more than it buys (profiles/r1_wgrad_splitk_sweep.txt).
int nf_gemm_tn_splits(int M, int N, int K) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int target = 2 * device_cus();
  if (const char* e = getenv("VINF_TN_TARGET_BLOCKS")) target = atoi(e);
  int splits = target / tiles;
  const int nkt = (K + BK - 1) / BK;
  if (splits > nkt / 4) splits = nkt / 4;
  return splits < 1 ? 1 : splits;
}

// dW[M][N] = dy[K][M]^T x[K][N] (fp32), db[M] = sum_k dy[k][M]; split-K slabs in `work`
// (nf_gemm_tn_workspace floats) reduced into dW/db by one extra launch.
void nf_launch_gemm_tn(const void* dy, long lddy, const void* x, long ldx, float* dW, long lddw,
                       float* db, int M, int N, int K, int splits, float* work,
                       hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  const int nkt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt;
  const int kts = (nkt + splits - 1) / splits;
  const int used = (nkt + kts - 1) / kts;
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)x; a.ldb = ldx;
  a.M = M; a.N = N; a.K = K; a.k_per_split = kts * BK;
  if (used == 1) {
    a.C = dW; a.ldc = lddw; a.c_split_stride = 0;
    a.dbias = db;
    launch<false, false, EPI_F32>(a, 1, stream);
    return;
  }
  const long slab = (long)M * N;
  a.C = work; a.ldc = N; a.c_split_stride = slab;
  a.dbias = db ? work + (long)used * slab : nullptr;
  launch<false, false, EPI_F32>(a, used, stream);
  const long total = (long)M * (N / 4) + (db ? M : 0);
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, work,
                     slab, used, dW, lddw, M, N, a.dbias, db);
  NF_HIP_CHECK(hipGetLastError());
}

// Masked variants (MADE): same kernels, with per-N-tile K ranges / per-tile skip flags.
void nf_launch_gemm_nt_masked(const void* x, long ldx, const void* W, long ldw, const void* bias,
                              void* y, long ldy, int M, int N, int K, int relu, const int* krange,
                              hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const bf16_t*)x; a.lda = ldx;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK; a.relu = relu;
  a.krange = krange;
  launch<true, true, EPI_BF16>(a, 1, stream);
}

void nf_launch_gemm_nn_masked(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                              long ld_aux, void* dx, long lddx, int dx_is_f32, int M, int N, int K,
                              const int* krange, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = dx; a.ldc = lddx;
  a.aux = (const bf16_t*)aux; a.ld_aux = ld_aux;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK;
  a.krange = krange;
  if (dx_is_f32) launch<true, false, EPI_F32>(a, 1, stream);
  else if (aux) launch<true, false, EPI_BF16_RELUMASK>(a, 1, stream);
  else launch<true, false, EPI_BF16>(a, 1, stream);
}

void nf_launch_gemm_tn_masked(const void* dy, long lddy, const void* x, long ldx, float* dW,
                              long lddw, float* db, int M, int N, int K, int splits, float* work,
                              const unsigned char* skip, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  const int nkt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt;
  const int kts = (nkt + splits - 1) / splits;
  const int used = (nkt + kts - 1) / kts;
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)x; a.ldb = ldx;
  a.M = M; a.N = N; a.K = K; a.k_per_split = kts * BK;
  a.skip = skip;
  if (used == 1) {
    a.C = dW; a.ldc = lddw; a.c_split_stride = 0;
    a.dbias = db;
    launch<false, false, EPI_F32>(a, 1, stream);
    return;
  }
  const long slab = (long)M * N;
  a.C = work; a.ldc = N; a.c_split_stride = slab;
  a.dbias = db ? work + (long)used * slab : nullptr;
  launch<false, false, EPI_F32>(a, used, stream);
  const long total = (long)M * (N / 4) + (db ? M : 0);
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, work,
                     slab, used, dW, lddw, M, N, a.dbias, db);
  NF_HIP_CHECK(hipGetLastError());
}
