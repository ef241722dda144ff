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
#include "gemm_tile.h"

#include <cstdlib>

namespace nf {
namespace gemm {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;       // one operand, one stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + B
constexpr int SMEM_BYTES = 2 * STAGE_BYTES;    // double buffered

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


// Per-lane LDS-DMA source pointers of one operand tile at k = k0, without the K clamp: valid
// for every full tile (k0 + BK <= K), reached by adding `step` per K-tile. The per-tile
// address arithmetic of stage_tile (row/K clamps, 64-bit multiplies: ~80 VALU per K-tile)
// then runs once per block; only a tail tile takes the clamped path.
template <bool KMAJOR>
struct TilePtrs {
  const bf16_t* p[4];
  long step;
};

template <bool KMAJOR>
__device__ __forceinline__ void tile_ptrs(TilePtrs<KMAJOR>& t, const bf16_t* __restrict__ base,
                                          long ld, int row0, int rows_total, int k0, int wave,
                                          int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    if (KMAJOR) {
      const int r = piece * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      int gr = row0 + r;
      gr = gr < rows_total ? gr : rows_total - 1;
      t.p[i] = base + (long)gr * ld + k0 + lc * 8;
    } else {
      const int kr = piece * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ mn_swz(kr);
      int gm = row0 + lc * 8;
      gm = gm < rows_total ? gm : rows_total - 8;
      t.p[i] = base + (long)(k0 + kr) * ld + gm;
    }
  }
  t.step = KMAJOR ? (long)BK : (long)BK * ld;
}

template <bool KMAJOR>
__device__ __forceinline__ void stage_ptrs(const TilePtrs<KMAJOR>& t, long off, char* lds_tile,
                                           int wave) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    __builtin_amdgcn_global_load_lds((const void*)(t.p[i] + off),
                                     (LDS_AS void*)(lds_tile + (wave * 4 + i) * 1024), 16, 0, 0);
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI>
__device__ __forceinline__ void gemm_body(const GemmArgs& a, int wg, int split, char* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int ntn = (a.N + BN - 1) / BN;
  const int tm = wg / ntn, tn = wg % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
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

  TilePtrs<A_KMAJOR> ta;
  TilePtrs<B_KMAJOR> tb;
  tile_ptrs<A_KMAJOR>(ta, a.A, a.lda, m0, a.M, kbeg, wave, lane);
  tile_ptrs<B_KMAJOR>(tb, a.B, a.ldb, n0, a.N, kbeg, wave, lane);
  long offa = 0, offb = 0;
  if (nkt > 0) {
    if (kbeg + BK <= a.K) {
      stage_ptrs<A_KMAJOR>(ta, 0, smem, wave);
      stage_ptrs<B_KMAJOR>(tb, 0, smem + TILE_BYTES, wave);
    } else {
      stage_tile<A_KMAJOR>(a.A, a.lda, m0, a.M, kbeg, a.K, smem, wave, lane);
      stage_tile<B_KMAJOR>(a.B, a.ldb, n0, a.N, kbeg, a.K, smem + TILE_BYTES, wave, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    if (kt + 1 < nkt) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
      const int k0 = kbeg + (kt + 1) * BK;
      offa += ta.step;
      offb += tb.step;
      if (k0 + BK <= a.K) {
        stage_ptrs<A_KMAJOR>(ta, offa, nxt, wave);
        stage_ptrs<B_KMAJOR>(tb, offb, nxt + TILE_BYTES, wave);
      } else {
        stage_tile<A_KMAJOR>(a.A, a.lda, m0, a.M, k0, a.K, nxt, wave, lane);
        stage_tile<B_KMAJOR>(a.B, a.ldb, n0, a.N, k0, a.K, nxt + TILE_BYTES, wave, lane);
      }
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
  if (a.staged) {  // main loop ended on a barrier: the whole 64 KiB is free
    epi_tile_staged<EPI, 4>(a, acc, m0 + wm * 64, n0 + wn * 64, split, smem + wave * 16384, lane);
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + c;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + g * 4;
      if (n >= a.N) continue;
      epi_store<EPI>(a, acc[i][j], m, n, split);
    }
  }
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI>
__global__ void __launch_bounds__(NTHR, 2) gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  gemm_body<A_KMAJOR, B_KMAJOR, EPI>(a, xcd_remap(blockIdx.x, ntm * ntn), blockIdx.y, smem);
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI>
__global__ void __launch_bounds__(NTHR, 2) gemm_group_kernel(GroupArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int id = xcd_remap(blockIdx.x, g.start[g.nprob]);
  int p = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (q < g.nprob && id >= g.start[q]) p = q;
  const GemmArgs& a = g.p[p];
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int local = id - g.start[p];
  gemm_body<A_KMAJOR, B_KMAJOR, EPI>(a, local % tiles, local / tiles, smem);
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

// Grouped split-K epilogue: problem p owns items [istart[p], istart[p+1]) laid out as in
// splitk_reduce_kernel.
struct ReduceGroup {
  const float* slabs[4];
  long slab_stride[4];
  int splits[4];
  float* out[4];
  long ld_out[4];
  int rows[4], cols[4];
  const float* dpart[4];
  float* db[4];
  const unsigned char* cmask[4];   // [rows][cols] 0/1 or null
  long istart[5];
  int nprob;
};

__global__ void __launch_bounds__(256) splitk_reduce_group_kernel(ReduceGroup r) {
  const long total = r.istart[r.nprob];
  for (long gidx = (long)blockIdx.x * blockDim.x + threadIdx.x; gidx < total;
       gidx += (long)gridDim.x * blockDim.x) {
    int p = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q)
      if (q < r.nprob && gidx >= r.istart[q]) p = q;
    const long idx = gidx - r.istart[p];
    const int cols = r.cols[p], c4 = cols >> 2, splits = r.splits[p];
    const long n_w = (long)r.rows[p] * c4;
    if (idx < n_w) {
      const int row = (int)(idx / c4), q = (int)(idx % c4);
      const float* sp = r.slabs[p] + (long)row * cols + 4 * q;
      float4 acc = *reinterpret_cast<const float4*>(sp);
      for (int k = 1; k < splits; ++k) {
        const float4 t = *reinterpret_cast<const float4*>(sp + k * r.slab_stride[p]);
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
      }
      if (r.cmask[p]) {
        const uchar4 mk = *reinterpret_cast<const uchar4*>(r.cmask[p] + (long)row * cols + 4 * q);
        acc.x = mk.x ? acc.x : 0.f; acc.y = mk.y ? acc.y : 0.f;
        acc.z = mk.z ? acc.z : 0.f; acc.w = mk.w ? acc.w : 0.f;
      }
      *reinterpret_cast<float4*>(r.out[p] + (long)row * r.ld_out[p] + 4 * q) = acc;
    } else {
      const int m = (int)(idx - n_w);
      float acc = 0.f;
      for (int k = 0; k < splits; ++k) acc += r.dpart[p][(long)k * r.rows[p] + m];
      r.db[p][m] = acc;
    }
  }
}

template <bool AK, bool BK_, int EPI>
static void launch(GemmArgs a, int splits, hipStream_t stream) {
  a.staged = staged_ok(a, EPI);
  if (a.mask_out && !a.staged) {
    fprintf(stderr, "vinf: ReLU bitmask output needs the staged epilogue (N %% 8, 16-B rows)\n");
    abort();
  }
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, splits), block(NTHR);
  hipLaunchKernelGGL((gemm_kernel<AK, BK_, EPI>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

}  // namespace gemm
}  // namespace nf

using namespace nf;
using namespace nf::gemm;

void nf_launch_gemm256_tn_group(const nf::gemm::GroupArgs& g, hipStream_t stream);

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

// Kernel choice (nf_gemm_set_mode): 0 auto, 1 the 128x128 kernel here, 2 the 256x256 8-phase
// kernel (gemm256.hip) for the M = batch products (forward / input-gradient), 3 also for the
// split-K weight gradients.
static int g_tile_mode = 0;

int nf_gemm_set_mode(int mode) {   // mode < 0: query; returns the previous mode
  const int prev = g_tile_mode;
  if (mode >= 0) g_tile_mode = mode > 3 ? 3 : mode;
  return prev;
}

static bool use_256(int M, int N, int K) {
  if (g_tile_mode == 1) return false;
  if (g_tile_mode >= 2) return true;
  // auto: enough 256x256 tiles to cover every CU once
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  return tiles >= device_cus() && K >= 256;
}

bool nf_gemm_prefer_256(int M, int N, int K) { return use_256(M, N, K); }

static bool use_256_tn() { return g_tile_mode == 3; }

// y[M][N] = act(x[M][K] W[N][K]^T + bias)   -> bf16
void nf_launch_gemm_nt(const void* x, long ldx, const void* W, long ldw, const void* bias, void* y,
                       long ldy, int M, int N, int K, int relu, hipStream_t stream,
                       void* mask_out, long ld_mask) {
  if (M <= 0 || N <= 0) return;
  if (use_256(M, N, K)) {
    nf_launch_gemm256_nt(x, ldx, W, ldw, bias, y, ldy, M, N, K, relu, stream, mask_out, ld_mask);
    return;
  }
  GemmArgs a{};
  a.A = (const bf16_t*)x; a.lda = ldx;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK; a.relu = relu;
  a.mask_out = (unsigned char*)mask_out; a.ld_mask = ld_mask;
  launch<true, true, EPI_BF16>(a, 1, stream);
}

// y[M][N] = x[M][K] W[N][K]^T -> fp32 (the module layers' bf16 precision path: bf16 operands,
// the fp32 accumulator stored as is)
void nf_launch_gemm_nt_f32out(const void* x, long ldx, const void* W, long ldw, float* y, long ldy,
                              int M, int N, int K, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const bf16_t*)x; a.lda = ldx;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK;
  launch<true, true, EPI_F32>(a, 1, stream);
}

// dx[M][N] = dy[M][K] W[K][N]  (* 1(aux>0) -> bf16)  or  (fp32 dx (+)= ...)
void nf_launch_gemm_nn(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                       long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                       int N, int K, hipStream_t stream, int aux_is_bits) {
  if (M <= 0 || N <= 0) return;
  if (use_256(M, N, K)) {
    nf_launch_gemm256_nn(dy, lddy, W, ldw, aux, ld_aux, dx, lddx, dx_is_f32, accumulate, M, N, K,
                         stream, aux_is_bits);
    return;
  }
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = dx; a.ldc = lddx;
  a.aux = (const bf16_t*)aux; a.ld_aux = ld_aux;
  a.aux_bits = aux_is_bits;
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
  if (use_256_tn()) {  // one 256x256 block per CU
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    int sp = device_cus() / tiles;
    const int nkt = (K + 63) / 64;
    if (sp > nkt / 4) sp = nkt / 4;
    return sp < 1 ? 1 : sp;
  }
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int target = 2 * device_cus();
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
  if (use_256_tn()) {  // 256x256 split-K kernel (gemm256.hip), splits from nf_gemm_tn_splits
    int sp = splits < 1 ? 1 : splits;
    if (sp == 1) {
      nf_launch_gemm256_tn_partials(dy, lddy, x, ldx, dW, lddw, 0, db, M, N, K, 1, stream);
      return;
    }
    const long slab = (long)M * N;
    float* dpart = db ? work + (long)sp * slab : nullptr;
    const int used = nf_launch_gemm256_tn_partials(dy, lddy, x, ldx, work, N, slab, dpart, M, N, K,
                                                   sp, stream);
    const long total = (long)M * (N / 4) + (db ? M : 0);
    long blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, work,
                       slab, used, dW, lddw, M, N, dpart, db);
    NF_HIP_CHECK(hipGetLastError());
    return;
  }
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
// krange256 (optional): the same K ranges for 256-column tiles; when given and the 256x256 kernel
// is the better fit (use_256), the product runs there.
void nf_launch_gemm_nt_masked(const void* x, long ldx, const void* W, long ldw, const void* bias,
                              void* y, long ldy, int M, int N, int K, int relu, const int* krange,
                              hipStream_t stream, const int* krange256) {
  if (M <= 0 || N <= 0) return;
  if (krange256 && use_256(M, N, K)) {
    nf_launch_gemm256_nt(x, ldx, W, ldw, bias, y, ldy, M, N, K, relu, stream, nullptr, 0,
                         krange256);
    return;
  }
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
                              long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                              int N, int K, const int* krange, hipStream_t stream,
                              const int* krange256, int krange256_segs, const void* Wt,
                              long ldwt) {
  if (M <= 0 || N <= 0) return;
  if (krange256 && use_256(M, N, K)) {   // with Wt = (W*M)^T [N][K]: the NT instantiation
    nf_launch_gemm256_nn(dy, lddy, Wt ? Wt : W, Wt ? ldwt : ldw, aux, ld_aux, dx, lddx, dx_is_f32,
                         accumulate, M, N, K, stream, 0, krange256, krange256_segs, Wt ? 1 : 0);
    return;
  }
  GemmArgs a{};
  a.A = (const bf16_t*)dy; a.lda = lddy;
  a.B = (const bf16_t*)W; a.ldb = ldw;
  a.C = dx; a.ldc = lddx;
  a.aux = (const bf16_t*)aux; a.ld_aux = ld_aux;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + BK - 1) / BK) * BK;
  a.krange = krange;
  if (dx_is_f32 && accumulate) launch<true, false, EPI_F32_ACC>(a, 1, stream);
  else if (dx_is_f32) launch<true, false, EPI_F32>(a, 1, stream);
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

// ---------------------------------------------------------------- grouped weight gradients
// Grouped weight gradients: the 256x256 kernel (one block per CU, S = CUs / tiles splits) beats
// the 128x128 one at long K (235 vs 246 us for the RealNVP conditioner at B = 32768,
// profiles/r1_wgrad_group_256.jsonl); it has no masked-tile skipping, so MADE groups stay on 128.
static bool group_use_256(int nprob, const NfTnProblem* pr) {
  if (g_tile_mode < 0) use_256(1, 1, 1);
  if (g_tile_mode == 3) return true;
  if (g_tile_mode != 0) return false;
  for (int p = 0; p < nprob; ++p)
    if (pr[p].skip || pr[p].K < 8192) return false;
  return true;
}

// All weight gradients of one conditioner MLP in ONE launch: a common split count S chosen so
// that S x (sum of tiles) fills one wave of resident blocks (2 per CU). Compared with one
// launch per layer this cuts the split count (3 vs 8-16 at B = 16384), so each block streams a
// 3x longer K range and the fp32 slab traffic drops by the same factor.
static int tn_group_splits(int nprob, const NfTnProblem* pr) {
  const bool t256 = group_use_256(nprob, pr);
  const int bm = t256 ? 256 : BM, bn = t256 ? 256 : BN;
  long tiles = 0;
  int cap = 1 << 30;
  for (int p = 0; p < nprob; ++p) {
    tiles += (long)((pr[p].M + bm - 1) / bm) * ((pr[p].N + bn - 1) / bn);
    const int c = ((pr[p].K + BK - 1) / BK) / 4;
    cap = c < cap ? c : cap;
  }
  const int target = (t256 ? 1 : 2) * device_cus();
  int S = (int)(target / (tiles > 0 ? tiles : 1));
  if (S > cap) S = cap;
  return S < 1 ? 1 : S;
}

long nf_gemm_tn_group_workspace(int nprob, const NfTnProblem* pr) {
  const int S = tn_group_splits(nprob, pr);
  if (S == 1) return 0;
  long w = 0;
  for (int p = 0; p < nprob; ++p) w += (long)S * pr[p].M * pr[p].N + (pr[p].db ? (long)S * pr[p].M : 0);
  return w;
}

void nf_launch_gemm_tn_group(int nprob, const NfTnProblem* pr, float* work, hipStream_t stream) {
  if (nprob < 1 || nprob > 4) return;
  const int S = tn_group_splits(nprob, pr);
  const bool t256 = group_use_256(nprob, pr);
  GroupArgs g{};
  ReduceGroup r{};
  g.nprob = nprob;
  r.nprob = nprob;
  g.start[0] = 0;
  r.istart[0] = 0;
  float* wp = work;
  for (int p = 0; p < nprob; ++p) {
    const NfTnProblem& q = pr[p];
    const int nkt = (q.K + BK - 1) / BK;
    const int kts = (nkt + S - 1) / S;
    const int used = (nkt + kts - 1) / kts;
    GemmArgs& a = g.p[p];
    a = GemmArgs{};
    a.A = (const bf16_t*)q.dy; a.lda = q.lddy;
    a.B = (const bf16_t*)q.x; a.ldb = q.ldx;
    a.M = q.M; a.N = q.N; a.K = q.K; a.k_per_split = kts * BK;
    a.skip = q.skip;
    a.cmask = q.cmask;
    r.cmask[p] = q.cmask;
    const int tb = t256 ? 256 : BM;
    const int tiles = ((q.M + tb - 1) / tb) * ((q.N + tb - 1) / tb);
    g.start[p + 1] = g.start[p] + tiles * used;
    if (S == 1 || used == 1) {
      a.C = q.dW; a.ldc = q.lddw; a.c_split_stride = 0;
      a.dbias = q.db;
      r.splits[p] = 0;  // nothing to reduce
      r.istart[p + 1] = r.istart[p];
      continue;
    }
    const long slab = (long)q.M * q.N;
    a.C = wp; a.ldc = q.N; a.c_split_stride = slab;
    a.dbias = q.db ? wp + (long)used * slab : nullptr;
    r.slabs[p] = wp; r.slab_stride[p] = slab; r.splits[p] = used;
    r.out[p] = q.dW; r.ld_out[p] = q.lddw; r.rows[p] = q.M; r.cols[p] = q.N;
    r.dpart[p] = a.dbias; r.db[p] = q.db;
    r.istart[p + 1] = r.istart[p] + (long)q.M * (q.N / 4) + (q.db ? q.M : 0);
    wp += (long)S * slab + (q.db ? (long)S * q.M : 0);
  }
  for (int p = 0; p < nprob; ++p) g.p[p].staged = staged_ok(g.p[p], EPI_F32);
  if (t256) {
    nf_launch_gemm256_tn_group(g, stream);
  } else {
    hipLaunchKernelGGL((gemm_group_kernel<false, false, EPI_F32>), dim3(g.start[nprob]), dim3(NTHR),
                       0, stream, g);
    NF_HIP_CHECK(hipGetLastError());
  }
  const long total = r.istart[nprob];
  if (total > 0) {
    long blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(splitk_reduce_group_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, r);
    NF_HIP_CHECK(hipGetLastError());
  }
}
