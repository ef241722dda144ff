// Two-blocks-per-CU ("ping-pong") persistent bf16 GEMM for gfx950: y = x W^T (+bias, ReLU,
// bitmask), both operands k-major (NT).
//
// Why: the 256x256 kernel (gemm256.hip) holds one 512-thread block per CU (128 KiB LDS ring,
// 256 VGPRs x 2 waves per SIMD), so a tile's epilogue - bias / ReLU / bitmask / bf16 stores,
// or the coupling transforms - runs while the MFMA pipe idles: 14-50 % of a tile's time in the
// RealNVP step (docs/PERF_NOTES.md, per-tile stamps). Here each block is 4 waves (2 x 2) on a
// 256 x 128 tile with a 72 KiB ring, so TWO independent blocks share every CU, one wave of
// each per SIMD: while one block stores its epilogue, the other block's MFMAs fill the pipe.
// The cost is arithmetic intensity (256x128 tiles fetch 1.5x the operand bytes per FLOP of
// 256x256), which the L2-resident LDS-DMA rate (~68 GB/s/CU, profiles/r3/mem_issue_bench*)
// still covers at ~1.3 PF/s.
//
// Measured (profiles/r3/pingpong_ab.jsonl, same box, interleaved): SLOWER than the 256x256
// kernel on every product it hosts - forward l2 183-185 vs 147-151 us, forward l1 93-94 vs
// 87-89, fused coupling backward 171-173 vs 155-163. The epilogues are bound by the CU's
// vector-memory pipeline (~26 GB/s/CU stores, profiles/r3/mem_issue_bench*.jsonl) and the
// 256x128 operand stream needs 1.5x the bytes per FLOP through that same pipeline, so there
// is no idle resource for the other block to fill. Kept opt-in (VINF_GEMM_PP, default 0) with
// its bitwise tests as the record of the experiment.
//
// Layout: wave w -> (wr, wc) = (w >> 1, w & 1), a 128 x 64 sub-tile as acc[4][8] of
// v_mfma_f32_16x16x32_bf16 (the gemm256 accumulator layout, so the staged epilogues of
// gemm_tile.h apply unchanged). K-tiles of 32: a stage is A [256 rows][64 B] + B [128 rows][64 B]
// (24 KiB), 16-B chunk c of row r stored at c ^ ((r >> 1) & 3) (conflict-free ds_read_b128 for
// every 16-row fragment under the CDNA4 lane grouping); 3 stages in a ring, stage kt + 2 issued
// right after the barrier that opens stage kt. Per stage per wave: 6 LDS-DMA, 12 ds_read_b128,
// 32 MFMAs. Tiles: block b takes tiles b, b + G, ... (XCD-remapped ids: an XCD's tiles are
// whole row panels, the weights stay L2-resident).
#include "gemm_tile.h"

#include <cstdlib>

namespace nf {
namespace gemm {
namespace pp {

constexpr int BM = 256, BN = 128, BK = 32, NTHR = 256, NST = 3;
constexpr int A_BYTES = BM * BK * 2;          // 16 KiB
constexpr int B_BYTES = BN * BK * 2;          // 8 KiB
constexpr int ST_BYTES = A_BYTES + B_BYTES;   // 24 KiB
constexpr int SMEM = NST * ST_BYTES;          // 72 KiB: two blocks per CU

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 3; }

// rows [row0, row0 + 16 * NP) x k [k0, k0 + 32) of a k-major operand into dst, one 1-KiB piece
// (16 rows x 64 B) per DMA; wave w issues pieces w, w + 4, ...
template <int NP>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ base, long ld, int row0,
                                      int rows_total, int k0, char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NP / 4; ++i) {
    const int p = wave + 4 * i;
    const int r = p * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ swz(r);
    int gr = row0 + r;
    gr = gr < rows_total ? gr : rows_total - 1;
    const bf16_t* src = base + (long)gr * ld + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(dst + p * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ v8s frag(const char* img, int r0, int lane) {
  const int r = r0 + (lane & 15);
  const int c = lane >> 4;
  return *(const LDS_AS v8s*)(img + r * 64 + ((c ^ swz(r)) << 4));
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI>
__global__ void __launch_bounds__(NTHR, 2) gemm_pp_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  const int G = gridDim.x, b = blockIdx.x;
  const int nk = a.K / BK;

  for (int s = 0; b + s * G < ntiles; ++s) {
    const int id = xcd_remap(b + s * G, ntiles);
    const int m0 = (id / ntn) * BM, n0 = (id % ntn) * BN;
    auto issue = [&](int kt) {
      char* st = smem + (kt % NST) * ST_BYTES;
      stage<16>(a.A, a.lda, m0, a.M, kt * BK, st, wave, lane);
      stage<8>(a.B, a.ldb, n0, a.N, kt * BK, st + A_BYTES, wave, lane);
    };
    v4f acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

    issue(0);
    if (nk > 1) issue(1);
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMA of stage kt done (stage kt + 1's six may stay in flight), then every
      // wave's: stage kt is in LDS, and every wave finished reading stage kt - 1, whose slot
      // stage kt + 2 reuses
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      if (kt + 2 < nk) issue(kt + 2);
      const char* st = smem + (kt % NST) * ST_BYTES;
      // B fragments and the first four A fragments, then the last four A reads fly under the
      // first 16 MFMAs (the compiler's counted lgkmcnt: LDS reads retire in order)
      v8s fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = frag(st + A_BYTES, wc * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = frag(st, wr * 128 + j * 16, lane);
#pragma unroll
      for (int j = 4; j < 8; ++j) fa[j] = frag(st, wr * 128 + j * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 4; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    bar();   // every wave's last operand reads done: the ring is the epilogue's staging space
    epi_tile_staged<EPI, 8>(a, acc, m0 + wr * 128, n0 + wc * 64, 0, smem + wave * 16384, lane);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bar();   // staging reads done before the next tile's DMA lands in the ring
  }
}

int device_cus() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
  }();
  return n;
}

}  // namespace pp
}  // namespace gemm
}  // namespace nf

using namespace nf::gemm;

// VINF_GEMM_PP (read at load) or nf_gemm_pp_set: bit 0 routes the forward products
// (nf_launch_gemm_nt), bit 1 the fused coupling backward (nf_launch_gemm256_nn_cpl, bf16 NT
// form) through gemm_pp_kernel
static int g_pp = [] {
  const char* e = getenv("VINF_GEMM_PP");
  return e ? atoi(e) : 0;
}();
int nf_gemm_pp_enabled() { return g_pp; }
void nf_gemm_pp_set(int mask) { g_pp = mask & 3; }

// Coupling-backward form (EPI_CPL_BWD, gemm_tile.h): `a` is the GemmArgs the 256x256 launcher
// built (NT: A = dy [M][K], B = W^T [N][K]); returns 0 when the shape does not fit this kernel.
int nf_launch_gemm_pp_cpl_bwd(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  auto al16 = [](const void* p) { return ((unsigned long)p & 15) == 0; };
  if (a.K % pp::BK || a.K < pp::BK || a.lda % 8 || a.ldb % 8 || !al16(a.A) || !al16(a.B) ||
      a.krange || a.f8_sa)
    return 0;
  a.k_per_split = a.K;
  a.staged = 1;
  const int ntiles = ((a.M + pp::BM - 1) / pp::BM) * ((a.N + pp::BN - 1) / pp::BN);
  const int cap = 2 * pp::device_cus();
  const int G = ntiles < cap ? ntiles : cap;
  hipLaunchKernelGGL(pp::gemm_pp_kernel<EPI_CPL_BWD>, dim3(G), dim3(pp::NTHR), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
  return 1;
}

// y [M][N] bf16 = x [M][K] W^T (W [N][K]), + bias, ReLU (+ bitmask of y > 0 into mask_out
// [M][N/8] bytes). Requires K % 32 == 0, 16-B aligned rows (ld % 8 == 0), N % 8 == 0.
// Returns 0 (and launches nothing) when the shape does not fit, so the caller can fall back.
int nf_launch_gemm_pp_nt(const void* x, long ldx, const void* W, long ldw, const void* bias,
                         void* y, long ldy, int M, int N, int K, int relu, void* mask_out,
                         long ld_mask, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 1;
  auto al16 = [](const void* p) { return ((unsigned long)p & 15) == 0; };
  if (K % pp::BK || K < pp::BK || ldx % 8 || ldw % 8 || ldy % 8 || N % 8 || !al16(x) ||
      !al16(W) || !al16(y))
    return 0;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)x; a.lda = ldx;
  a.B = (const nf::bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const nf::bf16_t*)bias;
  a.relu = relu;
  a.M = M; a.N = N; a.K = K; a.k_per_split = K;
  a.mask_out = (unsigned char*)mask_out; a.ld_mask = ld_mask;
  a.staged = staged_ok(a, EPI_BF16);
  if (!a.staged) return 0;
  const int ntiles = ((M + pp::BM - 1) / pp::BM) * ((N + pp::BN - 1) / pp::BN);
  const int cap = 2 * pp::device_cus();
  const int G = ntiles < cap ? ntiles : cap;
  hipLaunchKernelGGL(pp::gemm_pp_kernel<EPI_BF16>, dim3(G), dim3(pp::NTHR), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
  return 1;
}
