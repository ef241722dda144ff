// Batch-side NT products on 4 fat waves: C[m][n] = sum_k A[m][k] B[n][k], both operands k-major
// (forward y = act(x W^T + b) with the ReLU bitmask, input gradient dx = (dy Wt^T) * 1(bits)),
// one 256x256 output tile per block, bf16 output through the staged epilogue of gemm_tile.h.
//
// Opt-in A/B of the 4-wave design on the NT products (VINF_GEMM_NT4W=1; gemm256.hip's launch()
// keeps the 8-wave persistent kernel otherwise). The 4-wave TN kernel (gemm_tn4w.hip) beat the
// 8-wave schedule by 5 % with cache-resident operands and 25 % on real ones; an L2-resident
// activation did not speed the NT products up (profiles/r4/nt_probe_a_resident.jsonl), so their
// schedule was the candidate. Measured slower at the headline shapes (docs/PERF_NOTES.md
// "A 4-wave NT kernel", profiles/r4/nt4w_probe.jsonl): off by default.
//
// Geometry: 256 threads = 4 waves, wave w = (wr, wc) = (w >> 1, w & 1) owns tile rows
// [128 wr, +128) x cols [128 wc, +128) (256 fp32 accumulators per lane in AGPRs). BK = 64.
// LDS: 2 stages x 4 half-images x 16 KiB = 128 KiB; half-image h of a stage = k-major
// [128 rows][64 k] (gemm_tile.h layout: 16-B chunk c of row r at c ^ (r & 7)): h = 0 / 1: A rows
// m0 + [0, 128) / [128, 256), h = 2 / 3: B rows n0 + [0, 128) / [128, 256). Wave w stages
// half-image w (16 LDS-DMA instructions of 8 rows x 128 B: whole lines) and reads A half wr and
// B half wc. Per lane the swizzled source chunk of an instruction is (lane & 7) ^ (lane >> 3)
// for every instruction (the 8 rows of one start at a multiple of 8), so one 32-bit voffset
// serves all 16.
//
// Schedule per K-tile t (stage s = t & 1; F0 / F1 = fragments of k-steps 0 / 1):
//   reads F1(t)  |  MFMA F0(t) x 64  |  lgkmcnt(0), vmcnt(0) [K-tile t+1 landed], barrier  |
//   DMA K-tile t+2 -> stage s  |  reads F0(t+1)  |  MFMA F1(t) x 64
// (gemm_tn4w.hip tile_body with b128 fragment reads).
#include "gemm_tile.h"

#include <cstdlib>
#include <type_traits>

namespace nf {
namespace gemm {
namespace nt4w {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;
constexpr int HALF = 128 * 64 * 2;     // 16 KiB half-image
constexpr int STAGE = 4 * HALF;        // 64 KiB per K-tile

// stage rows [row0, row0 + 128) x k [k0, k0 + 64) of a k-major operand into a half-image
__device__ __forceinline__ void stage(const bf16_t* __restrict__ base, long ld, int row0, int k0,
                                      char* dst, unsigned voff) {
  const char* b = (const char*)base + ((long)row0 * ld + k0) * 2;
#pragma unroll
  for (int piece = 0; piece < 16; ++piece) {
    const char* row = b + (long)(piece * 8) * ld * 2;
    const unsigned lds = (unsigned)(unsigned long)(LDS_AS char*)(dst + piece * 1024);
    // saddr + voffset LDS-DMA in asm (see gemm_tn4w.hip stage): the K-loop's explicit vmcnt
    // waits + barriers are the only ordering
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1"
                 :: "v"(voff), "s"(row), "s"(lds) : "memory", "m0");
  }
}

__device__ __forceinline__ void mfma_acc(v4f& acc, const v8s& a, const v8s& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int EPI>
__global__ void __launch_bounds__(NTHR, 1) gemm_nt4w_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char st0[STAGE];
  __shared__ __attribute__((aligned(16))) char st1[STAGE];
  const int ntn = a.N / BN;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (id / ntn) * BM, n0 = (id % ntn) * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nkt = a.K / BK;   // even (launch_nt4w)

  const bf16_t* sbase = wave < 2 ? a.A : a.B;
  const long sld = wave < 2 ? a.lda : a.ldb;
  const int srow0 = wave < 2 ? m0 + wave * 128 : n0 + (wave - 2) * 128;
  const unsigned voff =
      (unsigned)((((lane >> 3) * sld) + (((lane & 7) ^ (lane >> 3)) << 3)) * 2);
  auto stp = [&](auto p_c) -> char* { return decltype(p_c)::value ? st1 : st0; };
  auto issue = [&](int t, auto p_c) {
    stage(sbase, sld, srow0, t * BK, stp(p_c) + wave * HALF, voff);
  };

  v4f acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  v8s fa[8], fb0[8], fb1[8];
  auto rd_a = [&](auto p_c, int ks, int j) {
    return read_frag<true>(stp(p_c) + wr * HALF, j * 16, ks, lane);
  };
  auto rd_b = [&](auto p_c, int ks, v8s (&fb)[8]) {
    const char* st = stp(p_c) + (2 + wc) * HALF;
#pragma unroll
    for (int i = 0; i < 8; ++i) fb[i] = read_frag<true>(st, i * 16, ks, lane);
  };
  auto kstep = [&](const v8s (&fb)[8], auto pn_c, int ksn, auto rd_c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) mfma_acc(acc[i][j], fb[i], fa[j]);
      if constexpr (decltype(rd_c)::value) fa[j] = rd_a(pn_c, ksn, j);
    }
  };

  using P0 = std::false_type;
  using P1 = std::true_type;
  issue(0, P0{});
  issue(1, P1{});
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) fa[j] = rd_a(P0{}, 0, j);
  rd_b(P0{}, 0, fb0);
  auto ktile = [&](int t, auto p_c, auto next_c, auto issue_c) {
    constexpr bool P = decltype(p_c)::value;
    constexpr bool NEXT = decltype(next_c)::value, ISSUE = decltype(issue_c)::value;
    using PN = std::integral_constant<bool, !P>;
    rd_b(p_c, 1, fb1);
    kstep(fb0, p_c, 1, std::true_type{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (NEXT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ISSUE) issue(t + 2, p_c);
    if constexpr (NEXT) rd_b(PN{}, 0, fb0);
    kstep(fb1, PN{}, 0, next_c);
  };
  using T = std::true_type;
  using F = std::false_type;
  int t = 0;
  for (; t + 2 < nkt; t += 2) {
    ktile(t, P0{}, T{}, T{});
    ktile(t + 1, P1{}, T{}, T{});
  }
  ktile(t, P0{}, T{}, F{});
  ktile(t + 1, P1{}, F{}, F{});

  // acc[i][j]: n = n0 + 128 wc + 16 i + 4 (lane >> 4) + r, m = m0 + 128 wr + 16 j + (lane & 15)
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  __syncthreads();   // every wave is past its last operand read: the LDS is free
  char* region = (wave < 2 ? st0 : st1) + (wave & 1) * 32768;   // 2 x 16 KiB per wave
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    v4f sub[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sub[i][j] = acc[4 * h + i][j];
    epi_tile_staged<EPI, 8>(a, sub, m0 + wr * 128, n0 + wc * 128 + h * 64, 0,
                            region + h * 16384, lane);
  }
}

}  // namespace nt4w

// VINF_GEMM_NT4W=1: the plain NT bf16 products (EPI_BF16 / EPI_BF16_RELUMASK, no K ranges,
// no split-K) on the 4-wave kernel. False: off, or a shape it does not take (the caller runs
// the 8-wave kernel).
static int g_nt4w = [] {
  const char* e = getenv("VINF_GEMM_NT4W");
  return e ? atoi(e) : 0;
}();

bool launch_nt4w(GemmArgs a, int epi, hipStream_t stream) {
  if (!g_nt4w) return false;
  if (epi != EPI_BF16 && epi != EPI_BF16_RELUMASK) return false;
  if (a.M % nt4w::BM || a.N % nt4w::BN || a.K % (2 * nt4w::BK) || a.K <= 0 || a.lda % 8 ||
      a.ldb % 8 || ((unsigned long)a.A & 15) || ((unsigned long)a.B & 15) || a.krange || a.skip)
    return false;
  a.staged = staged_ok(a, epi);
  if (!a.staged) return false;
  const int nblk = (a.M / nt4w::BM) * (a.N / nt4w::BN);
  if (epi == EPI_BF16)
    hipLaunchKernelGGL(nt4w::gemm_nt4w_kernel<EPI_BF16>, dim3(nblk), dim3(nt4w::NTHR), 0, stream, a);
  else
    hipLaunchKernelGGL(nt4w::gemm_nt4w_kernel<EPI_BF16_RELUMASK>, dim3(nblk), dim3(nt4w::NTHR), 0,
                       stream, a);
  NF_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace gemm
}  // namespace nf

int nf_gemm_nt4w_set(int on) {   // on < 0: query only; returns the previous setting
  const int prev = nf::gemm::g_nt4w;
  if (on >= 0) nf::gemm::g_nt4w = on ? 1 : 0;
  return prev;
}
