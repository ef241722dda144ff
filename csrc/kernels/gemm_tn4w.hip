// Weight-gradient (TN) products on 4 fat waves: dW[m][n] = sum_k dy[k][m] x[k][n] (+ db[m]),
// both operands batch-major (mn-major for this product), one 256x256 output tile per block.
//
// Why a second TN kernel: in gemm256_multi_kernel (8 waves, 128x64 per wave) every mn-major
// fragment costs two ds_read_b64_tr_b16 and feeds 4 (A) or 8 (B) MFMAs per k-step; the probe in
// docs/PERF_NOTES.md ("Weight gradients: the mn-major operand stream is the cost") puts the TN
// excess over the NT kernel in that read path. Here each wave owns 128 x 128 outputs (256 fp32
// accumulators per lane, AGPR-backed: one wave per SIMD, 512-register budget), so every
// transposed fragment feeds 8 MFMAs and the LDS reads per MFMA drop by a third
// (32 fragments per 128 MFMAs per K-tile instead of 24 per 64).
//
// Geometry: 256 threads = 4 waves, wave w = (wr, wc) = (w >> 1, w & 1) owns tile rows
// [128 wr, +128) x cols [128 wc, +128). BK = 64. LDS: 2 stages x 4 half-images x 16 KiB =
// 128 KiB; half-image h of a stage = mn-major [64 k][128 mn] (gemm_tile.h layout, 16-B chunk c of
// k-row k at c ^ mn_swz(k)): h = 0 / 1: dy rows m0 + [0, 128) / [128, 256); h = 2 / 3: x cols
// n0 + [0, 128) / [128, 256). Wave w stages half-image w of every K-tile (16 LDS-DMA
// instructions of 4 k-rows x 256 contiguous bytes: whole 128-B lines) and reads A half wr and
// B half wc only.
//
// Schedule per K-tile t (stage s = t & 1; F0 / F1 = fragments of k-steps 0 / 1, 64 VGPRs each):
//   reads F1(t)  |  MFMA F0(t) x 64  |  lgkmcnt(0), vmcnt(0) [K-tile t+1 landed], barrier  |
//   DMA K-tile t+2 -> stage s  |  reads F0(t+1)  |  MFMA F1(t) x 64
// one barrier per K-tile; the barrier both publishes K-tile t+1 and retires every wave's reads of
// stage s before it is restaged. K-tile t+1's DMA has the compute of one K-tile to land.
#include "tn_multi.h"

#include <cstdlib>
#include <type_traits>

namespace nf {
namespace gemm {
namespace tn4w {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;
constexpr int HALF = 128 * 64 * 2;     // 16 KiB half-image
constexpr int STAGE = 4 * HALF;        // 64 KiB per K-tile

// stage half-image `h` of the K-tile at k0 (wave-uniform h == wave): 16 pieces of 4 k-rows.
// Address = uniform row base (SGPRs: k-row k0 + 4 piece) + a per-lane 32-bit byte offset that
// takes two values (the chunk swizzle depends on bit 1 of the piece): saddr + voffset LDS-DMA,
// 2 VGPRs instead of 16 64-bit addresses
template <int NPIECE = 16>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ base, long ld, int col0,
                                      int cols_total, int k0, char* dst, int lane) {
  unsigned voff[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int kr = v * 8 + (lane >> 4);           // pieces with bit 1 = v
    const int lc = (lane & 15) ^ mn_swz(kr);
    int gm = col0 + lc * 8;
    gm = gm < cols_total ? gm : cols_total - 8;
    voff[v] = (unsigned)(((lane >> 4) * ld + gm) * 2);
  }
  const char* b = (const char*)base + (long)k0 * ld * 2;
#pragma unroll
  for (int piece = 0; piece < NPIECE; ++piece) {
    const char* row = b + (long)(piece * 4) * ld * 2;
    const unsigned lds = (unsigned)(unsigned long)(LDS_AS char*)(dst + piece * 1024);
    // saddr + voffset form in asm: the builtin hoisted 16 64-bit per-lane addresses out of the
    // loop (32 VGPRs the 256-accumulator body cannot spare), and reusing their temporaries for
    // LDS reads made the compiler drain the DMA queue. The compiler does not track these DMAs:
    // the K-loop's explicit vmcnt waits + barrier are the only ordering (see the schedule above)
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1"
                 :: "v"(voff[(piece >> 1) & 1]), "s"(row), "s"(lds) : "memory", "m0");
  }
}

// acc += A x B with the accumulator tied to one AGPR quad ("+a": destination == srcC). The
// builtin left the register allocator free to rename 256 loop-carried accumulators, and it
// shuffled them between AGPRs and VGPRs with ~300 v_accvgpr moves per K-tile. The compiler does
// not see an MFMA here: the epilogue pads the result-read hazard itself (s_nop before reading).
__device__ __forceinline__ void mfma_acc(v4f& acc, const v8s& a, const v8s& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <bool DODB>
__device__ __forceinline__ void tile_body(const GemmArgs& a, int m0, int n0, char* st0,
                                          char* st1) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nkt = a.K / BK;

  // this wave's DMA source: half-image `wave`
  const bf16_t* sbase = wave < 2 ? a.A : a.B;
  const long sld = wave < 2 ? a.lda : a.ldb;
  const int scol0 = wave < 2 ? m0 + wave * 128 : n0 + (wave - 2) * 128;
  const int stot = wave < 2 ? a.M : a.N;
  // the two stages are separate __shared__ objects and every access below names one at compile
  // time: the compiler then knows a DMA into one stage cannot alias a read of the other. With
  // one array it drains the LDS-DMA queue (s_waitcnt vmcnt(0)) before every transposed read
  // (ds_read_b64_tr_b16 is not disambiguated like plain LDS loads are), i.e. waits for the DMA
  // it just issued for a later K-tile
  auto stp = [&](auto p_c) -> char* { return decltype(p_c)::value ? st1 : st0; };
  auto issue = [&](int t, auto p_c) {
    stage(sbase, sld, scol0, stot, t * BK, stp(p_c) + wave * HALF, lane);
  };

  v4f acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  float dbs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dbs[j] = 0.f;

  // A fragments single-buffered (fragment j of the next k-step is read as soon as the 8 MFMAs
  // of this k-step that use it are issued), B fragments double-buffered: 96 fragment VGPRs, so
  // the 256 accumulators stay put in the AGPRs
  v8s fa[8], fb0[8], fb1[8];
  auto rd_a = [&](auto p_c, int ks, int j) {
    return read_frag<false>(stp(p_c) + wr * HALF, j * 16, ks, lane);
  };
  auto rd_b = [&](auto p_c, int ks, v8s (&fb)[8]) {
    const char* st = stp(p_c) + (2 + wc) * HALF;
#pragma unroll
    for (int i = 0; i < 8; ++i) fb[i] = read_frag<false>(st, i * 16, ks, lane);
  };
  auto db_add = [&](int j) {   // db[m]: the A fragment's 8 k-values of row (lane & 15), v_dot2
    if constexpr (DODB) {
      typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
      const v2bf one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned w = (unsigned)(unsigned short)fa[j][2 * e] |
                           ((unsigned)(unsigned short)fa[j][2 * e + 1] << 16);
        dbs[j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, w), one, dbs[j], false);
      }
    }
  };
  // one k-step: for each A fragment j its 8 MFMAs, then (RD) its successor from (tn, ksn)
  auto kstep = [&](const v8s (&fb)[8], auto pn_c, int ksn, auto rd_c) {
    constexpr bool RD = decltype(rd_c)::value;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        mfma_acc(acc[i][j], fb[i], fa[j]);
      db_add(j);
      if constexpr (RD) fa[j] = rd_a(pn_c, ksn, j);
    }
  };

  using P0 = std::false_type;
  using P1 = std::true_type;
  if (nkt > 0) {
    issue(0, P0{});
    issue(1, P1{});
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] = rd_a(P0{}, 0, j);
    rd_b(P0{}, 0, fb0);
    // K-tile t in stage P (compile time); NEXT: K-tile t+1 exists; ISSUE: K-tile t+2 exists
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
    // nkt is even (launch_tn4w_multi): pairs of K-tiles in stages 0, 1; the last pair drains
    int t = 0;
    for (; t + 2 < nkt; t += 2) {
      ktile(t, P0{}, T{}, T{});
      ktile(t + 1, P1{}, T{}, T{});
    }
    ktile(t, P0{}, T{}, F{});
    ktile(t + 1, P1{}, F{}, F{});
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j]: n = n0 + 128 wc + 16 i + 4 (lane >> 4) + r, m = m0 + 128 wr + 16 j + (lane & 15)
  const int g = lane >> 4, c = lane & 15;
  if (DODB && wc == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = dbs[j];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = m0 + wr * 128 + j * 16 + c;
      if (g == 0 && m < a.M) a.dbias[m] = v;
    }
  }
  // MFMA result -> VALU / v_accvgpr_read: 8-pass XDL needs 12 wait states after the last MFMA
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
    if (a.staged)
      epi_tile_staged<EPI_F32, 8>(a, sub, m0 + wr * 128, n0 + wc * 128 + h * 64, 0,
                                  region + h * 16384, lane);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + wr * 128 + j * 16 + c;
        if (m >= a.M) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = n0 + wc * 128 + h * 64 + i * 16 + g * 4;
          if (n < a.N) epi_store<EPI_F32>(a, sub[i][j], m, n, 0);
        }
      }
  }
}

// Deeper variant (VINF_TN4W_STAGES=4): 32-deep K-tiles in 4 stages of 32 KiB (separate
// __shared__ objects, compile-time stage per access), K-tile t+3 issued while t is computed, so
// up to 96 KiB per CU are in flight instead of 64; one barrier per 64 MFMAs.
template <bool DODB, int PD>
__device__ __forceinline__ void tile_body4(const GemmArgs& a, int m0, int n0, char* q0, char* q1,
                                           char* q2, char* q3) {
  constexpr int BK4 = 32, HALF4 = 128 * BK4 * 2;   // 8 KiB half-image
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nkt = a.K / BK4;   // a multiple of 4 (launch_tn4w_multi: K % 128 == 0)
  const bf16_t* sbase = wave < 2 ? a.A : a.B;
  const long sld = wave < 2 ? a.lda : a.ldb;
  const int scol0 = wave < 2 ? m0 + wave * 128 : n0 + (wave - 2) * 128;
  const int stot = wave < 2 ? a.M : a.N;
  auto stp = [&](auto q_c) -> char* {
    constexpr int Q = decltype(q_c)::value;
    return Q == 0 ? q0 : Q == 1 ? q1 : Q == 2 ? q2 : q3;
  };
  auto issue = [&](int t, auto q_c) {
    stage<8>(sbase, sld, scol0, stot, t * BK4, stp(q_c) + wave * HALF4, lane);
  };
  v4f acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  float dbs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dbs[j] = 0.f;
  v8s fa[8], fb0[8], fb1[8];
  auto rd_a = [&](auto q_c, int j) { return read_frag<false>(stp(q_c) + wr * HALF4, j * 16, 0, lane); };
  auto rd_b = [&](auto q_c, v8s (&fb)[8]) {
    const char* st = stp(q_c) + (2 + wc) * HALF4;
#pragma unroll
    for (int i = 0; i < 8; ++i) fb[i] = read_frag<false>(st, i * 16, 0, lane);
  };
  auto kstep = [&](const v8s (&fb)[8], auto qn_c, auto rd_c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) mfma_acc(acc[i][j], fb[i], fa[j]);
      if constexpr (DODB) {
        typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
        const v2bf one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned w = (unsigned)(unsigned short)fa[j][2 * e] |
                             ((unsigned)(unsigned short)fa[j][2 * e + 1] << 16);
          dbs[j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, w), one, dbs[j], false);
        }
      }
      if constexpr (decltype(rd_c)::value) fa[j] = rd_a(qn_c, j);
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  // PD: prefetch distance in K-tiles (K-tile t + PD issued while t is computed): 3 keeps up to
  // 96 KiB per CU in flight, 2 keeps 64 KiB (less of the XCD's 4 MiB L2 held by data in flight)
  issue(0, std::integral_constant<int, 0>{});
  issue(1, std::integral_constant<int, 1>{});
  if constexpr (PD == 3) {
    issue(2, std::integral_constant<int, 2>{});
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) fa[j] = rd_a(std::integral_constant<int, 0>{}, j);
  rd_b(std::integral_constant<int, 0>{}, fb0);
  // K-tile t in stage Q; W2: K-tile t+2 outstanding (wait vmcnt(8), else 0); NEXT: t+1 exists;
  // ISSUE: t+3 exists
  auto ktile = [&](int t, auto q_c, const v8s (&fbc)[8], v8s (&fbn)[8], auto w2_c, auto next_c,
                   auto issue_c) {
    constexpr int Q = decltype(q_c)::value;
    using QN = std::integral_constant<int, (Q + 1) & 3>;
    using QI = std::integral_constant<int, (Q + PD) & 3>;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (decltype(next_c)::value) {
      if constexpr (PD == 3 && decltype(w2_c)::value) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (decltype(issue_c)::value) issue(t + PD, QI{});
    if constexpr (decltype(next_c)::value) rd_b(QN{}, fbn);
    kstep(fbc, QN{}, next_c);
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  using Q2 = std::integral_constant<int, 2>;
  using Q3 = std::integral_constant<int, 3>;
  int t = 0;
  for (; t + 4 < nkt; t += 4) {
    ktile(t, Q0{}, fb0, fb1, T{}, T{}, T{});
    ktile(t + 1, Q1{}, fb1, fb0, T{}, T{}, T{});
    ktile(t + 2, Q2{}, fb0, fb1, T{}, T{}, T{});
    ktile(t + 3, Q3{}, fb1, fb0, T{}, T{}, T{});
  }
  // last four K-tiles: the first still issues K-tile nkt-1
  if constexpr (PD == 3) {
    ktile(t, Q0{}, fb0, fb1, T{}, T{}, T{});
    ktile(t + 1, Q1{}, fb1, fb0, T{}, T{}, F{});
  } else {   // K-tiles nkt-2, nkt-1 still to issue
    ktile(t, Q0{}, fb0, fb1, F{}, T{}, T{});
    ktile(t + 1, Q1{}, fb1, fb0, F{}, T{}, T{});
  }
  ktile(t + 2, Q2{}, fb0, fb1, F{}, T{}, F{});
  ktile(t + 3, Q3{}, fb1, fb0, F{}, F{}, F{});

  const int g = lane >> 4, c = lane & 15;
  if (DODB && wc == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = dbs[j];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = m0 + wr * 128 + j * 16 + c;
      if (g == 0 && m < a.M) a.dbias[m] = v;
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  __syncthreads();
  char* region = (wave == 0 ? q0 : wave == 1 ? q1 : wave == 2 ? q2 : q3);   // 32 KiB per wave
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    v4f sub[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sub[i][j] = acc[4 * h + i][j];
    if (a.staged)
      epi_tile_staged<EPI_F32, 8>(a, sub, m0 + wr * 128, n0 + wc * 128 + h * 64, 0,
                                  region + h * 16384, lane);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + wr * 128 + j * 16 + c;
        if (m >= a.M) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = n0 + wc * 128 + h * 64 + i * 16 + g * 4;
          if (n < a.N) epi_store<EPI_F32>(a, sub[i][j], m, n, 0);
        }
      }
  }
}

template <int PD>
__global__ void __launch_bounds__(NTHR, 1) gemm_tn4w4_kernel(g256::TnMulti t) {
  __shared__ __attribute__((aligned(16))) char q0[32768];
  __shared__ __attribute__((aligned(16))) char q1[32768];
  __shared__ __attribute__((aligned(16))) char q2[32768];
  __shared__ __attribute__((aligned(16))) char q3[32768];
  const int pos = xcd_remap(blockIdx.x, t.ntiles);
  const int id = t.tile0 + (t.use_perm ? (int)t.perm[pos] : pos);
  int p = 0;
  for (int q = 1; q < t.n; ++q)
    if (id >= t.d[q].start) p = q;
  const g256::TnDesc& d = t.d[p];
  GemmArgs a{};
  a.A = d.A; a.lda = d.lda;
  a.B = d.B; a.ldb = d.ldb;
  a.C = d.C; a.ldc = d.ldc;
  a.dbias = d.db;
  a.M = d.M; a.N = d.N; a.K = d.K;
  a.staged = d.staged;
  a.cmask = d.cmask;
  const int local = d.tiles ? (int)d.tiles[id - d.start] : id - d.start;
  const int ntn = (a.N + BN - 1) / BN;
  const int tm = local / ntn, tn = local % ntn;
  if (a.dbias != nullptr && tn == 0) tile_body4<true, PD>(a, tm * BM, tn * BN, q0, q1, q2, q3);
  else tile_body4<false, PD>(a, tm * BM, tn * BN, q0, q1, q2, q3);
}

__global__ void __launch_bounds__(NTHR, 1) gemm_tn4w_kernel(g256::TnMulti t) {
  __shared__ __attribute__((aligned(16))) char st0[STAGE];
  __shared__ __attribute__((aligned(16))) char st1[STAGE];
  const int pos = xcd_remap(blockIdx.x, t.ntiles);
  const int id = t.tile0 + (t.use_perm ? (int)t.perm[pos] : pos);
  int p = 0;
  for (int q = 1; q < t.n; ++q)
    if (id >= t.d[q].start) p = q;
  const g256::TnDesc& d = t.d[p];
  GemmArgs a{};
  a.A = d.A; a.lda = d.lda;
  a.B = d.B; a.ldb = d.ldb;
  a.C = d.C; a.ldc = d.ldc;
  a.dbias = d.db;
  a.M = d.M; a.N = d.N; a.K = d.K;
  a.staged = d.staged;
  a.cmask = d.cmask;
  const int local = d.tiles ? (int)d.tiles[id - d.start] : id - d.start;
  const int ntn = (a.N + BN - 1) / BN;
  const int tm = local / ntn, tn = local % ntn;
  if (a.dbias != nullptr && tn == 0) tile_body<true>(a, tm * BM, tn * BN, st0, st1);
  else tile_body<false>(a, tm * BM, tn * BN, st0, st1);
}

}  // namespace tn4w

bool launch_tn4w_multi(const g256::TnMulti& t, hipStream_t stream) {
  for (int i = 0; i < t.n; ++i) {
    const g256::TnDesc& d = t.d[i];
    // an even number of 64-deep K-tiles, 16-B operand rows (8 bf16 columns), 16-B aligned bases
    if (d.K % (2 * tn4w::BK) || d.M % 8 || d.N % 8 || d.lda % 8 || d.ldb % 8 ||
        ((unsigned long)d.A & 15) || ((unsigned long)d.B & 15))
      return false;
  }
  static const int stages = [] {
    const char* e = getenv("VINF_TN4W_STAGES");
    return e ? atoi(e) : 4;   // 4: profiles/r4/tn4w4_layout_probe.jsonl (2: tn4w_layout_probe)
  }();
  static const int pd = [] {
    const char* e = getenv("VINF_TN4W_PD");
    return e && atoi(e) == 2 ? 2 : 3;
  }();
  if (stages == 4 && pd == 2)
    hipLaunchKernelGGL(tn4w::gemm_tn4w4_kernel<2>, dim3(t.ntiles), dim3(tn4w::NTHR), 0, stream, t);
  else if (stages == 4)
    hipLaunchKernelGGL(tn4w::gemm_tn4w4_kernel<3>, dim3(t.ntiles), dim3(tn4w::NTHR), 0, stream, t);
  else
    hipLaunchKernelGGL(tn4w::gemm_tn4w_kernel, dim3(t.ntiles), dim3(tn4w::NTHR), 0, stream, t);
  NF_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace gemm
}  // namespace nf
