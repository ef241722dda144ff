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
// [128 wr, +128) x cols [128 wc, +128). K-tiles of 32 k in 4 LDS stages of 32 KiB; a stage holds
// four mn-major half-images [32 k][128 mn] (gemm_tile.h layout, 16-B chunk c of k-row k at
// c ^ mn_swz(k)): h = 0 / 1: dy rows m0 + [0, 128) / [128, 256); h = 2 / 3: x cols n0 + [0, 128)
// / [128, 256). Wave w stages half-image w of every K-tile (LDS-DMA pieces of 4 k-rows x 256
// contiguous bytes: whole 128-B lines) and reads A half wr and B half wc only. K-tile t + 3 is in
// flight while t is multiplied (tile_body4 below).

#include "tn_multi.h"

#include <cstdlib>
#include <type_traits>

namespace nf {
namespace gemm {
namespace tn4w {

// BK: the launch granule (launch_tn4w_multi needs K % (2 BK) == 0, i.e. a whole number of
// 4-K-tile loop iterations); the body itself runs 32-deep K-tiles in 4 stages of 32 KiB
// (tile_body4: BK4, HALF4)
constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;

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
#ifdef NF_PROBE_DMA_SAMEADDR   // timing probe: every lane of a piece reads the same 16 B
    voff[v] = 0;
#endif
  }
  const char* b = (const char*)base + (long)k0 * ld * 2;
#pragma unroll
  for (int piece = 0; piece < NPIECE; ++piece) {
#ifdef NF_PROBE_DMA_HALF       // timing probe: half the pieces
    if (piece & 1) continue;
#endif
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

// 32-deep K-tiles in 4 stages of 32 KiB (separate __shared__ objects, compile-time stage per
// access), K-tile t + PD issued while t is computed (PD = 3: up to 96 KiB per CU in flight); one
// barrier per 64 MFMAs. (A 2-stage body of 64-deep K-tiles, 64 KiB in flight, took 2193-2316 us
// per real multi-layer launch against 1959-2075 for this one: profiles/r4/tn4w4_layout_probe.jsonl;
// prefetch distance 2 2217-2234 us: profiles/r4/tn4w4_pd_layout.jsonl.)
// DBM: bit j set = this wave sums the bias gradient of its A row block j (rows 16 j of its
// 128-row half) with v_dot2 on the A fragments it already holds. Every row block of a row tile is
// owned by exactly one (column tile, wave) pair (gemm_tn4w4_kernel: db_mask), so the dot
// products are spread over the waves of the first two column tiles instead of all four waves of
// the first column tile each summing all eight blocks (half of it redundant: the two column
// waves hold the same A rows). Compile-time masks: a runtime mask test inside the unrolled
// K-step split the MFMA / ds_read / DMA schedule into basic blocks and cost more than it saved
// (docs/PERF_NOTES.md round 5, "dbhalf").
template <int DBM, int PD>
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
  // MFMAs of A fragment j (+ its bias-gradient dot products), then A fragment j of the next
  // K-tile into the freed registers
  // the next K-tile's B fragments: fragment 0 behind the DMA burst, fragment j behind the MFMAs
  // of A fragment j (one burst of all 16 reads after the first 8 MFMAs held the MFMA pipe:
  // real 13-layer launch 2210-2273 vs 2259-2313 us median, profiles/r6/tn4w_bspread_ab.jsonl)
  v8s* fbn_p = nullptr;
  auto mfma_j = [&](const v8s (&fb)[8], auto qn_c, auto rd_c, auto j_c) {
    constexpr int j = decltype(j_c)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) mfma_acc(acc[i][j], fb[i], fa[j]);
    if constexpr ((DBM >> j) & 1) {
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
    if constexpr (decltype(rd_c)::value && j > 0)
      fbn_p[j] = read_frag<false>(stp(qn_c) + (2 + wc) * HALF4, j * 16, 0, lane);
  };
  // A fragments 1..7 of a K-tile (fragment 0 is issued first, see ktile)
  auto kstep_from1 = [&](const v8s (&fb)[8], auto qn_c, auto rd_c) {
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 1>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 2>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 3>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 4>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 5>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 6>{});
    mfma_j(fb, qn_c, rd_c, std::integral_constant<int, 7>{});
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
#ifndef NF_PROBE_NOBAR   // timing probe: no block barrier per K-tile
    __builtin_amdgcn_s_barrier();
#endif
    __builtin_amdgcn_sched_barrier(0);
    // the first 8 MFMAs go out right after the barrier (their operands are already in
    // registers), the DMA issue and the next K-tile's B reads behind them: the MFMA pipe
    // restarts one instruction after the barrier instead of ~25 (whole step -0.13 ms on one
    // box, profiles/r5/tn4w_early_mfma_ab.jsonl)
    mfma_j(fbc, QN{}, next_c, std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_barrier(0);
#ifndef NF_PROBE_NODMA   // timing probes only (wrong results): no operand DMA in the K loop
    if constexpr (decltype(issue_c)::value) issue(t + PD, QI{});
#endif
    if constexpr (decltype(next_c)::value)
      fbn[0] = read_frag<false>(stp(QN{}) + (2 + wc) * HALF4, 0, 0, lane);
    fbn_p = fbn;
    __builtin_amdgcn_sched_barrier(0);
    kstep_from1(fbc, QN{}, next_c);
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
  if constexpr (DBM != 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!((DBM >> j) & 1)) continue;
      float v = dbs[j];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = m0 + wr * 128 + j * 16 + c;
      if (g == 0 && m < a.M) a.dbias[m] = v;
    }
  }
  // the accumulators are written by asm MFMAs the compiler cannot see: keep every epilogue read
  // of them below the pad (no v_accvgpr read may be scheduled above it)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
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
  // bias-gradient ownership: with >= 2 column tiles, column tile 0 sums row blocks 0-3 and
  // column tile 1 row blocks 4-7, each split between its two column waves (2 blocks per wave);
  // a single column tile gives each of its column waves 4 blocks
  const int wc = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1;
  const int m0 = tm * BM, n0 = tn * BN;
  // (a masked problem launches only its active tiles: there the first column tile alone owns
  // the row tile's bias gradient, split between its two column waves, as before)
  const bool spread = d.tiles == nullptr && ntn >= 2;
  if (a.dbias != nullptr && (spread ? tn < 2 : tn == 0)) {
    if (!spread) {
      if (wc == 0) tile_body4<0x0F, PD>(a, m0, n0, q0, q1, q2, q3);
      else tile_body4<0xF0, PD>(a, m0, n0, q0, q1, q2, q3);
    } else if (tn == 0) {
      if (wc == 0) tile_body4<0x03, PD>(a, m0, n0, q0, q1, q2, q3);
      else tile_body4<0x0C, PD>(a, m0, n0, q0, q1, q2, q3);
    } else {
      if (wc == 0) tile_body4<0x30, PD>(a, m0, n0, q0, q1, q2, q3);
      else tile_body4<0xC0, PD>(a, m0, n0, q0, q1, q2, q3);
    }
  } else {
    tile_body4<0, PD>(a, m0, n0, q0, q1, q2, q3);
  }
}

}  // namespace tn4w

bool launch_tn4w_multi(const g256::TnMulti& t, hipStream_t stream) {
  for (int i = 0; i < t.n; ++i) {
    const g256::TnDesc& d = t.d[i];
    // an even number of 64-deep K-tiles, 16-B operand rows (8 bf16 columns), 16-B aligned bases
    if (d.K <= 0 || d.K % (2 * tn4w::BK) || d.M % 8 || d.N % 8 || d.lda % 8 || d.ldb % 8 ||
        ((unsigned long)d.A & 15) || ((unsigned long)d.B & 15))
      return false;
  }
  hipLaunchKernelGGL(tn4w::gemm_tn4w4_kernel<3>, dim3(t.ntiles), dim3(tn4w::NTHR), 0, stream, t);
  NF_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace gemm
}  // namespace nf
