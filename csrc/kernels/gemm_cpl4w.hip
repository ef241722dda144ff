// Fused coupling-forward product on 4 fat waves (one per SIMD, 512 registers each):
//   [s_hat | t] = h W^T + b,  s = scale tanh(s_hat),  y = x e^s + t  (inverse: x = (y - t) e^-s)
// for the last conditioner product of an affine coupling layer (RealNVP; SURVEY §2.4
// coupling_fwd; reference transform /root/reference/normflows/normflows/flows.py:8-34).
//
// Why a second kernel for this product: Dh = 392 = 3 x 128 + 8. The 8-wave 256 x 256 kernel
// (gemm256.hip EPI_CPL_FWD) pairs the s_hat and t columns of 128 features per column tile, so
// the last 8 features take a fourth column tile that streams the whole 256-row activation panel
// for 16 useful columns (~30 us of a 170 us product at the headline shape,
// docs/PERF_NOTES.md round 5). Folding them into a 256-register wave spilled. Here a wave owns
// 64 rows x 272 columns = 136 features (s and t) in 272 AGPRs, so three column tiles cover
// 408 >= 392 features and no edge tile exists: 3/4 of the A-panel streams and ~20 % fewer
// MFMAs at the headline shape.
//
// Geometry: block = 256 threads = 4 waves, tile = 256 rows x 136 features. Wave w owns rows
// [64 w, +64) and every column: 17 column blocks of 16 (the B image rows):
//   block 2p / 2p+1 (p < 8): s_hat / t of features f0 + 16 p + [0, 16)
//   block 16: s_hat of features f0 + 128 + [0, 8) (cols 0..7), t of the same (cols 8..15).
// The MFMA runs transposed (A operand = W fragment, B operand = h fragment), so a lane holds 4
// consecutive columns of one row: the s_hat and t of the same 4 features sit in the same lane
// (blocks 2p, 2p+1) and the epilogue is register-only (block 16: one cross-half shuffle).
// K-tiles of 32 k in 4 LDS stages of 33 KiB (A [256][32] + B [272][32] bf16, 64-B rows, 16-B
// chunk c of row r at c ^ (((r >> 2) & 1) << 1): conflict-free ds_read_b128 for every lane group,
// host check: tests/test_realnvp_engine.py::test_cpl4w_lds_layout_conflict_free), K-tile t + 3 in flight while t is multiplied,
// one barrier per 68 MFMAs per wave. A and B fragments are double-buffered across K-tiles.
#include "cpl4w.h"
#include "gemm_tile.h"

#include <type_traits>

namespace nf {
namespace gemm {
namespace cpl4w {

constexpr int BM = 256, NFT = 136, NB = 17, BK = 32, NTHR = 256;
constexpr int A_IMG = BM * 64;         // 16 KiB
constexpr int B_IMG = NB * 16 * 64;    // 17 KiB
constexpr int STG = A_IMG + B_IMG;     // 33 KiB per K-tile stage
constexpr int NST = 4, PD = 3;


// chunk position of 16-B chunk c of image row r (64-B rows)
__device__ __forceinline__ int pos(int r, int c) { return c ^ (((r >> 2) & 1) << 1); }

// v_mfma_f32_16x16x32_bf16 with the accumulator tied to its AGPRs (see gemm_tn4w.hip mfma_acc)
// A wave has at most 256 AGPRs: blocks 0..15 accumulate there (256 registers), block 16 in
// VGPRs (the MFMA takes either as C / D; with "+a" for all 272 the allocator shuttled the extra
// ones through v_accvgpr moves around every MFMA)
__device__ __forceinline__ void mfma_acc(v4f& acc, const v8s& a, const v8s& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_accv(v4f& acc, const v8s& a, const v8s& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void dma(const char* src, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(src), "s"(lds) : "memory", "m0");
}

// W row of B-image row r of column tile f0
__device__ __forceinline__ int b_wrow(int r, int f0, int Dh) {
  const int j = r >> 4, b = r & 15;
  int f, t;
  if (j < 16) {
    f = f0 + 16 * (j >> 1) + b;
    t = j & 1;
  } else {
    f = f0 + 128 + (b & 7);
    t = b >> 3;
  }
  // features past Dh read the last valid s / t row (never stored); keeping every lane's row >=
  // the block's first row keeps the per-lane DMA offsets non-negative
  f = f < Dh ? f : Dh - 1;
  return t ? Dh + f : f;
}

// fragment of 16 image rows [r0, r0 + 16) x 32 k (the 16x16x32 operand layout: lane l holds
// row r0 + (l & 15), k = 8 (l >> 4) + [0, 8))
__device__ __forceinline__ v8s rd(const char* img, int r0, int lane) {
  const int r = r0 + (lane & 15), c = lane >> 4;
  return *(const LDS_AS v8s*)(img + r * 64 + (pos(r, c) << 4));
}

__global__ void __launch_bounds__(NTHR, 1) gemm_cpl4w_kernel(Args a) {
  // K-loop ring (132 KiB), reused by the epilogue's staging (4 waves x 34 KiB = 136 KiB)
  __shared__ __attribute__((aligned(16))) char smem[NST * STG > 4 * 2 * 64 * NFT * 2 ? NST * STG : 4 * 2 * 64 * NFT * 2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = ((a.M + BM - 1) / BM) * a.ntn;
  const int id = xcd_remap(blockIdx.x, ntiles);   // the ntn column tiles of a row tile: one XCD
  const int tm = id / a.ntn, tn = id % a.ntn;
  const int m0 = tm * BM, f0 = tn * NFT;
  const int nkt = a.K / BK;                        // a multiple of 4 (launcher: K % 128 == 0)

  // ---- DMA plan (loop-invariant): wave w stages A rows [64 w, +64) (4 pieces of 16 rows) and
  // B blocks [jb, jb + nb) (wave 0: 5, waves 1-3: 4). Piece = 16 image rows x 64 B = 1 KiB;
  // lane l writes row (l >> 2), position (l & 3), i.e. source chunk (l & 3) ^ ((l >> 4) & 1) * 2.
  const int csrc = (lane & 3) ^ (((lane >> 4) & 1) << 1);
  const int jb = wave == 0 ? 0 : 1 + 4 * wave, nb = wave == 0 ? 5 : 4;
  // A piece q of this wave at k = 0: rows m0 + 64 w + 16 q + [0, 16), a piece past M (M % 16 ==
  // 0: whole pieces) re-reads the last 16 rows (never stored)
  const char* pa[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int r0 = m0 + 64 * wave + 16 * q;
    r0 = r0 <= a.M - 16 ? r0 : a.M - 16;
    pa[q] = (const char*)a.A + (long)r0 * a.lda * 2;
  }
  const unsigned voa = (unsigned)(((long)(lane >> 2) * a.lda + csrc * 8) * 2);
  const char* pb[5];
  unsigned vob[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int j = jb + (q < nb ? q : nb - 1);
    // lane row of the block, clamped into the weight matrix (features >= Dh are computed on
    // duplicate rows and never stored)
    const int wl = b_wrow(16 * j + (lane >> 2), f0, a.Dh);   // < 2 Dh <= w_rows
    const int w0 = __builtin_amdgcn_readfirstlane(wl);   // row of lane 0 (uniform base)
    pb[q] = (const char*)a.W + (long)w0 * a.ldw * 2;
    vob[q] = (unsigned)(((long)(wl - w0) * a.ldw + csrc * 8) * 2);
  }
  const unsigned lds0 = (unsigned)(unsigned long)(LDS_AS char*)smem;
  auto issue = [&](int t, int st) {
    const long ko = (long)t * BK * 2;
    const unsigned sb = lds0 + st * STG;
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(pa[q] + ko, voa, sb + (64 * wave + 16 * q) * 64);
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (q < nb) dma(pb[q] + ko, vob[q], sb + A_IMG + (jb + q) * 1024);
  };

  v4f acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  v8s fa0[4], fa1[4], fb0[NB], fb1[NB];
  auto img_a = [&](int st) -> const char* { return smem + st * STG; };
  auto img_b = [&](int st) -> const char* { return smem + st * STG + A_IMG; };

  // prologue: K-tiles 0..2 in flight, wait for 0, its fragments into set 0
  issue(0, 0);
  issue(1, 1);
  issue(2, 2);
  if (wave == 0) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i) fa0[i] = rd(img_a(0), 64 * wave + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < NB; ++j) fb0[j] = rd(img_b(0), 16 * j, lane);

  // K-tile t from stage Q with fragments (fac, fbc); the next K-tile's fragments into (fan, fbn)
  // from stage Q + 1; K-tile t + 3 issued into stage Q + 3 (read last during K-tile t - 2).
  // Every K-tile runs the same code (no peeled tail: a separate tail made the register allocator
  // copy accumulators right behind the asm MFMAs that had not written them yet): the issue and
  // the wait depth are uniform branches.
  auto ktile = [&](int t, auto q_c, const v8s (&fac)[4], const v8s (&fbc)[NB], v8s (&fan)[4],
                   v8s (&fbn)[NB]) {
    constexpr int Q = decltype(q_c)::value;
    constexpr int QN = (Q + 1) & 3, QI = (Q + PD) & 3;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 2 < a.K / BK) {   // K-tile t + 2 may stay in flight
      if (wave == 0) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#ifndef NF_PROBE_NODMA   // timing probe (wrong results): no operand DMA in the K loop
    if (t + PD < nkt) issue(t + PD, QI);
#endif
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (j < 16) mfma_acc(acc[i][j], fbc[j], fac[i]);
        else mfma_accv(acc[i][j], fbc[j], fac[i]);
      }
      __builtin_amdgcn_sched_barrier(0);
      fbn[j] = rd(img_b(QN), 16 * j, lane);
      if (j < 4) fan[j] = rd(img_a(QN), 64 * wave + 16 * j, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  using Q2 = std::integral_constant<int, 2>;
  using Q3 = std::integral_constant<int, 3>;
  for (int t = 0; t < nkt; t += 4) {
    ktile(t, Q0{}, fa0, fb0, fa1, fb1);
    ktile(t + 1, Q1{}, fa1, fb1, fa0, fb0);
    ktile(t + 2, Q2{}, fa0, fb0, fa1, fb1);
    ktile(t + 3, Q3{}, fa1, fb1, fa0, fb0);
    if (t + 4 >= nkt) {   // the MFMA results need their wait states before the epilogue reads
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#ifdef NF_PROBE_NOEPI   // timing probe (wrong results): main loop only
  if (a.M < 0) a.y[lane] = acc[0][0][0] + acc[3][16][3];
  return;
#endif

  // ---- epilogue in two phases through LDS (the ring is idle: every wave drained its DMAs
  // before the last K-tile barrier, after which no stage is read for data).
  // Phase 1, fragment layout: lane l holds, for row block i, row 16 i + (l & 15) of the wave and
  // columns 16 j + 4 g + [0, 4), g = l >> 4. It adds the bias, rounds s_hat and t to bf16 (as
  // the stored s_hat the backward reads, and bitwise as the 8-wave kernel), parks both in the
  // wave's own LDS region [64 rows][136 features] x {s_hat, t}, and sums s for the log-det.
  // Phase 2, row layout: lane = 16-B chunk of 8 features of a row, so x loads and y / yb / st
  // stores run along rows (17 chunks = 544 B of fp32 per row) instead of 16 rows x 64 B per
  // instruction, which ran the first version's epilogue at half the store rate (~100 of 190 us).
  const int g = lane >> 4, rl = lane & 15;
  const int Dh = a.Dh;
  constexpr int RP = NFT * 2;                          // bytes per staged row (bf16)
  char* s_img = smem + wave * (2 * 64 * RP);           // [64][136] s_hat
  char* t_img = s_img + 64 * RP;                       // [64][136] t
  const float scale = a.scale;
  auto bf2 = [](unsigned w, int hi) -> float {
    return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16));
  };
  // bias of this lane's 4 features of each pair (s and t), loaded before x: a load's first use
  // waits for every older load (vmcnt counts in issue order)
  uint2 bs[9], bt[9];
#pragma unroll
  for (int p = 0; p < 9; ++p) {
    const int fp = f0 + (p < 8 ? 16 * p + 4 * g : 128 + 4 * (g & 1));
    bs[p] = bt[p] = make_uint2(0u, 0u);
    if (a.bias && fp < Dh) {
      bs[p] = *reinterpret_cast<const uint2*>(a.bias + fp);
      bt[p] = *reinterpret_cast<const uint2*>(a.bias + Dh + fp);
    }
  }
  // phase-2 operands next: this lane's x (17 chunks of 8 features) is in flight during phase 1
  const int nch = Dh - f0 < NFT ? (Dh - f0) / 8 : NFT / 8;   // valid chunks of this tile
  float4 xq[17][2];
#pragma unroll
  for (int it = 0; it < 17; ++it) {
    const int item = it * 64 + lane, row = item / 17, c = item % 17;
    const int m = m0 + 64 * wave + row;
    xq[it][0] = xq[it][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nch && m < a.M) {
      const float* xr = a.x + (long)m * a.ld_x + f0 + 8 * c;
      xq[it][0] = *reinterpret_cast<const float4*>(xr);
      xq[it][1] = *reinterpret_cast<const float4*>(xr + 4);
    }
  }
  float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < 9; ++p) {
    const int fl = p < 8 ? 16 * p + 4 * g : 128 + 4 * (g & 1);   // feature within the tile
    const int fp = f0 + fl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * i + rl;
      float sh[4], tv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned bsw = r < 2 ? bs[p].x : bs[p].y, btw = r < 2 ? bt[p].x : bt[p].y;
        if (p < 8) {
          sh[r] = acc[i][2 * p][r] + bf2(bsw, r & 1);
          tv[r] = acc[i][2 * p + 1][r] + bf2(btw, r & 1);
        } else {   // block 16: lanes g < 2 hold s_hat, g >= 2 the t of the same features
          sh[r] = acc[i][16][r] + bf2(bsw, r & 1);
          tv[r] = acc[i][16][r] + bf2(btw, r & 1);
        }
      }
      v2u so, to;
      so.x = (unsigned)f2bf(sh[0]) | ((unsigned)f2bf(sh[1]) << 16);
      so.y = (unsigned)f2bf(sh[2]) | ((unsigned)f2bf(sh[3]) << 16);
      to.x = (unsigned)f2bf(tv[0]) | ((unsigned)f2bf(tv[1]) << 16);
      to.y = (unsigned)f2bf(tv[2]) | ((unsigned)f2bf(tv[3]) << 16);
      if (p < 8 || g < 2) {
        *(LDS_AS v2u*)(s_img + row * RP + fl * 2) = so;
        if (fp < Dh) {
#pragma unroll
          for (int r = 0; r < 4; ++r) part[i] += scale * fast_tanhf(bf2(r < 2 ? so.x : so.y, r & 1));
        }
      }
      if (p < 8 || g >= 2) *(LDS_AS v2u*)(t_img + row * RP + fl * 2) = to;
    }
  }
  // log-det partials: the 4 lane groups hold disjoint features of the same rows
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = a.inverse ? -part[i] : part[i];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    const int m = m0 + 64 * wave + 16 * i + rl;
    if (g == 0 && m < a.M) {
      float* lp = a.ldjp + (long)tn * a.ld_ldjp + m;
      *lp = a.ldj_init ? v : *lp + v;
      if (a.ldj_init && tn == a.ntn - 1)   // rows no column tile owns
        for (int r = a.ntn; r < a.ldj_rows; ++r) a.ldjp[(long)r * a.ld_ldjp + m] = 0.f;
    }
  }
  // phase 2: 64 rows x 17 chunks of 8 features per wave, 17 passes of 64 lanes
#ifdef NF_PROBE_PH1ONLY   // timing probe (wrong results): no phase 2
  if (a.M < 0) a.y[lane] = xq[3][1].x + xq[16][0].y;
  return;
#endif
#ifdef NF_PROBE_NOSTORE   // timing probe (wrong results): phase 2 without its global stores
  float dummy = 0.f;
#endif
#pragma unroll
  for (int it = 0; it < 17; ++it) {
    const int item = it * 64 + lane, row = item / 17, c = item % 17;
    const int m = m0 + 64 * wave + row;
    if (c >= nch || m >= a.M) continue;
    const int f = f0 + 8 * c;
    const v4u su = *(const LDS_AS v4u*)(s_img + row * RP + c * 16);
    const v4u tu = *(const LDS_AS v4u*)(t_img + row * RP + c * 16);
    const float4 x0 = xq[it][0], x1 = xq[it][1];
    const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    const unsigned sw[4] = {su.x, su.y, su.z, su.w}, tw[4] = {tu.x, tu.y, tu.z, tu.w};
    float yv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sh = bf2(sw[e >> 1], e & 1), tv = bf2(tw[e >> 1], e & 1);
      const float sv = scale * fast_tanhf(sh);
      yv[e] = a.inverse ? (xs[e] - tv) * __expf(-sv) : fmaf(xs[e], __expf(sv), tv);
    }
#ifdef NF_PROBE_NOSTORE
    dummy += yv[0] + yv[3] + yv[5] + yv[7] + __uint_as_float(su.x);
    continue;
#endif
    float* yr = a.y + (long)m * a.ld_y + f;
    *reinterpret_cast<float4*>(yr) = make_float4(yv[0], yv[1], yv[2], yv[3]);
    *reinterpret_cast<float4*>(yr + 4) = make_float4(yv[4], yv[5], yv[6], yv[7]);
    if (a.yb) {
      uint4 o;
      o.x = (unsigned)f2bf(yv[0]) | ((unsigned)f2bf(yv[1]) << 16);
      o.y = (unsigned)f2bf(yv[2]) | ((unsigned)f2bf(yv[3]) << 16);
      o.z = (unsigned)f2bf(yv[4]) | ((unsigned)f2bf(yv[5]) << 16);
      o.w = (unsigned)f2bf(yv[6]) | ((unsigned)f2bf(yv[7]) << 16);
      *reinterpret_cast<uint4*>(a.yb + (long)m * a.ld_yb + f) = o;
    }
    if (a.st) *reinterpret_cast<v4u*>(a.st + (long)m * a.ld_st + f) = su;
  }
#ifdef NF_PROBE_NOSTORE
  if (a.M < 0) a.y[lane] = dummy;
#endif
  // the bf16 copy's pad columns [Dh, yb_width): zero, by the last column tile
  if (a.yb && tn == a.ntn - 1) {
    const int m = m0 + 64 * wave + lane;
    if (m < a.M)
      for (int c = Dh; c < a.yb_width; c += 8)
        *reinterpret_cast<uint4*>(a.yb + (long)m * a.ld_yb + c) = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace cpl4w

bool launch_cpl4w(const cpl4w::Args& a0, hipStream_t stream) {
  cpl4w::Args a = a0;
  a.ntn = (a.Dh + cpl4w::NFT - 1) / cpl4w::NFT;
  auto al = [](const void* p, int b) { return ((unsigned long)p & (b - 1)) == 0; };
  if (a.M <= 0 || a.K % 128 || a.M % 16 || a.Dh % 8 || a.w_rows < 2 * a.Dh || a.lda % 8 ||
      a.ldw % 8 || !al(a.A, 16) || !al(a.W, 16) || a.ld_x % 4 || a.ld_y % 4 || !al(a.x, 16) ||
      !al(a.y, 16) || (a.st && (a.ld_st % 8 || !al(a.st, 16))) ||
      (a.yb && (a.ld_yb % 8 || !al(a.yb, 16) || a.yb_width % 8 || a.yb_width < a.Dh)) ||
      (a.bias && !al(a.bias, 8)) || a.ldj_rows < a.ntn)
    return false;
  const int ntiles = ((a.M + cpl4w::BM - 1) / cpl4w::BM) * a.ntn;
  hipLaunchKernelGGL(cpl4w::gemm_cpl4w_kernel, dim3(ntiles), dim3(cpl4w::NTHR), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace gemm
}  // namespace nf
