// 256x256 bf16 MFMA GEMM with the CDNA4 8-phase pipelined schedule (gfx950).
//
// Same contract as gemm.hip (C[m][n] = sum_k Aop(m,k) Bop(n,k), fp32 accumulate, fused
// epilogues), used for the M = batch products of the flow conditioners (forward y = x W^T and
// input-gradient dx = dy W, M = 16384 per GPU), where the 128x128 two-barrier loop of gemm.hip
// stalls on the vmcnt(0) its barrier implies (~700 TF at K = 1024).
//
// Geometry: 512 threads = 8 waves as 2 (M) x 4 (N); block tile 256x256, BK = 64; each wave owns
// 128 (M) x 64 (N) = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).
// LDS: 2 K-tile buffers x 4 half-tiles x 16 KiB = 128 KiB (1 block / CU), staged by
// global_load_lds_dwordx4 (2 per thread per half-tile). A K-tile's operands are split into
// half-tiles by their *reader*, so each can be restaged as soon as its own readers are done:
//   A-lo = tile rows {0..63, 128..191}, A-hi = {64..127, 192..255}   (wave row-group wr reads
//          rows wr*128 + [0..63] from A-lo and wr*128 + [64..127] from A-hi)
//   B-lo = tile cols {wc*64 + 0..31}, B-hi = {wc*64 + 32..63}
// Per K-tile, 4 phases, 16 MFMAs (one 64x32 quadrant x K=64) each:
//   r1: read A-lo (8 frags) + B-lo (4)   mfma M0-3 x N0-1      issue half (t+1, B-hi)
//   r2: read B-hi (4)                    mfma M0-3 x N2-3      issue half (t+1, A-hi)
//   r3: read A-hi (8)                    mfma M4-7 x N2-3      issue half (t+2, A-lo)
//   r4: -                                mfma M4-7 x N0-1      issue half (t+2, B-lo)
// i.e. half j of K-tile t is issued at global phase 4t - 5 + j (prologue: 6 halves). Every
// phase ends its read section with a counted `s_waitcnt vmcnt(2*D)` that retires the half
// issued D phases earlier (never vmcnt(0) in the main loop), then raw s_barrier, lgkmcnt(0),
// setprio(1) MFMAs setprio(0), s_barrier (CDNA4 guide §5 "The 256^2 8-phase template").
//   RAW: a half issued at phase q is read at >= q + D + 1 (checked for every half, D = 3, 4).
//   WAR: a slot is restaged >= 2 phases after its last ds_read (the lgkmcnt(0) that retires a
//        lagging wave's reads sits one barrier after the issuing barrier).
// The two wave row-groups run one barrier apart (wr == 1 takes an extra barrier up front), so
// on each SIMD one wave issues its LDS reads / DMA while the other runs MFMAs.
#include "gemm_tile.h"
#include "wgrad_pack.h"
#include "tn_multi.h"
#include "cpl4w.h"

// Diagnostic build only (csrc/build.py --variant stamps -D NF_G256_STAMPS): every block records
// s_memrealtime (100 MHz, chip-global) at body entry, after the prologue wait, after the main
// loop, after issuing the epilogue, and after its stores have drained, into a buffer set with
// torch.ops.vinf.g256_set_stamps (8 slots per block). The shipped library compiles none of it.
#ifdef NF_G256_STAMPS
__device__ unsigned long long* nf_g256_stamp_buf;
#define NF_STAMP(i)                                                                            \
  do {                                                                                         \
    unsigned long long t_;                                                                     \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");             \
    unsigned long long* b_ = nf_g256_stamp_buf;                                                \
    if (threadIdx.x == 0 && b_) b_[((long)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = t_; \
  } while (0)
#else
#define NF_STAMP(i) \
  do {              \
  } while (0)
#endif

namespace nf {
namespace gemm {
namespace g256 {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int HALF_BYTES = 128 * 64 * 2;  // 16 KiB
// LDS ring of half-tiles: half j of K-tile t (h = 4t + j, j = issue order A-lo, B-lo, B-hi,
// A-hi) lives in slot h % NSLOT. Depth D = 4: NSLOT = 8 (two K-tile buffers, 128 KiB), half h
// issued at phase h - 5. Depth D = 4 + X: NSLOT = 8 + X and half h issued X phases earlier
// (h - 5 - X), every RAW / WAR distance unchanged; X = 2 fills the 160 KiB LDS and keeps 7-8
// half-tiles (~120 KiB) in flight instead of 4-5, for the long-K products whose operands miss
// L2 (a quarter of the weight-gradient fetches) and wait out HBM latency.
constexpr int ring_extra(int D) { return D > 4 ? D - 4 : 0; }
constexpr int smem_bytes(int D) { return (8 + ring_extra(D)) * HALF_BYTES; }
// slot order inside a buffer == issue order j
constexpr int H_ALO = 0, H_BLO = 1, H_BHI = 2, H_AHI = 3;

// local row (0..127) of a half-tile -> row of the 256-row block tile
__device__ __forceinline__ int half_row(bool is_a, bool hi, int lr) {
  return is_a ? (lr & 63) + ((lr >> 6) << 7) + (hi ? 64 : 0)
              : ((lr >> 5) << 6) + (lr & 31) + (hi ? 32 : 0);
}

// one 64x32 output quadrant x one K-tile: 16 bf16 16x16x32 MFMAs (8 without the tail's
// second k-step) or 8 e4m3 16x16x128 scaled MFMAs
#define NF_G256_QUAD(IO, JO, FB)                                                                  \
  do {                                                                                            \
    if constexpr (F8) {                                                                           \
      _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                             \
        const v8i fbi = cat16(FB[i][0], FB[i][1]);                                                \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                             \
          acc[IO + i][JO + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(                 \
              fbi, cat16(fa[j][0], fa[j][1]), acc[IO + i][JO + j], 0, 0, 0, 127, 0, 127);          \
      }                                                                                           \
    } else {                                                                                      \
      _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) if (ks == 0 || two)                        \
        _Pragma("unroll") for (int i = 0; i < 2; ++i)                                             \
          _Pragma("unroll") for (int j = 0; j < 4; ++j)                                           \
            acc[IO + i][JO + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                        \
                FB[i][ks], fa[j][ks], acc[IO + i][JO + j], 0, 0, 0);                              \
    }                                                                                             \
  } while (0)

// fragment column i = 0 of a quadrant only (bf16): the coupling forward's edge tile
#define NF_G256_QUAD_I0(IO, JO, FB)                                                                \
  do {                                                                                            \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) if (ks == 0 || two)                          \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                               \
        acc[IO][JO + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[0][ks], fa[j][ks],           \
                                                                  acc[IO][JO + j], 0, 0, 0);      \
  } while (0)

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v8i cat16(v8s lo, v8s hi) {
  const v4i l = __builtin_bit_cast(v4i, lo), h = __builtin_bit_cast(v4i, hi);
  return __builtin_shufflevector(l, h, 0, 1, 2, 3, 4, 5, 6, 7);
}

// EB: bytes per element (2 = bf16, 1 = e4m3); ld, k0, K in elements. A half-tile is 128 rows x
// 128 bytes either way (64 bf16 or 128 e4m3 k-values per row).
// pair_dh > 0 (EPI_CPL_FWD, B operand): tile row c < 128 -> weight row row0/2 + c, c >= 128 ->
// pair_dh + row0/2 + c - 128 (the s_hat and t rows of the same 128 features)
template <bool KMAJOR, int EB = 2>
__device__ __forceinline__ void stage_half(const bf16_t* __restrict__ base, long ld, int row0,
                                           int rows_total, int k0, int K, bool is_a, bool hi,
                                           char* dst, int wave, int lane, int pair_dh = 0) {
  constexpr int CE = 16 / EB;  // elements per 16-B chunk
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;  // 16 x 1 KiB
    const bf16_t* src;
    if (KMAJOR) {
      const int r = piece * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int tc = half_row(is_a, hi, r);
      int gr = pair_dh == 0 ? row0 + tc
                            : (tc < 128 ? (row0 >> 1) + tc : pair_dh + (row0 >> 1) + tc - 128);
      gr = gr < rows_total ? gr : rows_total - 1;
      int gk = k0 + lc * CE;
      gk = gk < K ? gk : K - CE;
      src = (const bf16_t*)((const char*)base + ((long)gr * ld + gk) * EB);
    } else if constexpr (EB == 1) {
      // e4m3, mn-major (the fp8 weight gradients, K = batch): a half is 128 k-rows x 128 m-bytes,
      // 8 k-rows per 1 KiB piece; 16-B chunk cm of k-row kr sits at chunk position
      // cm ^ f8mn_swz(kr) (the read side, read_frag_f8mn, applies the same involution)
      const int kr = piece * 8 + (lane >> 3);
      const int cm = (lane & 7) ^ f8mn_swz(kr);
      int gk = k0 + kr;
      gk = gk < K ? gk : K - 1;
      int gm = row0 + half_row(is_a, hi, cm * 16);
      gm = gm < rows_total ? gm : rows_total - 16;
      src = (const bf16_t*)((const char*)base + (long)gk * ld + gm);
    } else {
      const int kr = piece * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ mn_swz(kr);
      int gk = k0 + kr;
      gk = gk < K ? gk : K - 1;
      int gm = row0 + half_row(is_a, hi, lc * 8);
      gm = gm < rows_total ? gm : rows_total - 8;
      src = base + (long)gk * ld + gm;
    }
    // The DMA in asm, invisible to the compiler's wait-count pass. With the builtin it drains
    // the DMA queue (s_waitcnt vmcnt(0)) before every ds_read_b64_tr_b16 / _tr_b8 of the
    // mn-major operands (12 such drains in the weight-gradient kernel, none before the k-major
    // b128 reads): it cannot tell the slot being filled from the slot being read, so the
    // counted vmcnt ring degenerates to one phase of prefetch. Ordering is the schedule's own
    // counted vmcnt + barriers only (RAW / WAR distances in the header comment). Measured
    // (profiles/r4/asmdma_probe.jsonl): NN product 1782 -> 1612 us, TN 2238 -> 2158 us, NT
    // unchanged.
#ifdef NF_G256_STAMPS   // the stamps build's extra code leaves it in a VGPR otherwise
    const unsigned lds = __builtin_amdgcn_readfirstlane(
        (unsigned)(unsigned long)(LDS_AS char*)(dst + piece * 1024));
#else
    const unsigned lds = (unsigned)(unsigned long)(LDS_AS char*)(dst + piece * 1024);
#endif
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src), "s"(lds) : "memory", "m0");
  }
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void vmwait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

// retire every half issued at phase <= P - D; `cnt` = valid halves issued in (P - D, P]
template <int D>
__device__ __forceinline__ void vmwait_count(int cnt) {
  static_assert(D <= 6, "vmwait table");
  if (cnt >= D) vmwait<2 * D>();
  else if (cnt == 5) vmwait<10>();
  else if (cnt == 4) vmwait<8>();
  else if (cnt == 3) vmwait<6>();
  else if (cnt == 2) vmwait<4>();
  else if (cnt == 1) vmwait<2>();
  else vmwait<0>();
}

// EPI_CPL_FWD epilogue (GemmArgs::cf_*), in NP row passes. Per pass: 1) every wave parks
// bf16(acc + bias) of 128 / NP of its rows x 64 columns in its own LDS region
// (region_of(wave), 16 KiB / NP, the staged-epilogue image); 2) after a block barrier the 512
// threads walk the pass's 256 / NP rows x 128 features, thread = (row of 32, 16-B chunk of 8
// features), reading s_hat from the region of wave (wr, c/64) and t from wave (wr, 2 + c/64).
// NP = 2 lets the persistent kernel stage through the 64 KiB its LDS-DMA stream leaves free.
// F8: e4m3 operands, acc dequantised by f8_sa[0] * f8_sb[weight row] before the bias.
// cf_mode 1 (MAF): see GemmArgs::cf_mode; the e4m3 copy of u (f8_cq) is quantised from fp32 u.
template <int NP, bool F8 = false, typename RegionFn>
__device__ __forceinline__ void epi_coupling_fwd(const GemmArgs& a, const v4f (&acc)[4][8],
                                                 int m0, int n0, int wr, int wc,
                                                 RegionFn region_of, int lane, int tid_in = -1) {
  constexpr int RJ = 8 / NP, RROWS = 16 * RJ, ITS = 8 / NP;
  const int g = lane >> 4, c = lane & 15;
  const int j0 = n0 >> 1, tn = n0 / BN;
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, f8 = tid & 15, rsub = tid >> 4;
  const int ws = f8 >> 3, q = f8 & 7;
  const int jf = j0 + f8 * 8;                                    // first of this thread's 8 features
  const bool fok = jf < a.cf_dh;
  const bool maf = a.cf_mode != 0;
  // timing probes (docs/PERF_NOTES.md round 6, "MAF forward epilogue"; wrong results):
  // NF_PROBE_CF_NOSTORE drops the global stores, NF_PROBE_CF_NOXLOAD the x reads,
  // NF_PROBE_CF_NOEPI the whole epilogue (the accumulators kept live by one test)
#ifdef NF_PROBE_CF_NOSTORE
  const bool st_on = a.cf_scale == 1.2345e-30f;
#else
  constexpr bool st_on = true;
#endif
#ifdef NF_PROBE_CF_NOXLOAD
  constexpr bool xl_on = false;
#else
  constexpr bool xl_on = true;
#endif
#ifdef NF_PROBE_CF_NOEPI
  {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 1.2345e-30f) a.cf_y[tid] = s;
    return;
  }
#endif
  // bias (and e4m3 dequantisation scale) of the 4 columns of fragment i. AT_USE: read per pass,
  // ahead of the pass's x loads (held across the whole epilogue they spilled the e4m3 and
  // one-pass builds); otherwise (the persistent bf16 form) read once up front.
  constexpr bool AT_USE = F8 || NP == 1;
  // raw per fragment i: bias bits (4 bf16 in 2 dwords) and, e4m3, the 4 weight-row scales
  // (times f8_sa[0] at the use); kept packed so the per-pass preload stays small
  unsigned bq[4][2];
  float4 sq[4];
  auto col_params = [&](int i) {
    bq[i][0] = bq[i][1] = 0u;
    sq[i] = make_float4(1.f, 1.f, 1.f, 1.f);
#ifdef NF_PROBE_CF_NOCOLP   // timing probe: no bias / scale loads in the parking loop
    return;
#endif
    const int tc = wc * 64 + i * 16 + g * 4;                     // tile column (4 consecutive)
    const int f = j0 + (tc & 127);                               // feature
    const int row = tc < 128 ? f : a.cf_pair + f;                // weight / bias row
    if (a.bias && f < a.cf_dh) {
      const uint2 bb = *reinterpret_cast<const uint2*>(a.bias + row);
      bq[i][0] = bb.x; bq[i][1] = bb.y;
    }
    if constexpr (F8) {
      sq[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < a.cf_dh) sq[i] = *reinterpret_cast<const float4*>(a.f8_sb + row);
    }
  };
  float bpre[4][4];   // !AT_USE (persistent bf16): the bias as floats, converted once
  if constexpr (!AT_USE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      col_params(i);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        bpre[i][2 * e] = __uint_as_float(bq[i][e] << 16);
        bpre[i][2 * e + 1] = __uint_as_float(bq[i][e] & 0xffff0000u);
      }
    }
  }
  float qinv = 1.f, qamax = 0.f;
  if (a.f8_cq) {
    const float ap = *a.f8_q_amax_prev;
    const float qs = ap > 0.f ? ap / 448.f : 1.f;
    qinv = 1.f / qs;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.f8_q_scale_out = qs;
  }
  char* region = region_of(wr * 4 + wc);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (p) barrier();   // every wave's readback of the previous pass is done (its values were used)
    // AT_USE: the pass's bias / scale loads go out BEFORE its x loads. vmcnt retires in issue
    // order, so loaded at their use (inside the parking loop, behind the x loads) their first
    // wait also waited out every x row: the x round trip sat in front of the parking instead
    // of under it (e4m3 MAF forward 163 -> 139 us per call without those loads,
    // profiles/r6/maf_fwd_colparams_probe.txt)
    if constexpr (AT_USE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) col_params(i);
    }
    // this pass's x rows / previous log-det partials fetched up front: all in flight while the
    // accumulators are parked (the epilogue runs on every CU at once, so a load round trip per
    // row pair would sit exposed after the main loop)
    float4 xv[ITS][2];
    float lold[ITS];
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int lrow = it * 32 + rsub, wrr = lrow / RROWS, r = lrow % RROWS;
      const int m = m0 + wrr * 128 + p * RROWS + r;
      xv[it][0] = xv[it][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      lold[it] = 0.f;
      if (m < a.M && fok && xl_on) {
        if (a.cf_x_bf16) {   // 8 bf16 in xv[it][0]'s bits, expanded at the use
          const bf16_t* xr = reinterpret_cast<const bf16_t*>(a.cf_x) + (long)m * a.ld_cf_x + jf;
          xv[it][0] = __builtin_bit_cast(float4, *reinterpret_cast<const uint4*>(xr));
        } else {
          const float* xr = a.cf_x + (long)m * a.ld_cf_x + jf;
          xv[it][0] = *reinterpret_cast<const float4*>(xr);
          xv[it][1] = *reinterpret_cast<const float4*>(xr + 4);
        }
      }
      if (!a.cf_ldj_init && f8 == 0 && m < a.M) lold[it] = a.cf_ldj[(long)tn * a.ld_cf_ldj + m];
    }
#pragma unroll
    for (int jj = 0; jj < RJ; ++jj) {
      const int j = p * RJ + jj;
      const int row = jj * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float bv[4];
        if constexpr (AT_USE) {
          bv[0] = __uint_as_float(bq[i][0] << 16);
          bv[1] = __uint_as_float(bq[i][0] & 0xffff0000u);
          bv[2] = __uint_as_float(bq[i][1] << 16);
          bv[3] = __uint_as_float(bq[i][1] & 0xffff0000u);
        } else {
          bv[0] = bpre[i][0]; bv[1] = bpre[i][1]; bv[2] = bpre[i][2]; bv[3] = bpre[i][3];
        }
        float sv[4] = {1.f, 1.f, 1.f, 1.f};
        if constexpr (F8) {
          const float sa = a.f8_sa[0];
          sv[0] = sa * sq[i].x; sv[1] = sa * sq[i].y; sv[2] = sa * sq[i].z; sv[3] = sa * sq[i].w;
        }
        const unsigned lo = (unsigned)f2bf(fmaf(acc[i][j][0], sv[0], bv[0])) |
                            ((unsigned)f2bf(fmaf(acc[i][j][1], sv[1], bv[1])) << 16);
        const unsigned hi = (unsigned)f2bf(fmaf(acc[i][j][2], sv[2], bv[2])) |
                            ((unsigned)f2bf(fmaf(acc[i][j][3], sv[3], bv[3])) << 16);
        const int slot = i * 4 + g;
        *(LDS_AS v2u*)(region + bf_stage_off(row, slot)) = (v2u){lo, hi};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int lrow = it * 32 + rsub, wrr = lrow / RROWS, r = lrow % RROWS;
      const int m = m0 + wrr * 128 + p * RROWS + r;
      float part = 0.f;
      if (m < a.M) {
        if (fok) {
          const int off = r * 128 + ((q ^ (r & 7)) << 4);
          const bool swp = (r >> 3) & 1;   // bf_stage_off's half swap
          const v4u sh = bf_stage_fix(*(const LDS_AS v4u*)(region_of(wrr * 4 + ws) + off), swp);
          const v4u tt = bf_stage_fix(*(const LDS_AS v4u*)(region_of(wrr * 4 + 2 + ws) + off), swp);
          const float4 x0 = xv[it][0], x1 = xv[it][1];
          float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          if (a.cf_x_bf16) {
            const uint4 xb = __builtin_bit_cast(uint4, x0);
            const unsigned w4[4] = {xb.x, xb.y, xb.z, xb.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              xs[2 * e] = __uint_as_float(w4[e] << 16);
              xs[2 * e + 1] = __uint_as_float(w4[e] & 0xffff0000u);
            }
          }
          float y[8];
          if (maf) {   // shv = s_raw, tv = mu
            const float ib = __builtin_amdgcn_rcpf(a.cf_scale);   // v_rcp, not an IEEE division per row
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const unsigned us = sh[e >> 1], ut = tt[e >> 1];
              const float shv = __uint_as_float((e & 1) ? (us & 0xffff0000u) : (us << 16));
              const float tv = __uint_as_float((e & 1) ? (ut & 0xffff0000u) : (ut << 16));
              const float al = a.cf_scale * fast_tanhf(shv * ib);
              y[e] = (xs[e] - tv) * __expf(-al);
              part -= al;
            }
          } else if (a.cf_inverse) {   // x = (y - t) e^-s, ldj share -sum s
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const unsigned us = sh[e >> 1], ut = tt[e >> 1];
              const float shv = __uint_as_float((e & 1) ? (us & 0xffff0000u) : (us << 16));
              const float tv = __uint_as_float((e & 1) ? (ut & 0xffff0000u) : (ut << 16));
              const float sv = a.cf_scale * fast_tanhf(shv);
              y[e] = (xs[e] - tv) * __expf(-sv);
              part -= sv;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const unsigned us = sh[e >> 1], ut = tt[e >> 1];
              const float shv = __uint_as_float((e & 1) ? (us & 0xffff0000u) : (us << 16));
              const float tv = __uint_as_float((e & 1) ? (ut & 0xffff0000u) : (ut << 16));
              const float sv = a.cf_scale * fast_tanhf(shv);
              y[e] = fmaf(xs[e], __expf(sv), tv);
              part += sv;
            }
          }
          if (a.f8_cq && st_on) {   // e4m3 copy of y (the next fp8 product's operand), delayed scale
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              qamax = fmaxf(qamax, fabsf(y[e]));
              f[e] = fminf(fmaxf(y[e] * qinv, -448.f), 448.f);
            }
            int q0 = 0, q1 = 0;
            q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], q0, false);
            q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], q0, true);
            q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], q1, false);
            q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], q1, true);
            *reinterpret_cast<uint2*>(a.f8_cq + (long)m * a.ld_f8_cq + jf) =
                make_uint2((unsigned)q0, (unsigned)q1);
          }
          float* yr = a.cf_y + (long)m * a.ld_cf_y + jf;
          if (st_on && a.cf_y) {
            *reinterpret_cast<float4*>(yr) = make_float4(y[0], y[1], y[2], y[3]);
            *reinterpret_cast<float4*>(yr + 4) = make_float4(y[4], y[5], y[6], y[7]);
          }
          if (a.cf_yb && st_on) {
            uint4 o;
            o.x = (unsigned)f2bf(y[0]) | ((unsigned)f2bf(y[1]) << 16);
            o.y = (unsigned)f2bf(y[2]) | ((unsigned)f2bf(y[3]) << 16);
            o.z = (unsigned)f2bf(y[4]) | ((unsigned)f2bf(y[5]) << 16);
            o.w = (unsigned)f2bf(y[6]) | ((unsigned)f2bf(y[7]) << 16);
            *reinterpret_cast<uint4*>(a.cf_yb + (long)m * a.ld_cf_yb + jf) = o;
          }
          if (a.C && st_on)
            *reinterpret_cast<uint4*>((bf16_t*)a.C + (long)m * a.ldc + jf) =
                make_uint4(sh[0], sh[1], sh[2], sh[3]);
        } else if (a.cf_yb && jf < a.cf_yb_width) {   // zero the next operand's pad columns
          *reinterpret_cast<uint4*>(a.cf_yb + (long)m * a.ld_cf_yb + jf) = make_uint4(0, 0, 0, 0);
        }
      }
      // sum of s over this block's 128 features: the 16 threads of a row are 16 adjacent lanes
      part += __shfl_xor(part, 8);
      part += __shfl_xor(part, 4);
      part += __shfl_xor(part, 2);
      part += __shfl_xor(part, 1);
      if (f8 == 0 && m < a.M) {
        float* lp = a.cf_ldj + (long)tn * a.ld_cf_ldj + m;
        *lp = part + lold[it];
      }
    }
  }
  if (a.f8_cq) {   // one (mostly skipped) atomic per wave into the block's amax slot
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) qamax = fmaxf(qamax, __shfl_xor(qamax, off));
    if (lane == 0) amax_slot_atomic(a.f8_q_amax_cur, qamax);
  }
}

// F8: e4m3 operands (both k-major), one v_mfma_scale_f32_16x16x128_f8f6f4 per (i, j) and K-tile
// of 128 bytes in place of the two bf16 16x16x32 steps - the same LDS image and fragment reads
// (a lane's 32 k-bytes are the chunks g and g + 4 the bf16 steps read), 2x the FLOPs per
// MFMA cycle; block scales fixed at 2^0, the per-row / per-tensor scales applied in the epilogue.
template <bool A_KMAJOR, bool B_KMAJOR, int EPI, int D, bool DB, bool F8, bool DODB>
__device__ __forceinline__ void gemm256_body_impl(const GemmArgs& a, int wg, int split,
                                                  char* smem) {
  constexpr int BKE = F8 ? 2 * BK : BK;  // K-tile in elements
  constexpr int EB = F8 ? 1 : 2;
  constexpr int X = ring_extra(D), NSLOT = 8 + X;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int ntn = (a.N + BN - 1) / BN;
  const int tm = wg / ntn, tn = wg % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  int kbeg = split * a.k_per_split;
  int kend = kbeg + a.k_per_split;
  kend = kend < a.K ? kend : a.K;
  // optional second K segment [kbeg2, kend2) streamed after the first (K-tiles n1 .. nkt-1):
  // a MADE mask over a [mu | s] output pair is non-zero on one range in EACH half
  int kbeg2 = 0, kend2 = 0, n2 = 0;
  if (a.krange) {  // MADE weights: stream only the K-tiles where this N-tile's mask is non-zero
    const int segs = a.krange_segs == 2 ? 2 : 1;
    const int* r = a.krange + 2 * segs * tn;
    const int lo = (r[0] / BKE) * BKE, hi = r[1];
    kbeg = kbeg > lo ? kbeg : lo;
    kend = kend < hi ? kend : hi;
    if (F8 && kend > kbeg) {  // whole 128-byte K-tiles (the extra columns hold zero weights)
      kend = kbeg + ((kend - kbeg + BKE - 1) / BKE) * BKE;
      kend = kend < a.K ? kend : a.K;
    }
    if (segs == 2 && r[3] > r[2]) {  // (split-K is not combined with two segments)
      kbeg2 = (r[2] / BKE) * BKE;
      kend2 = r[3] < a.K ? r[3] : a.K;
      if (F8) {
        kend2 = kbeg2 + ((kend2 - kbeg2 + BKE - 1) / BKE) * BKE;
        kend2 = kend2 < a.K ? kend2 : a.K;
      }
      n2 = (kend2 - kbeg2 + BKE - 1) / BKE;
    }
  }
  const int n1 = kend > kbeg ? (kend - kbeg + BKE - 1) / BKE : 0;
  int nkt = n1 + n2;
  if (a.skip && a.skip[tm * ntn + tn] && !(DB && a.dbias != nullptr && tn == 0)) nkt = 0;

  v4f acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  // bias gradient db[m] = sum_k Aop(m,k) (weight-gradient launches, tn == 0 blocks: the DODB
  // instantiation). Wave wc sums A fragment j == wc of each A half - already in registers for
  // the MFMAs, 8 consecutive k of row (lane & 15) per k-step - with v_dot2_f32_bf16 against a
  // (1, 1) literal: 4 VALU per k-step in the MFMA shadow, no extra registers, LDS reads or
  // MFMAs (the former ones-fragment MFMA held 20 VGPRs, which spilled the 10-slot ring build).
  // The wave-uniform switch picks the fragment once per half (indexing fa[wc] per instruction
  // compiled to a branch ladder). dbs[h]: partial over this lane's k chunks; lanes are reduced
  // over (lane >> 4) in the epilogue.
  // (e4m3 weight gradients: the bias sums would spill the loop; fp8_colsum computes them)
  constexpr bool do_db = DODB && !F8;
  v8s fa[4][2], fbl[2][2], fbh[2][2];
  float dbs[2] = {0.f, 0.f};
  auto db_sum = [&](float& sacc, bool two_) {
    typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
    const v2bf one = {(__bf16)1.0f, (__bf16)1.0f};
    auto add = [&](const v8s (&f)[2]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 1 && !two_) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned w = (unsigned)(unsigned short)f[ks][2 * e] |
                             ((unsigned)(unsigned short)f[ks][2 * e + 1] << 16);
          sacc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, w), one, sacc, false);
        }
      }
    };
    switch (wc) {
      case 0: add(fa[0]); break;
      case 1: add(fa[1]); break;
      case 2: add(fa[2]); break;
      default: add(fa[3]); break;
    }
  };

  auto slot = [&](int t, int j) { return smem + ((4 * t + j) % NSLOT) * HALF_BYTES; };
  // issue half j of K-tile t (no-op past the end)
  auto issue = [&](int t, int j) {
    if (t >= nkt) return;
    char* dst = slot(t, j);
    const bool s2 = t >= n1;
    const int k0 = s2 ? kbeg2 + (t - n1) * BKE : kbeg + t * BKE;
    const int ke = s2 ? kend2 : kend;
    if (j == H_ALO || j == H_AHI)
      stage_half<A_KMAJOR, EB>(a.A, a.lda, m0, a.M, k0, ke, true, j == H_AHI, dst, wave, lane);
    else if constexpr (EPI == EPI_CPL_FWD)
      stage_half<B_KMAJOR, EB>(a.B, a.ldb, n0, a.cf_b_rows, k0, ke, false, j == H_BHI, dst, wave,
                               lane, a.cf_pair);
    else
      stage_half<B_KMAJOR, EB>(a.B, a.ldb, n0, a.N, k0, ke, false, j == H_BHI, dst, wave, lane);
  };
  auto issue_h = [&](int h) { issue(h >> 2, h & 3); };
  // valid halves issued at global phases (P - D, P]; half (t, j) is issued at 4t - 5 - X + j
  auto outstanding = [&](int P) {
    const int last = 4 * nkt - 6 - X;
    int hi = P < last ? P : last;
    int c = hi - (P - D);
    return c < 0 ? 0 : (c > D ? D : c);
  };

  NF_STAMP(0);
  if (nkt > 0) {
#pragma unroll
    for (int h = 0; h < 6 + X; ++h) issue_h(h);   // every half issued at phase <= 0
    vmwait_count<D>(outstanding(0));
    barrier();
    NF_STAMP(1);
    if (wr == 1) barrier();

    // One K-tile (4 phases). STEADY: every half this K-tile issues exists (t + 2 < nkt) and
    // the K-tile is a whole 64-deep step, so the issue bound checks, the runtime vmcnt ladder
    // and the tail branch inside the MFMA cluster all fold away (straight-line phases with a
    // fixed vmcnt(2D)); the generic form runs the last two K-tiles.
    auto ktile = [&](int t, auto steady_c) {
      constexpr bool S = decltype(steady_c)::value;
      const bool two = S || F8 ||
                       (t >= n1 ? (kend2 - (kbeg2 + (t - n1) * BK)) > 32
                                : (kend - (kbeg + t * BK)) > 32);
      const int P = 4 * t;
      auto issue_wait = [&](int h, int p) {
        if constexpr (S) {
          issue(h >> 2, h & 3);
          vmwait<2 * D>();
        } else {
          issue_h(h);
          vmwait_count<D>(outstanding(p));
        }
      };
      // ---- r1: M0-3 x N0-1
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fbl[i][ks] = read_frag_any<B_KMAJOR, F8>(slot(t, H_BLO), wc * 32 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fa[j][ks] = read_frag_any<A_KMAJOR, F8>(slot(t, H_ALO), wr * 64 + j * 16, ks, lane);
      issue_wait(4 * t + 6 + X, P + 1);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      NF_G256_QUAD(0, 0, fbl);
      if constexpr (do_db) db_sum(dbs[0], two);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- r2: M0-3 x N2-3
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fbh[i][ks] = read_frag_any<B_KMAJOR, F8>(slot(t, H_BHI), wc * 32 + i * 16, ks, lane);
      issue_wait(4 * t + 7 + X, P + 2);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      NF_G256_QUAD(2, 0, fbh);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- r3: M4-7 x N2-3
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fa[j][ks] = read_frag_any<A_KMAJOR, F8>(slot(t, H_AHI), wr * 64 + j * 16, ks, lane);
      issue_wait(4 * t + 8 + X, P + 3);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      NF_G256_QUAD(2, 4, fbh);
      if constexpr (do_db) db_sum(dbs[1], two);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- r4: M4-7 x N0-1 (no LDS reads)
      issue_wait(4 * t + 9 + X, P + 4);
      barrier();
      __builtin_amdgcn_s_setprio(1);
      NF_G256_QUAD(0, 4, fbl);
      __builtin_amdgcn_s_setprio(0);
      barrier();
    };
    // steady K-tiles: t + 2 < nkt, and (two K segments) not the first segment's last K-tile,
    // whose second 32-deep step may be absent
    int nsteady = nkt - 2;
    if (n2 > 0 && nsteady > n1 - 1) nsteady = n1 - 1;
    int t = 0;
    for (; t < nsteady; ++t) ktile(t, std::true_type{});
    for (; t < nkt; ++t) ktile(t, std::false_type{});
    if (wr == 0) barrier();
  }
  NF_STAMP(2);

  // ---------------------------------------------------------------- epilogue
  // acc[i][j]: n = n0 + wc*64 + i*16 + (lane>>4)*4 + r, m = m0 + wr*128 + j*16 + (lane&15)
  // lane-derived epilogue offsets from an opaque zero, so they are computed here: hoisted
  // above the K loop they stayed live across it at the 256-VGPR limit and were spilled
  int zt;
  asm volatile("s_mov_b32 %0, 0" : "=s"(zt));
  const int lane_e = lane + zt, tid_e = wave * 64 + lane_e;   // not v0: keeps it dead
  const int g = lane_e >> 4, c = lane_e & 15;
  if (do_db && a.dbias != nullptr) {   // dbs[h]: m = wr*128 + h*64 + wc*16 + (lane & 15)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v = dbs[h];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = m0 + wr * 128 + h * 64 + wc * 16 + c;
      if (g == 0 && m < a.M) a.dbias[(long)split * a.M + m] = v;
    }
  }
  if constexpr (EPI == EPI_CPL_FWD) {
    barrier();  // every wave is past its last operand read
    // e4m3 operands: two 64-row passes (half the x rows in flight) - the F8 main loop leaves
    // fewer registers, and one pass spilled (scratch 120 B/lane)
    epi_coupling_fwd<F8 ? 2 : 1, F8>(a, acc, m0, n0, wr, wc,
                                     [&](int w) { return smem + w * 16384; }, lane_e, tid_e);
#ifdef NF_G256_STAMPS
    NF_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    NF_STAMP(4);
#endif
    return;
  }
  if (a.staged) {
    barrier();  // every wave is past its last operand read; each wave reuses 16 KiB of LDS
    epi_tile_staged<EPI, 8, F8>(a, acc, m0 + wr * 128, n0 + wc * 64, split, smem + wave * 16384,
                                lane_e);
#ifdef NF_G256_STAMPS
    NF_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    NF_STAMP(4);
#endif
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = m0 + wr * 128 + j * 16 + c;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wc * 64 + i * 16 + g * 4;
      if (n >= a.N) continue;
      epi_store<EPI>(a, acc[i][j], m, n, split);
    }
  }
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI, int D, bool DB, bool F8 = false>
__device__ __forceinline__ void gemm256_body(const GemmArgs& a, int wg, int split, char* smem) {
  if constexpr (DB) {
    const int ntn = (a.N + BN - 1) / BN;
    if (a.dbias != nullptr && wg % ntn == 0) {
      gemm256_body_impl<A_KMAJOR, B_KMAJOR, EPI, D, DB, F8, true>(a, wg, split, smem);
      return;
    }
  }
  gemm256_body_impl<A_KMAJOR, B_KMAJOR, EPI, D, DB, F8, false>(a, wg, split, smem);
}

// ---------------------------------------------------------------------------------------------
// Persistent form for the plain products (no K ranges, no split-K, no bias gradient): grid =
// min(tiles, CUs) blocks of the same 8-phase schedule; block b computes tiles b, b + G, ...
// (XCD-remapped ids, so a block's tiles stay in its XCD's contiguous id range). The K-tiles of
// all of a block's tiles form ONE LDS-DMA stream (half h of the stream is issued at phase h - 5
// and lives in ring slot h % 8, exactly as inside one tile), so when a tile's last K-tile is
// done the next tile's first six half-tiles are already in flight: its prologue burst and the
// block turnover of the one-tile-per-block launch (~1.8 + 2.1 us per tile,
// profiles/r2_g256_stamps_b65536.jsonl) are gone, and the epilogue is the only per-tile cost
// outside the MFMA loop.
// LDS at a tile boundary (last K-tile T): halves 4T+4 .. 4T+9 are live in their slots; the slots
// of the last K-tile's B-hi / A-hi halves ((4T+2) % 8, (4T+3) % 8: read in its phases r2 / r3,
// restaged only in phases 1 / 2 of the next tile) and the 32 KiB above the ring are free.
// The epilogue stages through them: 8 KiB per wave (waves 0-3 in the free slot pair, 4-7 above
// the ring), i.e. bf16 outputs in two 64-row passes, fp32 outputs in their usual 32-row
// passes. WAR on the slot pair: every wave's staging reads are consumed by its own stores
// before the barrier that ends the epilogue, and the DMA into those slots is issued after it.
//
// DYN (persist mode 2): the same body with tiles CLAIMED at run time instead of the fixed list
// b, b + G, ...: XCD x's tiles (xcd_remap's contiguous range) are handed out by counter
// a.qctr[x]; a block claims from its own XCD's counter only. A block that
// starts late (its CU held by an RCCL kernel beside the backward) then takes fewer tiles, where a
// fixed list would hold the whole launch until it ran. One lane claims (QL: wave 3, lane 0),
// and claim latency stays off the critical path: tile s + 1 is claimed at the start of tile
// s - 1's epilogue and resolved after that epilogue's own vmcnt(0). LDS is full (ring + staging),
// so the id is published at the end of QL's own staging region (slot (4T + 7) % 8, T = the next
// tile's first stream K-tile), which nothing touches between the epilogue-ending barrier and
// the next tile's phase-2 DMA into that slot; every wave reads it at the loop top, before its
// first barrier of the tile (read + readfirstlane: complete before any wave can issue that DMA).
// A block's first tile is not claimed: XCD x's first nbx tiles belong to its nbx blocks in block
// order and the counter hands out the rest, so no claim round trip is ever exposed (a block that
// starts late delays one tile, not a list). Every block increments the done counter once, as it
// finishes; the last one zeroes the slot for the next launch that uses it. No block ever waits
// on another (no spin), so the grid always drains.
template <bool A_KMAJOR, bool B_KMAJOR, int EPI, bool DYN = false>
__device__ __forceinline__ void gemm256_persistent_body(const GemmArgs& a, char* smem) {
  static_assert(!(DYN && EPI == EPI_CPL_FWD), "the coupling forward reads other waves' staging");
  constexpr int D = 4, NSLOT = 8;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  const int G = gridDim.x, b = blockIdx.x;
  const int ns = DYN ? 0x7fffffff : (ntiles - b + G - 1) / G;   // tiles of this block
  // DYN claims (lane QL only)
  constexpr int QL = 192;
  auto qaddr = [&](int T_) {   // tile id published for the tile starting at stream K-tile T_
    return (volatile LDS_AS int*)(LDS_AS char*)(smem + ((4 * T_ + 7) & (NSLOT - 1)) * HALF_BYTES +
                                                 HALF_BYTES - 16);
  };
  // one lane's claim: the VGPR offset the compiler cannot see is zero keeps the atomic optimizer
  // from turning it into a wave-wide broadcast that waits for the result (vmcnt(0)) on the spot
  auto claim_add = [&](int x) {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return atomicAdd(a.qctr + x * QCTR_LINE + z, 1);
  };
  const int xcd = b & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
  auto xcount = [&](int x) { return x < r8 ? q8 + 1 : q8; };
  auto xbase = [&](int x) { return x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8; };
  // DYN: the XCD's first nbx tiles are the first tiles of its nbx blocks (block b = xcd + 8 i
  // takes tile i unclaimed); the counter hands out the rest
  const int nbx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);
  // tile id for the own-XCD claim `raw`; -1: the XCD's tiles are all taken (no stealing across
  // XCDs: RCCL's blocks spread over every XCD, and the claim code must stay register-cheap)
  auto resolve = [&](int raw) -> int {
    return raw + nbx < xcount(xcd) ? xbase(xcd) + raw + nbx : -1;
  };
  auto finished = [&](int old) {   // old: this block's pre-increment value of the done counter
    if (old == G - 1)
#pragma unroll
      for (int x = 0; x < 9; ++x) atomicExch(a.qctr + x * QCTR_LINE, 0);
  };
  const int nkt = (a.K + BK - 1) / BK;              // K-tiles per tile
  // Column rotation: with every block holding the same number of tiles and each XCD's step-s
  // ids a run of whole tile rows, block b's s-th tile takes column (tn + s) % ntn - still one
  // tile per (row, column) per step, same rows in flight per XCD, but every block now meets
  // each column tile once. Without it the blocks whose ids sit on the last column get ALL of
  // its cheap edge tiles (the coupling products' 8-feature / 136-column remainders) and the
  // others all of the full ones, and the launch lasts as long as the full-tile blocks.
  const bool rot = (G & 7) == 0 && ntiles % G == 0 && ((ntiles >> 3) % ntn) == 0 &&
                   ((G >> 3) % ntn) == 0;
  auto tile_org = [&](int s, int& m0, int& n0) {
    const int id = xcd_remap(b + s * G, ntiles);
    m0 = (id / ntn) * BM;
    n0 = (rot ? (id % ntn + s) % ntn : id % ntn) * BN;
  };
  auto tile_at = [&](int id, int& m0, int& n0) {   // DYN: claimed tile id
    m0 = (id / ntn) * BM;
    n0 = (id % ntn) * BN;
  };
  // stage half j of K-tile tk of the tile at (tm0, tn0) into the ring slot of stream half
  // 4 Tg + j
  auto issue_to = [&](int Tg, int tm0, int tn0, int tk, int j) {
    char* dst = smem + ((4 * Tg + j) & (NSLOT - 1)) * HALF_BYTES;
    const int k0 = tk * BK;
    if (j == H_ALO || j == H_AHI)
      stage_half<A_KMAJOR>(a.A, a.lda, tm0, a.M, k0, a.K, true, j == H_AHI, dst, wave, lane);
    else if constexpr (EPI == EPI_CPL_FWD)
      stage_half<B_KMAJOR>(a.B, a.ldb, tn0, a.cf_b_rows, k0, a.K, false, j == H_BHI, dst, wave,
                           lane, a.cf_pair);
    else
      stage_half<B_KMAJOR>(a.B, a.ldb, tn0, a.N, k0, a.K, false, j == H_BHI, dst, wave, lane);
  };

  v4f acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  v8s fa[4][2], fbl[2][2], fbh[2][2];

  // One K-tile (stream index T, index t in its tile) of the 8-phase schedule. Phase q issues
  // half 4T + 5 + q of the schedule: (t+1, B-hi), (t+1, A-hi), (t+2, A-lo), (t+2, B-lo) - only
  // while those are K-tiles of this tile. The next tile's first six halves are issued in one
  // burst at the tile boundary instead (they land during the epilogue), so the tile's last
  // K-tiles issue less and retire by the counts of the one-tile schedule's tail:
  //   MODE 0: t + 2 < nkt, four issues, vmcnt(2D) each phase (branch-free)
  //   MODE 1: t = nkt - 2, issues in phases 1-2, then vmcnt 6 / 4
  //   MODE 2: t = nkt - 1, no issues, vmcnt 2 / 0 / 0 / 0
  // FULL: the K-tile has both 32-deep k-steps (false only on a tile's last K-tile when
  //       K % 64 == 32, then `two` is the runtime answer).
  // EDGE (EPI_CPL_FWD tiles holding <= 16 features, e.g. the last 8 of Dh = 392): only the
  // s / t columns 0..15 and 128..143 are real, i.e. fragment 0 of the B-lo half of waves wc = 0
  // and 2; every other MFMA (and the B-hi fragment reads) of the tile is skipped. The DMA
  // stream, barriers and waits are the full tile's, so the ring schedule is unchanged.
  auto ktile = [&](int T, int t, int m0, int n0, bool two_rt, auto mode_c, auto full_c,
                   auto edge_c) {
    constexpr int MODE = decltype(mode_c)::value;
    constexpr bool E = decltype(edge_c)::value;
    const bool two = decltype(full_c)::value || two_rt;
    const bool e_act = (wc & 1) == 0;
    constexpr bool F8 = false;
    auto slot = [&](int j) { return smem + ((4 * T + j) & (NSLOT - 1)) * HALF_BYTES; };
    auto issue_wait = [&](auto q_c) {   // q = 1..4
      constexpr int q = decltype(q_c)::value;
      constexpr int j = q == 1 ? H_BHI : q == 2 ? H_AHI : q == 3 ? H_ALO : H_BLO;
      if constexpr (MODE == 0 || (MODE == 1 && q <= 2)) {
        issue_to(q <= 2 ? T + 1 : T + 2, m0, n0, q <= 2 ? t + 1 : t + 2, j);
        vmwait<2 * D>();
      } else if constexpr (MODE == 1) {
        vmwait<q == 3 ? 6 : 4>();
      } else {
        vmwait<q == 1 ? 2 : 0>();
      }
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fbl[i][ks] = read_frag<B_KMAJOR>(slot(H_BLO), wc * 32 + i * 16, ks, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fa[j][ks] = read_frag<A_KMAJOR>(slot(H_ALO), wr * 64 + j * 16, ks, lane);
    issue_wait(std::integral_constant<int, 1>{});
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if constexpr (E) {
      if (e_act) NF_G256_QUAD_I0(0, 0, fbl);
    } else {
      NF_G256_QUAD(0, 0, fbl);
    }
    __builtin_amdgcn_s_setprio(0);
    barrier();
    if constexpr (!E) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fbh[i][ks] = read_frag<B_KMAJOR>(slot(H_BHI), wc * 32 + i * 16, ks, lane);
    }
    issue_wait(std::integral_constant<int, 2>{});
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!E) NF_G256_QUAD(2, 0, fbh);
    __builtin_amdgcn_s_setprio(0);
    barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fa[j][ks] = read_frag<A_KMAJOR>(slot(H_AHI), wr * 64 + j * 16, ks, lane);
    issue_wait(std::integral_constant<int, 3>{});
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!E) NF_G256_QUAD(2, 4, fbh);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    issue_wait(std::integral_constant<int, 4>{});
    barrier();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (E) {
      if (e_act) NF_G256_QUAD_I0(0, 4, fbl);
    } else {
      NF_G256_QUAD(0, 4, fbl);
    }
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };

  if (ns <= 0) return;
  int m0, n0;
  int raw = 0;   // DYN, lane QL: the claim in flight (own-XCD counter value or done count)
  if constexpr (DYN) {
    // the first tile is static (see nbx): its DMA is issued at once, with tile 1's claim in
    // flight beside it, so no claim round trip precedes the block's first operand
    const int bi = b >> 3;
    const int id0 = bi < xcount(xcd) ? xbase(xcd) + bi : -1;
    if (id0 < 0) {   // (G <= ntiles: not taken; the done count must still reach G)
      if (threadIdx.x == QL) finished(claim_add(8));
      return;
    }
    if (threadIdx.x == QL) raw = claim_add(xcd);   // tile 1, resolved after the prologue's DMA wait
    tile_at(id0, m0, n0);
  } else {
    tile_org(0, m0, n0);
  }
  // prologue: the stream's first six halves (K-tile 0, and K-tile 1's A-lo / B-lo; nkt >= 2)
#pragma unroll
  for (int h = 0; h < 6; ++h) issue_to(h >> 2, m0, n0, h >> 2, h & 3);
  vmwait<0>();
  if constexpr (DYN) {
    if (threadIdx.x == QL) *qaddr(0) = resolve(raw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  barrier();
  const bool tail_half = (a.K - (nkt - 1) * BK) <= 32;   // a tile's last K-tile has one k-step
  int T = 0;
  for (int s = 0; s < ns; ++s) {
    // DYN: tile s + 1's id, published before tile s began (prologue / the previous epilogue)
    const int id_next = DYN ? __builtin_amdgcn_readfirstlane(*qaddr(T)) : 0;
    const bool has_next = DYN ? id_next >= 0 : s + 1 < ns;
    if (wr == 1) barrier();
    auto tile_loop = [&](auto edge_c) {
      for (int t = 0; t < nkt - 2; ++t, ++T)
        ktile(T, t, m0, n0, true, std::integral_constant<int, 0>{}, std::true_type{}, edge_c);
      ktile(T, nkt - 2, m0, n0, true, std::integral_constant<int, 1>{}, std::true_type{}, edge_c);
      ++T;
      ktile(T, nkt - 1, m0, n0, !tail_half, std::integral_constant<int, 2>{}, std::false_type{},
            edge_c);
      ++T;
    };
    if constexpr (EPI == EPI_CPL_FWD) {
      if (a.cf_dh - (n0 >> 1) <= 16) tile_loop(std::true_type{});
      else tile_loop(std::false_type{});
    } else {
      tile_loop(std::false_type{});
    }
    // the next tile's K-tile 0 and K-tile 1's A-lo / B-lo: stream halves 4T .. 4T+5, i.e. the
    // slots of K-tiles T-2 (all four, read long ago) and T-1's A-lo / B-lo (read in its phase
    // r1) - not the free pair the epilogue stages through
    int m0n = 0, n0n = 0;
    if (has_next) {
      if constexpr (DYN) tile_at(id_next, m0n, n0n);
      else tile_org(s + 1, m0n, n0n);
#pragma unroll
      for (int h = 0; h < 6; ++h) issue_to(T + (h >> 2), m0n, n0n, h >> 2, h & 3);
    }
    // DYN: claim tile s + 2 (or, on the last tile, count this block finished); the result is
    // used only after the epilogue's vmcnt(0)
    if constexpr (DYN) {
      if (threadIdx.x == QL) raw = claim_add(has_next ? xcd : 8);
    }
    if (wr == 0) barrier();
    // ---- epilogue of tile s through the free LDS (see above)
    const int fs = (4 * (T - 1) + 2) & (NSLOT - 1);   // free slot pair of the last K-tile
    char* region = wave < 4 ? smem + fs * HALF_BYTES + wave * 8192
                            : smem + NSLOT * HALF_BYTES + (wave - 4) * 8192;
    // the epilogue's lane-derived offsets from an opaque per-tile zero: hoisted above the tile
    // loop they stayed live across the MFMA loop at the 256-VGPR limit and were spilled
    int zt;
    asm volatile("s_mov_b32 %0, 0" : "=s"(zt));
    const int lane_e = lane + zt, tid_e = wave * 64 + lane_e;   // not v0: keeps it dead
    if constexpr (EPI == EPI_CPL_FWD) {
      epi_coupling_fwd<2>(a, acc, m0, n0, wr, wc,
                          [&](int w) {
                            return w < 4 ? smem + fs * HALF_BYTES + w * 8192
                                         : smem + NSLOT * HALF_BYTES + (w - 4) * 8192;
                          },
                          lane_e, tid_e);
    } else if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_RELUMASK) {
      // (DYN: offsets from the opaque lane too, else the claim's register spills them)
      const int lane_b = DYN ? lane_e : lane;
      epi_tile_staged<EPI, 4, false, 0, 8>(a, acc, m0 + wr * 128, n0 + wc * 64, 0, region,
                                           lane_b);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own readback done before re-staging
      epi_tile_staged<EPI, 4, false, 4, 8>(a, acc, m0 + wr * 128 + 64, n0 + wc * 64, 0, region,
                                           lane_b);
    } else {
      epi_tile_staged<EPI, 8>(a, acc, m0 + wr * 128, n0 + wc * 64, 0, region, lane_e);
    }
    // the next tile's six halves (and this epilogue's stores) retired, and every wave's staging
    // reads done before the stream restages the slot pair
    vmwait<0>();
    if constexpr (DYN) {   // tile s + 2's id, read at the top of tile s + 1 (stream K-tile T)
      if (threadIdx.x == QL) {
        if (has_next) *qaddr(T) = resolve(raw);
        else finished(raw);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    m0 = m0n;
    n0 = n0n;
    if (!has_next) break;
  }
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI, bool DYN = false>
__global__ void __launch_bounds__(NTHR, 1) gemm256_persistent_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[8 * HALF_BYTES + 8 * 4096];
  NF_STAMP(5);   // stamps build: block start / end (the body ends on vmcnt(0) + barrier)
  gemm256_persistent_body<A_KMAJOR, B_KMAJOR, EPI, DYN>(a, smem);
  NF_STAMP(6);
}

// Streamed K-tiles of column tile tn under a MADE K-range plan (one or two ranges).
__device__ __forceinline__ int krange_len(const GemmArgs& a, int tn) {
  const int segs = a.krange_segs == 2 ? 2 : 1;
  const int* r = a.krange + 2 * segs * tn;
  int len = r[1] > r[0] ? r[1] - r[0] : 0;
  if (segs == 2 && r[3] > r[2]) len += r[3] - r[2];
  return len;
}

template <bool A_KMAJOR, bool B_KMAJOR, int EPI, int D, bool DB, bool F8 = false>
__global__ void __launch_bounds__(NTHR, 1) gemm256_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes(D)];
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  if (!a.pair_tiles) {
    gemm256_body<A_KMAJOR, B_KMAJOR, EPI, D, DB, F8>(a, xcd_remap(blockIdx.x, ntm * ntn),
                                                      blockIdx.y, smem);
    return;
  }
  // MADE-masked products: column tiles stream very different K lengths (a triangular mask:
  // 1:2:3:4), and one tile per block leaves the launch waiting on the CUs that drew two long
  // tiles. Each block instead takes, for one row tile tm, the column tiles of rank p and
  // ntn-1-p in descending K length (equal sums for a triangular plan): one balanced round,
  // and the two tiles share the A row panel.
  const int half = ntn >> 1;
  const int b = xcd_remap(blockIdx.x, ntm * half);
  const int tm = b / half, p = b % half;
  int tn_a = 0, tn_b = 0;
  for (int c = 0; c < ntn; ++c) {  // rank by (length desc, index asc); uniform scalar loop
    const int lc = krange_len(a, c);
    int rank = 0;
    for (int o = 0; o < ntn; ++o) {
      const int lo = krange_len(a, o);
      rank += (lo > lc || (lo == lc && o < c)) ? 1 : 0;
    }
    if (rank == p) tn_a = c;
    if (rank == ntn - 1 - p) tn_b = c;
  }
  if (a.pair_alt && (b & 1)) {   // short tile first on odd blocks
    const int t = tn_a;
    tn_a = tn_b;
    tn_b = t;
  }
  gemm256_body<A_KMAJOR, B_KMAJOR, EPI, D, DB, F8>(a, tm * ntn + tn_a, 0, smem);
  __syncthreads();  // the second tile's LDS-DMA reuses what the first tile's epilogue staged
  gemm256_body<A_KMAJOR, B_KMAJOR, EPI, D, DB, F8>(a, tm * ntn + tn_b, 0, smem);
}

// grouped weight gradients (same block layout as gemm.hip's gemm_group_kernel)
template <int D>
__global__ void __launch_bounds__(NTHR, 1) gemm256_group_kernel(GroupArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes(D)];
  const int id = xcd_remap(blockIdx.x, g.start[g.nprob]);
  int p = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (q < g.nprob && id >= g.start[q]) p = q;
  const GemmArgs& a = g.p[p];
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int local = id - g.start[p];
  gemm256_body<false, false, EPI_F32, D, true>(a, local % tiles, local / tiles, smem);
}

// Weight gradients of MANY layers per launch (TnDesc / TnMulti: tn_multi.h)

// F8: every problem of the launch has e4m3 operands (mn-major, K % 128 == 0, ld in bytes):
// read through ds_read_b64_tr_b8 (read_frag_f8mn), dW = acc * s_dy * s_x, db = s_dy * row sums
// A_KM / B_KM: operand layouts of every problem (false = batch-major, the TN weight-gradient form;
// true = a transposed [M or N][batch] copy, k-major) - the layout A/B of wgrad_bench --probe
template <int D, bool F8 = false, bool A_KM = false, bool B_KM = false>
__global__ void __launch_bounds__(NTHR, 1) gemm256_multi_kernel(TnMulti t) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes(D)];
  const int pos = xcd_remap(blockIdx.x, t.ntiles);
  const int id = t.tile0 + (t.use_perm ? (int)t.perm[pos] : pos);
  int p = 0;
  for (int q = 1; q < t.n; ++q)
    if (id >= t.d[q].start) p = q;
  const TnDesc& d = t.d[p];
  GemmArgs a{};
  a.A = d.A; a.lda = d.lda;
  a.B = d.B; a.ldb = d.ldb;
  a.C = d.C; a.ldc = d.ldc;
  a.dbias = d.db;
  a.M = d.M; a.N = d.N; a.K = d.K;
  a.k_per_split = ((d.K + BK - 1) / BK) * BK;
  a.staged = d.staged;
  a.cmask = d.cmask;
  if constexpr (F8) {
    a.f8_sa = t.scales + (d.sidx & 0xffff);
    a.f8_sb = t.scales + (d.sidx >> 16);
  }
  const int local = d.tiles ? (int)d.tiles[id - d.start] : id - d.start;
  gemm256_body<A_KM, B_KM, EPI_F32, D, true, F8>(a, local, 0, smem);
}

// persistent plain products, nf_gemm256_set_persist: 1 (default) fixed tile lists, 2 tiles
// claimed at run time (the DP runner's multi-rank backward: RCCL kernels take CUs while a grid of
// one block per CU runs, and a fixed-list block that cannot start delays its whole list),
// 0 one block per tile
static int g_persist = 1;

// mode 2's claim counters: slots of QCTR_SLOT ints (8 per-XCD counters + the finished-block
// count, each on its own 128-B line so the 32 blocks of one XCD do not queue behind the other
// XCDs' claims on one line). Allocated and zeroed by the first nf_gemm256_set_persist(2)
// (outside any graph capture); each launch's last block re-zeroes its slot. Two pools:
//  - eager launches rotate over the QSLOTS_EAGER first slots (launches of one stream never
//    overlap; concurrent streams would need QSLOTS_EAGER launches in flight to meet);
//  - a launch recorded into a hipGraph keeps its slot for every replay, so it takes a slot of
//    its own from the capture pool, which no eager launch and no other captured launch ever
//    gets. A graph exec never runs concurrently with itself, so its replays may share. When the
//    capture pool is used up (QSLOTS_CAPT captured claim launches in one process) further
//    captures fall back to the fixed-list persistent kernel, with a one-time notice.
constexpr int QSLOTS_EAGER = 256, QSLOTS_CAPT = 7936, QSLOTS = QSLOTS_EAGER + QSLOTS_CAPT;
static int* g_qctr = nullptr;
static int g_qctr_dev = -1;
static unsigned g_qslot = 0;
static int g_qslot_capt = 0;

// counter slot for one claimed-tile launch on `stream`, or null (use the fixed lists)
inline int* claim_slot(hipStream_t stream) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return nullptr;
  if (cs == hipStreamCaptureStatusNone) return g_qctr + QCTR_SLOT * (g_qslot++ % QSLOTS_EAGER);
  if (g_qslot_capt >= QSLOTS_CAPT) {
    static bool told = false;
    if (!told) {
      fprintf(stderr, "vinf: claim-counter capture pool used up, captured launches use fixed "
                      "tile lists from now on\n");
      told = true;
    }
    return nullptr;
  }
  return g_qctr + QCTR_SLOT * (QSLOTS_EAGER + g_qslot_capt++);
}

// CUs the persistent grid leaves free (nf_gemm256_set_reserve): a multi-rank backward runs
// RCCL kernels beside the GEMMs, and a persistent block queued behind one would hold back its
// whole tile list; grid = min(tiles, CUs - reserve) keeps every block startable
static int g_reserve = 0;

// the RealNVP coupling-forward product on gemm_cpl4w.hip (nf_gemm_cpl4w): opt-in, measured
// slower at the headline shape (docs/PERF_NOTES.md round 6: its one-wave-per-SIMD epilogue
// runs at half the VALU issue rate of this kernel's two waves per SIMD); NF_CPL4W_ON build: on
#ifdef NF_CPL4W_ON
static int g_cpl4w = 1;
#else
static int g_cpl4w = 0;
#endif

// weight-gradient tile -> block packing by XCD (nf_gemm256_xcd_pack, on by default)
static int g_xcd_pack = 1;

// MADE column-tile pairing (nf_gemm256_set_pair): 0 off, 1 auto (when the paired grid still
// gives every CU a block), 2 always (tests)
static int g_pair = 1;

int device_cus_256() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
  }();
  return n;
}

// Paired MADE launches alternate: odd blocks run their short tile first, so half the CUs are in
// a main loop while the other half store their epilogue. The fused MAF epilogues move ~420 KB
// per tile and run at the chip's HBM rate when every CU stores at once; alternating took fwd2
// 172 -> 164 us (bf16) / 191 -> 178 (e4m3) and the fused backward 183 -> 166 / 178 -> 167 per
// layer (profiles/r2_maf_kernels.json)
inline bool pair_ok(const GemmArgs& a, int ntm, int ntn, int splits) {
  return g_pair && a.krange && splits == 1 && ntn % 2 == 0 &&
         (g_pair == 2 || (long)ntm * (ntn / 2) >= device_cus_256());
}

template <bool AK, bool BK_, int EPI, bool DB = false>
void launch(GemmArgs a, int splits, hipStream_t stream) {
  a.staged = staged_ok(a, EPI);
  if (a.mask_out && !a.staged) {
    fprintf(stderr, "vinf: ReLU bitmask output needs the staged epilogue (N %% 8, 16-B rows)\n");
    abort();
  }
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  // pair the column tiles of MADE-masked products (see gemm256_kernel)
  a.pair_tiles = pair_ok(a, ntm, ntn, splits);
  a.pair_alt = 1;
  // plain products run persistent (one continuous LDS-DMA stream per block, see
  // gemm256_persistent_body); nf_gemm256_set_persist(0) restores one tile per block
  const bool staged_epi = EPI == EPI_CPL_FWD || a.staged;
  if constexpr (!DB && AK) {
  if (g_persist && splits == 1 && !a.krange && !a.skip && !a.pair_tiles && staged_epi &&
      a.K > BK) {
    const int ntiles = ntm * ntn;
    int cus = (device_cus_256() - g_reserve) & ~7;   // whole XCD rounds: xcd_remap's b & 7
    cus = cus > 8 ? cus : 8;
    const int G = ntiles < cus ? ntiles : cus;
    // (mode 2 excludes the coupling forward: its epilogue reads other waves' staging regions,
    // where the claimed id is published; the engines run their forwards in mode 1)
    if constexpr (EPI != EPI_CPL_FWD) {
      int dev = -1;
      if (g_persist == 2 && g_qctr && hipGetDevice(&dev) == hipSuccess && dev == g_qctr_dev) {
        a.qctr = claim_slot(stream);
        if (a.qctr)
          hipLaunchKernelGGL((gemm256_persistent_kernel<AK, BK_, EPI, true>), dim3(G),
                             dim3(NTHR), 0, stream, a);
        else   // capture pool used up: fixed tile lists
          hipLaunchKernelGGL((gemm256_persistent_kernel<AK, BK_, EPI>), dim3(G), dim3(NTHR), 0,
                             stream, a);
        NF_HIP_CHECK(hipGetLastError());
        return;
      }
    }
    if (g_persist == 1) {
      hipLaunchKernelGGL((gemm256_persistent_kernel<AK, BK_, EPI>), dim3(G), dim3(NTHR), 0,
                         stream, a);
      NF_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  }
  dim3 grid(a.pair_tiles ? ntm * (ntn / 2) : ntm * ntn, splits), block(NTHR);
  hipLaunchKernelGGL((gemm256_kernel<AK, BK_, EPI, 4, DB>), grid, block, 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

// e4m3 operands (both k-major) on the one-tile-per-block kernel, MADE column tiles paired as in
// launch()
template <int EPI>
void launch_f8(GemmArgs a, hipStream_t stream) {
  a.staged = EPI == EPI_CPL_FWD ? 0 : staged_ok(a, EPI);
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  a.pair_tiles = pair_ok(a, ntm, ntn, 1);
  a.pair_alt = 1;
  const int nblk = a.pair_tiles ? ntm * (ntn / 2) : ntm * ntn;
  hipLaunchKernelGGL((gemm256_kernel<true, true, EPI, 4, false, true>), dim3(nblk), dim3(NTHR), 0,
                     stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

}  // namespace g256
}  // namespace gemm
}  // namespace nf

using namespace nf::gemm;

int nf_gemm256_set_pair(int mode) {   // mode < 0: query; returns the previous setting
  const int prev = g256::g_pair;
  if (mode >= 0) g256::g_pair = mode > 2 ? 2 : mode;
  return prev;
}
void nf_gemm256_set_persist(int mode) {
  using namespace g256;
  g_persist = mode == 2 ? 2 : mode ? 1 : 0;
  int dev = -1;
  if (g_persist == 2 && !g_qctr && hipGetDevice(&dev) == hipSuccess) {
    void* p = nullptr;
    if (hipMalloc(&p, QSLOTS * QCTR_SLOT * sizeof(int)) == hipSuccess &&
        hipMemset(p, 0, QSLOTS * QCTR_SLOT * sizeof(int)) == hipSuccess &&
        hipDeviceSynchronize() == hipSuccess) {
      g_qctr = (int*)p;
      g_qctr_dev = dev;
    } else {
      fprintf(stderr, "vinf: persist mode 2 counters unavailable, using one block per tile\n");
    }
  }
}
int nf_gemm256_set_reserve(int cus) {
  const int prev = g256::g_reserve;
  if (cus >= 0) g256::g_reserve = cus;
  return prev;
}
int nf_gemm256_xcd_pack(int on) {   // on < 0: query; returns the previous setting
  const int prev = g256::g_xcd_pack;
  if (on >= 0) g256::g_xcd_pack = on ? 1 : 0;
  return prev;
}
int nf_gemm256_get_persist() { return g256::g_persist; }

// y[M][N] = act(x[M][K] W[N][K]^T + bias) -> bf16
void nf_launch_gemm256_nt(const void* x, long ldx, const void* W, long ldw, const void* bias,
                          void* y, long ldy, int M, int N, int K, int relu, hipStream_t stream,
                          void* mask_out, long ld_mask, const int* krange) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)x; a.lda = ldx;
  a.B = (const nf::bf16_t*)W; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const nf::bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + 63) / 64) * 64; a.relu = relu;
  a.mask_out = (unsigned char*)mask_out; a.ld_mask = ld_mask;
  a.krange = krange;
  g256::launch<true, true, EPI_BF16>(a, 1, stream);
}

// dx[M][N] = dy[M][K] W[K][N]  (* 1(aux>0) -> bf16)  or  fp32 dx (+)= ...
void nf_launch_gemm256_nn(const void* dy, long lddy, const void* W, long ldw, const void* aux,
                          long ld_aux, void* dx, long lddx, int dx_is_f32, int accumulate, int M,
                          int N, int K, hipStream_t stream, int aux_is_bits, const int* krange,
                          int krange_segs, int w_kmajor) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.krange = krange;
  a.krange_segs = krange_segs;
  a.A = (const nf::bf16_t*)dy; a.lda = lddy;
  a.B = (const nf::bf16_t*)W; a.ldb = ldw;
  a.C = dx; a.ldc = lddx;
  a.aux = (const nf::bf16_t*)aux; a.ld_aux = ld_aux;
  a.aux_bits = aux_is_bits;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + 63) / 64) * 64;
  if (w_kmajor) {   // W given as Wt [N][K]: the NT instantiation (k-major fragment reads)
    if (dx_is_f32) {
      if (accumulate) g256::launch<true, true, EPI_F32_ACC>(a, 1, stream);
      else g256::launch<true, true, EPI_F32>(a, 1, stream);
    } else if (aux) {
      g256::launch<true, true, EPI_BF16_RELUMASK>(a, 1, stream);
    } else {
      g256::launch<true, true, EPI_BF16>(a, 1, stream);
    }
    return;
  }
  if (dx_is_f32) {
    if (accumulate) g256::launch<true, false, EPI_F32_ACC>(a, 1, stream);
    else g256::launch<true, false, EPI_F32>(a, 1, stream);
  } else if (aux) {
    g256::launch<true, false, EPI_BF16_RELUMASK>(a, 1, stream);
  } else {
    g256::launch<true, false, EPI_BF16>(a, 1, stream);
  }
}

// Input gradient dx[M][N] = dy[M][K] W[K][N] with W given transposed (Wt [N][K], k-major):
// the NT instantiation (b128 fragment reads of both operands) with the bf16 ReLU-mask (aux =
// activation or bitmask) or plain bf16 epilogue.
void nf_launch_gemm256_nt_dgrad(const void* dy, long lddy, const void* Wt, long ldwt,
                                const void* aux, long ld_aux, int aux_is_bits, void* dx,
                                long lddx, int M, int N, int K, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)dy; a.lda = lddy;
  a.B = (const nf::bf16_t*)Wt; a.ldb = ldwt;
  a.C = dx; a.ldc = lddx;
  a.aux = (const nf::bf16_t*)aux; a.ld_aux = ld_aux;
  a.aux_bits = aux_is_bits;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + 63) / 64) * 64;
  if (aux) g256::launch<true, true, EPI_BF16_RELUMASK>(a, 1, stream);
  else g256::launch<true, true, EPI_BF16>(a, 1, stream);
}

// Last conditioner product of coupling layer l with its coupling forward fused (EPI_CPL_FWD):
// W [2 Dh (+pad) rows][K], x/y fp32 [M][Dh], yb bf16 [M][>= yb_width] (or null), st bf16 [M][>= Dh]
// (s_hat written), ldjp fp32 [ceil(Dh/128)][M] per-column-tile partial sums of s.
void nf_launch_gemm256_nt_cpl(const void* h, long ldh, const void* W, long ldw, int w_rows,
                              const void* bias, void* st, long ld_st, int M, int K, int Dh,
                              const float* x, long ld_x, float* y, long ld_y, void* yb, long ld_yb,
                              int yb_width, float* ldjp, long ld_ldjp, int ldj_init, float scale,
                              hipStream_t stream, int inverse) {
  if (M <= 0) return;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)h; a.lda = ldh;
  a.B = (const nf::bf16_t*)W; a.ldb = ldw;
  a.C = st; a.ldc = ld_st;
  a.bias = (const nf::bf16_t*)bias;
  const int ntn = (Dh + 127) / 128;
  a.M = M; a.N = ntn * 256; a.K = K; a.k_per_split = ((K + 63) / 64) * 64;
  a.cf_x = x; a.ld_cf_x = ld_x;
  a.cf_y = y; a.ld_cf_y = ld_y;
  a.cf_yb = (nf::bf16_t*)yb; a.ld_cf_yb = ld_yb; a.cf_yb_width = yb_width;
  a.cf_ldj = ldjp; a.ld_cf_ldj = ld_ldjp; a.cf_ldj_init = ldj_init;
  a.cf_dh = Dh; a.cf_b_rows = w_rows; a.cf_scale = scale; a.cf_pair = Dh;
  a.cf_inverse = inverse;
  auto al16 = [](const void* p) { return ((unsigned long)p & 15) == 0; };
  if (Dh % 8 || w_rows < 2 * Dh || ld_x % 4 || ld_y % 4 || (st && ld_st % 8) ||
      (yb && (ld_yb % 8 || !al16(yb) || yb_width < Dh || yb_width % 8)) || !al16(x) || !al16(y) ||
      !al16(st) || (!st && !inverse)) {
    fprintf(stderr, "vinf: fused coupling-forward GEMM needs Dh %% 8 == 0, 16-B aligned rows and "
                    "2 Dh weight rows\n");
    abort();
  }
  if (g256::g_cpl4w) {   // the 4-fat-wave 136-feature tiles (gemm_cpl4w.hip): no edge tile
    cpl4w::Args c{};
    c.A = (const nf::bf16_t*)h; c.lda = ldh;
    c.W = (const nf::bf16_t*)W; c.ldw = ldw; c.w_rows = w_rows;
    c.bias = (const nf::bf16_t*)bias;
    c.st = (nf::bf16_t*)st; c.ld_st = ld_st;
    c.x = x; c.ld_x = ld_x; c.y = y; c.ld_y = ld_y;
    c.yb = (nf::bf16_t*)yb; c.ld_yb = ld_yb; c.yb_width = yb_width;
    c.ldjp = ldjp; c.ld_ldjp = ld_ldjp; c.ldj_rows = ntn; c.ldj_init = ldj_init;
    c.M = M; c.K = K; c.Dh = Dh; c.scale = scale; c.inverse = inverse;
    if (launch_cpl4w(c, stream)) return;
  }
  g256::launch<true, true, EPI_CPL_FWD>(a, 1, stream);
}
int nf_gemm_cpl4w(int on) {   // on < 0: query; returns the previous setting
  const int prev = g256::g_cpl4w;
  if (on >= 0) g256::g_cpl4w = on ? 1 : 0;
  return prev;
}

// Second MADE product of MAF layer l with the layer's transform fused (EPI_CPL_FWD, cf_mode 1):
// o = h (W2 * M2)^T + b2 = [mu | s_raw] is never stored; each 256-column tile holds the s_raw
// and mu columns of 128 features (W2 rows D + j and j), so the epilogue writes u = (x - mu)
// e^-alpha (fp32 u, bf16 ubf, optional e4m3 uq under a delayed scale), s_raw (bf16 [M][D], the
// backward's only use of o) and ldjp[tn][m] (-sum alpha over the tile's features, one owner per
// entry). h / W2 are bf16, or e4m3 (f8 = 1: hs = h's per-tensor scale, ws = W2's per-row scales).
// krange: [D / 128][2] K range of each paired tile (union of its mu and s_raw mask rows).
void nf_launch_gemm256_maf_fwd(const void* h, long ldh, int f8, const float* hs, const void* W,
                               long ldw, const float* ws, const void* bias, const int* krange,
                               void* s_out, long ld_s, int M, int K, int D, const float* x,
                               long ld_x, float* u, long ld_u, void* ubf, long ld_ub, float* ldjp,
                               long ld_ldjp, int ldj_init, float bound, void* uq, long lduq,
                               const float* q_amax_prev, float* q_scale_out, float* q_amax_cur,
                               hipStream_t stream, int x_bf16) {
  if (M <= 0) return;
  const int EB = f8 ? 1 : 2;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)h; a.lda = ldh;
  a.B = (const nf::bf16_t*)((const char*)W + (long)D * ldw * EB); a.ldb = ldw;   // s_raw rows
  a.C = s_out; a.ldc = ld_s;
  a.bias = bias ? (const nf::bf16_t*)bias + D : nullptr;
  const int ntn = D / 128;
  a.M = M; a.N = ntn * 256; a.K = K; a.k_per_split = f8 ? K : ((K + 63) / 64) * 64;
  a.krange = krange; a.krange_segs = 1;
  a.cf_x = x; a.ld_cf_x = ld_x; a.cf_x_bf16 = x_bf16;   // x_bf16: x points at bf16 (u may be null)
  a.cf_y = u; a.ld_cf_y = ld_u;
  a.cf_yb = (nf::bf16_t*)ubf; a.ld_cf_yb = ld_ub; a.cf_yb_width = D;
  a.cf_ldj = ldjp; a.ld_cf_ldj = ld_ldjp; a.cf_ldj_init = ldj_init;
  a.cf_dh = D; a.cf_b_rows = D; a.cf_scale = bound; a.cf_pair = -D; a.cf_mode = 1;
  a.f8_sa = hs; a.f8_sb = f8 ? ws + D : nullptr;
  a.f8_cq = (unsigned char*)uq; a.ld_f8_cq = lduq;
  a.f8_q_amax_prev = q_amax_prev; a.f8_q_scale_out = q_scale_out; a.f8_q_amax_cur = q_amax_cur;
  auto al16 = [](const void* p) { return ((unsigned long)p & 15) == 0; };
  if (D % 128 || ld_x % (x_bf16 ? 8 : 4) || (u && ld_u % 4) || ld_s % 8 ||
      (ubf && (ld_ub % 8 || !al16(ubf))) || (!u && !ubf) ||
      !al16(x) || (u && !al16(u)) || !al16(s_out) || !krange || (f8 && (K % 128 || !hs || !ws)) ||
      (uq && (!f8 || lduq % 8 || !q_amax_prev || !q_scale_out || !q_amax_cur)) ||
      (!f8 && K % 32)) {
    fprintf(stderr, "vinf: fused MAF-forward GEMM needs D %% 128 == 0, 16-B aligned rows, K "
                    "ranges, and (fp8) K %% 128 == 0 with both scales\n");
    abort();
  }
  if (f8) g256::launch_f8<EPI_CPL_FWD>(a, stream);
  else g256::launch<true, true, EPI_CPL_FWD>(a, 1, stream);
}

// Masked input gradient dx = relu'(h) * (dyq sa)(Wtq sb)^T on e4m3 operands (dyq [M][K] with a
// per-tensor scale, Wtq = (W*M)^T [N][K] with per-row scales), bf16 dx plus optionally its e4m3
// copy under a delayed scale (the next fp8 input-gradient product's operand).
void nf_launch_gemm256_fp8_dgrad(const void* dyq, long lddy, const float* sa, const void* wtq,
                                 long ldwt, const float* sb, const void* aux, long ld_aux,
                                 int aux_bits, void* dx, long lddx, int M, int N, int K,
                                 const int* krange, int krange_segs, void* dxq, long lddxq,
                                 const float* q_amax_prev, float* q_scale_out, float* q_amax_cur,
                                 hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)dyq; a.lda = lddy;
  a.B = (const nf::bf16_t*)wtq; a.ldb = ldwt;
  a.C = dx; a.ldc = lddx;
  a.aux = (const nf::bf16_t*)aux; a.ld_aux = ld_aux; a.aux_bits = aux_bits;
  a.M = M; a.N = N; a.K = K; a.k_per_split = K;
  a.krange = krange; a.krange_segs = krange_segs;
  a.f8_sa = sa; a.f8_sb = sb;
  a.f8_cq = (unsigned char*)dxq; a.ld_f8_cq = lddxq;
  a.f8_q_amax_prev = q_amax_prev; a.f8_q_scale_out = q_scale_out; a.f8_q_amax_cur = q_amax_cur;
  if (K % 128 || lddy % 16 || ldwt % 16 || N % 8 || !aux || !staged_ok(a, EPI_BF16_RELUMASK) ||
      (dxq && lddxq % 8)) {
    fprintf(stderr, "vinf: fp8 masked input gradient needs K %% 128 == 0, 16-B rows, N %% 8 == 0, "
                    "the ReLU operand and the staged epilogue\n");
    abort();
  }
  g256::launch_f8<EPI_BF16_RELUMASK>(a, stream);
}

// Conditioner input gradient of coupling layer l fused with the backward of coupling layer l-1
// (EPI_CPL_BWD, gemm_tile.h): gy = G[M][N] + dy[M][K] W[K][N] is consumed in the epilogue and
// never stored; dst/gx of layer l-1 are written instead.
void nf_launch_gemm256_nn_cpl(const void* dy, long lddy, const void* W, long ldw, const float* G,
                              long ldg, int M, int N, int K, const void* s_hat, long ld_s,
                              const float* x, long ld_x, void* dst, long ld_dst, int dst_pad,
                              float* gx, long ld_gx, int Dh, float scale, float c,
                              hipStream_t stream, int w_kmajor, const int* krange,
                              int krange_segs, int mode, const NfF8Operands* f8, int x_bf16,
                              int g_in_bf16, int gx_bf16) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  if (f8) {   // e4m3 dy (per-tensor scale) and Wt (per-row scales); optional e4m3 copy of dst
    a.f8_sa = f8->sa; a.f8_sb = f8->sb;
    a.f8_cq = (unsigned char*)f8->q; a.ld_f8_cq = f8->ldq;
    a.f8_q_amax_prev = f8->q_amax_prev; a.f8_q_scale_out = f8->q_scale_out;
    a.f8_q_amax_cur = f8->q_amax_cur;
  }
  // MAF (mode 1): the first MADE product's input gradient of layer l with the MAF backward of
  // layer l-1 (GemmArgs::cpl_mode), under the weight's per-tile K ranges
  a.krange = krange; a.krange_segs = krange_segs;
  a.cpl_mode = mode;
  a.A = (const nf::bf16_t*)dy; a.lda = lddy;
  a.B = (const nf::bf16_t*)W; a.ldb = ldw;
  a.C = (void*)G; a.ldc = ldg;
  a.aux = (const nf::bf16_t*)s_hat; a.ld_aux = ld_s;
  a.M = M; a.N = N; a.K = K; a.k_per_split = ((K + 63) / 64) * 64;
  a.cpl_x = x; a.ld_cpl_x = ld_x;
  a.cpl_gx = gx; a.ld_cpl_gx = ld_gx;
  a.cpl_dst = (nf::bf16_t*)dst; a.ld_cpl_dst = ld_dst;
  a.cpl_dh = Dh; a.cpl_pad = dst_pad;
  a.cpl_scale = scale; a.cpl_c = c;
  a.cpl_c_bf16 = g_in_bf16; a.cpl_gx_bf16 = gx_bf16;
  if ((g_in_bf16 || gx_bf16) && !x_bf16) {
    fprintf(stderr, "vinf: bf16 G chain in the fused backward needs the bf16-x form\n");
    abort();
  }
  // x_bf16 (EPI_CPL_BWD_XB): x is the bf16 copy of h_{l-1} (coupling) or the bf16 MAF state u
  const int epi = x_bf16 ? EPI_CPL_BWD_XB : EPI_CPL_BWD;
  // (the MAF engine's bf16_state option runs the MAF mode, e4m3 included, on bf16 u)
  if (x_bf16 && (!w_kmajor || ((g_in_bf16 || gx_bf16) && (f8 || mode)))) {
    fprintf(stderr, "vinf: bf16 x in the fused backward needs Wt (and the bf16 G chain the bf16 "
                    "coupling form)\n");
    abort();
  }
  if (Dh > N || dst_pad < 2 * Dh || dst_pad > Dh + N || !staged_ok(a, epi)) {
    fprintf(stderr, "vinf: fused coupling-backward GEMM needs Dh <= N, 2 Dh <= pad <= Dh + N, "
                    "4-element aligned rows and the staged epilogue\n");
    abort();
  }
  if (f8) {
    if (!w_kmajor || K % 128 || lddy % 16 || ldw % 16 || (f8->q && f8->ldq % 8)) {
      fprintf(stderr, "vinf: fp8 fused backward needs Wt, K %% 128 == 0 and 16-B rows\n");
      abort();
    }
    a.k_per_split = K;
    if (x_bf16) g256::launch_f8<EPI_CPL_BWD_XB>(a, stream);
    else g256::launch_f8<EPI_CPL_BWD>(a, stream);
    return;
  }
  if (x_bf16) {
    g256::launch<true, true, EPI_CPL_BWD_XB>(a, 1, stream);
    return;
  }
  if (w_kmajor) g256::launch<true, true, EPI_CPL_BWD>(a, 1, stream);   // W given as Wt [N][K]
  else g256::launch<true, false, EPI_CPL_BWD>(a, 1, stream);
}

// dW[M][N] (+ db[M]) = split-K partials of dy[K][M]^T x[K][N] written to `work` slabs (or
// straight to dW/db when splits == 1); the caller reduces them (gemm.hip).
int nf_launch_gemm256_tn_partials(const void* dy, long lddy, const void* x, long ldx, float* C,
                                  long ldc, long slab_stride, float* dbias, int M, int N, int K,
                                  int splits, hipStream_t stream) {
  const int nkt = (K + 63) / 64;
  if (splits < 1) splits = 1;
  if (splits > nkt) splits = nkt;
  const int kts = (nkt + splits - 1) / splits;
  const int used = (nkt + kts - 1) / kts;
  GemmArgs a{};
  a.A = (const nf::bf16_t*)dy; a.lda = lddy;
  a.B = (const nf::bf16_t*)x; a.ldb = ldx;
  a.C = C; a.ldc = ldc; a.c_split_stride = slab_stride;
  a.dbias = dbias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = kts * 64;
  g256::launch<false, false, EPI_F32, true>(a, used, stream);
  return used;
}

// y[M][N] = act((qx * sx) (qw * sw)^T + bias) -> bf16 (+ optional e4m3 copy of y), e4m3 operands
// with K (bytes) % 128 == 0; krange: per-256-column-tile K ranges of a MADE-masked weight
void nf_launch_gemm256_fp8_nt(const void* xq, long ldx, const float* sx, int sx_per_row,
                              const void* wq, long ldw, const float* sw, const void* bias, void* y,
                              long ldy, int M, int N, int K, int relu, const int* krange,
                              void* yq, long ldyq, const float* q_amax_prev, float* q_scale_out,
                              float* q_amax_cur, hipStream_t stream, unsigned char* mask_out,
                              long ld_mask) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.mask_out = mask_out; a.ld_mask = ld_mask;   // ReLU bitmask (y may then be null)
  a.A = (const nf::bf16_t*)xq; a.lda = ldx;
  a.B = (const nf::bf16_t*)wq; a.ldb = ldw;
  a.C = y; a.ldc = ldy;
  a.bias = (const nf::bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.k_per_split = K; a.relu = relu;
  a.krange = krange;
  a.f8_sa = sx; a.f8_sa_per_row = sx_per_row; a.f8_sb = sw;
  a.f8_cq = (unsigned char*)yq; a.ld_f8_cq = ldyq;
  a.f8_q_amax_prev = q_amax_prev; a.f8_q_scale_out = q_scale_out; a.f8_q_amax_cur = q_amax_cur;
  a.staged = staged_ok(a, EPI_BF16);
  if (K % 128 || ldx % 16 || ldw % 16 || N % 8 || !a.staged || (yq && ldyq % 8)) {
    fprintf(stderr, "vinf: gemm256_fp8_nt needs K %% 128 == 0, 16-B rows, N %% 8 == 0 and the "
                    "staged epilogue\n");
    abort();
  }
  const int ntm = (M + g256::BM - 1) / g256::BM, ntn = (N + g256::BN - 1) / g256::BN;
  a.pair_tiles = g256::pair_ok(a, ntm, ntn, 1);
  a.pair_alt = 1;
  const int nblk = a.pair_tiles ? ntm * (ntn / 2) : ntm * ntn;
  hipLaunchKernelGGL((g256::gemm256_kernel<true, true, EPI_BF16, 4, false, true>), dim3(nblk),
                     dim3(g256::NTHR), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

int nf_gemm256_tiles(int M, int N) {
  return ((M + g256::BM - 1) / g256::BM) * ((N + g256::BN - 1) / g256::BN);
}

// tiles are numbered problem after problem (row-major tiles inside a problem); the launch
// computes tiles [tile0, tile0 + ntiles) and may start or end inside a problem
void nf_launch_gemm256_tn_multi(int nprob, const NfTnProblem* pr, int tile0, int ntiles,
                                hipStream_t stream, const float* f8_scales, int layout) {
  if (ntiles <= 0) return;
  const bool f8 = f8_scales != nullptr;
  g256::TnMulti t{};
  t.scales = f8_scales;
  int base = 0;
  for (int p = 0; p < nprob; ++p) {
    const NfTnProblem& q = pr[p];
    const int tiles = q.ntiles_active >= 0 ? q.ntiles_active : nf_gemm256_tiles(q.M, q.N);
    if (base + tiles > tile0 && base < tile0 + ntiles) {
      if (t.n >= g256::TN_MULTI_MAX) {
        fprintf(stderr, "vinf: gemm256_tn_multi: more than %d problems in one launch\n",
                g256::TN_MULTI_MAX);
        abort();
      }
      if (f8 && (q.K % 128 || q.M % 16 || q.N % 16 || q.sa_idx < 0 || q.sb_idx < 0 ||
                 q.sa_idx > 0xffff || q.sb_idx > 0x7fff)) {
        fprintf(stderr, "vinf: gemm256_tn_multi e4m3: K %% 128, M/N %% 16, scale indices\n");
        abort();
      }
      if (q.skip || q.K % 32 || q.M % 8 || q.N % 8 || (q.cmask && q.lddw != q.N)) {
        fprintf(stderr, "vinf: gemm256_tn_multi: K %% 32, M/N %% 8, active-tile lists instead of "
                        "skip flags, dense dW with a cmask\n");
        abort();
      }
      g256::TnDesc& d = t.d[t.n++];
      d.A = (const nf::bf16_t*)q.dy; d.lda = (int)q.lddy;
      d.B = (const nf::bf16_t*)q.x; d.ldb = (int)q.ldx;
      d.C = q.dW; d.ldc = (int)q.lddw;
      d.db = f8 ? nullptr : q.db;   // e4m3: bias sums by nf_launch_fp8_colsum
      d.tiles = q.tiles;
      d.cmask = q.cmask;
      d.M = q.M; d.N = q.N; d.K = q.K;
      d.start = base;
      d.sidx = f8 ? (q.sa_idx | (q.sb_idx << 16)) : 0;
      GemmArgs a{};
      a.C = q.dW; a.ldc = q.lddw; a.N = q.N;
      d.staged = staged_ok(a, EPI_F32);
      if (f8 && !d.staged) {   // the dequantising epilogue is the staged one
        fprintf(stderr, "vinf: gemm256_tn_multi e4m3: dW must be 16-B aligned, N %% 4\n");
        abort();
      }
    }
    base += tiles;
  }
  if (tile0 + ntiles > base || t.n == 0) {
    fprintf(stderr, "vinf: gemm256_tn_multi: tile range [%d, %d) outside the %d tiles\n", tile0,
            tile0 + ntiles, base);
    abort();
  }
  t.tile0 = tile0;
  t.ntiles = ntiles;
  if (g256::g_xcd_pack && ntiles <= g256::TN_PERM_MAX) {
    int seg_lo[g256::TN_MULTI_MAX], seg_n[g256::TN_MULTI_MAX];
    for (int i = 0; i < t.n; ++i) {
      const int lo = t.d[i].start > tile0 ? t.d[i].start : tile0;
      const int hi_p = i + 1 < t.n ? t.d[i + 1].start : base;
      const int hi = hi_p < tile0 + ntiles ? hi_p : tile0 + ntiles;
      seg_lo[i] = lo - tile0;
      seg_n[i] = hi - lo;
    }
    t.use_perm = nf::wgrad_xcd_perm(t.n, seg_lo, seg_n, ntiles, t.perm) ? 1 : 0;
  }
  // 4-wave 128x128-per-wave TN kernel (gemm_tn4w.hip): the default bf16 launch (the real
  // multi-layer launch 2583 -> 1960 us median, profiles/r4/tn4w4_layout_probe.jsonl); layout 4
  // keeps the 8-wave kernel (A/B and bitwise tests), 3 forces the 4-wave one
  if (!f8 && (layout == 3 || layout == 0) && nf::gemm::launch_tn4w_multi(t, stream)) return;
  if (layout == 3 || layout == 4) layout = 0;
  if (layout != 0 && f8) {
    fprintf(stderr, "vinf: gemm256_tn_multi: transposed-operand layouts are bf16 only\n");
    abort();
  }
  if (layout == 1)
    hipLaunchKernelGGL((g256::gemm256_multi_kernel<4, false, false, true>), dim3(ntiles),
                       dim3(g256::NTHR), 0, stream, t);
  else if (layout == 2)
    hipLaunchKernelGGL((g256::gemm256_multi_kernel<4, false, true, false>), dim3(ntiles),
                       dim3(g256::NTHR), 0, stream, t);
  else if (f8)
    hipLaunchKernelGGL((g256::gemm256_multi_kernel<4, true>), dim3(ntiles), dim3(g256::NTHR), 0,
                       stream, t);
  else
    hipLaunchKernelGGL(g256::gemm256_multi_kernel<4>, dim3(ntiles), dim3(g256::NTHR), 0, stream, t);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_gemm256_tn_group(const GroupArgs& g, hipStream_t stream) {
  hipLaunchKernelGGL(g256::gemm256_group_kernel<4>, dim3(g.start[g.nprob]), dim3(g256::NTHR), 0,
                     stream, g);
  NF_HIP_CHECK(hipGetLastError());
}

#ifdef NF_G256_STAMPS
void nf_g256_set_stamps(void* p) {
  NF_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(nf_g256_stamp_buf), &p, sizeof(p)));
}
#endif
