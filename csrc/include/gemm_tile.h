// Shared pieces of the bf16 MFMA GEMM kernels (gemm.hip: 128x128 tile, gemm256.hip: 256x256
// 8-phase tile): argument block, epilogue kinds, LDS operand-image swizzles and fragment reads.
//
// LDS operand images (one 128 x 64 bf16 block, 16 KiB):
//   k-major  [128 rows][64 k]  : 16-B chunk c of row r stored at c ^ (r & 7)
//   mn-major [64 k][128 mn]    : 16-B chunk c of k-row k stored at c ^ mn_swz(k)
// both conflict-free for the fragment reads below (tools/lds_bank_model.py).
#pragma once
#include "nf_common.h"

#include <cstdio>
#include <cstdlib>

namespace nf {
namespace gemm {

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

enum Epi : int {
  EPI_BF16 = 0,          // C(bf16) = act(acc + bias)
  EPI_F32 = 1,           // C(fp32) = acc  (split-K slab when gridDim.y > 1)
  EPI_BF16_RELUMASK = 2, // C(bf16) = acc * 1(aux > 0)
  EPI_F32_ACC = 3,       // C(fp32) += acc
  EPI_CPL_BWD = 4,       // gy = C(fp32) + acc, then the affine-coupling backward of the previous
                         // flow layer (staged path only; see GemmArgs::cpl_*)
  EPI_CPL_FWD = 5,       // [s_hat | t] = acc + bias, then the affine-coupling forward of the same
                         // layer (gemm256 only; see GemmArgs::cf_*)
  EPI_CPL_BWD_XB = 6,    // EPI_CPL_BWD reading x = h_{l-1} as bf16 (the conditioner operand copy
                         // the forward wrote) instead of the fp32 state: 2 B less per element of
                         // an HBM-bound epilogue; x only enters dS_hat, which is stored in bf16
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
  int krange_segs;             // 2: krange is [ntn][4], two ranges per tile (gemm256 only)
  int pair_tiles;              // gemm256: each block computes two column tiles (set by launchers)
  int pair_alt;                // gemm256 paired tiles: odd blocks take the short tile first, so
                               // the CUs' epilogues (HBM-bound) do not all run at once
  const unsigned char* skip;   // [ntm*ntn] 1 -> tile entirely masked: write zeros, no MFMA, or null
  const unsigned char* cmask;  // [M][N] 0/1 applied to fp32 outputs (masked weight gradients), or null
  int staged;                  // 1 -> LDS-staged epilogue (set by the launchers, see staged_ok)
  // ReLU bitmask (1 bit per output, bit e of byte [m][n/8] <-> column n+e):
  unsigned char* mask_out;     // EPI_BF16 + relu: also write 1(y > 0) bits (staged path only)
  long ld_mask;                // bytes per mask row
  int aux_bits;                // EPI_BF16_RELUMASK: aux is such a bitmask (ld_aux in bytes)
  // EPI_CPL_BWD: the input gradient of coupling layer l's conditioner completes
  // gy = dL/dh_{l+1}, which is exactly the output gradient coupling layer l-1 needs. The
  // epilogue finishes gy (= old C + acc, never stored) and applies layer l-1's backward
  //   s = cpl_scale * tanh(s_hat)      (s_hat = aux, bf16, [M][ld_aux])
  //   dS_hat = (gy x e^s + cpl_c) (cpl_scale - s^2 / cpl_scale),  dT = gy,  gx = gy e^s
  // writing dst = [dS_hat | dT | 0-pad to cpl_pad] (bf16) and gx (fp32) for n < cpl_dh.
  const float* cpl_x; long ld_cpl_x;   // x = h_{l-1} (fp32; bf16 under EPI_CPL_BWD_XB)
  float* cpl_gx; long ld_cpl_gx;       // dL/dh_{l-1} (fp32, written)
  bf16_t* cpl_dst; long ld_cpl_dst;    // conditioner output gradient of layer l-1
  int cpl_dh, cpl_pad;
  float cpl_scale, cpl_c;
  // EPI_CPL_BWD_XB only: the G chain in bf16 - C (the partial dL/dh_{l+1}) read as bf16 and / or
  // gx written as bf16 (the engine keeps fp32 at the chain's two ends)
  int cpl_c_bf16, cpl_gx_bf16;
  // cpl_mode 1: the backward of MAF layer l-1 instead (models/maf_engine.py, csrc/kernels/maf.hip)
  //   u = (x - mu) e^-alpha, alpha = b tanh(s_raw / b)   (b = cpl_scale, s_raw = aux, x = u_{l-1})
  //   gx = gy e^-alpha,  dst = [dmu | ds_raw] = [-gx | (cpl_c - gy u)(1 - tanh^2)]
  int cpl_mode;
  // e4m3 operands (gemm256.hip FP8 instantiation, EPI_BF16): y = acc * f8_sa[m | 0] * f8_sb[n]
  // + bias, and optionally an e4m3 copy of the stored bf16 y with a delayed per-tensor scale
  // (q = e4m3(sat(y / s)), s = amax_prev / 448, amax_cur = max |y|) - the next fp8 GEMM's operand
  const float* f8_sa;
  int f8_sa_per_row;
  const float* f8_sb;
  unsigned char* f8_cq;
  long ld_f8_cq;
  const float* f8_q_amax_prev;
  float* f8_q_scale_out;
  float* f8_q_amax_cur;
  // EPI_CPL_FWD: the conditioner's last product with the coupling forward fused. Column tile tn
  // holds features j in [128 tn, 128 tn + 128): tile columns 0..127 read weight rows j (s_hat),
  // columns 128..255 rows cf_dh + j (t), so each block sees both halves of its features. The
  // epilogue writes y = x e^s + t (fp32, cf_y), its bf16 copy (cf_yb, zero pad to cf_yb_width),
  // s_hat (bf16, C at column j - what the backward recomputes s from) and this block's share of
  // sum_j s into cf_ldj[tn][m] (one owner per entry: deterministic, no atomics).
  const float* cf_x;
  long ld_cf_x;
  float* cf_y;
  long ld_cf_y;
  bf16_t* cf_yb;
  long ld_cf_yb;
  int cf_yb_width;
  float* cf_ldj;
  long ld_cf_ldj;
  int cf_ldj_init;
  int cf_dh, cf_b_rows;
  float cf_scale;
  // cf_pair: weight / bias / f8_sb row offset of tile columns 128..255 (coupling: cf_dh).
  // cf_mode 1: the MAF transform of the same layer instead of the coupling (B, bias, f8_sb
  // point at the s_raw rows, cf_pair = -D reaches the mu rows): columns 0..127 = s_raw,
  // 128..255 = mu, y = u = (x - mu) e^-alpha, alpha = cf_scale tanh(s_raw / cf_scale), the
  // ldj share is -sum alpha, C = s_raw; with f8_cq also the e4m3 copy of u (delayed scale)
  int cf_pair;
  int cf_mode;
  // cf_mode 0 inverse: x = (y - t) e^-s from the layer's output y (cf_x) into cf_y / cf_yb, the
  // ldj share is -sum s; C (s_hat) may be null
  int cf_inverse;
  // cf_x_bf16: cf_x holds bf16 (a bf16 flow state: the MAF engine's bf16_state option). cf_y may
  // be null (a bf16 state out: only cf_yb is written)
  int cf_x_bf16;
  // persistent launches with dynamic tile claims (gemm256.hip, persist mode 2): this launch's
  // counter slot, 8 per-XCD claim counters + 1 finished-block counter (one 128-B line each,
  // QCTR_LINE ints apart), zero at launch start and zeroed again by the launch's last block
  int* qctr;
};
constexpr int QCTR_LINE = 32, QCTR_SLOT = 9 * QCTR_LINE;

// The alignment the LDS-staged epilogue's 16-B row accesses need (host side); shapes that miss
// it take the fragment-layout stores.
inline bool staged_ok(const GemmArgs& a, int epi) {
  auto al = [](const void* p) { return ((unsigned long)p & 15) == 0; };
  if (epi == EPI_BF16 || epi == EPI_BF16_RELUMASK) {
    if (a.N % 8 || a.ldc % 8 || !al(a.C)) return false;
    if (epi == EPI_BF16_RELUMASK && !a.aux_bits && (a.ld_aux % 8 || !al(a.aux))) return false;
    return true;
  }
  if (epi == EPI_CPL_BWD || epi == EPI_CPL_BWD_XB) {
    const bool xok = epi == EPI_CPL_BWD ? al(a.cpl_x) : ((unsigned long)a.cpl_x & 7) == 0;
    const bool gxok = a.cpl_gx_bf16 ? ((unsigned long)a.cpl_gx & 7) == 0 : al(a.cpl_gx);
    if (a.cpl_dh % 4 || a.ld_cpl_x % 4 || a.ld_cpl_gx % 4 || a.ld_cpl_dst % 4 || a.ld_aux % 4 ||
        !xok || !gxok || ((unsigned long)a.cpl_dst & 7) || ((unsigned long)a.aux & 7))
      return false;
  }
  const bool c_ok = (epi == EPI_CPL_BWD_XB && a.cpl_c_bf16) ? ((unsigned long)a.C & 7) == 0
                                                           : al(a.C);
  return a.N % 4 == 0 && a.ldc % 4 == 0 && a.c_split_stride % 4 == 0 && c_ok;
}

// Grouped launch: up to 4 independent problems (the weight gradients of one conditioner MLP),
// blocks [start[p], start[p+1]) belong to problem p, split-major inside a problem so the column
// tiles sharing an A panel sit on consecutive (XCD-remapped) block ids.
struct GroupArgs {
  GemmArgs p[4];
  int start[5];
  int nprob;
};

__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

// e4m3 mn-major half-tile image: 128 k-rows x 128 m-bytes, 16-B chunk cm of k-row k at chunk
// position cm ^ f8mn_swz(k). A ds_read_b64_tr_b8 32-lane half reads one chunk column of 8
// k-rows per 16-lane group, the two groups 16 k-rows apart: (k & 1, chunk position) is then
// distinct over those 16 rows, i.e. the 32 lanes cover 64 distinct banks (conflict-free).
__device__ __forceinline__ int f8mn_swz(int k) { return ((k >> 1) & 3) | (((k >> 4) & 1) << 2); }

// e4m3 fragment of the scaled 16x16x128 MFMA from an mn-major image: 16 k-bytes
// [64 ks + 16 g, +16) of tile row r0 + (lane & 15), g = lane >> 4 - the k-set the k-major
// read_frag gives a lane, so A and B fragments of either layout pair up. Two
// ds_read_b64_tr_b8: per 16-lane group, lane 2q + p points at k-row kb + q, bytes 8p..8p+7 of
// the row's chunk; lane i receives byte i of those 8 rows (measured on gfx950:
// tools/tr8_probe.hip). The ISA needs EXEC all ones: every lane always reads.
__device__ __forceinline__ v8s read_frag_f8mn(const char* lds_tile, int r0, int ks, int lane) {
  typedef int v2i_ __attribute__((ext_vector_type(2)));
  const int g = lane >> 4, q = (lane & 15) >> 1, p = lane & 1, cm = r0 >> 4;
  int w[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = ks * 64 + g * 16 + h * 8 + q;
    const LDS_AS v2i_* ptr =
        (const LDS_AS v2i_*)(lds_tile + k * 128 + ((cm ^ f8mn_swz(k)) << 4) + p * 8);
    const v2i_ t = __builtin_amdgcn_ds_read_tr8_b64_v2i32((LDS_AS v2i_*)ptr);
    w[2 * h] = t[0];
    w[2 * h + 1] = t[1];
  }
  typedef int v4i_ __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(v8s, (v4i_){w[0], w[1], w[2], w[3]});
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

// bf16 fragments (either layout) and e4m3 fragments (k-major: the same 16-B row read; mn-major:
// read_frag_f8mn)
template <bool KMAJOR, bool F8>
__device__ __forceinline__ v8s read_frag_any(const char* lds_tile, int r0, int ks, int lane) {
  if constexpr (F8 && !KMAJOR) return read_frag_f8mn(lds_tile, r0, ks, lane);
  else return read_frag<KMAJOR>(lds_tile, r0, ks, lane);
}

// max(v, 0) in one VALU op: fmaxf (and fmed3(v, 0, inf), which the compiler folds back into
// it) compiles to v_max_f32 v, v, v (IEEE-mode NaN canonicalisation) + v_max_f32 v, 0, v
// (profiles/r4/relu_asm_step_ab.jsonl: -0.1 to -0.45 ms per headline step)
__device__ __forceinline__ float relu_f(float v) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
  return r;
}

// Epilogue for one accumulator fragment: 4 consecutive n of output row m.
template <int EPI>
__device__ __forceinline__ void epi_store(const GemmArgs& a, v4f v, int m, int n, int split) {
  if (EPI == EPI_BF16) {
    if (a.bias) {
      const ushort4 bb = *reinterpret_cast<const ushort4*>(a.bias + n);
      v[0] += bf2f(bb.x); v[1] += bf2f(bb.y); v[2] += bf2f(bb.z); v[3] += bf2f(bb.w);
    }
    if (a.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = relu_f(v[r]);
    }
    ushort4 o;
    o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
    *reinterpret_cast<ushort4*>((bf16_t*)a.C + (long)m * a.ldc + n) = o;
  } else if (EPI == EPI_BF16_RELUMASK) {
    if (a.aux_bits) {
      const unsigned b = ((const unsigned char*)a.aux)[(long)m * a.ld_aux + (n >> 3)] >> (n & 4);
      v[0] = (b & 1u) ? v[0] : 0.f; v[1] = (b & 2u) ? v[1] : 0.f;
      v[2] = (b & 4u) ? v[2] : 0.f; v[3] = (b & 8u) ? v[3] : 0.f;
    } else {
      const ushort4 h = *reinterpret_cast<const ushort4*>(a.aux + (long)m * a.ld_aux + n);
      // bf16 > 0  <=>  sign bit clear and not +0
      v[0] = (h.x != 0 && !(h.x & 0x8000)) ? v[0] : 0.f;
      v[1] = (h.y != 0 && !(h.y & 0x8000)) ? v[1] : 0.f;
      v[2] = (h.z != 0 && !(h.z & 0x8000)) ? v[2] : 0.f;
      v[3] = (h.w != 0 && !(h.w & 0x8000)) ? v[3] : 0.f;
    }
    ushort4 o;
    o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
    *reinterpret_cast<ushort4*>((bf16_t*)a.C + (long)m * a.ldc + n) = o;
  } else if (EPI == EPI_F32) {
    if (a.cmask) {
      const uchar4 mk = *reinterpret_cast<const uchar4*>(a.cmask + (long)m * a.N + n);
      v[0] = mk.x ? v[0] : 0.f; v[1] = mk.y ? v[1] : 0.f; v[2] = mk.z ? v[2] : 0.f; v[3] = mk.w ? v[3] : 0.f;
    }
    float* cp = (float*)a.C + (long)split * a.c_split_stride + (long)m * a.ldc + n;
    *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
  } else {  // EPI_F32_ACC
    float* cp = (float*)a.C + (long)m * a.ldc + n;
    float4 o = *reinterpret_cast<float4*>(cp);
    o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
    *reinterpret_cast<float4*>(cp) = o;
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 staging image of one wave's sub-tile: [rows][64 n] in 128-B rows, 16-B chunk q of row r
// at q ^ (r & 7), and the two 8-B halves of a chunk swapped on rows with bit 3 set. The swap makes
// the fragment writes conflict-free: a ds_write_b64 lane group (16 lanes = 16 rows r0..r0+15,
// one 8-B slot each) covers 32 distinct dwords of the 32-bank write space, where rows r and r+8
// used to land on the same two banks (2-way; SQ_LDS_BANK_CONFLICT 0.23-0.30 per LDS cycle on
// the bf16 epilogues). The 16-B readback reads the same chunk and swaps the halves back.
__device__ __forceinline__ int bf_stage_off(int row, int slot) {
  return row * 128 + (((slot >> 1) ^ (row & 7)) << 4) + (((slot & 1) ^ ((row >> 3) & 1)) << 3);
}
__device__ __forceinline__ v4u bf_stage_fix(v4u v, bool swapped) {
  return swapped ? (v4u){v[2], v[3], v[0], v[1]} : v;
}

// LDS-staged epilogue. In the fragment layout one store instruction covers 16 rows x 32 B
// (bf16) or 16 rows x 64 B (fp32): 16 partial cache lines per instruction, which made the
// output write, not the MFMAs, the per-tile fixed cost at K <= 1024 (~15 us per 256^2 tile).
// A wave instead parks its WM x 64 sub-tile in its own LDS region (free once the main loop
// is done) and reads it back as whole rows, so every global store / aux / cmask / accumulate
// access moves 16 B per lane and full 128-B lines.
//   bf16 region: [WM rows][64 n] (128 B rows), 16-B chunk q of row r at q ^ (r & 7); the
//                8-B fragment writes land 2-way at worst, the 16-B reads conflict-free.
//   fp32 region: [64 rows][64 n] (256 B rows) per pass, chunk q of row r at q ^ (r & 7).
// acc[i][j]: n = n0 + i*16 + (lane>>4)*4 + r, m = m0 + j*16 + (lane&15)  (m0/n0 = the wave's
// sub-tile origin), i < 4, j < NJ (WM = 16*NJ). Requires N % 8 == 0, ldc % 8 == 0 (bf16) /
// ldc % 4 == 0 (fp32) and a 16-B aligned C (checked by the launchers).
// J0 / NJA: the rows handled are accumulator blocks [J0, J0 + NJ) of a [4][NJA] array (m0 is the
// origin of block J0), so a caller short of LDS can stage a sub-tile in several calls.
template <int EPI, int NJ, bool F8 = false, int J0 = 0, int NJA = NJ>
__device__ __forceinline__ void epi_tile_staged(const GemmArgs& a, const v4f (&acc)[4][NJA],
                                                int m0, int n0, int split, char* region,
                                                int lane) {
  const int g = lane >> 4, c = lane & 15;
  if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_RELUMASK) {
    float bv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[i][r] = 0.f;
    if (EPI == EPI_BF16 && a.bias) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + i * 16 + g * 4;
        if (n < a.N) {
          const ushort4 bb = *reinterpret_cast<const ushort4*>(a.bias + n);
          bv[i][0] = bf2f(bb.x); bv[i][1] = bf2f(bb.y); bv[i][2] = bf2f(bb.z); bv[i][3] = bf2f(bb.w);
        }
      }
    }
    const bool relu = EPI == EPI_BF16 && a.relu;
    // fp8 operands: rank-1 dequantisation factor sa[m] * sb[n] (1 for bf16 operands)
    float sn[4][4], smj[NJ];
    constexpr bool f8 = F8 && (EPI == EPI_BF16 || EPI == EPI_BF16_RELUMASK);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) sn[i][r] = 1.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) smj[j] = 1.f;
    if constexpr (f8) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int n = n0 + i * 16 + g * 4;
        n = n < a.N ? n : a.N - 4;
        const float4 t = *reinterpret_cast<const float4*>(a.f8_sb + n);
        sn[i][0] = t.x; sn[i][1] = t.y; sn[i][2] = t.z; sn[i][3] = t.w;
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int m = m0 + j * 16 + c;
        m = m < a.M ? m : a.M - 1;
        smj[j] = a.f8_sa_per_row ? a.f8_sa[m] : a.f8_sa[0];
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int row = j * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v0 = fmaf(acc[i][J0 + j][0], smj[j] * sn[i][0], bv[i][0]);
        float v1 = fmaf(acc[i][J0 + j][1], smj[j] * sn[i][1], bv[i][1]);
        float v2 = fmaf(acc[i][J0 + j][2], smj[j] * sn[i][2], bv[i][2]);
        float v3 = fmaf(acc[i][J0 + j][3], smj[j] * sn[i][3], bv[i][3]);
        if (relu) { v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3); }
        const unsigned lo = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
        const unsigned hi = (unsigned)f2bf(v2) | ((unsigned)f2bf(v3) << 16);
        const int slot = i * 4 + g;  // 8-B slot of the 128-B row
        *(LDS_AS v2u*)(region + bf_stage_off(row, slot)) = (v2u){lo, hi};
      }
    }
    // aux rows (ReLU mask) for every readback row, in flight while the LDS writes drain
    const int q = lane & 7;
    uint4 hv[NJ * 2];
    unsigned hb[NJ * 2];
    if constexpr (EPI == EPI_BF16_RELUMASK) {
      if (a.aux_bits) {
#pragma unroll
        for (int it = 0; it < NJ * 2; ++it) {
          int m = m0 + it * 8 + (lane >> 3), n = n0 + q * 8;
          m = m < a.M ? m : a.M - 1;
          n = n < a.N ? n : a.N - 8;
          hb[it] = ((const unsigned char*)a.aux)[(long)m * a.ld_aux + (n >> 3)];
        }
      } else {
#pragma unroll
        for (int it = 0; it < NJ * 2; ++it) {
          int m = m0 + it * 8 + (lane >> 3), n = n0 + q * 8;
          m = m < a.M ? m : a.M - 1;
          n = n < a.N ? n : a.N - 8;
          hv[it] = *reinterpret_cast<const uint4*>(a.aux + (long)m * a.ld_aux + n);
        }
      }
    }
    float qinv = 1.f, qamax = 0.f;
    const bool f8out = F8 && (EPI == EPI_BF16 || EPI == EPI_BF16_RELUMASK) && a.f8_cq != nullptr;
    if (f8out) {
      const float ap = *a.f8_q_amax_prev;
      const float qs = ap > 0.f ? ap / 448.f : 1.f;
      qinv = 1.f / qs;
      if (blockIdx.x == 0 && threadIdx.x == 0) *a.f8_q_scale_out = qs;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < NJ * 2; ++it) {
      const int row = it * 8 + (lane >> 3);
      // (row >> 3) & 1 == it & 1: the half swap of bf_stage_off is a compile-time register swap
      const v4u v = bf_stage_fix(*(const LDS_AS v4u*)(region + row * 128 + ((q ^ (row & 7)) << 4)),
                                 (it & 1) != 0);
      const int m = m0 + row, n = n0 + q * 8;
      if (m < a.M && n < a.N) {
        uint4 o = make_uint4(v[0], v[1], v[2], v[3]);
        if constexpr (EPI == EPI_BF16_RELUMASK) {
          // keep element e iff aux_e > 0 (bf16: sign clear and not +0), per 16-bit half
          // branch-free, both halves at once: bit 15 / 31 of p is set iff that bf16 half is in
          // [1, 0x7fff] (> 0; see the bitmask epilogue below), and (p << 1) - (p >> 15)
          // widens each marked bit to its whole half (mod 2^32: bit 31's shifted-out carry is
          // what turns 0 - 0x10000 into 0xffff0000)
          auto keep = [](unsigned hw) {
            const unsigned p = ((hw & 0x7fff7fffu) + 0x7fff7fffu) & ~hw & 0x80008000u;
            return (p << 1) - (p >> 15);
          };
          if (a.aux_bits) {
            const unsigned b = hb[it];
            auto kb = [b](int e) {
              return ((b >> e) & 1u ? 0xffffu : 0u) | ((b >> (e + 1)) & 1u ? 0xffff0000u : 0u);
            };
            o.x &= kb(0); o.y &= kb(2); o.z &= kb(4); o.w &= kb(6);
          } else {
            const uint4 h = hv[it];
            o.x &= keep(h.x); o.y &= keep(h.y); o.z &= keep(h.z); o.w &= keep(h.w);
          }
        }
        if (EPI == EPI_BF16 && a.mask_out) {  // 1(y > 0) of the stored bf16, 8 bits per lane
          // branch-free: half h > 0 (bf16) <=> h in [1, 0x7fff] <=> bit 15 of
          // ((h & 0x7fff) + 0x7fff) & ~h; both halves at once (no carry: each sum <= 0xfffe),
          // then bits 15 / 31 of the 4 words gathered to bits 2e / 2e + 1 of one byte
          auto pos = [](unsigned w) { return ((w & 0x7fff7fffu) + 0x7fff7fffu) & ~w & 0x80008000u; };
          const unsigned t = (pos(o.x) >> 15) | (pos(o.y) >> 13) | (pos(o.z) >> 11) | (pos(o.w) >> 9);
          const unsigned bits = (t | (t >> 15)) & 0xffu;
          a.mask_out[(long)m * a.ld_mask + (n >> 3)] = (unsigned char)bits;
        }
        // (C may be null on the e4m3 paths that only need the e4m3 copy: MAF engine, e4m3
        // weight gradients)
        if (!F8 || a.C) *reinterpret_cast<uint4*>((bf16_t*)a.C + (long)m * a.ldc + n) = o;
        if (f8out) {
          const unsigned w4[4] = {o.x, o.y, o.z, o.w};
          float f[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[2 * e] = __uint_as_float(w4[e] << 16);
            f[2 * e + 1] = __uint_as_float(w4[e] & 0xffff0000u);
          }
          int q0 = 0, q1 = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            qamax = fmaxf(qamax, fabsf(f[e]));
            f[e] = fminf(fmaxf(f[e] * qinv, -448.f), 448.f);
          }
          q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], q0, false);
          q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], q0, true);
          q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], q1, false);
          q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], q1, true);
          *reinterpret_cast<uint2*>(a.f8_cq + (long)m * a.ld_f8_cq + n) =
              make_uint2((unsigned)q0, (unsigned)q1);
        }
      }
    }
    if (f8out) {  // one (mostly skipped) atomic per wave into the block's amax slot
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) qamax = fmaxf(qamax, __shfl_xor(qamax, off));
      if (lane == 0) amax_slot_atomic(a.f8_q_amax_cur, qamax);
    }
  } else {
    // fp32 path: passes of 32 rows (8 KiB of the wave's region). Every global operand a pass
    // reads (old C, and for EPI_CPL_BWD s_hat and x) is loaded for all its rows before the LDS
    // readback, from clamped addresses, so a pass waits out ONE load round trip. (Loading s_hat
    // / x per row inside the readback loop serialised 32 round trips per wave: the fused
    // coupling-backward epilogue took 52.6 us per tile, profiles/r2_g256_stamps_b65536.jsonl.)
    // 16-row accumulator blocks per pass (e4m3 fused backward: 1 - its loop leaves fewer
    // registers for the pass's preloaded operands, 264 B/lane of scratch at 2)
    constexpr bool CPLB = EPI == EPI_CPL_BWD || EPI == EPI_CPL_BWD_XB;
    constexpr bool XB = EPI == EPI_CPL_BWD_XB;   // x operand in bf16
    // timing probes of the fused backward epilogue (docs/PERF_NOTES.md round 6; wrong results):
    // NF_PROBE_CB_NOEPI no epilogue, NF_PROBE_CB_NOLOAD no C / s_hat / x reads,
    // NF_PROBE_CB_NOSTORE no gx / dst / e4m3 stores
#ifdef NF_PROBE_CB_NOEPI
    if constexpr (CPLB) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          s += acc[i][J0 + j][0] + acc[i][J0 + j][1] + acc[i][J0 + j][2] + acc[i][J0 + j][3];
      if (s == 1.2345e-30f) a.cpl_gx[lane] = s;
      return;
    }
#endif
#ifdef NF_PROBE_CB_NOSTORE
    const bool cb_st = a.cpl_scale == 1.2345e-30f;
#else
    constexpr bool cb_st = true;
#endif
    constexpr int PJ = (F8 && CPLB) ? 1 : 2;
    constexpr int PIT = PJ * 4;       // readback iterations (4 rows each) per pass
    // e4m3 operands (EPI_CPL_BWD): acc * f8_sa[0] * f8_sb[n], and with f8_cq the e4m3 copy of
    // dst = [dS | dT] (the next fp8 input-gradient product's operand) under a delayed scale
    constexpr bool f8c = F8 && CPLB;
    // e4m3 weight gradients (EPI_F32): dW = acc * sa * sb, both per-tensor scales
    float w8 = 1.f;
    if constexpr (F8 && EPI == EPI_F32) w8 = a.f8_sa[0] * a.f8_sb[0];
    float qinv = 1.f, qamax = 0.f;
    if (f8c && a.f8_cq) {
      const float ap = *a.f8_q_amax_prev;
      const float qs = ap > 0.f ? ap / 448.f : 1.f;
      qinv = 1.f / qs;
      if (blockIdx.x == 0 && threadIdx.x == 0) *a.f8_q_scale_out = qs;
    }
#pragma unroll
    for (int hj = 0; hj < NJ / PJ; ++hj) {
      if (hj) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int jj = 0; jj < PJ; ++jj) {
        const int row = jj * 16 + c;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *(LDS_AS v4f*)(region + row * 256 + (((i * 4 + g) ^ (row & 7)) << 4)) = acc[i][J0 + hj * PJ + jj];
      }
      // global operands of this pass's rows, in flight while the LDS writes drain
      const int q = lane & 15;
      float4 cv[PIT];
      float4 xp[PIT];
      ushort4 sp[PIT], xh[PIT];
#ifdef NF_PROBE_CB_NOLOAD
#pragma unroll
      for (int it = 0; it < PIT; ++it) {
        cv[it] = xp[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        sp[it] = xh[it] = make_ushort4(0, 0, 0, 0);
      }
      if constexpr (EPI == EPI_F32_ACC || (CPLB && false)) {
#else
      if constexpr (EPI == EPI_F32_ACC || CPLB) {
#endif
#pragma unroll
        for (int it = 0; it < PIT; ++it) {
          int m = m0 + hj * 16 * PJ + it * 4 + (lane >> 4), n = n0 + q * 4;
          m = m < a.M ? m : a.M - 1;
          n = n < a.N ? n : a.N - 4;
          if constexpr (XB) {
            if (a.cpl_c_bf16) {
              const ushort4 h =
                  *reinterpret_cast<const ushort4*>((const bf16_t*)a.C + (long)m * a.ldc + n);
              cv[it] = make_float4(bf2f(h.x), bf2f(h.y), bf2f(h.z), bf2f(h.w));
            } else {
              cv[it] = *reinterpret_cast<const float4*>((const float*)a.C + (long)m * a.ldc + n);
            }
          } else {
            cv[it] = *reinterpret_cast<const float4*>((const float*)a.C + (long)m * a.ldc + n);
          }
          if constexpr (CPLB) {
            const int nx = n < a.cpl_dh ? n : a.cpl_dh - 4;
            sp[it] = *reinterpret_cast<const ushort4*>(a.aux + (long)m * a.ld_aux + nx);
            if constexpr (XB)
              xh[it] = *reinterpret_cast<const ushort4*>(
                  reinterpret_cast<const bf16_t*>(a.cpl_x) + (long)m * a.ld_cpl_x + nx);
            else
              xp[it] = *reinterpret_cast<const float4*>(a.cpl_x + (long)m * a.ld_cpl_x + nx);
          }
        }
      }
      float sc8[4] = {1.f, 1.f, 1.f, 1.f};
      if constexpr (f8c) {
        int n = n0 + q * 4;
        n = n < a.N ? n : a.N - 4;
        const float4 t = *reinterpret_cast<const float4*>(a.f8_sb + n);
        const float s0 = a.f8_sa[0];
        sc8[0] = s0 * t.x; sc8[1] = s0 * t.y; sc8[2] = s0 * t.z; sc8[3] = s0 * t.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < PIT; ++it) {
        const int row = it * 4 + (lane >> 4);
        v4f v = *(const LDS_AS v4f*)(region + row * 256 + ((q ^ (row & 7)) << 4));
        if constexpr (f8c) {
          v[0] *= sc8[0]; v[1] *= sc8[1]; v[2] *= sc8[2]; v[3] *= sc8[3];
        }
        if constexpr (F8 && EPI == EPI_F32) {
          v[0] *= w8; v[1] *= w8; v[2] *= w8; v[3] *= w8;
        }
        const int m = m0 + hj * 16 * PJ + row, n = n0 + q * 4;
        if (m < a.M && n < a.N && cb_st) {
          if constexpr (CPLB) {
            const float4 o = cv[it];
            const float gy[4] = {o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]};
            bf16_t* drow = a.cpl_dst + (long)m * a.ld_cpl_dst;
            if (n < a.cpl_dh) {
              const ushort4 sh = sp[it];
              const float shv[4] = {bf2f(sh.x), bf2f(sh.y), bf2f(sh.z), bf2f(sh.w)};
              float xs[4];
              if constexpr (XB) {
                const ushort4 xv = xh[it];
                xs[0] = bf2f(xv.x); xs[1] = bf2f(xv.y); xs[2] = bf2f(xv.z); xs[3] = bf2f(xv.w);
              } else {
                const float4 xv = xp[it];
                xs[0] = xv.x; xs[1] = xv.y; xs[2] = xv.z; xs[3] = xv.w;
              }
              const float inv = __builtin_amdgcn_rcpf(a.cpl_scale);   // v_rcp (1 ulp): an IEEE division per element group here
              float gx[4], dsh[4], d1v[4];
              if (a.cpl_mode) {   // MAF: dst = [dmu | ds_raw], x = u of layer l-1
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float t = fast_tanhf(shv[e] * inv);
                  gx[e] = gy[e] * __expf(-a.cpl_scale * t);
                  dsh[e] = -gx[e];
                  d1v[e] = (a.cpl_c - gy[e] * xs[e]) * (1.f - t * t);
                }
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float sv = a.cpl_scale * fast_tanhf(shv[e]);
                  const float es = __expf(sv);
                  const float ds = fmaf(gy[e] * xs[e], es, a.cpl_c);
                  dsh[e] = ds * (a.cpl_scale - sv * sv * inv);
                  gx[e] = gy[e] * es;
                  d1v[e] = gy[e];
                }
              }
              if (XB && a.cpl_gx_bf16) {
                ushort4 gh;
                gh.x = f2bf(gx[0]); gh.y = f2bf(gx[1]); gh.z = f2bf(gx[2]); gh.w = f2bf(gx[3]);
                *reinterpret_cast<ushort4*>(reinterpret_cast<bf16_t*>(a.cpl_gx) +
                                            (long)m * a.ld_cpl_gx + n) = gh;
              } else {
                *reinterpret_cast<float4*>(a.cpl_gx + (long)m * a.ld_cpl_gx + n) =
                    make_float4(gx[0], gx[1], gx[2], gx[3]);
              }
              ushort4 d0, d1;
              d0.x = f2bf(dsh[0]); d0.y = f2bf(dsh[1]); d0.z = f2bf(dsh[2]); d0.w = f2bf(dsh[3]);
              d1.x = f2bf(d1v[0]); d1.y = f2bf(d1v[1]); d1.z = f2bf(d1v[2]); d1.w = f2bf(d1v[3]);
              if (!F8 || a.cpl_dst) {   // null (e4m3 only): the e4m3 copy alone (MAF engine)
                *reinterpret_cast<ushort4*>(drow + n) = d0;
                *reinterpret_cast<ushort4*>(drow + a.cpl_dh + n) = d1;
              }
              if (f8c && a.f8_cq) {
                float f0[4], f1[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  qamax = fmaxf(qamax, fmaxf(fabsf(dsh[e]), fabsf(d1v[e])));
                  f0[e] = fminf(fmaxf(dsh[e] * qinv, -448.f), 448.f);
                  f1[e] = fminf(fmaxf(d1v[e] * qinv, -448.f), 448.f);
                }
                int q0 = 0, q1 = 0;
                q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f0[0], f0[1], q0, false);
                q0 = __builtin_amdgcn_cvt_pk_fp8_f32(f0[2], f0[3], q0, true);
                q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f1[0], f1[1], q1, false);
                q1 = __builtin_amdgcn_cvt_pk_fp8_f32(f1[2], f1[3], q1, true);
                unsigned char* qr = a.f8_cq + (long)m * a.ld_f8_cq;
                *reinterpret_cast<int*>(qr + n) = q0;
                *reinterpret_cast<int*>(qr + a.cpl_dh + n) = q1;
              }
            } else if ((!F8 || a.cpl_dst) && a.cpl_dh + n < a.cpl_pad) {   // zero the dst pad [2 Dh, pad)
              *reinterpret_cast<ushort4*>(drow + a.cpl_dh + n) = make_ushort4(0, 0, 0, 0);
            }
          } else if (EPI == EPI_F32) {
            if (a.cmask) {
              const uchar4 mk = *reinterpret_cast<const uchar4*>(a.cmask + (long)m * a.N + n);
              v[0] = mk.x ? v[0] : 0.f; v[1] = mk.y ? v[1] : 0.f;
              v[2] = mk.z ? v[2] : 0.f; v[3] = mk.w ? v[3] : 0.f;
            }
            float* cp = (float*)a.C + (long)split * a.c_split_stride + (long)m * a.ldc + n;
            *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            const float4 o = cv[it];
            *reinterpret_cast<float4*>((float*)a.C + (long)m * a.ldc + n) =
                make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
          }
        }
      }
    }
    if (f8c && a.f8_cq) {   // one (mostly skipped) atomic per wave into the block's amax slot
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) qamax = fmaxf(qamax, __shfl_xor(qamax, off));
      if (lane == 0) amax_slot_atomic(a.f8_q_amax_cur, qamax);
    }
  }
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace gemm
}  // namespace nf
