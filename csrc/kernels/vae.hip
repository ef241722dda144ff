// Whole training step of the reference's main workload - the amortized planar-flow VAE of
// src/learning_mnist.py (encoder 784 -> 64 x3 -> 2dz + 2dz K + K, K per-sample planar flows,
// Bernoulli decoder dz -> 64 x3 -> 784; objective optimization.py:66-92 with the estimator
// fixes of inference/elbo.py) - in two launches instead of ~60 small ones (gfx950).
//
// The model has 145k parameters and the reference trains it at batch 128: every GEMM is a few
// hundred KFLOP and the composite step is launch-bound (0.61 ms in a hipGraph,
// profiles/r1_configs_final.jsonl). So:
//
// Phase 1 (vae_rows_kernel, one block per R = 8 rows, 8 waves): the forward (encoder, split,
// reparameterised z0 with in-kernel Philox noise, K planar layers with the u_hat
// reparameterisation, decoder, Bernoulli-from-logits + standard-normal log p, per-row free
// energy) and the whole input-gradient chain back to the encoder's first hidden layer, every
// activation in LDS. Each block writes the activations X and output gradients dY of every
// linear layer ([B][dim], row-major) for phase 2 - no weight-gradient atomics (16 blocks
// adding 145k gradients each would run at 16/256 of the chip's atomic rate).
// Phase 2 (vae_wgrad_kernel): all weight / bias gradients dW = dY^T X, db = sum_b dY as 64x64
// tiles with the batch as the reduction, plain stores into the flat gradient buffer; block 0
// also reduces the per-row free energies to the loss.
//
// fp32 throughout (VALU FMA; the f32-input MFMA runs at the same rate on gfx950): the
// reference trains in float64, and these products are far too small for bf16 MFMA to matter.
//
// Layouts in LDS: activations row-major [R][dim] (the next product reads float4 runs along
// its reduction dim), gradients transposed [dim][R] (the input-gradient product broadcasts the
// R values of one output as two float4 reads). Dense forward: LPO lanes per output each take
// float4 chunks of the reduction dim, then an xor-shuffle reduction over the LPO lanes.
// Dense input gradient: one lane per input feature, the outputs split over the 8 waves,
// partial sums combined through LDS.
#include "nf_common.h"

namespace nf {
namespace vae {

constexpr int R = 8;          // rows per block
constexpr int NW = 8;         // waves per block
constexpr int NT = NW * 64;
constexpr int H = 64;         // hidden width (wave width)
constexpr int MAXL = 4;       // hidden layers
constexpr int MAXZ = 64;      // latent dim
constexpr int MAXK = 8;       // planar layers
constexpr float LOG2PI = 1.8378770664093453f;

// Sum over aligned groups of N lanes (N = 16, 32, 64), result in every lane of the group:
// the steps inside a 16-lane row are DPP moves (quad_perm xor 1 / xor 2, row_half_mirror,
// row_mirror) that cost a VALU slot each, only the cross-row steps go through ds_bpermute.
// A chain of ds_bpermute shuffles costs an LDS round trip per step - the planar flow's dot
// products (six of them per layer per row) sit on the step's critical path.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, true));
}
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  v += dppf<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);   // row_half_mirror
  v += dppf<0x140>(v);   // row_mirror
  if constexpr (N >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (N >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ float wsum(float v) { return group_sum<64>(v); }

struct Mlp {                  // parameters of one FlatMLP: hidden W[l] [out][in], b[l], out Wo/bo
  const float* W[MAXL];
  const float* b[MAXL];
  const float* Wo;
  const float* bo;
};

struct RowsArgs {
  Mlp enc, dec;
  const float* x;            // [B][Din] binary images
  const float* eps_in;       // [B][dz] fixed noise (tests) or null -> Philox
  unsigned seed;
  const long* offset;        // device Philox offset (advanced once per step by the engine)
  const float* beta;         // device scalar
  float inv_b;               // 1 / B (the mean over the batch)
  int B, Din, dz, K, L, De;
  // phase-2 operands, row-major [B][dim]
  float* eact;               // [L][B][H] encoder hidden activations
  float* egrad;              // [L][B][H] their gradients (pre-activation, ReLU applied)
  float* gphi;               // [B][De] encoder output gradient
  float* zk;                 // [B][dz] decoder input
  float* dact;               // [L][B][H]
  float* dgrad;              // [L][B][H]
  float* dl;                 // [B][Din] logits gradient
  float* frow;               // [B] per-row free energy
  float* zk_out;             // optional [B][dz] z_K copy (tests), may be null
  float* ldj_out;            // optional [B]
};

// ------------------------------------------------------------------ block-level dense products
// Y = act(X W^T + b), X [R][ldx] in LDS (16-B aligned rows), W [O][I] global (I % 4 == 0),
// Y [R][ldy] (out_t = false) or transposed [O][R] (out_t = true) in LDS.
template <int LPO, int NCH>
__device__ __forceinline__ void dense_fwd(const float* X, int ldx, const float* __restrict__ W,
                                          const float* __restrict__ bias, int O, int I, float* Y,
                                          int ldy, bool relu, bool out_t, int wave, int lane) {
  // NCH: float4 chunks per lane (ceil(I / 4 / LPO)). The weights of the NEXT output group are
  // loaded before this group's FMAs / shuffle reduction, so one L2 round trip is exposed per
  // layer instead of one per output group.
  constexpr int OPW = 64 / LPO;
  const int sub = lane % LPO, og = lane / LPO;
  const int nch = I >> 2;
  auto load_w = [&](int o, float4 (&w)[NCH]) {
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
      const int c = sub + LPO * t;
      w[t] = (o < O && c < nch) ? *reinterpret_cast<const float4*>(W + (long)o * I + 4 * c)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float4 wc[NCH], wn[NCH];
  int o0 = wave * OPW;
  load_w(o0 + og, wc);
  for (; o0 < O; o0 += NW * OPW) {
    const int o = o0 + og;
    load_w(o + NW * OPW, wn);
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
      const int c = sub + LPO * t;
      if (c < nch) {
        const float4 w = wc[t];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float4 xv = *reinterpret_cast<const float4*>(X + r * ldx + 4 * c);
          acc[r] = fmaf(w.x, xv.x, fmaf(w.y, xv.y, fmaf(w.z, xv.z, fmaf(w.w, xv.w, acc[r]))));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = group_sum<LPO>(acc[r]);
    if (o < O && sub == 0) {
      const float bv = bias[o];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float v = acc[r] + bv;
        if (relu) v = fmaxf(v, 0.f);
        if (out_t) Y[o * R + r] = v;
        else Y[r * ldy + o] = v;
      }
    }
#pragma unroll
    for (int t = 0; t < NCH; ++t) wc[t] = wn[t];
  }
}

__device__ __forceinline__ void dense_fwd_any(const float* X, int ldx, const float* W,
                                              const float* bias, int O, int I, float* Y, int ldy,
                                              bool relu, bool out_t, int wave, int lane) {
  // lanes per output x float4 chunks per lane must cover I / 4 (I <= 1024)
  if (I > 512) dense_fwd<64, 4>(X, ldx, W, bias, O, I, Y, ldy, relu, out_t, wave, lane);
  else if (I > 256) dense_fwd<64, 2>(X, ldx, W, bias, O, I, Y, ldy, relu, out_t, wave, lane);
  else if (I > 128) dense_fwd<64, 1>(X, ldx, W, bias, O, I, Y, ldy, relu, out_t, wave, lane);
  else if (I > 64) dense_fwd<32, 1>(X, ldx, W, bias, O, I, Y, ldy, relu, out_t, wave, lane);
  else dense_fwd<16, 1>(X, ldx, W, bias, O, I, Y, ldy, relu, out_t, wave, lane);
}

// dX = dY W (dY transposed [O][R] in LDS, W [O][I] global, I <= 64), times 1(act > 0) when
// act ([R][lda] row-major) is given; dX transposed [I][R]. red: NW * R * 64 floats of LDS.
// Ends with a block barrier.
__device__ __forceinline__ void dense_dx(const float* dYt, const float* __restrict__ W, int O,
                                         int I, const float* act, int lda, float* dXt, float* red,
                                         int wave, int lane) {
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  const int per = (O + NW - 1) / NW;
  const int ob = wave * per, oe = min(O, ob + per);
  if (lane < I) {
#pragma unroll 8
    for (int o = ob; o < oe; ++o) {
      const float w = W[(long)o * I + lane];
      const float4 g0 = *reinterpret_cast<const float4*>(dYt + o * R);
      const float4 g1 = *reinterpret_cast<const float4*>(dYt + o * R + 4);
      acc[0] = fmaf(g0.x, w, acc[0]); acc[1] = fmaf(g0.y, w, acc[1]);
      acc[2] = fmaf(g0.z, w, acc[2]); acc[3] = fmaf(g0.w, w, acc[3]);
      acc[4] = fmaf(g1.x, w, acc[4]); acc[5] = fmaf(g1.y, w, acc[5]);
      acc[6] = fmaf(g1.z, w, acc[6]); acc[7] = fmaf(g1.w, w, acc[7]);
    }
  }
  float* mine = red + (wave * 64 + lane) * R;
  *reinterpret_cast<float4*>(mine) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(mine + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  __syncthreads();
  // combine: thread t -> (feature i = t / R, row r = t % R)
  for (int t = threadIdx.x; t < I * R; t += NT) {
    const int i = t / R, r = t % R;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[(w * 64 + i) * R + r];
    if (act && !(act[r * lda + i] > 0.f)) s = 0.f;
    dXt[i * R + r] = s;
  }
  __syncthreads();
}

// copy a row-major [R][ld] LDS block (first n columns) to global rows [row0 + r][n]
__device__ __forceinline__ void store_rows(const float* src, int ld, int n, float* dst, long row0,
                                           int nrows) {
  for (int t = threadIdx.x; t < R * n; t += NT) {
    const int r = t / n, c = t % n;
    if (r < nrows) dst[(row0 + r) * n + c] = src[r * ld + c];
  }
}
// transposed [n][R] LDS block -> global rows [row0 + r][n]
// src [n][R] (LDS, transposed) -> rows row0.. of dst with row pitch ld (>= n)
__device__ __forceinline__ void store_rows_t(const float* src, int n, float* dst, long row0,
                                             int nrows, int ld = 0) {
  if (ld <= 0) ld = n;
  for (int t = threadIdx.x; t < R * n; t += NT) {
    const int r = t / n, c = t % n;
    if (r < nrows) dst[(row0 + r) * ld + c] = src[c * R + r];
  }
}

__device__ __forceinline__ float softplusf_(float x) {
  return fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void __launch_bounds__(NT, 1) vae_rows_kernel(RowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long row0 = (long)blockIdx.x * R;
  const int nrows = (int)min((long)R, a.B - row0);
  const int Din = a.Din, dz = a.dz, K = a.K, L = a.L, De = a.De;
  const int ldx = Din, ldp = (De + 3) & ~3;
  // LDS carve-up (floats)
  float* xs = lds;                            // [R][Din]
  float* ea = xs + R * Din;                   // [L][R][H]
  float* phi = ea + MAXL * R * H;             // [R][ldp]
  float* zst = phi + R * ldp;                 // [R][MAXK + 1][64]
  float* epsb = zst + R * (MAXK + 1) * 64;    // [R][64]
  float* da = epsb + R * 64;                  // [L][R][H]
  float* lgt = da + MAXL * R * H;             // [Din][R] logits, then dL/dlogits
  float* gA = lgt + Din * R;                  // [64][R]
  float* gB = gA + 64 * R;                    // [64][R]
  float* gph = gB + 64 * R;                   // [De][R]
  float* red = gph + De * R;                  // [NW][64][R]
  float* zkb = red + NW * 64 * R;             // [R][64] decoder input (row-major)
  float* rs = zkb + R * 64;                   // per-row scalars [R][4]: lq0, ldj

  // ---- inputs
  for (int t = threadIdx.x; t < R * (Din / 4); t += NT) {
    const int r = t / (Din / 4), c = t % (Din / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < nrows) v = *reinterpret_cast<const float4*>(a.x + (row0 + r) * Din + 4 * c);
    *reinterpret_cast<float4*>(xs + r * ldx + 4 * c) = v;
  }
  __syncthreads();
  // ---- encoder
  const float* in = xs;
  int ldi = ldx, I = Din;
  for (int l = 0; l < L; ++l) {
    dense_fwd_any(in, ldi, a.enc.W[l], a.enc.b[l], H, I, ea + l * R * H, H, true, false, wave, lane);
    __syncthreads();
    in = ea + l * R * H; ldi = H; I = H;
  }
  dense_fwd_any(in, ldi, a.enc.Wo, a.enc.bo, De, I, phi, ldp, false, false, wave, lane);
  __syncthreads();
  const float beta = *a.beta;
  const float s = a.inv_b;
  // ---- base sample + planar flows: wave w owns row w, lane d owns latent coordinate d
  const int r = wave;
  const bool rok = r < nrows, dok = lane < dz;
  const float* pr = phi + r * ldp;
  if (rok) {
    float mu = dok ? pr[lane] : 0.f, lv = dok ? pr[dz + lane] : 0.f;
    float e = 0.f;
    if (dok) {
      if (a.eps_in) {
        e = a.eps_in[(row0 + r) * dz + lane];
      } else {
        const unsigned long long off = (unsigned long long)*a.offset;
        const Philox4 q = philox4x32_10((unsigned)(row0 + r), (unsigned)(lane >> 1),
                                        (unsigned)off, (unsigned)(off >> 32) ^ 0x5EAu, a.seed,
                                        0xA5A5u);
        float n0, n1;
        box_muller(q.x, q.y, n0, n1);
        e = (lane & 1) ? n1 : n0;
      }
    }
    float z = dok ? fmaf(__expf(0.5f * lv), e, mu) : 0.f;
    epsb[r * 64 + lane] = e;
    const float lq0 = -0.5f * dz * LOG2PI - 0.5f * wsum(lv) - 0.5f * wsum(e * e);
    float ldj = 0.f;
    for (int k = 0; k < K; ++k) {
      zst[(r * (MAXK + 1) + k) * 64 + lane] = z;
      const float w = dok ? pr[2 * dz + k * dz + lane] : 0.f;
      const float u = dok ? pr[2 * dz + K * dz + k * dz + lane] : 0.f;
      const float b = pr[2 * dz + 2 * K * dz + k];
      const float wu = wsum(w * u), nw = wsum(w * w);
      const float coef = nw > 0.f ? (-1.f + softplusf_(wu) - wu) / nw : 0.f;
      const float uh = fmaf(coef, w, u);
      const float h = tanhf(wsum(w * z) + b);
      const float eta = wsum(w * uh);
      ldj += __logf(fabsf(1.f + (1.f - h * h) * eta) + 1e-7f);
      z = fmaf(uh, h, z);
    }
    zst[(r * (MAXK + 1) + K) * 64 + lane] = z;
    zkb[r * 64 + lane] = z;
    if (lane == 0) { rs[r * 4 + 0] = lq0; rs[r * 4 + 1] = ldj; }
    if (dok) {
      a.zk[(row0 + r) * dz + lane] = z;
      if (a.zk_out) a.zk_out[(row0 + r) * dz + lane] = z;
    }
    if (lane == 0 && a.ldj_out) a.ldj_out[row0 + r] = ldj;
  } else {
    zkb[r * 64 + lane] = 0.f;
  }
  __syncthreads();
  // ---- decoder
  in = zkb; ldi = 64; I = dz;
  for (int l = 0; l < L; ++l) {
    dense_fwd_any(in, ldi, a.dec.W[l], a.dec.b[l], H, I, da + l * R * H, H, true, false, wave, lane);
    __syncthreads();
    in = da + l * R * H; ldi = H; I = H;
  }
  dense_fwd_any(in, ldi, a.dec.Wo, a.dec.bo, Din, I, lgt, 0, false, true, wave, lane);
  __syncthreads();
  // ---- log p(x, z_K), per-row free energy, dL/dlogits (in place)
  if (rok) {
    float lp = 0.f;
    for (int i = lane; i < Din; i += 64) {
      const float l = lgt[i * R + r], xv = xs[r * ldx + i];
      lp += xv * l - softplusf_(l);
      lgt[i * R + r] = -beta * s * (xv - sigmoidf_(l));
    }
    const float zK = zst[(r * (MAXK + 1) + K) * 64 + lane];
    lp = wsum(lp) - 0.5f * dz * LOG2PI - 0.5f * wsum(dok ? zK * zK : 0.f);
    if (lane == 0) a.frow[row0 + r] = rs[r * 4 + 0] - rs[r * 4 + 1] - beta * lp;
  } else {
    for (int i = lane; i < Din; i += 64) lgt[i * R + r] = 0.f;
  }
  __syncthreads();
  store_rows_t(lgt, Din, a.dl, row0, nrows);
  for (int l = 0; l < L; ++l) store_rows(da + l * R * H, H, H, a.dact + (long)l * a.B * H, row0, nrows);
  // ---- decoder input-gradient chain
  const float* gin = lgt;
  float* gout = gA;
  for (int l = L - 1; l >= 0; --l) {
    dense_dx(gin, l == L - 1 ? a.dec.Wo : a.dec.W[l + 1], l == L - 1 ? Din : H, H,
             da + l * R * H, H, gout, red, wave, lane);
    store_rows_t(gout, H, a.dgrad + (long)l * a.B * H, row0, nrows);
    gin = gout;
    gout = gout == gA ? gB : gA;
  }
  dense_dx(gin, a.dec.W[0], H, dz, nullptr, 0, gout, red, wave, lane);   // dL/dz_K (decoder)
  // ---- planar backward + reparameterisation: wave w owns row w
  if (rok) {
    const float zK = zst[(r * (MAXK + 1) + K) * 64 + lane];
    float g = dok ? gout[lane * R + r] + beta * s * zK : 0.f;   // + d(-beta log N(z_K))
    const float c = -s;                                          // dF / d ldj
    for (int k = K - 1; k >= 0; --k) {
      const float z = zst[(r * (MAXK + 1) + k) * 64 + lane];
      const float w = dok ? pr[2 * dz + k * dz + lane] : 0.f;
      const float u = dok ? pr[2 * dz + K * dz + k * dz + lane] : 0.f;
      const float b = pr[2 * dz + 2 * K * dz + k];
      const float wu = wsum(w * u), nw = wsum(w * w);
      const float sp = softplusf_(wu);
      const float coef = nw > 0.f ? (-1.f + sp - wu) / nw : 0.f;
      const float uh = fmaf(coef, w, u);
      const float h = tanhf(wsum(w * z) + b);
      const float hp = 1.f - h * h, hpp = -2.f * h * hp;
      const float eta = wsum(w * uh);
      const float psi = 1.f + hp * eta;
      const float ipsi = copysignf(1.f / (fabsf(psi) + 1e-7f), psi);
      const float rr = c * hp * ipsi;
      const float gu = wsum(g * uh);
      const float dA = gu * hp + c * hpp * eta * ipsi;
      const float dUh = g * h + rr * w;
      float dW = dA * z + rr * uh;
      float dU = dUh;
      if (nw > 0.f) {   // u_hat = u + coef(w.u, |w|^2) w
        const float t = wsum(dUh * w);
        const float sg = sigmoidf_(wu);                          // m'(x) = sigmoid(x)
        const float dcu = (sg - 1.f) / nw;                       // d coef / d(w.u)
        dU = fmaf(t * dcu, w, dUh);
        dW += coef * dUh + t * (dcu * u - 2.f * coef / nw * w);
      }
      g = fmaf(dA, w, g);
      if (dok) {
        gph[(2 * dz + k * dz + lane) * R + r] = dW;
        gph[(2 * dz + K * dz + k * dz + lane) * R + r] = dU;
      }
      if (lane == 0) gph[(2 * dz + 2 * K * dz + k) * R + r] = dA;
    }
    if (dok) {
      const float lv = pr[dz + lane], e = epsb[r * 64 + lane];
      gph[lane * R + r] = g;                                              // dF/dmu
      gph[(dz + lane) * R + r] = fmaf(g * e * 0.5f, __expf(0.5f * lv), -0.5f * s);   // dF/dlogvar
    }
  } else {
    for (int j = lane; j < De; j += 64) gph[j * R + r] = 0.f;
  }
  __syncthreads();
  store_rows_t(gph, De, a.gphi, row0, nrows, (De + 3) & ~3);   // 16-B aligned rows
  for (int l = 0; l < L; ++l) store_rows(ea + l * R * H, H, H, a.eact + (long)l * a.B * H, row0, nrows);
  // ---- encoder input-gradient chain (down to the first hidden layer's pre-activation)
  gin = gph;
  gout = gA;
  for (int l = L - 1; l >= 0; --l) {
    dense_dx(gin, l == L - 1 ? a.enc.Wo : a.enc.W[l + 1], l == L - 1 ? De : H, H,
             ea + l * R * H, H, gout, red, wave, lane);
    store_rows_t(gout, H, a.egrad + (long)l * a.B * H, row0, nrows);
    gin = gout;
    gout = gout == gA ? gB : gA;
  }
}

// ------------------------------------------------------------------ phase 2: weight gradients
constexpr int MAXP = 12;
struct WgProb {
  const float* dY;   // [B][ldy], ldy = O rounded up to a multiple of 4 (16-B aligned float4 rows)
  const float* X;    // [B][I]
  float* dW;         // [O][I]
  float* db;         // [O]
  int O, I, tiles_i, tile0, ldy;
};
struct WgArgs {
  WgProb p[MAXP];
  int np, B;
  const float* frow;
  float* loss;
  float inv_b;
};

// one 64 (o) x 64 (i) tile per block, 256 threads = 4 x 4 outputs each; the batch is staged in
// chunks of 128 rows (the reference batch in ONE chunk: a single memory round trip per block),
// float4 loads (O % 4 == 0 and I % 4 == 0 for every VAE layer); tn == 0 blocks also produce db
constexpr int WB = 128;
__global__ void __launch_bounds__(256) vae_wgrad_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) float wl[];
  float* sy = wl;                   // [WB][68]
  float* sx = wl + WB * 68;         // [WB][68]
  int p = 0;
  for (int q = 1; q < a.np; ++q)
    if ((int)blockIdx.x >= a.p[q].tile0) p = q;
  const WgProb& pb = a.p[p];
  const int local = blockIdx.x - pb.tile0;
  const int to = local / pb.tiles_i, ti = local % pb.tiles_i;
  const int o0 = to * 64, i0 = ti * 64;
  const int tid = threadIdx.x, ty = tid / 16, tx = tid % 16;   // outputs o0+4ty.., i0+4tx..
  float acc[4][4] = {};
  float accb[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b0 = 0; b0 < a.B; b0 += WB) {
    // 16 float4 per operand tile row-chunk: t -> (row bb, float4 column c4)
#pragma unroll 4
    for (int t = tid; t < WB * 16; t += 256) {
      const int bb = t / 16, c4 = (t % 16) * 4, bi = b0 + bb;
      float4 y = make_float4(0.f, 0.f, 0.f, 0.f), xv = y;
      if (bi < a.B && o0 + c4 < pb.O) y = *reinterpret_cast<const float4*>(pb.dY + (long)bi * pb.ldy + o0 + c4);
      if (bi < a.B && i0 + c4 < pb.I) xv = *reinterpret_cast<const float4*>(pb.X + (long)bi * pb.I + i0 + c4);
      *reinterpret_cast<float4*>(sy + bb * 68 + c4) = y;
      *reinterpret_cast<float4*>(sx + bb * 68 + c4) = xv;
    }
    __syncthreads();
    const int nb = min(WB, a.B - b0);
#pragma unroll 4
    for (int bb = 0; bb < nb; ++bb) {
      const float4 y4 = *reinterpret_cast<const float4*>(sy + bb * 68 + 4 * ty);
      const float4 x4 = *reinterpret_cast<const float4*>(sx + bb * 68 + 4 * tx);
      const float yv[4] = {y4.x, y4.y, y4.z, y4.w}, xv[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        accb[u] += yv[u];
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(yv[u], xv[v], acc[u][v]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int o = o0 + 4 * ty + u;
    if (o >= pb.O) continue;
    const int i = i0 + 4 * tx;
    if (i + 3 < pb.I) {
      *reinterpret_cast<float4*>(pb.dW + (long)o * pb.I + i) =
          make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (i + v < pb.I) pb.dW[(long)o * pb.I + i + v] = acc[u][v];
    }
    if (ti == 0 && tx == 0) pb.db[o] = accb[u];
  }
  if (blockIdx.x == 0) {   // loss = mean of the per-row free energies (fixed order)
    __shared__ float part[4];
    float v = 0.f;
    for (int i = tid; i < a.B; i += 256) v += a.frow[i];
    v = wave_sum(v);
    if ((tid & 63) == 0) part[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) *a.loss = (part[0] + part[1] + part[2] + part[3]) * a.inv_b;
  }
}

}  // namespace vae
}  // namespace nf

using namespace nf::vae;

size_t nf_vae_rows_lds_bytes(int Din, int dz, int K, int De) {
  (void)dz; (void)K;
  const int ldp = (De + 3) & ~3;
  const size_t f = (size_t)R * Din + MAXL * R * H + (size_t)R * ldp + R * (MAXK + 1) * 64 +
                   R * 64 + MAXL * R * H + (size_t)Din * R + 64 * R + 64 * R + (size_t)De * R +
                   NW * 64 * R + R * 64 + R * 4;
  return f * sizeof(float);
}

void nf_launch_vae_step(const NfVaeParams& prm, const float* x, const float* eps_in, unsigned seed,
                        const long* offset, const float* beta, int B, int Din, int dz, int K,
                        int L, float* ws_eact, float* ws_egrad, float* ws_gphi, float* ws_zk,
                        float* ws_dact, float* ws_dgrad, float* ws_dl, float* frow, float* loss,
                        float* zk_out, float* ldj_out, const NfVaeGrads& grd, hipStream_t stream) {
  RowsArgs a{};
  for (int l = 0; l < L; ++l) {
    a.enc.W[l] = prm.enc_W[l]; a.enc.b[l] = prm.enc_b[l];
    a.dec.W[l] = prm.dec_W[l]; a.dec.b[l] = prm.dec_b[l];
  }
  a.enc.Wo = prm.enc_Wo; a.enc.bo = prm.enc_bo;
  a.dec.Wo = prm.dec_Wo; a.dec.bo = prm.dec_bo;
  a.x = x; a.eps_in = eps_in; a.seed = seed; a.offset = offset; a.beta = beta;
  a.inv_b = 1.f / B;
  a.B = B; a.Din = Din; a.dz = dz; a.K = K; a.L = L; a.De = 2 * dz + 2 * dz * K + K;
  a.eact = ws_eact; a.egrad = ws_egrad; a.gphi = ws_gphi; a.zk = ws_zk;
  a.dact = ws_dact; a.dgrad = ws_dgrad; a.dl = ws_dl; a.frow = frow;
  a.zk_out = zk_out; a.ldj_out = ldj_out;
  const size_t lds = nf_vae_rows_lds_bytes(Din, dz, K, a.De);
  static bool attr_set = false;
  if (!attr_set) {
    NF_HIP_CHECK(hipFuncSetAttribute((const void*)vae_rows_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
    NF_HIP_CHECK(hipFuncSetAttribute((const void*)vae_wgrad_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(2 * WB * 68 * sizeof(float))));
    attr_set = true;
  }
  hipLaunchKernelGGL(vae_rows_kernel, dim3((B + R - 1) / R), dim3(NT), lds, stream, a);
  NF_HIP_CHECK(hipGetLastError());

  // phase 2: weight gradients of the 2 (L + 1) linears
  WgArgs w{};
  int tiles = 0;
  auto add = [&](const float* dY, const float* X, float* dW, float* db, int O, int I) {
    WgProb& q = w.p[w.np++];
    q.dY = dY; q.X = X; q.dW = dW; q.db = db; q.O = O; q.I = I; q.ldy = (O + 3) & ~3;
    q.tiles_i = (I + 63) / 64;
    q.tile0 = tiles;
    tiles += ((O + 63) / 64) * q.tiles_i;
  };
  const long BH = (long)B * H;
  add(ws_egrad, x, grd.enc_W[0], grd.enc_b[0], H, Din);
  for (int l = 1; l < L; ++l)
    add(ws_egrad + l * BH, ws_eact + (l - 1) * BH, grd.enc_W[l], grd.enc_b[l], H, H);
  add(ws_gphi, ws_eact + (L - 1) * BH, grd.enc_Wo, grd.enc_bo, a.De, H);
  add(ws_dgrad, ws_zk, grd.dec_W[0], grd.dec_b[0], H, dz);
  for (int l = 1; l < L; ++l)
    add(ws_dgrad + l * BH, ws_dact + (l - 1) * BH, grd.dec_W[l], grd.dec_b[l], H, H);
  add(ws_dl, ws_dact + (L - 1) * BH, grd.dec_Wo, grd.dec_bo, Din, H);
  w.B = B; w.frow = frow; w.loss = loss; w.inv_b = 1.f / B;
  hipLaunchKernelGGL(vae_wgrad_kernel, dim3(tiles), dim3(256), 2 * WB * 68 * sizeof(float),
                     stream, w);
  NF_HIP_CHECK(hipGetLastError());
}
