// Descriptor table of the multi-layer weight-gradient launches (gemm256.hip
// gemm256_multi_kernel, gemm_tn4w.hip gemm_tn4w_kernel): travels in the kernarg segment.
#pragma once
#include "gemm_tile.h"

namespace nf {
namespace gemm {
namespace g256 {

// Weight gradients of MANY layers per launch, no split-K. A launch covers the global tile range
// [tile0, tile0 + ntiles) of a problem list; every block owns one whole 256x256 output tile and
// streams the full K (= batch) range, so there are no fp32 slabs and no reduce launch, and the
// launch size is chosen by the caller (a multiple of the CU count: 40 tiles per RealNVP layer x
// 32 layers = 1280 = 5 x 256). The descriptors travel in the kernarg segment (scalar loads).
struct TnDesc {
  const bf16_t* A;
  const bf16_t* B;
  float* C;
  float* db;
  const unsigned short* tiles;   // active tile ids of a masked problem (others never launched)
  const unsigned char* cmask;    // [M][N] 0/1 applied to dW (MADE), or null
  int lda, ldb, ldc, M, N, K, start, staged;
  int sidx;                      // e4m3 launches: scale-pool indices of dy (low 16 bits) and x
};
constexpr int TN_MULTI_MAX = 40;   // 80-B descriptors: the table stays inside the 4 KiB kernarg
constexpr int TN_PERM_MAX = 256;   // + 512 B: 3724 B of kernarg with 40 descriptors
struct TnMulti {
  TnDesc d[TN_MULTI_MAX];
  int n, tile0, ntiles, use_perm;
  // XCD packing (gemm_wgrad_xcd_pack): block position -> tile offset. Positions
  // [x * ntiles/8, (x+1) * ntiles/8) run on XCD x (xcd_remap), so the permutation keeps each
  // problem's tiles - which share A / B panels - inside one XCD's L2 where they fit
  unsigned short perm[TN_PERM_MAX];
  const float* scales;   // e4m3 launches: per-tensor dequantisation scales, indexed by sidx
};
static_assert(sizeof(TnMulti) <= 4096, "TnMulti must fit the 4 KiB kernarg segment");

}  // namespace g256


// 4-wave 128x128-per-wave TN kernel (gemm_tn4w.hip); false: shape not supported (caller falls
// back to gemm256_multi_kernel)
bool launch_tn4w_multi(const g256::TnMulti& t, hipStream_t stream);

}  // namespace gemm
}  // namespace nf
