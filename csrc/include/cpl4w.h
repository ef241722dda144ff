// Fused coupling-forward product on 4 fat waves (gemm_cpl4w.hip): arguments and launcher.
#pragma once
#include "nf_common.h"

namespace nf {
namespace gemm {
namespace cpl4w {

struct Args {
  const bf16_t* A;     // h [M][K]
  long lda;
  const bf16_t* W;     // [w_rows][K]: rows [0, Dh) s_hat, [Dh, 2 Dh) t
  long ldw;
  int w_rows;
  const bf16_t* bias;  // [w_rows] or null
  bf16_t* st;          // s_hat [M][>= Dh] or null (inverse)
  long ld_st;
  const float* x;      // [M][Dh]
  long ld_x;
  float* y;            // [M][Dh]
  long ld_y;
  bf16_t* yb;          // [M][yb_width] or null
  long ld_yb;
  int yb_width;
  float* ldjp;         // [ldj_rows][M]
  long ld_ldjp;
  int ldj_rows, ldj_init;
  int M, K, Dh, ntn;
  float scale;
  int inverse;
};

}  // namespace cpl4w

// false: shape / alignment not supported (the caller runs the 8-wave EPI_CPL_FWD product)
bool launch_cpl4w(const cpl4w::Args& a, hipStream_t stream);

}  // namespace gemm
}  // namespace nf
