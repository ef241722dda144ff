// Batched bf16 transposes: one launch refreshes W^T for every conditioner weight of a model
// (models/realnvp.py `wt_dgrad`): the input-gradient GEMMs dx = dy W then run as dy (W^T)^T,
// the NT instantiation of gemm256 with both operands k-major (b128 LDS fragment reads) instead
// of the NN one (transposed ds_read_b64_tr_b16 reads of W), measured 5-7 % faster per product
// (profiles/r1_dgrad_nt_vs_nn.txt). The weights are small next to the activations (72 M
// parameters, 144 MB bf16 each way), so the per-step transpose costs tens of microseconds.
//
// Descriptors (TrDesc, a device table the caller builds once: the weight buffers never move)
// list src [rows][cols] (row stride lds) -> dst [cols][rows] (row stride ldd) and the first
// 64x64 tile of each problem; a block finds its problem by a binary search of the table, stages the tile in LDS with a padded row (no bank conflicts
// on the column read) and writes whole 128-B rows.
#include "nf_common.h"

namespace nf {

struct TrDesc {
  long src, dst;           // element addresses (bf16)
  int rows, cols;          // of src
  int lds, ldd;            // row strides (elements)
  int tile0, pad;
};

__global__ void __launch_bounds__(256) transpose_bf16_batched_kernel(const TrDesc* __restrict__ d,
                                                                     int n) {
  __shared__ __attribute__((aligned(16))) unsigned short t[64][66];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;          // last problem with tile0 <= b (tile0 ascending)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].tile0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const int p = lo;
  const TrDesc e = d[p];
  const int tcn = (e.cols + 63) / 64;
  const int local = b - e.tile0;
  const int r0 = (local / tcn) * 64, c0 = (local % tcn) * 64;
  const unsigned short* src = reinterpret_cast<const unsigned short*>(e.src);
  unsigned short* dst = reinterpret_cast<unsigned short*>(e.dst);
  const bool vec = ((e.src | e.dst) & 15) == 0 && ((e.lds | e.ldd | e.rows | e.cols) & 7) == 0;
  if (vec) {   // 16-B rows in and out: 2 chunks of 8 elements per thread each way
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = threadIdx.x + 256 * k, r = q >> 3, cc = (q & 7) * 8;
      const int gr = r0 + r, gc = c0 + cc;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < e.rows && gc < e.cols)
        v = *reinterpret_cast<const uint4*>(src + (long)gr * e.lds + gc);
      unsigned* tw = reinterpret_cast<unsigned*>(&t[r][cc]);
      tw[0] = v.x; tw[1] = v.y; tw[2] = v.z; tw[3] = v.w;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = threadIdx.x + 256 * k, j = q >> 3, rr = (q & 7) * 8;
      const int gj = c0 + j, gr = r0 + rr;
      if (gj >= e.cols || gr >= e.rows) continue;
      unsigned w[4];
#pragma unroll
      for (int h = 0; h < 4; ++h)
        w[h] = (unsigned)t[rr + 2 * h][j] | ((unsigned)t[rr + 2 * h + 1][j] << 16);
      *reinterpret_cast<uint4*>(dst + (long)gj * e.ldd + gr) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return;
  }
  // 256 threads: 2-element (4 B) column pairs x 8 row groups
  const int cp = (threadIdx.x & 31) * 2, rg = threadIdx.x >> 5;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = rg + 8 * i, gr = r0 + r, gc = c0 + cp;
    unsigned short v0 = 0, v1 = 0;
    if (gr < e.rows) {
      if (gc + 1 < e.cols && (((long)gr * e.lds + gc) & 1) == 0) {
        const unsigned w = *reinterpret_cast<const unsigned*>(src + (long)gr * e.lds + gc);
        v0 = (unsigned short)(w & 0xffffu);
        v1 = (unsigned short)(w >> 16);
      } else {
        if (gc < e.cols) v0 = src[(long)gr * e.lds + gc];
        if (gc + 1 < e.cols) v1 = src[(long)gr * e.lds + gc + 1];
      }
    }
    t[r][cp] = v0;
    t[r][cp + 1] = v1;
  }
  __syncthreads();
  // dst row = source column c0 + j, dst columns r0 .. r0 + 63
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int j = rg + 8 * i, gj = c0 + j, gr = r0 + cp;
    if (gj >= e.cols) continue;
    const unsigned short v0 = t[cp][j], v1 = t[cp + 1][j];
    unsigned short* o = dst + (long)gj * e.ldd + gr;
    if (gr + 1 < e.rows && (((long)gj * e.ldd + gr) & 1) == 0) {
      *reinterpret_cast<unsigned*>(o) = (unsigned)v0 | ((unsigned)v1 << 16);
    } else {
      if (gr < e.rows) o[0] = v0;
      if (gr + 1 < e.rows) o[1] = v1;
    }
  }
}

}  // namespace nf

void nf_launch_transpose_bf16_batched(const void* desc, int n, int total_tiles,
                                      hipStream_t stream) {
  if (n <= 0 || total_tiles <= 0) return;
  hipLaunchKernelGGL(nf::transpose_bf16_batched_kernel, dim3(total_tiles), dim3(256), 0, stream,
                     (const nf::TrDesc*)desc, n);
  NF_HIP_CHECK(hipGetLastError());
}
