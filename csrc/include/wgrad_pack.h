// Host-side planning for the weight-gradient launches (csrc/kernels/gemm256.hip
// nf_launch_gemm256_tn_multi): pack a launch's problem segments into the 8 XCD block ranges.
//
// A launch computes `ntiles` consecutive tiles (one per CU); block position p runs on XCD
// p / (ntiles / 8) after xcd_remap. Problem i owns the launch-relative tile range
// [seg_lo[i], seg_lo[i] + seg_n[i]). First-fit decreasing: the largest segments first, each into
// the fullest bin it fits in whole, else split over the emptiest bins. perm[p] = launch-relative
// tile run at position p; the result is a permutation of [0, ntiles).
//
// Pure host code without HIP dependencies, so tools/host_sanitize.cpp checks it under
// -fsanitize=address,undefined on the CPU.
#pragma once

namespace nf {

constexpr int WGRAD_PACK_MAX_SEGS = 64;

// returns false (perm untouched) when the shape is not packable: ntiles % 8 != 0, too many
// segments, or segments that do not tile [0, ntiles) exactly
inline bool wgrad_xcd_perm(int nseg, const int* seg_lo, const int* seg_n, int ntiles,
                           unsigned short* perm) {
  if (ntiles <= 0 || ntiles % 8 || nseg <= 0 || nseg > WGRAD_PACK_MAX_SEGS) return false;
  int total = 0;
  for (int i = 0; i < nseg; ++i) {
    if (seg_n[i] < 0 || seg_lo[i] < 0 || seg_lo[i] + seg_n[i] > ntiles) return false;
    total += seg_n[i];
  }
  if (total != ntiles) return false;
  const int cap = ntiles / 8;
  int order[WGRAD_PACK_MAX_SEGS];
  for (int i = 0; i < nseg; ++i) order[i] = i;
  for (int i = 1; i < nseg; ++i)   // stable insertion sort, largest segment first
    for (int j = i; j > 0 && seg_n[order[j]] > seg_n[order[j - 1]]; --j) {
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  int fill[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int oi = 0; oi < nseg; ++oi) {
    int lo = seg_lo[order[oi]], n = seg_n[order[oi]];
    while (n > 0) {
      int b = -1;   // the fullest bin that takes the whole rest, else the emptiest bin
      for (int x = 0; x < 8; ++x)
        if (cap - fill[x] >= n && (b < 0 || fill[x] > fill[b])) b = x;
      if (b < 0)
        for (int x = 0; x < 8; ++x)
          if (b < 0 || fill[x] < fill[b]) b = x;
      const int take = n < cap - fill[b] ? n : cap - fill[b];
      for (int k = 0; k < take; ++k) perm[b * cap + fill[b] + k] = (unsigned short)(lo + k);
      fill[b] += take;
      lo += take;
      n -= take;
    }
  }
  return true;
}

}  // namespace nf
