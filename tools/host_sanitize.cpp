// Host-code sanitizer check (AddressSanitizer + UndefinedBehaviorSanitizer, CPU only):
// randomized and edge-case runs of the pure-host planning code the launchers use.
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
//       -I csrc/include tools/host_sanitize.cpp -o /tmp/host_sanitize && /tmp/host_sanitize
// (tests/test_host_sanitizers.py builds and runs it; GPU code is never sanitized on this pool.)
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <vector>

#include "wgrad_pack.h"

static int fail(const char* what, int a, int b) {
  std::printf("FAIL %s (%d, %d)\n", what, a, b);
  return 1;
}

int main() {
  std::mt19937 rng(1234);
  int checked = 0;
  for (int iter = 0; iter < 20000; ++iter) {
    const int ntiles = 8 * (1 + (int)(rng() % 32));          // 8 .. 256
    // random partition of [0, ntiles) into 1 .. 40 segments
    const int want = 1 + (int)(rng() % 40);
    std::vector<int> cuts{0, ntiles};
    for (int i = 0; i < want - 1; ++i) cuts.push_back((int)(rng() % (ntiles + 1)));
    std::sort(cuts.begin(), cuts.end());
    std::vector<int> lo, n;
    for (size_t i = 0; i + 1 < cuts.size(); ++i) {
      lo.push_back(cuts[i]);
      n.push_back(cuts[i + 1] - cuts[i]);   // empty segments allowed (zero-length problems)
    }
    std::vector<unsigned short> perm(ntiles, 0xffff);
    if (!nf::wgrad_xcd_perm((int)lo.size(), lo.data(), n.data(), ntiles, perm.data()))
      return fail("valid partition rejected", ntiles, (int)lo.size());
    std::vector<int> seen(ntiles, 0);
    for (int p = 0; p < ntiles; ++p) {
      if (perm[p] >= ntiles) return fail("perm out of range", p, perm[p]);
      if (seen[perm[p]]++) return fail("perm not a bijection", p, perm[p]);
    }
    // a segment no larger than a bin, placed when every bin still had room for it, is whole
    // in one bin for the RealNVP-32 shape (16 / 16 / 8 tiles): checked separately below
    ++checked;
  }
  // RealNVP-32 launch: 6 layers x (16, 16, 8) + one 16 = 256 tiles -> every problem in one bin
  {
    std::vector<int> lo, n;
    int at = 0;
    for (int l = 0; l < 6; ++l)
      for (int s : {16, 16, 8}) { lo.push_back(at); n.push_back(s); at += s; }
    lo.push_back(at); n.push_back(16); at += 16;
    std::vector<unsigned short> perm(256);
    if (!nf::wgrad_xcd_perm((int)lo.size(), lo.data(), n.data(), 256, perm.data()))
      return fail("realnvp launch rejected", 256, (int)lo.size());
    for (size_t i = 0; i < lo.size(); ++i) {
      int bin = -1;
      for (int p = 0; p < 256; ++p)
        if (perm[p] >= lo[i] && perm[p] < lo[i] + n[i]) {
          if (bin < 0) bin = p / 32;
          else if (bin != p / 32) return fail("problem split across XCD bins", (int)i, p);
        }
    }
  }
  // malformed inputs are refused without touching perm
  {
    unsigned short perm[16];
    int lo[2] = {0, 8}, n[2] = {8, 9};
    if (nf::wgrad_xcd_perm(2, lo, n, 16, perm)) return fail("overlong segment accepted", 0, 0);
    int lo2[1] = {0}, n2[1] = {12};
    if (nf::wgrad_xcd_perm(1, lo2, n2, 12, perm)) return fail("ntiles % 8 accepted", 0, 0);
    if (nf::wgrad_xcd_perm(1, lo2, n2, 16, perm)) return fail("short cover accepted", 0, 0);
    int lo3[1] = {-1}, n3[1] = {16};
    if (nf::wgrad_xcd_perm(1, lo3, n3, 16, perm)) return fail("negative start accepted", 0, 0);
  }
  std::printf("host_sanitize ok: %d random packings\n", checked);
  return 0;
}
