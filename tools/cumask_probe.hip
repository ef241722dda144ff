// CU-mask stream probe (gfx950): which XCD / shader engine / CU each bit of a
// hipExtStreamCreateWithCUMask mask selects, and whether a hipGraph captured on a CU-masked
// stream keeps the mask when it is replayed.
//
//   hipcc -O3 --offload-arch=gfx950 tools/cumask_probe.hip -o cumask_probe && ./cumask_probe
//
// Output: one JSON line per mask bit {"bit", "xcc", "hw_id"} (HW_ID raw: CU_ID [11:8], SH_ID [12],
// SE_ID [15:13] on gfx9), then {"graph": ...} lines with the XCC ids seen by a 256-block kernel
// launched eagerly on a one-XCD mask, and replayed from a graph captured on that stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void where_kernel(unsigned* out, int spin) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  // keep the block resident a little so many blocks of one launch spread over the allowed CUs
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);   // ~0.1 us per 8 sleeps
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int words = (ncu + 31) / 32;
  unsigned* d = nullptr;
  CK(hipMalloc(&d, 2 * 1024 * sizeof(unsigned)));
  std::vector<unsigned> h(2 * 1024);
  for (int b = 0; b < ncu; ++b) {
    std::vector<uint32_t> m(words, 0u);
    m[b / 32] = 1u << (b % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
    hipLaunchKernelGGL(where_kernel, dim3(1), dim3(64), 0, s, d, 0);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, 2 * sizeof(unsigned), hipMemcpyDeviceToHost));
    printf("{\"bit\": %d, \"xcc\": %u, \"hw_id\": %u, \"cu\": %u, \"sh\": %u, \"se\": %u}\n", b,
           h[0] & 7u, h[1], (h[1] >> 8) & 15u, (h[1] >> 12) & 1u, (h[1] >> 13) & 7u);
    CK(hipStreamDestroy(s));
  }
  // multi-block launches under a few masks: distinct (XCC, HW_ID & CU/SH/SE) seen, eagerly and
  // replayed from a graph captured on the masked stream (1024 blocks, each resident ~20 us)
  hipStream_t plain;
  CK(hipStreamCreate(&plain));
  const int NB = 1024;
  unsigned* d2 = nullptr;
  CK(hipMalloc(&d2, 2 * NB * sizeof(unsigned)));
  std::vector<unsigned> h2(2 * NB);
  struct MaskCase { const char* name; std::vector<uint32_t> m; };
  std::vector<MaskCase> cases;
  cases.push_back({"bit0", std::vector<uint32_t>(words, 0u)});
  cases.back().m[0] = 1u;
  cases.push_back({"low16_of_each_word", std::vector<uint32_t>(words, 0x0000ffffu)});
  cases.push_back({"first_half_words", std::vector<uint32_t>(words, 0u)});
  for (int w = 0; w < words / 2; ++w) cases.back().m[w] = 0xffffffffu;
  cases.push_back({"even_bits", std::vector<uint32_t>(words, 0x55555555u)});
  auto census = [&](const char* mask, const char* how) {
    CK(hipMemcpy(h2.data(), d2, 2 * NB * sizeof(unsigned), hipMemcpyDeviceToHost));
    std::set<unsigned> xs, cus;
    for (int i = 0; i < NB; ++i) {
      xs.insert(h2[2 * i] & 7u);
      cus.insert(((h2[2 * i] & 7u) << 16) | ((h2[2 * i + 1] >> 8) & 0xffu));
    }
    printf("{\"mask\": \"%s\", \"how\": \"%s\", \"n_xcc\": %zu, \"n_cu\": %zu, \"xcc\": [", mask,
           how, xs.size(), cus.size());
    bool first = true;
    for (unsigned x : xs) {
      printf("%s%u", first ? "" : ", ", x);
      first = false;
    }
    printf("]}\n");
  };
  for (auto& c : cases) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, words, c.m.data()));
    hipLaunchKernelGGL(where_kernel, dim3(NB), dim3(64), 0, s, d2, 2000);
    CK(hipStreamSynchronize(s));
    census(c.name, "eager");
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(where_kernel, dim3(NB), dim3(64), 0, s, d2, 2000);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipMemset(d2, 0, 2 * NB * sizeof(unsigned)));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    census(c.name, "graph_on_masked_stream");
    CK(hipMemset(d2, 0, 2 * NB * sizeof(unsigned)));
    CK(hipGraphLaunch(ge, plain));
    CK(hipStreamSynchronize(plain));
    census(c.name, "graph_on_plain_stream");
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
  }
  hipLaunchKernelGGL(where_kernel, dim3(NB), dim3(64), 0, plain, d2, 2000);
  CK(hipStreamSynchronize(plain));
  census("none", "plain_stream");
  CK(hipStreamDestroy(plain));
  CK(hipFree(d2));
  CK(hipFree(d));
  return 0;
}
