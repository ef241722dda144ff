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
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);
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
  std::vector<int> bit_xcc(ncu, -1);
  for (int b = 0; b < ncu; ++b) {
    std::vector<uint32_t> m(words, 0u);
    m[b / 32] = 1u << (b % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
    hipLaunchKernelGGL(where_kernel, dim3(1), dim3(64), 0, s, d, 0);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, 2 * sizeof(unsigned), hipMemcpyDeviceToHost));
    bit_xcc[b] = (int)(h[0] & 7u);
    printf("{\"bit\": %d, \"xcc\": %u, \"hw_id\": %u, \"cu\": %u, \"sh\": %u, \"se\": %u}\n", b,
           h[0] & 7u, h[1], (h[1] >> 8) & 15u, (h[1] >> 12) & 1u, (h[1] >> 13) & 7u);
    CK(hipStreamDestroy(s));
  }
  // a mask of every bit that landed on XCC 0, then a 256-block launch: eager and graph replay
  std::vector<uint32_t> m(words, 0u);
  int nbits = 0;
  for (int b = 0; b < ncu; ++b)
    if (bit_xcc[b] == 0) {
      m[b / 32] |= 1u << (b % 32);
      ++nbits;
    }
  hipStream_t s, plain;
  CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
  CK(hipStreamCreate(&plain));
  auto report = [&](const char* tag) {
    CK(hipMemcpy(h.data(), d, 2 * 256 * sizeof(unsigned), hipMemcpyDeviceToHost));
    std::set<unsigned> xs;
    for (int i = 0; i < 256; ++i) xs.insert(h[2 * i] & 7u);
    printf("{\"graph\": \"%s\", \"mask_bits\": %d, \"xcc_seen\": [", tag, nbits);
    bool first = true;
    for (unsigned x : xs) {
      printf("%s%u", first ? "" : ", ", x);
      first = false;
    }
    printf("]}\n");
  };
  hipLaunchKernelGGL(where_kernel, dim3(256), dim3(64), 0, s, d, 200);
  CK(hipStreamSynchronize(s));
  report("eager_masked_stream");
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(where_kernel, dim3(256), dim3(64), 0, s, d, 200);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipMemset(d, 0xff, 2 * 256 * sizeof(unsigned)));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  report("graph_replayed_on_masked_stream");
  CK(hipMemset(d, 0xff, 2 * 256 * sizeof(unsigned)));
  CK(hipGraphLaunch(ge, plain));
  CK(hipStreamSynchronize(plain));
  report("graph_replayed_on_plain_stream");
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(plain));
  CK(hipFree(d));
  return 0;
}
