// Which XCD runs workgroup b of a one-block-per-CU launch (512 threads, 128 KiB LDS, like the
// 256x256 GEMM kernels)? The GEMMs' xcd_remap assumes b -> XCD b % 8 (round-robin dispatch).
//   hipcc -O3 --offload-arch=gfx950 tools/xcd_map_probe.hip -o xcd_map_probe && ./xcd_map_probe
// Output: one JSON line per launch size: the fraction of blocks with xcc == b % 8, and the XCD
// of the first 16 blocks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void __launch_bounds__(512, 1) where_kernel(unsigned* out, int spin) {
  __shared__ char lds[128 * 1024];
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  lds[threadIdx.x] = (char)xcc;   // keep the LDS allocation
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc & 7u) | ((unsigned)lds[5] << 8);
}

int main() {
  unsigned* d = nullptr;
  CK(hipMalloc(&d, 4096 * sizeof(unsigned)));
  std::vector<unsigned> h(4096);
  for (int nb : {256, 512, 1024}) {
    hipLaunchKernelGGL(where_kernel, dim3(nb), dim3(512), 0, 0, d, 200);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, nb * sizeof(unsigned), hipMemcpyDeviceToHost));
    int match = 0;
    for (int b = 0; b < nb; ++b) match += (h[b] & 7u) == (unsigned)(b % 8);
    printf("{\"blocks\": %d, \"frac_xcc_eq_b_mod_8\": %.3f, \"first16\": [", nb, match / (double)nb);
    for (int b = 0; b < 16; ++b) printf("%s%u", b ? ", " : "", h[b] & 7u);
    printf("]}\n");
  }
  CK(hipFree(d));
  return 0;
}
