#include <hip/hip_runtime.h>
#include <cstdio>
// gfx950 ds_read_b64_tr_b8 semantics probe. MODE 1 fills byte x with x and lets lane L point at
// bytes 8L..8L+7, so every output byte names its source (lane = v / 8, byte = v % 8).
#ifndef MODE
#define MODE 1
#endif
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(unsigned* out) {
  __shared__ unsigned char lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (unsigned char)(i & 255);
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 1, p = i & 1;
  // hypothesis: block = 8 rows x 16 bytes, row pitch 128 B; lane 2q+p -> row q, bytes 8p..8p+7
  const int addr = MODE == 0 ? g * 1024 + q * 128 + p * 8 : l * 8;   // MODE 1: lane L's own 8 bytes
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + addr));
  out[2 * l] = r[0]; out[2 * l + 1] = r[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 512);
  k<<<1, 64>>>(d);
  unsigned h[128]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 32; ++l) {
    const unsigned char* b = (const unsigned char*)&h[2 * l];
    printf("lane %2d:", l);
    for (int e = 0; e < 8; ++e) printf(" %3d", b[e]);
    printf("\n");
  }
  return 0;
}
