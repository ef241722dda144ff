// Per-CU vector-memory issue cost on gfx950: what a GEMM epilogue pays per wave-instruction.
//
// One 512-thread block per CU (the 256x256 GEMM's geometry); every wave issues NI memory
// instructions of one shape into its block's private region, then the block ends. Shapes:
//   width  : 1 (byte), 2, 4, 8 or 16 bytes per lane
//   rows   : how many distinct rows (row pitch `pitch` bytes) one wave-instruction covers;
//            lanes of a row are contiguous (lane stride = width), e.g. 16 B x 64 lanes in
//            rows = 4 -> 4 segments of 256 B (the staged fp32 epilogue's readback)
//   gap    : lane stride multiplier (2 -> every other 16-B slot, the coupling forward's y
//            stores: two instructions fill a line between them)
//   load   : loads instead of stores (all results folded into one dword store at the end)
// grid 256 blocks (all CUs) or 8 / 1 blocks (a lone CU per XCD: the per-CU limit without the
// chip's HBM share). Timed with hipEvents over several launches; prints one JSON line per case.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mem_issue_bench.hip -o /tmp/mem_issue_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

struct Shape {
  int width, rows, gap, load, ni;
  long pitch;
  int pair = 0;   // gap 2 only: odd instructions fill the other 16-B slots of the previous one's
                  // lines (the coupling-forward epilogue's two float4 stores per 8 features)
  int nx = 8;     // XCDs that work: blocks with (b % 8) < nx (blocks b and b + 8 share an XCD)
  int cu_div = 1; // of those, only blocks with ((b >> 3) % cu_div) == 0 work
};

template <int W>
struct VT;
template <> struct VT<1> { typedef unsigned char T; };
template <> struct VT<2> { typedef unsigned short T; };
template <> struct VT<4> { typedef unsigned T; };
template <> struct VT<8> { typedef uint2 T; };
template <> struct VT<16> { typedef uint4 T; };

template <int W>
__device__ __forceinline__ typename VT<W>::T mk(unsigned v) {
  typedef typename VT<W>::T T;
  if constexpr (W == 16) return make_uint4(v, v + 1, v + 2, v + 3);
  else if constexpr (W == 8) return make_uint2(v, v + 1);
  else return (T)v;
}
template <int W>
__device__ __forceinline__ unsigned fold(typename VT<W>::T x) {
  if constexpr (W == 16) return x.x ^ x.y ^ x.z ^ x.w;
  else if constexpr (W == 8) return x.x ^ x.y;
  else return (unsigned)x;
}

// region of block b: rows x pitch bytes; instruction i of wave w covers rows
// [(i * 8 + w) * rows, +rows), lane l -> row (l / lpr), byte (l % lpr) * W * gap
template <int W>
__global__ void __launch_bounds__(512, 1) mem_kernel(char* buf, long region, Shape s, unsigned* sink) {
  typedef typename VT<W>::T T;
  if ((int)(blockIdx.x & 7) >= s.nx || ((blockIdx.x >> 3) % s.cu_div) != 0) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lpr = 64 / s.rows;
  char* base = buf + (long)blockIdx.x * region;
  const long roff = (long)(lane / lpr) * s.pitch + (long)(lane % lpr) * W * s.gap;
  unsigned acc = 0;
  if (s.load) {
#pragma unroll 8
    for (int i = 0; i < s.ni; ++i) {
      const long r0 = (long)((i * 8 + w) * s.rows) * s.pitch;
      const T v = *(const T*)(base + r0 + roff);
      acc ^= fold<W>(v);
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
  } else {
#pragma unroll 8
    for (int i = 0; i < s.ni; ++i) {
      const int ii = s.pair ? (i >> 1) : i;
      const long r0 = (long)((ii * 8 + w) * s.rows) * s.pitch + (s.pair ? (i & 1) * W : 0);
      *(T*)(base + r0 + roff) = mk<W>(i ^ lane);
    }
  }
}

// LDS-DMA (global_load_lds, 16 B per lane) issue cost: the GEMM ring's operand stream. Wave w
// of block b issues NI DMA instructions; instruction i covers `rows` rows x (1024 / rows) B of
// its block's region (row pitch `pitch`, rows wrapping inside `foot` bytes, so a small footprint
// is L2-resident after the first pass) into a 16-KiB LDS ring, keeping INF in flight
// (s_waitcnt vmcnt(INF - 1) after each issue).
template <int INF>
__global__ void __launch_bounds__(512, 1) dma_kernel(const char* buf, long region, long foot, int rows,
                                                     long pitch, int ni, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char ring[8][16 * 1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lpr = 64 / rows;
  const char* base = buf + (long)blockIdx.x * region;
  const long roff = (long)(lane / lpr) * pitch + (long)(lane % lpr) * 16;
  const long nrows_foot = foot / pitch;
  for (int i = 0; i < ni; ++i) {
    const long r0 = ((long)(i * 8 + w) * rows) % nrows_foot;
    __builtin_amdgcn_global_load_lds((const void*)(base + r0 * pitch + roff),
                                     (__attribute__((address_space(3))) void*)(ring[w] + (i & 15) * 1024),
                                     16, 0, 0);
    if constexpr (INF == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (INF == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[w][lane] == 123 && ring[w][lane + 1] == 45) sink[blockIdx.x] = 1;
}

// Split lines: 16 rows x 64 B per instruction, the two 64-B halves of each 128-B line loaded
// by different instructions `lag` pairs apart (even instruction 2g: group g, half 0; odd
// instruction 2g + 1: group g - lag, half 1) - the TN ring's A-lo / A-hi pattern.
__global__ void __launch_bounds__(512, 1) dma_split_kernel(const char* buf, long region, int lag,
                                                           int ni, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char ring[8][16 * 1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long pitch = 2048;
  const char* base = buf + (long)blockIdx.x * region;
  for (int i = 0; i < ni; ++i) {
    const int half = i & 1;
    int grp = (i >> 1) - (half ? lag : 0);
    if (grp < 0) grp += ni / 2;
    const long r0 = ((long)(grp * 8 + w) * 16) % (region / pitch);   // rows wrap in the region
    const long off = r0 * pitch + (long)(lane >> 2) * pitch + half * 64 + (lane & 3) * 16;
    __builtin_amdgcn_global_load_lds((const void*)(base + off),
                                     (__attribute__((address_space(3))) void*)(ring[w] + (i & 15) * 1024),
                                     16, 0, 0);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[w][lane] == 123 && ring[w][lane + 1] == 45) sink[blockIdx.x] = 1;
}

// GEMM operand geometries, one private panel per block:
//   mode 0 (TN, mn-major operand): per instruction 2 k-rows x 512 B (the tile's 256 columns) at
//          row pitch `pitch`, k-rows advancing; the panel sits at column offset 512 * (b % 4)
//   mode 1 (NT, k-major operand): per instruction 8 rows x 128 B of a 256-row panel at row pitch
//          `pitch`; every 32 instructions (one K-tile's 256 rows) the column advances 128 B
// rows wrap inside the block's `foot` bytes (small foot = L2-resident after the first pass)
__global__ void __launch_bounds__(512, 1) dma_geom_kernel(const char* buf, long region, long foot,
                                                          int mode, long pitch, int ni,
                                                          unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char ring[8][16 * 1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* base = buf + (long)blockIdx.x * region;
  const long nrows = foot / pitch;
  for (int i = 0; i < ni; ++i) {
    const long q = (long)i * 8 + w;   // block-wide instruction index
    long off;
    if (mode == 0) {
      const long kr = (q * 2 + (lane >> 5)) % nrows;
      off = kr * pitch + 512 * (blockIdx.x & 3) + (lane & 31) * 16;
    } else {
      const long r = (q * 8) % 256 + (lane >> 3);
      const long col = ((q * 8 / 256) * 128) % pitch;
      off = (r % nrows) * pitch + col + (lane & 7) * 16;
    }
    __builtin_amdgcn_global_load_lds((const void*)(base + off),
                                     (__attribute__((address_space(3))) void*)(ring[w] + (i & 15) * 1024),
                                     16, 0, 0);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[w][lane] == 123 && ring[w][lane + 1] == 45) sink[blockIdx.x] = 1;
}

static void run_dma(char* buf, long region, unsigned* sink, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int ni = 2048;
  for (long foot : {64L << 10, 1L << 20, 64L << 20})
    for (int rows : {4, 8, 16})
      for (int inf : {4, 8, 16}) {
        const long pitch = 2048;   // a 1024-wide bf16 activation row
        auto launch = [&] {
          if (inf == 4) dma_kernel<4><<<cus, 512>>>(buf, region, foot, rows, pitch, ni, sink);
          else if (inf == 8) dma_kernel<8><<<cus, 512>>>(buf, region, foot, rows, pitch, ni, sink);
          else dma_kernel<16><<<cus, 512>>>(buf, region, foot, rows, pitch, ni, sink);
        };
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        const double bytes = 8.0 * ni * 1024;   // per block
        printf("{\"op\": \"dma\", \"rows\": %d, \"seg_bytes\": %d, \"inflight\": %d, "
               "\"foot_kb\": %ld, \"us\": %.2f, \"GBps_per_cu\": %.1f, \"TBps_total\": %.2f}\n",
               rows, 1024 / rows, inf, foot >> 10, us, bytes / us / 1e3, bytes * cus / us / 1e6);
        fflush(stdout);
      }
  struct G { int mode; long pitch; long foot; };
  const G geoms[] = {{0, 832, 1L << 20}, {0, 2048, 1L << 20}, {0, 8192, 1L << 20},
                     {1, 131072, 32L << 20},
                     {0, 832, 60L << 20}, {0, 1600, 60L << 20}, {0, 2048, 60L << 20},
                     {0, 8192, 60L << 20}, {1, 2048, 60L << 20}, {1, 131072, 60L << 20}};
  for (const G& gm : geoms) {
    auto launch = [&] { dma_geom_kernel<<<cus, 512>>>(buf, region, gm.foot, gm.mode, gm.pitch, ni, sink); };
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    const double bytes = 8.0 * ni * 1024;
    printf("{\"op\": \"dma_geom\", \"mode\": \"%s\", \"pitch\": %ld, \"foot_kb\": %ld, "
           "\"us\": %.2f, \"GBps_per_cu\": %.1f, \"TBps_total\": %.2f}\n",
           gm.mode ? "nt" : "tn", gm.pitch, gm.foot >> 10, us, bytes / us / 1e3,
           bytes * cus / us / 1e6);
    fflush(stdout);
  }
  for (int lag : {0, 2, 8, 32, 128}) {   // HBM footprint (ni/2 groups x 8 waves x 16 rows x 2 KB)
    auto launch = [&] { dma_split_kernel<<<cus, 512>>>(buf, region, lag, ni, sink); };
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    const double bytes = 8.0 * ni * 1024;
    printf("{\"op\": \"dma_split\", \"lag\": %d, \"us\": %.2f, \"GBps_per_cu\": %.1f, "
           "\"TBps_total\": %.2f}\n", lag, us, bytes / us / 1e3, bytes * cus / us / 1e6);
    fflush(stdout);
  }
}

int main(int argc, char** argv) {
  int dev_cus = 256;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  dev_cus = p.multiProcessorCount;
  const long region = 64L << 20;  // 64 MiB per block
  char* buf;
  CK(hipMalloc(&buf, region * dev_cus));
  CK(hipMemset(buf, 1, region * dev_cus));
  unsigned* sink;
  CK(hipMalloc(&sink, 4 * dev_cus));
  if (argc > 1 && std::string(argv[1]) == "dma") {
    run_dma(buf, region, sink, dev_cus);
    return 0;
  }
  std::vector<Shape> cases;
  // stores: (width, rows, gap), pitch 2048 (a bf16 1024-wide activation row) unless noted
  const int W[] = {1, 2, 4, 8, 16};
  const bool full = argc > 1 && std::string(argv[1]) == "full";
  for (int ld = 0; ld < 2 && full; ++ld) {
    for (int w : W) cases.push_back({w, 1, 1, ld, 256, 2048});           // contiguous
    cases.push_back({16, 2, 1, ld, 256, 2048});                          // 2 rows x 512 B
    cases.push_back({16, 4, 1, ld, 256, 2048});                          // 4 rows x 256 B
    cases.push_back({16, 8, 1, ld, 256, 2048});                          // 8 rows x 128 B
    cases.push_back({8, 4, 1, ld, 256, 2048});                           // 4 rows x 128 B
    cases.push_back({8, 8, 1, ld, 256, 2048});                           // 8 rows x 64 B
    cases.push_back({16, 4, 2, ld, 256, 2048});                          // 4 rows, every other 16 B
    cases.push_back({1, 8, 1, ld, 256, 128});                            // 8 rows x 8 B (ReLU bitmask)
    cases.push_back({16, 4, 1, ld, 256, 4096});                         // 4 rows x 256 B, fp32 rows
  }
  // per-XCD vs chip-wide limit: all 32 CUs of 1, 2, 4 or 8 XCDs, or 16 / 8 CUs of each
  for (int ld = 0; ld < 2; ++ld)
    for (int nx : {1, 2, 4, 8})
      for (int cd : {1, 2, 4}) {
        Shape t{16, 4, 1, ld, 256, 2048};
        t.nx = nx;
        t.cu_div = cd;
        cases.push_back(t);
      }
  for (int pr = 0; pr < 2; ++pr) {   // gap-2 stores alone vs filled by the next instruction
    Shape t{16, 4, 2, 0, 256, 2048};
    t.pair = pr;
    cases.push_back(t);
  }
  cases.push_back(Shape{16, 4, 1, 0, 256, 2048});   // contiguous reference
  const int grids[] = {dev_cus};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : cases) {
    for (int g : grids) {
      auto launch = [&] {
        switch (s.width) {
          case 1: mem_kernel<1><<<g, 512>>>(buf, region, s, sink); break;
          case 2: mem_kernel<2><<<g, 512>>>(buf, region, s, sink); break;
          case 4: mem_kernel<4><<<g, 512>>>(buf, region, s, sink); break;
          case 8: mem_kernel<8><<<g, 512>>>(buf, region, s, sink); break;
          default: mem_kernel<16><<<g, 512>>>(buf, region, s, sink); break;
        }
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      const int reps = 20;
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / reps;
      const double instr = 8.0 * s.ni;            // wave-instructions per working block
      const int working = [&] {
        int n = 0;
        for (int b = 0; b < g; ++b) n += (b % 8) < s.nx && ((b / 8) % s.cu_div) == 0;
        return n;
      }();
      const double bytes = instr * 64 * s.width;  // per block
      // cycles per wave-instruction per CU at an assumed 2.0 GHz (relative measure only)
      printf("{\"op\": \"%s\", \"width\": %d, \"rows\": %d, \"gap\": %d, \"pitch\": %ld, "
             "\"pair\": %d, \"blocks\": %d, \"xcds\": %d, \"working\": %d, \"us\": %.2f, \"GBps_per_cu\": %.1f, "
             "\"TBps_total\": %.2f, \"ns_per_instr\": %.2f}\n",
             s.load ? "load" : "store", s.width, s.rows, s.gap, s.pitch, s.pair, g, s.nx, working, us,
             bytes / us / 1e3, bytes * working / us / 1e6, us * 1e3 / instr);
      fflush(stdout);
    }
  }
  CK(hipFree(buf));
  return 0;
}
