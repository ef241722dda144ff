// Fused single-pass optimizers over one flat fp32 parameter buffer (gfx950).
//
// One launch updates every parameter of a model: p, m, v are flat fp32
// buffers and the kernel optionally writes the bf16 working copy that the
// MFMA GEMMs consume, so the master->bf16 cast costs no extra pass.
// Graph-capture friendly: the step count, an optional gradient multiplier
// (1/world for DP averaging, or a clip coefficient) and a skip flag (set by a
// non-finite guard) are all read from device memory.
//
// kind 0: Adam      (m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; bias-corrected)   [optimization.py:118]
// kind 1: RMSProp   (v = b2 v + (1-b2) g^2; p -= lr g / (sqrt(v) + eps))          [get_data.py:140]
// kind 2: SGD-mom.  (m = b1 m - (1-b1) g; p += lr m)  (autograd.misc.optimizers.sgd)[experimentation.py:109]
// kind 3: RMSProp+momentum (Lasagne style: v as above; m = b1 m - lr g/sqrt(v+eps); p += m) [theano_implement.py:187]
// weight_decay is decoupled (AdamW style) when > 0.
#include "nf_common.h"

namespace nf {

struct OptArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16_t* pbf;
  long n;
  float lr, b1, b2, eps, wd;
  const float* step_ptr;   // device step count (1-based after increment), may be null
  float step_host;
  const float* gscale_ptr; // device gradient multiplier, may be null
  float gscale_host;
  const float* skip_ptr;   // device flag; != 0 -> no update
  float warmup;            // > 0: lr ramps linearly over the first `warmup` steps (lr * min(1, t / warmup))
  int kind;
};

__device__ __forceinline__ void opt_update(const OptArgs& a, float& p, float g, float& m, float& v,
                                           float bc1, float bc2) {
  switch (a.kind) {
    case 0: {
      m = fmaf(a.b1, m, (1.f - a.b1) * g);
      v = fmaf(a.b2, v, (1.f - a.b2) * g * g);
      const float mh = m / bc1, vh = v / bc2;
      p -= a.lr * (mh / (sqrtf(vh) + a.eps) + a.wd * p);
      break;
    }
    case 1: {
      v = fmaf(a.b2, v, (1.f - a.b2) * g * g);
      p -= a.lr * (g / (sqrtf(v) + a.eps) + a.wd * p);
      break;
    }
    case 2: {
      m = fmaf(a.b1, m, -(1.f - a.b1) * g);
      p += a.lr * m - a.lr * a.wd * p;
      break;
    }
    default: {
      v = fmaf(a.b2, v, (1.f - a.b2) * g * g);
      m = fmaf(a.b1, m, -a.lr * g / sqrtf(v + a.eps));
      p += m - a.lr * a.wd * p;
      break;
    }
  }
}

typedef float f4v __attribute__((ext_vector_type(4)));

// NT = true: the read-once streams (g, m, v, p) are loaded and the master / moment streams are
// stored with nontemporal hints so they do not evict the bf16 copy (read by the transpose and
// the next step's GEMMs) from L2 / MALL.
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p, long i) {
  if constexpr (NT) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p) + i);
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return reinterpret_cast<const float4*>(p)[i];
  }
}

template <bool NT>
__device__ __forceinline__ void st4(float* p, long i, const float4& x) {
  if constexpr (NT) {
    f4v v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p) + i);
  } else {
    reinterpret_cast<float4*>(p)[i] = x;
  }
}

template <bool NT>
__global__ void __launch_bounds__(256) flat_optimizer_kernel(OptArgs a_) {
  OptArgs a = a_;
  if (a.skip_ptr && *a.skip_ptr != 0.f) return;
  const float step = a.step_ptr ? *a.step_ptr : a.step_host;
  const float gs = a.gscale_ptr ? *a.gscale_ptr : a.gscale_host;
  const float bc1 = 1.f - powf(a.b1, step);
  const float bc2 = 1.f - powf(a.b2, step);
  // linear learning-rate warm-up, read from the device step so a captured graph replays it: the
  // first bias-corrected Adam step is a sign step of size lr on EVERY parameter, which at 72 M
  // parameters and 32 coupling layers throws the flow far off (ldj -1 -> -1500 in one step)
  if (a.warmup > 0.f && step < a.warmup) a.lr *= fmaxf(step, 1.f) / a.warmup;
  const long n4 = a.n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = ld4<NT>(a.p, i);
    const float4 g = ld4<NT>(a.g, i);
    float4 m = a.m ? ld4<NT>(a.m, i) : make_float4(0, 0, 0, 0);
    float4 v = a.v ? ld4<NT>(a.v, i) : make_float4(0, 0, 0, 0);
    opt_update(a, p.x, g.x * gs, m.x, v.x, bc1, bc2);
    opt_update(a, p.y, g.y * gs, m.y, v.y, bc1, bc2);
    opt_update(a, p.z, g.z * gs, m.z, v.z, bc1, bc2);
    opt_update(a, p.w, g.w * gs, m.w, v.w, bc1, bc2);
    st4<NT>(a.p, i, p);
    if (a.m) st4<NT>(a.m, i, m);
    if (a.v) st4<NT>(a.v, i, v);
    if (a.pbf) {
      ushort4 o;
      o.x = f2bf(p.x); o.y = f2bf(p.y); o.z = f2bf(p.z); o.w = f2bf(p.w);
      reinterpret_cast<ushort4*>(a.pbf)[i] = o;
    }
  }
  // scalar tail
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    float p = a.p[i], m = a.m ? a.m[i] : 0.f, v = a.v ? a.v[i] : 0.f;
    opt_update(a, p, a.g[i] * gs, m, v, bc1, bc2);
    a.p[i] = p;
    if (a.m) a.m[i] = m;
    if (a.v) a.v[i] = v;
    if (a.pbf) a.pbf[i] = f2bf(p);
  }
}

// Sum of squares + non-finite detection over a flat buffer: partial sums per block.
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ x, long n,
                                                             float* __restrict__ partial) {
  __shared__ float scratch[16];
  float acc = 0.f;
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // four independent float4 loads in flight per thread (512 blocks = 8 waves per CU)
  float acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const float4 v0 = reinterpret_cast<const float4*>(x)[i];
    const float4 v1 = reinterpret_cast<const float4*>(x)[i + stride];
    const float4 v2 = reinterpret_cast<const float4*>(x)[i + 2 * stride];
    const float4 v3 = reinterpret_cast<const float4*>(x)[i + 3 * stride];
    acc += v0.x * v0.x + v0.y * v0.y + v0.z * v0.z + v0.w * v0.w;
    acc1 += v1.x * v1.x + v1.y * v1.y + v1.z * v1.z + v1.w * v1.w;
    acc2 += v2.x * v2.x + v2.y * v2.y + v2.z * v2.z + v2.w * v2.w;
    acc3 += v3.x * v3.x + v3.y * v3.y + v3.z * v3.z + v3.w * v3.w;
  }
  for (; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc += (acc1 + acc2) + acc3;
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    acc += x[i] * x[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Finalise: total = sum(partial); writes total, guard flag (1 if non-finite) and
// clip multiplier min(1, max_norm / sqrt(total)) * base_scale.
__global__ void __launch_bounds__(256) sumsq_finalize_kernel(const float* __restrict__ partial,
                                                              int np, float* __restrict__ out_sumsq,
                                                              float* __restrict__ out_skip,
                                                              float* __restrict__ out_scale,
                                                              float max_norm, float base_scale) {
  __shared__ float scratch[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    const float total = acc * base_scale * base_scale;
    if (out_sumsq) *out_sumsq = total;
    const bool bad = !isfinite(total);
    if (out_skip) *out_skip = bad ? 1.f : 0.f;
    if (out_scale) {
      float sc = base_scale;
      if (max_norm > 0.f && !bad) {
        const float nrm = sqrtf(total);
        if (nrm > max_norm) sc *= max_norm / (nrm + 1e-6f);
      }
      *out_scale = sc;
    }
  }
}

}  // namespace nf

using namespace nf;

void nf_launch_flat_optimizer(int kind, float* p, const float* g, float* m, float* v, void* pbf,
                              long n, float lr, float b1, float b2, float eps, float wd,
                              const float* step_ptr, float step_host, const float* gscale_ptr,
                              float gscale_host, const float* skip_ptr, float warmup,
                              hipStream_t stream) {
  if (n <= 0) return;
  OptArgs a;
  a.p = p; a.g = g; a.m = m; a.v = v; a.pbf = (bf16_t*)pbf; a.n = n;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  a.step_ptr = step_ptr; a.step_host = step_host;
  a.gscale_ptr = gscale_ptr; a.gscale_host = gscale_host;
  a.skip_ptr = skip_ptr; a.kind = kind; a.warmup = warmup;
  // nontemporal loads / stores (446 -> 397 us for the headline's 72.2M parameters against plain
  // ones, tools/opt_probe.py), grid capped at 2048 blocks (grid-stride loop)
  long blocks = ((n >> 2) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(flat_optimizer_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  NF_HIP_CHECK(hipGetLastError());
}

void nf_launch_sumsq_guard(const float* x, long n, float* partial, int npartial, float* out_sumsq,
                           float* out_skip, float* out_scale, float max_norm, float base_scale,
                           hipStream_t stream) {
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(npartial), dim3(256), 0, stream, x, n, partial);
  NF_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(sumsq_finalize_kernel, dim3(1), dim3(256), 0, stream, partial, npartial,
                     out_sumsq, out_skip, out_scale, max_norm, base_scale);
  NF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Collective-occupancy emulator (diagnostics only): `blocks` workgroups of 256 threads that each
// hold a CU slot for `usec` microseconds (s_memrealtime is a 100 MHz clock), launched on a side
// stream where a DP gradient bucket's all-reduce would run. Lets a 1-GPU box measure how the
// compute kernels behave when RCCL's channel blocks occupy CUs mid-backward. Every wave exits
// on the time bound.
namespace nf {
__global__ void __launch_bounds__(256) cu_hold_kernel(long long ticks, int* sink) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  int n = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    ++n;
  }
  if (n < 0 && sink) sink[threadIdx.x] = n;  // never taken: keeps the loop observable
}
}  // namespace nf

void nf_launch_cu_hold(int blocks, float usec, hipStream_t stream) {
  if (blocks <= 0 || usec <= 0.f) return;
  const long long ticks = (long long)(usec * 100.0f);
  hipLaunchKernelGGL(nf::cu_hold_kernel, dim3(blocks), dim3(256), 0, stream, ticks, (int*)nullptr);
  NF_HIP_CHECK(hipGetLastError());
}
