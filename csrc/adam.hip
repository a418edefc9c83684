// Fused multi-tensor Adam (L2 weight decay, torch.optim.Adam semantics) over ONE flat fp32 buffer.
// Reference: utils/train_utils.py:45 (Adam(lr, weight_decay=1e-8)), SURVEY K13.
// Memory-bound: 4 streams in (p, g, m, v) + 3 out -> float4 per lane, grid-stride, one launch per step.
#include "common.h"

// DEV: hyper-parameters read from a device state block (HIP-graph replay: the captured launch cannot
// bake host scalars that change every step); state = {step, lr, 1/bc1, 1/sqrt(bc2)} in fp64.
template <bool DEV>
__global__ __launch_bounds__(256) void adam_flat_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    long long n, float lr, float b1, float b2, float eps, float wd, float inv_bc1, float inv_sqrt_bc2,
    const double* __restrict__ state) {
  if constexpr (DEV) {
    lr = (float)state[1];
    inv_bc1 = (float)state[2];
    inv_sqrt_bc2 = (float)state[3];
  }
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = ga[j] + wd * pa[j];
      ma[j] = b1 * ma[j] + (1.f - b1) * gr;
      va[j] = b2 * va[j] + (1.f - b2) * gr * gr;
      float denom = sqrtf(va[j]) * inv_sqrt_bc2 + eps;
      pa[j] -= lr * inv_bc1 * ma[j] / denom;
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  // scalar tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    long long i = (n4 << 2) + threadIdx.x;
    float gr = g[i] + wd * p[i];
    m[i] = b1 * m[i] + (1.f - b1) * gr;
    v[i] = b2 * v[i] + (1.f - b2) * gr * gr;
    p[i] -= lr * inv_bc1 * m[i] / (sqrtf(v[i]) * inv_sqrt_bc2 + eps);
  }
}

DPA_API int dpa_adam_flat(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
                          float b2, float eps, float wd, float bc1, float bc2, hipStream_t stream) {
  if (n <= 0) return 0;
  int grid = dpa_grid((n + 3) / 4, 256, 4096);
  hipLaunchKernelGGL(adam_flat_kernel<false>, dim3(grid), dim3(256), 0, stream, p, g, m, v, n, lr, b1, b2, eps,
                     wd, 1.f / bc1, 1.f / sqrtf(bc2), nullptr);
  return (int)hipGetLastError();
}

// state[0] += 1 and the bias corrections of the new step, in fp64 (same rounding as the host path)
__global__ void adam_tick_kernel(double* state, double b1, double b2) {
  const double t = state[0] + 1.0;
  state[0] = t;
  state[2] = 1.0 / (1.0 - pow(b1, t));
  state[3] = 1.0 / sqrt(1.0 - pow(b2, t));
}

// graph-capturable step: tick + update, all hyper-parameters from `state` (lr = state[1], set by the host)
DPA_API int dpa_adam_flat_dev(float* p, const float* g, float* m, float* v, long long n, double* state, double b1,
                              double b2, float eps, float wd, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(1), 0, stream, state, b1, b2);
  int grid = dpa_grid((n + 3) / 4, 256, 4096);
  hipLaunchKernelGGL(adam_flat_kernel<true>, dim3(grid), dim3(256), 0, stream, p, g, m, v, n, 0.f, (float)b1,
                     (float)b2, eps, wd, 0.f, 0.f, (const double*)state);
  return (int)hipGetLastError();
}

DPA_API int dpa_version() { return 1; }
DPA_API const char* dpa_error_string(int e) { return hipGetErrorString((hipError_t)e); }
