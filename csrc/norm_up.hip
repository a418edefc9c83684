// BatchNorm(+ReLU) and bilinear x2 up-sampling for the UNet variant blocks on gfx950: NHWC bf16
// activations, fp32 statistics and math, 16-byte accesses (8 channels per lane).
//
// The reference UNet has neither op (model/unet_parts.py:6-17 is Conv+ReLU, :51-54 ConvTranspose2d);
// the north-star DoubleConv = Conv2d+BN+ReLU and the bilinear Up path are the variants listed next
// to it (model/modelsummary.txt:153-247).  Semantics follow torch.nn.BatchNorm2d (training: biased
// batch variance for normalisation, unbiased for running_var, running stats updated with
// `momentum`; eval: running stats) and F.interpolate(scale_factor=2, mode="bilinear",
// align_corners=False).
//
// Batch statistics are a deterministic two-level reduction (no float atomics): bn_partial_kernel
// gives every block one row of per-channel partial sums in a slab [nblk][2][C] (256 threads = R
// pixel rows x G groups of 8 channels, consecutive rows = consecutive pixels, so a block streams a
// contiguous R*C*2-byte span when G*8 == C); bn_*_finalize_kernel sums the rows in a fixed order,
// one block per channel.  The same pair computes the backward sums (sum g, sum g*(z-mean)).
#include "common.h"

#include "conv_args.h"   // pool_code

// ------------------------------------------------------------------------------ batch statistics
// MODE 0: s = sum z, q = sum z^2          (a = z)
// MODE 1: s = sum g, q = sum g*(z - mean)  (a = g, z = conv output, mean = saved[c])
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(const bf16_t* __restrict__ a, int lda, const bf16_t* __restrict__ z,
                                                         int ldz, const float* __restrict__ saved, long P, int C, int G,
                                                         float* __restrict__ slab) {
  __shared__ float red[256 * 16];
  const int tid = threadIdx.x;
  const int R = 256 / G;
  const int g = tid % G, r = tid / G;
  const int c0 = (blockIdx.y * G + g) * 8;
  float s[8], q[8], mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s[k] = 0.f;
    q[k] = 0.f;
    mu[k] = MODE ? saved[c0 + k] : 0.f;
  }
  for (long p = (long)blockIdx.x * R + r; p < P; p += (long)gridDim.x * R) {
    const uint4 u = *reinterpret_cast<const uint4*>(a + p * lda + c0);
    const unsigned* pu = &u.x;
    if (MODE == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v0 = lo_bf(pu[e]), v1 = hi_bf(pu[e]);
        s[2 * e] += v0; q[2 * e] = fmaf(v0, v0, q[2 * e]);
        s[2 * e + 1] += v1; q[2 * e + 1] = fmaf(v1, v1, q[2 * e + 1]);
      }
    } else {
      const uint4 w = *reinterpret_cast<const uint4*>(z + p * ldz + c0);
      const unsigned* pw = &w.x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g0 = lo_bf(pu[e]), g1 = hi_bf(pu[e]);
        s[2 * e] += g0; q[2 * e] = fmaf(g0, lo_bf(pw[e]) - mu[2 * e], q[2 * e]);
        s[2 * e + 1] += g1; q[2 * e + 1] = fmaf(g1, hi_bf(pw[e]) - mu[2 * e + 1], q[2 * e + 1]);
      }
    }
  }
  float* row = red + r * (G * 16) + g * 16;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    row[k] = s[k];
    row[8 + k] = q[k];
  }
  __syncthreads();
  for (int j = tid; j < G * 16; j += 256) {
    float acc = 0.f;
    for (int rr = 0; rr < R; ++rr) acc += red[rr * G * 16 + j];
    const int gg = j >> 4, k = j & 15;
    const int c = (blockIdx.y * G + gg) * 8 + (k & 7);
    slab[(long)blockIdx.x * 2 * C + (k >> 3) * C + c] = acc;
  }
}

// one block per channel: fixed-order sums of the slab rows
__device__ __forceinline__ void slab_pair(const float* slab, int nblk, int C, int c, float* red, float& s, float& q) {
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    a += slab[(long)i * 2 * C + c];
    b += slab[(long)i * 2 * C + C + c];
  }
  s = block_sum_256(a, red);
  q = block_sum_256(b, red);
}

// Fold a tall slab [rows][K] into [ceil(rows/R)][K] (block b sums rows bR..bR+R-1, threads across
// the K columns: coalesced rows, fixed order).  The conv epilogues write one slab row per block --
// tens of thousands at full resolution -- and the one-block-per-channel finalize would otherwise walk
// all of them serially.
__global__ __launch_bounds__(256) void slab_fold_kernel(const float* __restrict__ in, int rows, int K, int R,
                                                        float* __restrict__ out) {
  const int r0 = blockIdx.x * R, r1 = min(rows, r0 + R);
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float acc = 0.f;
    for (int r = r0; r < r1; ++r) acc += in[(long)r * K + k];
    out[(long)blockIdx.x * K + k] = acc;
  }
}

DPA_API int dpa_slab_fold(const float* in, int rows, int K, int nout, float* out, hipStream_t st) {
  if (rows <= 0 || K <= 0 || nout <= 0) return (int)hipErrorInvalidValue;
  const int R = (rows + nout - 1) / nout;
  hipLaunchKernelGGL(slab_fold_kernel, dim3((rows + R - 1) / R), dim3(256), 0, st, in, rows, K, R, out);
  return (int)hipGetLastError();
}

// Forward coefficients y = z*coef[c] + coef[C+c].  train: batch statistics (saved = mean, invstd
// for the backward; running stats updated in place); eval (slab == null): running statistics.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ slab, int nblk, int C, long P,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float eps, float momentum, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, float* __restrict__ coef,
                                                          float* __restrict__ saved) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float mean, var;
  if (slab) {
    float s, q;
    slab_pair(slab, nblk, C, c, red, s, q);
    const double m = (double)s / (double)P;
    double v = (double)q / (double)P - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  if (threadIdx.x != 0) return;
  const float invstd = 1.f / sqrtf(var + eps);
  const float sc = gamma[c] * invstd;
  coef[c] = sc;
  coef[C + c] = beta[c] - mean * sc;
  if (slab) {
    saved[c] = mean;
    saved[C + c] = invstd;
    if (rmean) {
      const float unbiased = P > 1 ? var * (float)((double)P / (double)(P - 1)) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
    }
  }
}

// Backward coefficients dz = a*g + b*z + c (torch batch_norm_backward, training mode):
//   xhat = (z-mean)*invstd,  dz = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat))
// and dgamma += sum g*xhat, dbeta += sum g (accumulated into the flat fp32 gradient buffer).
// gy_mode (slab from the dgrad epilogue, csrc/halo.hip EPI 5): the second column is sum g*y with
// y = relu(gamma xhat + beta) the BN output; g vanishes where y == 0, elsewhere xhat = (y - beta)/gamma,
// so sum g*xhat = (sum g*y - beta sum g) / gamma.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ slab, int nblk, int C, long P,
                                                              const float* __restrict__ gamma, const float* __restrict__ saved,
                                                              float* __restrict__ coef3, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, const float* __restrict__ beta,
                                                              int gy_mode) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float sg, sgz;
  slab_pair(slab, nblk, C, c, red, sg, sgz);
  if (threadIdx.x != 0) return;
  const float mean = saved[c], invstd = saved[C + c];
  const float sgx = gy_mode ? (sgz - beta[c] * sg) / gamma[c] : sgz * invstd;
  if (dgamma) dgamma[c] += sgx;
  if (dbeta) dbeta[c] += sg;
  const float sc = gamma[c] * invstd;
  const float inv_p = (float)(1.0 / (double)P);
  const float b = -sc * invstd * sgx * inv_p;
  coef3[c] = sc;
  coef3[C + c] = b;
  coef3[2 * C + c] = -sc * sg * inv_p - b * mean;
}

// ------------------------------------------------------------------------------ elementwise passes
// y = relu?(z*coef[c] + coef[C+c]); y may be a channel slice of a wider tensor (concat half)
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ z, int ldz, bf16_t* __restrict__ y, int ldy,
                                                       const float* __restrict__ coef, long P, int C, int relu) {
  const int CC = C >> 3;
  const long tot = P * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long p = i / CC;
    const int c0 = cc * 8;
    const uint4 u = *reinterpret_cast<const uint4*>(z + p * ldz + c0);
    const unsigned* pu = &u.x;
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v0 = fmaf(lo_bf(pu[e]), coef[c0 + 2 * e], coef[C + c0 + 2 * e]);
      float v1 = fmaf(hi_bf(pu[e]), coef[c0 + 2 * e + 1], coef[C + c0 + 2 * e + 1]);
      if (relu) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
      }
      o[e] = pack_bf2(v0, v1);
    }
    *reinterpret_cast<uint4*>(y + p * ldy + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Encoder DoubleConv output: y = relu(bn(z)) AND its 2x2/s2 max-pool + window codes in one pass
// (even H, W).  One thread per (window, 8 channels): reads the 4 z pixels once, writes the 4 y
// pixels, the pooled pixel and the codes the pool backward consumes -- the separate max-pool pass
// would re-read all of y.  Pools the STORED (bf16-rounded) y, like maxpool2_kernel.
__global__ __launch_bounds__(256) void bn_apply_pool_kernel(const bf16_t* __restrict__ z, int ldz, bf16_t* __restrict__ y,
                                                            int ldy, bf16_t* __restrict__ pool, int ldp,
                                                            unsigned char* __restrict__ code, const float* __restrict__ coef,
                                                            int N, int H, int W, int C, int relu) {
  const int Ho = H >> 1, Wo = W >> 1, CC = C >> 3;
  const long tot = (long)N * Ho * Wo * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long op = i / CC;
    const int ow = (int)(op % Wo);
    const long t = op / Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const int c0 = cc * 8;
    const long p00 = ((long)(n * H + 2 * oh) * W + 2 * ow);
    const long pix[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    float v[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 u = *reinterpret_cast<const uint4*>(z + pix[q] * ldz + c0);
      const unsigned* pu = &u.x;
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v0 = fmaf(lo_bf(pu[e]), coef[c0 + 2 * e], coef[C + c0 + 2 * e]);
        float v1 = fmaf(hi_bf(pu[e]), coef[c0 + 2 * e + 1], coef[C + c0 + 2 * e + 1]);
        if (relu) {
          v0 = fmaxf(v0, 0.f);
          v1 = fmaxf(v1, 0.f);
        }
        o[e] = pack_bf2(v0, v1);
        v[q][2 * e] = lo_bf(o[e]);
        v[q][2 * e + 1] = hi_bf(o[e]);
      }
      if (y) *reinterpret_cast<uint4*>(y + pix[q] * ldy + c0) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    unsigned o[4], cd[2] = {0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int a = 2 * k, b = 2 * k + 1;
      const float l = fmaxf(fmaxf(v[0][a], v[1][a]), fmaxf(v[2][a], v[3][a]));
      const float h = fmaxf(fmaxf(v[0][b], v[1][b]), fmaxf(v[2][b], v[3][b]));
      o[k] = pack_bf2(l, h);
      const unsigned cl = pool_code(v[0][a], v[1][a], v[2][a], v[3][a]);
      const unsigned ch = pool_code(v[0][b], v[1][b], v[2][b], v[3][b]);
      cd[k >> 1] |= (cl | ch << 8) << (16 * (k & 1));
    }
    *reinterpret_cast<uint4*>(pool + op * ldp + c0) = make_uint4(o[0], o[1], o[2], o[3]);
    if (code) *reinterpret_cast<uint2*>(code + op * C + c0) = make_uint2(cd[0], cd[1]);
  }
}

// dz = coef3[c]*g + coef3[C+c]*z + coef3[2C+c]
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ g, int ldg, const bf16_t* __restrict__ z,
                                                           int ldz, const float* __restrict__ coef3, bf16_t* __restrict__ dz,
                                                           int lddz, long P, int C) {
  const int CC = C >> 3;
  const long tot = P * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long p = i / CC;
    const int c0 = cc * 8;
    const uint4 ug = *reinterpret_cast<const uint4*>(g + p * ldg + c0);
    const uint4 uz = *reinterpret_cast<const uint4*>(z + p * ldz + c0);
    const unsigned* pg = &ug.x;
    const unsigned* pz = &uz.x;
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + 2 * e;
      const float v0 = fmaf(coef3[c], lo_bf(pg[e]), fmaf(coef3[C + c], lo_bf(pz[e]), coef3[2 * C + c]));
      const float v1 = fmaf(coef3[c + 1], hi_bf(pg[e]), fmaf(coef3[C + c + 1], hi_bf(pz[e]), coef3[2 * C + c + 1]));
      o[e] = pack_bf2(v0, v1);
    }
    *reinterpret_cast<uint4*>(dz + p * lddz + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// G = channel groups of 8 per block (power of two dividing C/8, <= 32) and the block grid
static bool bn_shape(long P, int C, int& G, dim3& grid) {
  if (C <= 0 || (C & 7) || P <= 0) return false;
  const int CG = C / 8;
  G = 1;
  while (G * 2 <= 32 && CG % (G * 2) == 0) G *= 2;
  const int R = 256 / G;
  long nbx = (P + R - 1) / R;
  if (nbx > 512) nbx = 512;
  grid = dim3((unsigned)nbx, (unsigned)(CG / G));
  return true;
}

DPA_API int dpa_bn_slab_rows(long long P, int C) {
  int G;
  dim3 grid;
  return bn_shape(P, C, G, grid) ? (int)grid.x : 0;
}

// training forward: statistics of z -> coef (scale, shift), saved (mean, invstd), running stats;
// eval forward (train == 0): coef from the running statistics.  Then y = relu?(bn(z)).
DPA_API int dpa_bn_fwd(const bf16_t* z, int ldz, bf16_t* y, int ldy, long long P, int C, const float* gamma, const float* beta,
                       float eps, float momentum, float* rmean, float* rvar, float* slab, float* coef, float* saved, int train,
                       int relu, int slab_rows, bf16_t* pool, int ldp, unsigned char* code, int N, int H, int W,
                       hipStream_t st) {
  int G;
  dim3 grid;
  if (!bn_shape(P, C, G, grid) || (ldz & 7) || (ldy & 7)) return (int)hipErrorInvalidValue;
  if (pool && ((ldp & 7) || (H & 1) || (W & 1) || (long)N * H * W != (long)P)) return (int)hipErrorInvalidValue;
  if (train) {
    // slab_rows > 0: the producing conv already wrote the partial sums (igemm_stream EPI 4)
    if (slab_rows <= 0)
      hipLaunchKernelGGL(bn_partial_kernel<0>, grid, dim3(256), 0, st, z, ldz, (const bf16_t*)nullptr, 0,
                         (const float*)nullptr, (long)P, C, G, slab);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, slab, slab_rows > 0 ? slab_rows : (int)grid.x, C,
                       (long)P, gamma, beta, eps, momentum, rmean, rvar, coef, saved);
  } else {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, (const float*)nullptr, 0, C, (long)P, gamma, beta, eps,
                       momentum, rmean, rvar, coef, saved);
  }
  // coefficients only (y == pool == null): the consumer applies the BN + ReLU on load (IgemmArgs::xbn);
  // y == null with pool: only the pooled tensor and its window codes (the consumers of y read z on load)
  if (y == nullptr && pool == nullptr) return (int)hipGetLastError();
  if (y == nullptr && !(pool && relu)) return (int)hipErrorInvalidValue;
  if (pool) {
    const long tot = (long)P / 4 * (C / 8);
    hipLaunchKernelGGL(bn_apply_pool_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, z, ldz, y, ldy, pool, ldp,
                       code, coef, N, H, W, C, relu);
    return (int)hipGetLastError();
  }
  const long tot = (long)P * (C / 8);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, z, ldz, y, ldy, coef, (long)P, C, relu);
  return (int)hipGetLastError();
}

// training backward coefficients only: dz = coef3[c] g + coef3[C+c] z + coef3[2C+c] (dgamma/dbeta
// accumulated) -- for a consumer that forms dz itself on load (csrc/bwd_stream.hip BN mode)
DPA_API int dpa_bn_bwd_coef(const bf16_t* g, int ldg, const bf16_t* z, int ldz, long long P, int C, const float* gamma,
                            const float* saved, float* slab, float* coef3, float* dgamma, float* dbeta,
                            const float* beta, int slab_rows, hipStream_t st) {
  int G;
  dim3 grid;
  if (!bn_shape(P, C, G, grid) || (ldg & 7) || (ldz & 7)) return (int)hipErrorInvalidValue;
  if (slab_rows > 0 && beta == nullptr) return (int)hipErrorInvalidValue;
  if (slab_rows <= 0)
    hipLaunchKernelGGL(bn_partial_kernel<1>, grid, dim3(256), 0, st, g, ldg, z, ldz, saved, (long)P, C, G, slab);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, slab, slab_rows > 0 ? slab_rows : (int)grid.x, C,
                     (long)P, gamma, saved, coef3, dgamma, dbeta, beta, slab_rows > 0 ? 1 : 0);
  return (int)hipGetLastError();
}

// training backward: g = dL/d(bn output) (ReLU mask already applied by the consumer) -> dz,
// dgamma/dbeta accumulated.  coef3: scratch [3C].
DPA_API int dpa_bn_bwd(const bf16_t* g, int ldg, const bf16_t* z, int ldz, bf16_t* dz, int lddz, long long P, int C,
                       const float* gamma, const float* saved, float* slab, float* coef3, float* dgamma, float* dbeta,
                       const float* beta, int slab_rows, hipStream_t st) {
  int G;
  dim3 grid;
  if (!bn_shape(P, C, G, grid) || (ldg & 7) || (ldz & 7) || (lddz & 7)) return (int)hipErrorInvalidValue;
  // slab_rows > 0: (sum g, sum g*y) partials already written by the producing dgrad (needs beta)
  if (slab_rows > 0 && beta == nullptr) return (int)hipErrorInvalidValue;
  if (slab_rows <= 0)
    hipLaunchKernelGGL(bn_partial_kernel<1>, grid, dim3(256), 0, st, g, ldg, z, ldz, saved, (long)P, C, G, slab);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, slab, slab_rows > 0 ? slab_rows : (int)grid.x, C,
                     (long)P, gamma, saved, coef3, dgamma, dbeta, beta, slab_rows > 0 ? 1 : 0);
  const long tot = (long)P * (C / 8);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, g, ldg, z, ldz, coef3, dz, lddz,
                     (long)P, C);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ bilinear x2
// torch upsample_bilinear2d, align_corners=False, scale 2: src = max((o + 0.5)/2 - 0.5, 0)
__device__ __forceinline__ void up_src(int o, int I, int& i0, int& i1, float& l1) {
  const float src = fmaxf((o + 0.5f) * 0.5f - 0.5f, 0.f);
  i0 = min((int)src, I - 1);
  i1 = min(i0 + 1, I - 1);
  l1 = src - (float)i0;
}

// y[n][oh][ow][c] (2h x 2w, y may be the second half of a concat buffer) from x[n][h][w][c]
__global__ __launch_bounds__(256) void up2_fwd_kernel(const bf16_t* __restrict__ x, int ldx, bf16_t* __restrict__ y, int ldy,
                                                      int N, int h, int w, int C) {
  const int CC = C >> 3, Ho = 2 * h, Wo = 2 * w;
  const long tot = (long)N * Ho * Wo * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long op = i / CC;
    const int ow = (int)(op % Wo);
    const long t = op / Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
    int h0, h1, w0, w1;
    float lh, lw;
    up_src(oh, h, h0, h1, lh);
    up_src(ow, w, w0, w1, lw);
    const long base = (long)n * h * w;
    const bf16_t* xc = x + cc * 8;
    const uint4 a = *reinterpret_cast<const uint4*>(xc + (base + (long)h0 * w + w0) * ldx);
    const uint4 b = *reinterpret_cast<const uint4*>(xc + (base + (long)h0 * w + w1) * ldx);
    const uint4 c = *reinterpret_cast<const uint4*>(xc + (base + (long)h1 * w + w0) * ldx);
    const uint4 d = *reinterpret_cast<const uint4*>(xc + (base + (long)h1 * w + w1) * ldx);
    const unsigned *pa = &a.x, *pb = &b.x, *pc = &c.x, *pd = &d.x;
    const float h0l = 1.f - lh, w0l = 1.f - lw;
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v0 = h0l * (w0l * lo_bf(pa[e]) + lw * lo_bf(pb[e])) + lh * (w0l * lo_bf(pc[e]) + lw * lo_bf(pd[e]));
      const float v1 = h0l * (w0l * hi_bf(pa[e]) + lw * hi_bf(pb[e])) + lh * (w0l * hi_bf(pc[e]) + lw * hi_bf(pd[e]));
      o[e] = pack_bf2(v0, v1);
    }
    *reinterpret_cast<uint4*>(y + op * ldy + cc * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// weight of input index i in output o's interpolation (0 if o does not touch i)
__device__ __forceinline__ float up_weight(int o, int I, int i) {
  int i0, i1;
  float l1;
  up_src(o, I, i0, i1, l1);
  return (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
}

// Backward as a gather (deterministic, no atomics): dx[i][j] = sum over the <= 5x5 output
// neighbourhood o in [2i-2, 2i+2] of w_h(o, i) w_w(o', j) g[o][o'].
__global__ __launch_bounds__(256) void up2_bwd_kernel(const bf16_t* __restrict__ g, int ldg, bf16_t* __restrict__ dx, int lddx,
                                                      int N, int h, int w, int C) {
  const int CC = C >> 3, Ho = 2 * h, Wo = 2 * w;
  const long tot = (long)N * h * w * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long ip = i / CC;
    const int iw = (int)(ip % w);
    const long t = ip / w;
    const int ih = (int)(t % h);
    const int n = (int)(t / h);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int oh0 = max(2 * ih - 2, 0), oh1 = min(2 * ih + 2, Ho - 1);
    const int ow0 = max(2 * iw - 2, 0), ow1 = min(2 * iw + 2, Wo - 1);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const float wh = up_weight(oh, h, ih);
      if (wh == 0.f) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const float ww = up_weight(ow, w, iw);
        if (ww == 0.f) continue;
        const float wt = wh * ww;
        const uint4 u = *reinterpret_cast<const uint4*>(g + (((long)n * Ho + oh) * Wo + ow) * ldg + cc * 8);
        const unsigned* pu = &u.x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] = fmaf(wt, lo_bf(pu[e]), acc[2 * e]);
          acc[2 * e + 1] = fmaf(wt, hi_bf(pu[e]), acc[2 * e + 1]);
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + ip * lddx + cc * 8) =
        make_uint4(pack_bf2(acc[0], acc[1]), pack_bf2(acc[2], acc[3]), pack_bf2(acc[4], acc[5]), pack_bf2(acc[6], acc[7]));
  }
}

DPA_API int dpa_up2_fwd(const bf16_t* x, int ldx, bf16_t* y, int ldy, int N, int h, int w, int C, hipStream_t st) {
  if ((C & 7) || (ldx & 7) || (ldy & 7) || h < 1 || w < 1) return (int)hipErrorInvalidValue;
  const long tot = (long)N * 4 * h * w * (C / 8);
  hipLaunchKernelGGL(up2_fwd_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, x, ldx, y, ldy, N, h, w, C);
  return (int)hipGetLastError();
}

DPA_API int dpa_up2_bwd(const bf16_t* g, int ldg, bf16_t* dx, int lddx, int N, int h, int w, int C, hipStream_t st) {
  if ((C & 7) || (ldg & 7) || (lddx & 7) || h < 1 || w < 1) return (int)hipErrorInvalidValue;
  const long tot = (long)N * h * w * (C / 8);
  hipLaunchKernelGGL(up2_bwd_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, g, ldg, dx, lddx, N, h, w, C);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ fp32 forms
// The fp32 engine (models/hip_unet_f32.py: the reference's precision, utils/train_utils.py:60-61) for the
// BatchNorm and bilinear variants: the same statistics / finalize kernels above (the slab is fp32 either
// way), fp32 NHWC activations read and written 4 channels (16 B) per lane.
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_f32_kernel(const float* __restrict__ a, int lda, const float* __restrict__ z,
                                                             int ldz, const float* __restrict__ saved, long P, int C, int G,
                                                             float* __restrict__ slab) {
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x;
  const int R = 256 / G;
  const int g = tid % G, r = tid / G;
  const int c0 = (blockIdx.y * G + g) * 4;
  float s[4], q[4], mu[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s[k] = 0.f;
    q[k] = 0.f;
    mu[k] = MODE ? saved[c0 + k] : 0.f;
  }
  for (long p = (long)blockIdx.x * R + r; p < P; p += (long)gridDim.x * R) {
    const float4 u = *reinterpret_cast<const float4*>(a + p * lda + c0);
    const float v[4] = {u.x, u.y, u.z, u.w};
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[k] += v[k];
        q[k] = fmaf(v[k], v[k], q[k]);
      }
    } else {
      const float4 w = *reinterpret_cast<const float4*>(z + p * ldz + c0);
      const float zz[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[k] += v[k];
        q[k] = fmaf(v[k], zz[k] - mu[k], q[k]);
      }
    }
  }
  float* row = red + r * (G * 8) + g * 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    row[k] = s[k];
    row[4 + k] = q[k];
  }
  __syncthreads();
  for (int j = tid; j < G * 8; j += 256) {
    float acc = 0.f;
    for (int rr = 0; rr < R; ++rr) acc += red[rr * G * 8 + j];
    const int gg = j >> 3, k = j & 7;
    const int c = (blockIdx.y * G + gg) * 4 + (k & 3);
    slab[(long)blockIdx.x * 2 * C + (k >> 2) * C + c] = acc;
  }
}

// y = relu?(z*coef[c] + coef[C+c])
__global__ __launch_bounds__(256) void bn_apply_f32_kernel(const float* __restrict__ z, int ldz, float* __restrict__ y, int ldy,
                                                           const float* __restrict__ coef, long P, int C, int relu) {
  const int CC = C >> 2;
  const long tot = P * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % CC) * 4;
    const long p = i / CC;
    const float4 u = *reinterpret_cast<const float4*>(z + p * ldz + c0);
    float v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = fmaf(v[k], coef[c0 + k], coef[C + c0 + k]);
      if (relu) v[k] = fmaxf(v[k], 0.f);
    }
    *reinterpret_cast<float4*>(y + p * ldy + c0) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// dz = coef3[c]*g + coef3[C+c]*z + coef3[2C+c]
__global__ __launch_bounds__(256) void bn_bwd_apply_f32_kernel(const float* __restrict__ g, int ldg, const float* __restrict__ z,
                                                               int ldz, const float* __restrict__ coef3, float* __restrict__ dz,
                                                               int lddz, long P, int C) {
  const int CC = C >> 2;
  const long tot = P * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % CC) * 4;
    const long p = i / CC;
    const float4 ug = *reinterpret_cast<const float4*>(g + p * ldg + c0);
    const float4 uz = *reinterpret_cast<const float4*>(z + p * ldz + c0);
    const float gv[4] = {ug.x, ug.y, ug.z, ug.w}, zv[4] = {uz.x, uz.y, uz.z, uz.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = fmaf(coef3[c0 + k], gv[k], fmaf(coef3[C + c0 + k], zv[k], coef3[2 * C + c0 + k]));
    *reinterpret_cast<float4*>(dz + p * lddz + c0) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

static bool bn_shape_f32(long P, int C, int& G, dim3& grid) {
  if (C <= 0 || (C & 3) || P <= 0) return false;
  const int CG = C / 4;
  G = 1;
  while (G * 2 <= 32 && CG % (G * 2) == 0) G *= 2;
  const int R = 256 / G;
  long nbx = (P + R - 1) / R;
  if (nbx > 512) nbx = 512;
  grid = dim3((unsigned)nbx, (unsigned)(CG / G));
  return true;
}

DPA_API int dpa_bn_slab_rows_f32(long long P, int C) {
  int G;
  dim3 grid;
  return bn_shape_f32(P, C, G, grid) ? (int)grid.x : 0;
}

// BN(+ReLU) forward, fp32: train -> batch statistics (saved = mean, invstd; running stats updated), eval ->
// running statistics; then y = relu?(bn(z))
DPA_API int dpa_bn_fwd_f32(const float* z, int ldz, float* y, int ldy, long long P, int C, const float* gamma,
                           const float* beta, float eps, float momentum, float* rmean, float* rvar, float* slab, float* coef,
                           float* saved, int train, int relu, hipStream_t st) {
  int G;
  dim3 grid;
  if (!bn_shape_f32(P, C, G, grid) || (ldz & 3) || (ldy & 3)) return (int)hipErrorInvalidValue;
  if (train) {
    hipLaunchKernelGGL(bn_partial_f32_kernel<0>, grid, dim3(256), 0, st, z, ldz, (const float*)nullptr, 0,
                       (const float*)nullptr, (long)P, C, G, slab);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, slab, (int)grid.x, C, (long)P, gamma, beta, eps,
                       momentum, rmean, rvar, coef, saved);
  } else {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, (const float*)nullptr, 0, C, (long)P, gamma, beta, eps,
                       momentum, rmean, rvar, coef, saved);
  }
  const long tot = (long)P * (C / 4);
  hipLaunchKernelGGL(bn_apply_f32_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, z, ldz, y, ldy, coef, (long)P, C,
                     relu);
  return (int)hipGetLastError();
}

// BN backward, fp32: g = dL/d(bn output) with the ReLU mask applied -> dz; dgamma / dbeta accumulated
DPA_API int dpa_bn_bwd_f32(const float* g, int ldg, const float* z, int ldz, float* dz, int lddz, long long P, int C,
                           const float* gamma, const float* saved, float* slab, float* coef3, float* dgamma, float* dbeta,
                           hipStream_t st) {
  int G;
  dim3 grid;
  if (!bn_shape_f32(P, C, G, grid) || (ldg & 3) || (ldz & 3) || (lddz & 3)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_partial_f32_kernel<1>, grid, dim3(256), 0, st, g, ldg, z, ldz, saved, (long)P, C, G, slab);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, slab, (int)grid.x, C, (long)P, gamma, saved, coef3,
                     dgamma, dbeta, (const float*)nullptr, 0);
  const long tot = (long)P * (C / 4);
  hipLaunchKernelGGL(bn_bwd_apply_f32_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, g, ldg, z, ldz, coef3, dz,
                     lddz, (long)P, C);
  return (int)hipGetLastError();
}

// bilinear x2 (align_corners=False), fp32 NHWC, 4 channels per lane
__global__ __launch_bounds__(256) void up2_fwd_f32_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y, int ldy,
                                                          int N, int h, int w, int C) {
  const int CC = C >> 2, Ho = 2 * h, Wo = 2 * w;
  const long tot = (long)N * Ho * Wo * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long op = i / CC;
    const int ow = (int)(op % Wo);
    const long t = op / Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
    int h0, h1, w0, w1;
    float lh, lw;
    up_src(oh, h, h0, h1, lh);
    up_src(ow, w, w0, w1, lw);
    const long base = (long)n * h * w;
    const float* xc = x + cc * 4;
    const float4 a = *reinterpret_cast<const float4*>(xc + (base + (long)h0 * w + w0) * ldx);
    const float4 b = *reinterpret_cast<const float4*>(xc + (base + (long)h0 * w + w1) * ldx);
    const float4 c = *reinterpret_cast<const float4*>(xc + (base + (long)h1 * w + w0) * ldx);
    const float4 d = *reinterpret_cast<const float4*>(xc + (base + (long)h1 * w + w1) * ldx);
    const float h0l = 1.f - lh, w0l = 1.f - lw;
    float4 o;
    o.x = h0l * (w0l * a.x + lw * b.x) + lh * (w0l * c.x + lw * d.x);
    o.y = h0l * (w0l * a.y + lw * b.y) + lh * (w0l * c.y + lw * d.y);
    o.z = h0l * (w0l * a.z + lw * b.z) + lh * (w0l * c.z + lw * d.z);
    o.w = h0l * (w0l * a.w + lw * b.w) + lh * (w0l * c.w + lw * d.w);
    *reinterpret_cast<float4*>(y + op * ldy + cc * 4) = o;
  }
}

__global__ __launch_bounds__(256) void up2_bwd_f32_kernel(const float* __restrict__ g, int ldg, float* __restrict__ dx, int lddx,
                                                          int N, int h, int w, int C) {
  const int CC = C >> 2, Ho = 2 * h, Wo = 2 * w;
  const long tot = (long)N * h * w * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long ip = i / CC;
    const int iw = (int)(ip % w);
    const long t = ip / w;
    const int ih = (int)(t % h);
    const int n = (int)(t / h);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int oh0 = max(2 * ih - 2, 0), oh1 = min(2 * ih + 2, Ho - 1);
    const int ow0 = max(2 * iw - 2, 0), ow1 = min(2 * iw + 2, Wo - 1);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const float wh = up_weight(oh, h, ih);
      if (wh == 0.f) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const float ww = up_weight(ow, w, iw);
        if (ww == 0.f) continue;
        const float wt = wh * ww;
        const float4 u = *reinterpret_cast<const float4*>(g + (((long)n * Ho + oh) * Wo + ow) * ldg + cc * 4);
        acc[0] = fmaf(wt, u.x, acc[0]);
        acc[1] = fmaf(wt, u.y, acc[1]);
        acc[2] = fmaf(wt, u.z, acc[2]);
        acc[3] = fmaf(wt, u.w, acc[3]);
      }
    }
    *reinterpret_cast<float4*>(dx + ip * lddx + cc * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

DPA_API int dpa_up2_fwd_f32(const float* x, int ldx, float* y, int ldy, int N, int h, int w, int C, hipStream_t st) {
  if ((C & 3) || (ldx & 3) || (ldy & 3) || h < 1 || w < 1) return (int)hipErrorInvalidValue;
  const long tot = (long)N * 4 * h * w * (C / 4);
  hipLaunchKernelGGL(up2_fwd_f32_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, x, ldx, y, ldy, N, h, w, C);
  return (int)hipGetLastError();
}

DPA_API int dpa_up2_bwd_f32(const float* g, int ldg, float* dx, int lddx, int N, int h, int w, int C, hipStream_t st) {
  if ((C & 3) || (ldg & 3) || (lddx & 3) || h < 1 || w < 1) return (int)hipErrorInvalidValue;
  const long tot = (long)N * h * w * (C / 4);
  hipLaunchKernelGGL(up2_bwd_f32_kernel, dim3(dpa_grid(tot, 256, 16384)), dim3(256), 0, st, g, ldg, dx, lddx, N, h, w, C);
  return (int)hipGetLastError();
}
