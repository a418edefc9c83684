// Memory-bound UNet kernels for gfx950 (everything that is not a GEMM), all NHWC bf16, 16-byte
// vector accesses (8 channels per lane), fp32 math:
//   * input conversion fp32 NCHW [B,3,H,W] -> bf16 NHWC8 (zero channels 3..7)  
//   * 2x2/s2 max-pool, reading the skip from the decoder's concat buffer        (K5 fwd)
//   * fused max-pool backward + skip-gradient add + ReLU-backward mask          (K5 bwd + K7 + K4 bwd)
//   * batched weight packing fp32 PyTorch layout -> bf16 GEMM layouts (one launch per step)
//   * fused 1x1 segmap + sigmoid + BCE + Dice partial sums, and its fused backward (K8-K11)
// Reference semantics: model/unet_parts.py:26-41 (MaxPool2d(2,2)), model/unet_model.py:10-11
// (segmap, Sigmoid), utils/utils.py:9-25 (BCE - log Dice, global over the batch).
#include "common.h"
#include "conv_args.h"

#include <hip/hip_ext.h>

#include <type_traits>
#include <vector>

// ------------------------------------------------------------------------------ input conversion
__global__ __launch_bounds__(256) void nchw3_to_nhwc8_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int B,
                                                             int C, int HW) {
  const long tot = (long)B * HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const long b = i / HW, p = i - b * HW;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < C && c < 8; ++c) v[c] = x[(b * C + c) * HW + p];
    uint4 o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
    *reinterpret_cast<uint4*>(y + i * 8) = o;
  }
}
DPA_API int dpa_input_nhwc8(const float* x, bf16_t* y, int B, int C, int H, int W, hipStream_t st) {
  if (C > 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(nchw3_to_nhwc8_kernel, dim3(dpa_grid((long)B * H * W, 256, 8192)), dim3(256), 0, st, x, y, B, C, H * W);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ max-pool 2x2 / s2
// Floor semantics (nn.MaxPool2d(2,2)); first maximum in scan order wins (matches PyTorch).
__global__ __launch_bounds__(256) void maxpool2_kernel(const bf16_t* __restrict__ x, int ldx, bf16_t* __restrict__ y, int ldy,
                                                       int N, int H, int W, int C, unsigned char* __restrict__ code) {
  const int Ho = H / 2, Wo = W / 2, CC = C / 8;
  const long tot = (long)N * Ho * Wo * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long op = i / CC;
    const int ow = (int)(op % Wo);
    const long t = op / Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const long p00 = ((long)(n * H + 2 * oh) * W + 2 * ow);
    const uint4 a = *reinterpret_cast<const uint4*>(x + p00 * ldx + cc * 8);
    const uint4 b = *reinterpret_cast<const uint4*>(x + (p00 + 1) * ldx + cc * 8);
    const uint4 c = *reinterpret_cast<const uint4*>(x + (p00 + W) * ldx + cc * 8);
    const uint4 d = *reinterpret_cast<const uint4*>(x + (p00 + W + 1) * ldx + cc * 8);
    const unsigned int* pa = &a.x; const unsigned int* pb = &b.x; const unsigned int* pc = &c.x; const unsigned int* pd = &d.x;
    unsigned int o[4], cd[2] = {0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float l = fmaxf(fmaxf(lo_bf(pa[k]), lo_bf(pb[k])), fmaxf(lo_bf(pc[k]), lo_bf(pd[k])));
      float h = fmaxf(fmaxf(hi_bf(pa[k]), hi_bf(pb[k])), fmaxf(hi_bf(pc[k]), hi_bf(pd[k])));
      o[k] = pack_bf2(l, h);
      if (code) {
        const unsigned cl = pool_code(lo_bf(pa[k]), lo_bf(pb[k]), lo_bf(pc[k]), lo_bf(pd[k]));
        const unsigned ch = pool_code(hi_bf(pa[k]), hi_bf(pb[k]), hi_bf(pc[k]), hi_bf(pd[k]));
        cd[k >> 1] |= (cl | ch << 8) << (16 * (k & 1));
      }
    }
    *reinterpret_cast<uint4*>(y + op * ldy + cc * 8) = make_uint4(o[0], o[1], o[2], o[3]);
    if (code) *reinterpret_cast<uint2*>(code + op * C + cc * 8) = make_uint2(cd[0], cd[1]);
  }
}
DPA_API int dpa_maxpool2(const bf16_t* x, int ldx, bf16_t* y, int ldy, int N, int H, int W, int C, unsigned char* code,
                         hipStream_t st) {
  if ((C & 7) || (ldx & 7) || (ldy & 7)) return (int)hipErrorInvalidValue;
  const long tot = (long)N * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(maxpool2_kernel, dim3(dpa_grid(tot, 256, 8192)), dim3(256), 0, st, x, ldx, y, ldy, N, H, W, C, code);
  return (int)hipGetLastError();
}

// Max-pool backward from window codes (even H, W): one thread per (2x2 window, 8 channels).  The
// window's code and dpool are loaded once for its 4 pixels, all 4 dskip loads are issued before
// any math (4 independent 16-B loads in flight per lane), and the index math is one div chain per
// window.  A wave covers 64/CC consecutive windows of one pooled row: each of its loads/stores
// touches full 64-B runs of the two full-resolution rows.
//   g[p][c] = (dskip[p][c] + (argmax(window)[c] == q(p) ? dpool[window][c] : 0)) * mask_q(p)[c]
// BNS: the pooled tensor y (= the skip) is a BatchNorm+ReLU output: also the BN backward's partial sums of the
// STORED bf16 g, sum g[c] and sum g[c] * y[c], per block -> bnslab[block][2][C] (no statistics pass over g, z).
// A thread's channel chunk is fixed (256 % C/8 == 0 for C <= 512), so per-thread sums reduce per chunk.
// ZBN (with BNS): `y` holds the BN input z (dense) and y = relu(z * coef[c] + coef[C + c]) is formed on load
// with bn_apply_pool_kernel's arithmetic -- the skip y itself may be a strided concat half (ldy = 2C), z is not.
template <bool BNS = false, bool ZBN = false>
__global__ __launch_bounds__(256) void pool_bwd_code_kernel(const unsigned char* __restrict__ code,
                                                            const bf16_t* __restrict__ dskip, int ldd,
                                                            const bf16_t* __restrict__ dpool, int ldp,
                                                            bf16_t* __restrict__ g, int ldg, int N, int H, int W, int C,
                                                            const bf16_t* __restrict__ y, int ldy, float* __restrict__ bnslab,
                                                            const float* __restrict__ coef) {
  const int CC = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const unsigned tot = (unsigned)N * Ho * Wo * CC;
  float sg[BNS ? 8 : 1], sgy[BNS ? 8 : 1], zsc[ZBN ? 8 : 1], zsh[ZBN ? 8 : 1];
  if constexpr (BNS) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sg[k] = sgy[k] = 0.f;
  }
  if constexpr (ZBN) {        // this thread's channel chunk is fixed (see below)
    const int c0 = (int)((blockIdx.x * blockDim.x + threadIdx.x) % (unsigned)CC) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      zsc[k] = coef[c0 + k];
      zsh[k] = coef[C + c0 + k];
    }
  }
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
    const unsigned cc = i % CC, win = i / CC;
    const unsigned ow = win % Wo, noh = win / Wo;          // noh = n * Ho + oh
    const size_t p00 = (size_t)noh * 2 * W + 2 * ow;        // (n*H + 2*oh) * W + 2*ow
    const size_t pix[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    const uint2 cw = *reinterpret_cast<const uint2*>(code + (size_t)win * C + cc * 8);
    const uint4 dp = *reinterpret_cast<const uint4*>(dpool + (size_t)win * ldp + cc * 8);
    uint4 ds[4], yv[BNS ? 4 : 1];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      ds[q] = dskip ? *reinterpret_cast<const uint4*>(dskip + pix[q] * ldd + cc * 8) : make_uint4(0u, 0u, 0u, 0u);
    if constexpr (BNS) {      // issued with the other loads: 8 independent 16-B loads in flight per lane
#pragma unroll
      for (int q = 0; q < 4; ++q) yv[q] = *reinterpret_cast<const uint4*>(y + pix[q] * ldy + cc * 8);
    }
    const unsigned* pd = &dp.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned* ps = &ds[q].x;
      unsigned o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned c2 = (k < 2 ? cw.x : cw.y) >> (16 * (k & 1));   // codes of channels 2k, 2k+1
        const unsigned cl = c2 & 0xffu, ch = (c2 >> 8) & 0xffu;
        float lo = lo_bf(ps[k]) + ((cl & 3u) == (unsigned)q ? lo_bf(pd[k]) : 0.f);
        float hi = hi_bf(ps[k]) + ((ch & 3u) == (unsigned)q ? hi_bf(pd[k]) : 0.f);
        lo = (cl >> (2 + q)) & 1u ? lo : 0.f;
        hi = (ch >> (2 + q)) & 1u ? hi : 0.f;
        o[k] = pack_bf2(lo, hi);
      }
      *reinterpret_cast<uint4*>(g + pix[q] * ldg + cc * 8) = make_uint4(o[0], o[1], o[2], o[3]);
      if constexpr (BNS) {
        const unsigned* py = &yv[q].x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float g0 = lo_bf(o[k]), g1 = hi_bf(o[k]);
          unsigned yk = py[k];
          if constexpr (ZBN)
            yk = pack_bf2(fmaxf(fmaf(lo_bf(yk), zsc[2 * k], zsh[2 * k]), 0.f),
                          fmaxf(fmaf(hi_bf(yk), zsc[2 * k + 1], zsh[2 * k + 1]), 0.f));
          sg[2 * k] += g0;
          sg[2 * k + 1] += g1;
          sgy[2 * k] = fmaf(g0, lo_bf(yk), sgy[2 * k]);
          sgy[2 * k + 1] = fmaf(g1, hi_bf(yk), sgy[2 * k + 1]);
        }
      }
    }
  }
  if constexpr (BNS) {
    // thread t holds chunk t % CC; the 256 / CC threads of a chunk are summed in thread order
    __shared__ float red[256][17];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[threadIdx.x][k] = sg[k];
      red[threadIdx.x][8 + k] = sgy[k];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * C; j += 256) {
      const int which = j / C, c = j - which * C, chunk = c >> 3, k = c & 7;
      float acc = 0.f;
      for (int t = chunk; t < 256; t += CC) acc += red[t][8 * which + k];
      bnslab[(long)blockIdx.x * 2 * C + j] = acc;
    }
  }
}
// blocks of a launch (rows of its BN slab): dpa_pool_bwd_code_blocks
DPA_API int dpa_pool_bwd_code_blocks(int N, int H, int W, int C) {
  return dpa_grid((long)N * (H / 2) * (W / 2) * (C / 8), 256, 16384);
}

// y / bnslab (or null): the BatchNorm partial sums of g against y (pool_bwd_code_kernel BNS), C <= 512;
// coef (or null, needs bnslab): y is the BN input z, relu(bn(z)) formed on load (ZBN)
DPA_API int dpa_pool_bwd_code(const unsigned char* code, const bf16_t* dskip, int ldd, const bf16_t* dpool, int ldp,
                              bf16_t* g, int ldg, int N, int H, int W, int C, const bf16_t* y, int ldy, float* bnslab,
                              const float* coef, hipStream_t st) {
  if ((C & 7) || (ldd & 7) || (ldp & 7) || (ldg & 7) || (H & 1) || (W & 1)) return (int)hipErrorInvalidValue;
  if (bnslab && (!y || (ldy & 7) || C > 512)) return (int)hipErrorInvalidValue;
  if (coef && !bnslab) return (int)hipErrorInvalidValue;
  const long tot = (long)N * (H / 2) * (W / 2) * (C / 8);
  if ((long)N * H * W * (C / 8) >= (1l << 31)) return (int)hipErrorInvalidValue;
  const dim3 grid(dpa_pool_bwd_code_blocks(N, H, W, C));
#define DPA_PB(BN, ZB) hipLaunchKernelGGL((pool_bwd_code_kernel<BN, ZB>), grid, dim3(256), 0, st, code, dskip, ldd, dpool, ldp, g, ldg, N, H, W, C, y, ldy, bnslab, coef)
  if (coef)
    DPA_PB(true, true);
  else if (bnslab)
    DPA_PB(true, false);
  else
    DPA_PB(false, false);
#undef DPA_PB
  (void)tot;
  return (int)hipGetLastError();
}

// g[p][c] = (dskip[p][c] + (p is the window argmax ? dpool[p/2][c] : 0)) * (skip[p][c] > 0)
// dskip may be null (no decoder contribution).  Pixels outside the pooled area (odd H/W) get only dskip.
__global__ __launch_bounds__(256) void pool_bwd_kernel(const bf16_t* __restrict__ skip, int lds, const bf16_t* __restrict__ dskip,
                                                       int ldd, const bf16_t* __restrict__ dpool, int ldp, bf16_t* __restrict__ g,
                                                       int ldg, int N, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CC = C / 8;
  const int Hw = (H + 1) / 2, Ww = (W + 1) / 2;   // windows covering every pixel
  const long tot = (long)N * Hw * Ww * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long op = i / CC;
    const int ow = (int)(op % Ww);
    const long t = op / Ww;
    const int oh = (int)(t % Hw);
    const int n = (int)(t / Hw);
    const bool pooled = oh < Ho && ow < Wo;
    float dp[8];
    if (pooled) {
      const uint4 v = *reinterpret_cast<const uint4*>(dpool + ((long)(n * Ho + oh) * Wo + ow) * ldp + cc * 8);
      const unsigned int* pv = &v.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) { dp[2 * k] = lo_bf(pv[k]); dp[2 * k + 1] = hi_bf(pv[k]); }
    }
    float sv[4][8];
    long pix[4];
    bool in[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * oh + (q >> 1), w = 2 * ow + (q & 1);
      in[q] = h < H && w < W;
      pix[q] = ((long)(n * H + h) * W + w);
      if (in[q]) {
        const uint4 v = *reinterpret_cast<const uint4*>(skip + pix[q] * lds + cc * 8);
        const unsigned int* pv = &v.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) { sv[q][2 * k] = lo_bf(pv[k]); sv[q][2 * k + 1] = hi_bf(pv[k]); }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) sv[q][k] = 0.f;
      }
    }
    int am[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int best = 0;
      float bv = sv[0][k];
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (sv[q][k] > bv) { bv = sv[q][k]; best = q; }
      am[k] = best;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!in[q]) continue;
      float o[8];
      if (dskip) {
        const uint4 v = *reinterpret_cast<const uint4*>(dskip + pix[q] * ldd + cc * 8);
        const unsigned int* pv = &v.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[2 * k] = lo_bf(pv[k]); o[2 * k + 1] = hi_bf(pv[k]); }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (pooled && am[k] == q) o[k] += dp[k];
        if (!(sv[q][k] > 0.f)) o[k] = 0.f;
      }
      *reinterpret_cast<uint4*>(g + pix[q] * ldg + cc * 8) =
          make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
    }
  }
}
DPA_API int dpa_pool_bwd(const bf16_t* skip, int lds, const bf16_t* dskip, int ldd, const bf16_t* dpool, int ldp, bf16_t* g,
                         int ldg, int N, int H, int W, int C, hipStream_t st) {
  if ((C & 7) || (lds & 7) || (ldd & 7) || (ldp & 7) || (ldg & 7)) return (int)hipErrorInvalidValue;
  const long tot = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(dpa_grid(tot, 256, 8192)), dim3(256), 0, st, skip, lds, dskip, ldd, dpool, ldp, g, ldg,
                     N, H, W, C);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ weight packing
// One launch packs every layer: blockIdx.y selects a descriptor.
//   mode 0: Conv2d fwd     dst[co][tap*Cs + ci]      = W[co][ci][tap]          (Ngemm=Cout, K=9*Cs)
//   mode 1: Conv2d dgrad   dst[ci][tap*Cout + co]    = W[co][ci][8-tap]        (Ngemm=Cin,  K=9*Cout)
//   mode 2: ConvT fwd      dst[(2i+j)*Cout+co][ci]   = W[ci][co][i][j]         (Ngemm=4*Cout, K=Cin)
//   mode 3: ConvT dgrad    dst[ci][(2i+j)*Cout+co]   = W[ci][co][i][j]         (Ngemm=Cin, K=4*Cout)
//   mode 4: Conv1x1 fwd    dst[co][ci]               = W[co][ci]               (Ngemm=Cout, K=Cin)
//   mode 5: Conv1x1 dgrad  dst[ci][co]               = W[co][ci]               (Ngemm=Cin,  K=Cout)
// k >= K (padding to Kpad) and ci >= Cin (first-layer channel padding) are zero.
struct PackDesc {
  long long src;   // device address of the fp32 weight (PyTorch layout)
  long long dst;   // element offset in the packed bf16 buffer
  int mode, Cout, Cin, Cs, Ngemm, Kpad;
};
// Conv2d modes 0 / 1 go one thread per (GEMM row, channel) over all 9 taps: the thread reads the 9 contiguous
// taps W[co][ci][0..8] (36 B; consecutive lanes read consecutive 36-B runs in mode 0) and writes 9 packed values,
// each store coalesced across lanes (consecutive channels).  The per-element form below gathered mode 1 with a
// Cin*36-B lane stride (one cache line per element): 1.08 ms per UNet-XL step for ~0.25 GB of weights.
// 32-bit index math throughout (the host checks Ngemm * Kpad < 2^31).
template <typename OutT>
__device__ __forceinline__ void pack_store(OutT* p, long idx, float v) {
  if constexpr (std::is_same<OutT, float>::value) p[idx] = v;
  else p[idx] = f2bf(v);
}
template <typename OutT>
__global__ __launch_bounds__(256) void pack_kernel(OutT* __restrict__ packed, const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  const unsigned stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (d.mode == 0 || d.mode == 1) {
    const float* W = reinterpret_cast<const float*>(d.src);
    OutT* dst = packed + d.dst;
    const int C = d.mode == 0 ? d.Cs : d.Cout;      // channels per tap in the packed row
    const unsigned rows = (unsigned)d.Ngemm * (unsigned)C;
    for (unsigned i = t0; i < rows; i += stride) {
      const unsigned n = i / (unsigned)C, c = i - n * (unsigned)C;
      float w[9];
      // mode 0: row n = co, channel c = ci (ci >= Cin: first-layer padding); mode 1: row n = ci (n >= Cin:
      // GEMM-N padding), channel c = co, taps flipped
      const bool ok = d.mode == 0 ? (int)c < d.Cin : (int)n < d.Cin;
      const float* src = W + (d.mode == 0 ? ((long)n * d.Cin + c) * 9 : ((long)c * d.Cin + n) * 9);
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t] = ok ? src[t] : 0.f;
      const long row = (long)n * d.Kpad;
#pragma unroll
      for (int t = 0; t < 9; ++t) pack_store(dst, row + t * C + c, d.mode == 0 ? w[t] : w[8 - t]);
    }
    // K padding columns [9 C, Kpad) of every row
    const unsigned padw = (unsigned)(d.Kpad - 9 * C), npad = (unsigned)d.Ngemm * padw;
    for (unsigned i = t0; i < npad; i += stride) {
      const unsigned n = i / padw, k = 9 * C + (i - n * padw);
      pack_store(dst, (long)n * d.Kpad + k, 0.f);
    }
    return;
  }
  const long tot = (long)d.Ngemm * d.Kpad;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / d.Kpad), k = (int)(i - (long)n * d.Kpad);
    float v = 0.f;
    const float* W = reinterpret_cast<const float*>(d.src);
    if (d.mode == 0) {
      const int tap = k / d.Cs, ci = k - tap * d.Cs;
      if (tap < 9 && ci < d.Cin) v = W[((long)n * d.Cin + ci) * 9 + tap];
    } else if (d.mode == 1) {
      const int tap = k / d.Cout, co = k - tap * d.Cout;
      if (tap < 9 && n < d.Cin) v = W[((long)co * d.Cin + n) * 9 + (8 - tap)];
    } else if (d.mode == 2) {
      const int ij = n / d.Cout, co = n - ij * d.Cout;
      if (k < d.Cin) v = W[((long)k * d.Cout + co) * 4 + ij];
    } else if (d.mode == 3) {
      const int ij = k / d.Cout, co = k - ij * d.Cout;
      if (ij < 4) v = W[((long)n * d.Cout + co) * 4 + ij];
    } else if (d.mode == 4) {
      if (k < d.Cin) v = W[(long)n * d.Cin + k];
    } else {
      if (k < d.Cout) v = W[(long)k * d.Cin + n];
    }
    if constexpr (std::is_same<OutT, float>::value) packed[d.dst + i] = v;
    else packed[d.dst + i] = f2bf(v);
  }
}
DPA_API int dpa_pack_weights(const float* flat, bf16_t* packed, const void* descs, int ndesc, long long max_elems,
                             hipStream_t st) {
  if (ndesc <= 0) return 0;
  if (max_elems >= (1ll << 31)) return (int)hipErrorInvalidValue;   // 32-bit index math
  dim3 grid(dpa_grid(max_elems, 256, 1024), ndesc);
  (void)flat;
  hipLaunchKernelGGL(pack_kernel<bf16_t>, grid, dim3(256), 0, st, packed, reinterpret_cast<const PackDesc*>(descs));
  return (int)hipGetLastError();
}
// the fp32 engine's packed weights (models/hip_unet_f32.py): the same layouts, fp32 values; mode 1 rows
// n >= Cin (GEMM-N padded to a multiple of 32) are zero
DPA_API int dpa_pack_weights_f32(float* packed, const void* descs, int ndesc, long long max_elems, hipStream_t st) {
  if (ndesc <= 0) return 0;
  if (max_elems >= (1ll << 31)) return (int)hipErrorInvalidValue;   // 32-bit index math
  dim3 grid(dpa_grid(max_elems, 256, 1024), ndesc);
  hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(256), 0, st, packed, reinterpret_cast<const PackDesc*>(descs));
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ head + loss
// z = b + sum_c y[p][c] w[c];  p = sigmoid(z);  BCE with log clamped at -100 (torch.nn.BCELoss);
// partial sums S = [sum BCE, sum p*[t==1], sum p, sum [t==1]] per block -> slab [grid][4].
// If probs != null, p is also written (inference).
#define HEAD_MAXC 64
template <int C>
__device__ __forceinline__ void load_row(const bf16_t* y, float* v) {
#pragma unroll
  for (int k = 0; k < C / 8; ++k) {
    const uint4 u = *reinterpret_cast<const uint4*>(y + k * 8);
    const unsigned int* pu = &u.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[8 * k + 2 * e] = lo_bf(pu[e]); v[8 * k + 2 * e + 1] = hi_bf(pu[e]); }
  }
}

// ZBN: the row holds the last decoder conv's pre-BN output z and y = relu(bn(z)) is formed on load with
// bn_apply_kernel's arithmetic (fp32 fma, ReLU, bf16 rounding), so y is never stored: coef = [scale C | shift C]
template <int C, bool ZBN>
__device__ __forceinline__ void load_row_bn(const bf16_t* y, const float* sc, const float* sh, float* v) {
  load_row<C>(y, v);
  if constexpr (ZBN) {
#pragma unroll
    for (int c = 0; c < C; c += 2) {
      const unsigned o = pack_bf2(fmaxf(fmaf(v[c], sc[c], sh[c]), 0.f), fmaxf(fmaf(v[c + 1], sc[c + 1], sh[c + 1]), 0.f));
      v[c] = lo_bf(o);
      v[c + 1] = hi_bf(o);
    }
  }
}

template <int C, bool ZBN = false>
__global__ __launch_bounds__(256) void head_fwd_kernel(const bf16_t* __restrict__ y, int ldy, const float* __restrict__ w,
                                                       const float* __restrict__ b, const float* __restrict__ t,
                                                       float* __restrict__ slab, float* __restrict__ probs, long P,
                                                       const float* __restrict__ coef) {
  __shared__ float red[4];
  float wv[C], sc[ZBN ? C : 1], sh[ZBN ? C : 1];
#pragma unroll
  for (int c = 0; c < C; ++c) wv[c] = w[c];
  if constexpr (ZBN) {
#pragma unroll
    for (int c = 0; c < C; ++c) { sc[c] = coef[c]; sh[c] = coef[C + c]; }
  }
  const float bias = b[0];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    float v[C];
    load_row_bn<C, ZBN>(y + i * ldy, sc, sh, v);
    float z = bias;
#pragma unroll
    for (int c = 0; c < C; ++c) z = fmaf(v[c], wv[c], z);
    const float p = fast_sigmoid(z);
    if (probs) probs[i] = p;
    if (t) {
      const float tt = t[i];
      const float lp = fmaxf(__logf(p), -100.f), l1p = fmaxf(__logf(1.f - p), -100.f);
      s0 -= tt * lp + (1.f - tt) * l1p;
      const float one = tt == 1.f ? 1.f : 0.f;
      s1 += p * one;
      s2 += p;
      s3 += one;
    }
  }
  if (!slab) return;
  s0 = block_sum_256(s0, red);
  s1 = block_sum_256(s1, red);
  s2 = block_sum_256(s2, red);
  s3 = block_sum_256(s3, red);
  if (threadIdx.x == 0) {
    float* o = slab + 4 * (long)blockIdx.x;
    o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3;
  }
}

// deterministic sum of the [nblk][K] slab into out[K]: one block per column, fixed order
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int nblk, int K, float* __restrict__ out,
                                                       int accumulate) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) s += slab[(long)i * K + k];
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) out[k] = accumulate ? out[k] + s : s;
}

static int head_grid(long P) { return dpa_grid(P, 256, 2048); }

// coef (or null): y is the pre-BN output z of a BatchNorm+ReLU layer, y = relu(z * coef[c] + coef[C + c])
// formed on load (head_fwd_kernel ZBN), C = 32 / 64
DPA_API int dpa_head_fwd(const bf16_t* y, int ldy, int C, const float* w, const float* b, const float* t, float* slab,
                         float* S, float* probs, long long P, const float* coef, hipStream_t st) {
  const int grid = head_grid(P);
  if ((ldy & 7) || (coef && C != 32 && C != 64)) return (int)hipErrorInvalidValue;
#define DPA_HF(Cv, ZB) hipLaunchKernelGGL((head_fwd_kernel<Cv, ZB>), dim3(grid), dim3(256), 0, st, y, ldy, w, b, t, slab, probs, (long)P, coef)
  switch (C) {
    case 8: DPA_HF(8, false); break;
    case 16: DPA_HF(16, false); break;
    case 32: if (coef) DPA_HF(32, true); else DPA_HF(32, false); break;
    case 64: if (coef) DPA_HF(64, true); else DPA_HF(64, false); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DPA_HF
  if (slab && S) hipLaunchKernelGGL(slab_sum_kernel, dim3(4), dim3(256), 0, st, slab, grid, 4, S, 0);
  return (int)hipGetLastError();
}

// Backward.  dS[4] = dLoss/dS (from autograd).  Per pixel (torch formulas: BCE backward
// (p - t) / max(p(1-p), 1e-12), sigmoid backward g*p*(1-p)):
//   dp = dS0 * (p-t)/max(p(1-p),1e-12) + dS1*[t==1] + dS2 ;  dz = dp * p * (1-p)
//   gy[p][c] = dz * w[c] * (y[p][c] > 0)      (ReLU backward of the last decoder conv)
//   dw[c] += dz * y[p][c] ;  db += dz          (block partials -> slab [grid][C+1])
// BNS: the last decoder conv is followed by BatchNorm + ReLU (y = its output): also the BN backward's partial
// sums of the STORED bf16 gradient, sum gy[c] and sum gy[c] * y[c], per block -> bnslab[block][2][C] (the
// conv epilogues' EPI 5 convention), so the BN backward needs no statistics pass over (gy, z)
template <int C, bool BNS = false, bool ZBN = false>
__global__ __launch_bounds__(256) void head_bwd_kernel(const bf16_t* __restrict__ y, int ldy, const float* __restrict__ w,
                                                       const float* __restrict__ b, const float* __restrict__ t,
                                                       const float* __restrict__ dS, bf16_t* __restrict__ gy, int ldg,
                                                       float* __restrict__ slab, long P, float* __restrict__ bnslab,
                                                       const float* __restrict__ coef) {
  __shared__ float red[4];
  float wv[C], dw[C], sc[ZBN ? C : 1], sh[ZBN ? C : 1];
  if constexpr (ZBN) {
#pragma unroll
    for (int c = 0; c < C; ++c) { sc[c] = coef[c]; sh[c] = coef[C + c]; }
  }
  float sg[BNS ? C : 1], sgy[BNS ? C : 1];
#pragma unroll
  for (int c = 0; c < C; ++c) { wv[c] = w[c]; dw[c] = 0.f; }
  if constexpr (BNS) {
#pragma unroll
    for (int c = 0; c < C; ++c) sg[c] = sgy[c] = 0.f;
  }
  const float bias = b[0];
  const float d0 = dS[0], d1 = dS[1], d2 = dS[2];
  float db = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    float v[C];
    load_row_bn<C, ZBN>(y + i * ldy, sc, sh, v);
    float z = bias;
#pragma unroll
    for (int c = 0; c < C; ++c) z = fmaf(v[c], wv[c], z);
    const float p = fast_sigmoid(z);
    const float tt = t[i];
    const float one = tt == 1.f ? 1.f : 0.f;
    const float dz = head_dz(p, tt, one, d0, d1, d2);
    db += dz;
    unsigned int o[C / 2];
#pragma unroll
    for (int c = 0; c < C; c += 2) {
      dw[c] = fmaf(dz, v[c], dw[c]);
      dw[c + 1] = fmaf(dz, v[c + 1], dw[c + 1]);
      const float g0 = v[c] > 0.f ? dz * wv[c] : 0.f;
      const float g1 = v[c + 1] > 0.f ? dz * wv[c + 1] : 0.f;
      o[c / 2] = pack_bf2(g0, g1);
      if constexpr (BNS) {
        const float q0 = lo_bf(o[c / 2]), q1 = hi_bf(o[c / 2]);
        sg[c] += q0;
        sg[c + 1] += q1;
        sgy[c] = fmaf(q0, v[c], sgy[c]);
        sgy[c + 1] = fmaf(q1, v[c + 1], sgy[c + 1]);
      }
    }
    if (gy) {                  // null: statistics pass (the gradient is formed again on load by its consumer)
#pragma unroll
      for (int k = 0; k < C / 8; ++k)
        *reinterpret_cast<uint4*>(gy + i * ldg + 8 * k) = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    }
  }
  float* out = slab + (long)blockIdx.x * (C + 1);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float s = block_sum_256(dw[c], red);
    if (threadIdx.x == 0) out[c] = s;
  }
  const float s = block_sum_256(db, red);
  if (threadIdx.x == 0) out[C] = s;
  if constexpr (BNS) {
    float* bo = bnslab + (long)blockIdx.x * 2 * C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float a0 = block_sum_256(sg[c], red);
      if (threadIdx.x == 0) bo[c] = a0;
      const float a1 = block_sum_256(sgy[c], red);
      if (threadIdx.x == 0) bo[C + c] = a1;
    }
  }
}

// gw: segmap weight grad [C] (+=), gb: bias grad [1] (+=); contiguous in the flat buffer is not assumed.
__global__ void head_grad_finish(const float* __restrict__ tmp, float* __restrict__ gw, float* __restrict__ gb, int C) {
  const int c = threadIdx.x;
  if (c < C) gw[c] += tmp[c];
  if (c == C) gb[0] += tmp[C];
}

// bnslab (or null): [head_grid(P)][2][C] BatchNorm backward partial sums of gy (head_bwd_kernel BNS), C = 32 / 64
// coef (or null, needs bnslab): y is the pre-BN z, y = relu(bn(z)) formed on load as in dpa_head_fwd;
// gy (or null, needs bnslab): null = only the segmap gradients and the BN partial sums (the fused conv
// backward's head + BN mode forms the gradient itself, csrc/bwd_stream.hip)
DPA_API int dpa_head_bwd(const bf16_t* y, int ldy, int C, const float* w, const float* b, const float* t, const float* dS,
                         bf16_t* gy, int ldg, float* slab, float* tmp, float* gw, float* gb, long long P, float* bnslab,
                         const float* coef, hipStream_t st) {
  const int grid = head_grid(P);
  if ((ldy & 7) || (ldg & 7) || (bnslab && C != 32 && C != 64) || (coef && !bnslab) || (!gy && !bnslab))
    return (int)hipErrorInvalidValue;
#define DPA_HB(Cv, BN, ZB) hipLaunchKernelGGL((head_bwd_kernel<Cv, BN, ZB>), dim3(grid), dim3(256), 0, st, y, ldy, w, b, t, dS, gy, ldg, slab, (long)P, bnslab, coef)
  switch (C) {
    case 8: DPA_HB(8, false, false); break;
    case 16: DPA_HB(16, false, false); break;
    case 32: if (coef) DPA_HB(32, true, true); else if (bnslab) DPA_HB(32, true, false); else DPA_HB(32, false, false); break;
    case 64: if (coef) DPA_HB(64, true, true); else if (bnslab) DPA_HB(64, true, false); else DPA_HB(64, false, false); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DPA_HB
  hipLaunchKernelGGL(slab_sum_kernel, dim3(C + 1), dim3(256), 0, st, slab, grid, C + 1, tmp, 0);
  hipLaunchKernelGGL(head_grad_finish, dim3(1), dim3(128), 0, st, tmp, gw, gb, C);
  return (int)hipGetLastError();
}

DPA_API int dpa_head_slab_blocks(long long P) { return head_grid(P); }

// segmap gradients from a [nblk][C+1] slab written elsewhere (the fused conv backward's head mode)
DPA_API int dpa_head_grad_from_slab(const float* slab, int nblk, int C, float* tmp, float* gw, float* gb, hipStream_t st) {
  hipLaunchKernelGGL(slab_sum_kernel, dim3(C + 1), dim3(256), 0, st, slab, nblk, C + 1, tmp, 0);
  hipLaunchKernelGGL(head_grad_finish, dim3(1), dim3(128), 0, st, tmp, gw, gb, C);
  return (int)hipGetLastError();
}

// zero-fill (the flat gradient buffer before a step): a DMA-engine memset, no compute kernel
DPA_API int dpa_zero(void* p, long long nbytes, hipStream_t st) {
  if (nbytes < 0) return (int)hipErrorInvalidValue;
  return (int)hipMemsetAsync(p, 0, (size_t)nbytes, st);
}

// Per-channel sums of a bf16 NHWC tensor (P pixels, C channels at row stride ld), ADDED to out[C]: the bias
// gradient of a transposed conv whose weight gradient runs on the dense GEMM (wgrad_gemm.hip up mode, which
// has no bias column).  Thread t owns the 8-channel chunk t % (C / 8) (C / 8 divides 256), so per-thread sums
// reduce per chunk in thread order in LDS; one slab row per block, then slab_sum_kernel (fixed order).
__global__ __launch_bounds__(256) void chan_sum_bf16_kernel(const bf16_t* __restrict__ g, long P, int C, int ld,
                                                            float* __restrict__ slab) {
  const int CC = C >> 3;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const long tot = P * CC;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const long px = i / CC;
    const int cc = (int)(i - px * CC);
    const uint4 v = *reinterpret_cast<const uint4*>(g + px * ld + cc * 8);
    const unsigned* u = &v.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s[2 * k] += lo_bf(u[k]);
      s[2 * k + 1] += hi_bf(u[k]);
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[threadIdx.x][k] = s[k];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int chunk = c >> 3, k = c & 7;
    float t = 0.f;
    for (int th = chunk; th < 256; th += CC) t += red[th][k];
    slab[(long)blockIdx.x * C + c] = t;
  }
}
DPA_API int dpa_chan_sum_bf16(const bf16_t* g, long long P, int C, int ld, float* slab, int nblk, float* out,
                              hipStream_t st) {
  if ((C & 7) || (ld & 7) || C > 2048 || (256 % (C / 8)) || nblk < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(chan_sum_bf16_kernel, dim3(nblk), dim3(256), 0, st, g, (long)P, C, ld, slab);
  hipLaunchKernelGGL(slab_sum_kernel, dim3(C), dim3(256), 0, st, slab, nblk, C, out, 1);
  return (int)hipGetLastError();
}

DPA_API int dpa_slab_sum(const float* slab, int nblk, int K, float* out, hipStream_t st) {
  hipLaunchKernelGGL(slab_sum_kernel, dim3(K), dim3(256), 0, st, slab, nblk, K, out, 0);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------ loss from partials
// loss = S0/n - dice * log(2 S1 / (S2 + S3 + 1e-15))   (reference utils/utils.py:14-25)
// One thread: the scalar tail of the loss that eager torch spends ~8 launches on (and ~8 more in
// backward).  out = [loss, dL/dS0..3]; the backward scales the stored derivative by the incoming
// gradient.  fp32 throughout, same operation order as the torch formula.
__global__ void loss_finish_kernel(const float* __restrict__ S, float inv_n, int dice, float* __restrict__ out) {
  const float s0 = S[0], s1 = S[1], s2 = S[2], s3 = S[3];
  float loss = s0 * inv_n;
  float d1 = 0.f, d2 = 0.f;
  if (dice) {
    const float u = s2 + s3 + 1e-15f;
    loss = loss - logf(2.f * s1 / u);
    d1 = -1.f / s1;
    d2 = 1.f / u;
  }
  out[0] = loss;
  out[1] = inv_n;
  out[2] = d1;
  out[3] = d2;
  out[4] = d2;
}
__global__ void loss_grad_kernel(const float* __restrict__ g, const float* __restrict__ coef, float scale,
                                 float* __restrict__ dS) {
  const int i = threadIdx.x;
  if (i < 4) dS[i] = g[0] * scale * coef[i];
}
DPA_API int dpa_loss_finish(const float* S, float inv_n, int dice, float* out, hipStream_t st) {
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(1), 0, st, S, inv_n, dice, out);
  return (int)hipGetLastError();
}
DPA_API int dpa_loss_grad(const float* g, const float* coef, float scale, float* dS, hipStream_t st) {
  hipLaunchKernelGGL(loss_grad_kernel, dim3(1), dim3(64), 0, st, g, coef, scale, dS);
  return (int)hipGetLastError();
}

// ---- communication-slot probe (VERDICT r5 #3c): a stand-in for an RCCL all-reduce bucket launched while
// the backward's one-workgroup-per-CU GEMMs hold the CUs.  RCCL's ring kernels run a few workgroups
// (one per channel) that stream the bucket through L2/HBM; this kernel has that geometry -- `blocks`
// workgroups of 256 threads copying `n` float4 -- and each workgroup's lanes stamp the constant 100 MHz
// clock when the workgroup starts and when it ends (stamp[2 * block + {0, 1}], vector stores), so the host
// can separate "waited for a CU" from "ran slowly beside the GEMMs".
__global__ __launch_bounds__(256) void comm_probe_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                         long n, unsigned long long* __restrict__ stamp) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = src[i];
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x < 64 && lane < 2) stamp[2 * blockIdx.x + lane] = lane == 0 ? t0 : t1;
}
DPA_API int dpa_comm_probe(const void* src, void* dst, long long n16, int blocks, unsigned long long* stamp,
                           hipStream_t st) {
  if (blocks < 1 || blocks > 1024 || n16 < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(comm_probe_kernel, dim3(blocks), dim3(256), 0, st, (const float4*)src, (float4*)dst, (long)n16,
                     stamp);
  return (int)hipGetLastError();
}

// A compute stream restricted to all CUs but `reserve` of them (hipExtStreamCreateWithCUMask), spread evenly
// over the CU index range: the backward's one-workgroup-per-CU GEMMs then always leave CUs on which an RCCL
// bucket's kernels start at once (VERDICT r5 #3c; the measured trade-off: BASELINE.md round 6).
DPA_API int dpa_stream_create_cumask(int device, int reserve, void** out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return (int)e;
  const int n = prop.multiProcessorCount;
  if (reserve < 0 || reserve >= n) return (int)hipErrorInvalidValue;
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  const int every = reserve > 0 ? n / reserve : n + 1;
  int kept = 0;
  for (int i = 0; i < n; ++i) {
    const bool res = reserve > 0 && (i % every) == every - 1 && (i / every) < reserve;
    if (!res) {
      mask[i / 32] |= 1u << (i % 32);
      ++kept;
    }
  }
  hipStream_t s;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) return (int)e;
  *out = (void*)s;
  return kept;      // >= 0: the number of CUs the stream may use
}
