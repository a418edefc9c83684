// Implicit-GEMM convolution on MFMA (gfx950), NHWC bf16 activations, fp32 accumulation.
//
// One kernel family covers every "k-contiguous" conv-shaped product of the UNet step
// (SURVEY §2.5 K1, K2, K6 fwd/dgrad; reference model/unet_parts.py:10-12,51-54):
//   * conv3x3 forward          y[p][co]  = relu(b + sum_{tap,ci} x[p+off(tap)][ci] * W[co][tap][ci])
//   * conv3x3 dgrad            dx[p][ci] = (sum_{tap,co} g[p+off(tap)][co] * Wflip[ci][tap][co]) * (x>0)
//   * transposed-conv forward  y[2h+i][2w+j][co] = b + sum_ci x[h][w][ci] * W[ci][co][i][j]  (scatter)
//   * transposed-conv dgrad    dx[h][w][ci] = (sum_{i,j,co} g[2h+i][2w+j][co] * W[ci][co][i][j]) * (x>0)
//
// GEMM view: M = output pixels (gathered rows of the source tensor, zero padding by predication),
// N = output channels (rows of the packed weight matrix), K = taps x source channels.  Both
// operands are K-contiguous in memory, staged global -> registers -> LDS (double buffered, one
// barrier per K-step; the next tile's loads are issued before this tile's MFMAs) with an XOR
// swizzle that makes every ds_read_b128 fragment read conflict-free (see tools/lds_banks.py).
// MFMA: v_mfma_f32_16x16x32_bf16 with A = weights (rows = out channels) and B = pixels, so each
// lane ends with 4 consecutive channels of one pixel -> 8-byte bf16 stores.  Epilogue fuses bias,
// ReLU, the ReLU-backward mask of the *next* tensor, accumulation and the transposed-conv scatter.
// Block -> tile mapping is XCD-aware (channel tiles of one pixel tile share an XCD's L2).
#include "common.h"

#include "conv_args.h"

template <int BP, int BC, int BK, int WP, int WC>
__global__ __launch_bounds__(64 * (BP / WP) * (BC / WC)) void igemm_kernel(IgemmArgs a) {
  constexpr int NT = 64 * (BP / WP) * (BC / WC);   // 4 or 8 waves
  constexpr int CPR = BK / 8;               // 16-byte chunks per LDS row
  constexpr int RPP = NT / CPR;             // rows covered by one pass of the block
  constexpr int LP = (BP + RPP - 1) / RPP;  // pixel-row loads per thread
  constexpr int LW = (BC + RPP - 1) / RPP;  // weight-row loads per thread
  constexpr int NWC = BC / WC;
  constexpr int NWP = BP / WP;
  static_assert(NWC * NWP == 4 || NWC * NWP == 8, "4 or 8 waves per block");
  static_assert(BP % RPP == 0 && (BC % RPP == 0 || (BC * CPR) % 64 == 0), "loader tiling");
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int RB = BK * 2;                // LDS row bytes
  __shared__ __attribute__((aligned(16))) char lds[2][(BP + BC) * RB];

  const int M = a.N * a.Ho * a.Wo;
  const int nct = a.Ngemm / BC;
  const int npt = (M + BP - 1) / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  const int pt = bid / nct, ct = bid - pt * nct;
  const int m0 = pt * BP, c0 = ct * BC;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid / NWC, wc = wid - wp * NWC;
  const int lchunk = tid % CPR;
  const int lrow = tid / CPR;

  // Per-thread loader state, computed ONCE: each pixel row's byte offset at tap (0,0) and a bit mask
  // of the taps that land inside the image (zero padding).  When a K-step never straddles a tap
  // (Cs % BK == 0, every layer except tiny ones) the tap is wave-uniform, so a K-step costs one
  // scalar division and ~4 VALU per row (the old per-lane divisions and bounds math made the loader
  // VALU-bound beside the MFMAs).
  unsigned pbase[LP];
  unsigned tmask[LP];
  const int taps = a.KH * a.KW;
#pragma unroll
  for (int i = 0; i < LP; ++i) {
    const int r = lrow + i * RPP;
    const int m = m0 + r;
    const bool pok = (r < BP) && (m < M);
    const int mm = pok ? m : 0;
    const int hw = a.Ho * a.Wo;
    const int pn = mm / hw;
    const int rem = mm - pn * hw;
    const int ph = rem / a.Wo, pw = rem - (rem / a.Wo) * a.Wo;
    const int h0 = ph * a.stride - a.pad, w0 = pw * a.stride - a.pad;
    unsigned msk = 0;
    for (int t = 0; t < taps; ++t) {
      const int kh = t / a.KW, kw = t - (t / a.KW) * a.KW;
      const int ih = h0 + kh, iw = w0 + kw;
      if (pok && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) msk |= 1u << t;
    }
    tmask[i] = msk;
    // offset of (h0, w0) may be "negative" (padding): unsigned wrap-around is undone by the tap delta
    pbase[i] = (unsigned)((((pn * a.Hs + h0) * a.Ws + w0) * a.ldx) * 2);
  }
  const int S = a.Kpad / BK;
  const bool uniform_tap = (a.Cs % BK) == 0;
  u32x4_t pr[LP], wr[LW];

  // Zero padding by the buffer unit's range check: an out-of-image tap gets an offset beyond
  // num_records and reads 0 -- no branch, no select, every load issued back to back (a branch
  // around each load makes hipcc wait vmcnt(0) per load: guide §5 ".s traps" (c)).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  unsigned woff[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) woff[i] = (unsigned)(((c0 + lrow + i * RPP) * a.Kpad + lchunk * 8) * 2);
  auto gload = [&](int s) {
    int tap, ci;
    if (uniform_tap) {
      tap = (s * BK) / a.Cs;                           // wave-uniform (scalar)
      ci = s * BK - tap * a.Cs + lchunk * 8;
    } else {
      const int k0 = (s * CPR + lchunk) * 8;
      tap = k0 / a.Cs;
      ci = k0 - tap * a.Cs;
    }
    const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
    const unsigned delta = (unsigned)(((kh * a.Ws + kw) * a.ldx + ci) * 2);
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      const bool ok = tap < taps && ((tmask[i] >> tap) & 1u);
      pr[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? pbase[i] + delta : 0x80000000u, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      if (BC % RPP == 0 || tid < BC * CPR)
        wr[i] = __builtin_amdgcn_raw_buffer_load_b128(wrs, woff[i] + s * BK * 2, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
    char* P = lds[buf];
    char* Wt = lds[buf] + BP * RB;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      const int r = lrow + i * RPP;
      *reinterpret_cast<u32x4_t*>(P + r * RB + swz_nk<BK>(r, lchunk) * 16) = pr[i];
    }
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int r = lrow + i * RPP;
      if (BC % RPP == 0 || tid < BC * CPR) *reinterpret_cast<u32x4_t*>(Wt + r * RB + swz_nk<BK>(r, lchunk) * 16) = wr[i];
    }
  };

  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int buf = s & 1;
    if (s + 1 < S) gload(s + 1);
    // keep the prefetch issue above and the LDS stores below the MFMAs: without the fences hipcc
    // hoists the next tile's ds_writes (and so their vmcnt waits) in front of this tile's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    const char* P = lds[buf];
    const char* Wt = lds[buf] + BP * RB;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8_t af[TC], bfr[TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        const int row = wc * WC + ic * 16 + (lane & 15);
        af[ic] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RB + swz_nk<BK>(row, chunk) * 16);
      }
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const int row = wp * WP + ip * 16 + (lane & 15);
        bfr[ip] = *reinterpret_cast<const bf16x8_t*>(P + row * RB + swz_nk<BK>(row, chunk) * 16);
      }
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip)
          acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < S) lstore(buf ^ 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // 32-bit buffer addressing (extents < 2 GiB per launch): no 64-bit pointer math per element.
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.mask ? a.mask : a.y), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int m = m0 + wp * WP + ip * 16 + (lane & 15);
    if (m >= M) continue;
    unsigned ybase;
    if (a.mode == 0) {
      ybase = (unsigned)m * (unsigned)a.ldy;
    } else {
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, rem = m - n * hw, h = rem / a.Wo, w = rem - (rem / a.Wo) * a.Wo;
      ybase = (unsigned)(((n * 2 * a.Ho + 2 * h) * (2 * a.Wo) + 2 * w) * a.ldy);
    }
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int nidx = c0 + wc * WC + ic * 16 + 4 * (lane >> 4);
      int co = nidx;
      unsigned off = ybase + nidx;
      if (a.mode == 1) {
        const int ij = nidx / a.Cout;
        co = nidx - ij * a.Cout;
        off = ybase + (unsigned)(((ij >> 1) * (2 * a.Wo) + (ij & 1)) * a.ldy + co);
      }
      float v0 = acc[ic][ip][0], v1 = acc[ic][ip][1], v2 = acc[ic][ip][2], v3 = acc[ic][ip][3];
      if (a.bias) {
        const float* b = a.bias + co;   // views into the flat fp32 buffer: only 4-byte aligned
        v0 += b[0]; v1 += b[1]; v2 += b[2]; v3 += b[3];
      }
      if (a.relu) {
        v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3);
      }
      if (a.mask && co < a.mask_ch) {
        const u32x2_t mk = __builtin_amdgcn_raw_buffer_load_b64(mr, ((unsigned)m * (unsigned)a.ldm + co) * 2, 0, 0);
        v0 = lo_bf(mk.x) > 0.f ? v0 : 0.f;
        v1 = hi_bf(mk.x) > 0.f ? v1 : 0.f;
        v2 = lo_bf(mk.y) > 0.f ? v2 : 0.f;
        v3 = hi_bf(mk.y) > 0.f ? v3 : 0.f;
      }
      if (a.accumulate) {
        const u32x2_t o = __builtin_amdgcn_raw_buffer_load_b64(yr, off * 2, 0, 0);
        v0 += lo_bf(o.x); v1 += hi_bf(o.x); v2 += lo_bf(o.y); v3 += hi_bf(o.y);
      }
      const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
      if (!split_store(a, (unsigned)m, co, packed)) __builtin_amdgcn_raw_buffer_store_b64(packed, yr, off * 2, 0, 0);
    }
  }
}

template <int BP, int BC, int BK, int WP, int WC>
static int launch_igemm(const IgemmArgs& a, hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  const int grid = ((M + BP - 1) / BP) * (a.Ngemm / BC);
  hipLaunchKernelGGL((igemm_kernel<BP, BC, BK, WP, WC>), dim3(grid), dim3(64 * (BP / WP) * (BC / WC)), 0, st, a);
  return (int)hipGetLastError();
}

// cfg: 0 = auto.  Tile families (BP x BC x BK): 1: 128x128x32  2: 128x128x64  3: 128x64x32
//      4: 128x64x64  5: 256x32x32  6: 256x32x64  7: 64x128x64 (small-M deep layers)
//      8: 256x128x64 (8 waves)  9: 128x256x64 (8 waves)
DPA_API int dpa_igemm(const IgemmArgs* args, int cfg, hipStream_t st) {
  IgemmArgs a = *args;
  if ((a.Cs & 7) || (a.ldx & 7) || (a.ldy & 3) || (a.Kpad & 31) || (a.Ngemm & 31) || a.x2 || a.xbn) return (int)hipErrorInvalidValue;
  if (a.mode == 1 && (a.Cout & 3)) return (int)hipErrorInvalidValue;
  if (cfg == 0) {
    const long M = (long)a.N * a.Ho * a.Wo;
    const bool k64 = (a.Kpad % 64) == 0;
    if (a.Ngemm % 128 == 0) cfg = (M <= 16384 && a.Ngemm >= 256) ? (k64 ? 7 : 1) : (k64 ? 2 : 1);
    else if (a.Ngemm % 64 == 0) cfg = k64 ? 4 : 3;
    else cfg = k64 ? 6 : 5;
  }
  switch (cfg) {
    case 1: if (a.Ngemm % 128) break; return launch_igemm<128, 128, 32, 64, 64>(a, st);
    case 2: if (a.Ngemm % 128 || a.Kpad % 64) break; return launch_igemm<128, 128, 64, 64, 64>(a, st);
    case 3: if (a.Ngemm % 64) break; return launch_igemm<128, 64, 32, 64, 32>(a, st);
    case 4: if (a.Ngemm % 64 || a.Kpad % 64) break; return launch_igemm<128, 64, 64, 64, 32>(a, st);
    case 5: return launch_igemm<256, 32, 32, 64, 32>(a, st);
    case 6: if (a.Kpad % 64) break; return launch_igemm<256, 32, 64, 64, 32>(a, st);
    case 7: if (a.Ngemm % 128 || a.Kpad % 64) break; return launch_igemm<64, 128, 64, 32, 64>(a, st);
    case 8: if (a.Ngemm % 128 || a.Kpad % 64) break; return launch_igemm<256, 128, 64, 64, 64>(a, st);   // 8 waves
    case 9: if (a.Ngemm % 256 || a.Kpad % 64) break; return launch_igemm<128, 256, 64, 64, 64>(a, st);   // 8 waves
    default: break;
  }
  return (int)hipErrorInvalidValue;
}
