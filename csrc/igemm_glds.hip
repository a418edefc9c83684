// Implicit-GEMM convolution with LDS-DMA staging (gfx950), for the deep UNet layers
// (64x64 / 32x32 grids, 256-1024 channels: enc.conv4, mid, dec.conv1 and the transposed convs;
// SURVEY §2.5 K1/K2/K6, reference model/unet_parts.py:10-12,51-54).
//
// Why a second GEMM core: the register-staged kernel in igemm.hip spends more LDS cycles than
// MFMA cycles per K-step -- ds_write_b128 moves only ~79 B/clk/CU (MI355X_MICROARCH §LDS) and a
// 128x128x64 step writes 32 KB and reads 64 KB -- so it stalls near 800 TF.  Here both operands go
// HBM/L2 -> LDS by `buffer_load_dwordx4 ... lds` (no VGPR round trip, no ds_write), three stages
// deep, with counted `s_waitcnt vmcnt(N)` + raw `s_barrier` so two K-steps of loads stay in flight
// across each barrier (cdna_hip_programming.md "Pipelining across barriers").
//
// Tile: BC (output channels = rows of the packed weights) x BP (pixels) x 64 (K), 8 waves.
// LDS images are [rows][64] bf16 (128-B rows) with the 16-B chunk XOR swizzle swz_nk<64>; the DMA
// writes lane-linearly, so the swizzle is applied on the SOURCE address (lane l of a wave fetches
// chunk (l&7) ^ (row&7) of its row and lands in slot l&7).  Zero padding / M tail: the buffer
// unit's range check (offset 0x80000000 -> zeros written to LDS), no branches in the loader.
// Epilogue = igemm.hip's (bias, ReLU, ReLU-backward mask, accumulate, transposed-conv scatter).
#include "common.h"

#include "conv_args.h"

#include <type_traits>


// Logical tile id -> (pixel tile, channel tile).  Consecutive ids run on one XCD (xcd_remap), so
// ~32 consecutive ids share an L2: with many channel tiles, group them as 8 pixel tiles x (ids / 8)
// channel tiles instead of one pixel tile x 32 channel tiles (the whole weight panel per K-step):
// 12 distinct operand tiles per K-step instead of 33.  With 1-2 channel tiles (the UNet) the order is
// the plain row-major one.
__device__ __forceinline__ void glds_tile(int L, int npt, int nct, int& pt, int& ct) {
  if (nct < 4) {
    pt = L / nct;
    ct = L - pt * nct;
    return;
  }
  constexpr int GM = 8;
  const int g = L / (GM * nct), r = L - g * GM * nct;
  const int gm = min(GM, npt - g * GM);
  pt = g * GM + r % gm;
  ct = r / gm;
}

// K-tile s -> (tap, first channel).  Slice-major order (all taps of one 64-channel slice, then the next
// slice) when the packed K has no padding: consecutive K-tiles then gather the SAME channel slice at
// 9 neighbouring pixel offsets, so the pixel lines a K-tile fetches were mostly fetched by the previous
// one and are still in the XCD's L2 (tap-major order re-reads a line only Cs/64 K-tiles later, after
// ~8 MB of other traffic went through the 4 MB L2).  The weight block of (tap, ci) is the 128-B
// column block tap*Cs + ci of the packed [Ngemm][Kpad] matrix in either order.
__device__ __forceinline__ void ktile_coords(const IgemmArgs& a, int s, int BK, int taps, bool slm, int& tap, int& ci) {
  if (slm) {
    const int sl = s / taps;
    tap = s - sl * taps;
    ci = sl * BK;
  } else {
    tap = (s * BK) / a.Cs;                           // Cs % BK == 0: one tap per K-step (scalar)
    ci = s * BK - tap * a.Cs;
  }
}

// epilogue (as igemm.hip): bias, ReLU, ReLU-backward mask, accumulate, transposed-conv scatter.
// Output base of GEMM row (pixel) m: NHWC row, or the (2h, 2w) corner of its 2x2 block (mode 1).
__device__ __forceinline__ unsigned glds_ybase(const IgemmArgs& a, int m) {
  if (a.mode == 0) return (unsigned)m * (unsigned)a.ldy;
  const int hw = a.Ho * a.Wo;
  const int n = m / hw, rem = m - n * hw, h = rem / a.Wo, w = rem - (rem / a.Wo) * a.Wo;
  return (unsigned)(((n * 2 * a.Ho + 2 * h) * (2 * a.Wo) + 2 * w) * a.ldy);
}

// four consecutive GEMM columns nidx..nidx+3 of pixel m
__device__ __forceinline__ void glds_store4(const IgemmArgs& a, __amdgpu_buffer_rsrc_t yr, __amdgpu_buffer_rsrc_t mr,
                                            int m, unsigned ybase, int nidx, float v0, float v1, float v2, float v3) {
  int co = nidx;
  unsigned off = ybase + nidx;
  if (a.mode == 1) {
    const int ij = nidx / a.Cout;
    co = nidx - ij * a.Cout;
    off = ybase + (unsigned)(((ij >> 1) * (2 * a.Wo) + (ij & 1)) * a.ldy + co);
  }
  if (a.bias) {
    const float* b = a.bias + co;
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

// 16x16 accumulator tiles: pixel = lane & 15, channels 4*(lane >> 4) + 0..3
template <int TC, int TP, int WC, int WP>
__device__ __forceinline__ void glds_epilogue(const IgemmArgs& a, f32x4_t (&acc)[TC][TP], int M, int m0, int c0,
                                              int wc, int wp, int lane) {
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.mask ? a.mask : a.y), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int m = m0 + wp * WP + ip * 16 + (lane & 15);
    if (m >= M) continue;
    const unsigned ybase = glds_ybase(a, m);
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
      glds_store4(a, yr, mr, m, ybase, c0 + wc * WC + ic * 16 + 4 * (lane >> 4), acc[ic][ip][0], acc[ic][ip][1],
                  acc[ic][ip][2], acc[ic][ip][3]);
  }
}

// Specialised epilogues (EP 1: plain conv forward -- optional bias, optional ReLU; EP 2: dgrad with the
// ReLU-backward mask only; EP 3: dgrad split into the two dense halves of a concat gradient): straight-line code with the row offsets computed once per pixel fragment.
// The generic epilogue carries every mode (scatter, split, accumulate, mask) behind runtime branches:
// ~5000 instructions that cost 10-20 % of a deep layer's time (profiles/experiments_r03_late.txt).
// Out-of-range pixels store to an offset past the buffer's range check (dropped) instead of branching.
// PM: the EP 2 mask fragments were loaded by the caller up front (pmk[ip * TC + ic]), so their latency
// overlaps the K loop instead of opening the epilogue.
// PB: likewise the EP 1 bias values (pbias[ic * 4 + e]).
template <int TC, int TP, int WC, int WP, int EP, bool PM = false, bool PB = false>
__device__ __forceinline__ void glds_epilogue_fast(const IgemmArgs& a, f32x4_t (&acc)[TC][TP], int M, int m0, int c0,
                                                   int wc, int wp, int lane, const u32x2_t* pmk = nullptr,
                                                   const float* pbias = nullptr) {
  static_assert(EP == 1 || EP == 2 || EP == 3, "fast epilogue kinds");
  static_assert(!PM || EP == 2, "preloaded masks: EP 2");
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)(EP == 2 ? a.mask : a.y), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t y2r = __builtin_amdgcn_make_buffer_rsrc((void*)(EP == 3 ? a.y2 : a.y), 0, 0x7fffffff, 0x00020000);
  const int cb = c0 + wc * WC + 4 * (lane >> 4);
  float bias[TC][4];
  const bool relu = a.relu != 0;
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[ic][e] = 0.f;
  if constexpr (PB) {
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) bias[ic][e] = pbias[ic * 4 + e];
  } else if (EP == 1 && a.bias) {
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) bias[ic][e] = a.bias[cb + ic * 16 + e];   // (flat parameter views: 4-B aligned)
  }
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int m = m0 + wp * WP + ip * 16 + (lane & 15);
    const bool ok = m < M;
    const unsigned yo = ok ? (unsigned)m * (unsigned)a.ldy * 2u + (unsigned)cb * 2u : 0x80000000u;
    const unsigned yo2 = EP == 3 ? (unsigned)m * (unsigned)a.ldy2 * 2u : 0u;
    u32x2_t mk[TC];
    if constexpr (PM) {
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) mk[ic] = pmk[ip * TC + ic];
    } else if constexpr (EP == 2) {
      const unsigned mo = ok ? (unsigned)m * (unsigned)a.ldm * 2u + (unsigned)cb * 2u : 0x80000000u;
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) mk[ic] = __builtin_amdgcn_raw_buffer_load_b64(mr, mo + ic * 32, 0, 0);
    }
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      float v0 = acc[ic][ip][0] + bias[ic][0], v1 = acc[ic][ip][1] + bias[ic][1];
      float v2 = acc[ic][ip][2] + bias[ic][2], v3 = acc[ic][ip][3] + bias[ic][3];
      if (EP == 1 && relu) {
        v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3);
      }
      if constexpr (EP == 2) {
        if (cb + ic * 16 < a.mask_ch) {
          v0 = lo_bf(mk[ic].x) > 0.f ? v0 : 0.f;
          v1 = hi_bf(mk[ic].x) > 0.f ? v1 : 0.f;
          v2 = lo_bf(mk[ic].y) > 0.f ? v2 : 0.f;
          v3 = hi_bf(mk[ic].y) > 0.f ? v3 : 0.f;
        }
      }
      const u32x2_t pk = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
      if constexpr (EP == 3) {
        // split output: a 16-channel group lies wholly below or above `split` (split % 16 == 0), so the
        // target tensor is wave-uniform per group
        if (c0 + wc * WC + ic * 16 < a.split)
          __builtin_amdgcn_raw_buffer_store_b64(pk, yr, yo + ic * 32, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b64(pk, y2r, ok ? yo2 + (unsigned)(cb + ic * 16 - a.split) * 2u : 0x80000000u, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(pk, yr, yo + ic * 32, 0, 0);
      }
    }
  }
}

// sum over the 16 lanes of a DPP row (every lane gets it; lane order of the adds is fixed per lane):
// row rotations by 8, 4, 2, 1 on the VALU (ds_bpermute / __shfl_xor goes through the LDS unit and
// serialises: 128 of them cost ~4 us per workgroup in this epilogue)
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xf, 0xf, false));
  return v;
}

// EP 1 / 2 plus the BatchNorm partial sums of the STORED bf16 values for the producing conv's BN (row-block
// kernels, 4 pixel waves x 2 channel waves): forward (EP 1: bias, no ReLU): sum y, sum y^2; backward (EP 2,
// mask = the BN output): sum g, sum g * mask.  One slab row per 256-pixel tile, bnslab[m0 / 256][2][Ngemm],
// reduced in a fixed order (16-lane DPP row sum, then the 4 pixel waves in order).
// Channel fragments outermost so only one fragment's sums are live (acc already holds 128 VGPRs).
// bred: 4 x 2BC floats of the kernel's own LDS that no wave reads any more (a separate __shared__
// array makes hipcc wait vmcnt(0) before every fragment read of the K loop: it cannot tell the second
// LDS object from the LDS-DMA destination -- +15 % on the 128-channel layers).
template <int TC, int TP, int WC, int WP, int EP>
__device__ __forceinline__ void glds_epilogue_bns(const IgemmArgs& a, f32x4_t (&acc)[TC][TP], int M, int m0, int c0,
                                                  int wc, int wp, int lane, float* bred_) {
  static_assert(EP == 1 || EP == 2, "BN partial sums: EP 1 / 2");
  constexpr int BC = 2 * WC;
  float (*bred)[2 * BC] = reinterpret_cast<float (*)[2 * BC]>(bred_);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)(EP == 2 ? a.mask : a.y), 0, 0x7fffffff, 0x00020000);
  const int cb = c0 + wc * WC + 4 * (lane >> 4);
  unsigned yo[TP], mo[TP];
  float okf[TP];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int m = m0 + wp * WP + ip * 16 + (lane & 15);
    const bool ok = m < M;
    okf[ip] = ok ? 1.f : 0.f;
    yo[ip] = ok ? (unsigned)m * (unsigned)a.ldy * 2u + (unsigned)cb * 2u : 0x80000000u;
    mo[ip] = EP == 2 && ok ? (unsigned)m * (unsigned)a.ldm * 2u + (unsigned)cb * 2u : 0x80000000u;
  }
#pragma unroll
  for (int ic = 0; ic < TC; ++ic) {
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (EP == 1 && a.bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bias[e] = a.bias[cb + ic * 16 + e];
    }
    u32x2_t mk[TP];
    if constexpr (EP == 2) {
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) mk[ip] = __builtin_amdgcn_raw_buffer_load_b64(mr, mo[ip] + ic * 32, 0, 0);
    }
    float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[ic][ip][e] + bias[e];
      float f[4];
      if constexpr (EP == 2) {
        f[0] = lo_bf(mk[ip].x); f[1] = hi_bf(mk[ip].x); f[2] = lo_bf(mk[ip].y); f[3] = hi_bf(mk[ip].y);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f[e] > 0.f ? v[e] : 0.f;      // host: mask_ch == Ngemm
      }
      const u32x2_t pk = u32x2_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
      __builtin_amdgcn_raw_buffer_store_b64(pk, yr, yo[ip] + ic * 32, 0, 0);
      const float st[4] = {okf[ip] * lo_bf(pk.x), okf[ip] * hi_bf(pk.x), okf[ip] * lo_bf(pk.y), okf[ip] * hi_bf(pk.y)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] += st[e];
        q[e] = fmaf(st[e], EP == 2 ? f[e] : st[e], q[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[e] = row16_sum(s[e]);
      q[e] = row16_sum(q[e]);
      if ((lane & 15) == 0) {
        const int c = wc * WC + ic * 16 + 4 * (lane >> 4) + e;
        bred[wp][c] = s[e];
        bred[wp][BC + c] = q[e];
      }
    }
  }
  // LDS-only barrier: __syncthreads' release fence would first wait for every output store of the
  // block to be acknowledged (vmcnt(0)), several us per block with one 132-KB block per CU
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  float* row = a.bnslab + (long)(m0 / 256) * 2 * a.Ngemm;
  for (int k = threadIdx.x; k < 2 * BC; k += blockDim.x) {
    const float t = (bred[0][k] + bred[1][k]) + (bred[2][k] + bred[3][k]);
    row[k < BC ? c0 + k : a.Ngemm + c0 + (k - BC)] = t;
  }
}

// epilogue kind for a launch: 1 / 2 when the specialised code covers it, else 0 (generic)
static inline int glds_ep_kind(const IgemmArgs& a) {
  if (a.mode != 0 || a.accumulate || (a.ldy & 3)) return 0;
  if (a.y2 != nullptr)     // split dgrad (the two halves of a concat gradient)
    return (a.mask == nullptr && a.bias == nullptr && !a.relu && (a.split % 16) == 0 && (a.ldy2 & 3) == 0) ? 3 : 0;
  if (a.mask == nullptr) return (a.Ngemm % 16) == 0 ? 1 : 0;
  if (a.bias == nullptr && !a.relu && (a.ldm & 3) == 0) return 2;
  return 0;
}

template <int BC, int BP, int WC, int WP, int ST, int BK, bool PRE = false>
__global__ __launch_bounds__(512) void igemm_glds_kernel(IgemmArgs a) {
  constexpr int NWC = BC / WC, NWP = BP / WP;
  static_assert(NWC * NWP == 8, "8 waves");
  constexpr int RBY = BK * 2;                 // bytes per LDS row
  constexpr int CPR = RBY / 16;               // 16-B chunks per row
  constexpr int RPI = 64 / CPR;               // rows one wave-instruction (1 KB) fills
  constexpr int RA = BC / (8 * RPI), RP = BP / (8 * RPI);   // DMA rounds per stage per wave
  static_assert(RA * 8 * RPI == BC && RP * 8 * RPI == BP, "loader tiling");
  constexpr int LPS = RA + RP;                // DMA instructions per stage per wave
  constexpr int TC = WC / 16, TP = WP / 16;
  constexpr int STAGE = (BC + BP) * RBY;
  __shared__ __attribute__((aligned(16))) char lds[ST * STAGE];

  const int M = a.N * a.Ho * a.Wo;
  const int nct = a.Ngemm / BC;
  const int npt = (M + BP - 1) / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  int pt, ct;
  glds_tile(bid, npt, nct, pt, ct);
  const int m0 = pt * BP, c0 = ct * BC;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % NWC, wp = wid / NWC;

  // loader geometry: in round j this wave fills rows j*8*RPI + wid*RPI + lane/CPR, slot lane%CPR; the
  // swizzle depends on row bits the round offset does not touch, and XOR is its own inverse
  const int lrow = wid * RPI + lane / CPR;
  const int lchunk = swz_nk<BK>(lrow, lane % CPR);

  unsigned pbase[RP], tmask[RP];
  const int taps = a.KH * a.KW;
#pragma unroll
  for (int j = 0; j < RP; ++j) {
    const int m = m0 + j * 8 * RPI + lrow;
    const bool pok = m < M;
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
    tmask[j] = msk;
    pbase[j] = (unsigned)((((pn * a.Hs + h0) * a.Ws + w0) * a.ldx) * 2 + lchunk * 16);
  }
  unsigned woff[RA];
#pragma unroll
  for (int j = 0; j < RA; ++j) woff[j] = (unsigned)(((c0 + j * 8 * RPI + lrow) * a.Kpad) * 2 + lchunk * 16);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  const int S = a.Kpad / BK;

  const bool slm = !(a.korder & 1) && a.Kpad == taps * a.Cs;
  auto issue = [&](int s) {
    char* base = lds + (s % ST) * STAGE;
    int tap, ci;
    ktile_coords(a, s, BK, taps, slm, tap, ci);
    const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
    const unsigned delta = (unsigned)(((kh * a.Ws + kw) * a.ldx + ci) * 2);
    const unsigned wk = (unsigned)((tap * a.Cs + ci) * 2);
#pragma unroll
    for (int j = 0; j < RA; ++j)
      dma16(wrs, base + (j * 8 * RPI + wid * RPI) * RBY, woff[j] + wk);
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const bool ok = tap < taps && ((tmask[j] >> tap) & 1u);
      dma16(xr, base + (BC + j * 8 * RPI + wid * RPI) * RBY, ok ? pbase[j] + delta : 0x80000000u);
    }
  };

  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < ST - 1; ++s)
    if (s < S) issue(s);

  for (int s = 0; s < S; ++s) {
    // own DMAs of step s done (the ST-2 newer steps may stay in flight), then everyone's
    if (s + ST - 2 < S) wait_vm<(ST - 2) * LPS>();
    else wait_vm<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + ST - 1 < S) issue(s + ST - 1);           // refills the buffer consumed at step s-1
    __builtin_amdgcn_sched_barrier(0);
    const char* Wt = lds + (s % ST) * STAGE;
    const char* P = Wt + BC * RBY;
    if constexpr (PRE) {
      // every fragment of the K-step into registers first (96 VGPRs), then the MFMAs back to back:
      // the compiler's default interleave issues two reads per eight MFMAs and waits lgkmcnt(0) on them
      bf16x8_t af[BK / 32][TC], bfr[BK / 32][TP];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) {
          const int row = wp * WP + ip * 16 + (lane & 15);
          bfr[kk][ip] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          const int row = wc * WC + ic * 16 + (lane & 15);
          af[kk][ic] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int ic = 0; ic < TC; ++ic)
#pragma unroll
          for (int ip = 0; ip < TP; ++ip)
            acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][ic], bfr[kk][ip], acc[ic][ip], 0, 0, 0);
    } else {
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8_t af[TC], bfr[TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        const int row = wc * WC + ic * 16 + (lane & 15);
        af[ic] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + (swz_nk<BK>(row, chunk) << 4));
      }
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const int row = wp * WP + ip * 16 + (lane & 15);
        bfr[ip] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + (swz_nk<BK>(row, chunk) << 4));
      }
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip)
          acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
    }
    }
  }

  glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
}

// ------------------------------------------------------------------------------------------------
// Persistent variant (cfg 8-10): one workgroup per CU walks a list of output tiles and keeps the
// LDS-DMA pipeline running ACROSS tile boundaries -- the first K-steps of tile j+1 are issued during
// the last K-steps of tile j and land while tile j's epilogue stores its outputs -- instead of one
// workgroup per tile, where every tile pays the first loads' HBM latency and its epilogue on an
// otherwise idle CU (one 128-144 KB workgroup fits a CU, so nothing else overlaps them).  That
// ramp is ~5-15 % of a tile at K = 2304-4608 and far more at the short K of the transposed convs
// and the K = 1152 layers.  Tiles are dealt in XCD-contiguous chunks (workgroup b runs on XCD b & 7,
// its slot b >> 3 takes every (grid/8)-th tile of that XCD's chunk), so the ~32 tiles an XCD works on
// at a time are neighbours sharing halo rows and weights in its L2.
template <int BC, int BP, int WC, int WP, int ST, int BK>
__global__ __launch_bounds__(512) void igemm_glds_pers_kernel(IgemmArgs a) {
  constexpr int NWC = BC / WC, NWP = BP / WP;
  static_assert(NWC * NWP == 8, "8 waves");
  constexpr int RBY = BK * 2, CPR = RBY / 16, RPI = 64 / CPR;
  constexpr int RA = BC / (8 * RPI), RP = BP / (8 * RPI);
  static_assert(RA * 8 * RPI == BC && RP * 8 * RPI == BP, "loader tiling");
  constexpr int LPS = RA + RP;
  constexpr int TC = WC / 16, TP = WP / 16;
  constexpr int STAGE = (BC + BP) * RBY;
  __shared__ __attribute__((aligned(16))) char lds[ST * STAGE];

  const int M = a.N * a.Ho * a.Wo;
  const int nct = a.Ngemm / BC;
  const int T = ((M + BP - 1) / BP) * nct;
  const int G8 = gridDim.x >> 3, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int q = T >> 3, r = T & 7;
  const int cstart = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int clen = q + (xcd < r ? 1 : 0);
  const int J = slot < clen ? (clen - slot + G8 - 1) / G8 : 0;
  if (J == 0) return;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % NWC, wp = wid / NWC;
  const int lrow = wid * RPI + lane / CPR;
  const int lchunk = swz_nk<BK>(lrow, lane % CPR);
  const int taps = a.KH * a.KW;
  const int hw = a.Ho * a.Wo;

  // loader geometry of tile j of this workgroup's list
  auto geo = [&](int j, unsigned (&pb)[RP], unsigned (&tm)[RP], unsigned (&wo)[RA], int& m0, int& c0) {
    const int t = cstart + slot + j * G8;
    int pt, ct;
    glds_tile(t, (M + BP - 1) / BP, nct, pt, ct);
    m0 = pt * BP;
    c0 = ct * BC;
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int m = m0 + i * 8 * RPI + lrow;
      const bool pok = m < M;
      const int mm = pok ? m : 0;
      const int pn = mm / hw;
      const int rem = mm - pn * hw;
      const int ph = rem / a.Wo, pw = rem - ph * a.Wo;
      const int h0 = ph * a.stride - a.pad, w0 = pw * a.stride - a.pad;
      unsigned msk = 0;
      for (int k = 0; k < taps; ++k) {
        const int kh = k / a.KW, kw = k - kh * a.KW;
        const int ih = h0 + kh, iw = w0 + kw;
        if (pok && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) msk |= 1u << k;
      }
      tm[i] = msk;
      pb[i] = (unsigned)((((pn * a.Hs + h0) * a.Ws + w0) * a.ldx) * 2 + lchunk * 16);
    }
#pragma unroll
    for (int i = 0; i < RA; ++i) wo[i] = (unsigned)(((c0 + i * 8 * RPI + lrow) * a.Kpad) * 2 + lchunk * 16);
  };

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  const int S = a.Kpad / BK;
  const int GT = J * S;
  const bool slm = !(a.korder & 1) && a.Kpad == taps * a.Cs;

  // one geometry set: the next tile's overwrites the current one at K-step S-ST+1, after the current
  // tile's last DMA was issued (the epilogue keeps only the tile origin)
  unsigned pb[RP], tm[RP], wo[RA];
  int m0, c0, m0g, c0g;
  geo(0, pb, tm, wo, m0g, c0g);

  // K-step sk of the tile whose geometry is loaded into stage buffer b
  auto issue = [&](int b, int sk) {
    char* base = lds + b * STAGE;
    int tap, ci;
    ktile_coords(a, sk, BK, taps, slm, tap, ci);
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const unsigned delta = (unsigned)(((kh * a.Ws + kw) * a.ldx + ci) * 2);
    const unsigned wk = (unsigned)((tap * a.Cs + ci) * 2);
#pragma unroll
    for (int i = 0; i < RA; ++i) dma16(wrs, base + (i * 8 * RPI + wid * RPI) * RBY, wo[i] + wk);
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const bool ok = tap < taps && ((tm[i] >> tap) & 1u);
      dma16(xr, base + (BC + i * 8 * RPI + wid * RPI) * RBY, ok ? pb[i] + delta : 0x80000000u);
    }
  };

  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < ST - 1; ++s) issue(s, s);      // host guarantees S >= ST - 1

  int g = 0;
  for (int j = 0; j < J; ++j) {
    m0 = m0g;
    c0 = c0g;
    for (int s = 0; s < S; ++s, ++g) {
      // after an epilogue (its loads/stores share the counter) drain; else keep ST-2 steps in flight
      if ((s == 0 && j > 0) || g + ST - 2 >= GT) wait_vm<0>();
      else wait_vm<(ST - 2) * LPS>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (g + ST - 1 < GT) {
        const int sk = s + ST - 1;
        if (sk == S) geo(j + 1, pb, tm, wo, m0g, c0g);
        issue((g + ST - 1) % ST, sk >= S ? sk - S : sk);
      }
      __builtin_amdgcn_sched_barrier(0);
      const char* Wt = lds + (g % ST) * STAGE;
      const char* P = Wt + BC * RBY;
      // all fragments first (see igemm_glds_kernel PRE) where the registers allow it: the 256x256 tile's
      // 128 accumulators + 96 fragment registers + the persistent loop's state would spill
      constexpr bool PRE = TC * TP * 4 + (TC + TP) * (BK / 32) * 4 <= 192;
      if constexpr (!PRE) {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
        bf16x8_t af[TC], bfr[TP];
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          const int row = wc * WC + ic * 16 + (lane & 15);
          af[ic] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) {
          const int row = wp * WP + ip * 16 + (lane & 15);
          bfr[ip] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
#pragma unroll
        for (int ic = 0; ic < TC; ++ic)
#pragma unroll
          for (int ip = 0; ip < TP; ++ip)
            acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
      }
      } else {
      bf16x8_t af[BK / 32][TC], bfr[BK / 32][TP];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) {
          const int row = wp * WP + ip * 16 + (lane & 15);
          bfr[kk][ip] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          const int row = wc * WC + ic * 16 + (lane & 15);
          af[kk][ic] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + (swz_nk<BK>(row, chunk) << 4));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int ic = 0; ic < TC; ++ic)
#pragma unroll
          for (int ip = 0; ip < TP; ++ip)
            acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][ic], bfr[kk][ip], acc[ic][ip], 0, 0, 0);
      }
    }
    glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int BC, int BP, int WC, int WP, int ST, int BK = 64>
static int launch_glds_pers(const IgemmArgs& a, hipStream_t st) {
  if (a.Kpad / BK < ST - 1) return (int)hipErrorInvalidValue;
  const int M = a.N * a.Ho * a.Wo;
  const int tiles = ((M + BP - 1) / BP) * (a.Ngemm / BC);
  int grid = cu_count();
  if (grid > tiles) grid = tiles;
  grid = (grid + 7) & ~7;                     // XCD chunks: a multiple of 8 workgroups
  hipLaunchKernelGGL((igemm_glds_pers_kernel<BC, BP, WC, WP, ST, BK>), dim3(grid), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Ping-pong, steady-state form (cfg 14): a 256 x 256 tile in four MFMA phases per K-tile (one 64 x 32
// accumulator quadrant each) with the two wave halves one barrier apart, and a half-tile LDS-DMA
// schedule; the K loop body is straight-line code: the K-tile coordinates of the two tiles in
// flight (s+1, s+2) advance incrementally (no per-issue integer division), every phase of the steady
// loop issues its half-tile and waits a constant vmcnt(8), and the last two K-tiles are a peeled tail
// with compile-time waits.  Per phase: B fragments first, then A (as the 8-phase template orders them).
template <int EP = 0>       // epilogue kind (glds_ep_kind)
__global__ __launch_bounds__(512) void igemm_pp2_kernel(IgemmArgs a) {
  constexpr int BC = 256, BP = 256, WC = 128, WP = 64, TC = 8, TP = 4, RBY = 128;
  constexpr int STAGE = (BC + BP) * RBY;
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int M = a.N * a.Ho * a.Wo;
  const int nct = a.Ngemm / BC;
  const int npt = (M + BP - 1) / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  int pt, ct;
  glds_tile(bid, npt, nct, pt, ct);
  const int m0 = pt * BP, c0 = ct * BC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid & 1, wp = wid >> 1, grp = wid >> 2;
  const int lr = lane >> 3;
  const int lchunk = (lane & 7) ^ lr;
  unsigned woff[2][2], pbase[2][2], tmask[2][2];
  const int taps = a.KH * a.KW;
  const int hw = a.Ho * a.Wo;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      woff[h][j] = (unsigned)(((c0 + j * 128 + h * 64 + wid * 8 + lr) * a.Kpad) * 2 + lchunk * 16);
      const int m = m0 + (2 * j + grp) * 64 + h * 32 + (wid & 3) * 8 + lr;
      const bool pok = m < M;
      const int mm = pok ? m : 0;
      const int pn = mm / hw;
      const int rem = mm - pn * hw;
      const int ph = rem / a.Wo, pw = rem - ph * a.Wo;
      const int h0 = ph * a.stride - a.pad, w0 = pw * a.stride - a.pad;
      unsigned msk = 0;
      for (int t = 0; t < taps; ++t) {
        const int kh = t / a.KW, kw = t - kh * a.KW;
        const int ih = h0 + kh, iw = w0 + kw;
        if (pok && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) msk |= 1u << t;
      }
      tmask[h][j] = msk;
      pbase[h][j] = (unsigned)((((pn * a.Hs + h0) * a.Ws + w0) * a.ldx) * 2 + lchunk * 16);
    }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  const int S = a.Kpad / 64;                   // host guarantees S >= 2
  const bool slm = !(a.korder & 1) && a.Kpad == taps * a.Cs;

  // K-tile coordinates, advanced one K-tile at a time (wave-uniform scalars)
  struct KC { int tap, ci, kh, kw; };
  auto knext = [&](KC c) {
    bool tapinc = true;
    if (!slm) {
      c.ci += 64;
      tapinc = c.ci == a.Cs;
      if (tapinc) c.ci = 0;
    }
    if (tapinc) {
      if (++c.tap == taps) {
        c.tap = c.kh = c.kw = 0;
        if (slm) c.ci += 64;
      } else if (++c.kw == a.KW) {
        c.kw = 0;
        ++c.kh;
      }
    }
    return c;
  };
  auto issueA = [&](int h, int buf, KC c) {
    char* base = lds + buf * STAGE;
    const unsigned wk = (unsigned)((c.tap * a.Cs + c.ci) * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(wrs, base + (j * 128 + h * 64 + wid * 8) * RBY, woff[h][j] + wk);
  };
  auto issueB = [&](int h, int buf, KC c) {
    char* base = lds + buf * STAGE + BC * RBY;
    const unsigned delta = (unsigned)(((c.kh * a.Ws + c.kw) * a.ldx + c.ci) * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = (tmask[h][j] >> c.tap) & 1u;
      dma16(xr, base + ((2 * j + grp) * 64 + h * 32 + (wid & 3) * 8) * RBY, ok ? pbase[h][j] + delta : 0x80000000u);
    }
  };

  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  KC k0{0, 0, 0, 0};
  KC k1 = knext(k0);
  issueA(0, 0, k0);
  issueB(0, 0, k0);
  issueB(1, 0, k0);
  issueA(1, 0, k0);
  issueA(0, 1, k1);
  issueB(0, 1, k1);
  wait_vm<8>();
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();       // the second half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  bf16x8_t af[4][2], bfr[2][2][2];
  auto readA = [&](const char* Wt, int h) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ic = 0; ic < 4; ++ic) {
        const int row = wc * WC + h * 64 + ic * 16 + (lane & 15);
        const int chunk = kk * 4 + (lane >> 4);
        af[ic][kk] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + ((chunk ^ (row & 7)) << 4));
      }
  };
  auto readB = [&](const char* P, int h) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ip = 0; ip < 2; ++ip) {
        const int row = wp * WP + h * 32 + ip * 16 + (lane & 15);
        const int chunk = kk * 4 + (lane >> 4);
        bfr[h][ip][kk] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + ((chunk ^ (row & 7)) << 4));
      }
  };
  auto mfma_quad = [&](int qa, int qb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ic = 0; ic < 4; ++ic)
#pragma unroll
        for (int ip = 0; ip < 2; ++ip)
          acc[qa * 4 + ic][qb * 2 + ip] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic][kk], bfr[qb][ip][kk], acc[qa * 4 + ic][qb * 2 + ip], 0, 0, 0);
  };
  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // steady state: K-tiles s < S-2 issue halves of s+1 (B1, A1) and s+2 (A0, B0)
  KC kc1 = k1, kc2 = knext(k1);
  int s = 0;
  for (; s < S - 2; ++s) {
    const int b = s & 1;
    const char* Wt = lds + b * STAGE;
    const char* P = Wt + BC * RBY;
    readB(P, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(Wt, 0);
    issueB(1, b ^ 1, kc1);
    wait_vm<8>();
    sync_in();
    mfma_quad(0, 0);
    sync_out();
    readB(P, 1);
    issueA(1, b ^ 1, kc1);
    wait_vm<8>();
    sync_in();
    mfma_quad(0, 1);
    sync_out();
    readA(Wt, 1);
    issueA(0, b, kc2);
    sync_in();
    mfma_quad(1, 1);
    sync_out();
    issueB(0, b, kc2);
    wait_vm<8>();
    sync_in();
    mfma_quad(1, 0);
    sync_out();
    kc1 = kc2;
    kc2 = knext(kc2);
  }
  {  // K-tile S-2: halves of S-1 still to issue; nothing of S
    const int b = s & 1;
    const char* Wt = lds + b * STAGE;
    const char* P = Wt + BC * RBY;
    readB(P, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(Wt, 0);
    issueB(1, b ^ 1, kc1);
    wait_vm<8>();
    sync_in();
    mfma_quad(0, 0);
    sync_out();
    readB(P, 1);
    issueA(1, b ^ 1, kc1);
    wait_vm<8>();
    sync_in();
    mfma_quad(0, 1);
    sync_out();
    readA(Wt, 1);
    sync_in();
    mfma_quad(1, 1);
    sync_out();
    wait_vm<4>();                              // A0/B0 of S-1 (B1, A1 of S-1 may stay in flight)
    sync_in();
    mfma_quad(1, 0);
    sync_out();
    ++s;
  }
  {  // K-tile S-1
    const int b = s & 1;
    const char* Wt = lds + b * STAGE;
    const char* P = Wt + BC * RBY;
    readB(P, 0);
    __builtin_amdgcn_sched_barrier(0);
    readA(Wt, 0);
    wait_vm<2>();                              // B1 of S-1
    sync_in();
    mfma_quad(0, 0);
    sync_out();
    readB(P, 1);
    wait_vm<0>();                              // A1 of S-1
    sync_in();
    mfma_quad(0, 1);
    sync_out();
    readA(Wt, 1);
    sync_in();
    mfma_quad(1, 1);
    sync_out();
    sync_in();
    mfma_quad(1, 0);
    sync_out();
  }
  if (!grp) __builtin_amdgcn_s_barrier();      // balance the second half's extra barrier

  if constexpr (EP != 0) glds_epilogue_fast<TC, TP, WC, WP, EP>(a, acc, M, m0, c0, wc, wp, lane);
  else glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
}

// ------------------------------------------------------------------------------------------------
// Row-block ping-pong (cfg 14 with row-block pixel staging, 3x3 s1 p1 convs whose 256-pixel tiles are
// whole image rows, W in {32, 64, 128, 256}, or 256-pixel parts of rows, W % 256 == 0).  cfg 14 stages the pixel operand per K-tile = per (tap,
// 64-channel slice): the three kw taps of a kernel row fetch three 1-pixel-shifted copies of the same
// rows (32 KB each).  Here the pixel half-tiles of a kernel row kh are fetched ONCE as blocks of four
// 34-pixel row segments (the 32 pixels of a wave's quadrant + the kw halo; 17 KB) and the kw = 0,1,2
// K-tiles read them at a 0/1/2-row offset: per kernel row 96 KB of weights + 34 KB of pixels instead
// of 96 + 96 KB.  The K order (slice-major, taps kh-major) and hence every accumulation is the same as
// cfg 14's: bitwise-equal output.  Weight half-tiles keep cfg 14's schedule (p1 -> A1(s+1), p2 ->
// A0(s+2)); the pixel blocks of kernel-row group g+1 are issued during the first two K-tiles of group g
// (p3 of t = 0 -> B0, p0 of t = 1 -> B1) into the other of two group buffers.  The K loop runs one
// kernel-row group (three K-tiles) per iteration with every position's wait a constant: the number of
// DMA instructions this wave issued after the unit it needs (wave 0 issues the 17th instruction of
// each pixel block, so its counts are one higher per block).
// BC = 128 (the 128-output-channel convs / dgrads of the 128^2 level): the same schedule with 64 channels
// per wave (2 x 32-row quadrant halves, 8 MFMAs per quadrant, one weight DMA instruction per half-tile);
// 100 KB of LDS instead of 132.
template <int EP, int BC = 256, bool BNS = false>
__global__ __launch_bounds__(512) void igemm_pp2h_kernel(IgemmArgs a) {
  static_assert(BC == 256 || BC == 128, "channel tile");
  constexpr int BP = 256, WC = BC / 2, WP = 64, TC = WC / 16, TP = 4, RBY = 128;
  constexpr int QA = WC / 2;                   // weight rows per wave and quadrant half
  constexpr int NIC = QA / 16;                 // weight fragments per quadrant half
  constexpr int AI = BC / 128;                 // weight DMA instructions per half-tile per wave
  constexpr int ASTAGE = BC * RBY;             // weight K-tile image (32 / 16 KB)
  constexpr int SEG = 34;                      // pixel rows per quadrant segment (32 + kw halo)
  constexpr int BHALF = 4 * SEG * RBY;         // one pixel half-block (17 KB, 17 DMA instructions)
  static_assert(2 * BHALF >= 4 * 2 * BC * 4, "BN sums staging fits one pixel group buffer");
  __shared__ __attribute__((aligned(16))) char lds[2 * ASTAGE + 4 * BHALF];
  char* const Bimg = lds + 2 * ASTAGE;

  const int M = a.N * a.Ho * a.Wo;
  const int W = a.Wo, H = a.Ho, HW = H * W;
  const int nct = a.Ngemm / BC;
  const int npt = M / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  int pt, ct;
  glds_tile(bid, npt, nct, pt, ct);
  const int m0 = pt * BP, c0 = ct * BC;
  const int img = m0 / HW, p0 = m0 - img * HW;               // tile = pixels p0 .. p0 + 255 of image img
                                                             // (whole rows, or a part of one row for W >= 512)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid & 1, wp = wid >> 1, grp = wid >> 2;
  const int lr = lane >> 3;
  const int lchunk = (lane & 7) ^ lr;
  // weight half-tile h = rows {w*WC + h*QA + [0, QA) : w = 0, 1}; instruction i = j*8 + wid of it covers
  // its rows 8i .. 8i+7 (channel wave (8i) / QA, row (8i) % QA of that wave's half)
  unsigned woff[2][AI];
  int wdst[2][AI];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int i8 = 8 * (j * 8 + wid);
      const int row = (i8 / QA) * WC + h * QA + i8 % QA;
      wdst[h][j] = row * RBY;
      woff[h][j] = (unsigned)(((c0 + row + lr) * a.Kpad) * 2 + lchunk * 16);
    }
  // pixel block DMA: instruction i of a half-block fills LDS rows 8i .. 8i+7; wave w issues i = w, 8 + w
  // and wave 0 also i = 16.  LDS row q -> quadrant segment q / 34, pixel (q % 34) - 1 of the segment's
  // 32 columns; for kernel row kh the image row is the segment's row + kh - 1.
  const int NI = wid == 0 ? 3 : 2;
  int bbase[2][3];                             // byte offset of the (kh = 0) source pixel, per half / instruction
  unsigned bvalid[2][3];                       // bit kh: source row of kernel row kh inside the image
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int i = j < 2 ? j * 8 + wid : 16;
      const int q = 8 * i + lr;
      const int sg = q / SEG, loc = q - sg * SEG;
      const int pq = sg * 64 + h * 32;                        // first pixel of the quadrant segment
      const int r = (p0 + pq) / W, col = (p0 + pq) % W + loc - 1;
      const bool cok = col >= 0 && col < W && (j < 2 || wid == 0);
      unsigned vb = 0;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int ih = r + kh - 1;
        if (cok && ih >= 0 && ih < H) vb |= 1u << kh;
      }
      bvalid[h][j] = vb;
      bbase[h][j] = (((img * a.Hs + r - 1) * a.Ws + col) * a.ldx) * 2 + lchunk * 16;
    }
  const int rowB = W * a.ldx * 2;              // bytes per image row
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  const int S = a.Kpad / 64;                   // 9 K-tiles per 64-channel slice; host: S >= 9
  const int G = S / 3;                         // kernel-row groups

  // K-tile coordinates (tap, 64-channel slice), advanced one K-tile at a time (no division)
  struct KC { int tap, ci; };
  auto knext = [&](KC c) {
    if (++c.tap == 9) { c.tap = 0; c.ci += 64; }
    return c;
  };
  auto issueA = [&](int h, int buf, KC c) {
    const unsigned wk = (unsigned)((c.tap * a.Cs + c.ci) * 2);
    char* base = lds + buf * ASTAGE;
#pragma unroll
    for (int j = 0; j < AI; ++j) dma16(wrs, base + wdst[h][j], woff[h][j] + wk);
  };
  // pixel half-block h of kernel row kh, slice ci, into group buffer gb (2 instructions; wave 0: 3)
  auto issueB = [&](int h, int gb, int kh, int ci) {
    char* base = Bimg + (gb * 2 + h) * BHALF;
    const int add = kh * rowB + ci * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = (bvalid[h][j] >> kh) & 1u;
      dma16(xr, base + (j * 8 + wid) * 1024, ok ? (unsigned)(bbase[h][j] + add) : 0x80000000u);
    }
    if (wid == 0) {
      const bool ok = (bvalid[h][2] >> kh) & 1u;
      dma16(xr, base + 16 * 1024, ok ? (unsigned)(bbase[h][2] + add) : 0x80000000u);
    }
  };
  // the waits count the DMA instructions this wave issued after the staged unit it needs; a pixel
  // block is 3 instructions in wave 0 and 2 in the others (static per position in the group)
  const bool w0 = wid == 0;

  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // 128-channel dgrad: the ReLU-mask fragments of the epilogue (32 VGPRs) are loaded before the first
  // DMA; they are older than every staged unit, so the constant waits below are unchanged
  constexpr bool PM = EP == 2 && BC == 128 && !BNS;
  constexpr bool PB = EP == 1 && BC == 128 && !BNS;   // likewise the forward bias (16 VGPRs)
  float pbias[PB ? TC * 4 : 1];
  if constexpr (PB) {
    const int cb = c0 + wc * WC + 4 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < TC * 4; ++k) pbias[k] = a.bias ? a.bias[cb + (k >> 2) * 16 + (k & 3)] : 0.f;
  }
  u32x2_t pmk[PM ? TP * TC : 1];
  if constexpr (PM) {
    const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)a.mask, 0, 0x7fffffff, 0x00020000);
    const int cb = c0 + wc * WC + 4 * (lane >> 4);
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) {
      const int m = m0 + wp * WP + ip * 16 + (lane & 15);
      const unsigned mo = m < M ? (unsigned)m * (unsigned)a.ldm * 2u + (unsigned)cb * 2u : 0x80000000u;
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) pmk[ip * TC + ic] = __builtin_amdgcn_raw_buffer_load_b64(mr, mo + ic * 32, 0, 0);
    }
  }

  // prologue: weights of K-tiles 0 (both halves) and 1 (half 0), pixel blocks of group 0
  const KC k0{0, 0};
  KC kA1 = knext(k0);                          // K-tile s+1 (A1 issue at p1 of s)
  issueA(0, 0, k0);
  issueB(0, 0, 0, 0);
  issueB(1, 0, 0, 0);
  issueA(1, 0, k0);
  issueA(0, 1, kA1);
  KC kA0 = knext(kA1);                         // K-tile s+2 (A0 issue at p2 of s)
  // waits below: "2 * AI" = two weight half-tiles, "+ 3 / + 2" = one pixel half-block (wave 0 / others)
  if (w0) wait_vm<2 * AI + 3>(); else wait_vm<2 * AI + 2>();   // A0(0), B0(0): newer are B1(0), A1(0), A0(1)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();       // the second half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  bf16x8_t af[NIC][2], bfr[2][2][2];
  auto readA = [&](const char* Wt, int h) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ic = 0; ic < NIC; ++ic) {
        const int row = wc * WC + h * QA + ic * 16 + (lane & 15);
        const int chunk = kk * 4 + (lane >> 4);
        af[ic][kk] = *reinterpret_cast<const bf16x8_t*>(Wt + row * RBY + ((chunk ^ (row & 7)) << 4));
      }
  };
  // B quadrant h of group buffer gb at kw: segment rows wp*34 + ip*16 + (lane & 15) + kw
  auto readB = [&](int gb, int h, int kw) {
    const char* P = Bimg + (gb * 2 + h) * BHALF;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ip = 0; ip < 2; ++ip) {
        const int row = wp * SEG + ip * 16 + (lane & 15) + kw;
        const int chunk = kk * 4 + (lane >> 4);
        bfr[h][ip][kk] = *reinterpret_cast<const bf16x8_t*>(P + row * RBY + ((chunk ^ (row & 7)) << 4));
      }
  };
  auto mfma_quad = [&](int qa, int qb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ic = 0; ic < NIC; ++ic)
#pragma unroll
        for (int ip = 0; ip < 2; ++ip)
          acc[qa * NIC + ic][qb * 2 + ip] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic][kk], bfr[qb][ip][kk], acc[qa * NIC + ic][qb * 2 + ip], 0, 0, 0);
  };
  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // one kernel-row group (3 K-tiles, kw = 0, 1, 2) of group buffer gb; LAST: no next group, and the
  // K-tiles beyond S are not issued.  kh2/ci2 = kernel row / slice of the next group.
  auto group = [&](auto LASTc, int gb, int bA, int kh2, int ci2) {
    constexpr bool LAST = decltype(LASTc)::value;
    // ---- t = 0 (weights buffer bA)
    {
      const char* Wt = lds + bA * ASTAGE;
      readB(gb, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      readA(Wt, 0);
      wait_vm<2 * AI>();                       // B1 of this group (conservative: newer >= 2 half-tiles)
      sync_in();
      mfma_quad(0, 0);
      sync_out();
      readB(gb, 1, 0);
      issueA(1, bA ^ 1, kA1);
      wait_vm<2 * AI>();                       // A1 of this K-tile
      sync_in();
      mfma_quad(0, 1);
      sync_out();
      readA(Wt, 1);
      issueA(0, bA, kA0);
      sync_in();
      mfma_quad(1, 1);
      sync_out();
      if constexpr (!LAST) {
        issueB(0, gb ^ 1, kh2, ci2);
        if (w0) wait_vm<2 * AI + 3>(); else wait_vm<2 * AI + 2>();   // A0 of K-tile t = 1
      } else {
        wait_vm<2 * AI>();
      }
      sync_in();
      mfma_quad(1, 0);
      sync_out();
      kA1 = kA0;
      kA0 = knext(kA0);
    }
    // ---- t = 1 (weights buffer bA ^ 1)
    {
      const char* Wt = lds + (bA ^ 1) * ASTAGE;
      readB(gb, 0, 1);
      __builtin_amdgcn_sched_barrier(0);
      readA(Wt, 0);
      if constexpr (!LAST) issueB(1, gb ^ 1, kh2, ci2);
      sync_in();
      mfma_quad(0, 0);
      sync_out();
      readB(gb, 1, 1);
      issueA(1, bA, kA1);
      if constexpr (!LAST) {
        if (w0) wait_vm<2 * AI + 6>(); else wait_vm<2 * AI + 4>();   // A1 of this K-tile
      } else {
        wait_vm<2 * AI>();
      }
      sync_in();
      mfma_quad(0, 1);
      sync_out();
      readA(Wt, 1);
      if constexpr (!LAST) issueA(0, bA ^ 1, kA0);
      sync_in();
      mfma_quad(1, 1);
      sync_out();
      if constexpr (!LAST) {
        if (w0) wait_vm<2 * AI + 6>(); else wait_vm<2 * AI + 4>();   // A0 of K-tile t = 2
      } else {
        wait_vm<AI>();
      }
      sync_in();
      mfma_quad(1, 0);
      sync_out();
      kA1 = kA0;
      kA0 = knext(kA0);
    }
    // ---- t = 2 (weights buffer bA)
    {
      const char* Wt = lds + bA * ASTAGE;
      readB(gb, 0, 2);
      __builtin_amdgcn_sched_barrier(0);
      readA(Wt, 0);
      sync_in();
      mfma_quad(0, 0);
      sync_out();
      readB(gb, 1, 2);
      if constexpr (!LAST) {
        issueA(1, bA ^ 1, kA1);
        wait_vm<2 * AI>();                     // A1 of this K-tile
      } else {
        wait_vm<0>();
      }
      sync_in();
      mfma_quad(0, 1);
      sync_out();
      readA(Wt, 1);
      if constexpr (!LAST) issueA(0, bA, kA0);
      sync_in();
      mfma_quad(1, 1);
      sync_out();
      if constexpr (!LAST) wait_vm<2 * AI>();  // A0 of the next group's first K-tile (+ its B0, older)
      sync_in();
      mfma_quad(1, 0);
      sync_out();
      kA1 = kA0;
      kA0 = knext(kA0);
    }
  };

  // K-tile s = 3 g + t uses weights buffer s & 1: (g & 1, !(g & 1), g & 1) within group g
  int kh = 0, ci = 0;
#pragma unroll 1
  for (int g = 0; g < G - 1; ++g) {
    int kh2 = kh + 1, ci2 = ci;
    if (kh2 == 3) { kh2 = 0; ci2 += 64; }
    group(std::integral_constant<bool, false>{}, g & 1, g & 1, kh2, ci2);
    kh = kh2;
    ci = ci2;
  }
  group(std::integral_constant<bool, true>{}, (G - 1) & 1, (G - 1) & 1, 0, 0);
  if (!grp) __builtin_amdgcn_s_barrier();      // balance the second half's extra barrier

  // BN sums: staged in the pixel group buffer the last kernel-row group does not use (last read in
  // group G-2, before barriers every wave has passed; no DMA targets it any more)
  if constexpr (BNS)
    glds_epilogue_bns<TC, TP, WC, WP, EP>(a, acc, M, m0, c0, wc, wp, lane,
                                          reinterpret_cast<float*>(Bimg + ((((G - 1) & 1) ^ 1) * 2) * BHALF));
  else if constexpr (PM) glds_epilogue_fast<TC, TP, WC, WP, EP, true>(a, acc, M, m0, c0, wc, wp, lane, pmk);
  else if constexpr (PB) glds_epilogue_fast<TC, TP, WC, WP, EP, false, true>(a, acc, M, m0, c0, wc, wp, lane, nullptr, pbias);
  else if constexpr (EP != 0) glds_epilogue_fast<TC, TP, WC, WP, EP>(a, acc, M, m0, c0, wc, wp, lane);
  else glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
}

// ------------------------------------------------------------------------------------------------
// Slice-staged implicit GEMM (cfg 18: 128 output channels x 512 pixels), conv3x3 s1 p1 on tiles of R
// whole image rows (W in {32, 64, 128}).  The template also has a 256 x 256 form (BC = 256); measured
// slower than igemm_pp2h_kernel<EP, 256> on every 256-channel layer (profiles/kbench_sl_b256_r04.txt),
// it is not instantiated.
//
// Why: the row-block kernel (pp2h) stages the pixel operand once per (kernel row, 64-channel slice)
// and the weights once per K-tile for every 256-pixel tile; at 128 output channels that is 28 KB of
// LDS-DMA per 4.2 MFLOP K-tile (150 FLOP/B), and measured it runs at ~2500 cycles per K-tile whatever
// the barrier structure (a two-phase variant with half the barriers measured bitwise-equal and
// exactly as fast, profiles/kbench_rb2_b256_r04.txt; removed) -- the DMA traffic per FLOP, not the
// MFMA schedule, bounds it.  Here a tile's pixel operand is staged ONCE
// per 32-channel slice as an (R+2) x (W+2) image with its zero halo and all 9 taps read from it, and the
// 128-channel tile covers 512 pixels: per 32-deep K-tile 8 KB of weights + 5.5 KB of pixels for
// 4.2 MFLOP (310 FLOP/B, half the DMA instructions per MFMA of pp2h's 128-channel form).
//
// Geometry: 8 waves, each a 128-channel x 64-pixel tile (TC 8 x TP 4 accumulators, one 16x16x32 MFMA
// per (channel, pixel) fragment and tap): 1 x 8 waves at 128 channels, 2 x 4 at 256.  LDS rows are
// 64 B (32 channels) with the chunk swizzle swz64 (conflict-free ds_read_b128 for 16 consecutive rows
// from any first row -- the pixel reads of a tap start anywhere).  A "step" = (slice, kernel row): the
// 3 kw taps of that row, 96 MFMAs per wave; the step's weights (3 taps x BC rows) and the next slice's
// image are double-buffered and issued at the start of the previous step, which ends with
// __syncthreads (vmcnt(0): they had a whole step to land).
__device__ __forceinline__ int swz64(int row) { return ((row >> 2) & 1) << 1; }

template <int EP, int BC>
__global__ __launch_bounds__(512) void igemm_sl_kernel(IgemmArgs a) {
  static_assert(BC == 128 || BC == 256, "channel tile");
  constexpr int NCW = BC / 128, NPW = 8 / NCW, WC = 128, WP = 64, TC = 8, TP = 4;
  constexpr int BP = NPW * WP;                       // 512 / 256 pixels
  constexpr int RB = 64;                             // LDS row bytes (32 channels)
  constexpr int WSTEP = 3 * BC * RB;                 // one step's weights: 24 / 48 KB
  constexpr int PIMG = BC == 128 ? 49 * 1024 : 25 * 1024;   // largest (R+2)(W+2) image, whole DMA instructions
  constexpr int NWI = 3 * BC / 16 / 8;               // weight DMA instructions per wave per step: 3 / 6
  constexpr int MI = (PIMG / 1024 + 7) / 8;          // pixel DMA instruction slots per wave per image: 7 / 4
  __shared__ __attribute__((aligned(16))) char lds[2 * WSTEP + 2 * PIMG];
  char* const Pimg = lds + 2 * WSTEP;

  const int W = a.Wo, H = a.Ho, HW = H * W;
  const int lw = 31 - __builtin_clz(W);             // W is a power of two (host)
  const int R = BP >> lw;                            // image rows per tile
  const int W2 = W + 2;
  const int NPX = (R + 2) * W2;                      // pixels of the slice image
  const int NPI = (NPX + 15) >> 4;                   // DMA instructions per image
  const int M = a.N * HW;
  const int nct = a.Ngemm / BC, npt = M / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  int pt, ct;
  glds_tile(bid, npt, nct, pt, ct);
  const int m0 = pt * BP, c0 = ct * BC;
  const int img = m0 / HW, r0 = (m0 - img * HW) >> lw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % NCW, wp = wid / NCW;
  const int lq = lane >> 2, lc = lane & 3;

  // weight DMA: step instruction u = wid + 8 v covers tap kw = u / (BC/16), rows 16 (u % (BC/16)) + lq
  unsigned wsrc[NWI];
#pragma unroll
  for (int v = 0; v < NWI; ++v) {
    const int u = wid + 8 * v;
    const int kw = u / (BC / 16), row = 16 * (u % (BC / 16)) + lq;
    wsrc[v] = (unsigned)(((c0 + row) * a.Kpad + kw * a.Cs) * 2 + ((lc ^ swz64(row)) << 4));
  }
  // pixel DMA: image instruction i = wid + 8 m covers image pixels 16 i + lq (flattened (R+2) x (W+2))
  unsigned psrc[MI];
  unsigned pvalid = 0;
#pragma unroll
  for (int m = 0; m < MI; ++m) {
    const int P = 16 * (wid + 8 * m) + lq;
    const int rr = P / W2, cc = P - rr * W2;
    const int row = r0 - 1 + rr, col = cc - 1;
    const bool ok = P < NPX && row >= 0 && row < H && col >= 0 && col < W;
    pvalid |= (ok ? 1u : 0u) << m;
    psrc[m] = (unsigned)((((img * a.Hs + row) * a.Ws + col) * a.ldx) * 2 + ((lc ^ swz64(P)) << 4));
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);

  auto issueW = [&](int buf, int sl, int kh) {
    const unsigned add = (unsigned)((kh * 3 * a.Cs + sl * 32) * 2);
    char* base = lds + buf * WSTEP;
#pragma unroll
    for (int v = 0; v < NWI; ++v) dma16(wrs, base + (wid + 8 * v) * 1024, wsrc[v] + add);
  };
  // the pixel instructions m = kh, kh + 3, ... of slice sl's image (a third of it per step)
  auto issueP = [&](int buf, int sl, int kh) {
    char* base = Pimg + buf * PIMG;
#pragma unroll
    for (int m = 0; m < MI; ++m) {
      if (m % 3 != kh || wid + 8 * m >= NPI) continue;   // wave-uniform
      const bool ok = (pvalid >> m) & 1u;
      dma16(xr, base + (wid + 8 * m) * 1024, ok ? psrc[m] + (unsigned)(sl * 64) : 0x80000000u);
    }
  };

  // fragment addresses: A row = wc*128 + ic*16 + (lane & 15); B output pixel q -> image pixel base
  const int chunk = lane >> 4;
  int pb[TP];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int q = wp * WP + ip * 16 + (lane & 15);
    pb[ip] = (q >> lw) * W2 + (q & (W - 1));
  }
  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int NSL = a.Cs / 32, NS = NSL * 3;
  issueW(0, 0, 0);
#pragma unroll
  for (int k = 0; k < 3; ++k) issueP(0, 0, k);
  wait_vm<0>();                                      // this wave's DMAs have landed ...
  __syncthreads();                                   // ... and every wave's

  int sl = 0, kh = 0;
#pragma unroll 1
  for (int j = 0; j < NS; ++j) {
    int kh2 = kh + 1, sl2 = sl;
    if (kh2 == 3) { kh2 = 0; ++sl2; }
    if (j + 1 < NS) issueW((j + 1) & 1, sl2, kh2);
    if (sl + 1 < NSL) issueP((sl + 1) & 1, sl + 1, kh);
    const char* Wb = lds + (j & 1) * WSTEP;
    const char* Pb = Pimg + (sl & 1) * PIMG;
    const int poff = kh * W2;
    // fragments of tap kw+1 are read while the MFMAs of tap kw run (two register sets)
    auto rd = [&](int kw, bf16x8_t (&af)[TC], bf16x8_t (&bf)[TP]) {
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        const int row = wc * WC + ic * 16 + (lane & 15);
        af[ic] = *reinterpret_cast<const bf16x8_t*>(Wb + (kw * BC + row) * RB + ((chunk ^ swz64(row)) << 4));
      }
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const int P = pb[ip] + poff + kw;
        bf[ip] = *reinterpret_cast<const bf16x8_t*>(Pb + P * RB + ((chunk ^ swz64(P)) << 4));
      }
    };
    auto mm = [&](const bf16x8_t (&af)[TC], const bf16x8_t (&bf)[TP]) {
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip)
          acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bf[ip], acc[ic][ip], 0, 0, 0);
    };
    bf16x8_t a0[TC], b0[TP], a1[TC], b1[TP];
    rd(0, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    rd(1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mm(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    rd(2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mm(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mm(a0, b0);
    if (j + 1 < NS) {
      wait_vm<0>();
      __syncthreads();
    }
    sl = sl2;
    kh = kh2;
  }

  if constexpr (EP != 0) glds_epilogue_fast<TC, TP, WC, WP, EP>(a, acc, M, m0, c0, wc, wp, lane);
  else glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
}

// ds_read_b128 as inline asm with an immediate offset (see igemm_slp_kernel)
template <int OFF = 0>
__device__ __forceinline__ bf16x8_t lds_read128_i(unsigned addr) {
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

// Slice-staged kernel on the ping-pong schedule (cfg 18's default since round 6; the kernel above stays as
// DPA_NO_SLPP=1).  Same tile, slice images and fragments as igemm_sl_kernel<EP, 128>, but the K loop is
// one phase per tap -- 12 fragment reads, then 32 MFMAs per wave -- with the two wave halves one barrier
// apart (one half issues its MFMAs while the other reads its fragments and issues DMA), instead of three
// taps per step ending in vmcnt(0) + __syncthreads with every wave waiting at once (35-45 % MFMA,
// profiles/pmc_b128_512_r05_end.txt).  Weights are staged per tap: a ring of six 8-KB tap buffers, the
// tap of phase g + 4 issued at phase g (into the buffer phase g - 2 read: two phases, i.e. both halves,
// past its last read), so each has ~3 phases to land; the next slice's image is issued in slots 1-4 of
// the 9 phases of the current slice (2 instructions per wave per phase, zero-fill dummies past the
// image) into the other image buffer.  Every wave issues the same DMA count per phase, so the waits are
// compile-time vmcnt values (slice loop unrolled by its 9 phases).
//
// BC = 64 (round 6, the 64-output-channel convs the row-halo kernel took: 256^2 128 -> 64 forward, 128^2 dgrads
// into 64 channels): 8 waves of 64 channels x 64 pixels (16 MFMAs per phase), 512-pixel tiles of whole rows
// up to W = 256 (R = 2: a 4 x 258-pixel image, 65 KB per buffer); the 4-KB tap weights are 4 DMA
// instructions, so waves 4-7 issue a zero-fill dummy into the dump area (uniform vmcnt); the next slice's
// image goes out 3 slots per phase in phases 1-3.
template <int EP, int BC>
__global__ __launch_bounds__(512) void igemm_slp_kernel(IgemmArgs a) {
  static_assert(BC == 64 || BC == 128 || BC == 256, "channel tile");
  constexpr int WC = BC == 64 ? 64 : 128, TC = WC / 16, TP = 4, WP = 64, RB = 64;
  constexpr int NCW = BC / WC, BP = 8 / NCW * WP;    // 1 x 8 waves, 512 pixels / 2 x 4 waves, 256 pixels
  constexpr int TAPB = BC * RB;                      // one tap's weights: 4 / 8 / 16 KB
  constexpr int NWW = BC == 64 ? 1 : BC / 128;       // weight DMA instructions per wave per phase
  // largest (R+2)(W+2) image in whole DMA instructions: 64 channels W <= 256 (R >= 2), 128 channels W <= 128
  // (R >= 4), 256 channels W <= 64
  constexpr int PIMG = BC == 64 ? 65 * 1024 : BC == 128 ? 49 * 1024 : 25 * 1024;
  constexpr int MI = BC == 64 ? 9 : BC == 128 ? 7 : 4;   // pixel DMA slots per wave per image (8 x MI >= PIMG / 1 KB)
  constexpr int SPP = BC == 64 ? 3 : 2;              // image slots issued per phase
  constexpr int NPQ = (MI + SPP - 1) / SPP;          // phases 1 .. NPQ of a slice issue them
  // phase 8's wait allows the slots of phases 5 .. 8 outstanding: the next image must be out by phase 4
  static_assert(NPQ <= 4, "image issue window");
  __shared__ __attribute__((aligned(1024))) char lds[6 * TAPB + 2 * PIMG + 1024];
  char* const Pimg = lds + 6 * TAPB;
  char* const dump = lds + 6 * TAPB + 2 * PIMG;

  const int W = a.Wo, H = a.Ho, HW = H * W;
  const int lw = 31 - __builtin_clz(W);             // W is a power of two (host)
  const int R = BP >> lw;                            // image rows per tile
  const int W2 = W + 2;
  const int NPX = (R + 2) * W2;                      // pixels of the slice image
  const int NPI = (NPX + 15) >> 4;                   // DMA instructions per image
  const int M = a.N * HW;
  const int nct = a.Ngemm / BC, npt = M / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  int pt, ct;
  glds_tile(bid, npt, nct, pt, ct);
  const int m0 = pt * BP, c0 = ct * BC;
  const int img = m0 / HW, r0 = (m0 - img * HW) >> lw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % NCW, wp = wid / NCW, grp = wid >> 2;
  const int lq = lane >> 2, lc = lane & 3;

  // tap-weight DMA: BC / 16 instructions of 16 rows; wave w -> rows 16 (w + 8 v) + lq
  unsigned wsrc[NWW];
#pragma unroll
  for (int v = 0; v < NWW; ++v) {
    const int wrow = 16 * (wid + 8 * v) + lq;
    wsrc[v] = (unsigned)(((c0 + wrow) * a.Kpad) * 2 + ((lc ^ swz64(wrow)) << 4));
  }
  // pixel DMA: image instruction i = wid + 8 m covers image pixels 16 i + lq (flattened (R+2) x (W+2))
  unsigned psrc[MI];
  unsigned pvalid = 0;
#pragma unroll
  for (int m = 0; m < MI; ++m) {
    const int P = 16 * (wid + 8 * m) + lq;
    const int rr = P / W2, cc = P - rr * W2;
    const int row = r0 - 1 + rr, col = cc - 1;
    const bool ok = P < NPX && row >= 0 && row < H && col >= 0 && col < W;
    pvalid |= (ok ? 1u : 0u) << m;
    psrc[m] = (unsigned)((((img * a.Hs + row) * a.Ws + col) * a.ldx) * 2 + ((lc ^ swz64(P)) << 4));
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);

  const int NSL = a.Cs / 32, NPH = NSL * 9;          // slices, phases (slice-major, then kh, then kw)
  // the weights of phase g (tap (g % 9) / 3, (g % 9) % 3 of slice g / 9) into ring buffer g % 6
  auto issueW = [&](int g) {
    const int sl = g / 9, t = g - 9 * sl;
    const bool real = BC != 64 || wid < 4;             // BC 64: waves 4-7 issue a dummy (wave-uniform)
    const bool ok = g < NPH && real;
#pragma unroll
    for (int v = 0; v < NWW; ++v)
      dma16(wrs, real ? lds + (g % 6) * TAPB + (wid + 8 * v) * 1024 : dump,
            ok ? wsrc[v] + (unsigned)((t * a.Cs + sl * 32) * 2) : 0x80000000u);
  };
  // pixel slot m of slice sl's image into image buffer sl & 1 (dummies past the image / the slices)
  auto issueP = [&](int sl, int m) {
    const bool real = m < MI && wid + 8 * m < NPI;
    const int mm = m < MI ? m : 0;
    const bool ok = real && sl < NSL && ((pvalid >> mm) & 1u);
    char* dst = real ? Pimg + (sl & 1) * PIMG + (wid + 8 * m) * 1024 : dump;
    dma16(xr, dst, ok ? psrc[mm] + (unsigned)(sl * 64) : 0x80000000u);
  };

  // fragment addresses: A row = ic*16 + (lane & 15); B output pixel q -> image pixel base
  const int chunk = lane >> 4;
  int pb[TP];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int q = wp * WP + ip * 16 + (lane & 15);
    pb[ip] = (q >> lw) * W2 + (q & (W - 1));
  }
  f32x4_t acc[TC][TP];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: slice 0's image (SPP NPQ slots) and the weights of phases 0-3
#pragma unroll
  for (int m = 0; m < SPP * NPQ; ++m) issueP(0, m);
  issueW(0);
  issueW(1);
  issueW(2);
  issueW(3);
  wait_vm<3 * NWW>();                                // image 0 and phase 0's weights landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();             // the second half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this phase's fragment reads
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  bf16x8_t af[TC], bf[TP];
  // fragment reads as inline asm: a plain LDS load makes hipcc wait vmcnt(0) first while any LDS-DMA is in
  // flight (it cannot tell the load from the DMA destination); sync_in waits lgkmcnt(0) itself
  const unsigned lds0 = (unsigned)(size_t)LDS_PTR(char, lds);
  const unsigned aoff = (unsigned)((wc * WC + (lane & 15)) * RB + ((chunk ^ swz64(lane & 15)) << 4));   // + ic * 16 rows
  // phase Q (compile-time position in the slice) of slice sl
  auto phase = [&](int sl, auto Qc) {
    constexpr int Q = decltype(Qc)::value, KH = Q / 3, KW = Q % 3;
    const int g = 9 * sl + Q;
    const unsigned wa = lds0 + (unsigned)((g % 6) * TAPB) + aoff;
    const unsigned pbase = lds0 + (unsigned)(6 * TAPB + (sl & 1) * PIMG);
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) af[ic] = lds_read128_i(wa + (unsigned)(ic * 16 * RB));
    const int poff = KH * W2 + KW;
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) {
      int pq = pb[ip];
      asm volatile("" : "+v"(pq));                   // per-phase address math (not 36 hoisted registers)
      const int P = pq + poff;
      bf[ip] = lds_read128_i(pbase + (unsigned)(P * RB + ((chunk ^ swz64(P)) << 4)));
    }
    issueW(g + 4);
    if constexpr (Q >= 1 && Q <= NPQ) {
#pragma unroll
      for (int u = 0; u < SPP; ++u) issueP(sl + 1, SPP * (Q - 1) + u);
    }
    // outstanding after W(g + 1): W(g + 2 .. g + 4) and the image slots of phases g - 3 .. g
    constexpr int P0 = (Q >= 1 && Q <= NPQ) ? SPP : 0, P1 = (Q - 1 >= 1 && Q - 1 <= NPQ) ? SPP : 0;
    constexpr int P2 = (Q - 2 >= 1 && Q - 2 <= NPQ) ? SPP : 0, P3 = (Q - 3 >= 1 && Q - 3 <= NPQ) ? SPP : 0;
    wait_vm<3 * NWW + P0 + P1 + P2 + P3>();
    sync_in();
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int ip = 0; ip < TP; ++ip)
        acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bf[ip], acc[ic][ip], 0, 0, 0);
    sync_out();
  };
#pragma unroll 1
  for (int sl = 0; sl < NSL; ++sl) {
    phase(sl, std::integral_constant<int, 0>{});
    phase(sl, std::integral_constant<int, 1>{});
    phase(sl, std::integral_constant<int, 2>{});
    phase(sl, std::integral_constant<int, 3>{});
    phase(sl, std::integral_constant<int, 4>{});
    phase(sl, std::integral_constant<int, 5>{});
    phase(sl, std::integral_constant<int, 6>{});
    phase(sl, std::integral_constant<int, 7>{});
    phase(sl, std::integral_constant<int, 8>{});
  }
  wait_vm<0>();                                      // no DMA may land after the workgroup ends
  if (!grp) __builtin_amdgcn_s_barrier();            // balance the second half's extra barrier

  if constexpr (EP != 0) glds_epilogue_fast<TC, TP, WC, WP, EP>(a, acc, M, m0, c0, wc, wp, lane);
  else glds_epilogue<TC, TP, WC, WP>(a, acc, M, m0, c0, wc, wp, lane);
}

static int SL_PINGPONG = 1;         // DPA_NO_SLPP=1 -> 0 (set at library load, ops/_lib.py)
static int SLP256 = 0;              // DPA_SLP256=1: 256-channel convs on W <= 64 take igemm_slp_kernel<EP, 256>
DPA_API void dpa_igemm_set_slpp(int on) { SL_PINGPONG = on; }
DPA_API void dpa_igemm_set_slp256(int on) { SLP256 = on; }

// 256-channel slice-staged ping-pong eligible: W in {32, 64}, whole 256-pixel tiles, Cs % 32, unpadded K
static inline bool slp256_ok(const IgemmArgs& a) {
  const int W = a.Wo;
  return a.mode == 0 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Hs == a.Ho && a.Ws == a.Wo &&
         a.Kpad == 9 * a.Cs && (a.Cs % 32) == 0 && a.Ngemm % 256 == 0 && (a.ldx & 7) == 0 && (W == 32 || W == 64) &&
         ((long)a.Ho * W) % 256 == 0;
}

// 64-channel slice-staged ping-pong eligible (cfg 19): W a power of two in [32, 256], whole 512-pixel tiles
static inline bool slp64_ok(const IgemmArgs& a) {
  const int W = a.Wo;
  return a.mode == 0 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Hs == a.Ho && a.Ws == a.Wo &&
         a.Kpad == 9 * a.Cs && (a.Cs % 32) == 0 && a.Ngemm % 64 == 0 && (a.ldx & 7) == 0 &&
         (W == 32 || W == 64 || W == 128 || W == 256) && ((long)a.Ho * W) % 512 == 0;
}

// slice-staged eligible: conv3x3 s1 p1 on one grid, K = 9 Cs unpadded, 32-channel slices, tiles of whole
// rows of one image: W a power of two in [32, 128] (256-channel form: [32, 64])
static inline bool sl_ok(const IgemmArgs& a) {
  const int W = a.Wo;
  return a.mode == 0 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Hs == a.Ho && a.Ws == a.Wo &&
         a.Kpad == 9 * a.Cs && (a.Cs % 32) == 0 && a.Ngemm % 128 == 0 && (a.ldx & 7) == 0 &&
         (W == 32 || W == 64 || W == 128) && ((long)a.Ho * W) % 512 == 0;
}

// row-block staging eligible: conv3x3 s1 p1, slice-major K (Kpad == 9 Cs, Cs % 64 == 0), tiles = whole rows
static inline bool pp2h_ok(const IgemmArgs& a) {
  const int W = a.Wo;
  return a.mode == 0 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Hs == a.Ho && a.Ws == a.Wo &&
         !(a.korder & 1) && a.Kpad == 9 * a.Cs && (a.Cs % 64) == 0 && (W == 32 || W == 64 || W == 128 || W % 256 == 0) &&
         ((long)a.Ho * W) % 256 == 0 && a.Ngemm % 256 == 0;
}

// the 128-channel form (cfg 15): same conditions with Ngemm % 128
static inline bool pp2h128_ok(const IgemmArgs& a) {
  IgemmArgs b = a;
  b.Ngemm = 256;
  return pp2h_ok(b) && a.Ngemm % 128 == 0;
}

template <int BC, int BP, int WC, int WP, int ST, int BK = 64, bool PRE = false>
static int launch_glds(const IgemmArgs& a, hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  const int grid = ((M + BP - 1) / BP) * (a.Ngemm / BC);
  hipLaunchKernelGGL((igemm_glds_kernel<BC, BP, WC, WP, ST, BK, PRE>), dim3(grid), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// cfg 0 = auto.  Tile families (all LDS-DMA, MFMA 16x16x32 bf16):
//   1: 256 (ch) x 128 (px), 3 stages      2: 128 x 256, 3 stages      4: 128 x 128, 4 stages
//   8: 256 x 256 persistent (one workgroup per CU walking XCD-contiguous tiles; short K)
//   14: 256 x 256 ping-pong: row-block pixel staging (igemm_pp2h_kernel) on whole-row tiles of 3x3 s1 p1
//       convs, per-K-tile staging (igemm_pp2_kernel) otherwise
//   15: 128 x 256 row-block ping-pong (igemm_pp2h_kernel<EP, 128>)
//   18 (variant 262144): slice-staged 128 x 512 (igemm_sl_kernel) -- the auto choice for 128-output-channel
//       layers it takes (3-16 % faster than cfg 15 on every 128-channel 512^2-UNet layer,
//       profiles/kbench_sl_b256_r04.txt), cfg 15 where it does not
//   19 (variant 524288): slice-staged ping-pong 64 x 512 (igemm_slp_kernel<EP, 64>), W <= 256
// Flags: +32 no persistent kernel in the auto choice (a side stream owns CUs), +2048 generic epilogue
// (tests), +8192 cfg 14 without row blocks (tests), +1048576 no slice-staged kernel in the auto choice.
// Requires Cs % 64 == 0 (a K-step never straddles a tap; slice-staged: Cs % 32), Kpad % 64 == 0,
// Ngemm % BC == 0.
DPA_API int dpa_igemm_glds(const IgemmArgs* args, int cfg, hipStream_t st) {
  IgemmArgs a = *args;
  if (cfg & 32) a.korder |= 2;          // no persistent kernel in the auto choice
  const bool no_fast_ep = cfg & 2048;   // the generic epilogue (tests)
  const bool no_rowblock = cfg & 8192;  // cfg 14 with per-K-tile pixel staging (tests)
  const bool no_sl = cfg & 1048576;     // auto: no slice-staged kernel (A/B switch)
  cfg = (cfg & 262144) ? 18 : (cfg & 524288) ? 19 : (cfg & 15);
  const bool sl = cfg == 18 || cfg == 19;
  if ((a.Cs & (sl ? 31 : 63)) || (a.Kpad & 63) || (a.ldx & 7) || (a.ldy & 3) || a.KH * a.KW > 32 || (a.korder & 1) || a.x2 || a.xbn)
    return (int)hipErrorInvalidValue;
  if (a.bnslab) {
    // BatchNorm partial sums (bnslab[M / 256][2][Ngemm]): only the row-block kernels' EP 1 / 2 epilogues
    // carry them (cfg 0 -> 14 / 15 by the channel count); anything else is refused, never silently skipped
    const long M = (long)a.N * a.Ho * a.Wo;
    const int ep = glds_ep_kind(a);
    if (no_fast_ep || no_rowblock || (ep != 1 && ep != 2) || (ep == 1 && a.relu) ||
        (ep == 2 && a.mask_ch != a.Ngemm) || M % 256)
      return (int)hipErrorInvalidValue;
    if (cfg == 0) cfg = a.Ngemm % 256 == 0 ? 14 : 15;
    const bool ok = cfg == 14 ? (pp2h_ok(a) && a.Kpad >= 128) : cfg == 15 ? pp2h128_ok(a) : false;
    if (!ok) return (int)hipErrorInvalidValue;
    const int BCt = cfg == 14 ? 256 : 128;
    const int grid = (int)(M / 256) * (a.Ngemm / BCt);
    if (cfg == 14) {
      if (ep == 1) hipLaunchKernelGGL((igemm_pp2h_kernel<1, 256, true>), dim3(grid), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((igemm_pp2h_kernel<2, 256, true>), dim3(grid), dim3(512), 0, st, a);
    } else {
      if (ep == 1) hipLaunchKernelGGL((igemm_pp2h_kernel<1, 128, true>), dim3(grid), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((igemm_pp2h_kernel<2, 128, true>), dim3(grid), dim3(512), 0, st, a);
    }
    return (int)hipGetLastError();
  }
  if (a.mode == 1 && (a.Cout & 3)) return (int)hipErrorInvalidValue;
  if (cfg == 0) {
    // largest tile that still gives >= 512 workgroups (2 per CU; one 131-147 KB workgroup fits a CU):
    // a microbatched pipeline stage or a small batch has few output pixels at the deep levels
    // (XL bottleneck, 2 images: 2048 pixels x 2048 channels = 64 tiles of 256x256 for 256 CUs)
    const long M = (long)a.N * a.Ho * a.Wo;
    auto grid_of = [&](long bc, long bp) { return ((M + bp - 1) / bp) * (a.Ngemm / bc); };
    // short K (<= 8 K-steps: the transposed convs' forward and up-path dgrads): the persistent kernel,
    // which hides each tile's first-load latency and epilogue behind the neighbouring tile, is 3-9 %
    // faster there (profiles/kbench_glds_shortk_b256_r02.txt, interleaved); otherwise the ping-pong
    // steady-state kernel, 4-10 % faster than the 2-stage 256 x 256 tile on every deep layer and 1.38 vs
    // 1.18 PF on a plain 8192^3 GEMM (profiles/kbench_glds_pp2_b256_r03.txt)
    if (a.Ngemm % 256 == 0 && grid_of(256, 256) >= 512)
      cfg = (a.Kpad <= 8 * 64 && !(a.korder & 2)) ? 8 : 14;
    // 128-output-channel layers on whole rows of <= 128 pixels: the slice-staged 128 x 512 kernel when
    // its tiles fill every CU once
    else if (a.Ngemm % 128 == 0 && !no_sl && !no_rowblock && sl_ok(a) && grid_of(128, 512) >= 256)
      cfg = 18;
    // small grids (pipeline microbatches, small batches): the 128-channel row-block kernel when its
    // 128 x 256 tiles still fill every CU once -- it replaces the 3-stage 128 x 256 kernel (cfg 2) and,
    // at 256..511 of its tiles, the 128 x 128 one (cfg 4: twice the tiles at lower efficiency)
    else if (a.Ngemm % 128 == 0 && grid_of(128, 256) >= 256 && !no_rowblock && pp2h128_ok(a))
      cfg = 15;
    else if (a.Ngemm % 128 == 0 && grid_of(128, 256) >= 512) cfg = 2;
    else if (a.Ngemm % 256 == 0 && grid_of(256, 128) >= 512) cfg = 1;
    else cfg = 4;
  }
  const int ep = no_fast_ep ? 0 : glds_ep_kind(a);
  // launch kernel template K<EP> with the specialised epilogue of this launch
// the same for K<EP, BCv>
#define DPA_EP_LAUNCH2(K, BCv, grid)                                                               \
  do {                                                                                             \
    if (ep == 1) hipLaunchKernelGGL((K<1, BCv>), dim3(grid), dim3(512), 0, st, a);                 \
    else if (ep == 2) hipLaunchKernelGGL((K<2, BCv>), dim3(grid), dim3(512), 0, st, a);            \
    else if (ep == 3) hipLaunchKernelGGL((K<3, BCv>), dim3(grid), dim3(512), 0, st, a);            \
    else hipLaunchKernelGGL((K<0, BCv>), dim3(grid), dim3(512), 0, st, a);                         \
    return (int)hipGetLastError();                                                                 \
  } while (0)
#define DPA_EP_LAUNCH(K, grid)                                                                     \
  do {                                                                                             \
    if (ep == 1) hipLaunchKernelGGL((K<1>), dim3(grid), dim3(512), 0, st, a);                      \
    else if (ep == 2) hipLaunchKernelGGL((K<2>), dim3(grid), dim3(512), 0, st, a);                 \
    else if (ep == 3) hipLaunchKernelGGL((K<3>), dim3(grid), dim3(512), 0, st, a);                 \
    else hipLaunchKernelGGL((K<0>), dim3(grid), dim3(512), 0, st, a);                              \
    return (int)hipGetLastError();                                                                 \
  } while (0)
  const int M = a.N * a.Ho * a.Wo;
  switch (cfg) {
    case 1: if (a.Ngemm % 256) break; return launch_glds<256, 128, 64, 64, 3, 64, true>(a, st);
    case 2: if (a.Ngemm % 128) break; return launch_glds<128, 256, 64, 64, 3, 64, true>(a, st);
    case 4: if (a.Ngemm % 128) break; return launch_glds<128, 128, 64, 32, 4, 64, true>(a, st);
    case 8: if (a.Ngemm % 256) break; return launch_glds_pers<256, 256, 128, 64, 2>(a, st);
    case 14: {
      if (a.Ngemm % 256 || a.Kpad < 128) break;     // the steady loop + peeled tail need S >= 2
      const int grid = ((M + 255) / 256) * (a.Ngemm / 256);
      if (SLP256 && !no_rowblock && slp256_ok(a)) DPA_EP_LAUNCH2(igemm_slp_kernel, 256, grid);
      if (!no_rowblock && pp2h_ok(a)) DPA_EP_LAUNCH(igemm_pp2h_kernel, grid);
      DPA_EP_LAUNCH(igemm_pp2_kernel, grid);
    }
    case 15: {
      if (!pp2h128_ok(a)) break;
      const int grid = (M / 256) * (a.Ngemm / 128);
      if (ep == 1) hipLaunchKernelGGL((igemm_pp2h_kernel<1, 128>), dim3(grid), dim3(512), 0, st, a);
      else if (ep == 2) hipLaunchKernelGGL((igemm_pp2h_kernel<2, 128>), dim3(grid), dim3(512), 0, st, a);
      else if (ep == 3) hipLaunchKernelGGL((igemm_pp2h_kernel<3, 128>), dim3(grid), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((igemm_pp2h_kernel<0, 128>), dim3(grid), dim3(512), 0, st, a);
      return (int)hipGetLastError();
    }
    case 18: {
      if (!sl_ok(a)) break;
      const int grid = (M / 512) * (a.Ngemm / 128);
      if (SL_PINGPONG) DPA_EP_LAUNCH2(igemm_slp_kernel, 128, grid);
      if (ep == 1) hipLaunchKernelGGL((igemm_sl_kernel<1, 128>), dim3(grid), dim3(512), 0, st, a);
      else if (ep == 2) hipLaunchKernelGGL((igemm_sl_kernel<2, 128>), dim3(grid), dim3(512), 0, st, a);
      else if (ep == 3) hipLaunchKernelGGL((igemm_sl_kernel<3, 128>), dim3(grid), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((igemm_sl_kernel<0, 128>), dim3(grid), dim3(512), 0, st, a);
      return (int)hipGetLastError();
    }
    case 19: {
      if (!slp64_ok(a)) break;
      const int grid = (M / 512) * (a.Ngemm / 64);
      DPA_EP_LAUNCH2(igemm_slp_kernel, 64, grid);
    }
    default: break;
  }
#undef DPA_EP_LAUNCH
#undef DPA_EP_LAUNCH2
  return (int)hipErrorInvalidValue;
}
