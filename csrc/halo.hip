// Row-halo variants of the 3x3 convolution kernels for the full-resolution, low-channel layers of
// the UNet (SURVEY §7.4 "Conv kernels on gfx950: MFMA efficiency collapses for C=32/64 full-res
// layers ... you need NHWC tiles that reuse the 3x3 halo from LDS").
//
// The generic kernels (igemm.hip, wgrad.hip) gather every tap separately, so each input pixel is
// fetched 9 times through L2; at 32-64 channels that traffic, not the MFMAs, sets the speed.  Here a
// tile is a run of consecutive pixels of ONE image row; the three input rows it touches (plus one
// pixel of halo on each side) are staged once into LDS and all 9 taps read shifted windows of them:
// 3*(BP+2)/BP ~= 3x the tile instead of 9x.
//
//   igemm_halo : conv3x3 s1 p1 forward / dgrad (mode 0 epilogue: bias, ReLU, ReLU-mask, accumulate)
//                K loop = 32-channel slices of the source (Cs % 32 == 0), 9 taps per slice from LDS.
//   wgrad_halo : conv3x3 weight gradient; the B operand (layer input) is staged as 3 images of
//                34 rows (kh = 0..2, w0-1 .. w0+32) and tap (kh, kw) reads rows kw .. kw+31.
// Both require the tile to stay inside one image row (W % tile == 0), checked on the host.
#include "conv_args.h"

// ------------------------------------------------------------------------------------ igemm_halo
// ROWS output rows per block share one staging of each weight slice (the weights are ~60% of a
// slice's LDS writes at 64-128 output channels, and ds_write bandwidth, not the MFMAs, bounds this
// kernel): ROWS = 2 stages 4 input rows + the weights for twice the MFMAs of ROWS = 1.
// (BC/WC) x (BP/WP) waves: 4, or 8 for the 128-channel tile (one staging of the input rows serves
// all 128 output channels -- the dgrads into 128 channels from 64 have only 2 K-slices to amortise it).
//
// DPP = true: the kernel is LDS-read bound (each pixel fragment feeds only TC MFMAs), so the three
// kw taps of a kernel row share ONE read of the pixel fragments: kw = 1, 2 are the kw = 0 fragments
// shifted by 1, 2 pixels inside each 16-lane row (the MFMA B layout puts pixels along lane & 15),
// built with row_shl DPP moves whose vacated lanes take the head of the next fragment (row_ror):
// TP + 1 ds_read_b128 per (kh, row) instead of 3 * TP.  Measured (kbench --hvar 4 8 5 9 7 10, batch
// 128): within -5..+1% of the LDS-read versions on every UNet shape, so the fragment reads are not
// what bounds this kernel (the per-slice staging barrier is); kept as cfg 8-10, not auto.
// B-fragment lanes l: pixel (l & 15), channel chunk (l >> 4).  Result lane i = cur[i + KW] for
// i + KW < 16, else nxt[i + KW - 16].
template <int KW>
__device__ __forceinline__ bf16x8_t shift_px(const bf16x8_t cur, const bf16x8_t nxt) {
  const u32x4_t c = __builtin_bit_cast(u32x4_t, cur), n = __builtin_bit_cast(u32x4_t, nxt);
  u32x4_t o;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    // row_ror:(16-KW): lane i <- n[(i + KW) & 15]; row_shl:KW: lane i <- c[i + KW], invalid lanes keep old
    const int nr = __builtin_amdgcn_mov_dpp((int)n[d], 0x120 + (16 - KW), 0xf, 0xf, false);
    o[d] = (unsigned)__builtin_amdgcn_update_dpp(nr, (int)c[d], 0x100 + KW, 0xf, 0xf, false);
  }
  return __builtin_bit_cast(bf16x8_t, o);
}

template <int BP, int BC, int WP, int WC, int ROWS = 1, bool DPP = false>
__global__ __launch_bounds__(64 * (BC / WC) * (BP / WP)) void igemm_halo_kernel(IgemmArgs a) {
  constexpr int HR = BP + 2;              // pixels per halo row
  constexpr int PROWS = (ROWS + 2) * HR;  // staged pixel rows (64 B = 32 channels each)
  constexpr int PBYTES = PROWS * 64;
  constexpr int WRB = 9 * 64;             // weight row bytes: 9 taps x 32 channels (576 = 64 mod 256)
  constexpr int NWC = BC / WC, NWP = BP / WP, NT = 64 * NWC * NWP;
  static_assert(NT == 256 || NT == 512, "4 or 8 waves");
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int PCH = PROWS * 4, WCH = BC * 36, CH = PCH + WCH;   // 16-B chunks per slice
  constexpr int L = (CH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char lds[PBYTES + BC * WRB];
  char* const Pimg = lds;
  char* const Wimg = lds + PBYTES;

  const int tilesPerRow = (a.Wo + BP - 1) / BP;     // the last tile of a row may be partial (ragged W)
  const int rowGroups = (a.Ho + ROWS - 1) / ROWS;
  const int npt = a.N * rowGroups * tilesPerRow;
  const int nct = a.Ngemm / BC;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  const int pt = bid / nct, ct = bid - pt * nct;
  const int c0 = ct * BC;
  const int rowid = pt / tilesPerRow;               // n * rowGroups + row group (uniform)
  const int w0 = (pt - rowid * tilesPerRow) * BP;
  const int n = rowid / rowGroups, h = (rowid - n * rowGroups) * ROWS;
  const long m0 = ((long)n * a.Ho + h) * a.Wo + w0;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid / NWC, wc = wid - wp * NWC;
  // one image per block: 64-bit image base, 32-bit offsets inside it (whole batch in one launch)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long)n * a.Hs * a.Ws * a.ldx), 0, (int)a.ximg, 0x00020000);

  f32x4_t acc[ROWS][TC][TP];
#pragma unroll
  for (int rr = 0; rr < ROWS; ++rr)
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) acc[rr][ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // per-thread staging plan, computed once: global byte offsets (slice 0) + LDS offsets
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  unsigned goff[L];
  int lsto[L];
  bool isw[L], gok[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int c = tid + j * NT;
    isw[j] = c >= PCH;
    if (c < PCH) {
      const int row = c >> 2, cc = c & 3;
      const int kh = row / HR, col = row - kh * HR;
      const int ih = h + kh - 1, iw = w0 + col - 1;
      gok[j] = ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
      goff[j] = (unsigned)(((ih * a.Ws + iw) * a.ldx + cc * 8) * 2);
      lsto[j] = row * 64 + (swz_nk<32>(row, cc) << 4);
    } else {
      const int cw = c - PCH, r = cw / 36, k = cw - r * 36;     // k = tap*4 + chunk
      const int tap = k >> 2, cc = k & 3;
      gok[j] = c < CH;
      goff[j] = (unsigned)(((c0 + r) * a.Kpad + tap * a.Cs + cc * 8) * 2);
      lsto[j] = c < CH ? PBYTES + r * WRB + tap * 64 + (swz_nk<32>(r, cc) << 4) : -1;
    }
  }
  u32x4_t reg[L];
  auto sload = [&](int s) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      if (isw[j]) {
        if (gok[j]) reg[j] = __builtin_amdgcn_raw_buffer_load_b128(wr, goff[j] + s * 64, 0, 0);
      } else {
        reg[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, gok[j] ? goff[j] + s * 64 : 0x80000000u, 0, 0);
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int j = 0; j < L; ++j)
      if (lsto[j] >= 0) *reinterpret_cast<u32x4_t*>(lds + lsto[j]) = reg[j];
  };

  // slices of 32 source channels; slice s+1 is fetched into registers while slice s computes
  const int S = a.Cs / 32;
  sload(0);
  for (int s = 0; s < S; ++s) {
    if (s > 0) __syncthreads();          // slice s-1 fully consumed
    sstore();
    __syncthreads();
    if (s + 1 < S) sload(s + 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DPP) {
      const int chunk = lane >> 4;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        bf16x8_t af[3][TC];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int ic = 0; ic < TC; ++ic) {
            const int r = wc * WC + ic * 16 + (lane & 15);
            af[kw][ic] = *reinterpret_cast<const bf16x8_t*>(Wimg + r * WRB + (kh * 3 + kw) * 64 +
                                                             (swz_nk<32>(r, chunk) << 4));
          }
#pragma unroll
        for (int rr = 0; rr < ROWS; ++rr) {
          bf16x8_t fr[TP + 1];   // fr[TP]: only its lanes 0-1 of each row (the right halo) are used
#pragma unroll
          for (int ip = 0; ip <= TP; ++ip) {
            const int r = (kh + rr) * HR + wp * WP + ip * 16 + (lane & 15);
            fr[ip] = *reinterpret_cast<const bf16x8_t*>(Pimg + r * 64 + (swz_nk<32>(r, chunk) << 4));
          }
          bf16x8_t b1[TP], b2[TP];
#pragma unroll
          for (int ip = 0; ip < TP; ++ip) {
            b1[ip] = shift_px<1>(fr[ip], fr[ip + 1]);
            b2[ip] = shift_px<2>(fr[ip], fr[ip + 1]);
          }
          // kw outer: consecutive MFMAs hit different accumulators
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[rr][ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][ic], fr[ip], acc[rr][ic][ip], 0, 0, 0);
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[rr][ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][ic], b1[ip], acc[rr][ic][ip], 0, 0, 0);
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[rr][ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2][ic], b2[ip], acc[rr][ic][ip], 0, 0, 0);
        }
      }
    } else
    // ---- 9 taps x (TC x TP) MFMAs from LDS
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - kh * 3;
      const int chunk = lane >> 4;
      bf16x8_t af[TC], bfr[TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        const int r = wc * WC + ic * 16 + (lane & 15);
        af[ic] = *reinterpret_cast<const bf16x8_t*>(Wimg + r * WRB + tap * 64 + (swz_nk<32>(r, chunk) << 4));
      }
#pragma unroll
      for (int rr = 0; rr < ROWS; ++rr) {
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) {
          const int r = (kh + rr) * HR + wp * WP + ip * 16 + (lane & 15) + kw;
          bfr[ip] = *reinterpret_cast<const bf16x8_t*>(Pimg + r * 64 + (swz_nk<32>(r, chunk) << 4));
        }
#pragma unroll
        for (int ic = 0; ic < TC; ++ic)
#pragma unroll
          for (int ip = 0; ip < TP; ++ip)
            acc[rr][ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[rr][ic][ip], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue (mode 0): bias, ReLU, ReLU-backward mask, accumulate; 8-byte bf16 stores
#pragma unroll
  for (int rr = 0; rr < ROWS; ++rr) {
  if (h + rr >= a.Ho) break;
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    if (w0 + wp * WP + ip * 16 + (lane & 15) >= a.Wo) continue;     // ragged last tile
    const long m = m0 + (long)rr * a.Wo + wp * WP + ip * 16 + (lane & 15);
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int co = c0 + wc * WC + ic * 16 + 4 * (lane >> 4);
      float v0 = acc[rr][ic][ip][0], v1 = acc[rr][ic][ip][1], v2 = acc[rr][ic][ip][2], v3 = acc[rr][ic][ip][3];
      if (a.bias) {
        const float* b = a.bias + co;
        v0 += b[0]; v1 += b[1]; v2 += b[2]; v3 += b[3];
      }
      if (a.relu) {
        v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3);
      }
      if (a.mask && co < a.mask_ch) {
        const uint2 mk = *reinterpret_cast<const uint2*>(a.mask + m * a.ldm + co);
        v0 = lo_bf(mk.x) > 0.f ? v0 : 0.f;
        v1 = hi_bf(mk.x) > 0.f ? v1 : 0.f;
        v2 = lo_bf(mk.y) > 0.f ? v2 : 0.f;
        v3 = hi_bf(mk.y) > 0.f ? v3 : 0.f;
      }
      uint2* dst = reinterpret_cast<uint2*>(a.y + m * a.ldy + co);
      if (a.accumulate) {
        const uint2 o = *dst;
        v0 += lo_bf(o.x); v1 += hi_bf(o.x); v2 += lo_bf(o.y); v3 += hi_bf(o.y);
      }
      const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
      if (!split_store(a, (unsigned)m, co, packed)) *reinterpret_cast<u32x2_t*>(dst) = packed;
    }
  }
  }
}

template <int BP, int BC, int WP, int WC, int ROWS = 1, bool DPP = false>
static int launch_igemm_halo(const IgemmArgs& a, hipStream_t st) {
  const int grid = a.N * ((a.Ho + ROWS - 1) / ROWS) * ((a.Wo + BP - 1) / BP) * (a.Ngemm / BC);
  hipLaunchKernelGGL((igemm_halo_kernel<BP, BC, WP, WC, ROWS, DPP>), dim3(grid), dim3(64 * (BC / WC) * (BP / WP)), 0, st, a);
  return (int)hipGetLastError();
}

// Returns hipErrorInvalidValue (nothing launched) when the shape is not eligible; the caller then
// uses dpa_igemm.  cfg: 0 auto, 1: 256x32, 2: 128x64, 3: 128x32, 4: 128x64 two rows, 5: 128x32 two rows,
// 6: 128x128 two rows 8 waves (4 ch x 2 px), 7: 128x128 two rows 8 waves (2 ch x 4 px),
// 8 / 9 / 10: cfg 4 / 5 / 7 with DPP-shifted pixel fragments (one LDS read per kernel row)
// a row of W pixels in tiles of bp: whole tiles, or a partial last tile that keeps >= 85 % of the
// tile pixels useful (640x960: widths 960 / 480 / 240 / 120 in 128-pixel tiles are 94 % useful)
// the per-image buffer binding (IgemmArgs::ximg) must cover one whole image of x: a short extent would
// read zeros past it instead of failing
static bool ximg_ok(const IgemmArgs& a) {
  // a dual input (a.x2) holds Cs / 2 channels per tensor, each tensor with this extent
  return (long)a.ximg >= ((long)a.Hs * a.Ws - 1) * a.ldx * 2 + (long)(a.x2 ? a.Cs / 2 : a.Cs) * 2;
}

static bool tiles_ok(int W, int bp) {
  const int t = (W + bp - 1) / bp;
  return W >= 16 && (W % bp == 0 || W * 100 >= 85 * t * bp);
}

DPA_API int dpa_igemm_halo(const IgemmArgs* args, int cfg, hipStream_t st) {
  const IgemmArgs& a = *args;
  if (a.mode != 0 || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || (a.Cs % 32) || (a.ldx & 7) ||
      (a.ldy & 3) || a.Hs != a.Ho || a.Ws != a.Wo || a.Kpad < 9 * a.Cs || !ximg_ok(a) || a.x2 || a.xbn)
    return (int)hipErrorInvalidValue;
  if (cfg == 0) {
    if (a.Ngemm == 32 && tiles_ok(a.Wo, 256)) cfg = 1;
    // two output rows per block: 20-25% faster than one row on every 512^2 UNet shape
    // (profiles/kbench_b32_512.txt halo.c4/c5 vs c2/c3)
    else if (a.Ngemm % 64 == 0 && a.Ngemm <= 128 && tiles_ok(a.Wo, 128)) cfg = 4;
    else if (a.Ngemm % 32 == 0 && a.Ngemm <= 64 && tiles_ok(a.Wo, 128)) cfg = 5;
    else return (int)hipErrorInvalidValue;
  }
  switch (cfg) {
    case 1: if (!tiles_ok(a.Wo, 256) || a.Ngemm % 32) break; return launch_igemm_halo<256, 32, 64, 32>(a, st);
    case 2: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 64, 32>(a, st);
    case 3: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 32) break; return launch_igemm_halo<128, 32, 32, 32>(a, st);
    case 4: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 64, 32, 2>(a, st);
    case 5: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 32) break; return launch_igemm_halo<128, 32, 32, 32, 2>(a, st);
    case 6: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 128) break; return launch_igemm_halo<128, 128, 64, 32, 2>(a, st);
    case 7: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 128) break; return launch_igemm_halo<128, 128, 32, 64, 2>(a, st);
    case 8: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 64, 32, 2, true>(a, st);
    case 9: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 32) break; return launch_igemm_halo<128, 32, 32, 32, 2, true>(a, st);
    case 10: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 128) break; return launch_igemm_halo<128, 128, 32, 64, 2, true>(a, st);
    // (cfg 13 is 4-5 % faster than cfg 4 alone at 256^2 128 -> 64, 2972 vs 3113 us at b256, but the step is 0.4 %
    // slower with it: 3158 / 3165 vs 3171 / 3183 img/s on one box, profiles/kbench_slp64_halo_r06.txt -- not auto)
    // more output rows per staging of the weight slice (the weights are half of the staged bytes at 64
    // output channels): 3 rows x 4 waves / 8 waves (two blocks per CU), 4 rows x 8 waves, 256 x 2 rows x 8 waves
    case 11: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 64, 32, 3>(a, st);
    case 12: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 32, 32, 3>(a, st);
    case 13: if (!tiles_ok(a.Wo, 128) || a.Ngemm % 64) break; return launch_igemm_halo<128, 64, 32, 32, 4>(a, st);
    case 14: if (!tiles_ok(a.Wo, 256) || a.Ngemm % 64) break; return launch_igemm_halo<256, 64, 64, 32, 2>(a, st);
    default: break;
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------ wgrad_halo
// conv3x3 weight gradient, pixel chunks of 32 inside one row.  out[tap][m][n] as in wgrad.hip.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void wgrad_halo_kernel(WgradArgs a) {
  constexpr int NWN = BN / WN, NW = (BM / WM) * NWN, NT = 64 * NW;
  constexpr int CPRA = BM / 8, CPRB = BN / 8, RBA = BM * 2, RBB = BN * 2;
  constexpr int BR = 34;                                   // B rows per kh image
  constexpr int IMGA = 32 * RBA, IMGB = BR * RBB;
  constexpr int CHA = 32 * CPRA, CH = CHA + 3 * BR * CPRB;
  constexpr int L = (CH + NT - 1) / NT;
  constexpr int TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) char lds[IMGA + 3 * IMGB];

  const int nmt = a.M / BM;
  const int nnt = (a.Nc + BN - 1) / BN;
  const int tiles = nmt * nnt;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const long P = (long)a.N * a.Hg * a.Wg;
  const long pbeg = (long)split * a.pix_per_split;
  long pend = pbeg + a.pix_per_split;
  if (pend > P) pend = P;
  const int nst = (int)((pend - pbeg) / 32);            // P % 32 == 0 (host check)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid - wm * NWN;
  const bool do_bias = a.bslab != nullptr && nt == 0;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)a.abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)a.bbytes, 0x00020000);

  u32x4_t reg[L];
  auto gload = [&](int st) {
    const int p0 = (int)(pbeg + (long)st * 32);           // 32 pixels of one row
    const int hw = a.Hg * a.Wg;
    const int n = p0 / hw, rem = p0 - n * hw, h = rem / a.Wg, w0 = rem - h * a.Wg;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int c = tid + j * NT;
      if (c < CH) {
        if (c < CHA) {
          const int r = c / CPRA, cc = c - r * CPRA;
          const int ch = m0 + cc * 8;
          const bool ok = ch < a.M;
          const unsigned off = ok ? (unsigned)((((n * a.HA + h) * a.WA + w0 + r) * a.lda + ch) * 2) : 0x80000000u;
          reg[j] = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
        } else {
          const int cl = c - CHA, img = cl / (BR * CPRB), rr = cl - img * (BR * CPRB);
          const int r = rr / CPRB, cc = rr - r * CPRB;
          const int ih = h + img - 1, iw = w0 + r - 1, ch = n0 + cc * 8;
          const bool ok = ih >= 0 && ih < a.HB && iw >= 0 && iw < a.WB && ch < a.Nc;
          const unsigned off = ok ? (unsigned)((((n * a.HB + ih) * a.WB + iw) * a.ldb + ch) * 2) : 0x80000000u;
          reg[j] = __builtin_amdgcn_raw_buffer_load_b128(br, off, 0, 0);
        }
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int c = tid + j * NT;
      if (c < CH) {
        if (c < CHA) {
          const int r = c / CPRA, cc = c - r * CPRA;
          *reinterpret_cast<u32x4_t*>(lds + r * RBA + ((cc ^ swz_kk<RBA>(r)) << 4)) = reg[j];
        } else {
          const int cl = c - CHA, img = cl / (BR * CPRB), rr = cl - img * (BR * CPRB);
          const int r = rr / CPRB, cc = rr - r * CPRB;
          *reinterpret_cast<u32x4_t*>(lds + IMGA + img * IMGB + r * RBB + ((cc ^ swz_kk<RBB>(r)) << 4)) = reg[j];
        }
      }
    }
  };

  f32x4_t acc[9][TM][TN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[t][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  if (nst > 0) {
    gload(0);
    lstore();
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) gload(st + 1);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8_t af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = tr_frag<RBA>(lds, wm * WM + i * 16, lane);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t - kh * 3;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bf16x8_t bf = tr_frag<RBB>(lds + IMGA + kh * IMGB, wn * WN + j * 16, lane, kw);
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[t][i][j], 0, 0, 0);
      }
    }
    if (do_bias && tid < BM) {
      const int ch = tid >> 3, e = tid & 7;
      for (int r = 0; r < 32; ++r)
        bsum += bf2f(*reinterpret_cast<const bf16_t*>(lds + r * RBA + ((ch ^ swz_kk<RBA>(r)) << 4) + e * 2));
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (st + 1 < nst) {
      lstore();
      __syncthreads();
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nn = n0 + wn * WN + j * 16 + (lane & 15);
        if (nn >= a.Nc) continue;
        const int mb = m0 + wm * WM + i * 16 + 4 * (lane >> 4);
        float* dst = a.slab + (((long)split * 9 + t) * a.M + mb) * a.Nc + nn;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(long)r * a.Nc] = acc[t][i][j][r];
      }
  if (do_bias && tid < BM) a.bslab[(long)split * a.M + m0 + tid] = bsum;
}

template <int BM, int BN, int WM, int WN>
static int launch_wgrad_halo(const WgradArgs& a, hipStream_t st) {
  const int tiles = (a.M / BM) * ((a.Nc + BN - 1) / BN);
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  hipLaunchKernelGGL((wgrad_halo_kernel<BM, BN, WM, WN>), dim3(tiles * a.splits), dim3(NT), 0, st, a);
  return (int)hipGetLastError();
}

// cfg: 1: 32x32 (4 waves of 16x16)  2: 64x32  3: 32x64  4: 64x64;  0 = auto
DPA_API int dpa_wgrad_halo(const WgradArgs* args, int cfg, hipStream_t st) {
  const WgradArgs& a = *args;
  if ((a.M & 31) || (a.lda & 7) || (a.ldb & 7) || (a.pix_per_split & 31) || (a.Wg & 31) || a.splits < 1 || a.s != 1 ||
      a.pad != 1 || a.KW != 3 || a.HA != a.Hg || a.WA != a.Wg || a.HB != a.Hg || a.WB != a.Wg || (a.Nc & 31))
    return (int)hipErrorInvalidValue;
  if (cfg == 0) cfg = (a.M % 64 == 0) ? (a.Nc % 64 == 0 ? 4 : 2) : (a.Nc % 64 == 0 ? 3 : 1);
  switch (cfg) {
    case 1: return launch_wgrad_halo<32, 32, 16, 16>(a, st);
    case 2: if (a.M % 64) break; return launch_wgrad_halo<64, 32, 32, 16>(a, st);
    case 3: return launch_wgrad_halo<32, 64, 16, 32>(a, st);
    case 4: if (a.M % 64) break; return launch_wgrad_halo<64, 64, 32, 32>(a, st);
    default: break;
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------ igemm_stream
// Row-streaming conv3x3 (s1 p1) for Ngemm, Cs in {32, 64}: one block owns an image column strip
// [w0, w0+BP) x rows [h0, h0+RH) and ALL output channels.  The packed weights stay resident in LDS
// for the block's lifetime; input rows stream through a 4-slot LDS ring (3 rows in use + 1 being
// prefetched), so every input pixel is read from HBM ~once ((RH+2)/RH x (BP+2)/BP) and every
// output pixel written once: the layer runs near streaming bandwidth instead of gathering each
// pixel 9 times through L2.
// At K = 9*32 an output tile gets only 9 MFMAs, so the VALU work around them (addresses, epilogue)
// decides the speed: every per-lane byte offset (loader, LDS fragments, output, mask) is computed
// once per block in 32 bits, rows only add a wave-uniform scalar, and all global traffic goes
// through buffer instructions (32-bit offsets, range-checked zero padding, no 64-bit math).
// LDS images are [.. ][rows][32 channels] 64-B-row nk images (swz_nk<32>, conflict-free).
// EPI: 0 plain epilogue, 1 + fused 2x2 max-pool (and window codes), 2 split output (a.y2), 3 fused
// head, 4/5 BatchNorm partials (forward / backward), 6 plain forward (no mask / accumulate); the
// pool registers and branches exist only in the instantiations that use them.
template <int BP, int NG, int CS, int RH, int WCS, int EPI>
__global__ __launch_bounds__(256 * WCS) void igemm_stream_kernel(IgemmArgs a) {
  constexpr int NT = 256 * WCS;               // 4 waves along the pixels x WCS along the channels
  constexpr int HR = BP + 2;                  // pixels per staged input row
  constexpr int KS = CS / 32;                 // 32-channel slices
  constexpr int WBYTES = 9 * KS * NG * 64;    // [tap][ks][NG][32]
  constexpr int SLOT = KS * HR * 64;          // one input row: [ks][HR][32]
  constexpr int WP = BP / 4, TP = WP / 16, WCN = NG / WCS, TC = WCN / 16;
  static_assert(TP >= 1 && TC >= 1, "tile");
  constexpr int RCH = KS * HR * 4;            // 16-B chunks per input row
  // dual input (KS == 2, a.x2): channels 32-63 come from a second dense tensor.  Its chunks are laid
  // out plane-major with each plane padded to whole waves, so every wave's loads use ONE buffer
  // resource; for every strip width this needs no more load slots than the interleaved mapping
  constexpr int PL = (HR * 4 + 63) / 64 * 64;
  constexpr int LR0 = (RCH + NT - 1) / NT, LR1 = KS == 2 ? (2 * PL + NT - 1) / NT : 0;
  constexpr int LR = LR0 > LR1 ? LR0 : LR1;
  __shared__ __attribute__((aligned(16))) char lds[WBYTES + 4 * SLOT];
  char* const Wimg = lds;
  char* const Ring = lds + WBYTES;

  const int stripsW = (a.Wo + BP - 1) / BP;                // the last strip may be partial (ragged W)
  const int segsH = (a.Ho + RH - 1) / RH;
  const int bid = blockIdx.x;                               // streaming: no L2 reuse to chase
  const int n = bid / (segsH * stripsW);
  const int rem = bid - n * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * BP;
  const int h0 = hs * RH;
  const int tid = threadIdx.x, lane = tid & 63, wp = (tid >> 6) & 3, wc = tid >> 8;
  // one image per block: 64-bit image bases, 32-bit offsets inside the image (any batch size)
  const long opix = (long)n * a.Ho * a.Wo;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long)n * a.Hs * a.Ws * a.ldx), 0, (int)a.ximg, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + opix * a.ldy), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.mask ? a.mask + opix * a.ldm : a.y), 0, 0x7fffffff, 0x00020000);
  const bool dual = KS == 2 && a.x2 != nullptr;
  const __amdgpu_buffer_rsrc_t x2r = dual ? __builtin_amdgcn_make_buffer_rsrc((void*)(a.x2 + (long)n * a.Hs * a.Ws * a.ldx), 0, (int)a.ximg, 0x00020000) : xr;

  // resident weights: packed [NG][Kpad] with k = tap*CS + ci
  for (int c = tid; c < 9 * KS * NG * 4; c += NT) {
    const int cc = c & 3, row = (c >> 2) % NG, tk = (c >> 2) / NG;       // tk = tap*KS + ks
    const int tap = tk / KS, ks = tk - tap * KS;
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(a.w + (long)row * a.Kpad + tap * CS + ks * 32 + cc * 8);
    *reinterpret_cast<u32x4_t*>(Wimg + (tk * NG + row) * 64 + (swz_nk<32>(row, cc) << 4)) = v;
  }
  // ---- per-thread loader constants (row-invariant)
  unsigned loff[LR];
  int lsto[LR];
  bool lok[LR], lpl[LR];      // lpl: this wave's chunk j comes from x2 (wave-uniform)
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
  for (int j = 0; j < LR; ++j) {
    const int c = tid + j * NT;
    int cc = c & 3, px = (c >> 2) % HR, ks = (c >> 2) / HR, xch = ks * 32;
    bool live = c < RCH;
    lpl[j] = false;
    if (dual) {
      ks = (wv * 64 + j * NT) / PL;
      const int cl = c - ks * PL;
      live = ks < 2 && cl < HR * 4;
      cc = cl & 3, px = cl >> 2, xch = 0;
      lpl[j] = ks == 1;
    }
    const int iw = w0 + px - 1;
    lok[j] = live && iw >= 0 && iw < a.Ws;
    loff[j] = (unsigned)((iw * a.ldx + xch + cc * 8) * 2);
    lsto[j] = live ? (ks * HR + px) * 64 + (swz_nk<32>(px, cc) << 4) : -1;
  }
  const unsigned rowbytes_x = (unsigned)(a.Ws * a.ldx * 2);
  // BN-on-load (EPI 4, a.xbn): the input is the PRE-BatchNorm output z of the layer below and the
  // loader stores y = relu(z * xbn[c] + xbn[CS + c]) into the ring -- bn_apply's exact arithmetic,
  // so the layer below never writes y (its BN+ReLU pass over HBM disappears); padding stays zero.
  // With a dual input only x (channels < 32) is a BN input; x2 is stored as loaded
  constexpr bool XBN = EPI == 4;
  __shared__ float xbc[XBN ? 2 * CS : 1];
  const bool xbn = XBN && a.xbn != nullptr;
  if constexpr (XBN) {
    if (xbn) {
      // a dual input's coefficients cover x only: [scale 32 | shift 32] -> xbc[0, 32) and xbc[CS, CS + 32)
      for (int i = tid; i < (dual ? 64 : 2 * CS); i += NT) xbc[dual && i >= 32 ? CS + i - 32 : i] = a.xbn[i];
      __syncthreads();
    }
  }
  // two register sets: a row's loads are issued two rows before it is stored into the ring
  struct RowRegs {
    u32x4_t v[LR];
    bool rok;
  };
  RowRegs setA, setB;
  auto rload = [&](int ih, RowRegs& R) {
    const bool rok = ih >= 0 && ih < a.Hs;                     // wave-uniform
    R.rok = rok;
    const unsigned rbase = (unsigned)ih * rowbytes_x;
#pragma unroll
    for (int j = 0; j < LR; ++j) {
      const unsigned off = (rok && lok[j]) ? rbase + loff[j] : 0x80000000u;
      R.v[j] = __builtin_amdgcn_raw_buffer_load_b128(lpl[j] ? x2r : xr, off, 0, 0);
    }
  };
  // BN-on-load transform of a loaded row (registers only).  The row loop runs it right after its
  // MFMAs, inside the same scheduling region, so the VALU work overlaps the MFMA drain instead of
  // sitting between the epilogue and the ring store.
  auto xform = [&](RowRegs& R) {
    if constexpr (XBN) {
      if (xbn && R.rok) {
#pragma unroll
        for (int j = 0; j < LR; ++j) {
          if (!lok[j] || lpl[j]) continue;     // dual input: x2 (plane 1) is read as is
          // chunk j's first channel: slice ks (plane for a dual input) * 32 + (c & 3) * 8
          const int c = tid + j * NT;
          const int cb = (dual ? (lpl[j] ? 32 : 0) : ((c >> 2) / HR) * 32) + (c & 3) * 8;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float2 sc = *reinterpret_cast<const float2*>(xbc + cb + 2 * k);
            const float2 sh = *reinterpret_cast<const float2*>(xbc + CS + cb + 2 * k);
            R.v[j][k] = pack_bf2(fmaxf(fmaf(lo_bf(R.v[j][k]), sc.x, sh.x), 0.f),
                                 fmaxf(fmaf(hi_bf(R.v[j][k]), sc.y, sh.y), 0.f));
          }
        }
      }
    }
  };
  auto rstore = [&](int slot, const RowRegs& R) {
#pragma unroll
    for (int j = 0; j < LR; ++j)
      if (lsto[j] >= 0) *reinterpret_cast<u32x4_t*>(Ring + slot * SLOT + lsto[j]) = R.v[j];
  };
  // ---- per-lane LDS fragment offsets and epilogue constants
  const int chunk = lane >> 4;
  int aoff[TC];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic) {
    const int row = wc * WCN + ic * 16 + (lane & 15);
    aoff[ic] = row * 64 + (swz_nk<32>(row, chunk) << 4);
  }
  int boff[TP][3];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int px = wp * WP + ip * 16 + (lane & 15) + kw;
      boff[ip][kw] = px * 64 + (swz_nk<32>(px, chunk) << 4);
    }
  float bias[TC][4];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[ic][e] = a.bias ? a.bias[wc * WCN + ic * 16 + 4 * chunk + e] : 0.f;
  unsigned yl[TP], ml[TP];
  bool pv[TP];                  // pixel inside the row (false only in a ragged last strip)
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int pl = w0 + wp * WP + ip * 16 + (lane & 15);
    pv[ip] = pl < a.Wo;
    // out-of-row pixels: an offset past the range check -> their stores are dropped, mask loads read 0
    yl[ip] = pv[ip] ? (unsigned)((pl * a.ldy + wc * WCN + 4 * chunk) * 2) : 0x80000000u;
    ml[ip] = pv[ip] ? (unsigned)((pl * a.ldm + wc * WCN + 4 * chunk) * 2) : 0x80000000u;
  }
  // forward epilogues (pool, head, BN statistics, plain forward EPI 6) never mask or accumulate: with
  // those paths compiled out, no epilogue load shares the in-order vmcnt queue with the two-rows-ahead
  // prefetch, which a runtime-dead mask load otherwise forced to drain every row (s_waitcnt vmcnt(0))
  constexpr bool MAYMASK = EPI == 0 || EPI == 2 || EPI == 5;
  const bool has_mask = MAYMASK && a.mask != nullptr;
  // fused 2x2 max-pool (encoder conv2 -> next level input): even rows keep their horizontally
  // max-reduced values in registers, odd rows finish the window and write the pooled pixel.
  constexpr bool do_pool = EPI == 1;
  const long ppix = (long)n * (a.Ho >> 1) * (a.Wo >> 1);
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)(do_pool ? a.pool + ppix * a.ldp : a.y), 0, 0x7fffffff, 0x00020000);
  constexpr int PT = do_pool ? TP : 1, PC = do_pool ? TC : 1;
  u32x2_t ptop[PT][PC], ptop2[PT][PC];       // even row of the window (stored bf16): own / partner pixel

  // fused segmentation head (EPI 3): segmap weights of this lane's channels, BCE/Dice partials
  constexpr bool do_head = EPI == 3;
  float hwv[do_head ? TC : 1][4];
  float hsum[4] = {0.f, 0.f, 0.f, 0.f};
  // the head's target of each output pixel of a row is loaded at the START of the row (issued before the
  // row prefetch, like the mask): loaded in the epilogue its latency was exposed once per row
  const __amdgpu_buffer_rsrc_t tgr = __builtin_amdgcn_make_buffer_rsrc((void*)(do_head ? a.tgt + opix : (const float*)a.y),
                                                                       0, do_head ? a.Ho * a.Wo * 4 : 0, 0x00020000);
  if constexpr (do_head) {
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) hwv[ic][e] = a.hw[wc * WCN + ic * 16 + 4 * chunk + e];
  }

  // fused BatchNorm statistics: EPI 4 (forward, conv -> BN) sum z, sum z^2 of the stored output;
  // EPI 5 (backward, dgrad with the ReLU mask y = relu(bn(z)) of the BN layer below) sum g, sum g*y
  // of the stored masked gradient -- with sum g*(z - mean) = (sum g*y - beta sum g) / (gamma invstd)
  // on the mask's support, the BN backward needs no statistics pass over (g, z)
  constexpr bool do_bn = EPI == 4 || EPI == 5;
  float bsum[do_bn ? TC : 1][4], bsq[do_bn ? TC : 1][4];
  if constexpr (do_bn) {
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) bsum[ic][e] = bsq[ic][e] = 0.f;
  }

  // prologue: input rows h0-1, h0, h0+1 -> slots 0, 1, 2; row h0+2 in flight
  const int nrows = min(RH, a.Ho - h0);
#pragma unroll 1
  for (int j = 0; j < 3; ++j) {
    rload(h0 - 1 + j, setA);
    xform(setA);
    rstore(j, setA);
  }
  if (nrows > 1) rload(h0 + 2, setA);
  __syncthreads();

  // row r: `cur` holds row h0+r+2 (issued during row r-1); row h0+r+3 is issued into `nxt`
  auto row = [&](int r, RowRegs& cur, RowRegs& nxt) {
    const int orow = n * a.Ho + h0 + r;                        // global output row (pointer-math epilogues)
    const unsigned ybase = (unsigned)(h0 + r) * (unsigned)(a.Wo * a.ldy * 2);   // inside this image
    const unsigned mbase = (unsigned)(h0 + r) * (unsigned)(a.Wo * a.ldm * 2);
    // ReLU-mask of this output row: issued before the MFMAs so its latency hides under them, and
    // before the row prefetch, so waiting for it does not wait for the prefetch (in-order vmcnt)
    u32x2_t mk[TP][TC];
    if (has_mask) {
#pragma unroll
      for (int ip = 0; ip < TP; ++ip)
#pragma unroll
        for (int ic = 0; ic < TC; ++ic)
          mk[ip][ic] = (wc * WCN + ic * 16 < a.mask_ch) ? __builtin_amdgcn_raw_buffer_load_b64(mr, mbase + ml[ip] + ic * 32, 0, 0)
                                             : u32x2_t{0x3f803f80u, 0x3f803f80u};
    }
    float ttp[do_head ? TP : 1];
    if constexpr (do_head) {
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const unsigned px = (unsigned)((h0 + r) * a.Wo + w0 + wp * WP + ip * 16 + (lane & 15));
        ttp[ip] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(tgr, (chunk == 0 && pv[ip]) ? px * 4u : 0x80000000u, 0, 0));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (r + 2 < nrows) rload(h0 + r + 3, nxt);
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t acc[TC][TP];
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const char* S = Ring + ((r + kh) & 3) * SLOT;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int tk = (kh * 3 + kw) * KS + ks;
          bf16x8_t af[TC], bfr[TP];
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
            af[ic] = *reinterpret_cast<const bf16x8_t*>(Wimg + tk * NG * 64 + aoff[ic]);
#pragma unroll
          for (int ip = 0; ip < TP; ++ip)
            bfr[ip] = *reinterpret_cast<const bf16x8_t*>(S + ks * HR * 64 + boff[ip][kw]);
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
        }
      }
    }
    if (r + 1 < nrows) xform(cur);      // BN-on-load of the row stored below (overlaps the MFMA drain)
    // epilogue for output row h0 + r: 32-bit buffer offsets = per-lane constant + uniform row base
#pragma unroll
    for (int ip = 0; ip < TP; ++ip) {
      float hdot = 0.f;
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        float v0 = acc[ic][ip][0] + bias[ic][0], v1 = acc[ic][ip][1] + bias[ic][1];
        float v2 = acc[ic][ip][2] + bias[ic][2], v3 = acc[ic][ip][3] + bias[ic][3];
        if (a.relu) {
          v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3);
        }
        if (has_mask) {
          v0 = lo_bf(mk[ip][ic].x) > 0.f ? v0 : 0.f;
          v1 = hi_bf(mk[ip][ic].x) > 0.f ? v1 : 0.f;
          v2 = lo_bf(mk[ip][ic].y) > 0.f ? v2 : 0.f;
          v3 = hi_bf(mk[ip][ic].y) > 0.f ? v3 : 0.f;
        }
        const unsigned yo = ybase + yl[ip] + ic * 32;
        if (MAYMASK && a.accumulate) {
          const u32x2_t o = __builtin_amdgcn_raw_buffer_load_b64(yr, yo, 0, 0);
          v0 += lo_bf(o.x); v1 += hi_bf(o.x); v2 += lo_bf(o.y); v3 += hi_bf(o.y);
        }
        const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
        if constexpr (EPI == 2) {
          if (pv[ip])
            split_store(a, (unsigned)(orow * a.Wo + w0 + wp * WP + ip * 16 + (lane & 15)), wc * WCN + ic * 16 + 4 * chunk,
                        packed);
        } else
          __builtin_amdgcn_raw_buffer_store_b64(packed, yr, yo, 0, 0);
        if constexpr (do_bn) {     // statistics of the STORED bf16 values, like a separate pass
          const float pz = pv[ip] ? 1.f : 0.f;                  // out-of-row pixels add nothing
          const float q[4] = {pz * lo_bf(packed.x), pz * hi_bf(packed.x), pz * lo_bf(packed.y), pz * hi_bf(packed.y)};
          float f[4] = {q[0], q[1], q[2], q[3]};
          if constexpr (EPI == 5) {
            f[0] = lo_bf(mk[ip][ic].x); f[1] = hi_bf(mk[ip][ic].x); f[2] = lo_bf(mk[ip][ic].y); f[3] = hi_bf(mk[ip][ic].y);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bsum[ic][e] += q[e];
            bsq[ic][e] = fmaf(q[e], f[e], bsq[ic][e]);
          }
        }
        if constexpr (do_head) {   // the head sees the STORED bf16 values, like a separate pass would
          hdot = fmaf(lo_bf(packed.x), hwv[ic][0], hdot);
          hdot = fmaf(hi_bf(packed.x), hwv[ic][1], hdot);
          hdot = fmaf(lo_bf(packed.y), hwv[ic][2], hdot);
          hdot = fmaf(hi_bf(packed.y), hwv[ic][3], hdot);
        }
        if constexpr (do_pool) {
          // pool the STORED bf16 values (identical to max-pooling the tensor afterwards).  They are
          // post-ReLU (>= 0; the host requires relu with pool), so the window max and argmax run on
          // the packed channel pairs as 16-bit integers.  Even lanes hold pixel w (left), their
          // xor-1 partner pixel w+1 (right).
          const u32x2_t pq = u32x2_t{(unsigned)__shfl_xor((int)packed.x, 1, 64), (unsigned)__shfl_xor((int)packed.y, 1, 64)};
          const int hrow = h0 + r;
          if ((hrow & 1) == 0) {
            ptop[ip][ic] = packed;
            ptop2[ip][ic] = pq;
          } else if (hrow < 2 * (a.Ho >> 1) && (lane & 1) == 0 && pv[ip]) {
            const int pw = (w0 + wp * WP + ip * 16 + (lane & 15)) >> 1;
            const unsigned lidx = (unsigned)((hrow >> 1) * (a.Wo >> 1) + pw);       // inside this image
            const size_t pidx = (size_t)ppix + lidx;
            const unsigned po = (lidx * a.ldp + wc * WCN + ic * 16 + 4 * chunk) * 2;
            const u32x2_t tl = ptop[ip][ic], tr = ptop2[ip][ic];
            const u32x2_t mx = u32x2_t{pk_max16(pk_max16(tl.x, tr.x), pk_max16(packed.x, pq.x)),
                                       pk_max16(pk_max16(tl.y, tr.y), pk_max16(packed.y, pq.y))};
            __builtin_amdgcn_raw_buffer_store_b64(mx, pr, po, 0, 0);
            if (a.pcode) {
              const unsigned code = pool_code2(tl.x, tr.x, packed.x, pq.x) | pool_code2(tl.y, tr.y, packed.y, pq.y) << 16;
              *reinterpret_cast<unsigned*>(a.pcode + (size_t)pidx * a.Ngemm + wc * WCN + ic * 16 + 4 * chunk) = code;
            }
          }
        }
      }
      if constexpr (do_head) {
        // the pixel's 32 channels live in lanes l, l^16, l^32, l^48 of this wave
        hdot += __shfl_xor(hdot, 16, 64);
        hdot += __shfl_xor(hdot, 32, 64);
        if (chunk == 0 && pv[ip]) {
          const unsigned pix = (unsigned)(orow * a.Wo + w0 + wp * WP + ip * 16 + (lane & 15));
          const float z = hdot + a.hb[0];
          const float p = fast_sigmoid(z);
          if (a.hprob) a.hprob[pix] = p;
          const float tt = ttp[ip];
          const float lp = fmaxf(__logf(p), -100.f), l1p = fmaxf(__logf(1.f - p), -100.f);
          const float one = tt == 1.f ? 1.f : 0.f;
          hsum[0] -= tt * lp + (1.f - tt) * l1p;
          hsum[1] += p * one;
          hsum[2] += p;
          hsum[3] += one;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (r + 1 < nrows) rstore((r + 3) & 3, cur);
    __syncthreads();
  };
#pragma unroll 1
  for (int r = 0; r < nrows; r += 2) {
    row(r, setA, setB);
    if (r + 1 < nrows) row(r + 1, setB, setA);
  }
  if constexpr (do_bn) {
    // lanes l and l^1..l^15 hold the same channels (different pixels): butterfly over the 16, then
    // the 4 pixel waves in a fixed order -> one deterministic slab row per block
    __shared__ float bred[4][2 * NG];
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s = bsum[ic][e], q = bsq[ic][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          q += __shfl_xor(q, o, 64);
        }
        if ((lane & 15) == 0) {
          const int c = wc * WCN + ic * 16 + 4 * chunk + e;
          bred[wp][c] = s;
          bred[wp][NG + c] = q;
        }
      }
    __syncthreads();
    for (int k = tid; k < 2 * NG; k += NT)
      a.bnslab[(long)blockIdx.x * 2 * NG + k] = (bred[0][k] + bred[1][k]) + (bred[2][k] + bred[3][k]);
  }
  if constexpr (do_head) {
    static_assert(!do_head || NT == 256, "head epilogue reduces over 256 threads");
    __shared__ float hred[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = block_sum_256(hsum[k], hred);
      if (tid == 0) a.hslab[(long)blockIdx.x * 4 + k] = v;
    }
  }
}

// First layer (Cin = 3 padded to 8): K = 9 taps x 8 channels.  A 32-deep MFMA k-step covers 4 taps,
// one per 16-lane group, so each lane reads its tap's 16 bytes straight from the row ring at pixel
// (p + kw) of slot (r + kh): no im2col, 3 k-steps (taps 9..11 have zero weights).
// BNS: the conv is followed by BatchNorm (bias, no ReLU): also sum y, sum y^2 of the stored bf16 output per
// block -> a.bnslab[block][2][32], as igemm_stream_kernel's EPI 4 (no statistics pass over the 512^2 output)
// NG = 64: the UNet-XL first conv (3 -> 64), the same schedule with twice the output tiles per wave.
template <int BP, int RH, bool BNS = false, int NG = 32>
__global__ __launch_bounds__(256) void igemm_stream8_kernel(IgemmArgs a) {
  static_assert(NG == 32 || NG == 64, "output channels");
  constexpr int HR = BP + 2, SLOT = HR * 16;
  constexpr int WP = BP / 4, TP = WP / 16, TC = NG / 16;
  __shared__ __attribute__((aligned(16))) char lds[3 * NG * 64 + 4 * SLOT];
  char* const Wimg = lds;
  char* const Ring = lds + 3 * NG * 64;
  const int stripsW = (a.Wo + BP - 1) / BP, segsH = (a.Ho + RH - 1) / RH;
  const int bid = blockIdx.x;
  const int n = bid / (segsH * stripsW);
  const int rem = bid - n * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * BP, h0 = hs * RH;
  const int tid = threadIdx.x, lane = tid & 63, wp = tid >> 6;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long)n * a.Hs * a.Ws * a.ldx), 0, (int)a.ximg, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + (long)n * a.Ho * a.Wo * a.ldy), 0, 0x7fffffff, 0x00020000);
  // weights [co][96] -> [kstep][co][64 B] (swz_nk<32>)
  for (int c = tid; c < 3 * NG * 4; c += 256) {
    const int cc = c & 3, row = (c >> 2) % NG, s = (c >> 2) / NG;
    const u32x4_t v = (s * 32 + cc * 8 < a.Kpad) ? *reinterpret_cast<const u32x4_t*>(a.w + (long)row * a.Kpad + s * 32 + cc * 8)
                                                 : u32x4_t{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4_t*>(Wimg + (s * NG + row) * 64 + (swz_nk<32>(row, cc) << 4)) = v;
  }
  const int iw_l = w0 + tid - 1;
  const bool lcol = tid < HR && iw_l >= 0 && iw_l < a.Ws;
  const unsigned rowbytes = (unsigned)(a.Ws * a.ldx * 2);
  u32x4_t reg;
  auto rload = [&](int ih) {
    const bool ok = lcol && ih >= 0 && ih < a.Hs;
    reg = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (unsigned)ih * rowbytes + (unsigned)(iw_l * a.ldx * 2)
                                                       : 0x80000000u, 0, 0);
  };
  auto rstore = [&](int slot) {
    if (tid < HR) *reinterpret_cast<u32x4_t*>(Ring + slot * SLOT + tid * 16) = reg;
  };
  const int chunk = lane >> 4;
  int aoff[TC];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic) {
    const int row = ic * 16 + (lane & 15);
    aoff[ic] = row * 64 + (swz_nk<32>(row, chunk) << 4);
  }
  float bias[TC][4];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[ic][e] = a.bias ? a.bias[ic * 16 + 4 * chunk + e] : 0.f;
  unsigned yl[TP];
  float pz[TP];                 // 1 for pixels inside the row (the statistics skip a ragged strip's tail)
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int pl = w0 + wp * WP + ip * 16 + (lane & 15);
    yl[ip] = pl < a.Wo ? (unsigned)((pl * a.ldy + 4 * chunk) * 2) : 0x80000000u;   // ragged strip: dropped
    pz[ip] = pl < a.Wo ? 1.f : 0.f;
  }
  float bsum[BNS ? TC : 1][4], bsq[BNS ? TC : 1][4];
  if constexpr (BNS) {
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) bsum[ic][e] = bsq[ic][e] = 0.f;
  }
#pragma unroll 1
  for (int j = 0; j < 3; ++j) {
    rload(h0 - 1 + j);
    rstore(j);
  }
  __syncthreads();
  const int nrows = min(RH, a.Ho - h0);
#pragma unroll 1
  for (int r = 0; r < nrows; ++r) {
    if (r + 1 < nrows) rload(h0 + r + 2);
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t acc[TC][TP];
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int tap = 4 * s + chunk;                     // this lane group's tap
      const int kh = tap / 3, kw = tap - kh * 3;
      const bool real = tap < 9;
      bf16x8_t af[TC], bfr[TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) af[ic] = *reinterpret_cast<const bf16x8_t*>(Wimg + s * NG * 64 + aoff[ic]);
      const char* S = Ring + ((r + (real ? kh : 0)) & 3) * SLOT;
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const int px = wp * WP + ip * 16 + (lane & 15) + (real ? kw : 0);
        bfr[ip] = *reinterpret_cast<const bf16x8_t*>(S + px * 16);   // weights of taps >= 9 are zero
      }
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip)
          acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
    }
    const unsigned ybase = (unsigned)(h0 + r) * (unsigned)(a.Wo * a.ldy * 2);
#pragma unroll
    for (int ip = 0; ip < TP; ++ip)
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        float v0 = acc[ic][ip][0] + bias[ic][0], v1 = acc[ic][ip][1] + bias[ic][1];
        float v2 = acc[ic][ip][2] + bias[ic][2], v3 = acc[ic][ip][3] + bias[ic][3];
        if (a.relu) {
          v0 = relu_f(v0); v1 = relu_f(v1); v2 = relu_f(v2); v3 = relu_f(v3);
        }
        const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
        __builtin_amdgcn_raw_buffer_store_b64(packed, yr, ybase + yl[ip] + ic * 32, 0, 0);
        if constexpr (BNS) {     // statistics of the STORED bf16 values
          const float q[4] = {pz[ip] * lo_bf(packed.x), pz[ip] * hi_bf(packed.x), pz[ip] * lo_bf(packed.y),
                              pz[ip] * hi_bf(packed.y)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bsum[ic][e] += q[e];
            bsq[ic][e] = fmaf(q[e], q[e], bsq[ic][e]);
          }
        }
      }
    __builtin_amdgcn_sched_barrier(0);
    if (r + 1 < nrows) rstore((r + 3) & 3);
    __syncthreads();
  }
  if constexpr (BNS) {
    // lanes l ^ 1..15 hold the same channels of other pixels: butterfly over the 16, then the 4 waves in a
    // fixed order -> one deterministic slab row per block
    __shared__ float bred[4][2 * NG];
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sv = bsum[ic][e], qv = bsq[ic][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          sv += __shfl_xor(sv, o, 64);
          qv += __shfl_xor(qv, o, 64);
        }
        if ((lane & 15) == 0) {
          const int c = ic * 16 + 4 * chunk + e;
          bred[wp][c] = sv;
          bred[wp][NG + c] = qv;
        }
      }
    __syncthreads();
    for (int k = tid; k < 2 * NG; k += 256)
      a.bnslab[(long)blockIdx.x * 2 * NG + k] = (bred[0][k] + bred[1][k]) + (bred[2][k] + bred[3][k]);
  }
}

template <int BP, int RH, int NG>
static int launch_igemm_stream8(const IgemmArgs& a, hipStream_t st) {
  const int grid = a.N * ((a.Ho + RH - 1) / RH) * ((a.Wo + BP - 1) / BP);
  if (a.bnslab) {   // conv followed by BatchNorm: statistics in the epilogue (bias only, plain store)
    if (a.relu || a.mask || a.accumulate || a.y2 || a.hslab) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((igemm_stream8_kernel<BP, RH, true, NG>), dim3(grid), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((igemm_stream8_kernel<BP, RH, false, NG>), dim3(grid), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

template <int BP, int NG, int CS, int RH, int WCS>
static int launch_igemm_stream(const IgemmArgs& a, hipStream_t st) {
  const int grid = a.N * ((a.Ho + RH - 1) / RH) * ((a.Wo + BP - 1) / BP);
  if (a.pool) {   // encoder conv2 (NG == CS): pool + window codes fused
    if constexpr (NG == CS) {
      hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 1>), dim3(grid), dim3(256 * WCS), 0, st, a);
      return (int)hipGetLastError();
    }
    return (int)hipErrorInvalidValue;
  }
  if (a.hslab) {  // last decoder conv + fused segmentation head / loss partials
    if constexpr (NG == 32 && WCS == 1) {
      hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 3>), dim3(grid), dim3(256 * WCS), 0, st, a);
      return (int)hipGetLastError();
    }
    return (int)hipErrorInvalidValue;
  }
  if (a.bnslab) { // BatchNorm partial sums in the epilogue: forward statistics (no mask) or backward (mask)
    if (a.y2 || a.accumulate || a.relu || (a.mask && a.mask_ch < a.Ngemm)) return (int)hipErrorInvalidValue;
    if (a.mask)
      hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 5>), dim3(grid), dim3(256 * WCS), 0, st, a);
    else
      hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 4>), dim3(grid), dim3(256 * WCS), 0, st, a);
    return (int)hipGetLastError();
  }
  if (a.y2) {     // decoder conv1 dgrad over the concat (NG = 2 CS): skip / up gradients as dense tensors
    if constexpr (NG == 2 * CS) {
      hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 2>), dim3(grid), dim3(256 * WCS), 0, st, a);
      return (int)hipGetLastError();
    }
    return (int)hipErrorInvalidValue;
  }
  if (a.mask == nullptr && !a.accumulate)    // plain forward conv: the epilogue without mask / accumulate
    hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 6>), dim3(grid), dim3(256 * WCS), 0, st, a);
  else
    hipLaunchKernelGGL((igemm_stream_kernel<BP, NG, CS, RH, WCS, 0>), dim3(grid), dim3(256 * WCS), 0, st, a);
  return (int)hipGetLastError();
}

// auto variant (measured at batch 128, tools/kbench.py --svar): 128-pixel strips where the LDS fits
// them (Cs = Ngemm = 64 included: 8 waves, 140 KB, 10-20% over 64-pixel strips), 64-pixel strips
// when the row width does not divide by 128
static int stream_auto_variant(const IgemmArgs& a) {
  int v;
  if (a.Cs == 32 && a.Ngemm == 32) v = 1;
  else if (a.Cs == 64 && a.Ngemm == 32) v = 2;
  else v = 3;                                  // Ngemm = 64 with Cs = 32 or 64
  if ((v == 1 || v == 3) && a.Wo % 128) v += 1;
  return v;
}

// blocks the streaming launch of `a` (variant 0) uses -- rows of the fused head's slab
DPA_API int dpa_igemm_stream_blocks(const IgemmArgs* args) {
  const IgemmArgs& a = *args;
  if (a.Cs == 8 && (a.Ngemm == 32 || a.Ngemm == 64)) return a.N * ((a.Ho + 31) / 32) * ((a.Wo + 127) / 128);   // igemm_stream8<128, 32>
  const int variant = stream_auto_variant(a);
  const int bp = (variant == 1 || variant == 3) ? 128 : 64;
  const int strips = (a.Wo + bp - 1) / bp;
  const long blocks32 = (long)a.N * ((a.Ho + 31) / 32) * strips;
  const int rh = blocks32 >= 1024 ? 32 : 16;
  return a.N * ((a.Ho + rh - 1) / rh) * strips;
}

// Eligible: conv3x3 s1 p1 mode 0, Ngemm and Cs in {32, 64}, Wo >= 16 (a ragged last strip is masked), Ho >= 1.
// With a.pool set the kernel also writes the 2x2/s2 max-pool of y (floor semantics).
// variant: 0 auto, 1: BP128 x 4 waves, 2: BP64 x 4 waves, 3: BP128 x 8 waves, 4: BP64 x 8 waves
DPA_API int dpa_igemm_stream(const IgemmArgs* args, int variant, hipStream_t st) {
  const IgemmArgs& a = *args;
  // any row width: a partial last strip masks its out-of-row pixels (loads read zeros, stores are
  // dropped); the fused pool needs whole 2x2 windows along the row (even width)
  if (a.mode != 0 || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || (a.ldx & 7) || (a.ldy & 3) ||
      a.Hs != a.Ho || a.Ws != a.Wo || a.Wo < 16 || a.Kpad < 9 * a.Cs || !ximg_ok(a) ||
      (a.pool && ((a.ldp & 3) || (a.Wo & 1) || !a.relu)) || (a.x2 && (a.Cs != 64 || a.ldx < 32)) ||
      (a.xbn && (a.bnslab == nullptr || a.mask || a.pool || a.hslab || a.Cs == 8)))     // BN-on-load: the EPI 4 kernels only
    return (int)hipErrorInvalidValue;
  if (a.Cs == 8 && a.Ngemm == 32 && !a.pool) return launch_igemm_stream8<128, 32, 32>(a, st);
  if (a.Cs == 8 && a.Ngemm == 64 && !a.pool && !a.hslab && !a.mask && !a.accumulate && !a.y2 && !a.x2)
    return launch_igemm_stream8<128, 32, 64>(a, st);
  if (variant == 0) variant = stream_auto_variant(a);
  const int bp = (variant == 1 || variant == 3) ? 128 : 64;
  const long blocks32 = (long)a.N * ((a.Ho + 31) / 32) * ((a.Wo + bp - 1) / bp);
  const int rh = blocks32 >= 1024 ? 32 : 16;
#define DPA_STREAM(NGv, CSv)                                                                               \
  if (a.Ngemm == NGv && a.Cs == CSv) {                                                                    \
    switch (variant * 100 + rh) {                                                                         \
      case 132: return launch_igemm_stream<128, NGv, CSv, 32, 1>(a, st);                                  \
      case 116: return launch_igemm_stream<128, NGv, CSv, 16, 1>(a, st);                                  \
      case 232: return launch_igemm_stream<64, NGv, CSv, 32, 1>(a, st);                                   \
      case 216: return launch_igemm_stream<64, NGv, CSv, 16, 1>(a, st);                                   \
      case 332: if (NGv % 32) break; return launch_igemm_stream<128, NGv, CSv, 32, 2>(a, st);             \
      case 316: if (NGv % 32) break; return launch_igemm_stream<128, NGv, CSv, 16, 2>(a, st);             \
      case 432: if (NGv % 32) break; return launch_igemm_stream<64, NGv, CSv, 32, 2>(a, st);              \
      case 416: if (NGv % 32) break; return launch_igemm_stream<64, NGv, CSv, 16, 2>(a, st);              \
      default: break;                                                                                     \
    }                                                                                                     \
  }
  DPA_STREAM(32, 32)
  DPA_STREAM(32, 64)
  DPA_STREAM(64, 32)
  DPA_STREAM(64, 64)
#undef DPA_STREAM
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------ wgrad_stream
// Row-streaming conv3x3 weight gradient.  A block owns one (BM out-ch x BN in-ch) tile and an
// image strip [w0, w0+BP) x rows [h0, h0+RH) (its split).  Per output row it stages the gradient
// row g[h][w0..w0+BP) (A) and streams the layer-input rows through a 4-slot ring (B, BP+2 pixels
// incl. halo), so every input/gradient pixel is read ~once.  Three waves, one per kernel row kh:
// wave kh accumulates the taps (kh, 0..2) against ring slot (r + kh) with a pixel shift kw, i.e.
// dW[co][kh][kw][ci] += sum_px g[h][px][co] * x[h+kh-1][px+kw-1][ci].  Fragments come from the
// [pixel][channel] LDS images through ds_read_b64_tr_b16 (conflict-free swizzles, any row shift).
// Bias gradient: the loader threads sum the gradient chunks they stage, reduced once per block.
// the two ds_read_b64_tr_b16 of a transposed fragment (tr_frag) at precomputed byte offsets
__device__ __forceinline__ bf16x8_t tr_pair_off(const char* base, int off0, int off1) {
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off1));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int BM, int BN, int BP, int RH, bool ABN = false>
__global__ __launch_bounds__(192) void wgrad_stream_kernel(WgradArgs a, int ipb) {
  constexpr int NT = 192;
  constexpr int HR = BP + 2;
  constexpr int CPRA = BM / 8, CPRB = BN / 8, RBA = BM * 2, RBB = BN * 2;
  constexpr int IMGA = BP * RBA, SLOTB = HR * RBB;
  constexpr int CHA = BP * CPRA, CHB = HR * CPRB;
  constexpr int LA = (CHA + NT - 1) / NT, LB = (CHB + NT - 1) / NT;
  constexpr int TM = BM / 16, TN = BN / 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * IMGA + 4 * SLOTB];
  __shared__ float bred[BM];
  __shared__ float abc[ABN ? 3 * BM : 4];       // ABN: this tile's dz coefficients [3][BM]
  char* const Aimg = lds;
  char* const Ring = lds + 2 * IMGA;

  const int nmt = a.M / BM, nnt = (a.Nc + BN - 1) / BN, tiles = nmt * nnt;
  const int stripsW = (a.Wg + BP - 1) / BP, segsH = (a.Hg + RH - 1) / RH;   // ragged last strip allowed
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;     // split = (image group, hs, ws)
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ig = split / (segsH * stripsW);                      // images [ig*ipb, ig*ipb + ipb)
  const int rem = split - ig * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * BP, h0 = hs * RH;
  const int nrows = min(RH, a.Hg - h0);
  const int nimg = min(ipb, a.N - ig * ipb);
  const int tid = threadIdx.x, lane = tid & 63, kh = tid >> 6;
  const bool do_bias = a.bslab != nullptr && nt == 0;
  // one image at a time: 64-bit image bases (rebound per image below), 32-bit offsets inside it;
  // a.abytes / a.bbytes are the extents of ONE image here, so one launch covers any batch
  __amdgpu_buffer_rsrc_t ar, br, zr;

  // per-thread loader constants
  unsigned aoff[LA], boff[LB];
  int asto[LA], bsto[LB];
  bool bok[LB];
  if constexpr (ABN) {
    for (int i = tid; i < 3 * BM; i += NT) abc[i] = a.abn[(i / BM) * a.M + m0 + i % BM];
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int c = tid + j * NT, px = c / CPRA, cc = c - px * CPRA;
    // gradient pixels past the row (ragged last strip) read as zeros: they add nothing to dW / db
    aoff[j] = w0 + px < a.Wg ? (unsigned)(((w0 + px) * a.lda + m0 + cc * 8) * 2) : 0x80000000u;
    asto[j] = c < CHA ? px * RBA + ((cc ^ swz_kk<RBA>(px)) << 4) : -1;
  }
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int c = tid + j * NT, px = c / CPRB, cc = c - px * CPRB;
    const int iw = w0 + px - 1;
    bok[j] = c < CHB && iw >= 0 && iw < a.WB && n0 + cc * 8 < a.Nc;   // channel tail (first layer: 8 of 16)
    boff[j] = (unsigned)((iw * a.ldb + n0 + cc * 8) * 2);
    bsto[j] = c < CHB ? px * RBB + ((cc ^ swz_kk<RBB>(px)) << 4) : -1;
  }
  const unsigned arow = (unsigned)(a.WA * a.lda * 2), brow = (unsigned)(a.WB * a.ldb * 2);
  u32x4_t ra[LA], rb[LB], rz[ABN ? LA : 1];
  int n = ig * ipb;
  auto load_a = [&](int h) {
    const unsigned base = (unsigned)h * arow;
#pragma unroll
    for (int j = 0; j < LA; ++j) ra[j] = __builtin_amdgcn_raw_buffer_load_b128(ar, asto[j] >= 0 ? base + aoff[j] : 0x80000000u, 0, 0);
    if constexpr (ABN) {
#pragma unroll
      for (int j = 0; j < LA; ++j) rz[j] = __builtin_amdgcn_raw_buffer_load_b128(zr, asto[j] >= 0 ? base + aoff[j] : 0x80000000u, 0, 0);
    }
  };
  // ABN: (g, z) chunk -> dz chunk; pixels past the row stay zero (they add nothing to dW / db)
  auto xform_a = [&]() {
    if constexpr (ABN) {
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const int c = tid + j * NT, cb = (c % CPRA) * 8;
        const bool ok = asto[j] >= 0 && aoff[j] != 0x80000000u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = cb + 2 * e;
          const float v0 = fmaf(abc[ch], lo_bf(ra[j][e]), fmaf(abc[BM + ch], lo_bf(rz[j][e]), abc[2 * BM + ch]));
          const float v1 = fmaf(abc[ch + 1], hi_bf(ra[j][e]), fmaf(abc[BM + ch + 1], hi_bf(rz[j][e]), abc[2 * BM + ch + 1]));
          ra[j][e] = ok ? pack_bf2(v0, v1) : 0u;
        }
      }
    }
  };
  auto load_b = [&](int ih) {
    const bool rok = ih >= 0 && ih < a.HB;
    const unsigned base = (unsigned)ih * brow;
#pragma unroll
    for (int j = 0; j < LB; ++j)
      rb[j] = __builtin_amdgcn_raw_buffer_load_b128(br, (rok && bok[j]) ? base + boff[j] : 0x80000000u, 0, 0);
  };
  // bias gradient: wave 0 sums the staged gradient row from LDS; lane owns channel chunk lane % CPRA
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto store_a = [&](int buf) {
#pragma unroll
    for (int j = 0; j < LA; ++j)
      if (asto[j] >= 0) *reinterpret_cast<u32x4_t*>(Aimg + buf * IMGA + asto[j]) = ra[j];
  };
  auto store_b = [&](int slot) {
#pragma unroll
    for (int j = 0; j < LB; ++j)
      if (bsto[j] >= 0) *reinterpret_cast<u32x4_t*>(Ring + slot * SLOTB + bsto[j]) = rb[j];
  };

  f32x4_t acc[3][TM][TN];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[kw][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // transposed-fragment addressing (tr_frag) with the per-lane parts precomputed: fragment (column
  // tile c, k-step ks, half h) sits at base + ((2c << 4) ^ sw4[h]) + const -- the swizzle only sees row
  // bits that ks*32 and the column tile do not touch, so per fragment one XOR + one add remain (the
  // per-fragment swizzle arithmetic was more VALU issue than the MFMAs it fed)
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int fcol = (fp & 1) * 8 + (fp >> 1) * 16;            // byte offset of this lane's 4 columns
  int swA[2], swB[3][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    swA[h] = swz_kk<RBA>(8 * fg + fq + 4 * h) << 4;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) swB[kw][h] = swz_kk<RBB>(kw + 8 * fg + fq + 4 * h) << 4;
  }
  const int baseA = (8 * fg + fq) * RBA + fcol, baseB = (8 * fg + fq) * RBB + fcol;

#pragma unroll 1
  for (int im = 0; im < nimg; ++im, ++n) {
  ar = __builtin_amdgcn_make_buffer_rsrc((void*)(a.atab ? a.atab[n] : a.A + (long)n * a.HA * a.WA * a.lda), 0, (int)a.abytes, 0x00020000);
  br = __builtin_amdgcn_make_buffer_rsrc((void*)(a.btab ? a.btab[n] : a.B + (long)n * a.HB * a.WB * a.ldb), 0, (int)a.bbytes, 0x00020000);
  if constexpr (ABN) zr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.az + (long)n * a.HA * a.WA * a.lda), 0, (int)a.abytes, 0x00020000);
  // prologue: input rows h0-1, h0, h0+1 -> ring slots 0..2; gradient row h0 -> A buffer 0
  if (nrows > 0) {
#pragma unroll 1
    for (int j = 0; j < 3; ++j) {
      load_b(h0 - 1 + j);
      store_b(j);
    }
    load_a(h0);
    xform_a();
    store_a(0);
  }
  __syncthreads();
#pragma unroll 1
  for (int r = 0; r < nrows; ++r) {
    const bool more = r + 1 < nrows;
    if (more) {
      load_a(h0 + r + 1);
      load_b(h0 + r + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* Ai = Aimg + (r & 1) * IMGA;
    const char* Bi = Ring + ((r + kh) & 3) * SLOTB;
#pragma unroll
    for (int ks = 0; ks < BP / 32; ++ks) {
      bf16x8_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = tr_pair_off(Ai + ks * 32 * RBA, baseA + (((2 * i) << 4) ^ swA[0]), baseA + 4 * RBA + (((2 * i) << 4) ^ swA[1]));
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const char* Bk = Bi + (ks * 32 + kw) * RBB;
          const bf16x8_t bf = tr_pair_off(Bk, baseB + (((2 * j) << 4) ^ swB[kw][0]), baseB + 4 * RBB + (((2 * j) << 4) ^ swB[kw][1]));
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[kw][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[kw][i][j], 0, 0, 0);
        }
    }
    if (do_bias && kh == 0) {
#pragma unroll
      for (int c = lane; c < CHA; c += 64) {
        const int px = c / CPRA, cc = c - px * CPRA;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(Ai + px * RBA + ((cc ^ swz_kk<RBA>(px)) << 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bsum[2 * e] += lo_bf(v[e]);
          bsum[2 * e + 1] += hi_bf(v[e]);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      xform_a();
      store_a((r + 1) & 1);
      store_b((r + 3) & 3);
    }
    __syncthreads();
  }
  }   // images of this split
  // epilogue: this split's partial dW for taps (kh, 0..2)
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nn = n0 + j * 16 + (lane & 15);
        if (nn >= a.Nc) continue;
        const int mb = m0 + i * 16 + 4 * (lane >> 4);
        float* dst = a.slab + (((long)split * 9 + kh * 3 + kw) * a.M + mb) * a.Nc + nn;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) dst[(long)rr * a.Nc] = acc[kw][i][j][rr];
      }
  if (do_bias) {
    for (int c = tid; c < BM; c += NT) bred[c] = 0.f;
    __syncthreads();
    if (kh == 0) {
      const int cc = lane % CPRA;
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&bred[cc * 8 + e], bsum[e]);
    }
    __syncthreads();
    for (int c = tid; c < BM; c += NT) a.bslab[(long)split * a.M + m0 + c] = bred[c];
  }
}

template <int BM, int BN, int BP, int RH, bool ABN = false>
static int launch_wgrad_stream(const WgradArgs& a, int ipb, hipStream_t st) {
  const int tiles = (a.M / BM) * ((a.Nc + BN - 1) / BN);
  hipLaunchKernelGGL((wgrad_stream_kernel<BM, BN, BP, RH, ABN>), dim3(tiles * a.splits), dim3(192), 0, st, a, ipb);
  return (int)hipGetLastError();
}

// A split = ipb consecutive images x one (row segment, column strip): splits must equal
// ceil(N/ipb) * ceil(Hg/RH) * (Wg/BP).  More images per split = fewer fp32 slabs to reduce (the
// reduction's bytes otherwise grow with the batch).  cfg picks (BM, BN): 1: 32x32  2: 64x32  3: 32x64
// 4: 32x16 with Nc == 8 (the first layer's 8-padded RGB input; channels 8..15 read as zeros).
// (A 64x64 tile measured 5-20% slower than 64x32 / 32x64 on every UNet shape at batch 128.)
DPA_API int dpa_wgrad_stream(const WgradArgs* args, int cfg, int bp, int rh, int ipb, hipStream_t st) {
  const WgradArgs& a = *args;
  if (ipb < 1 || (a.lda & 7) || (a.ldb & 7) || a.s != 1 || a.pad != 1 || a.KW != 3 || a.HA != a.Hg || a.WA != a.Wg ||
      a.HB != a.Hg || a.WB != a.Wg || a.Wg < 8 ||
      a.splits != ((a.N + ipb - 1) / ipb) * ((a.Hg + rh - 1) / rh) * ((a.Wg + bp - 1) / bp))
    return (int)hipErrorInvalidValue;
  // BatchNorm backward on load of the gradient: the first layer's tile only (the other 32/64-channel
  // layers of a BN model take the fused backward, csrc/bwd_stream.hip, which does the same on load)
  if (a.abn != nullptr || a.az != nullptr) {
    if (!(a.abn && a.az) || a.atab || cfg != 4 || a.Nc != 8 || a.M % 32 || bp != 64) return (int)hipErrorInvalidValue;
    if (rh == 64) return launch_wgrad_stream<32, 16, 64, 64, true>(a, ipb, st);
    if (rh == 32) return launch_wgrad_stream<32, 16, 64, 32, true>(a, ipb, st);
    return (int)hipErrorInvalidValue;
  }
#define DPA_WS(C, BMv, BNv, BPv, RHv)                                                              \
  if (cfg == C && bp == BPv && rh == RHv && a.M % BMv == 0 && a.Nc % BNv == 0) return launch_wgrad_stream<BMv, BNv, BPv, RHv>(a, ipb, st);
  DPA_WS(1, 32, 32, 64, 64)
  DPA_WS(2, 64, 32, 64, 64)
  DPA_WS(3, 32, 64, 64, 64)
  DPA_WS(1, 32, 32, 64, 32)
  DPA_WS(2, 64, 32, 64, 32)
  DPA_WS(3, 32, 64, 64, 32)
  DPA_WS(1, 32, 32, 32, 64)
  DPA_WS(2, 64, 32, 32, 64)
  DPA_WS(3, 32, 64, 32, 64)
  DPA_WS(1, 32, 32, 32, 32)
  DPA_WS(2, 64, 32, 32, 32)
  DPA_WS(3, 32, 64, 32, 32)
#undef DPA_WS
  if (cfg == 4 && a.Nc == 8 && a.M % 32 == 0 && bp == 64) {
    if (rh == 64) return launch_wgrad_stream<32, 16, 64, 64>(a, ipb, st);
    if (rh == 32) return launch_wgrad_stream<32, 16, 64, 32>(a, ipb, st);
  }
  return (int)hipErrorInvalidValue;
}
