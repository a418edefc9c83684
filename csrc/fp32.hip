// fp32 training path (the reference's precision, utils/train_utils.py:60-61): fp32 storage, fp32 MFMA
// (v_mfma_f32_16x16x4_f32, IEEE fp32 products, fp32 accumulation) for every conv-shaped product of the
// UNet step, plus the fp32 elementwise ops around them.  The bf16 engine's kernels (halo.hip,
// igemm_glds.hip, bwd_stream.hip ...) are bf16-specialised; this is a separate, deliberately simple
// family -- correctness and precision first, the bf16 path is the fast one.
//
//   igemm_f32_kernel : implicit GEMM, NHWC fp32 (reference
//                      model/unet_parts.py:10-12,51-54):
//       conv3x3 forward  y[p][co] = relu?(b + sum_{tap,ci} x[p + off(tap)][ci] W[co][tap][ci])
//       conv3x3 dgrad    dx[p][ci] = sum_{tap,co} g[p + off(tap)][co] Wflip[ci][tap][co]
//       transposed conv forward (mode 1: 2x2/s2 scatter of n = (2i+j) Cout + co)
//       transposed conv dgrad (KH = KW = 2, stride 2 gather)
//     GEMM M = output pixels, N = output channels, K = taps x source channels (16-deep K-steps of
//     float4 chunks that never straddle a tap: Cs % 4 == 0).  Register-staged, double-buffered LDS.
//   wgrad_f32_kernel : dW[m][tap][n] = sum_p A[p][m] B[p*s + d(tap) - pad][n] (K3), split over pixel
//                      ranges into fp32 slab rows [split][tap][M][Nc] that dpa_wgrad_reduce sums in a
//                      fixed order; the bias gradient sum_p A[p][m] rides along (A = the output gradient).
//   elementwise       : ReLU backward, 2x2 max-pool with window codes and its backward, the segmentation
//                       head (1x1 conv + sigmoid + BCE/Dice partial sums) and its backward, NCHW -> NHWC4.
//
// MFMA operand order: the 16x16x4 f32 MFMA takes one K value per lane (lane group q = lane >> 4 holds
// k = q).  Each lane reads a float4 of 4 consecutive K values of its row from LDS and issues 4 MFMAs
// with elements 0..3: K is summed in the permuted order (4q + e) -- the same for both operands, so the
// product is the same sum in another order (fp32 rounding differs from a sequential sum by ~1 ulp).
#include "common.h"

typedef float f32x4v __attribute__((ext_vector_type(4)));

struct F32ConvArgs {
  const float* x;       // source [N][Hs][Ws][ldx]
  const float* w;       // packed weights [Ngemm][Kpad] fp32, k = tap * Cs + ci (zero beyond KH*KW*Cs)
  const float* bias;    // [Cout] or null
  float* y;             // output (mode 0: [N][Ho][Wo][ldy]; mode 1: [N][2Ho][2Wo][ldy])
  const float* mask;    // optional ReLU-backward mask on the output grid (y = 0 where mask <= 0)
  int ldx, ldy, ldm, mask_ch;
  int N, Ho, Wo, Hs, Ws, Cs;
  int KH, KW, stride, pad;
  int Ngemm, Kpad, mode, relu, accumulate, Cout;
  int wide;             // 1: the 256-pixel 8-wave tile for GEMM-N % 128 == 0 (ops/fp32.py IGEMM_WIDE)
  int halo;             // 1: 3x3 / s1 / p1 convs with GEMM-N == 32 (or 64, 2): conv3_halo_f32_kernel
};

struct F32WgradArgs {
  const float* A;       // [N][Hg][Wg][lda]: M channels (the output gradient for a conv)
  const float* B;       // [N][HB][WB][ldb]: Nc channels, read at (h*s + kh - pad, w*s + kw - pad)
  float* slab;          // [splits][T][M][Nc]
  float* bslab;         // [splits][M] (sum of A over the split's pixels) or null
  int lda, ldb, N, Hg, Wg, HB, WB, M, Nc, s, pad, KH, KW;
  long pix_per_split;   // pixels per split (multiple of 32; halo form: of 64, in stage order)
  int splits;
  int halo;             // 1: the 3x3 / s1 / p1 form with the B halo staged per 2 x 32-pixel stage; 2: 64 columns as 2 x 32;
                        //    3: the first layer's 4-channel form (wgrad_c4_f32_kernel)
  int big;              // 1: allow the 256 x 256 tile (M % 256 == 0, >= 256 columns)
  int px;               // 1: pixel-major LDS images (no loader transpose), PX form of wgrad_f32_kernel
};

namespace {

constexpr int F_BK = 16;             // K-step granularity of the implicit GEMM (Kpad % 16 == 0)

// conflict-free ds_read_b128 of 16 consecutive rows at one chunk: 64-B rows (4 chunks) rotate the
// chunk every 4 rows, 128-B rows (8 chunks) every 2 rows -- 16 distinct 16-B bank groups either way
template <int CPR>
__device__ __forceinline__ int fswzk(int row, int chunk) {
  if constexpr (CPR == 4) return chunk ^ ((row >> 2) & 3);
  else return chunk ^ ((row >> 1) & 7);
}

// weight-gradient operand rows: additionally XOR row bits 4..6, so the loader's rotated 4-row micro-block
// stores (rows 4q + (j + q) % 4 across a 16-lane group) are conflict-free as well as the 16-row reads
__device__ __forceinline__ int wswz(int row, int chunk) { return chunk ^ (((row >> 1) ^ (row >> 4)) & 7); }

__device__ __forceinline__ f32x4_t mfma4(const f32x4v& a, const f32x4v& b, f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

}  // namespace

// BP pixels x BC channels per block, BK-deep K-steps, NW waves (NWP along the pixels x NWC along the channels);
// NW = 8 with BP = 256: twice the MFMA work per barrier and per staged weight row (the deep layers)
template <int BP, int BC, int NWP, int BK, int NW = 4>
__global__ __launch_bounds__(64 * NW) void igemm_f32_kernel(F32ConvArgs a) {
  constexpr int NWC = NW / NWP, WP = BP / NWP, WC = BC / NWC, TP = WP / 16, TC = WC / 16;
  static_assert(NWP * NWC == NW && TP >= 1 && TC >= 1 && (BK == 16 || BK == 32), "tile");
  constexpr int CPR = BK / 4, RPP = 64 * NW / CPR;   // float4 chunks per LDS row, rows per loader pass
  constexpr int RB = BK * 4;                         // LDS row bytes
  constexpr int LP = BP / RPP, LW = (BC + RPP - 1) / RPP;
  static_assert(BP % RPP == 0, "loader tiling");
  __shared__ __attribute__((aligned(16))) char lds[2][(BP + BC) * RB];

  const int M = a.N * a.Ho * a.Wo;
  const int nct = a.Ngemm / BC, npt = (M + BP - 1) / BP;
  const int bid = xcd_remap(blockIdx.x, npt * nct);
  const int pt = bid / nct, ct = bid - pt * nct;
  const int m0 = pt * BP, c0 = ct * BC;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid / NWC, wc = wid - wp * NWC;
  const int lchunk = tid % CPR, lrow = tid / CPR;  // RPP rows x CPR chunks per pass
  const int taps = a.KH * a.KW;

  // per pixel row: (n, h0, w0) of tap (0, 0) and the in-image taps
  int pn[LP], ph0[LP], pw0[LP];
  unsigned tmask[LP];
#pragma unroll
  for (int i = 0; i < LP; ++i) {
    const int m = m0 + lrow + i * RPP;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    const int hw = a.Ho * a.Wo;
    pn[i] = mm / hw;
    const int rem = mm - pn[i] * hw;
    const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
    ph0[i] = oh * a.stride - a.pad;
    pw0[i] = ow * a.stride - a.pad;
    unsigned msk = 0;
    for (int t = 0; t < taps; ++t) {
      const int kh = t / a.KW, kw = t - kh * a.KW;
      const int ih = ph0[i] + kh, iw = pw0[i] + kw;
      if (ok && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) msk |= 1u << t;
    }
    tmask[i] = msk;
  }
  const int S = a.Kpad / BK;
  f32x4v pr[LP], wr[LW];
  auto gload = [&](int s) {
    const int k0 = s * BK + lchunk * 4;
    const int tap = k0 / a.Cs, ci = k0 - tap * a.Cs;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      if (tap < taps && ((tmask[i] >> tap) & 1u)) {
        const long off = ((long)(pn[i] * a.Hs + ph0[i] + kh) * a.Ws + pw0[i] + kw) * a.ldx + ci;
        pr[i] = *reinterpret_cast<const f32x4v*>(a.x + off);
      } else {
        pr[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int r = lrow + i * RPP;
      if (r < BC) wr[i] = *reinterpret_cast<const f32x4v*>(a.w + (long)(c0 + r) * a.Kpad + s * BK + lchunk * 4);
    }
  };
  auto lstore = [&](int buf) {
    char* P = lds[buf];
    char* Wt = lds[buf] + BP * RB;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      const int r = lrow + i * RPP;
      *reinterpret_cast<f32x4v*>(P + r * RB + fswzk<CPR>(r, lchunk) * 16) = pr[i];
    }
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int r = lrow + i * RPP;
      if (r < BC) *reinterpret_cast<f32x4v*>(Wt + r * RB + fswzk<CPR>(r, lchunk) * 16) = wr[i];
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
  const int q = lane >> 4;
  for (int s = 0; s < S; ++s) {
    const int buf = s & 1;
    if (s + 1 < S) gload(s + 1);
    const char* P = lds[buf];
    const char* Wt = lds[buf] + BP * RB;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = kk * 4 + q;
      f32x4v af[TC], bfr[TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic) {
        const int row = wc * WC + ic * 16 + (lane & 15);
        af[ic] = *reinterpret_cast<const f32x4v*>(Wt + row * RB + fswzk<CPR>(row, ch) * 16);
      }
#pragma unroll
      for (int ip = 0; ip < TP; ++ip) {
        const int row = wp * WP + ip * 16 + (lane & 15);
        bfr[ip] = *reinterpret_cast<const f32x4v*>(P + row * RB + fswzk<CPR>(row, ch) * 16);
      }
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = mfma4(af[ic], bfr[ip], acc[ic][ip]);
    }
    if (s + 1 < S) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds 4 consecutive GEMM columns (4 q + r) of pixel (lane & 15)
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int m = m0 + wp * WP + ip * 16 + (lane & 15);
    if (m >= M) continue;
    long ybase;
    if (a.mode == 0) {
      ybase = (long)m * a.ldy;
    } else {
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, rem = m - n * hw, h = rem / a.Wo, w = rem - (rem / a.Wo) * a.Wo;
      ybase = ((long)(n * 2 * a.Ho + 2 * h) * (2 * a.Wo) + 2 * w) * a.ldy;
    }
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int nidx = c0 + wc * WC + ic * 16 + 4 * q;
      int co = nidx;
      long off = ybase + nidx;
      if (a.mode == 1) {
        const int ij = nidx / a.Cout;
        co = nidx - ij * a.Cout;
        off = ybase + (long)((ij >> 1) * (2 * a.Wo) + (ij & 1)) * a.ldy + co;
      }
      f32x4v v = f32x4v{acc[ic][ip][0], acc[ic][ip][1], acc[ic][ip][2], acc[ic][ip][3]};
      if (a.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += a.bias[co + r];
      }
      if (a.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (a.mask && co < a.mask_ch) {
        const f32x4v mk = *reinterpret_cast<const f32x4v*>(a.mask + (long)m * a.ldm + co);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = mk[r] > 0.f ? v[r] : 0.f;
      }
      if (a.accumulate) v += *reinterpret_cast<const f32x4v*>(a.y + off);
      *reinterpret_cast<f32x4v*>(a.y + off) = v;
    }
  }
}

// 3x3 / stride 1 / pad 1 conv over 32-channel input slices with a narrow GEMM-N (32 output columns per
// block): the implicit GEMM above re-fetches every input pixel once per tap (9x) for only 32 output
// channels -- 16 FLOP per byte through L1 / L2, the bound of the 32-channel full-resolution layers
// (70-86 TF/s, profiles/f32_kbench_b16_512_r05_px.txt).  Here a block stages the 10 x 34 input halo of its
// 8 x 32 output pixels once per 32-channel slice ([pixel][32 ch], 128-B rows, chunk ^ (pixel & 7) so 8
// consecutive pixels at any tap shift read distinct bank groups) together with the slice's 9 taps of
// weights ([tap][n][32 k], fswzk<8>), and every tap reads its operands from LDS: 80 KB per block (2 per
// CU), ~4x fewer fetched bytes per FLOP.  Wave w computes output rows 2w, 2w + 1 (4 pixel tiles x 2
// channel tiles).  K runs tap-major within a slice in 16-deep slabs, the permuted 4q + e order as above.
// Same epilogue (bias / ReLU / mask / accumulate) as igemm_f32_kernel, mode 0.
__global__ __launch_bounds__(256) void conv3_halo_f32_kernel(F32ConvArgs a) {
  constexpr int BR = 8, BW = 32, HR = BR + 2, HW = BW + 2, HP = HR * HW, RB = 128;
  __shared__ __attribute__((aligned(16))) char lds[(HP + 9 * 32) * RB];
  char* Hs = lds;
  char* Ws = lds + HP * RB;
  const int nct = a.Ngemm / 32, nwt = a.Wo / BW, nht = a.Ho / BR;
  const int total = a.N * nht * nwt * nct;
  const int bid = xcd_remap(blockIdx.x, total);
  const int ct = bid % nct, pt = bid / nct;
  const int n = pt / (nht * nwt), rem = pt - n * (nht * nwt), hb = rem / nwt, wb = rem - hb * nwt;
  const int h0 = hb * BR, w0 = wb * BW, c0 = ct * 32;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4, l16 = lane & 15;

  f32x4_t acc[2][4];
#pragma unroll
  for (int ic = 0; ic < 2; ++ic)
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int cs = 0; cs < a.Cs; cs += 32) {
    if (cs) __syncthreads();
    // halo slice: HP pixels x 8 chunks, chunk-fastest across threads
    constexpr int HI = (HP * 8 + 255) / 256;
    f32x4v hv[HI];
#pragma unroll
    for (int i = 0; i < HI; ++i) {          // all loads in flight before the first store
      const int u = tid + 256 * i, p = u >> 3, c = u & 7, hr = p / HW, hc = p - hr * HW;
      const int ih = h0 - 1 + hr, iw = w0 - 1 + hc;
      hv[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (u < HP * 8 && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws)
        hv[i] = *reinterpret_cast<const f32x4v*>(a.x + ((long)(n * a.Hs + ih) * a.Ws + iw) * a.ldx + cs + 4 * c);
    }
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int u = tid + 256 * i, p = u >> 3, c = u & 7;
      if (u < HP * 8) *reinterpret_cast<f32x4v*>(Hs + p * RB + ((c ^ (p & 7)) << 4)) = hv[i];
    }
    // weights of the slice: row (tap, n) = the packed row c0 + n at k = tap * Cs + cs
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int u = tid + 256 * i, row = u >> 3, c = u & 7, tap = row >> 5, nn = row & 31;
      *reinterpret_cast<f32x4v*>(Ws + row * RB + fswzk<8>(row, c) * 16) =
          *reinterpret_cast<const f32x4v*>(a.w + (long)(c0 + nn) * a.Kpad + tap * a.Cs + cs + 4 * c);
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - 3 * kh;
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        const int ch = 4 * sl + q;
        f32x4v af[2], bf[4];
#pragma unroll
        for (int ic = 0; ic < 2; ++ic) {
          const int row = tap * 32 + ic * 16 + l16;
          af[ic] = *reinterpret_cast<const f32x4v*>(Ws + row * RB + fswzk<8>(row, ch) * 16);
        }
#pragma unroll
        for (int ip = 0; ip < 4; ++ip) {
          const int p = (2 * wid + (ip >> 1) + kh) * HW + 16 * (ip & 1) + l16 + kw;
          bf[ip] = *reinterpret_cast<const f32x4v*>(Hs + p * RB + ((ch ^ (p & 7)) << 4));
        }
#pragma unroll
        for (int ic = 0; ic < 2; ++ic)
#pragma unroll
          for (int ip = 0; ip < 4; ++ip) acc[ic][ip] = mfma4(af[ic], bf[ip], acc[ic][ip]);
      }
    }
  }

  // epilogue: lane holds 4 consecutive output channels (4 q + r) of pixel l16 of each pixel tile
#pragma unroll
  for (int ip = 0; ip < 4; ++ip) {
    const long m = ((long)n * a.Ho + h0 + 2 * wid + (ip >> 1)) * a.Wo + w0 + 16 * (ip & 1) + l16;
#pragma unroll
    for (int ic = 0; ic < 2; ++ic) {
      const int co = c0 + ic * 16 + 4 * q;
      const long off = m * a.ldy + co;
      f32x4v v = f32x4v{acc[ic][ip][0], acc[ic][ip][1], acc[ic][ip][2], acc[ic][ip][3]};
      if (a.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += a.bias[co + r];
      }
      if (a.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (a.mask && co < a.mask_ch) {
        const f32x4v mk = *reinterpret_cast<const f32x4v*>(a.mask + m * a.ldm + co);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = mk[r] > 0.f ? v[r] : 0.f;
      }
      if (a.accumulate) v += *reinterpret_cast<const f32x4v*>(a.y + off);
      *reinterpret_cast<f32x4v*>(a.y + off) = v;
    }
  }
}

// Weight gradient: dW[m][col] = sum_p A[p][m] B'[p][col], col = tap * Nc + n, B'[p][col] = B at pixel p's tap
// position.  BM (A channels) x BN (columns) per block, 2 BN threads: BN = 128 -> 4 waves (2 x 2 of 64 x 64
// for BM = 128, else 1 x 4); BN = 256 -> 8 waves (2 x 4; 128 x 64 each for BM = 256: the deep layers, half
// the staged operand bytes per FLOP of the 128 x 128 tile, one block of 128 KB LDS per CU).
// K = 32 pixels per stage.  LDS holds both operands K-contiguous ([channel / column][32 px], 128-B rows,
// fswzk<8> swizzle), as the conv kernel does, so an MFMA operand is one ds_read_b128 per 4 MFMAs (K in
// the permuted 4q + e order, the same for both operands).  The loader transposes in registers: a thread
// loads a 4-pixel x 4-channel micro-block (4 float4, channel-contiguous in NHWC) and writes it as 4
// float4 rows of 4 pixels.  Next stage's loads in registers during the current one; one barrier per
// stage.  The bias gradient sum_p A[p][m] rides along in the blocks of column tile 0.
//
// PX = true: the same GEMM with PIXEL-major LDS images ([32 px][BM + 4] / [32 px][BN + 4] floats, channels
// contiguous as in NHWC): the loader stores each thread's float4s as they were loaded (no register
// transpose), and an MFMA operand is 4 ds_read_b32 of one channel column (rows 4q + e; the +4-float row
// pad puts rows 4 apart 16 banks apart: conflict-free halves).  Same MFMA sequence per accumulator -> the
// same result bit for bit.
template <int BM, int BN, bool PX = false>
__global__ __launch_bounds__(2 * BN) void wgrad_f32_kernel(F32WgradArgs a) {
  constexpr int BK = 32, RB = BK * 4;                           // LDS row bytes (8 chunks of 4 px)
  constexpr int NT = 2 * BN, NW = NT / 64;                      // one B micro-block per thread per stage
  constexpr int NWM = BM >= 128 ? 2 : 1, NWN = NW / NWM, WM = BM / NWM, WN = BN / NWN, TM = WM / 16, TN = WN / 16;
  constexpr int QA = BM / 4, UA = QA * (BK / 4);                // A micro-blocks (4 ch x 4 px) per stage
  constexpr int QB = BN / 4;                                    // B: BN/4 x 8 micro-blocks
  static_assert(TM >= 1 && TN >= 1 && UA <= NT && QB * (BK / 4) == NT, "tile");
  constexpr int SA = BM + 4, SB = BN + 4;                       // PX: floats per pixel row
  constexpr int STAGE = PX ? BK * (SA + SB) * 4 : (BM + BN) * RB;
  __shared__ __attribute__((aligned(16))) char lds[2][STAGE];

  const int T = a.KH * a.KW, Ncols = T * a.Nc;
  const int nmt = a.M / BM, nnt = (Ncols + BN - 1) / BN, tiles = nmt * nnt;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);     // a split's tiles (same pixels) share an XCD's L2
  const int split = bid / tiles, tile = bid - split * tiles;
  const int nt = tile / nmt, mt = tile - nt * nmt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int P = a.N * a.Hg * a.Wg, hw = a.Hg * a.Wg;
  const int p0 = (int)((long)split * a.pix_per_split);
  const int p1 = p0 + (int)a.pix_per_split < P ? p0 + (int)a.pix_per_split : P;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4, l16 = lane & 15;
  const int wm = wid / NWN, wn = wid - wm * NWN;
  // loader micro-blocks: A channels m0 + 4 qa, pixels 4 pa ..; B columns n0 + 4 qb -> (tap, n), pixels 4 pb ..
  const bool has_a = tid < UA;
  const int qa = tid % QA, pa = tid / QA;
  const int qb = tid % QB, pbq = tid / QB;
  const int bcol = n0 + 4 * qb;
  const bool bok = bcol < Ncols;
  const int btap = bok ? bcol / a.Nc : 0, bn = bcol - btap * a.Nc;
  const int bkh = btap / a.KW, bkw = btap - bkh * a.KW;
  const bool do_bias = a.bslab != nullptr && nt == 0;
  f32x4v bsum = f32x4v{0.f, 0.f, 0.f, 0.f};
  f32x4v va[4], vb[4];

  auto gload = [&](int pb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int p = pb + 4 * pa + e;
      va[e] = has_a && p < p1 ? *reinterpret_cast<const f32x4v*>(a.A + (long)p * a.lda + m0 + 4 * qa)
                              : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    // (n, h, w) of the quad's first pixel, then stepped one pixel at a time (one division per quad)
    const int pq0 = pb + 4 * pbq;
    int n = pq0 / hw, h = (pq0 - n * hw) / a.Wg, w = pq0 - n * hw - h * a.Wg;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      vb[e] = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (bok && pq0 + e < p1) {
        const int bh = h * a.s + bkh - a.pad, bw = w * a.s + bkw - a.pad;
        if (bh >= 0 && bh < a.HB && bw >= 0 && bw < a.WB)
          vb[e] = *reinterpret_cast<const f32x4v*>(a.B + ((long)(n * a.HB + bh) * a.WB + bw) * a.ldb + bn);
      }
      if (++w == a.Wg) {
        w = 0;
        if (++h == a.Hg) h = 0, ++n;
      }
    }
  };
  // column jj of a 4 x 4 micro-block (selects, no dynamic register indexing)
  auto colv = [](const f32x4v (&v)[4], int jj) {
    f32x4v o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = jj == 0 ? v[e][0] : jj == 1 ? v[e][1] : jj == 2 ? v[e][2] : v[e][3];
    return o;
  };
  auto lstore = [&](int buf) {
    if constexpr (PX) {
      float* As = reinterpret_cast<float*>(lds[buf]);
      float* Bs = As + BK * SA;
      if (has_a) {
#pragma unroll
        for (int e = 0; e < 4; ++e) *reinterpret_cast<f32x4v*>(As + (4 * pa + e) * SA + 4 * qa) = va[e];
        if (do_bias) bsum += va[0] + va[1] + va[2] + va[3];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) *reinterpret_cast<f32x4v*>(Bs + (4 * pbq + e) * SB + 4 * qb) = vb[e];
      return;
    }
    char* As = lds[buf];
    char* Bs = lds[buf] + BM * RB;
    if (has_a) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {           // rotated by the channel quad: both row parities per store
        const int jj = (j + qa) & 3, r = 4 * qa + jj;
        *reinterpret_cast<f32x4v*>(As + r * RB + wswz(r, pa) * 16) = colv(va, jj);
      }
      if (do_bias) bsum += va[0] + va[1] + va[2] + va[3];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = (j + qb) & 3, r = 4 * qb + jj;
      *reinterpret_cast<f32x4v*>(Bs + r * RB + wswz(r, pbq) * 16) = colv(vb, jj);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int S = (p1 - p0 + BK - 1) / BK;
  gload(p0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int buf = s & 1;
    if (s + 1 < S) gload(p0 + (s + 1) * BK);
    if constexpr (PX) {
      const float* As = reinterpret_cast<const float*>(lds[buf]) + wm * WM + l16;
      const float* Bs = reinterpret_cast<const float*>(lds[buf]) + BK * SA + wn * WN + l16;
#pragma unroll
      for (int kb = 0; kb < BK / 16; ++kb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 16 * kb + 4 * q + e;
          float av[TM], bv[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) av[i] = As[row * SA + i * 16];
#pragma unroll
          for (int j = 0; j < TN; ++j) bv[j] = Bs[row * SB + j * 16];
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      if (s + 1 < S) lstore(buf ^ 1);
      __syncthreads();
      continue;
    }
    const char* As = lds[buf];
    const char* Bs = lds[buf] + BM * RB;
#pragma unroll
    for (int kb = 0; kb < BK / 16; ++kb) {
      const int ch = 4 * kb + q;
      f32x4v af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + l16;
        af[i] = *reinterpret_cast<const f32x4v*>(As + r * RB + wswz(r, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + l16;
        bf[j] = *reinterpret_cast<const f32x4v*>(Bs + r * RB + wswz(r, ch) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma4(af[i], bf[j], acc[i][j]);
    }
    if (s + 1 < S) lstore(buf ^ 1);
    __syncthreads();
  }
  // slab[split][tap][m][n]: lane holds rows (m) 4 q + r of column l16
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + l16;
    if (col >= Ncols) continue;
    const int tap = col / a.Nc, n = col - tap * a.Nc;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + 4 * q + r;
        a.slab[(((long)split * T + tap) * a.M + m) * a.Nc + n] = acc[i][j][r];
      }
  }
  if (do_bias) {                                  // A micro-block rows pa -> sum over the 8 pixel quads
    float* red = reinterpret_cast<float*>(lds[0]);
    if (has_a) *reinterpret_cast<f32x4v*>(&red[pa * BM + 4 * qa]) = bsum;
    __syncthreads();
    if (tid < BM) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < BK / 4; ++k) sum += red[k * BM + tid];
      a.bslab[(long)split * a.M + m0 + tid] = sum;
    }
  }
}

// 3x3 / stride-1 / pad-1 weight gradient for the shallow levels (B channels NC = 32 / 64, A channels in
// blocks of 32): a stage is a 2-row x 32-pixel patch; its B halo (4 rows x 34 pixels x NC) is fetched
// once and stored K-contiguous in three column-shifted copies ([kw][halo row][n][32 px], one per kernel
// column, so every tap's operand is an aligned float4 of 4 pixels), and all 9 taps read from it: B is
// fetched ~1.2x per pixel instead of once per tap-column tile.  Block = 32 A channels x all 9 NC columns:
// (m-tile, n-tile) pairs over the 4 waves, each pair with its 9 taps in registers; one ds_read_b128 per 4
// MFMAs as in the generic form.  Single LDS buffer, the next stage's loads in registers during the
// current one.  Stages are enumerated (n, row pair, 32-px segment); a split is a contiguous range of
// stages, reduced like the generic form.
template <int NC>
__global__ __launch_bounds__(256) void wgrad3_f32_kernel(F32WgradArgs a) {
  constexpr int SR = 2, SW = 32, RB = 128;                      // stage rows, pixels per row, LDS row bytes
  constexpr int NT = NC / 16, PW = 2 * NT / 4;                  // n-tiles, (mt, nt) pairs per wave
  constexpr int QN = NC / 4, UB = (SR + 2) * 8 * QN, LBI = UB / 256;   // B micro-blocks (4 ch x 4 shifted px)
  static_assert(PW >= 1 && 2 * NT % 4 == 0 && UB % 256 == 0, "tile");
  constexpr int AROWS = SR * 32, BROWS = 3 * (SR + 2) * NC;     // A rows (r, m); B rows (kw, hr, n)
  __shared__ __attribute__((aligned(16))) char lds[(AROWS + BROWS) * RB];

  const int nmb = a.M / 32, nnb = a.Nc / NC, per_split = nmb * nnb;   // nnb = 2: 64 B channels as two 32-column halves
  const int bid = xcd_remap(blockIdx.x, per_split * a.splits);  // a split's blocks (same B halo) share an L2
  const int split = bid / per_split, rb0 = bid - split * per_split, nb = rb0 / nmb, mb = rb0 - nb * nmb;
  const int m0 = mb * 32, n0 = nb * NC;
  const int segs = a.Wg / SW, per_img = (a.Hg / SR) * segs;
  const int nst = a.N * per_img;
  const int sps = (int)(a.pix_per_split / (SR * SW));
  const int st0 = split * sps, st1 = st0 + sps < nst ? st0 + sps : nst;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4, l16 = lane & 15;
  const int mt = wid & 1, nt0 = (wid >> 1) * PW;
  // A micro-blocks (threads < 128): channels m0 + 4 qa, pixel quad pq (row pq / 8, chunk pq % 8)
  const bool has_a = tid < 128;
  const int qa = tid & 7, pq = (tid >> 3) & 15;
  const bool do_bias = a.bslab != nullptr && nb == 0;
  f32x4v bsum = f32x4v{0.f, 0.f, 0.f, 0.f};
  f32x4v va[4], vb[LBI][6];

  auto gload = [&](int st) {
    const int n = st / per_img, rem = st - n * per_img, hp = rem / segs;
    const int h0 = hp * SR, w0 = (rem - hp * segs) * SW;
    if (has_a) {
      const long pix = ((long)n * a.Hg + h0 + (pq >> 3)) * a.Wg + w0 + 4 * (pq & 7);
#pragma unroll
      for (int e = 0; e < 4; ++e) va[e] = *reinterpret_cast<const f32x4v*>(a.A + (pix + e) * a.lda + m0 + 4 * qa);
    }
#pragma unroll
    for (int i = 0; i < LBI; ++i) {
      const int u = tid + 256 * i, nq = u % QN, rest = u / QN, hr = rest >> 3, j = rest & 7;
      const int ih = h0 - 1 + hr;
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const int iw = w0 - 1 + 4 * j + e;
        vb[i][e] = f32x4v{0.f, 0.f, 0.f, 0.f};
        if (ih >= 0 && ih < a.HB && iw >= 0 && iw < a.WB)
          vb[i][e] = *reinterpret_cast<const f32x4v*>(a.B + ((long)(n * a.HB + ih) * a.WB + iw) * a.ldb + n0 + 4 * nq);
      }
    }
  };
  auto lstore = [&]() {
    if (has_a) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = (pq >> 3) * 32 + 4 * qa + c;
        *reinterpret_cast<f32x4v*>(lds + r * RB + fswzk<8>(r, pq & 7) * 16) = f32x4v{va[0][c], va[1][c], va[2][c], va[3][c]};
      }
      if (do_bias) bsum += va[0] + va[1] + va[2] + va[3];
    }
    char* Bs = lds + AROWS * RB;
#pragma unroll
    for (int i = 0; i < LBI; ++i) {
      const int u = tid + 256 * i, nq = u % QN, rest = u / QN, hr = rest >> 3, j = rest & 7;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int r = (kw * (SR + 2) + hr) * NC + 4 * nq + c;
          *reinterpret_cast<f32x4v*>(Bs + r * RB + fswzk<8>(r, j) * 16) =
              f32x4v{vb[i][kw][c], vb[i][kw + 1][c], vb[i][kw + 2][c], vb[i][kw + 3][c]};
        }
    }
  };

  f32x4_t acc[PW][9];
#pragma unroll
  for (int p = 0; p < PW; ++p)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[p][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (st0 < st1) gload(st0);
  for (int st = st0; st < st1; ++st) {
    lstore();
    __syncthreads();
    if (st + 1 < st1) gload(st + 1);
    const char* Bs = lds + AROWS * RB;
#pragma unroll
    for (int r = 0; r < SR; ++r)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int ch = 4 * cb + q;
        const int ra = r * 32 + mt * 16 + l16;
        const f32x4v af = *reinterpret_cast<const f32x4v*>(lds + ra * RB + fswzk<8>(ra, ch) * 16);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int p = 0; p < PW; ++p) {
            const int rb = ((t % 3) * (SR + 2) + r + t / 3) * NC + (nt0 + p) * 16 + l16;
            const f32x4v bf = *reinterpret_cast<const f32x4v*>(Bs + rb * RB + fswzk<8>(rb, ch) * 16);
            acc[p][t] = mfma4(af, bf, acc[p][t]);
          }
      }
    __syncthreads();
  }
  // slab[split][tap][m][n]: lane holds rows (m) 4 q + r of column l16
#pragma unroll
  for (int p = 0; p < PW; ++p)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + mt * 16 + 4 * q + r, n = (nt0 + p) * 16 + l16;
        a.slab[(((long)split * 9 + t) * a.M + m) * a.Nc + n0 + n] = acc[p][t][r];
      }
  if (do_bias) {                             // 16 pixel quads x 32 channels
    float* red = reinterpret_cast<float*>(lds);
    if (has_a) *reinterpret_cast<f32x4v*>(&red[pq * 32 + 4 * qa]) = bsum;
    __syncthreads();
    if (tid < 32) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sum += red[k * 32 + tid];
      a.bslab[(long)split * a.M + m0 + tid] = sum;
    }
  }
}

// First-layer weight gradient (3x3 / s1 / p1, 4 input channels -- the 3-channel image padded --, 32 output
// channels): 36 GEMM columns, so the 128-column tile of wgrad_f32_kernel is 72 % padding (0.57 ms at b16,
// 512^2, 13 TF/s).  Here the MFMA columns are (tap, channel) pairs plus one column of ones (the bias
// gradient), 3 n-tiles of 16, and both operands come straight from global memory: lane (q, l16) reads the
// output-gradient channel l16 of pixel 4 ks + q (64 B per 16 lanes) and the input value of its column at
// that pixel's tap position (L1 / L2 hits: the input is 16 B per pixel).  A wave walks 64-pixel row
// segments of its block's range; the 4 waves' sums meet in LDS in a fixed order and the block writes one
// slab row [9][32][4] (+ the bias row) for dpa_wgrad_reduce.
__global__ __launch_bounds__(256) void wgrad_c4_f32_kernel(F32WgradArgs a) {
  __shared__ float red[4][24][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4, l16 = lane & 15;
  const int segs = a.Wg / 64, units = a.N * a.Hg * segs;
  const int upb = (int)(a.pix_per_split / 64);
  const int u0 = blockIdx.x * upb, u1 = u0 + upb < units ? u0 + upb : units;
  // this lane's column of each n-tile: (tap offset, channel) or the ones column (36) or padding
  int dh[3], dw[3], cc[3], kind[3];
#pragma unroll
  for (int nt = 0; nt < 3; ++nt) {
    const int j = nt * 16 + l16, tap = j >> 2;
    kind[nt] = j < 36 ? 0 : j == 36 ? 1 : 2;
    dh[nt] = tap / 3 - 1;
    dw[nt] = tap % 3 - 1;
    cc[nt] = j & 3;
  }
  f32x4_t acc[2][3];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int u = u0 + wid; u < u1; u += 4) {
    const int n = u / (a.Hg * segs), rem = u - n * (a.Hg * segs), h = rem / segs, w0 = (rem - h * segs) * 64;
    const float* Ar = a.A + ((long)(n * a.Hg + h) * a.Wg + w0) * a.lda;
    float av[16][2], bv[16][3];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int w = w0 + 4 * ks + q;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) av[ks][mt] = Ar[(long)(4 * ks + q) * a.lda + mt * 16 + l16];
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const int ih = h + dh[nt], iw = w + dw[nt];
        float v = kind[nt] == 1 ? 1.f : 0.f;
        if (kind[nt] == 0 && ih >= 0 && ih < a.HB && iw >= 0 && iw < a.WB)
          v = a.B[((long)(n * a.HB + ih) * a.WB + iw) * a.ldb + cc[nt]];
        bv[ks][nt] = v;
      }
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks][mt], bv[ks][nt], acc[mt][nt], 0, 0, 0);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][(mt * 3 + nt) * 4 + r][lane] = acc[mt][nt][r];
  __syncthreads();
  // thread: lane L, 6 of the 24 (mt, nt, r) values; lane L of those holds rows 4 q + r, column l16
  const int L = lane, qq = L >> 4, col = L & 15;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int e = wid * 6 + i, mt = e / 12, nt = (e / 4) % 3, r = e & 3;
    const float v = ((red[0][e][L] + red[1][e][L]) + red[2][e][L]) + red[3][e][L];
    const int m = mt * 16 + 4 * qq + r, j = nt * 16 + col;
    if (j < 36) a.slab[(((long)blockIdx.x * 9 + (j >> 2)) * 32 + m) * 4 + (j & 3)] = v;
    else if (j == 36 && a.bslab) a.bslab[(long)blockIdx.x * 32 + m] = v;
  }
}

// ------------------------------------------------------------------------------------ elementwise
// y = g * (r > 0) over n floats (float4)
__global__ __launch_bounds__(256) void relu_bwd_f32_kernel(const float* __restrict__ g, const float* __restrict__ r,
                                                           float* __restrict__ y, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4v gv = reinterpret_cast<const f32x4v*>(g)[i], rv = reinterpret_cast<const f32x4v*>(r)[i];
    f32x4v o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = rv[e] > 0.f ? gv[e] : 0.f;
    reinterpret_cast<f32x4v*>(y)[i] = o;
  }
}

// 2x2/s2 max-pool (floor), NHWC dense C channels; code = argmax window position (first maximum,
// window order tl, tr, bl, br -- torch max_pool2d's choice)
__global__ __launch_bounds__(256) void maxpool2_f32_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                                           unsigned char* __restrict__ code, int N, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1;
  const long tot = (long)N * Ho * Wo * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int wo = (int)(pix % Wo), ho = (int)((pix / Wo) % Ho), n = (int)(pix / ((long)Wo * Ho));
    const float* b = x + (((long)n * H + 2 * ho) * W + 2 * wo) * ldx + c;
    const float v0 = b[0], v1 = b[ldx], v2 = b[(long)W * ldx], v3 = b[(long)W * ldx + ldx];
    float m = v0;
    unsigned k = 0;
    if (v1 > m) { m = v1; k = 1; }
    if (v2 > m) { m = v2; k = 2; }
    if (v3 > m) { m = v3; k = 3; }
    y[i] = m;
    code[i] = (unsigned char)k;
  }
}

// dx[2h+i][2w+j][c] = (code == 2i+j) ? g[h][w][c] : 0 over the whole input grid (odd last row/col: 0)
__global__ __launch_bounds__(256) void maxpool2_bwd_f32_kernel(const float* __restrict__ g, const unsigned char* __restrict__ code,
                                                               float* __restrict__ dx, int N, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1;
  const long tot = (long)N * H * W * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((long)W * H));
    const int ho = h >> 1, wo = w >> 1;
    float v = 0.f;
    if (ho < Ho && wo < Wo) {
      const long o = (((long)n * Ho + ho) * Wo + wo) * C + c;
      if (code[o] == (unsigned)((h & 1) * 2 + (w & 1))) v = g[o];
    }
    dx[i] = v;
  }
}

// encoder DoubleConv output gradient in one pass: ge = (y > 0) * (gs + [code == window position] gp) --
// the skip gradient (gs, pixel stride lds, may be null), the max-pool backward and the ReLU backward
// that autograd would run as three passes (scatter, add, mask); NHWC fp32, 4 channels per thread
__global__ __launch_bounds__(256) void enc_out_bwd_f32_kernel(const float* __restrict__ gs, int lds,
                                                              const float* __restrict__ gp,
                                                              const unsigned char* __restrict__ code,
                                                              const float* __restrict__ y, int ldy, float* __restrict__ ge,
                                                              int N, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1, C4 = C >> 2;
  const long tot = (long)N * H * W * C4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const long pix = i / C4;
    const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((long)W * H));
    f32x4v v = gs ? *reinterpret_cast<const f32x4v*>(gs + pix * lds + c) : f32x4v{0.f, 0.f, 0.f, 0.f};
    const int ho = h >> 1, wo = w >> 1;
    if (gp && ho < Ho && wo < Wo) {
      const long o = (((long)n * Ho + ho) * Wo + wo) * C + c;
      const f32x4v g = *reinterpret_cast<const f32x4v*>(gp + o);
      const unsigned k = (unsigned)((h & 1) * 2 + (w & 1));
      const uchar4 cd = *reinterpret_cast<const uchar4*>(code + o);
      v[0] += cd.x == k ? g[0] : 0.f;
      v[1] += cd.y == k ? g[1] : 0.f;
      v[2] += cd.z == k ? g[2] : 0.f;
      v[3] += cd.w == k ? g[3] : 0.f;
    }
    const f32x4v yv = *reinterpret_cast<const f32x4v*>(y + pix * ldy + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = yv[e] > 0.f ? v[e] : 0.f;
    *reinterpret_cast<f32x4v*>(ge + pix * C + c) = v;
  }
}

// segmentation head forward: z = b + sum_c w[c] y[p][c], p = sigmoid(z); per-block partial sums of
// [BCE(p, t), p * [t == 1], p, [t == 1]] (reference utils/utils.py:9-25, log clamped at -100 like
// torch's BCELoss) -> slab[block][4]; optional probabilities out
__global__ __launch_bounds__(256) void head_f32_kernel(const float* __restrict__ y, int C, const float* __restrict__ w,
                                                       const float* __restrict__ b, const float* __restrict__ t, long P,
                                                       float* __restrict__ slab, float* __restrict__ probs) {
  __shared__ float red[4][256];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    float z = b[0];
    for (int c = 0; c < C; ++c) z = fmaf(w[c], y[i * C + c], z);
    const float p = 1.f / (1.f + expf(-z));
    if (probs) probs[i] = p;
    if (t) {
      const float tt = t[i];
      const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
      s0 += -(tt * lp + (1.f - tt) * l1p);
      const float one = tt == 1.f ? 1.f : 0.f;
      s1 += p * one;
      s2 += p;
      s3 += one;
    }
  }
  if (!t) return;
  red[0][threadIdx.x] = s0; red[1][threadIdx.x] = s1; red[2][threadIdx.x] = s2; red[3][threadIdx.x] = s3;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x < 4) slab[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// The same head forward with L = C / 4 lanes per pixel, each loading one float4 of the pixel's row: a wave
// reads 64 / L whole rows per instruction (coalesced 1-KB runs at C = 32) instead of 64 lanes each walking
// its own row one float at a time (0.41 ms for 2.5 M pixels of 32 channels,
// profiles/hip_fp32_b4_640x960_summary_r06.txt).  z's channel sum: lane partials, then an xor tree over
// the pixel's lanes; the loss terms from lane 0 of each pixel (the formulas above).
template <int C>
__global__ __launch_bounds__(256) void head_f32_vec_kernel(const float* __restrict__ y, const float* __restrict__ w,
                                                           const float* __restrict__ b, const float* __restrict__ t,
                                                           long P, float* __restrict__ slab, float* __restrict__ probs) {
  constexpr int L = C / 4, PPB = 256 / L;          // lanes per pixel, pixels per block iteration
  __shared__ float red[4][256];
  const int sub = threadIdx.x % L;
  const f32x4v wv = *reinterpret_cast<const f32x4v*>(w + 4 * sub);
  const float bb = b[0];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (long i = (long)blockIdx.x * PPB + threadIdx.x / L; i < P; i += (long)gridDim.x * PPB) {
    const f32x4v v = *reinterpret_cast<const f32x4v*>(y + i * C + 4 * sub);
    float z = fmaf(wv[3], v[3], fmaf(wv[2], v[2], fmaf(wv[1], v[1], wv[0] * v[0])));
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
    z += bb;
    if (sub == 0) {
      const float p = 1.f / (1.f + expf(-z));
      if (probs) probs[i] = p;
      if (t) {
        const float tt = t[i];
        const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
        s0 += -(tt * lp + (1.f - tt) * l1p);
        const float one = tt == 1.f ? 1.f : 0.f;
        s1 += p * one;
        s2 += p;
        s3 += one;
      }
    }
  }
  if (!t) return;
  red[0][threadIdx.x] = s0; red[1][threadIdx.x] = s1; red[2][threadIdx.x] = s2; red[3][threadIdx.x] = s3;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x < 4) slab[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// head backward: dL/dz per pixel from dS (gradient w.r.t. the four partial sums), torch's BCE backward through
// the sigmoid (common.h head_dz, shared with the bf16 head kernels); gy[p][c] = dz w[c]; per-block partials of
// sum_p dz y[p][c] (C) and sum_p dz (1) -> slab[block][C + 1].  L = C / 4 lanes per pixel (float4 loads of y
// and stores of gy, as above); every lane
// of a pixel forms dz itself; channel partials of dz y in the 4 channels a lane owns, reduced per block in
// LDS in a fixed order (rows = the block's pixel slots), the bias partial (dz) from lane 0 of each pixel.
// relu: gy is also ReLU-backward masked by y > 0 (y = the last decoder block's ReLU output, so its ReLU
// backward pass over the full-resolution gradient disappears; the parameter partials use dz as before).
template <int C>
__global__ __launch_bounds__(256) void head_bwd_f32_vec_kernel(const float* __restrict__ y, const float* __restrict__ w,
                                                               const float* __restrict__ b, const float* __restrict__ t,
                                                               const float* __restrict__ dS, long P, float* __restrict__ gy,
                                                               float* __restrict__ slab, int relu) {
  constexpr int L = C / 4, PPB = 256 / L;
  __shared__ float red[PPB][C + 1];
  const int sub = threadIdx.x % L, slot = threadIdx.x / L;
  const f32x4v wv = *reinterpret_cast<const f32x4v*>(w + 4 * sub);
  const float bb = b[0], d0 = dS[0], d1 = dS[1], d2 = dS[2];
  f32x4v acc = f32x4v{0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  for (long i = (long)blockIdx.x * PPB + slot; i < P; i += (long)gridDim.x * PPB) {
    const f32x4v v = *reinterpret_cast<const f32x4v*>(y + i * C + 4 * sub);
    float z = fmaf(wv[3], v[3], fmaf(wv[2], v[2], fmaf(wv[1], v[1], wv[0] * v[0])));
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
    z += bb;
    const float p = 1.f / (1.f + expf(-z));
    const float tt = t[i];
    const float dz = head_dz(p, tt, tt == 1.f ? 1.f : 0.f, d0, d1, d2);
    f32x4v o = dz * wv;
    if (relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = v[r] > 0.f ? o[r] : 0.f;
    }
    *reinterpret_cast<f32x4v*>(gy + i * C + 4 * sub) = o;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaf(dz, v[r], acc[r]);
    accb += dz;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[slot][4 * sub + r] = acc[r];
  if (sub == 0) red[slot][C] = accb;
  __syncthreads();
  if ((int)threadIdx.x <= C) {
    float s = 0.f;
    for (int k = 0; k < PPB; ++k) s += red[k][threadIdx.x];
    slab[(long)blockIdx.x * (C + 1) + threadIdx.x] = s;
  }
}


// NCHW fp32 (C <= 4) -> NHWC fp32 with 4 channels (zero padded)
__global__ __launch_bounds__(256) void nchw_to_nhwc4_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int N,
                                                                int C, long HW) {
  const long tot = (long)N * HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW, p = i - n * HW;
    f32x4v v = f32x4v{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; ++c) v[c] = x[(n * C + c) * HW + p];
    reinterpret_cast<f32x4v*>(y)[i] = v;
  }
}

// per-channel sums of an NHWC tensor into slab[block][C] (bias gradient of the transposed conv): block b
// sums pixels b, b + gridDim.x, ... ; thread (c, r) takes channel c (+ 256 k for C > 256) of row group r
__global__ __launch_bounds__(256) void channel_sum_f32_kernel(const float* __restrict__ g, long P, int C, int ld,
                                                              float* __restrict__ slab) {
  __shared__ float red[256];
  const int R = C < 256 ? 256 / C : 1;               // host: C < 256 divides 256
  const int r = threadIdx.x / (C < 256 ? C : 256);
  for (int c = threadIdx.x % (C < 256 ? C : 256); c < C; c += 256) {
    float s = 0.f;
    for (long p = (long)blockIdx.x * R + r; p < P; p += (long)gridDim.x * R) s += g[p * ld + c];
    __syncthreads();
    red[threadIdx.x] = s;
    __syncthreads();
    if (r == 0) {
      for (int k = 1; k < R; ++k) s += red[k * C + c];
      slab[(long)blockIdx.x * C + c] = s;
    }
  }
}

static unsigned egrid(long n) { return (unsigned)(n / 256 + 1 < 8192 ? n / 256 + 1 : 8192); }

// Eligible: Cs % 4 == 0 (a float4 chunk never straddles a tap), Kpad % 16 == 0, Kpad >= KH*KW*Cs,
// Ngemm % 32 == 0, 16-B aligned strides; mode 1 also Cout % 4 == 0.
// Tiles (32-deep K-steps when Kpad % 32 == 0): Ngemm % 128 == 0 -> 128 px x 128 ch (K32); Ngemm % 64 == 0 ->
// 128 x 64; else 128 x 32; Ngemm 64 over <= 64 / Ngemm 32 over 32 input channels: 256 x Ngemm with 16-deep
// K-steps (the 32-deep 256-pixel form measured 5-17 % slower: 72-80 KB of LDS).
DPA_API int dpa_igemm_f32(const F32ConvArgs* args, hipStream_t st) {
  const F32ConvArgs& a = *args;
  if ((a.Cs & 3) || (a.Kpad % F_BK) || a.Kpad < a.KH * a.KW * a.Cs || (a.Ngemm & 31) || (a.ldx & 3) || (a.ldy & 3) ||
      (a.mask && (a.ldm & 3)) || (a.mode == 1 && (a.Cout & 3)) || a.KH * a.KW > 32 || a.N < 1)
    return (int)hipErrorInvalidValue;
  const long M = (long)a.N * a.Ho * a.Wo;
  const bool k32 = a.Kpad % 32 == 0;
  if (a.halo && a.mode == 0 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Hs == a.Ho &&
      a.Ws == a.Wo && a.Ho % 8 == 0 && a.Wo % 32 == 0 && a.Cs % 32 == 0 && a.Kpad >= 9 * a.Cs &&
      (a.Ngemm == 32 || (a.halo == 2 && a.Ngemm == 64))) {
    const dim3 grid((unsigned)(M / 256 * (a.Ngemm / 32)));
    hipLaunchKernelGGL(conv3_halo_f32_kernel, grid, dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  if (k32 && a.mode == 0 && ((a.Ngemm == 64 && a.Cs <= 64) || (a.Ngemm == 32 && a.Cs == 32))) {
    // narrow GEMM-N over few input channels: 256-pixel tiles, 16-deep K-steps (36-40 KB LDS)
    const dim3 grid((unsigned)((M + 255) / 256));
    if (a.Ngemm == 64) hipLaunchKernelGGL((igemm_f32_kernel<256, 64, 4, 16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((igemm_f32_kernel<256, 32, 4, 16>), grid, dim3(256), 0, st, a);
  } else if (a.Ngemm % 128 == 0 && k32 && a.wide && ((M + 255) / 256) * (a.Ngemm / 128) >= 512) {
    // one 96 KB block of 8 waves per CU: only with >= 2 blocks per CU of work (a 32^2 deep layer at b16 has
    // 256 and runs 30 % slower on it, profiles/f32_kbench_b16_512_r05_wide.txt)
    const dim3 grid((unsigned)(((M + 255) / 256) * (a.Ngemm / 128)));
    if (a.Ngemm == 128 || a.mode == 1) hipLaunchKernelGGL((igemm_f32_kernel<256, 128, 4, 16, 8>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((igemm_f32_kernel<256, 128, 4, 32, 8>), grid, dim3(512), 0, st, a);
  } else if (a.Ngemm % 128 == 0 && k32) {
    const dim3 grid((unsigned)(((M + 127) / 128) * (a.Ngemm / 128)));
    // 16-deep K-steps (32 KB of LDS, 3 waves / SIMD) measured faster for a single 128-wide GEMM-N tile and
    // the transposed conv's scatter; 32-deep for the wider layers (profiles/f32_kbench_b16_512_r04.txt)
    if (a.Ngemm == 128 || a.mode == 1) hipLaunchKernelGGL((igemm_f32_kernel<128, 128, 2, 16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((igemm_f32_kernel<128, 128, 2, 32>), grid, dim3(256), 0, st, a);
  } else if (a.Ngemm % 64 == 0) {
    const dim3 grid((unsigned)(((M + 127) / 128) * (a.Ngemm / 64)));
    if (k32) hipLaunchKernelGGL((igemm_f32_kernel<128, 64, 2, 32>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((igemm_f32_kernel<128, 64, 2, 16>), grid, dim3(256), 0, st, a);
  } else {
    const dim3 grid((unsigned)(((M + 127) / 128) * (a.Ngemm / 32)));
    if (k32) hipLaunchKernelGGL((igemm_f32_kernel<128, 32, 4, 32>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((igemm_f32_kernel<128, 32, 4, 16>), grid, dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

// Eligible: M % 32 == 0, Nc % 4 == 0, lda / ldb % 4 == 0, pix_per_split % 32 == 0, splits covering all
// pixels.  BM = 128 / 64 / 32 A channels per tile (the largest dividing M).
// block tile rows (A channels); 256 -> the 256 x 256 8-wave tile (deep layers, opt-in by the host's `big`)
static int wgrad_f32_bm(int M, int Ncols, int big) {   // ops/fp32.py wgrad_f32_tile mirrors it
  if (big && M == 256 && Ncols >= 9 * 256) return 256;
  return M % 128 == 0 ? 128 : M % 64 == 0 ? 64 : 32;
}

DPA_API int dpa_wgrad_f32(const F32WgradArgs* args, hipStream_t st) {
  const F32WgradArgs& a = *args;
  const long P = (long)a.N * a.Hg * a.Wg;
  if ((a.M & 31) || (a.Nc & 3) || (a.lda & 3) || (a.ldb & 3) || a.pix_per_split < 32 || (a.pix_per_split % 32) ||
      a.splits < 1 || (long)a.splits * a.pix_per_split < P || (long)(a.splits - 1) * a.pix_per_split >= P ||
      a.KH * a.KW < 1 || P >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if (a.halo == 3) {      // first layer: 4 input channels, 32 outputs, 64-pixel row segments per split unit
    if (a.KH != 3 || a.KW != 3 || a.s != 1 || a.pad != 1 || a.HB != a.Hg || a.WB != a.Wg || a.Nc != 4 || a.M != 32 ||
        (a.Wg % 64) || (a.pix_per_split % 64))
      return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(wgrad_c4_f32_kernel, dim3((unsigned)a.splits), dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  if (a.halo) {
    if (a.KH != 3 || a.KW != 3 || a.s != 1 || a.pad != 1 || a.HB != a.Hg || a.WB != a.Wg || (a.Hg & 1) ||
        (a.Wg % 32) || (a.pix_per_split % 64) || (a.Nc != 32 && a.Nc != 64))
      return (int)hipErrorInvalidValue;
    // halo == 2 with 64 columns: the 32-column kernel over each half (56 KB of LDS, 2 blocks per CU, vs one
    // 104 KB block of the 64-column form)
    const bool halves = a.Nc == 64 && a.halo == 2;
    const dim3 grid((unsigned)((a.M / 32) * (halves ? 2 : 1) * a.splits));
    if (a.Nc == 32 || halves) hipLaunchKernelGGL(wgrad3_f32_kernel<32>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(wgrad3_f32_kernel<64>, grid, dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  const int T = a.KH * a.KW, bm = wgrad_f32_bm(a.M, T * a.Nc, a.big), bn = bm == 256 ? 256 : 128;
  const long tiles = (long)(a.M / bm) * ((T * a.Nc + bn - 1) / bn);
  const dim3 grid((unsigned)(tiles * a.splits));
  if (a.px) {
    if (bm == 256) hipLaunchKernelGGL((wgrad_f32_kernel<256, 256, true>), grid, dim3(512), 0, st, a);
    else if (bm == 128) hipLaunchKernelGGL((wgrad_f32_kernel<128, 128, true>), grid, dim3(256), 0, st, a);
    else if (bm == 64) hipLaunchKernelGGL((wgrad_f32_kernel<64, 128, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((wgrad_f32_kernel<32, 128, true>), grid, dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  if (bm == 256) hipLaunchKernelGGL((wgrad_f32_kernel<256, 256>), grid, dim3(512), 0, st, a);
  else if (bm == 128) hipLaunchKernelGGL((wgrad_f32_kernel<128, 128>), grid, dim3(256), 0, st, a);
  else if (bm == 64) hipLaunchKernelGGL((wgrad_f32_kernel<64, 128>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((wgrad_f32_kernel<32, 128>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

DPA_API int dpa_relu_bwd_f32(const float* g, const float* r, float* y, long long n, hipStream_t st) {
  if (n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(relu_bwd_f32_kernel, dim3(egrid(n / 4)), dim3(256), 0, st, g, r, y, (long)(n / 4));
  return (int)hipGetLastError();
}

DPA_API int dpa_maxpool2_f32(const float* x, int ldx, float* y, unsigned char* code, int N, int H, int W, int C,
                             hipStream_t st) {
  if (H < 2 || W < 2 || C < 1) return (int)hipErrorInvalidValue;
  if (ldx < C) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool2_f32_kernel, dim3(egrid((long)N * (H / 2) * (W / 2) * C)), dim3(256), 0, st, x, ldx, y, code, N, H,
                     W, C);
  return (int)hipGetLastError();
}

DPA_API int dpa_maxpool2_bwd_f32(const float* g, const unsigned char* code, float* dx, int N, int H, int W, int C,
                                 hipStream_t st) {
  if (H < 2 || W < 2 || C < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool2_bwd_f32_kernel, dim3(egrid((long)N * H * W * C)), dim3(256), 0, st, g, code, dx, N, H, W, C);
  return (int)hipGetLastError();
}

DPA_API int dpa_enc_out_bwd_f32(const float* gs, int lds, const float* gp, const unsigned char* code, const float* y,
                                int ldy, float* ge, int N, int H, int W, int C, hipStream_t st) {
  if (H < 1 || W < 1 || (C & 3) || (gs && (lds & 3)) || (ldy & 3) || ldy < C || (gp && (H < 2 || W < 2)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(enc_out_bwd_f32_kernel, dim3(egrid((long)N * H * W * (C / 4))), dim3(256), 0, st, gs, lds, gp, code, y,
                     ldy, ge, N, H, W, C);
  return (int)hipGetLastError();
}

// head forward over P pixels of C channels: slab needs blocks * 4 floats (blocks = dpa_head_f32_blocks)
DPA_API int dpa_head_f32_blocks(long long P) { return (int)(P / 256 + 1 < 1024 ? P / 256 + 1 : 1024); }

DPA_API int dpa_head_f32(const float* y, int C, const float* w, const float* b, const float* t, long long P, float* slab,
                         float* probs, hipStream_t st) {
  if (C < 1) return (int)hipErrorInvalidValue;
  const dim3 grid(dpa_head_f32_blocks(P));
  switch (C) {
    case 8: hipLaunchKernelGGL(head_f32_vec_kernel<8>, grid, dim3(256), 0, st, y, w, b, t, (long)P, slab, probs); break;
    case 16: hipLaunchKernelGGL(head_f32_vec_kernel<16>, grid, dim3(256), 0, st, y, w, b, t, (long)P, slab, probs); break;
    case 32: hipLaunchKernelGGL(head_f32_vec_kernel<32>, grid, dim3(256), 0, st, y, w, b, t, (long)P, slab, probs); break;
    case 64: hipLaunchKernelGGL(head_f32_vec_kernel<64>, grid, dim3(256), 0, st, y, w, b, t, (long)P, slab, probs); break;
    default: hipLaunchKernelGGL(head_f32_kernel, grid, dim3(256), 0, st, y, C, w, b, t, (long)P, slab, probs);
  }
  return (int)hipGetLastError();
}

DPA_API int dpa_head_bwd_f32(const float* y, int C, const float* w, const float* b, const float* t, const float* dS,
                             long long P, float* gy, float* slab, int relu, hipStream_t st) {
  const dim3 grid(dpa_head_f32_blocks(P));
  switch (C) {
    case 8: hipLaunchKernelGGL(head_bwd_f32_vec_kernel<8>, grid, dim3(256), 0, st, y, w, b, t, dS, (long)P, gy, slab, relu); break;
    case 16: hipLaunchKernelGGL(head_bwd_f32_vec_kernel<16>, grid, dim3(256), 0, st, y, w, b, t, dS, (long)P, gy, slab, relu); break;
    case 32: hipLaunchKernelGGL(head_bwd_f32_vec_kernel<32>, grid, dim3(256), 0, st, y, w, b, t, dS, (long)P, gy, slab, relu); break;
    case 64: hipLaunchKernelGGL(head_bwd_f32_vec_kernel<64>, grid, dim3(256), 0, st, y, w, b, t, dS, (long)P, gy, slab, relu); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

DPA_API int dpa_nchw_to_nhwc4_f32(const float* x, float* y, int N, int C, long long HW, hipStream_t st) {
  if (C < 1 || C > 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(nchw_to_nhwc4_f32_kernel, dim3(egrid((long)N * HW)), dim3(256), 0, st, x, y, N, C, (long)HW);
  return (int)hipGetLastError();
}

// slab rows = dpa_head_f32_blocks(P) (same grid policy)
DPA_API int dpa_channel_sum_f32(const float* g, long long P, int C, int ld, float* slab, hipStream_t st) {
  if (C < 1 || (C < 256 && 256 % C) || (C > 256 && C % 256)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(channel_sum_f32_kernel, dim3(dpa_head_f32_blocks(P)), dim3(256), 0, st, g, (long)P, C, ld, slab);
  return (int)hipGetLastError();
}
