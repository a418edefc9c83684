// Weight gradients of the UNet convolutions on MFMA (gfx950): split-K over pixels, all taps of a
// tile inside one block, deterministic two-stage reduction (reference
// layers model/unet_parts.py:10-12 Conv2d, :51-54 ConvTranspose2d).
//
//   out[tap][m][n] = sum_{p in pixel grid} A[srcA(p,tap)][m] * B[srcB(p,tap)][n]
//     conv3x3   : A = grad of conv output g[p][co] (tap independent), B = conv input x shifted by the
//                 tap (zero padded)                 -> dW[co][ci][kh][kw]
//     convT 2x2 : A = grad of the upsampled output gathered at (2h+i, 2w+j), B = input x[p][ci]
//                 -> dW[ci][co][i][j]
//
// GEMM K is the pixel dimension (up to N*H*W = 8.4M at 512^2, batch 32), so each block handles one
// (m-tile, n-tile) pair for ALL taps over a contiguous range of pixels (its split) and writes an fp32
// slab; `dpa_wgrad_reduce` sums the slabs in a fixed order (bitwise reproducible, no atomics) and
// accumulates into the flat fp32 gradient buffer in the PyTorch parameter layout.
//
// Both operands are channel-contiguous in memory with K (=pixels) as the row index, so tiles are
// staged as [32 pixels][channels] LDS images (16-B chunks, XOR swizzled) and fragments are read with
// the gfx950 transposed LDS read ds_read_b64_tr_b16, conflict-free for 64/128/256-byte rows.
// The tap-independent operand is staged once per pixel chunk and reused by all taps (9 for conv).
// Bias gradients (sum of A over pixels) come from the n-tile-0 blocks' LDS images.
#include "conv_args.h"



template <int BM, int BN, int WM, int WN, int T, bool TAPA>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void wgrad_kernel(WgradArgs a) {
  constexpr int NWN = BN / WN, NW = (BM / WM) * NWN, NT = 64 * NW;
  constexpr int TA = TAPA ? T : 1, TB = TAPA ? 1 : T;
  constexpr int CPRA = BM / 8, CPRB = BN / 8, RBA = BM * 2, RBB = BN * 2;
  constexpr int IMGA = 32 * RBA, IMGB = 32 * RBB;
  constexpr int CHA = TA * CPRA, CH = CHA + TB * CPRB;   // 16-B chunks per pixel per stage
  constexpr int SLOTS = NT / 32;
  constexpr int L = (CH + SLOTS - 1) / SLOTS;
  constexpr int TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) char lds[TA * IMGA + TB * IMGB];

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
  const int nst = (int)((pend - pbeg + 31) / 32);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid - wm * NWN;
  const int lpx = tid / SLOTS, lslot = tid - lpx * SLOTS;
  const bool do_bias = a.bslab != nullptr && nt == 0;

  u32x4_t reg[L];
  // zero padding / channel tails via the buffer range check (no branch per load, see igemm.hip)
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)a.abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)a.bbytes, 0x00020000);
  auto gload = [&](int st) {
    const long p = pbeg + (long)st * 32 + lpx;
    const bool pok = p < pend;
    int n = 0, h = 0, w = 0;
    {
      const int hw = a.Hg * a.Wg;
      const int pp = pok ? (int)p : 0;
      n = pp / hw;
      const int rem = pp - n * hw;
      h = rem / a.Wg;
      w = rem - h * a.Wg;
    }
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int c = lslot + j * SLOTS;
      if (c < CH) {
        const bool isA = c < CHA;
        const int cl = isA ? c : c - CHA;
        const int cpr = isA ? CPRA : CPRB;
        const int tap = cl / cpr, cc = cl - tap * cpr;
        const bool dep = (isA == TAPA);
        int ih = h, iw = w;
        const int H = isA ? a.HA : a.HB, W = isA ? a.WA : a.WB;
        if (dep) {
          const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
          ih = h * a.s + kh - a.pad;
          iw = w * a.s + kw - a.pad;
        }
        const int ch = (isA ? m0 : n0) + cc * 8;
        const int nch = isA ? a.M : a.Nc;
        const bool ok = pok && ih >= 0 && ih < H && iw >= 0 && iw < W && ch < nch;
        const int ld = isA ? a.lda : a.ldb;
        const unsigned off = ok ? (unsigned)((((n * H + ih) * W + iw) * ld + ch) * 2) : 0x80000000u;
        reg[j] = isA ? __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0) : __builtin_amdgcn_raw_buffer_load_b128(br, off, 0, 0);
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int c = lslot + j * SLOTS;
      if (c < CH) {
        if (c < CHA) {
          const int tap = c / CPRA, cc = c - tap * CPRA;
          *reinterpret_cast<u32x4_t*>(lds + tap * IMGA + lpx * RBA + ((cc ^ swz_kk<RBA>(lpx)) << 4)) = reg[j];
        } else {
          const int cl = c - CHA, tap = cl / CPRB, cc = cl - tap * CPRB;
          *reinterpret_cast<u32x4_t*>(lds + TA * IMGA + tap * IMGB + lpx * RBB + ((cc ^ swz_kk<RBB>(lpx)) << 4)) = reg[j];
        }
      }
    }
  };

  f32x4_t acc[T][TM][TN];
#pragma unroll
  for (int t = 0; t < T; ++t)
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
    if constexpr (TAPA) {
      bf16x8_t bf[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = tr_frag<RBB>(lds + TA * IMGA, wn * WN + j * 16, lane);
#pragma unroll
      for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8_t af = tr_frag<RBA>(lds + t * IMGA, wm * WM + i * 16, lane);
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[t][i][j], 0, 0, 0);
        }
      }
    } else {
      bf16x8_t af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag<RBA>(lds, wm * WM + i * 16, lane);
#pragma unroll
      for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const bf16x8_t bf = tr_frag<RBB>(lds + TA * IMGA + t * IMGB, wn * WN + j * 16, lane);
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[t][i][j], 0, 0, 0);
        }
      }
    }
    if (do_bias && tid < BM) {
      const int ch = tid >> 3, e = tid & 7;
#pragma unroll
      for (int t = 0; t < TA; ++t)
        for (int r = 0; r < 32; ++r) {
          const bf16_t v = *reinterpret_cast<const bf16_t*>(lds + t * IMGA + r * RBA + ((ch ^ swz_kk<RBA>(r)) << 4) + e * 2);
          bsum += bf2f(v);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (st + 1 < nst) {
      lstore();
      __syncthreads();
    }
  }

  // epilogue: fp32 partial slab for this split
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (n >= a.Nc) continue;
        const int mb = m0 + wm * WM + i * 16 + 4 * (lane >> 4);
        float* dst = a.slab + (((long)split * T + t) * a.M + mb) * a.Nc + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(long)r * a.Nc] = acc[t][i][j][r];
      }
  if (do_bias && tid < BM) a.bslab[(long)split * a.M + m0 + tid] = bsum;
}

template <int BM, int BN, int WM, int WN, int T, bool TAPA>
static int launch_wgrad(const WgradArgs& a, hipStream_t st) {
  const int tiles = (a.M / BM) * ((a.Nc + BN - 1) / BN);
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, T, TAPA>), dim3(tiles * a.splits), dim3(NT), 0, st, a);
  return (int)hipGetLastError();
}

// kind: 0 = conv3x3 (T=9, B tap-dependent), 1 = transposed conv 2x2/s2 (T=4, A tap-dependent),
//       2 = conv1x1 (T=1; the bilinear Up path's projection).
// cfg: 0 = auto; otherwise a tile id (see switch).  M % BM == 0 is required.
DPA_API int dpa_wgrad(const WgradArgs* args, int kind, int cfg, hipStream_t st) {
  const WgradArgs& a = *args;
  if ((a.M & 31) || (a.lda & 7) || (a.ldb & 7) || (a.pix_per_split & 31) || a.splits < 1) return (int)hipErrorInvalidValue;
  if (cfg == 0) {
    if (kind == 0) cfg = (a.Nc <= 16) ? 1 : (a.M >= 64 && a.Nc >= 32) ? 3 : 2;
    // transposed conv: the 64 x 128 tile is ~30% faster than 64 x 64 on D1/D2 at batch 128 (kbench --dwcfg)
    else if (kind == 1) cfg = (a.M % 64 == 0 && a.Nc % 128 == 0) ? 14 : (a.M >= 64 && a.Nc >= 64) ? 12 : 11;
    else cfg = (a.M % 64 == 0 && a.Nc >= 64) ? 22 : 21;
  }
  if (kind == 0) {
    switch (cfg) {
      case 1: if (a.M % 32) break; return launch_wgrad<32, 16, 16, 16, 9, false>(a, st);   // first layer (Cin<=16)
      case 2: if (a.M % 32) break; return launch_wgrad<32, 32, 16, 16, 9, false>(a, st);
      case 3: if (a.M % 64) break; return launch_wgrad<64, 32, 32, 16, 9, false>(a, st);
      case 4: if (a.M % 64) break; return launch_wgrad<64, 64, 32, 32, 9, false>(a, st);
      default: break;
    }
  } else if (kind == 2) {
    switch (cfg) {
      case 21: if (a.M % 32) break; return launch_wgrad<32, 32, 16, 16, 1, false>(a, st);
      case 22: if (a.M % 64) break; return launch_wgrad<64, 64, 32, 32, 1, false>(a, st);
      default: break;
    }
  } else {
    switch (cfg) {
      case 11: if (a.M % 32) break; return launch_wgrad<32, 32, 16, 16, 4, true>(a, st);
      case 12: if (a.M % 64) break; return launch_wgrad<64, 64, 32, 32, 4, true>(a, st);
      case 13: if (a.M % 128) break; return launch_wgrad<128, 64, 64, 32, 4, true>(a, st);
      case 14: if (a.M % 64) break; return launch_wgrad<64, 128, 32, 64, 4, true>(a, st);
      default: break;
    }
  }
  return (int)hipErrorInvalidValue;
}

// Sum the split slabs and accumulate into the PyTorch-layout fp32 gradient:
//   mode 0 (Conv2d OIHW):          gw[m][n][tap]          (m = out ch, n = in ch < Nreal)
//   mode 1 (ConvTranspose2d IOHW): gw[n][m][tap]          (n = in ch, m = out ch)
// Block = 32 consecutive slab elements x 8 split groups (coalesced 128-B rows, 8 independent load
// streams per element), partial sums combined through LDS in a fixed order -> deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab,
                                                           float* __restrict__ gw, float* __restrict__ gb, int splits, int T,
                                                           int M, int Nc, int Nreal, int mode, int rmul) {
  __shared__ float part[8][33];
  const long tot = (long)T * M * Nc;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const long nblk_w = (tot + 31) / 32;
  for (long b = blockIdx.x; b < nblk_w + (bslab ? (M + 31) / 32 : 0); b += gridDim.x) {
    const bool isb = b >= nblk_w;
    const long idx = isb ? (b - nblk_w) * 32 + tx : b * 32 + tx;
    const long lim = isb ? M : tot;
    const float* src = isb ? bslab : slab;
    const long stride = (isb ? M : tot) * rmul;
    float s = 0.f;
    if (idx < lim) {
#pragma unroll 8
      for (int k = ty; k < splits; k += 8) s += src[(long)k * stride + idx];
    }
    part[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && idx < lim) {
      float r = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) r += part[g][tx];
      if (isb) {
        gb[idx] += r;
      } else {
        const int n = (int)(idx % Nc);
        const int m = (int)((idx / Nc) % M);
        const int t = (int)(idx / ((long)Nc * M));
        if (n < Nreal) {
          const long dst = mode == 0 ? ((long)m * Nreal + n) * T + t : ((long)n * M + m) * T + t;
          gw[dst] += r;
        }
      }
    }
    __syncthreads();
  }
}

// Quad version (T*M*Nc and M multiples of 4): a thread sums 4 consecutive slab elements (16-B loads)
// over the splits k = g, g + G, ...; the G split groups of a quad are combined through LDS in a fixed
// order.  G is chosen from the shape alone (enough threads to cover the chip, no more groups than
// splits), so the summation order -- and the result bits -- do not change from run to run.  Compared
// with wgrad_reduce_kernel: 4x fewer load instructions, no idle split rows when splits < 8, and
// every thread of a block busy in the grid-stride loop.
template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const float* __restrict__ slab, const float* __restrict__ bslab,
                                                            float* __restrict__ gw, float* __restrict__ gb, int splits,
                                                            int T, int M, int Nc, int Nreal, int mode, int rmul) {
  constexpr int Q = 256 / G;                   // quads per block
  __shared__ f32x4_t part[G][Q];
  const long totq = (long)T * M * Nc / 4, mq = bslab ? M / 4 : 0;
  const int tq = threadIdx.x % Q, tg = threadIdx.x / Q;
  const long nblk = (totq + mq + Q - 1) / Q;
  for (long b = blockIdx.x; b < nblk; b += gridDim.x) {
    const long q = b * Q + tq;
    const bool isb = q >= totq;
    const long qi = isb ? q - totq : q;
    const bool ok = isb ? qi < mq : true;
    const float* src = isb ? bslab : slab;
    const long stride = (isb ? M : totq * 4) * rmul;
    f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (ok) {
#pragma unroll 4
      for (int k = tg; k < splits; k += G) s += *reinterpret_cast<const f32x4_t*>(src + (long)k * stride + qi * 4);
    }
    part[tg][tq] = s;
    __syncthreads();
    if (tg == 0 && ok) {
      f32x4_t r = part[0][tq];
#pragma unroll
      for (int g = 1; g < G; ++g) r += part[g][tq];
      if (isb) {
#pragma unroll
        for (int e = 0; e < 4; ++e) gb[qi * 4 + e] += r[e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long idx = qi * 4 + e;
          const int n = (int)(idx % Nc);
          const int m = (int)((idx / Nc) % M);
          const int t = (int)(idx / ((long)Nc * M));
          if (n < Nreal) gw[mode == 0 ? ((long)m * Nreal + n) * T + t : ((long)n * M + m) * T + t] += r[e];
        }
      }
    }
    __syncthreads();
  }
}

// Tiled version for the Conv2d layout with few splits (mode 0, Nreal == Nc, Nc % 64 == 0, T <= 9).
// The two kernels above read the slab coalesced but scatter their read-modify-write of gw at a stride
// of T floats, so every T-slice of a weight-sized slab sweeps all of gw's cache lines again: with one
// to four splits (the deep layers of a small (micro)batch) that transpose, not the summation, is the
// cost (a 2048x2048 conv: 0.9 ms).  Here a block owns (m, 64 consecutive n) for all T taps: it sums the
// splits into LDS (4 split groups, fixed combine order), then adds the [64 n][T] tile to gw as ONE
// contiguous run of 64*T floats.  Blocks past the weight tiles sum the bias slab, 64 channels each.
__global__ __launch_bounds__(256) void wgrad_reduce_tile_kernel(const float* __restrict__ slab,
                                                                const float* __restrict__ bslab, float* __restrict__ gw,
                                                                float* __restrict__ gb, int splits, int T, int M, int Nc,
                                                                int rmul) {
  __shared__ float part[4][9][64];
  __shared__ float out[64 * 9];
  const long tot = (long)T * M * Nc;
  const int ntn = Nc / 64;
  const long ntile = (long)M * ntn, nbias = bslab ? (M + 63) / 64 : 0;
  const int n = threadIdx.x & 63, grp = threadIdx.x >> 6;
  for (long b = blockIdx.x; b < ntile + nbias; b += gridDim.x) {
    if (b < ntile) {
      const int m = (int)(b / ntn), n0 = (int)(b - (long)m * ntn) * 64;
      for (int t = 0; t < T; ++t) {
        const float* src = slab + ((long)t * M + m) * Nc + n0 + n;
        float acc = 0.f;
#pragma unroll 4
        for (int k = grp; k < splits; k += 4) acc += src[(long)k * rmul * tot];
        part[grp][t][n] = acc;
      }
      __syncthreads();
      for (int o = threadIdx.x; o < 64 * T; o += 256) {
        const int t = o >> 6, nn = o & 63;
        out[nn * T + t] = ((part[0][t][nn] + part[1][t][nn]) + part[2][t][nn]) + part[3][t][nn];
      }
      __syncthreads();
      float* dst = gw + ((long)m * Nc + n0) * T;
      for (int o = threadIdx.x; o < 64 * T; o += 256) dst[o] += out[o];
      __syncthreads();
    } else {
      const int m0 = (int)(b - ntile) * 64;
      float acc = 0.f;
      if (m0 + n < M)
        for (int k = grp; k < splits; k += 4) acc += bslab[(long)k * rmul * M + m0 + n];
      part[grp][0][n] = acc;
      __syncthreads();
      if (grp == 0 && m0 + n < M) gb[m0 + n] += ((part[0][0][n] + part[1][0][n]) + part[2][0][n]) + part[3][0][n];
      __syncthreads();
    }
  }
}

// Few elements over thousands of splits (the first conv's [9][32][8] weight gradient from a row-streaming
// kernel with one slab row per block): the kernels above give each element ONE block-column of threads,
// so a 2304-element slab is summed by 73 blocks walking 16k rows -- 0.9 ms, latency bound.  Stage 1 sums
// groups of R consecutive rows IN PLACE into the group's first row (one thread per element, coalesced,
// (elements / 256) x groups blocks); the reduce kernels then walk every R-th row (rmul).  Fixed order.
// gridDim.y < groups: each block walks groups blockIdx.y, + gridDim.y, ... (the same per-group sums): beside
// a busy kernel on the other stream, thousands of 256-thread blocks wait for dispatch far longer than
// they run (0.44 ms vs 6 us alone for the first conv's slab, profiles/hip_b256_512_summary_r06.txt)
__global__ __launch_bounds__(256) void wgrad_presum_kernel(float* __restrict__ slab, float* __restrict__ bslab, int splits,
                                                           long tot, int M, int R) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const bool isb = e >= tot;
  if (e >= tot + (bslab ? M : 0)) return;
  float* src = isb ? bslab + (e - tot) : slab + e;
  const long stride = isb ? M : tot;
  const int groups = (splits + R - 1) / R;
  for (int gi = blockIdx.y; gi < groups; gi += gridDim.y) {
    const int r0 = gi * R, r1 = min(splits, r0 + R);
    float s = 0.f;
#pragma unroll 8
    for (int k = r0; k < r1; ++k) s += src[(long)k * stride];
    src[(long)r0 * stride] = s;
  }
}

static int WGRAD_PRESUM = 1;        // DPA_NO_WGRAD_PRESUM=1 -> 0 (set at library load, ops/_lib.py)
static int WGRAD_PRESUM_Y = 0;      // DPA_WGRAD_PRESUM_Y: cap on the presum grid's group dimension (0 = one block per group)
DPA_API void dpa_wgrad_set_presum(int on) { WGRAD_PRESUM = on; }
DPA_API void dpa_wgrad_set_presum_y(int y) { WGRAD_PRESUM_Y = y; }

// g: -1 auto, 0 the 32-element kernel, > 0 the quad kernel with g split groups, -2 the tiled kernel
// (tools/kbench_reduce.py).  The slabs are scratch: the presum stage (many splits, few elements) writes them.
DPA_API int dpa_wgrad_reduce_cfg(const float* slab_in, const float* bslab_in, float* gw, float* gb, int splits, int T, int M,
                                 int Nc, int Nreal, int mode, int g, hipStream_t st) {
  const long tot = (long)T * M * Nc;
  float* slab = const_cast<float*>(slab_in);
  float* bslab = const_cast<float*>(bslab_in);
  const bool tile_ok = mode == 0 && Nreal == Nc && Nc % 64 == 0 && T <= 9;
  int rmul = 1;
  if (WGRAD_PRESUM && splits >= 1024 && tot <= 65536) {
    constexpr int R = 32;
    const long el = tot + (bslab ? M : 0);
    const unsigned groups = (unsigned)((splits + R - 1) / R);
    const unsigned gy = WGRAD_PRESUM_Y > 0 && (unsigned)WGRAD_PRESUM_Y < groups ? (unsigned)WGRAD_PRESUM_Y : groups;
    hipLaunchKernelGGL(wgrad_presum_kernel, dim3((unsigned)((el + 255) / 256), gy), dim3(256), 0, st, slab, bslab, splits,
                       tot, M, R);
    splits = (int)groups;
    rmul = R;
  }
  if (g == -1) {
    // measured on the UNet / UNet-XL slab shapes (profiles/kbench_reduce_r02.txt): tiled for few
    // splits, quad kernel with 4-8 groups for a moderate count, the 32-element kernel for thousands
    if (tile_ok && splits <= 16) g = -2;
    else if (splits >= 1024 || tot < 65536 || (mode == 1 && splits > 32)) g = 0;
    else if (mode == 1) g = splits <= 8 ? 4 : 8;
    else g = splits <= 32 ? 4 : 8;
  }
  if (g == -2) {
    if (!tile_ok) return (int)hipErrorInvalidValue;
    const long nb = (long)M * (Nc / 64) + (bslab ? (M + 63) / 64 : 0);
    hipLaunchKernelGGL(wgrad_reduce_tile_kernel, dim3((unsigned)(nb < 16384 ? nb : 16384)), dim3(256), 0, st, slab, bslab,
                       gw, gb, splits, T, M, Nc, rmul);
    return (int)hipGetLastError();
  }
  if (g != 0 && tot % 4 == 0 && M % 4 == 0 && ((size_t)slab & 15) == 0 && (!bslab || ((size_t)bslab & 15) == 0)) {
    // G split groups per quad (chosen above or by the caller)
    const long quads = tot / 4 + (bslab ? M / 4 : 0);
    const int G = g;
    const long nb = (quads + (256 / G) - 1) / (256 / G);
    const dim3 grid((unsigned)(nb < 8192 ? nb : 8192));
#define DPA_RED4(Gv) \
    if (G == Gv) { hipLaunchKernelGGL(wgrad_reduce4_kernel<Gv>, grid, dim3(256), 0, st, slab, bslab, gw, gb, splits, T, M, Nc, Nreal, mode, rmul); return (int)hipGetLastError(); }
    DPA_RED4(1) DPA_RED4(2) DPA_RED4(4) DPA_RED4(8) DPA_RED4(16) DPA_RED4(32) DPA_RED4(64)
#undef DPA_RED4
    return (int)hipErrorInvalidValue;
  }
  const long nb = (tot + 31) / 32 + (bslab ? (M + 31) / 32 : 0);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(nb < 8192 ? nb : 8192)), dim3(256), 0, st, slab, bslab, gw, gb,
                     splits, T, M, Nc, Nreal, mode, rmul);
  return (int)hipGetLastError();
}

DPA_API int dpa_wgrad_reduce(const float* slab, const float* bslab, float* gw, float* gb, int splits, int T, int M, int Nc,
                             int Nreal, int mode, hipStream_t st) {
  return dpa_wgrad_reduce_cfg(slab, bslab, gw, gb, splits, T, M, Nc, Nreal, mode, -1, st);
}
