// Deep-layer conv3x3 weight gradient on an LDS-DMA row pipeline (gfx950): the 128/256/512-channel
// layers of the UNet's lower levels (reference model/unet_parts.py:10-12 -- enc.conv3/conv4, mid,
// dec.conv1/conv2 at 128^2 and 64^2).
//
// As a GEMM: dW[tap][co][ci] = sum_p g[p][co] * x[p + delta(tap)][ci] -- M = Cout, N = 9 x Cin,
// K = the pixels (B*H*W, up to 4.2 M at batch 256).  The row-streaming wgrad (halo.hip
// wgrad_stream) owns 64 x 32 output tiles with three 64-lane waves and one register-staged row in
// flight: every gradient / input row is re-fetched by 8-32 tiles and the per-row latency is
// exposed (38 % MFMA issue, profiles/pmc_b128_512_r02_end.txt).  Here:
//   * one workgroup (12 waves) owns BM = 128 output channels x BN = 64 input channels x all 9 taps
//     (73,728 fp32 accumulators, 96 per lane): 386 FLOP per staged byte instead of 192;
//   * K runs along one image row strip at a time (BP = 64 pixels of row h): the gradient row
//     g[h][w0..w0+63][co0..co0+127] and the input rows x[h-1..h+1][w0-1..w0+64][ci0..ci0+63] (a ring
//     of rows, each fetched once) are staged by LDS-DMA (`buffer_load ... lds`: no VGPR round trip,
//     no ds_write), D row bundles deep with counted `s_waitcnt vmcnt` and raw barriers
//     (cdna_hip_programming.md "Pipelining across barriers"), so D rows of HBM latency hide behind
//     the MFMAs of the current one;
//   * the three kernel-column taps kw read the same staged input row shifted by kw pixels (rows of
//     the [pixel][channel] LDS image), the kernel-row taps kh three ring slots;
//   * fragments are read with ds_read_b64_tr_b16 from [pixel][channel] images (the MFMA K dimension
//     = pixels is the strided one in NHWC) whose 16-B chunks are XOR-swizzled on the DMA's SOURCE
//     address (the DMA writes lane-linearly; swz_kk, conflict-free transposed reads).
// Twelve waves: wave w handles kernel row kh = w / 4 (its three taps kw share the ring slot of input
// row h + kh - 1), output channels ((w % 4) & 1) * 64 .. +63 and input channels ((w % 4) >> 1) * 32 ..
// +31: per 32-pixel k-step 4 + 6 fragment reads feed 24 MFMAs, 96 accumulator registers per lane
// (three waves per SIMD).
// One workgroup per (image, row segment, column strip) x (co tile, ci tile): its partial dW goes to
// fp32 slab rows [split][tap][M][Nc] and dpa_wgrad_reduce sums them in a fixed order (bitwise
// reproducible), exactly like the other weight-gradient kernels; the bias gradient (the row sums of
// g) is accumulated by the ci-tile-0 workgroups from the staged gradient rows.
#include "conv_args.h"

namespace {

constexpr int WR_BM = 128, WR_BN = 64, WR_BP = 64;
constexpr int WR_RBA = WR_BM * 2;                 // gradient row image: [64 px][128 co], 256 B rows
constexpr int WR_RBB = WR_BN * 2;                 // input row image: [72 px][64 ci], 128 B rows
constexpr int WR_AIMG = WR_BP * WR_RBA;           // 16 KB
constexpr int WR_BROWS = 72;                      // px w0-1 .. w0+70 (66 used), 9 DMA instructions
constexpr int WR_BIMG = WR_BROWS * WR_RBB;        // 9 KB

// two ds_read_b64_tr_b16 of one transposed fragment (see conv_args.h tr_frag) at byte offsets
__device__ __forceinline__ bf16x8_t wr_tr(const char* base, int off0, int off1) {
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off1));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// the same two reads as inline asm: the builtin makes hipcc wait vmcnt(0) before every read while an
// LDS-DMA is in flight (it cannot tell the read from the DMA's destination) -- that drained the row
// pipeline before each row's first fragment read.  The asm reads are invisible to the wait-count pass:
// the kernel waits lgkmcnt(0) itself before the MFMAs that consume them (wr_lgkm0).
__device__ __forceinline__ s16x4_t wr_trld(unsigned addr) {
  s16x4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ bf16x8_t wr_join(s16x4_t v0, s16x4_t v1) {
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}
__device__ __forceinline__ void wr_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace

// D: row bundles in flight beyond the one being consumed.  LDS: (D+1) gradient rows + (D+3) input
// rows + the bias scratch, one workgroup per CU.
template <int D>
__global__ __launch_bounds__(768) void wgrad_rows_kernel(WgradArgs a, int rh) {
  constexpr int NA = D + 1, NB = D + 3;
  constexpr int BIAS_OFF = NA * WR_AIMG + NB * WR_BIMG;
  __shared__ __attribute__((aligned(16))) char lds[BIAS_OFF + 4 * WR_BM];   // all LDS in ONE array
  char* const Abuf = lds;
  char* const Bbuf = lds + NA * WR_AIMG;
  float* const bred = reinterpret_cast<float*>(lds + BIAS_OFF);

  const int nmt = a.M / WR_BM, nnt = a.Nc / WR_BN, tiles = nmt * nnt;
  const int stripsW = (a.Wg + WR_BP - 1) / WR_BP, segsH = (a.Hg + rh - 1) / rh;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;        // a split's tiles share one XCD's L2
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * WR_BM, n0 = nt * WR_BN;
  const int n = split / (segsH * stripsW);
  const int rem = split - n * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * WR_BP, h0 = hs * rh;
  const int nrows = min(rh, a.Hg - h0);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool do_bias = a.bslab != nullptr && nt == 0;

  // one image per workgroup: 64-bit image bases, 32-bit offsets inside the image
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.atab ? a.atab[n] : a.A + (long)n * a.HA * a.WA * a.lda), 0, (int)a.abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.btab ? a.btab[n] : a.B + (long)n * a.HB * a.WB * a.ldb), 0, (int)a.bbytes, 0x00020000);

  // ---- DMA plan per row bundle: 16 gradient-row instructions (4 pixel rows x 16 chunks of 1 KB
  // each) and 9 input-row instructions (8 pixel rows x 8 chunks).  Wave w issues gradient
  // instruction w; waves 0-3 also gradient instructions 12-15, waves 4-11 input instructions 0-7 and
  // wave 0 input instruction 8: 3 instructions per bundle for wave 0, 2 for the others.  Lane ->
  // (row, LDS slot); the slot holds global chunk slot ^ swz(row) (source-side swizzle).
  const int ia0 = wid, ia1 = wid < 4 ? 12 + wid : -1;                // gradient instructions
  const int ib0 = wid >= 4 ? wid - 4 : -1, ib1 = wid == 0 ? 8 : -1;  // input-row instructions
  auto a_off = [&](int ins) -> unsigned {
    const int px = 4 * ins + (lane >> 4), slot = lane & 15;
    const int ch = slot ^ swz_kk<WR_RBA>(px);
    return (w0 + px < a.Wg) ? (unsigned)(((w0 + px) * a.lda + m0 + ch * 8) * 2) : 0x80000000u;
  };
  auto b_off = [&](int ins) -> unsigned {
    const int row = 8 * ins + (lane >> 3), slot = lane & 7;
    const int ch = slot ^ swz_kk<WR_RBB>(row);
    const int iw = w0 - 1 + row;
    return (row < WR_BP + 2 && iw >= 0 && iw < a.WB) ? (unsigned)((iw * a.ldb + n0 + ch * 8) * 2) : 0x80000000u;
  };
  const unsigned aoff0 = a_off(ia0), aoff1 = ia1 >= 0 ? a_off(ia1) : 0x80000000u;
  const unsigned boff0 = ib0 >= 0 ? b_off(ib0) : 0x80000000u, boff1 = ib1 >= 0 ? b_off(ib1) : 0x80000000u;
  const unsigned arow = (unsigned)(a.WA * a.lda * 2), brow = (unsigned)(a.WB * a.ldb * 2);
  auto issue_a = [&](int t) {                           // gradient row h0 + t -> A buffer t % NA
    char* dst = Abuf + (t % NA) * WR_AIMG;
    const unsigned base = (unsigned)(h0 + t) * arow;
    dma16(ar, dst + ia0 * 1024, aoff0 == 0x80000000u ? aoff0 : base + aoff0);
    if (ia1 >= 0) dma16(ar, dst + ia1 * 1024, aoff1 == 0x80000000u ? aoff1 : base + aoff1);
  };
  auto issue_b = [&](int b) {                           // input row h0 + b (b = -1 .. nrows) -> slot (b+1) % NB
    char* dst = Bbuf + ((b + 1) % NB) * WR_BIMG;
    const int ih = h0 + b;
    const bool rok = ih >= 0 && ih < a.HB;
    const unsigned base = (unsigned)(rok ? ih : 0) * brow;
    if (ib0 >= 0) dma16(br, dst + ib0 * 1024, (rok && boff0 != 0x80000000u) ? base + boff0 : 0x80000000u);
    if (ib1 >= 0) dma16(br, dst + ib1 * 1024, (rok && boff1 != 0x80000000u) ? base + boff1 : 0x80000000u);
  };

  // ---- fragment addressing (conv_args.h tr_frag with the per-lane parts precomputed)
  const int kh = wid >> 2, wq = wid & 3, wco = wq & 1, wci = wq >> 1;
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int fcol = (fp & 1) * 8 + (fp >> 1) * 16;
  const int baseA = (8 * fg + fq) * WR_RBA + fcol, baseB = (8 * fg + fq) * WR_RBB + fcol;
  int offA[4][2], offB[3][2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int swa = swz_kk<WR_RBA>(8 * fg + fq + 4 * h) << 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) offA[i][h] = baseA + 4 * h * WR_RBA + (((2 * (wco * 4 + i)) << 4) ^ swa);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int swb = swz_kk<WR_RBB>(kw + 8 * fg + fq + 4 * h) << 4;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        offB[kw][j][h] = baseB + (kw + 4 * h) * WR_RBB + (((2 * (wci * 2 + j)) << 4) ^ swb);
    }
  }

  f32x4_t acc[3][4][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[kw][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // bias: threads 0..511 sum 8 output channels (chunk tid & 15) over pixel rows (tid >> 4) and +32
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool bias_lane = do_bias && tid < 512;

  // ---- prologue: input rows -1, 0; then bundles 0 .. D-1 = {gradient row t, input row t+1}
  issue_b(-1);
  issue_b(0);
#pragma unroll
  for (int t = 0; t < D; ++t)
    if (t < nrows) {
      issue_a(t);
      issue_b(t + 1);
    }

#pragma unroll 1
  for (int t = 0; t < nrows; ++t) {
    // bundle t (and everything before it) has landed for this wave; bundles t+1 .. t+D-1 may fly
    const int fly = min(D - 1, nrows - 1 - t);
    if (wid == 0) {
      if (fly >= 2) wait_vm<6>(); else if (fly == 1) wait_vm<3>(); else wait_vm<0>();
    } else {
      if (fly >= 2) wait_vm<4>(); else if (fly == 1) wait_vm<2>(); else wait_vm<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();                      // every wave's DMAs of bundle t are in LDS,
    __builtin_amdgcn_sched_barrier(0);                 // every wave finished step t-1's reads
    if (t + D < nrows) {
      issue_a(t + D);
      issue_b(t + D + 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* Ai = Abuf + (t % NA) * WR_AIMG;
    const char* Bi = Bbuf + ((t + kh) % NB) * WR_BIMG;   // input row h0 + t + kh - 1
    const unsigned ua = (unsigned)(size_t)LDS_PTR(char, Ai), ub = (unsigned)(size_t)LDS_PTR(char, Bi);
#pragma unroll
    for (int ks = 0; ks < WR_BP / 32; ++ks) {
      // A fragments + the kw = 0 B pair, then per kw: the next pair's reads behind this pair's MFMAs
      s16x4_t ra[4][2], rb[2][2][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) ra[i][h] = wr_trld(ua + ks * 32 * WR_RBA + offA[i][h]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) rb[0][j][h] = wr_trld(ub + ks * 32 * WR_RBB + offB[0][j][h]);
      wr_lgkm0();
      bf16x8_t af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = wr_join(ra[i][0], ra[i][1]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int cur = kw & 1;
        if (kw < 2) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) rb[cur ^ 1][j][h] = wr_trld(ub + ks * 32 * WR_RBB + offB[kw + 1][j][h]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8_t bf = wr_join(rb[cur][j][0], rb[cur][j][1]);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[kw][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[kw][i][j], 0, 0, 0);
        }
        if (kw < 2) wr_lgkm0();
      }
    }
    if (bias_lane) {
      const int ch = tid & 15;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int px = (tid >> 4) + 32 * k;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(Ai + px * WR_RBA + ((ch ^ swz_kk<WR_RBA>(px)) << 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bsum[2 * e] += lo_bf(v[e]);
          bsum[2 * e + 1] += hi_bf(v[e]);
        }
      }
    }
  }

  // ---- epilogue: this split's partial dW[tap][co][ci] (C/D layout: ci = lane & 15, co = 4*(lane>>4)+r)
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int co = m0 + wco * 64 + i * 16 + 4 * (lane >> 4);
        const int ci = n0 + wci * 32 + j * 16 + (lane & 15);
        float* dst = a.slab + (((long)split * 9 + kh * 3 + kw) * a.M + co) * a.Nc + ci;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(long)r * a.Nc] = acc[kw][i][j][r];
      }
  if (do_bias) {
    __syncthreads();                                    // no DMA in flight any more
    for (int c = tid; c < WR_BM; c += 768) bred[c] = 0.f;
    __syncthreads();
    if (bias_lane) {
      const int ch = tid & 15;
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&bred[ch * 8 + e], bsum[e]);
    }
    __syncthreads();
    for (int c = tid; c < WR_BM; c += 768) a.bslab[(long)split * a.M + m0 + c] = bred[c];
  }
}

// Rows of output per workgroup: rh (whole images by default: the prologue's two input rows and the
// pipeline ramp are paid once per image segment).  splits must equal N * ceil(Hg / rh) * ceil(Wg / 64).
// Eligible: conv3x3 s1 p1 (A = the output gradient, B = the layer input, same grid), M % 128 == 0,
// Nc % 64 == 0, 16-B aligned channel strides; a ragged last strip reads zeros past the row.
DPA_API int dpa_wgrad_rows(const WgradArgs* args, int rh, int depth, hipStream_t st) {
  const WgradArgs& a = *args;
  if ((a.M % WR_BM) || (a.Nc % WR_BN) || (a.lda & 7) || (a.ldb & 7) || a.s != 1 || a.pad != 1 || a.KW != 3 ||
      a.HA != a.Hg || a.WA != a.Wg || a.HB != a.Hg || a.WB != a.Wg || a.Wg < 8 || rh < 1 ||
      a.splits != a.N * ((a.Hg + rh - 1) / rh) * ((a.Wg + WR_BP - 1) / WR_BP))
    return (int)hipErrorInvalidValue;
  const int tiles = (a.M / WR_BM) * (a.Nc / WR_BN);
  const dim3 grid(tiles * a.splits);
  if (depth == 3)
    hipLaunchKernelGGL((wgrad_rows_kernel<3>), grid, dim3(768), 0, st, a, rh);
  else if (depth == 1)
    hipLaunchKernelGGL((wgrad_rows_kernel<1>), grid, dim3(768), 0, st, a, rh);
  else
    hipLaunchKernelGGL((wgrad_rows_kernel<2>), grid, dim3(768), 0, st, a, rh);
  return (int)hipGetLastError();
}
