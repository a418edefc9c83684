// Deep-layer conv3x3 weight gradient as a dense LDS-DMA GEMM on the ping-pong schedule of
// igemm_glds.hip's cfg 14 (gfx950; reference model/unet_parts.py:10-12 -- enc.conv4, mid, dec.conv1/2 at
// 64^2 / 32^2).
//
// As a GEMM: dW[co][tap, ci] = sum_p g[p][co] * x[p + delta(tap)][ci] -- M = Cout, N = 9 x Cin
// (tap-major columns), K = pixels.  The row-streaming (halo.hip wgrad_stream) and row-pipeline
// (wgrad_rows.hip) kernels reuse a staged input row for the three kw taps but run 64 x 32 / 128 x 64
// output tiles at 0.73-1.0 PF; the forward/dgrad GEMMs of the same layers reach 1.2-1.33 PF on the
// 256 x 256 ping-pong core.  Here the weight gradient IS that core:
//   * 256 (co) x 256 (tap, ci) output tile, 64-pixel K-steps, two K-tile buffers of four 16-KB
//     half-tiles (A0/A1: gradient channels co0 + [0,128) / [128,256), B0/B1: columns n0 + [0,128) /
//     [128,256)), each a [64 px][128 ch] image with 256-B rows, filled by LDS-DMA
//     (`buffer_load ... lds`) with the 16-B chunks XOR-swizzled on the SOURCE address (swz_kk<256>);
//   * the B operand of column (tap, ci) at pixel (h, w) is x[h + kh - 1][w + kw - 1][ci]: the DMA
//     source offset is a per-lane constant plus the K-step's pixel base; zero padding by the buffer
//     unit's range check (offset 0x80000000 -> zeros), per lane and K-step;
//   * fragments are transposed reads (ds_read_b64_tr_b16, conv_args.h tr_frag): the MFMA K dimension
//     is the pixel, the strided one in NHWC;
//   * waves 0-3 and 4-7 (one of each per SIMD) run one barrier apart: while one issues a quadrant's 16
//     MFMAs the other reads the next quadrant's fragments and issues one half-tile of DMA; the K loop
//     is straight-line code with constant vmcnt waits, the last two K-tiles a peeled tail
//     (cfg 14's schedule: p0 -> B1(s+1), p1 -> A1(s+1), p2 -> A0(s+2), p3 -> B0(s+2));
//   * the bias gradient (sum_p g[p][co]) rides along in the column-tile-0 workgroups: one extra MFMA
//     per A fragment against a ones fragment, spread over the four column waves.
// One workgroup per (image group, tile): K = all pixels of ipS images; its partial dW goes to fp32 slab
// rows [split][tap][M][Nc] that dpa_wgrad_reduce sums in a fixed order (bitwise reproducible).
#include "conv_args.h"

#include <type_traits>

namespace {

constexpr int WG_RB = 256;                 // bytes per LDS image row: 128 channels
constexpr int WG_HALF = 64 * WG_RB;        // one half-tile image: 64 pixels x 128 channels
constexpr int WG_STAGE = 4 * WG_HALF;      // A0 A1 B0 B1

// ds_read_b64_tr_b16 as inline asm.  The builtin makes hipcc wait vmcnt(0) before every read while an
// LDS-DMA is in flight (it cannot tell the read from the DMA's destination), which drains the DMA
// pipeline every phase; the asm read is invisible to the wait-count pass, so the kernel waits
// lgkmcnt(0) itself before the MFMAs that consume the fragments (sync_in) -- no other code reads them.
template <int OFF>
__device__ __forceinline__ s16x4_t trld(unsigned addr) {
  s16x4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

__device__ __forceinline__ bf16x8_t tr_join(s16x4_t v0, s16x4_t v1) {
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// K-step coordinates: byte offsets of the 64-pixel step's first pixel in A and B (consecutive K-steps
// are consecutive pixels of the split's contiguous images) and its (h, w) for the zero-padding masks
struct WKC {
  unsigned oa, ob;
  int h, w, n;            // n: image inside the split (the transposed-conv mode's B addressing)
};

}  // namespace

__global__ __launch_bounds__(512) void wgrad_gemm_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * WG_STAGE];

  const int H = a.Hg, W = a.Wg, HW = H * W;
  // up mode (KW == 2): the weight gradient of a transposed conv k2 s2, dW[ci][tap][co] = sum_p x[p][ci] *
  // g[2p + (i, j)][co] -- A = the layer input x on the low-resolution grid, B = the output gradient on the
  // 2x grid, 4 taps at (2h + i, 2w + j); no padding
  const bool up = a.KW == 2;
  const int T = up ? 4 : 9;
  const int Ncols = T * a.Nc;
  const int nmt = a.M / 256, nnt = (Ncols + 255) / 256, tiles = nmt * nnt;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;   // a split's tiles share an XCD's L2
  const int mt = tile / nnt, nt = tile - mt * nnt;
  const int m0 = mt * 256, n0 = nt * 256;
  const int ips = a.pix_per_split;                             // images per split
  const int nimg0 = split * ips;
  const int nimg = min(ips, a.N - nimg0);
  const int spi = HW / 64;                                     // K-steps per image
  const int S = nimg * spi;                                    // host guarantees S >= 2
  const bool do_bias = a.bslab != nullptr && nt == 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid & 1, wp = wid >> 1, grp = wid >> 2;

  // split's image range: 64-bit bases, 32-bit offsets inside it (host: < 2^31 bytes)
  // (per-image tables -- the microbatches of a pipeline stage: the host makes every split's images
  // consecutive images of ONE tensor, so the split's first image pointer is its base)
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.atab ? a.atab[nimg0] : a.A + (long)nimg0 * HW * a.lda), 0, (int)a.abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.btab ? a.btab[nimg0] : a.B + (long)nimg0 * (up ? 4 : 1) * HW * a.ldb), 0, (int)a.bbytes, 0x00020000);

  // ---- per-lane DMA constants.  Half-tile image = 16 instructions of 1 KB (4 pixel rows x 16
  // chunks); wave wid issues instructions wid and 8 + wid.  Lane l: pixel row r = 4 ins + (l >> 4),
  // LDS slot l & 15 <- global chunk (l & 15) ^ swz_kk<256>(r).
  unsigned laneA[2][2], laneB[2][2];
  int dh[2][2], dw[2][2];
  bool colok[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ins = j * 8 + wid;
    const int r = 4 * ins + (lane >> 4);
    const int ch = (lane & 15) ^ swz_kk<WG_RB>(r);
    const int lh = W >= 64 ? 0 : r / W, lw = W >= 64 ? r : r - (r / W) * W;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      laneA[h][j] = (unsigned)(((lh * W + lw) * a.lda + m0 + h * 128 + ch * 8) * 2);
      const int col = n0 + h * 128 + ch * 8;
      const int tap = col / a.Nc, ci = col - tap * a.Nc;
      const int kh = tap / 3, kw = tap - kh * 3;
      colok[h][j] = col < Ncols;
      dh[h][j] = lh + kh - 1;
      dw[h][j] = lw + kw - 1;
      laneB[h][j] = up ? (unsigned)((((2 * lh + (tap >> 1)) * 2 * W + 2 * lw + (tap & 1)) * a.ldb + ci) * 2)
                       : (unsigned)((((lh + kh - 1) * W + (lw + kw - 1)) * a.ldb + ci) * 2);
    }
  }
  const unsigned rowA = (unsigned)(64 * a.lda * 2), rowB = (unsigned)(64 * a.ldb * 2);   // bytes per K-step

  auto knext = [&](WKC c) {
    c.oa += rowA;
    c.ob += rowB;
    if (W >= 64) {
      c.w += 64;
      if (c.w == W) { c.w = 0; ++c.h; }
    } else {
      c.h += 64 / W;
    }
    if (c.h == H) {
      c.h = 0;
      ++c.n;
    }
    return c;
  };
  auto issueA = [&](int h, int buf, WKC c) {
    char* base = lds + buf * WG_STAGE + h * WG_HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(ar, base + (j * 8 + wid) * 1024, c.oa + laneA[h][j]);
  };
  auto issueB = [&](int h, int buf, WKC c) {
    char* base = lds + buf * WG_STAGE + (2 + h) * WG_HALF;
    if (up) {
      const unsigned ob = (unsigned)((((c.n * 2 * H + 2 * c.h) * 2 * W) + 2 * c.w) * a.ldb * 2);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(br, base + (j * 8 + wid) * 1024, colok[h][j] ? ob + laneB[h][j] : 0x80000000u);
      return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int hh = c.h + dh[h][j], ww = c.w + dw[h][j];
      const bool ok = colok[h][j] && hh >= 0 && hh < H && ww >= 0 && ww < W;
      dma16(br, base + (j * 8 + wid) * 1024, ok ? c.ob + laneB[h][j] : 0x80000000u);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int ic = 0; ic < 8; ++ic)
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t bacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  const s16x8_t ones_s = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, ones_s);

  WKC k0{0u, 0u, 0, 0, 0};
  WKC k1 = knext(k0);
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

  // per-lane LDS byte offsets of the transposed fragment reads (conv_args.h tr_frag's addressing) inside
  // a half image, k rows 0..31: [fragment][first / second 4-row block]
  const unsigned lds0 = (unsigned)(size_t)LDS_PTR(char, lds);
  unsigned toA[4][2], toB[2][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 8 * g + q + 4 * h;
#pragma unroll
      for (int ic = 0; ic < 4; ++ic) {
        const int col = wc * 64 + ic * 16 + 4 * p;
        toA[ic][h] = lds0 + (unsigned)(r * WG_RB + (((col >> 3) ^ swz_kk<WG_RB>(r)) << 4) + (col & 7) * 2);
      }
#pragma unroll
      for (int ip = 0; ip < 2; ++ip) {
        const int col = wp * 32 + ip * 16 + 4 * p;
        toB[ip][h] = lds0 + (unsigned)(r * WG_RB + (((col >> 3) ^ swz_kk<WG_RB>(r)) << 4) + (col & 7) * 2);
      }
    }
  }
  s16x4_t ra[4][2][2], rb[2][2][2][2];          // raw reads: [frag][kk][block]
  bf16x8_t af[4][2], bfr[2][2][2];
  // A quadrant QA of this wave: channels QA*128 + wc*64 + ic*16 of half-image QA (stage offset sto)
  auto readA = [&](unsigned sto, auto QAc) {
    constexpr int O = decltype(QAc)::value * WG_HALF;
#pragma unroll
    for (int ic = 0; ic < 4; ++ic) {
      ra[ic][0][0] = trld<O>(toA[ic][0] + sto);
      ra[ic][0][1] = trld<O>(toA[ic][1] + sto);
      ra[ic][1][0] = trld<O + 32 * WG_RB>(toA[ic][0] + sto);
      ra[ic][1][1] = trld<O + 32 * WG_RB>(toA[ic][1] + sto);
    }
  };
  // B quadrant QB: columns QB*128 + wp*32 + ip*16 of half-image 2 + QB
  auto readB = [&](unsigned sto, auto QBc) {
    constexpr int QB = decltype(QBc)::value;
    constexpr int O = (2 + QB) * WG_HALF;
#pragma unroll
    for (int ip = 0; ip < 2; ++ip) {
      rb[QB][ip][0][0] = trld<O>(toB[ip][0] + sto);
      rb[QB][ip][0][1] = trld<O>(toB[ip][1] + sto);
      rb[QB][ip][1][0] = trld<O + 32 * WG_RB>(toB[ip][0] + sto);
      rb[QB][ip][1][1] = trld<O + 32 * WG_RB>(toB[ip][1] + sto);
    }
  };
  // after the reads have landed (sync_in's lgkmcnt(0)): assemble the MFMA operands
  auto joinA = [&]() {
#pragma unroll
    for (int ic = 0; ic < 4; ++ic)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[ic][kk] = tr_join(ra[ic][kk][0], ra[ic][kk][1]);
  };
  auto joinB = [&](int qb) {
#pragma unroll
    for (int ip = 0; ip < 2; ++ip)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bfr[qb][ip][kk] = tr_join(rb[qb][ip][kk][0], rb[qb][ip][kk][1]);
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
  // bias: column wave wp sums A fragment ic = wp of the quadrant (both k halves)
  // (wp is wave-uniform: scalar branches with compile-time fragment indices -- a runtime-indexed
  // fragment array would live in scratch)
  auto bias_mfma = [&](int qa, const bf16x8_t& f0, const bf16x8_t& f1) {
    bacc[qa] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, ones, bacc[qa], 0, 0, 0);
    bacc[qa] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, ones, bacc[qa], 0, 0, 0);
  };
  auto bias_quad = [&](int qa) {
    if (do_bias) {
      if (wp == 0) bias_mfma(qa, af[0][0], af[0][1]);
      else if (wp == 1) bias_mfma(qa, af[1][0], af[1][1]);
      else if (wp == 2) bias_mfma(qa, af[2][0], af[2][1]);
      else bias_mfma(qa, af[3][0], af[3][1]);
    }
  };
  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this phase's asm fragment reads
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  WKC kc1 = k1, kc2 = knext(k1);
  int s = 0;
  for (; s < S - 2; ++s) {
    const unsigned sto = (unsigned)((s & 1) * WG_STAGE);
    const int nb = (s & 1) ^ 1, cb = s & 1;
    readB(sto, std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_barrier(0);
    readA(sto, std::integral_constant<int, 0>{});
    issueB(1, nb, kc1);
    wait_vm<8>();
    sync_in();
    joinB(0);
    joinA();
    mfma_quad(0, 0);
    bias_quad(0);
    sync_out();
    readB(sto, std::integral_constant<int, 1>{});
    issueA(1, nb, kc1);
    wait_vm<8>();
    sync_in();
    joinB(1);
    mfma_quad(0, 1);
    sync_out();
    readA(sto, std::integral_constant<int, 1>{});
    issueA(0, cb, kc2);
    sync_in();
    joinA();
    mfma_quad(1, 1);
    bias_quad(1);
    sync_out();
    issueB(0, cb, kc2);
    wait_vm<8>();
    sync_in();
    mfma_quad(1, 0);
    sync_out();
    kc1 = kc2;
    kc2 = knext(kc2);
  }
  {  // K-tile S-2: the halves of S-1 still to issue
    const unsigned sto = (unsigned)((s & 1) * WG_STAGE);
    const int nb = (s & 1) ^ 1;
    readB(sto, std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_barrier(0);
    readA(sto, std::integral_constant<int, 0>{});
    issueB(1, nb, kc1);
    wait_vm<8>();
    sync_in();
    joinB(0);
    joinA();
    mfma_quad(0, 0);
    bias_quad(0);
    sync_out();
    readB(sto, std::integral_constant<int, 1>{});
    issueA(1, nb, kc1);
    wait_vm<8>();
    sync_in();
    joinB(1);
    mfma_quad(0, 1);
    sync_out();
    readA(sto, std::integral_constant<int, 1>{});
    sync_in();
    joinA();
    mfma_quad(1, 1);
    bias_quad(1);
    sync_out();
    wait_vm<4>();                              // A0/B0 of S-1
    sync_in();
    mfma_quad(1, 0);
    sync_out();
    ++s;
  }
  {  // K-tile S-1
    const unsigned sto = (unsigned)((s & 1) * WG_STAGE);
    readB(sto, std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_barrier(0);
    readA(sto, std::integral_constant<int, 0>{});
    wait_vm<2>();                              // B1 of S-1
    sync_in();
    joinB(0);
    joinA();
    mfma_quad(0, 0);
    bias_quad(0);
    sync_out();
    readB(sto, std::integral_constant<int, 1>{});
    wait_vm<0>();                              // A1 of S-1
    sync_in();
    joinB(1);
    mfma_quad(0, 1);
    sync_out();
    readA(sto, std::integral_constant<int, 1>{});
    sync_in();
    joinA();
    mfma_quad(1, 1);
    bias_quad(1);
    sync_out();
    sync_in();
    mfma_quad(1, 0);
    sync_out();
  }
  if (!grp) __builtin_amdgcn_s_barrier();      // balance the second half's extra barrier

  // ---- epilogue: partial dW of this split.  Accumulator (16x16): column = lane & 15, row (co) =
  // 4 (lane >> 4) + r.  acc[qa*4 + ic][qb*2 + ip]: co = m0 + qa*128 + wc*64 + ic*16 + ...,
  // column = n0 + qb*128 + wp*32 + ip*16 + (lane & 15) = (tap, ci)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int ip = 0; ip < 2; ++ip) {
      const int col = n0 + qb * 128 + wp * 32 + ip * 16 + (lane & 15);
      if (col >= Ncols) continue;
      const int tap = col / a.Nc, ci = col - tap * a.Nc;
      float* dst = a.slab + (((long)split * T + tap) * a.M + m0 + wc * 64 + 4 * (lane >> 4)) * a.Nc + ci;
#pragma unroll
      for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int ic = 0; ic < 4; ++ic)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            dst[(long)(qa * 128 + ic * 16 + r) * a.Nc] = acc[qa * 4 + ic][qb * 2 + ip][r];
    }
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a.bslab[(long)split * a.M + m0 + qa * 128 + wc * 64 + wp * 16 + 4 * (lane >> 4) + r] = bacc[qa][r];
  }
}

// Eligible: conv3x3 s1 p1 (A = the output gradient, B = the layer input, same pixel grid), M % 256 == 0,
// Nc % 8 == 0, W % 64 == 0 or W == 32, H * W % 64 == 0, 16-B aligned channel strides; with per-image
// tables every split's images must be consecutive images of one tensor (host); pix_per_split = images per split (splits = ceil(N / ips)), >= 2 K-steps per split
// (the ragged last split included: the steady loop and its peeled tail need S >= 2),
// each split's images addressable with 32-bit offsets (abytes / bbytes = ips images).
DPA_API int dpa_wgrad_gemm(const WgradArgs* args, hipStream_t st) {
  const WgradArgs& a = *args;
  const int ips = a.pix_per_split;
  if (a.KW == 2) {
    // transposed conv k2 s2 (up mode): A = x [N][Hg][Wg][lda] (M = its channels), B = the output gradient
    // [N][2Hg][2Wg][ldb]; columns (tap, co), 4 taps; no bias from this kernel (bslab must be null)
    if ((a.M % 256) || ((4 * a.Nc) % 256) || (a.Nc % 8) || (a.lda & 7) || (a.ldb & 7) || a.s != 2 || a.pad != 0 ||
        a.bslab != nullptr || a.atab || a.btab || a.HA != a.Hg || a.WA != a.Wg || a.HB != 2 * a.Hg ||
        a.WB != 2 * a.Wg || (a.Wg % 64 && (a.Wg > 64 || 64 % a.Wg)) || ((a.Hg * a.Wg) % 64) || ips < 1 ||
        a.splits != (a.N + ips - 1) / ips || (long)ips * a.Hg * a.Wg / 64 < 2 ||
        (long)((a.N - 1) % ips + 1) * a.Hg * a.Wg / 64 < 2 || a.lda < a.M || a.ldb < a.Nc ||
        (long)ips * a.Hg * a.Wg * a.lda * 2 > (long)a.abytes || (long)ips * 4 * a.Hg * a.Wg * a.ldb * 2 > (long)a.bbytes)
      return (int)hipErrorInvalidValue;
    const int tiles = (a.M / 256) * (4 * a.Nc / 256);
    hipLaunchKernelGGL(wgrad_gemm_kernel, dim3(tiles * a.splits), dim3(512), 0, st, a);
    return (int)hipGetLastError();
  }
  if ((a.M % 256) || (a.Nc % 8) || (a.lda & 7) || (a.ldb & 7) || a.s != 1 || a.pad != 1 || a.KW != 3 ||
      a.HA != a.Hg || a.WA != a.Wg || a.HB != a.Hg || a.WB != a.Wg || (a.Wg % 64 && a.Wg != 32) ||
      ((a.Hg * a.Wg) % 64) || (!a.atab != !a.btab) || ips < 1 || a.splits != (a.N + ips - 1) / ips ||
      (long)ips * a.Hg * a.Wg / 64 < 2 || (long)((a.N - 1) % ips + 1) * a.Hg * a.Wg / 64 < 2 ||
      a.lda < a.M || a.ldb < a.Nc ||
      (long)ips * a.Hg * a.Wg * a.lda * 2 > (long)a.abytes || (long)ips * a.Hg * a.Wg * a.ldb * 2 > (long)a.bbytes)
    return (int)hipErrorInvalidValue;
  const int tiles = (a.M / 256) * ((9 * a.Nc + 255) / 256);
  hipLaunchKernelGGL(wgrad_gemm_kernel, dim3(tiles * a.splits), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}
