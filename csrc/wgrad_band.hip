// Deep-layer conv3x3 weight gradient with band-staged input rows (gfx950; reference
// model/unet_parts.py:10-12 -- enc.conv4, mid, dec.conv1 at 64^2 / 32^2).
//
// wgrad_gemm.hip runs dW[co][tap, ci] = sum_p g[p][co] x[p + delta(tap)][ci] as a plain 256 x 256 GEMM:
// per 64-pixel K-step it stages 32 KB of gradient (A) and 32 KB of tap-shifted input (B) by LDS-DMA, 8.4
// MFLOP per 64 KB = 128 FLOP/B.  Measured (profiles/pmc_b128_512_r05_end.txt) it sits at 41 % MFMA with a
// third of its wave cycles in waits: at ~12-13 B/clk/CU of LDS-DMA (MI355X_MICROARCH §latency table) that
// is the rate its bytes per FLOP allow (128 FLOP/B x 12.5 B/clk x 2.4 GHz x 256 CUs ~ 1 PF).  The nine B
// columns blocks of one input channel are nine shifted views of the SAME pixels, so here the tile spans the
// taps instead of the channels:
//   * workgroup tile = 256 output channels x (9 taps x 32 input channels) = 256 x 288;
//   * a K-step = 64 output pixels = R = 64 / W whole image rows; B is staged ONCE per K-step as the
//     (R + 2) x (W + 2) input band [rows h0-1 .. h0+R][cols -1 .. W] x 32 channels (64-B pixel rows) and all
//     nine taps read it at a (kh rows, kw pixels) offset: 32 KB A + 12 KB B per 9.4 MFLOP = 214 FLOP/B;
//   * zero padding: band rows outside the image by the buffer unit's range check (offset 0x80000000 ->
//     zeros), the two halo columns (always outside the image at W <= 64) zeroed once at the start;
//   * three K-step buffers (A and B), each K-step's loads issued two steps ahead; the 8 waves are 4 (64
//     output channels) x 2 (144 columns = 9 fragments) and the two column halves run one barrier apart
//     (wgrad_gemm.hip's ping-pong: one half issues its 36 MFMAs while the other reads fragments and DMAs);
//     a phase = one 32-pixel half of the K-step;
//   * fragments are transposed reads (ds_read_b64_tr_b16): the MFMA K dimension is the pixel;
//   * bias gradient (sum_p g[p][co]) in the channel-tile-0 workgroups: one MFMA per A fragment against a
//     ones fragment, two fragments per column half.
// One workgroup per (image group, tile); partial dW -> fp32 slab rows [split][tap][M][Nc] that
// dpa_wgrad_reduce sums in a fixed order (bitwise reproducible), exactly as wgrad_gemm.hip.
#include "conv_args.h"

#include <type_traits>

namespace {

// ds_read_b64_tr_b16 as inline asm (see wgrad_gemm.hip: the builtin makes hipcc drain the DMA pipeline
// before every read); the kernel waits lgkmcnt(0) itself before the MFMAs that consume the fragments
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

constexpr int BA_RB = 512;                // A image row: 256 gradient channels of one pixel
constexpr int BA_BYTES = 64 * BA_RB;      // one K-step of A: 64 pixels
constexpr int BB_RB = 64;                 // B image row: 32 input channels of one pixel
constexpr int NBUF = 3;                   // K-step buffers (loads run two steps ahead)

template <int W>
struct Band {
  static_assert(W == 32 || W == 64, "band staging covers 32- and 64-pixel rows");
  static constexpr int R = 64 / W;                      // image rows per K-step
  static constexpr int SP = W == 64 ? 80 : 48;          // LDS pixel rows per band row (>= W + 2, multiple of 16)
  static constexpr int ROWS = R + 2;                    // band rows
  static constexpr int B_BYTES = ROWS * SP * BB_RB;     // 15360 / 12288 (1-KB multiple)
  static constexpr int NBI_REAL = ROWS * W / 16;        // 1-KB DMA instructions per band: 12 / 8
  static constexpr int NBI = (NBI_REAL + 7) / 8;        // per wave (the surplus ones are zero-fill dummies)
  static constexpr int STAGE = BA_BYTES + B_BYTES;
  static constexpr int LDS = NBUF * STAGE + 1024;       // + a 1-KB dump for the dummy DMAs
};

}  // namespace

template <int W>
__global__ __launch_bounds__(512) void wgrad_band_kernel(WgradArgs a) {
  using G = Band<W>;
  __shared__ __attribute__((aligned(1024))) char lds[G::LDS];

  const int H = a.Hg;
  const int nct = a.Nc / 32, tiles = (a.M / 256) * nct;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;   // a split's tiles share an XCD's L2
  const int mt = tile / nct, ct = tile - mt * nct;
  const int m0 = mt * 256, ci0 = ct * 32;
  const int ips = a.pix_per_split;                             // images per split
  const int nimg0 = split * ips;
  const int nimg = min(ips, a.N - nimg0);
  const int spi = H / G::R;                                    // K-steps per image
  const int S = nimg * spi;
  const bool do_bias = a.bslab != nullptr && ct == 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wid & 3, nh = wid >> 2;                       // channel group, column half (= ping-pong half)

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.atab ? a.atab[nimg0] : a.A + (long)nimg0 * H * W * a.lda), 0, (int)a.abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.btab ? a.btab[nimg0] : a.B + (long)nimg0 * H * W * a.ldb), 0, (int)a.bbytes, 0x00020000);

  // ---- per-lane DMA constants.  A: K-step image [64 px][256 ch], 32 instructions of 1 KB (2 pixel rows
  // x 32 chunks); wave w issues instructions kk*16 + w and kk*16 + 8 + w of half kk.  Lane l: pixel row
  // 2 ins + (l >> 5), slot l & 31 <- global chunk (l & 31) ^ swz_kk<512>(row) (row & 15 is the same for
  // every instruction of the wave).
  const int arow = 2 * wid + (lane >> 5);
  const unsigned laneA = (unsigned)((arow * a.lda + m0 + (((lane & 31) ^ swz_kk<BA_RB>(arow)) * 8)) * 2);
  const unsigned rowA = (unsigned)(64 * a.lda * 2), insA = (unsigned)(16 * a.lda * 2);   // per K-step / per 16 px
  // B: band row r, 16-pixel block pb (instruction i = r * (W / 16) + pb); lane l: pixel 1 + 16 pb + (l >> 2)
  // of the band row, slot l & 3 <- chunk (l & 3) ^ swz_kk<64>(LDS row).  Source offset relative to the
  // K-step's first pixel; the row is valid iff 0 <= h0 - 1 + r < H.
  int laneB[G::NBI], bDst[G::NBI], bRow[G::NBI];
#pragma unroll
  for (int j = 0; j < G::NBI; ++j) {
    const int i = wid + 8 * j;
    const bool real = i < G::NBI_REAL;
    const int r = real ? i / (W / 16) : 0, pb = real ? i - r * (W / 16) : 0;
    const int c = 1 + 16 * pb + (lane >> 2);
    const int lr = r * G::SP + c;
    laneB[j] = (((r - 1) * W + 16 * pb + (lane >> 2)) * a.ldb + ci0 + (((lane & 3) ^ swz_kk<BB_RB>(lr)) * 8)) * 2;
    bDst[j] = real ? BA_BYTES + (r * G::SP + 1 + 16 * pb) * BB_RB : -1;   // -1: dummy (dump area)
    bRow[j] = r;
  }
  const unsigned rowB = (unsigned)(64 * a.ldb * 2);

  // zero the halo columns (band pixels 0 and W + 1 of every row of every buffer): never written by the DMA
  for (int e = tid; e < NBUF * G::ROWS * 2 * 4; e += 512) {
    const int chunk = e & 3, side = (e >> 2) & 1, rb = e >> 3;
    const int buf = rb / G::ROWS, r = rb - buf * G::ROWS;
    const int lr = r * G::SP + (side ? W + 1 : 0);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4_t*>(
        LDS_PTR(char, lds + buf * G::STAGE + BA_BYTES + lr * BB_RB + chunk * 16)) = u32x4_t{0u, 0u, 0u, 0u};
  }

  // K-step issue: A half kk and (kk == 1) the band of step sq into buffer bf; steps >= S load zeros
  // (range check) so every wave's vmcnt sequence is the same in every step
  auto issueA = [&](int kk, int bf, int sq) {
    char* base = lds + bf * G::STAGE + kk * (BA_BYTES / 2);
    const bool ok = sq < S;
    const unsigned o = (unsigned)sq * rowA + laneA + (unsigned)kk * 2 * insA;
    dma16(ar, base + wid * 1024, ok ? o : 0x80000000u);
    dma16(ar, base + (8 + wid) * 1024, ok ? o + insA : 0x80000000u);
  };
  auto issueB = [&](int bf, int sq, int h0) {
    char* base = lds + bf * G::STAGE;
#pragma unroll
    for (int j = 0; j < G::NBI; ++j) {
      const int h = h0 - 1 + bRow[j];
      const bool ok = sq < S && bDst[j] >= 0 && h >= 0 && h < H;
      const int o = (int)((unsigned)sq * rowB) + laneB[j];
      dma16(br, bDst[j] >= 0 ? base + bDst[j] : lds + NBUF * G::STAGE, ok ? (unsigned)o : 0x80000000u);
    }
  };

  // prologue: K-steps 0 and 1
  issueA(0, 0, 0);
  issueA(1, 0, 0);
  issueB(0, 0, 0);
  {
    const int t1 = spi > 1 ? 1 : 0;
    issueA(0, 1, 1);
    issueA(1, 1, 1);
    issueB(1, 1, t1 * G::R);
  }
  wait_vm<4 + G::NBI>();                                       // step 0 landed (step 1 may be in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // the halo zeros
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (nh) __builtin_amdgcn_s_barrier();                        // the second half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  // per-lane LDS byte offsets of the transposed fragment reads (conv_args.h tr_frag's addressing): lane
  // (g, q, p) reads k rows 8g + q + 4h, 4 columns at 4p
  const unsigned lds0 = (unsigned)(size_t)LDS_PTR(char, lds);
  // Only fragment 0 / channel half 0 is kept: the other A fragments (16 columns = chunk bits 1-2) and
  // the second 16-channel half of B (chunk bit 1) differ by an XOR of the chunk field, which the
  // swizzles (XOR of chunk bits 1-3) commute with -- (addr ^ ic*32), (addr ^ 32) on 1-KB-aligned stages.
  unsigned aoff[2], boff[3][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 8 * g + q + 4 * h;
      const int col = cg * 64 + 4 * p;
      aoff[h] = (unsigned)(r * BA_RB + (((col >> 3) ^ swz_kk<BA_RB>(r)) << 4) + (col & 7) * 2);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int rr = r + kw, cb = 4 * p;                   // band rows start at multiples of 16 LDS rows
        boff[kw][h] = (unsigned)(BA_BYTES + rr * BB_RB + (((cb >> 3) ^ swz_kk<BB_RB>(rr)) << 4) + (cb & 7) * 2);
      }
    }
  }

  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  const s16x8_t ones_s = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, ones_s);

  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // this phase's asm fragment reads
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // the K loop and epilogue, specialised per column half (its taps are compile-time)
  auto run = [&](auto NHc) {
    constexpr int NH = decltype(NHc)::value;
    f32x4_t acc[4][9];
#pragma unroll
    for (int ic = 0; ic < 4; ++ic)
#pragma unroll
      for (int f = 0; f < 9; ++f) acc[ic][f] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    f32x4_t bacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
    s16x4_t ra[4][2], rb[9][2];

    // one phase: 32-pixel half KK of the K-step in buffer `stage` (LDS byte offset)
    auto reads = [&](unsigned stage, auto KKc) {
      constexpr int KK = decltype(KKc)::value;
      // B fragments: F = NH * 9 + f -> tap F >> 1 (kh, kw), channel half F & 1; band row (KK * 32) / W + kh,
      // band pixel (KK * 32) % W + kw
#define DPA_BAND_B(f)                                                                          \
  {                                                                                            \
    constexpr int F = NH * 9 + (f), tap = F >> 1, jj = F & 1, kh = tap / 3, kw = tap % 3;     \
    constexpr int O = (((KK * 32) / W + kh) * Band<W>::SP + (KK * 32) % W) * BB_RB;          \
    rb[f][0] = trld<O>((boff[kw][0] + stage) ^ (jj * 32u));                                    \
    rb[f][1] = trld<O>((boff[kw][1] + stage) ^ (jj * 32u));                                    \
  }
      DPA_BAND_B(0) DPA_BAND_B(1) DPA_BAND_B(2) DPA_BAND_B(3) DPA_BAND_B(4)
      DPA_BAND_B(5) DPA_BAND_B(6) DPA_BAND_B(7) DPA_BAND_B(8)
#undef DPA_BAND_B
      constexpr int OA = KK * 32 * BA_RB;
      const unsigned a0 = aoff[0] + stage, a1 = aoff[1] + stage;
#pragma unroll
      for (int ic = 0; ic < 4; ++ic) {
        ra[ic][0] = trld<OA>(a0 ^ (ic * 32u));
        ra[ic][1] = trld<OA>(a1 ^ (ic * 32u));
      }
    };
    auto mfmas = [&]() {
      bf16x8_t af[4];
#pragma unroll
      for (int ic = 0; ic < 4; ++ic) af[ic] = tr_join(ra[ic][0], ra[ic][1]);
#pragma unroll
      for (int f = 0; f < 9; ++f) {
        const bf16x8_t bf = tr_join(rb[f][0], rb[f][1]);
#pragma unroll
        for (int ic = 0; ic < 4; ++ic)
          acc[ic][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bf, acc[ic][f], 0, 0, 0);
      }
      if (do_bias) {
        bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[NH * 2], ones, bacc[0], 0, 0, 0);
        bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[NH * 2 + 1], ones, bacc[1], 0, 0, 0);
      }
    };

    int tq = 2 % spi, hq = tq * G::R;                         // image row of the step being issued (s + 2)
    int cur = 0, iss = 2;
    for (int s = 0; s < S; ++s) {
      const unsigned stage = lds0 + (unsigned)(cur * G::STAGE);
      // phase 0: pixels 0-31 of step s; issue A half 0 of step s + 2
      reads(stage, std::integral_constant<int, 0>{});
      issueA(0, iss, s + 2);
      sync_in();
      mfmas();
      sync_out();
      // phase 1: pixels 32-63; issue A half 1 and the band of step s + 2; this wave's A(s + 1), B(s + 1)
      // landed before the barrier (the first one after which any wave reads step s + 1 is the next)
      reads(stage, std::integral_constant<int, 1>{});
      issueA(1, iss, s + 2);
      issueB(iss, s + 2, hq);
      wait_vm<4 + G::NBI>();
      sync_in();
      mfmas();
      sync_out();
      cur = cur == NBUF - 1 ? 0 : cur + 1;
      iss = iss == NBUF - 1 ? 0 : iss + 1;
      if (++tq == spi) tq = 0;
      hq = tq * G::R;
    }
    wait_vm<0>();                                              // no DMA may land after the workgroup ends
    if (!NH) __builtin_amdgcn_s_barrier();                     // balance the second half's extra barrier

    // ---- epilogue: accumulator (16x16) column = lane & 15, row (co) = 4 (lane >> 4) + r;
    // acc[ic][f]: co = m0 + cg*64 + ic*16 + ..., column F = NH*9 + f = (tap F >> 1, ci ci0 + (F & 1)*16 + lane & 15)
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      const int F = NH * 9 + f, tap = F >> 1;
      const int ci = ci0 + (F & 1) * 16 + (lane & 15);
      float* dst = a.slab + (((long)split * 9 + tap) * a.M + m0 + cg * 64 + 4 * (lane >> 4)) * a.Nc + ci;
#pragma unroll
      for (int ic = 0; ic < 4; ++ic)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(long)(ic * 16 + r) * a.Nc] = acc[ic][f][r];
    }
    if (do_bias && (lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          a.bslab[(long)split * a.M + m0 + cg * 64 + (NH * 2 + i) * 16 + 4 * (lane >> 4) + r] = bacc[i][r];
    }
  };
  if (nh) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
}

// ------------------------------------------------------------------------------------------------
// 128-output-channel form (the 128^2 level of the reference UNet -- enc.conv3, dec.conv2 -- and any grid with
// W % 64 == 0): 128 co x (9 taps x 64 ci) = 128 x 576 per workgroup; a K-step = 64 pixels of ONE image row
// (w0 = 0, 64, ...).  The band is 3 rows x 72 pixels x 64 channels (128-B pixel rows): band pixel c <-> image
// column w0 - 1 + c, nine 1-KB DMA instructions per row whose lanes outside the image read zeros (per-lane
// range check) -- at interior strips the halo columns are real pixels.  16 KB A + 27 KB B per 9.4 MFLOP.
// Waves: 2 (64 output channels) x 4 (16-channel quarter j of the 64, all nine taps): every wave's taps are
// compile-time and its quarter is an XOR of the fragment address (chunk bits 1-2, which the swizzle
// commutes with).  Splits are ranges of K-steps (pix_per_split pixels, a multiple of 64): a split may start
// inside an image (256 K-steps per 128^2 image).
namespace {
constexpr int B1_RB = 128;                       // B pixel row: 64 input channels
constexpr int B1_SP = 80;                        // LDS pixel rows per band row (72 used)
constexpr int B1_BYTES = 3 * B1_SP * B1_RB;      // 30720
constexpr int A1_RB = 256;                       // A pixel row: 128 gradient channels
constexpr int A1_BYTES = 64 * A1_RB;             // 16384
constexpr int S1 = A1_BYTES + B1_BYTES;          // 47104 per K-step buffer
constexpr int NBI1 = 4;                          // 27 band instructions over 8 waves (5 zero-fill dummies)
constexpr int LDS1 = NBUF * S1 + 1024;
}  // namespace

__global__ __launch_bounds__(512) void wgrad_band128_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS1];

  const int H = a.Hg, W = a.Wg, HW = H * W;
  const int spi = HW / 64;                                     // K-steps per image
  const long stot = (long)a.N * spi;
  const int sps = a.pix_per_split / 64;                        // K-steps per split
  const int nct = a.Nc / 64, tiles = (a.M / 128) * nct;
  const int bid = xcd_remap(blockIdx.x, tiles * a.splits);
  const int split = bid / tiles, tile = bid - split * tiles;   // a split's tiles share an XCD's L2
  const int mt = tile / nct, ct = tile - mt * nct;
  const int m0 = mt * 128, ci0 = ct * 64;
  const long gs0 = (long)split * sps;                          // the split's first K-step
  const int S = (int)min((long)sps, stot - gs0);
  const int n0 = (int)(gs0 / spi), ls0 = (int)(gs0 - (long)n0 * spi);
  const bool do_bias = a.bslab != nullptr && ct == 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wid & 1, jq = wid >> 1, grp = wid >> 2;      // channel group, channel quarter, ping-pong half

  // buffers from the split's first image; per-image tables: the host keeps a split inside one tensor and
  // passes its extent (abytes / bbytes), else everything up to the batch's end (clamped to 31 bits)
  const unsigned arec = a.atab ? a.abytes : (unsigned)min((long)(a.N - n0) * HW * a.lda * 2, 0x7fffffffL);
  const unsigned brec = a.btab ? a.bbytes : (unsigned)min((long)(a.N - n0) * HW * a.ldb * 2, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.atab ? a.atab[n0] : a.A + (long)n0 * HW * a.lda), 0, (int)arec, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.btab ? a.btab[n0] : a.B + (long)n0 * HW * a.ldb), 0, (int)brec, 0x00020000);

  // ---- DMA constants.  A: [64 px][128 ch], 16 instructions of 1 KB (4 pixel rows x 16 chunks); wave w
  // issues instruction kk*8 + w of half kk; lane l: pixel row 4 ins + (l >> 4), slot l & 15 <- chunk
  // (l & 15) ^ swz_kk<256>(row).
  const int arow = 4 * wid + (lane >> 4);
  const unsigned laneA = (unsigned)((arow * a.lda + m0 + (((lane & 15) ^ swz_kk<A1_RB>(arow)) * 8)) * 2);
  const unsigned stepA = (unsigned)(64 * a.lda * 2), halfA = (unsigned)(32 * a.lda * 2);
  // B: band row r, 8-pixel block ib (instruction i = 9 r + ib); lane l: band pixel c = 8 ib + (l >> 3), slot
  // l & 7 <- chunk (l & 7) ^ swz_kk<128>(LDS row); source relative to the K-step's first pixel (h0, w0)
  int laneB[NBI1], bDst[NBI1], bRow[NBI1], bCol[NBI1];
#pragma unroll
  for (int jj = 0; jj < NBI1; ++jj) {
    const int i = wid + 8 * jj;
    const bool real = i < 27;
    const int r = real ? i / 9 : 0, ib = real ? i - 9 * r : 0;
    const int c = 8 * ib + (lane >> 3);
    const int lr = r * B1_SP + c;
    laneB[jj] = (((r - 1) * W + (c - 1)) * a.ldb + ci0 + (((lane & 7) ^ swz_kk<B1_RB>(lr)) * 8)) * 2;
    bDst[jj] = real ? A1_BYTES + (r * B1_SP + 8 * ib) * B1_RB : -1;
    bRow[jj] = r;
    bCol[jj] = 8 * ib - 1;                                     // + (lane >> 3): image column - w0
  }
  const int l3 = lane >> 3;
  const unsigned stepB = (unsigned)(64 * a.ldb * 2);

  auto issueA = [&](int kk, int bf, int s, int lsq) {          // lsq: K-step index relative to image n0
    const bool ok = s < S;
    dma16(ar, lds + bf * S1 + kk * (A1_BYTES / 2) + wid * 1024,
          ok ? (unsigned)lsq * stepA + laneA + (unsigned)kk * halfA : 0x80000000u);
  };
  auto issueB = [&](int bf, int s, int lsq, int h0, int w0) {
#pragma unroll
    for (int jj = 0; jj < NBI1; ++jj) {
      const int h = h0 - 1 + bRow[jj], w = w0 + bCol[jj] + l3;
      const bool ok = s < S && bDst[jj] >= 0 && h >= 0 && h < H && w >= 0 && w < W;
      const int o = (int)((unsigned)lsq * stepB) + laneB[jj];
      dma16(br, bDst[jj] >= 0 ? lds + bf * S1 + bDst[jj] : lds + NBUF * S1, ok ? (unsigned)o : 0x80000000u);
    }
  };
  // image row / column of the K-step ls (relative to image n0)
  auto coords = [&](int ls, int& h0, int& w0) {
    const int t = ls % spi;
    h0 = (t * 64) / W;
    w0 = t * 64 - h0 * W;
  };

  int h0, w0;
  coords(ls0, h0, w0);
  issueA(0, 0, 0, ls0);
  issueA(1, 0, 0, ls0);
  issueB(0, 0, ls0, h0, w0);
  coords(ls0 + 1, h0, w0);
  issueA(0, 1, 1, ls0 + 1);
  issueA(1, 1, 1, ls0 + 1);
  issueB(1, 1, ls0 + 1, h0, w0);
  wait_vm<2 + NBI1>();                                         // step 0 landed (step 1 may be in flight)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();                       // the second half runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  // fragment read offsets (tr_frag addressing; lane (g, q, p) reads k rows 8g + q + 4h, 4 columns at 4p):
  // A fragment 0 of the wave's 64 channels (fragment ic: ^ ic * 32); B with the wave's quarter folded in
  const unsigned lds0 = (unsigned)(size_t)LDS_PTR(char, lds);
  unsigned aoff[2], boff[3][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 8 * g + q + 4 * h;
      const int col = cg * 64 + 4 * p;
      aoff[h] = (unsigned)(r * A1_RB + (((col >> 3) ^ swz_kk<A1_RB>(r)) << 4) + (col & 7) * 2);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int rr = r + kw, cb = jq * 16 + 4 * p;         // band rows start at multiples of 16 LDS rows
        boff[kw][h] = (unsigned)(A1_BYTES + rr * B1_RB + (((cb >> 3) ^ swz_kk<B1_RB>(rr)) << 4) + (cb & 7) * 2);
      }
    }
  }

  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  const s16x8_t ones_s = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, ones_s);

  f32x4_t acc[4][9];
#pragma unroll
  for (int ic = 0; ic < 4; ++ic)
#pragma unroll
    for (int f = 0; f < 9; ++f) acc[ic][f] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t bacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  s16x4_t ra[4][2], rb[9][2];

  auto reads = [&](unsigned stage, auto KKc) {
    constexpr int KK = decltype(KKc)::value;
#define DPA_BAND1_B(f)                                                                         \
  {                                                                                            \
    constexpr int kh = (f) / 3, kw = (f) % 3;                                                  \
    constexpr int O = (kh * B1_SP + KK * 32) * B1_RB;                                          \
    rb[f][0] = trld<O>(boff[kw][0] + stage);                                                   \
    rb[f][1] = trld<O>(boff[kw][1] + stage);                                                   \
  }
    DPA_BAND1_B(0) DPA_BAND1_B(1) DPA_BAND1_B(2) DPA_BAND1_B(3) DPA_BAND1_B(4)
    DPA_BAND1_B(5) DPA_BAND1_B(6) DPA_BAND1_B(7) DPA_BAND1_B(8)
#undef DPA_BAND1_B
    constexpr int OA = KK * 32 * A1_RB;
    const unsigned a0 = aoff[0] + stage, a1 = aoff[1] + stage;
#pragma unroll
    for (int ic = 0; ic < 4; ++ic) {
      ra[ic][0] = trld<OA>(a0 ^ (ic * 32u));
      ra[ic][1] = trld<OA>(a1 ^ (ic * 32u));
    }
  };
  auto mfmas = [&]() {
    bf16x8_t af[4];
#pragma unroll
    for (int ic = 0; ic < 4; ++ic) af[ic] = tr_join(ra[ic][0], ra[ic][1]);
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      const bf16x8_t bf = tr_join(rb[f][0], rb[f][1]);
#pragma unroll
      for (int ic = 0; ic < 4; ++ic)
        acc[ic][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bf, acc[ic][f], 0, 0, 0);
    }
    if (do_bias) {                                             // quarters 0 / 1 sum fragments 0-1 / 2-3
      if (jq == 0) {
        bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], ones, bacc[0], 0, 0, 0);
        bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], ones, bacc[1], 0, 0, 0);
      } else if (jq == 1) {
        bacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], ones, bacc[0], 0, 0, 0);
        bacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[3], ones, bacc[1], 0, 0, 0);
      }
    }
  };
  auto sync_in = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  int lsq = ls0 + 2;                                           // the step being issued (s + 2), rel. to image n0
  coords(lsq, h0, w0);
  int cur = 0, iss = 2;
  for (int s = 0; s < S; ++s) {
    const unsigned stage = lds0 + (unsigned)(cur * S1);
    reads(stage, std::integral_constant<int, 0>{});
    issueA(0, iss, s + 2, lsq);
    sync_in();
    mfmas();
    sync_out();
    reads(stage, std::integral_constant<int, 1>{});
    issueA(1, iss, s + 2, lsq);
    issueB(iss, s + 2, lsq, h0, w0);
    wait_vm<2 + NBI1>();                                       // A(s + 1), B(s + 1) of this wave landed
    sync_in();
    mfmas();
    sync_out();
    cur = cur == NBUF - 1 ? 0 : cur + 1;
    iss = iss == NBUF - 1 ? 0 : iss + 1;
    ++lsq;
    w0 += 64;
    if (w0 == W) {
      w0 = 0;
      if (++h0 == H) h0 = 0;
    }
  }
  wait_vm<0>();                                                // no DMA may land after the workgroup ends
  if (!grp) __builtin_amdgcn_s_barrier();                      // balance the second half's extra barrier

  // ---- epilogue: acc[ic][f]: co = m0 + cg*64 + ic*16 + 4 (lane >> 4) + r, tap f, ci = ci0 + jq*16 + (lane & 15)
  const int ci = ci0 + jq * 16 + (lane & 15);
#pragma unroll
  for (int f = 0; f < 9; ++f) {
    float* dst = a.slab + (((long)split * 9 + f) * a.M + m0 + cg * 64 + 4 * (lane >> 4)) * a.Nc + ci;
#pragma unroll
    for (int ic = 0; ic < 4; ++ic)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(long)(ic * 16 + r) * a.Nc] = acc[ic][f][r];
  }
  if (do_bias && jq < 2 && (lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a.bslab[(long)split * a.M + m0 + cg * 64 + (2 * jq + i) * 16 + 4 * (lane >> 4) + r] = bacc[i][r];
  }
}

// Eligible: conv3x3 s1 p1 (A = the output gradient, B = the layer input, same pixel grid), W in {32, 64},
// H % (64 / W) == 0, M % 256 == 0, Nc % 32 == 0, 16-B aligned channel strides; per-image tables as
// wgrad_gemm.hip (every split's images consecutive images of one tensor); pix_per_split = images per split
// (splits = ceil(N / ips)); each split's images addressable with 32-bit offsets.
DPA_API int dpa_wgrad_band(const WgradArgs* args, hipStream_t st) {
  const WgradArgs& a = *args;
  const int ips = a.pix_per_split;
  if ((a.M % 256) || (a.Nc % 32) || a.Nc < 32 || (a.lda & 7) || (a.ldb & 7) || a.s != 1 || a.pad != 1 ||
      a.KW != 3 || a.HA != a.Hg || a.WA != a.Wg || a.HB != a.Hg || a.WB != a.Wg || (a.Wg != 64 && a.Wg != 32) ||
      (a.Hg % (64 / a.Wg)) || (!a.atab != !a.btab) || ips < 1 || a.N < 1 || a.splits != (a.N + ips - 1) / ips ||
      a.lda < a.M || a.ldb < a.Nc ||
      (long)ips * a.Hg * a.Wg * a.lda * 2 > (long)a.abytes || (long)ips * a.Hg * a.Wg * a.ldb * 2 > (long)a.bbytes ||
      (long)ips * a.Hg * a.Wg * a.lda * 2 >= (1L << 31) || (long)ips * a.Hg * a.Wg * a.ldb * 2 >= (1L << 31))
    return (int)hipErrorInvalidValue;
  const int tiles = (a.M / 256) * (a.Nc / 32);
  if (a.Wg == 64)
    hipLaunchKernelGGL(wgrad_band_kernel<64>, dim3(tiles * a.splits), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL(wgrad_band_kernel<32>, dim3(tiles * a.splits), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// Eligible: conv3x3 s1 p1 on one grid, W % 64 == 0, M % 128 == 0, Nc % 64 == 0, 16-B aligned channel strides;
// pix_per_split = pixels per split (a positive multiple of 64), splits = ceil(N H W / pix_per_split); a split's
// span from its first image addressable with 32-bit offsets; per-image tables: whole-image splits
// (pix_per_split % (H W) == 0) inside one tensor, abytes / bbytes = a split's extent.
DPA_API int dpa_wgrad_band128(const WgradArgs* args, hipStream_t st) {
  const WgradArgs& a = *args;
  const long HW = (long)a.Hg * a.Wg, pps = a.pix_per_split;
  if ((a.M % 128) || a.M < 128 || (a.Nc % 64) || a.Nc < 64 || (a.lda & 7) || (a.ldb & 7) || a.s != 1 ||
      a.pad != 1 || a.KW != 3 || a.HA != a.Hg || a.WA != a.Wg || a.HB != a.Hg || a.WB != a.Wg || a.Wg < 64 ||
      (a.Wg % 64) || a.Hg < 1 || a.N < 1 || (!a.atab != !a.btab) || pps < 64 || (pps % 64) ||
      a.splits != ((long)a.N * HW + pps - 1) / pps || a.lda < a.M || a.ldb < a.Nc ||
      (pps + 2 * HW) * a.lda * 2 >= (1L << 31) || (pps + 2 * HW) * a.ldb * 2 >= (1L << 31))
    return (int)hipErrorInvalidValue;
  if (a.atab && ((pps % HW) || pps * a.lda * 2 > (long)a.abytes || pps * a.ldb * 2 > (long)a.bbytes))
    return (int)hipErrorInvalidValue;
  const int tiles = (a.M / 128) * (a.Nc / 64);
  hipLaunchKernelGGL(wgrad_band128_kernel, dim3(tiles * a.splits), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}
