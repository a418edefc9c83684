// Fused backward of a full-resolution conv3x3 (s1 p1) for 32/64-channel layers: input gradient AND
// weight + bias gradient in ONE pass over the row stream (reference layers: the 512^2 / 256^2
// conv_blocks of model/unet_parts.py:9-14; SURVEY K2 + K3 + K4-bwd).
//
// Why: at these widths both backward GEMMs are bound by HBM traffic, not MFMAs.  Run separately,
// the dgrad reads g (the ReLU-masked output gradient) and the layer input x (for ReLU mask of the
// input gradient) and writes dx, and the weight gradient reads g and x AGAIN: 5 activation-sized
// passes per conv (21.5 GB per 32->32 conv at 512^2, batch 256).  Here one block streams the rows
// of an image column strip once: g rows go through one 4-slot LDS ring, x rows through another,
// and for every output row the block
//   * computes the dx row from the three g rows in the ring with the dgrad weights resident in LDS
//     (the igemm_stream schedule: 9 taps x 32-channel slices of 16x16x32 bf16 MFMAs),
//   * masks it with x > 0 read from the x ring (EPI 0: the input is a ReLU output), or splits it
//     into the two halves of a concat gradient (EPI 1), or stores it as is (EPI 2),
//   * accumulates dW[tap][co][ci] += sum_px g[h][px][co] * x[h+kh-1][px+kw-1][ci] from the same ring
//     slots (transposed LDS reads, ds_read_b64_tr_b16; fp32 accumulators live in registers for the
//     whole block), and db[co] += sum_px g[h][px][co],
// so every byte of g and x is read from HBM ~once ((BP+2)/BP) and dx written once: 3 passes.
// Each block writes its partial dW / db as fp32 slab rows; dpa_wgrad_reduce sums them in a fixed
// order (bitwise reproducible) into the flat gradient buffer.
//
// Wave roles: dx row = WPX waves along the pixels x WCS along the channels (as igemm_stream);
// weight gradient = wave w owns input-channel tile (w % NTI), output-channel tiles
// [msp*MTW, msp*MTW + MTW) (msp = w / NTI % MSPL) for all 9 taps, over the pixel k-steps
// pg + j*PG of the row (pg = w / (NTI*MSPL)); the PG pixel groups write separate slab rows.
#include "conv_args.h"

struct BwdArgs {
  const bf16_t* g;      // gradient w.r.t. the conv output [N][H][W][ldg], CO channels (ReLU mask applied)
  const bf16_t* x;      // conv input [N][H][W][ldx], CI channels
  const bf16_t* wd;     // dgrad-packed weights [CI][Kd]: k = tap*CO + co (pack mode 1, taps flipped)
  bf16_t* y;            // dx [N][H][W][ldy] (EPI 1: channels < split)
  bf16_t* y2;           // EPI 1: channels >= split -> y2[..][c - split]
  float* slab;          // [nblocks*PG][9][CO][CI] partial weight gradients
  float* bslab;         // [nblocks*PG][CO] partial bias gradients (rows of pixel group > 0 zero) or null
  int ldg, ldx, ldy, ldy2, split, Kd;
  int N, H, W;
  int rh, ipb;          // rows per block, images per block
  unsigned gbytes, xbytes;  // addressable bytes of ONE image of g / x (buffer offsets are per image)
  // HEAD mode (last decoder conv feeding the fused segmentation head): `g` is the conv's OUTPUT y and
  // the gradient is formed on load, g = dz * hw[c] * (y > 0) with z = hb + sum_c hw[c] y[c],
  // p = sigmoid(z), dz from the BCE/Dice partial-sum gradient dS (head_bwd_kernel's formula);
  // the segmap gradients sum_p dz*y[c], sum_p dz go to hslab[block][C+1].
  const float* tgt; const float* hw; const float* hb; const float* dS; float* hslab;
  // POOL mode (encoder conv2 whose output was max-pooled with window codes): `g` is the skip gradient
  // dskip (or null) and the gradient is formed on load as in pool_bwd_code_kernel,
  //   g[p][c] = (dskip[p][c] + (argmax(window)[c] == q(p) ? dpool[window][c] : 0)) * mask_q(p)[c]
  const unsigned char* pcode; const bf16_t* dpool; int ldp;
  // W1 mode (POOL, 32 -> 32, the first encoder level): the input gradient of this conv is the output
  // gradient of the level's FIRST conv (input x1: the 8-channel padded image [N][H][W][8]), whose only
  // remaining use is that conv's weight + bias gradient.  It is not stored: each dx row goes (ReLU-
  // masked, bf16) into an LDS buffer and the next row step accumulates dW1[tap][co][ci] +=
  // sum_px dx[h][px][co] * x1[h+kh-1][px+kw-1][ci] from it and an x1 row ring; partials go to
  // slab1 [nblocks][9][32][8] / bslab1 [nblocks][32].
  const bf16_t* x1; float* slab1; float* bslab1; unsigned x1bytes;
  // BN mode (the conv is followed by BatchNorm + ReLU): `g` is the ReLU-masked gradient of the BN
  // output and the conv-output gradient is formed on load with bn_bwd_apply's formula,
  //   dz = bncoef[c] g + bncoef[CO + c] z + bncoef[2 CO + c]     (z: the BN input, ldz == ldg),
  // zero outside the image (the conv's zero padding), so the dz pass over HBM never happens.
  const bf16_t* z; const float* bncoef;
  // BN statistics of the layer BELOW (its ReLU output is this conv's input x, the dx mask): per block
  // and channel, sum dx and sum dx*x of the stored masked dx -> bnslab[block][2][CI] (the partial
  // sums igemm_stream's EPI 5 writes; bn_bwd_finalize_kernel's gy mode consumes them)
  float* bnslab;
  // HEAD mode: the forward's per-pixel probability p = sigmoid(z) [N*H*W] (igemm_stream's fused head
  // epilogue writes it), read per pixel instead of the 32-channel dot + sigmoid
  const float* hprob;
  // dual input (CI == 64): channels 32-63 of x come from this second tensor, laid out like x (same
  // ldx, xbytes) -- the decoder conv over [skip | up] without a concat buffer
  const bf16_t* x2;
  // BN-on-load of x (BN mode 2: x is the ReLU output of a BatchNorm layer below): x holds that layer's
  // pre-BN output z and the loader forms relu(z * xbn[c] + xbn[CI + c]) (the forward's bn_apply
  // arithmetic) -- the BN output is never stored in the forward
  const float* xbn;
  // HEAD + BN mode (the last decoder conv is followed by BatchNorm + ReLU and then the head): `g` is the
  // conv's pre-BN output z (the BN input, also `z`) and the head gradient of y = relu(z * ybn[c] +
  // ybn[CO + c]) is formed on load (p from hprob), then the BN backward (bncoef) -- neither the BN output
  // nor the head gradient is ever stored.  The segmap gradients come from the statistics pass before.
  const float* ybn;
};

// 8 consecutive k (pixel rows roff+8g .. +7) of 16 channels starting at col0, from an nk image
// ([rows][32 channels], 64-B rows, swz_nk<32> chunk swizzle): the tr_frag of conv_args.h for the
// dgrad-friendly layout of the g ring.
__device__ __forceinline__ bf16x8_t tr_frag_nk32(const char* img, int col0, int lane, int roff) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = col0 + 4 * p;
  const int ch = col >> 3, hb = (col & 7) * 2;
  const int r0 = roff + 8 * g + q, r1 = r0 + 4;
  const char* a0 = img + r0 * 64 + (swz_nk<32>(r0, ch) << 4) + hb;
  const char* a1 = img + r1 * 64 + (swz_nk<32>(r1, ch) << 4) + hb;
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, a0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, a1));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// the two ds_read_b64_tr_b16 of a transposed fragment at precomputed byte offsets (see tr_frag)
__device__ __forceinline__ bf16x8_t tr_pair(const char* base, int off0, int off1) {
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + off1));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// (head + BN mode: one 8-wave block per CU -- its registers do not fit two 4-wave blocks without spilling)
template <int BP, int CI, int CO, int NW, int PG, int EPI, bool HEAD, bool POOL, bool W1, int BNM>
__global__ __launch_bounds__(64 * NW, (HEAD && BNM) ? 1 : 2) void bwd_stream_kernel(BwdArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int HR = BP + 2;                   // ring row: BP pixels + 1 halo pixel each side
  constexpr int KSO = CO / 32;                 // 32-channel slices of g
  constexpr int WBYTES = 9 * KSO * CI * 64;    // dgrad weights [tap][ks][CI][32] (nk)
  constexpr int GSLOT = KSO * HR * 64;         // g row [ks][HR][32] (nk)
  constexpr int RBX = CI * 2;                  // x row image [HR][CI] (kk)
  constexpr int XSLOT = HR * RBX;
  constexpr int WCS = NW == 8 ? 2 : 1, WPX = NW / WCS;
  constexpr int WP = BP / WPX, TP = WP / 16;
  constexpr int WCN = CI / WCS, TC = WCN / 16;
  constexpr int NTI = CI / 16, MTI = CO / 16;
  constexpr int MSPL = NW / (NTI * PG), MTW = MTI / MSPL;
  constexpr int KST = BP / 32 / PG;            // pixel k-steps per wave per row
  static_assert(TP >= 1 && TC >= 1 && MSPL >= 1 && NTI * MSPL * PG == NW && MTW * MSPL == MTI && (BP / 32) % PG == 0,
                "tile");
  static_assert(!HEAD || (CO == 32 && EPI == 0), "head mode: 32-channel last decoder conv");
  static_assert(!(HEAD && POOL), "one gradient source");
  static_assert(!W1 || (POOL && CI == 32 && CO == 32 && EPI == 0 && BP % 32 == 0), "W1 mode");
  // BNM: 0 none, 1 BatchNorm backward on load, 2 that + the layer below's BN statistics from dx
  constexpr bool BNL = BNM >= 1, BNS = BNM == 2;
  static_assert(!BNM || !(POOL || W1), "BN mode: plain or head gradient source");
  static_assert(!(HEAD && BNM == 1), "head + BN: with the layer below's BN statistics (mode 2)");
  static_assert(!BNS || EPI == 0, "BN statistics of the layer below need the masked dx");
  // W1: x1 row ring (5 slots: the delayed dW1 step still reads row h-2 while row h+2 is stored),
  // dx row double buffer [BP][32] (nk, swz_nk<32>), per-wave tiles of the 32 x (9 taps x 8) dW1
  constexpr int X1SLOT = HR * 16, G1SLOT = BP * 64;
  constexpr int W1BYTES = W1 ? 5 * X1SLOT + 2 * G1SLOT : 0;
  constexpr int GCH = KSO * HR * 4, XCH = HR * (CI / 8);         // 16-B chunks per ring row
  // dual input (CI == 64, a.x2): plane-major x chunks, each 32-channel plane padded to whole waves
  // so every wave's loads use one buffer resource (no more load slots than the interleaved mapping)
  constexpr int PLX = (HR * 4 + 63) / 64 * 64;
  constexpr int LX0 = (XCH + NT - 1) / NT, LX1 = CI == 64 ? (2 * PLX + NT - 1) / NT : 0;
  constexpr int LG = (GCH + NT - 1) / NT, LX = LX0 > LX1 ? LX0 : LX1;
  constexpr int BCH = BP * 4 * KSO, LBI = (BCH + NT - 1) / NT;   // bias: chunks of the g row's BP pixels
  __shared__ __attribute__((aligned(16))) char lds[WBYTES + 4 * GSLOT + 4 * XSLOT + W1BYTES];
  __shared__ __attribute__((aligned(16))) float bnc[BNL ? 3 * CO : 4];   // BN mode: the dz coefficients
  constexpr bool HBN = HEAD && BNL;             // head gradient of relu(bn(z)) formed on load, then dz
  __shared__ __attribute__((aligned(16))) float ybc[HBN ? 3 * CO : 4];   // HBN: [scale | shift | segmap w]
  // x = relu(bn(z)) formed on load (a.xbn): BN mode 2, and mode 1 with a dual input (x only, not x2 --
  // the decoder conv over [skip | up] whose skip is the encoder BN's input z)
  constexpr bool XBN = BNL;
  // where the row loop runs the loader transforms (rxform): in BN mode 2 at 64 input channels right after the
  // dx MFMAs.  Mode 1 keeps them next to the ring store: early, the dual-input split kernel (64 -> 32,
  // EPI 1) took 8.37 vs 7.77 ms per b256 step and the halves kernel 5.97 vs 6.01 (kernel traces,
  // profiles/bn_mode1_early_vs_late_r05.txt; the end-to-end A/B, +0.3 %, was within noise)
  constexpr bool EARLY_XFORM = BNS && CI == 64;
  __shared__ __attribute__((aligned(16))) float xbc[XBN ? 2 * CI : 4];
  char* const Wimg = lds;
  char* const Gring = lds + WBYTES;
  char* const Xring = Gring + 4 * GSLOT;
  char* const X1ring = Xring + 4 * XSLOT;
  char* const G1buf = X1ring + 5 * X1SLOT;

  const int stripsW = (a.W + BP - 1) / BP, segsH = (a.H + a.rh - 1) / a.rh;   // ragged last strip allowed
  const int split_id = blockIdx.x;
  const int ig = split_id / (segsH * stripsW);
  const int rem = split_id - ig * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * BP, h0 = hs * a.rh;
  const int nrows = min(a.rh, a.H - h0);
  const int nimg = min(a.ipb, a.N - ig * a.ipb);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid % WPX, wc = wid / WPX;                      // dx role
  const int nt = wid % NTI, msp = (wid / NTI) % MSPL, pg = wid / (NTI * MSPL);   // dW role
  // buffer resources are rebuilt per image (32-bit offsets stay inside one image at any batch size)
  __amdgpu_buffer_rsrc_t gr, xr, x2r, yr, y2r, tr, hpr, pr, cr, x1r, zr;
  const bool has_g = !POOL || a.g != nullptr;
  const bool dual = CI == 64 && a.x2 != nullptr;
  auto bind = [&](int img) {
    const long pix = (long)img * a.H * a.W;
    if constexpr (POOL) {
      const long win = (long)img * (a.H >> 1) * (a.W >> 1);
      pr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.dpool + win * a.ldp), 0, 0x7fffffff, 0x00020000);
      cr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.pcode + win * CO), 0, 0x7fffffff, 0x00020000);
    }
    if constexpr (HEAD) {
      tr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.tgt + pix), 0, a.H * a.W * 4, 0x00020000);
      hpr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.hprob + pix), 0, a.H * a.W * 4, 0x00020000);
    }
    if constexpr (W1) x1r = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x1 + pix * 8), 0, (int)a.x1bytes, 0x00020000);
    if constexpr (BNL) zr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.z + pix * a.ldg), 0, (int)a.gbytes, 0x00020000);
    gr = __builtin_amdgcn_make_buffer_rsrc((void*)(has_g ? a.g + pix * a.ldg : a.x), 0, has_g ? (int)a.gbytes : 0, 0x00020000);
    xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + pix * a.ldx), 0, (int)a.xbytes, 0x00020000);
    x2r = dual ? __builtin_amdgcn_make_buffer_rsrc((void*)(a.x2 + pix * a.ldx), 0, (int)a.xbytes, 0x00020000) : xr;
    yr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + pix * a.ldy), 0, 0x7fffffff, 0x00020000);
    y2r = __builtin_amdgcn_make_buffer_rsrc((void*)(EPI == 1 ? a.y2 + pix * a.ldy2 : a.y), 0, 0x7fffffff, 0x00020000);
  };

  // resident dgrad weights: packed [CI][Kd], k = tap*CO + ks*32 + c
  for (int c = tid; c < 9 * KSO * CI * 4; c += NT) {
    const int cc = c & 3, row = (c >> 2) % CI, tk = (c >> 2) / CI;   // tk = tap*KSO + ks
    const int tap = tk / KSO, ks = tk - tap * KSO;
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(a.wd + (long)row * a.Kd + tap * CO + ks * 32 + cc * 8);
    *reinterpret_cast<u32x4_t*>(Wimg + (tk * CI + row) * 64 + (swz_nk<32>(row, cc) << 4)) = v;
  }
  const bool xbn = XBN && a.xbn != nullptr;
  if constexpr (BNL) {
    for (int i = tid; i < 3 * CO; i += NT) bnc[i] = a.bncoef[i];
    if constexpr (HBN)       // (the segmap weights in LDS too: registers are the limit of this mode)
      for (int i = tid; i < 3 * CO; i += NT) ybc[i] = i < 2 * CO ? a.ybn[i] : a.hw[i - 2 * CO];
    if (xbn)   // dual input: x's coefficients only, [scale 32 | shift 32] -> xbc[0, 32) and xbc[CI, CI + 32)
      for (int i = tid; i < (dual ? 64 : 2 * CI); i += NT) xbc[dual && i >= 32 ? CI + i - 32 : i] = a.xbn[i];
    __syncthreads();
  }
  // ---- loader constants
  unsigned goff[LG], xoff[LX];
  int gsto[LG], xsto[LX];
  bool gok[LG], xok[LX], xpl[LX];     // xpl: this wave's x chunk j comes from x2 (wave-uniform)
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
  for (int j = 0; j < LG; ++j) {
    const int c = tid + j * NT;
    const int cc = c & 3, px = (c >> 2) % HR, ks = (c >> 2) / HR;
    const int iw = w0 + px - 1;
    gok[j] = c < GCH && iw >= 0 && iw < a.W;
    goff[j] = (unsigned)((iw * a.ldg + ks * 32 + cc * 8) * 2);
    gsto[j] = c < GCH ? (ks * HR + px) * 64 + (swz_nk<32>(px, cc) << 4) : -1;
  }
#pragma unroll
  for (int j = 0; j < LX; ++j) {
    const int c = tid + j * NT;
    int px = c / (CI / 8), cc = c - px * (CI / 8), xc = cc * 8;
    bool live = c < XCH;
    xpl[j] = false;
    if (dual) {
      const int pl = (wid_s * 64 + j * NT) / PLX, cl = c - pl * PLX;
      live = pl < 2 && cl < HR * 4;
      px = cl >> 2, xc = (cl & 3) * 8, cc = pl * 4 + (cl & 3);
      xpl[j] = pl == 1;
    }
    const int iw = w0 + px - 1;
    xok[j] = live && iw >= 0 && iw < a.W;
    xoff[j] = (unsigned)((iw * a.ldx + xc) * 2);
    xsto[j] = live ? px * RBX + ((cc ^ swz_kk<RBX>(px)) << 4) : -1;
  }
  const unsigned growb = (unsigned)(a.W * a.ldg * 2), xrowb = (unsigned)(a.W * a.ldx * 2);
  // ring rows are BP + 2 pixels, so the last register chunk of a row is live in one wave only: the
  // other waves skip its (HEAD/POOL) gradient transform on a wave-uniform branch
  bool glive[LG];
#pragma unroll
  for (int j = 0; j < LG; ++j) glive[j] = wid_s * 64 + j * NT < GCH;
  // W1: one 16-B chunk (8 channels) per ring pixel
  const bool x1ok = W1 && tid < HR && w0 + tid - 1 >= 0 && w0 + tid - 1 < a.W;
  const unsigned x1off = (unsigned)((w0 + tid - 1) * 16), x1rowb = (unsigned)(a.W * 16);
  // HEAD: segmap weights of this thread's 8 channels (cc = tid & 3 for every chunk it loads), the
  // target offset of each chunk's pixel, and whether the pixel is this block's own (not halo)
  float hwv[8], hdw[8], hd0 = 0.f, hd1 = 0.f, hd2 = 0.f, hdb = 0.f;
  // POOL: per chunk the window column's byte offsets into dpool / codes and the pixel's column parity
  unsigned ppo[POOL ? LG : 1], pco[POOL ? LG : 1], pq[POOL ? LG : 1];
  if constexpr (POOL) {
#pragma unroll
    for (int j = 0; j < LG; ++j) {
      const int c = tid + j * NT;
      const int cc = c & 3, px = (c >> 2) % HR, ks = (c >> 2) / HR;
      const int iw = max(w0 + px - 1, 0);
      ppo[j] = (unsigned)(((iw >> 1) * a.ldp + ks * 32 + cc * 8) * 2);
      pco[j] = (unsigned)((iw >> 1) * CO + ks * 32 + cc * 8);
      pq[j] = (unsigned)(iw & 1);
    }
  }
  unsigned tpo[HEAD ? LG : 1];
  bool hval[HEAD ? LG : 1];
  if constexpr (HEAD) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      hwv[e] = HBN ? 0.f : a.hw[(tid & 3) * 8 + e];
      hdw[e] = 0.f;
    }
    hd0 = a.dS[0]; hd1 = a.dS[1]; hd2 = a.dS[2];
#pragma unroll
    for (int j = 0; j < LG; ++j) {
      const int c = tid + j * NT, px = (c >> 2) % HR;
      tpo[j] = (unsigned)(w0 + px - 1) * 4u;
      hval[j] = c < GCH && px >= 1 && px <= BP;
    }
  }
  // two register sets: the loads of a row are issued two rows before it is stored into the ring
  // (one row of compute was too short to cover the load latency at 1-2 blocks per CU)
  struct RowRegs {
    u32x4_t g[LG], x[LX];
    unsigned t[HEAD ? LG : 1];            // HEAD: target bits of each chunk's pixel
    unsigned p[HEAD ? LG : 1];            // HEAD: the forward's probability of each chunk's pixel
    u32x4_t pd[POOL ? LG : 1];            // POOL: the pooled gradient of each chunk's window
    u32x2_t pc[POOL ? LG : 1];            // POOL: the window codes of the chunk's 8 channels
    u32x4_t x1[1];                        // W1: the x1 chunk of this thread's pixel
    u32x4_t z[BNL ? LG : 1];              // BN: the BN input chunk at the gradient chunk's position
  };
  RowRegs setA, setB;
  int n = ig * a.ipb;
  auto rload = [&](int ih, RowRegs& R) {
    const bool rok = ih >= 0 && ih < a.H;                     // wave-uniform
    const unsigned gb = (unsigned)ih * growb, xb = (unsigned)ih * xrowb;
    if constexpr (!HBN) {                      // HEAD + BN: the gradient is formed from z (R.z) alone
#pragma unroll
      for (int j = 0; j < LG; ++j)
        R.g[j] = __builtin_amdgcn_raw_buffer_load_b128(gr, (rok && gok[j]) ? gb + goff[j] : 0x80000000u, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < LX; ++j)
      R.x[j] = __builtin_amdgcn_raw_buffer_load_b128(xpl[j] ? x2r : xr, (rok && xok[j]) ? xb + xoff[j] : 0x80000000u, 0, 0);
    if constexpr (W1) R.x1[0] = __builtin_amdgcn_raw_buffer_load_b128(x1r, (rok && x1ok) ? (unsigned)ih * x1rowb + x1off : 0x80000000u, 0, 0);
    if constexpr (BNL) {
#pragma unroll
      for (int j = 0; j < LG; ++j) R.z[j] = __builtin_amdgcn_raw_buffer_load_b128(zr, (rok && gok[j]) ? gb + goff[j] : 0x80000000u, 0, 0);
    }
    if constexpr (HEAD) {
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        const unsigned o = (rok && gok[j]) ? (unsigned)(ih * a.W) * 4u + tpo[j] : 0x80000000u;
        R.t[j] = __builtin_amdgcn_raw_buffer_load_b32(tr, o, 0, 0);
        R.p[j] = __builtin_amdgcn_raw_buffer_load_b32(hpr, o, 0, 0);
      }
    }
    if constexpr (POOL) {
      const unsigned wrow = (unsigned)(ih >> 1) * (unsigned)(a.W >> 1);
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        const bool ok = rok && gok[j];
        R.pd[j] = __builtin_amdgcn_raw_buffer_load_b128(pr, ok ? (wrow * a.ldp) * 2u + ppo[j] : 0x80000000u, 0, 0);
        R.pc[j] = __builtin_amdgcn_raw_buffer_load_b64(cr, ok ? wrow * CO + pco[j] : 0x80000000u, 0, 0);
      }
    }
  };
  // register transforms of a loaded row (gradient formed on load, BN-on-load of x).  The row loop runs
  // them right after the dx MFMAs, in the same scheduling region, so their VALU work overlaps the
  // MFMAs instead of sitting between the epilogue and the ring store
  auto rxform = [&](RowRegs& R, int ih) {
    if constexpr (POOL) {                       // (dskip, dpool, code) chunk -> gradient chunk
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        if (!glive[j]) continue;
        const unsigned q = (unsigned)((ih & 1) * 2) + pq[j];
        const u32x4_t ps = R.g[j], pd = R.pd[j];
        unsigned o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const unsigned c2 = (k < 2 ? R.pc[j].x : R.pc[j].y) >> (16 * (k & 1));   // codes of channels 2k, 2k+1
          const unsigned cl = c2 & 0xffu, ch = (c2 >> 8) & 0xffu;
          float lo = lo_bf(ps[k]) + ((cl & 3u) == q ? lo_bf(pd[k]) : 0.f);
          float hi = hi_bf(ps[k]) + ((ch & 3u) == q ? hi_bf(pd[k]) : 0.f);
          lo = (cl >> (2 + q)) & 1u ? lo : 0.f;
          hi = (ch >> (2 + q)) & 1u ? hi : 0.f;
          o[k] = pack_bf2(lo, hi);
        }
        R.g[j] = u32x4_t{o[0], o[1], o[2], o[3]};
      }
    }
    if constexpr (HBN) {                        // z chunk -> head gradient of y = relu(bn(z)) (into R.g)
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        if (!glive[j]) continue;
        const int cb = (tid & 3) * 8;
        const float p = __uint_as_float(R.p[j]);
        const float tt = __uint_as_float(R.t[j]);
        const float dz = head_dz(p, tt, tt == 1.f ? 1.f : 0.f, hd0, hd1, hd2);
        unsigned o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 sc = *reinterpret_cast<const float2*>(ybc + cb + 2 * e);
          const float2 sh = *reinterpret_cast<const float2*>(ybc + CO + cb + 2 * e);
          // y as the forward's BN pass would have stored it (bf16); ReLU mask y > 0
          const unsigned yq = pack_bf2(fmaxf(fmaf(lo_bf(R.z[j][e]), sc.x, sh.x), 0.f),
                                       fmaxf(fmaf(hi_bf(R.z[j][e]), sc.y, sh.y), 0.f));
          const float2 hw2 = *reinterpret_cast<const float2*>(ybc + 2 * CO + cb + 2 * e);
          o[e] = pack_bf2(lo_bf(yq) > 0.f ? dz * hw2.x : 0.f, hi_bf(yq) > 0.f ? dz * hw2.y : 0.f);
        }
        R.g[j] = u32x4_t{o[0], o[1], o[2], o[3]};
      }
    }
    if constexpr (BNL) {                        // (g, z) chunk -> conv-output gradient chunk
      const bool rok = ih >= 0 && ih < a.H;
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        if (!glive[j]) continue;
        const int c = tid + j * NT;
        const int cb = ((c >> 2) / HR) * 32 + (c & 3) * 8;       // first channel of the chunk
        const bool ok = rok && gok[j];                            // padding stays zero
        unsigned o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {     // two channels at a time: few coefficient registers live
          const float2 ca = *reinterpret_cast<const float2*>(bnc + cb + 2 * k);
          const float2 cz = *reinterpret_cast<const float2*>(bnc + CO + cb + 2 * k);
          const float2 cc = *reinterpret_cast<const float2*>(bnc + 2 * CO + cb + 2 * k);
          const float lo = fmaf(ca.x, lo_bf(R.g[j][k]), fmaf(cz.x, lo_bf(R.z[j][k]), cc.x));
          const float hi = fmaf(ca.y, hi_bf(R.g[j][k]), fmaf(cz.y, hi_bf(R.z[j][k]), cc.y));
          o[k] = ok ? pack_bf2(lo, hi) : 0u;
        }
        R.g[j] = u32x4_t{o[0], o[1], o[2], o[3]};
      }
    }
    if constexpr (HEAD && !HBN) {               // y chunk -> gradient chunk (+ segmap gradient partials)
      const bool rowv = ih >= h0 && ih < h0 + nrows;
#pragma unroll
      for (int j = 0; j < LG; ++j) {
        if (!glive[j]) continue;
        float yv[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          yv[2 * e] = lo_bf(R.g[j][e]);
          yv[2 * e + 1] = hi_bf(R.g[j][e]);
        }
        const float p = __uint_as_float(R.p[j]);  // the forward's sigmoid(z) (no 32-channel dot here)
        const float tt = __uint_as_float(R.t[j]);
        const float one = tt == 1.f ? 1.f : 0.f;
        const float dz = head_dz(p, tt, one, hd0, hd1, hd2);
        unsigned o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = pack_bf2(yv[2 * e] > 0.f ? dz * hwv[2 * e] : 0.f, yv[2 * e + 1] > 0.f ? dz * hwv[2 * e + 1] : 0.f);
        R.g[j] = u32x4_t{o[0], o[1], o[2], o[3]};
        if (rowv && hval[j]) {
#pragma unroll
          for (int e = 0; e < 8; ++e) hdw[e] = fmaf(dz, yv[e], hdw[e]);
          if ((tid & 3) == 0) hdb += dz;
        }
      }
    }
    if constexpr (XBN) {                        // z chunk -> relu(bn(z)) chunk (padding stays zero)
      const bool rok = ih >= 0 && ih < a.H;
      if (xbn && rok) {
#pragma unroll
        for (int j = 0; j < LX; ++j) {
          if (!xok[j] || (dual && xpl[j])) continue;
          const int cb = dual ? (tid & 3) * 8 : (tid % (CI / 8)) * 8;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float2 sc = *reinterpret_cast<const float2*>(xbc + cb + 2 * k);
            const float2 sh = *reinterpret_cast<const float2*>(xbc + CI + cb + 2 * k);
            R.x[j][k] = pack_bf2(fmaxf(fmaf(lo_bf(R.x[j][k]), sc.x, sh.x), 0.f),
                                 fmaxf(fmaf(hi_bf(R.x[j][k]), sc.y, sh.y), 0.f));
          }
        }
      }
    }
  };
  auto rstore = [&](int slot, RowRegs& R, int ih) {
#pragma unroll
    for (int j = 0; j < LG; ++j)
      if (gsto[j] >= 0) *reinterpret_cast<u32x4_t*>(Gring + slot * GSLOT + gsto[j]) = R.g[j];
#pragma unroll
    for (int j = 0; j < LX; ++j)
      if (xsto[j] >= 0) *reinterpret_cast<u32x4_t*>(Xring + slot * XSLOT + xsto[j]) = R.x[j];
    if constexpr (W1)
      if (tid < HR) *reinterpret_cast<u32x4_t*>(X1ring + ((ih - h0 + 1) % 5) * X1SLOT + tid * 16) = R.x1[0];
  };
  // ---- dx role: LDS fragment offsets, mask offsets, output offsets
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
  int moff[TP][TC];
  unsigned yoff[TP][TC];
  bool hi[TP][TC];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip)
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int px = wp * WP + ip * 16 + (lane & 15);
      const int c0 = wc * WCN + ic * 16 + 4 * chunk;
      moff[ip][ic] = (px + 1) * RBX + (((c0 >> 3) ^ swz_kk<RBX>(px + 1)) << 4) + ((c0 >> 2) & 1) * 8;
      hi[ip][ic] = EPI == 1 && c0 >= a.split;
      // pixels past the row (ragged last strip): offset past the range check, the store is dropped
      yoff[ip][ic] = w0 + px >= a.W ? 0x80000000u
                   : hi[ip][ic] ? (unsigned)(((w0 + px) * a.ldy2 + c0 - a.split) * 2)
                                : (unsigned)(((w0 + px) * a.ldy + c0) * 2);
    }
  const unsigned yrowb = (unsigned)(a.W * a.ldy * 2), y2rowb = (unsigned)(a.W * (EPI == 1 ? a.ldy2 : a.ldy) * 2);
  float bsm[BNS ? TC : 1][4], bsq[BNS ? TC : 1][4];      // BN statistics of the layer below (per lane)
#pragma unroll
  for (int ic = 0; ic < (BNS ? TC : 1); ++ic)
#pragma unroll
    for (int e = 0; e < 4; ++e) bsm[ic][e] = bsq[ic][e] = 0.f;

  // ---- dW role: per-lane byte offsets of the transposed fragments inside a ring slot (row-invariant;
  // computing the swizzled addresses per row cost more VALU issue than the MFMAs they feed)
  int gta[KST][MTW][2], xta[KST][3][2];
  {
    const int g8 = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int j = 0; j < KST; ++j) {
      const int k0 = (pg + j * PG) * 32;
#pragma unroll
      for (int mm = 0; mm < MTW; ++mm) {
        const int m = msp * MTW + mm, col = (m & 1) * 16 + 4 * p, ch = col >> 3, hb = (col & 7) * 2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int rr = 1 + k0 + 8 * g8 + q + 4 * h;
          gta[j][mm][h] = (m >> 1) * HR * 64 + rr * 64 + (swz_nk<32>(rr, ch) << 4) + hb;
        }
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int col = nt * 16 + 4 * p, ch = col >> 3, hb = (col & 7) * 2;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int rr = k0 + kw + 8 * g8 + q + 4 * h;
          xta[j][kw][h] = rr * RBX + ((ch ^ swz_kk<RBX>(rr)) << 4) + hb;
        }
      }
    }
  }
  // ---- dW role accumulators: [tap][co tile] for input-channel tile nt
  f32x4_t accw[9][MTW];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int m = 0; m < MTW; ++m) accw[t][m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum[LBI][8];
#pragma unroll
  for (int i = 0; i < LBI; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[i][e] = 0.f;
  const bool do_bias = a.bslab != nullptr;
  // ---- W1 role: the 10 tiles u = mt1*5 + t1 (co tile mt1, n-tile t1 = taps 2*t1, 2*t1+1) go round-robin
  // over the waves, each over all BP/32 pixel k-steps.  Columns 8..15 of n-tile 4 (a tap 9 that does
  // not exist) are fed ones instead: D[co][8] = sum_px dx[px][co] is conv1's bias gradient.
  constexpr int NTL1 = (10 + NW - 1) / NW, KS1 = BP / 32;
  int g1a[NTL1][2], x1a[NTL1][2], x1kh[NTL1];
  f32x4_t acc1[NTL1];
  if constexpr (W1) {
    const int g8 = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int i = 0; i < NTL1; ++i) {
      const int u = wid + i * NW, mt1 = u / 5, t1 = u - mt1 * 5;
      const int col = mt1 * 16 + 4 * p, ch = col >> 3, hb = (col & 7) * 2;
      const int tap = 2 * t1 + (p >> 1);
      const bool ok = u < 10 && tap < 9;
      const int kh = ok ? tap / 3 : 0, kw = ok ? tap % 3 : 0;
      x1kh[i] = kh;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = 8 * g8 + q + 4 * h;          // + 32 per k-step: same swizzle, +32 rows
        g1a[i][h] = rr * 64 + (swz_nk<32>(rr, ch) << 4) + hb;
        x1a[i][h] = (kw + rr) * 16 + (p & 1) * 8;
      }
      acc1[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }
  // dW1 += dx[h0+r-1]^T x1[h0+r-2+kh] for the dx row stored into G1buf during row step r-1
  auto w1_row = [&](int r) {
    const char* G1 = G1buf + ((r - 1) & 1) * G1SLOT;
#pragma unroll
    for (int i = 0; i < NTL1; ++i) {
      const int u = wid + i * NW;
      if (u >= 10) continue;                                     // wave-uniform
      const char* XS = X1ring + ((r - 1 + x1kh[i]) % 5) * X1SLOT;
      const bool ones = u % 5 == 4 && (lane & 15) >= 8;
#pragma unroll
      for (int k = 0; k < KS1; ++k) {
        const bf16x8_t ga = tr_pair(G1 + k * 32 * 64, g1a[i][0], g1a[i][1]);
        bf16x8_t xb = tr_pair(XS + k * 32 * 16, x1a[i][0], x1a[i][1]);
        if (ones) xb = __builtin_bit_cast(bf16x8_t, u32x4_t{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
        acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, xb, acc1[i], 0, 0, 0);
      }
    }
  };
  int g1o[TP][TC];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip)
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int px = wp * WP + ip * 16 + (lane & 15), c0 = wc * WCN + ic * 16 + 4 * chunk;
      g1o[ip][ic] = px * 64 + (swz_nk<32>(px, c0 >> 3) << 4) + ((c0 >> 2) & 1) * 8;
    }

#pragma unroll 1
  for (int im = 0; im < nimg; ++im, ++n) {
    bind(n);
    if (nrows > 0) {
#pragma unroll 1
      for (int j = 0; j < 3; ++j) {           // rows h0-1, h0, h0+1 -> slots 0..2
        rload(h0 - 1 + j, setA);
        rxform(setA, h0 - 1 + j);
        rstore(j, setA, h0 - 1 + j);
      }
      if (nrows > 1) rload(h0 + 2, setA);      // in flight during row 0
    }
    __syncthreads();
    // row r: `cur` holds row h0+r+2 (issued during row r-1); row h0+r+3 is issued into `nxt`
    auto row = [&](int r, RowRegs& cur, RowRegs& nxt) {
      if (r + 2 < nrows) rload(h0 + r + 3, nxt);
      __builtin_amdgcn_sched_barrier(0);
      const char* Gm = Gring + ((r + 1) & 3) * GSLOT;             // g row h
      const char* Xm = Xring + ((r + 1) & 3) * XSLOT;             // x row h (mask)
      // ---------------- dx row h
      f32x4_t acc[TC][TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* S = Gring + ((r + kh) & 3) * GSLOT;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int ks = 0; ks < KSO; ++ks) {
            const int tk = (kh * 3 + kw) * KSO + ks;
            bf16x8_t af[TC], bfr[TP];
#pragma unroll
            for (int ic = 0; ic < TC; ++ic) af[ic] = *reinterpret_cast<const bf16x8_t*>(Wimg + tk * CI * 64 + aoff[ic]);
#pragma unroll
            for (int ip = 0; ip < TP; ++ip) bfr[ip] = *reinterpret_cast<const bf16x8_t*>(S + ks * HR * 64 + boff[ip][kw]);
#pragma unroll
            for (int ic = 0; ic < TC; ++ic)
#pragma unroll
              for (int ip = 0; ip < TP; ++ip)
                acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
          }
      }
      // BN mode 2 at 64 input channels transforms the row stored below right after the dx MFMAs
      // (overlapping them: 4.63 -> 3.75 ms per 64 -> 64 call at b256); the 32-channel and pool / head
      // modes measured faster with the transform next to the ring store (profiles/*_r04_onload*.txt)
      if constexpr (EARLY_XFORM)
        if (r + 1 < nrows) rxform(cur, h0 + r + 2);
      // ---------------- dW += g[h]^T x[h+kh-1] (this wave: input-channel tile nt, pixel group pg)
#pragma unroll
      for (int j = 0; j < KST; ++j) {
        bf16x8_t ga[MTW];
#pragma unroll
        for (int mm = 0; mm < MTW; ++mm) ga[mm] = tr_pair(Gm, gta[j][mm][0], gta[j][mm][1]);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const char* XS = Xring + ((r + kh) & 3) * XSLOT;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const bf16x8_t xb = tr_pair(XS, xta[j][kw][0], xta[j][kw][1]);
#pragma unroll
            for (int m = 0; m < MTW; ++m)
              accw[kh * 3 + kw][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[m], xb, accw[kh * 3 + kw][m], 0, 0, 0);
          }
        }
      }
      if constexpr (W1)
        if (r > 0) w1_row(r);
      // ---------------- db: sum of the g row's BP pixels (chunk c = (ks*BP + px)*4 + cc; cc = tid & 3)
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < LBI; ++i) {
          const int c = tid + i * NT;
          if (c < BCH) {
            const int cc = c & 3, px = ((c >> 2) % BP) + 1, ks = (c >> 2) / BP;
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>(Gm + ks * HR * 64 + px * 64 + (swz_nk<32>(px, cc) << 4));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bsum[i][2 * e] += lo_bf(v[e]);
              bsum[i][2 * e + 1] += hi_bf(v[e]);
            }
          }
        }
      }
      // ---------------- dx epilogue (mask from the x ring, split store)
      const unsigned orow = (unsigned)(h0 + r);
#pragma unroll
      for (int ip = 0; ip < TP; ++ip)
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          float v0 = acc[ic][ip][0], v1 = acc[ic][ip][1], v2 = acc[ic][ip][2], v3 = acc[ic][ip][3];
          u32x2_t mk = u32x2_t{0u, 0u};
          if constexpr (EPI == 0) {
            mk = *reinterpret_cast<const u32x2_t*>(Xm + moff[ip][ic]);
            v0 = lo_bf(mk.x) > 0.f ? v0 : 0.f;
            v1 = hi_bf(mk.x) > 0.f ? v1 : 0.f;
            v2 = lo_bf(mk.y) > 0.f ? v2 : 0.f;
            v3 = hi_bf(mk.y) > 0.f ? v3 : 0.f;
          }
          const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
          if constexpr (BNS) {     // statistics of the STORED masked dx (out-of-row pixels have x = 0)
            const float q[4] = {lo_bf(packed.x), hi_bf(packed.x), lo_bf(packed.y), hi_bf(packed.y)};
            const float m[4] = {lo_bf(mk.x), hi_bf(mk.x), lo_bf(mk.y), hi_bf(mk.y)};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bsm[ic][e] += q[e];
              bsq[ic][e] = fmaf(q[e], m[e], bsq[ic][e]);
            }
          }
          if constexpr (W1)                      // dx row -> LDS only (bf16, as it would be stored)
            *reinterpret_cast<u32x2_t*>(G1buf + (r & 1) * G1SLOT + g1o[ip][ic]) = packed;
          else if (EPI == 1 && hi[ip][ic])
            __builtin_amdgcn_raw_buffer_store_b64(packed, y2r, orow * y2rowb + yoff[ip][ic], 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b64(packed, yr, orow * yrowb + yoff[ip][ic], 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
      if (r + 1 < nrows) {
        if constexpr (!EARLY_XFORM) rxform(cur, h0 + r + 2);
        rstore((r + 3) & 3, cur, h0 + r + 2);
      }
      __syncthreads();
    };
#pragma unroll 1
    for (int r = 0; r < nrows; r += 2) {
      row(r, setA, setB);
      if (r + 1 < nrows) row(r + 1, setB, setA);
    }
    if constexpr (W1) {                          // the last dx row of this image
      if (nrows > 0) w1_row(nrows);
      __syncthreads();
    }
  }
  if constexpr (BNS) {
    // lanes l, l^1 .. l^15 hold the same channels (different pixels): butterfly over the 16, then the
    // WPX pixel waves in a fixed order -> one deterministic bnslab row per block
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);                 // [WPX][2][CI] (the rings are free)
#pragma unroll
    for (int ic = 0; ic < TC; ++ic)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sm = bsm[ic][e], sq = bsq[ic][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          sm += __shfl_xor(sm, o, 64);
          sq += __shfl_xor(sq, o, 64);
        }
        if ((lane & 15) == 0) {
          const int c = wc * WCN + ic * 16 + 4 * chunk + e;
          red[(wp * 2) * CI + c] = sm;
          red[(wp * 2 + 1) * CI + c] = sq;
        }
      }
    __syncthreads();
    for (int k = tid; k < 2 * CI; k += NT) {
      float t = 0.f;
      for (int w = 0; w < WPX; ++w) t += red[w * 2 * CI + k];
      a.bnslab[(long)split_id * 2 * CI + k] = t;
    }
    __syncthreads();
  }
  // ---------------- partial weight gradient of this (block, pixel group): slab row blockIdx*PG + pg
  const long srow = (long)split_id * PG + pg;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const int ci = nt * 16 + (lane & 15);
      const int co = (msp * MTW + m) * 16 + 4 * (lane >> 4);
      float* dst = a.slab + ((srow * 9 + t) * CO + co) * CI + ci;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[(long)e * CI] = accw[t][m][e];
    }
  if (do_bias) {
    // deterministic: partials by chunk index in LDS, then per channel a fixed-order sum
    float* part = reinterpret_cast<float*>(lds);               // BCH*8 floats (rings are free now)
    static_assert(BCH * 8 * 4 <= WBYTES + 4 * GSLOT + 4 * XSLOT, "bias scratch");
#pragma unroll
    for (int i = 0; i < LBI; ++i) {
      const int c = tid + i * NT;
      if (c < BCH)
#pragma unroll
        for (int e = 0; e < 8; ++e) part[c * 8 + e] = bsum[i][e];
    }
    __syncthreads();
    for (int co = tid; co < CO * PG; co += NT) {
      const int q = co / CO, cch = co - q * CO;                  // q > 0: zero rows of the other groups
      float s = 0.f;
      if (q == 0) {
        const int ks = cch >> 5, cc = (cch & 31) >> 3, e = cch & 7;
        for (int px = 0; px < BP; ++px) s += part[((ks * BP + px) * 4 + cc) * 8 + e];
      }
      a.bslab[((long)split_id * PG + q) * CO + cch] = s;
    }
  }
  if constexpr (HEAD && !HBN) {
    // segmap gradient partials: per thread 8 channels (cc = tid & 3) + dz sum; fixed-order reduction
    __syncthreads();
    float* hp = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int e = 0; e < 8; ++e) hp[tid * 9 + e] = hdw[e];
    hp[tid * 9 + 8] = hdb;
    __syncthreads();
    if (tid < 33) {
      float sacc = 0.f;
      if (tid < 32) {
        const int cc = tid >> 3, e = tid & 7;
        for (int t2 = cc; t2 < NT; t2 += 4) sacc += hp[t2 * 9 + e];
      } else {
        for (int t2 = 0; t2 < NT; t2 += 4) sacc += hp[t2 * 9 + 8];
      }
      a.hslab[(long)split_id * 33 + tid] = sacc;
    }
  }
  if constexpr (W1) {
    // dW1 partials -> slab1 row split_id: D element (co = mt1*16 + 4*(lane>>4) + e, n = lane&15) of
    // n-tile t1 is (tap 2*t1 + n/8, ci n%8); n-tile 4, n == 8 is the bias partial
    const int n1 = lane & 15;
#pragma unroll
    for (int i = 0; i < NTL1; ++i) {
      const int u = wid + i * NW, mt1 = u / 5, t1 = u - mt1 * 5, tap = 2 * t1 + (n1 >> 3);
      const int co = mt1 * 16 + 4 * (lane >> 4);
      if (u < 10 && tap < 9) {
        float* dst = a.slab1 + (((long)split_id * 9 + tap) * 32 + co) * 8 + (n1 & 7);
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e * 8] = acc1[i][e];
      } else if (u < 10 && n1 == 8) {
#pragma unroll
        for (int e = 0; e < 4; ++e) a.bslab1[(long)split_id * 32 + co + e] = acc1[i][e];
      }
    }
  }
}

template <int BP, int CI, int CO, int NW, int PG, int EPI, bool HEAD = false, bool POOL = false, bool W1 = false, int BNM = 0>
static int launch_bwd_stream(const BwdArgs& a, hipStream_t st) {
  const int blocks = ((a.N + a.ipb - 1) / a.ipb) * ((a.H + a.rh - 1) / a.rh) * ((a.W + BP - 1) / BP);
  hipLaunchKernelGGL((bwd_stream_kernel<BP, CI, CO, NW, PG, EPI, HEAD, POOL, W1, BNM>), dim3(blocks), dim3(64 * NW), 0, st, a);
  return (int)hipGetLastError();
}

// Tile (BP pixels x NW waves) per channel pair; pixel groups per block (slab rows per block).
static int bwd_cfg(int ci, int co, int* bp, int* nw) {
  if (ci == 32 && co == 32) { *bp = 64; *nw = 4; return 2; }
  if (ci == 64 && co == 32) { *bp = 64; *nw = 8; return 2; }
  if (ci == 32 && co == 64) { *bp = 64; *nw = 8; return 2; }
  if (ci == 64 && co == 64) { *bp = 64; *nw = 8; return 1; }
  return 0;
}

// Slab rows per block for (ci, co) (0: not supported) and the pixel strip width.
DPA_API int dpa_bwd_stream_pool_ok(int ci, int co) { return ci == 32 && co == 32; }

DPA_API int dpa_bwd_stream_geom(int ci, int co, int* bp) {
  int nw = 0;
  return bwd_cfg(ci, co, bp, &nw);
}

// W1 runs 8 waves (one block per CU, 198 VGPRs): at 4 waves the extra accumulators spill 208 B/lane.
// Measured at batch 256, 512^2: 6.05 ms vs 4.08 ms (pool-mode kernel) + 1.2 ms (separate conv1
// weight gradient) -- the 8-wave row step reads ~60% more LDS per pixel row -- so the engine keeps
// the separate path unless DPA_FUSED_W1=1.
#ifndef W1_NW
#define W1_NW 8
#endif
// epi: 0 dx masked by x > 0, 1 dx split at `split` into y / y2, 2 dx plain.
DPA_API int dpa_bwd_stream(const BwdArgs* args, int ci, int co, int epi, hipStream_t st) {
  const BwdArgs& a = *args;
  int bp = 0, nw = 0;
  // a ragged last strip (W % bp != 0) is masked in the plain / split / masked modes; the fused pool,
  // head and first-conv modes need whole strips
  const bool fused_mode = a.pcode != nullptr || a.hslab != nullptr || a.x1 != nullptr;
  if (!bwd_cfg(ci, co, &bp, &nw) || (fused_mode && a.W % bp) || a.W < 16 || (a.ldg & 7) || (a.ldx & 7) || (a.ldy & 3) ||
      a.rh < 1 || a.ipb < 1 ||
      a.Kd < 9 * co || (epi == 1 && (a.y2 == nullptr || (a.ldy2 & 3) || a.split % 16 || a.split <= 0 || a.split >= ci)) ||
      (a.x2 && (ci != 64 || a.ldx < 32 || fused_mode)) || (a.xbn && (a.z == nullptr || (a.bnslab == nullptr && a.x2 == nullptr))))
    return (int)hipErrorInvalidValue;
  // BN modes: the gradient source is plain (no pool / head / first-conv fold); statistics for the
  // layer below only with the masked dx
  const bool bn = a.z != nullptr;
  if (bn && (a.bncoef == nullptr || fused_mode || (a.bnslab != nullptr && epi != 0))) return (int)hipErrorInvalidValue;
  if (!bn && a.bnslab != nullptr) return (int)hipErrorInvalidValue;
#define DPA_BWD(CIv, COv, BPv, NWv, PGv)                                                              \
  if (ci == CIv && co == COv) {                                                                        \
    if (bn && a.bnslab) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 0, false, false, false, 2>(a, st); \
    if (bn && epi == 1) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 1, false, false, false, 1>(a, st); \
    if (bn && epi == 2) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 2, false, false, false, 1>(a, st); \
    if (bn) return (int)hipErrorInvalidValue;                                                          \
    if (epi == 0) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 0>(a, st);                         \
    if (epi == 1) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 1>(a, st);                         \
    if (epi == 2) return launch_bwd_stream<BPv, CIv, COv, NWv, PGv, 2>(a, st);                         \
  }
  if (a.pcode != nullptr) {    // fused max-pool backward: the full-resolution encoder conv2 (32 -> 32)
    // (the 64 -> 64 instantiation spilled 104 B/lane at two waves per SIMD: kept on pool_bwd_code)
    if (a.dpool == nullptr || (a.H & 1) || (a.ldp & 7) || epi != 0 || a.hslab != nullptr) return (int)hipErrorInvalidValue;
    if (ci != 32 || co != 32) return (int)hipErrorInvalidValue;
    if (a.x1 != nullptr) {     // + the first conv's weight gradient from the unstored input gradient
      if (a.slab1 == nullptr || a.bslab1 == nullptr) return (int)hipErrorInvalidValue;
      return launch_bwd_stream<64, 32, 32, W1_NW, 2, 0, false, true, true>(a, st);
    }
    return launch_bwd_stream<64, 32, 32, 4, 2, 0, false, true>(a, st);
  }
  if (a.ybn != nullptr) {     // head + BN: the last decoder conv 32 -> 32 of a BN model (its BN statistics
    // and the segmap gradients from the head statistics pass; the layer below's BN sums from dx)
    if (ci == 32 && co == 32 && epi == 0 && bn && a.bnslab && a.tgt && a.hw && a.hb && a.dS && a.hprob && !a.hslab &&
        !a.pcode && !a.x1 && a.W % 64 == 0)
      return launch_bwd_stream<64, 32, 32, 8, 2, 0, true, false, false, 2>(a, st);
    return (int)hipErrorInvalidValue;
  }
  if (a.hslab != nullptr) {                        // fused head backward: last decoder conv 32 -> 32
    if (ci == 32 && co == 32 && epi == 0 && a.tgt && a.hw && a.hb && a.dS && a.hprob)
      return launch_bwd_stream<64, 32, 32, 4, 2, 0, true>(a, st);
    return (int)hipErrorInvalidValue;
  }
  DPA_BWD(32, 32, 64, 4, 2)
  DPA_BWD(64, 32, 64, 8, 2)
  DPA_BWD(32, 64, 64, 8, 2)
  DPA_BWD(64, 64, 64, 8, 1)
#undef DPA_BWD
  return (int)hipErrorInvalidValue;
}
