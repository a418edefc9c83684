// Fused forward of the first encoder level's DoubleConv + max-pool (reference model/unet_parts.py:9-14
// and :26-30 at 512^2: conv3x3(3->32)+ReLU, conv3x3(32->32)+ReLU, 2x2 max-pool).
//
// Run as two streaming kernels (igemm_stream8 then igemm_stream with the pool epilogue), the 32-channel
// intermediate a1 is written to HBM by the first and read back by the second: at 512^2 that re-read
// is a quarter of the level's forward traffic.  Here one block streams the image rows of a column
// strip once and keeps a1 in an LDS row ring:
//   iteration t (a1 row k = h0-1+t, output row h = k-2):
//     conv1: a1 row k from the x8 row ring (3 k-steps of 4 taps x 8 channels, as igemm_stream8) ->
//            bf16 into a1-ring slot t&3 (+ the strip's two halo pixels) and, for the block's own rows,
//            to HBM (the backward needs a1);
//     conv2: output row h from a1 rows h-1..h+1 (ring slots (t-3..t-1)&3, written in earlier
//            iterations) -> bias, ReLU, skip store, 2x2 max-pool + window codes (igemm_stream EPI 1);
//   one barrier per iteration; x8 rows are prefetched two rows ahead through two register sets.
// a1 rows / pixels outside the image are stored as zeros (conv2's zero padding), not relu(bias).
// Same MFMA sequences and bf16 roundings as the two-kernel path, so the outputs are bitwise equal
// (tests/test_dconv_fwd.py).  Measured: no faster than the two kernels at batch 256 (4.18 ms vs
// 1.40 + 2.73 ms; tools/ab_dconv.sh) -- like them it is bound by per-row latency (one barrier per row,
// 2-3 waves per SIMD), not by the HBM bytes the fusion removes -- so it is opt-in (DPA_FUSED_DCONV1=1).
#include "conv_args.h"

struct DconvArgs {
  const bf16_t* x;        // [N][H][W][8] (3 real channels)
  const bf16_t* w1;       // packed [32][kp1] (k = tap*8 + ci; taps 9..11 zero)
  const float* b1;
  const bf16_t* w2;       // packed [32][kp2] (k = tap*32 + ci)
  const float* b2;
  bf16_t* a1;             // [N][H][W][32]   conv1 output (for the backward)
  bf16_t* y;              // [N][H][W][ldy]  conv2 output (the skip: concat-buffer half)
  bf16_t* pool;           // [N][H/2][W/2][ldp]
  unsigned char* pcode;   // [N][H/2][W/2][32] window codes, or null
  int N, H, W, ldy, ldp, kp1, kp2, rh;
};

template <int BP>
__global__ __launch_bounds__(256) void dconv1_fwd_kernel(DconvArgs a) {
  constexpr int NG = 32, WP = BP / 4, TP = WP / 16, TC = 2;
  constexpr int HX = BP + 4;                 // x8 ring pixels: w0-2 .. w0+BP+1
  constexpr int HA = BP + 2;                 // a1 ring pixels: w0-1 .. w0+BP
  constexpr int XSLOT = HX * 16, ASLOT = HA * 64;
  __shared__ __attribute__((aligned(16))) char lds[3 * NG * 64 + 9 * NG * 64 + 4 * XSLOT + 4 * ASLOT];
  char* const W1img = lds;
  char* const W2img = lds + 3 * NG * 64;
  char* const Xring = W2img + 9 * NG * 64;
  char* const Aring = Xring + 4 * XSLOT;

  const int stripsW = a.W / BP, segsH = (a.H + a.rh - 1) / a.rh;
  const int bid = blockIdx.x;
  const int n = bid / (segsH * stripsW);
  const int rem = bid - n * segsH * stripsW;
  const int hs = rem / stripsW;
  const int w0 = (rem - hs * stripsW) * BP, h0 = hs * a.rh;
  const int nrows = min(a.rh, a.H - h0);
  const int tid = threadIdx.x, lane = tid & 63, wp = tid >> 6, chunk = lane >> 4;
  const long pix = (long)n * a.H * a.W;       // per-image buffer bases: 32-bit offsets at any batch
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + pix * 8), 0, a.H * a.W * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)(a.a1 + pix * 32), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + pix * a.ldy), 0, 0x7fffffff, 0x00020000);
  const long ppix = (long)n * (a.H >> 1) * (a.W >> 1);
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.pool + ppix * a.ldp), 0, 0x7fffffff, 0x00020000);

  // resident weights: conv1 [kstep][co][64 B], conv2 [tap][co][64 B] (swz_nk<32>)
  for (int c = tid; c < 3 * NG * 4; c += 256) {
    const int cc = c & 3, row = (c >> 2) % NG, s = (c >> 2) / NG;
    const u32x4_t v = (s * 32 + cc * 8 < a.kp1) ? *reinterpret_cast<const u32x4_t*>(a.w1 + (long)row * a.kp1 + s * 32 + cc * 8)
                                                : u32x4_t{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4_t*>(W1img + (s * NG + row) * 64 + (swz_nk<32>(row, cc) << 4)) = v;
  }
  for (int c = tid; c < 9 * NG * 4; c += 256) {
    const int cc = c & 3, row = (c >> 2) % NG, tap = (c >> 2) / NG;
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(a.w2 + (long)row * a.kp2 + tap * 32 + cc * 8);
    *reinterpret_cast<u32x4_t*>(W2img + (tap * NG + row) * 64 + (swz_nk<32>(row, cc) << 4)) = v;
  }
  // ---- x8 loader: thread tid < HX owns ring pixel tid (image column w0-2+tid)
  const int iwx = w0 - 2 + tid;
  const bool xok = tid < HX && iwx >= 0 && iwx < a.W;
  const unsigned xoff = (unsigned)iwx * 16u, xrowb = (unsigned)a.W * 16u;
  auto rload = [&](int ih, u32x4_t& R) {
    const bool ok = xok && ih >= 0 && ih < a.H;
    R = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (unsigned)ih * xrowb + xoff : 0x80000000u, 0, 0);
  };
  auto rstore = [&](int slot, const u32x4_t& R) {
    if (tid < HX) *reinterpret_cast<u32x4_t*>(Xring + slot * XSLOT + tid * 16) = R;
  };
  // ---- conv1 fragments (as igemm_stream8): lane group `chunk` = the tap of each 4-tap k-step
  int a1off[TC];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic) {
    const int row = ic * 16 + (lane & 15);
    a1off[ic] = row * 64 + (swz_nk<32>(row, chunk) << 4);
  }
  float bias1[TC][4], bias2[TC][4];
#pragma unroll
  for (int ic = 0; ic < TC; ++ic)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bias1[ic][e] = a.b1[ic * 16 + 4 * chunk + e];
      bias2[ic][e] = a.b2[ic * 16 + 4 * chunk + e];
    }
  // the strip's two a1 halo pixels (ring index 0 and HA-1) are one extra 16-lane tile computed by
  // wave 0: lane p16 = 0 -> pixel w0-1, every other lane -> pixel w0+BP (duplicates, stored once)
  const int p16 = lane & 15;
  const int hq = p16 == 0 ? -1 : BP;                         // strip coordinate of the halo pixel
  const bool hq_in = (w0 + hq) >= 0 && (w0 + hq) < a.W;
  // ---- conv2 fragments (as igemm_stream over the a1 ring) and epilogue constants
  int boff[TP][3];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int px = wp * WP + ip * 16 + p16 + kw;
      boff[ip][kw] = px * 64 + (swz_nk<32>(px, chunk) << 4);
    }
  // a1 ring store offsets of this lane's 4 channels (c0 = ic*16 + 4*chunk) at ring pixel p+1
  int ast[TP][TC], hst[TC];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip)
#pragma unroll
    for (int ic = 0; ic < TC; ++ic) {
      const int q = wp * WP + ip * 16 + p16 + 1, c0 = ic * 16 + 4 * chunk;
      ast[ip][ic] = q * 64 + (swz_nk<32>(q, c0 >> 3) << 4) + ((c0 >> 2) & 1) * 8;
    }
#pragma unroll
  for (int ic = 0; ic < TC; ++ic) {
    const int q = hq + 1, c0 = ic * 16 + 4 * chunk;
    hst[ic] = q * 64 + (swz_nk<32>(q, c0 >> 3) << 4) + ((c0 >> 2) & 1) * 8;
  }
  unsigned al[TP], yl[TP];
#pragma unroll
  for (int ip = 0; ip < TP; ++ip) {
    const int pl = w0 + wp * WP + ip * 16 + p16;
    al[ip] = (unsigned)((pl * 32 + 4 * chunk) * 2);
    yl[ip] = (unsigned)((pl * a.ldy + 4 * chunk) * 2);
  }
  float ptop[TP][TC][4], ptop2[TP][TC][4];

  u32x4_t xa, xb;                              // x8 prefetch registers (two rows ahead)
  // prologue: x rows h0-2 .. h0 -> slots 0..2, row h0+1 in flight
#pragma unroll 1
  for (int j = 0; j < 3; ++j) {
    rload(h0 - 2 + j, xa);
    rstore(j, xa);
  }
  rload(h0 + 1, xb);
  __syncthreads();

  // iteration t: `cur` holds x row h0+t+1 (loaded during t-1), x row h0+t+2 is loaded into `nxt`
  auto step = [&](int t, u32x4_t& cur, u32x4_t& nxt) {
    const int k = h0 - 1 + t;                  // a1 row produced now
    const bool c1 = t <= nrows + 1;            // a1 rows h0-1 .. h0+nrows
    if (t + 1 <= nrows + 1) rload(h0 + t + 2, nxt);
    __builtin_amdgcn_sched_barrier(0);
    // ---------------- conv1 -> a1 row k
    if (c1) {
      char* As = Aring + (t & 3) * ASLOT;
      if (k >= 0 && k < a.H) {
        f32x4_t acc[TC][TP], hacc[TC];
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          hacc[ic] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tap = 4 * s + chunk;
          const int kh = tap / 3, kw = tap - kh * 3;
          const bool real = tap < 9;
          bf16x8_t af[TC], bfr[TP];
#pragma unroll
          for (int ic = 0; ic < TC; ++ic) af[ic] = *reinterpret_cast<const bf16x8_t*>(W1img + s * NG * 64 + a1off[ic]);
          const char* S = Xring + ((t + (real ? kh : 0)) & 3) * XSLOT;   // x row k-1+kh
#pragma unroll
          for (int ip = 0; ip < TP; ++ip) {
            const int px = wp * WP + ip * 16 + p16 + 1 + (real ? kw : 0);  // ring index of pixel p-1+kw
            bfr[ip] = *reinterpret_cast<const bf16x8_t*>(S + px * 16);
          }
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
          if (wp == 0) {
            const bf16x8_t hb = *reinterpret_cast<const bf16x8_t*>(S + (hq + 1 + (real ? kw : 0)) * 16);
#pragma unroll
            for (int ic = 0; ic < TC; ++ic) hacc[ic] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], hb, hacc[ic], 0, 0, 0);
          }
        }
        const bool own = k >= h0 && k < h0 + nrows;
        const unsigned abase = (unsigned)k * (unsigned)(a.W * 64);
#pragma unroll
        for (int ip = 0; ip < TP; ++ip)
#pragma unroll
          for (int ic = 0; ic < TC; ++ic) {
            const float v0 = fmaxf(acc[ic][ip][0] + bias1[ic][0], 0.f), v1 = fmaxf(acc[ic][ip][1] + bias1[ic][1], 0.f);
            const float v2 = fmaxf(acc[ic][ip][2] + bias1[ic][2], 0.f), v3 = fmaxf(acc[ic][ip][3] + bias1[ic][3], 0.f);
            const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
            *reinterpret_cast<u32x2_t*>(As + ast[ip][ic]) = packed;
            if (own) __builtin_amdgcn_raw_buffer_store_b64(packed, ar, abase + al[ip] + ic * 32, 0, 0);
          }
        if (wp == 0 && p16 < 2) {
#pragma unroll
          for (int ic = 0; ic < TC; ++ic) {
            u32x2_t packed = u32x2_t{0u, 0u};
            if (hq_in) {
              const float v0 = fmaxf(hacc[ic][0] + bias1[ic][0], 0.f), v1 = fmaxf(hacc[ic][1] + bias1[ic][1], 0.f);
              const float v2 = fmaxf(hacc[ic][2] + bias1[ic][2], 0.f), v3 = fmaxf(hacc[ic][3] + bias1[ic][3], 0.f);
              packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
            }
            *reinterpret_cast<u32x2_t*>(As + hst[ic]) = packed;
          }
        }
      } else {                                 // padding row of conv2's input: zeros
        for (int c = tid; c < HA * 4; c += 256) *reinterpret_cast<u32x4_t*>(As + c * 16) = u32x4_t{0u, 0u, 0u, 0u};
      }
    }
    // ---------------- conv2 -> output row h = k - 2 from a1 rows h-1 .. h+1
    if (t >= 3) {
      const int r = t - 3, h = h0 + r;
      f32x4_t acc[TC][TP];
#pragma unroll
      for (int ic = 0; ic < TC; ++ic)
#pragma unroll
        for (int ip = 0; ip < TP; ++ip) acc[ic][ip] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* S = Aring + ((t - 3 + kh) & 3) * ASLOT;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int tk = kh * 3 + kw;
          bf16x8_t af[TC], bfr[TP];
#pragma unroll
          for (int ic = 0; ic < TC; ++ic) af[ic] = *reinterpret_cast<const bf16x8_t*>(W2img + tk * NG * 64 + a1off[ic]);
#pragma unroll
          for (int ip = 0; ip < TP; ++ip) bfr[ip] = *reinterpret_cast<const bf16x8_t*>(S + boff[ip][kw]);
#pragma unroll
          for (int ic = 0; ic < TC; ++ic)
#pragma unroll
            for (int ip = 0; ip < TP; ++ip)
              acc[ic][ip] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ic], bfr[ip], acc[ic][ip], 0, 0, 0);
        }
      }
      const unsigned ybase = (unsigned)h * (unsigned)(a.W * a.ldy * 2);
#pragma unroll
      for (int ip = 0; ip < TP; ++ip)
#pragma unroll
        for (int ic = 0; ic < TC; ++ic) {
          const float v0 = fmaxf(acc[ic][ip][0] + bias2[ic][0], 0.f), v1 = fmaxf(acc[ic][ip][1] + bias2[ic][1], 0.f);
          const float v2 = fmaxf(acc[ic][ip][2] + bias2[ic][2], 0.f), v3 = fmaxf(acc[ic][ip][3] + bias2[ic][3], 0.f);
          const u32x2_t packed = u32x2_t{pack_bf2(v0, v1), pack_bf2(v2, v3)};
          __builtin_amdgcn_raw_buffer_store_b64(packed, yr, ybase + yl[ip] + ic * 32, 0, 0);
          // 2x2 max-pool of the STORED values (igemm_stream EPI 1)
          float q[4] = {lo_bf(packed.x), hi_bf(packed.x), lo_bf(packed.y), hi_bf(packed.y)};
          float pq[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) pq[e] = __shfl_xor(q[e], 1, 64);
          if ((h & 1) == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              ptop[ip][ic][e] = q[e];
              ptop2[ip][ic][e] = pq[e];
            }
          } else if (h < 2 * (a.H >> 1) && (lane & 1) == 0) {
            const int pw = (w0 + wp * WP + ip * 16 + p16) >> 1;
            const unsigned pidx = (unsigned)((h >> 1) * (a.W >> 1) + pw);
            float mx[4];
            unsigned code = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              mx[e] = fmaxf(fmaxf(q[e], pq[e]), fmaxf(ptop[ip][ic][e], ptop2[ip][ic][e]));
              code |= pool_code(ptop[ip][ic][e], ptop2[ip][ic][e], q[e], pq[e]) << (8 * e);
            }
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack_bf2(mx[0], mx[1]), pack_bf2(mx[2], mx[3])}, pr,
                                                  (pidx * a.ldp + ic * 16 + 4 * chunk) * 2, 0, 0);
            if (a.pcode)
              *reinterpret_cast<unsigned*>(a.pcode + (ppix + pidx) * 32 + ic * 16 + 4 * chunk) = code;
          }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t <= nrows) rstore((t + 3) & 3, cur);   // x row h0+t+1: read by conv1 from iteration t+1 on
    __syncthreads();
  };
  const int T = nrows + 3;
#pragma unroll 1
  for (int t = 0; t < T; t += 2) {
    step(t, xb, xa);
    if (t + 1 < T) step(t + 1, xa, xb);
  }
}

// Rows per block: whole image columns when the batch alone fills the chip, else row segments
// (2 halo rows of conv1 recomputed per segment).  rh must be even (pool windows stay in a block).
// bp: 0 auto (64-pixel strips: 45 KB of LDS and fewer registers -> more waves per CU), 64 or 128
DPA_API int dpa_dconv1_fwd(const DconvArgs* args, int bp, hipStream_t st) {
  const DconvArgs& a = *args;
  const int BP = bp == 128 ? 128 : 64;
  if (a.W % BP || (a.H & 1) || (a.rh & 1) || a.rh < 2 || (a.ldy & 3) || (a.ldp & 3) || a.kp1 < 72 || a.kp2 < 288 ||
      a.x == nullptr || a.a1 == nullptr || a.y == nullptr || a.pool == nullptr || (long)a.H * a.W * 64 > 0x7fffffffL)
    return (int)hipErrorInvalidValue;
  const int blocks = a.N * ((a.H + a.rh - 1) / a.rh) * (a.W / BP);
  if (BP == 128) hipLaunchKernelGGL(dconv1_fwd_kernel<128>, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dconv1_fwd_kernel<64>, dim3(blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
