// Argument blocks and LDS helpers shared by the convolution kernels (igemm.hip, wgrad.hip, halo.hip).
#pragma once
#include "common.h"

struct IgemmArgs {
  const bf16_t* x;      // source activations [N][Hs][Ws][ldx] (channel offset folded into the pointer)
  const bf16_t* w;      // packed weights [Ngemm][Kpad] bf16
  const float* bias;    // [Cout] fp32 or null
  bf16_t* y;            // output (channel offset folded into the pointer)
  const bf16_t* mask;   // ReLU-backward mask source (same pixel grid as y, mode 0) or null
  int ldx, ldy, ldm, mask_ch;
  int N, Ho, Wo;        // GEMM-M pixel grid
  int Hs, Ws, Cs;       // source grid and channels gathered per tap (Cs % 8 == 0)
  int KH, KW, stride, pad;
  int Ngemm, Kpad;      // GEMM N, K padded to a multiple of BK (packed weights zero-filled)
  int mode;             // 0: y[m][n]   1: transposed-conv 2x2/s2 scatter, n = (2i+j)*Cout + co
  int relu, accumulate, Cout;
  unsigned xbytes;      // bytes addressable from x (< 2^31; the host splits larger batches by image)
  bf16_t* pool;         // optional fused 2x2/s2 max-pool output [N][Ho/2][Wo/2][ldp] (stream kernels)
  int ldp;
  unsigned char* pcode; // optional with pool: per (window, channel) code = argmax(2b) | (4 pixels > 0) << 2,
                        // dense [N][Ho/2][Wo/2][Ngemm] bytes: the max-pool backward needs nothing else
  bf16_t* y2;           // optional split output (mode 0, no accumulate): channels >= split go to
  int ldy2, split;      // y2[m][co - split] -- the two halves of a concat gradient as dense tensors
  // optional fused segmentation head (streaming kernel, last decoder conv, Ngemm == 32): per pixel
  // z = hb + sum_c y[c] hw[c], p = sigmoid(z), BCE/Dice partial sums vs tgt -> hslab[block][4]
  const float* hw; const float* hb; const float* tgt; float* hslab;
  // optional BatchNorm batch statistics of the stored (bf16) output (streaming kernel, conv followed
  // by BN): per block, per channel sum and sum of squares -> bnslab[block][2][Ngemm] (bn_finalize)
  float* bnslab;
  int korder;           // LDS-DMA kernels: bit 0 = tap-major K-tile order (default slice-major when K is
                        // unpadded), bit 1 = no persistent kernel in the auto choice (A/B switches)
  unsigned ximg;        // bytes addressable from ONE image of x: the row-streaming / row-halo kernels
                        // bind one image per block (64-bit base, 32-bit offsets inside it), so they take
                        // the whole batch in one launch whatever its size (no 2 GiB chunking)
  float* hprob;         // fused head (optional): the per-pixel probability p = sigmoid(z) [N*Ho*Wo] fp32,
                        // kept for the head backward (bwd_stream HEAD mode reads it instead of re-deriving
                        // it from the 32-channel output)
  const bf16_t* x2;     // dual input (row-streaming kernel, Cs == 64 only): channels 32-63 of the conv input
                        // come from this second tensor, laid out like x ([N][Hs][Ws][ldx], same ximg) --
                        // a decoder conv over [skip | up] reads the two dense halves, no concat buffer
  const float* xbn;     // BN-on-load (row-streaming kernel with BN statistics, EPI 4): x holds the layer
                        // below's pre-BatchNorm output z; the loader forms relu(z * xbn[c] + xbn[Cs + c])
};

// 2x2 window code from the four (bf16-rounded) values in window order tl, tr, bl, br: first
// occurrence of the maximum (torch max_pool2d / the old pool_bwd order) and the ReLU masks.
__device__ __forceinline__ unsigned pool_code(float tl, float tr, float bl, float br) {
  const unsigned it = tr > tl ? 1u : 0u, ib = br > bl ? 3u : 2u;
  const float mt = fmaxf(tl, tr), mb = fmaxf(bl, br);
  return (mb > mt ? ib : it) | (unsigned)(tl > 0.f) << 2 | (unsigned)(tr > 0.f) << 3 | (unsigned)(bl > 0.f) << 4 |
         (unsigned)(br > 0.f) << 5;
}

// pool_code of two channels at once from packed non-negative bf16 pairs (window order tl, tr, bl, br):
// the code of the low halves in bits 0-7, of the high halves in bits 8-15
__device__ __forceinline__ unsigned pool_code2(unsigned tl, unsigned tr, unsigned bl, unsigned br) {
  const unsigned mt = pk_max16(tl, tr), mb = pk_max16(bl, br);
  const unsigned it = pk_gt16(tr, tl), ib = pk_gt16(br, bl), sel = pk_gt16(mb, mt);
  const unsigned b0 = (sel & ib) | (~sel & it);                   // argmax bit 0, bit 1 = sel
  // flag bits at 15 / 31 -> code bit k at k / 16 + k, then the high code to bits 8-13
  unsigned x = b0 >> 15;
  x |= sel >> 14;
  x |= pk_nz16(tl) >> 13;
  x |= pk_nz16(tr) >> 12;
  x |= pk_nz16(bl) >> 11;
  x |= pk_nz16(br) >> 10;
  return (x & 0x3fu) | ((x >> 8) & 0x3f00u);
}

// split-output store (see IgemmArgs::y2); returns false when the output is not split
__device__ __forceinline__ bool split_store(const IgemmArgs& a, unsigned m, int co, u32x2_t v) {
  if (a.y2 == nullptr) return false;
  bf16_t* p = co >= a.split ? a.y2 + (size_t)m * a.ldy2 + (co - a.split) : a.y + (size_t)m * a.ldy + co;
  *reinterpret_cast<u32x2_t*>(p) = v;
  return true;
}

struct WgradArgs {
  const bf16_t* A; const bf16_t* B;
  float* slab;          // [splits][T][M][Nc]
  float* bslab;         // [splits][M] or null (bias gradient partials)
  int lda, ldb;
  int N, Hg, Wg;        // pixel grid p = (n, h, w)
  int HA, WA, HB, WB;   // spatial dims of A and B tensors
  int M, Nc;            // channels of A (GEMM rows) and B (GEMM cols, may be < tile width: zero filled)
  int s, pad, KW;       // tap-dependent operand is read at (h*s + kh - pad, w*s + kw - pad)
  int pix_per_split, splits;
  unsigned abytes, bbytes;  // addressable bytes of A / B (< 2^31; the host splits larger batches)
  // optional per-image base pointers (device arrays of N entries): image n of A / B starts at
  // atab[n] / btab[n] instead of A / B + n * image size -- one weight-gradient launch over the images
  // of several tensors of the same per-image layout (the microbatches of a pipeline stage)
  const bf16_t* const* atab; const bf16_t* const* btab;
  // BatchNorm backward on load of A (wgrad_stream, the first conv): A is the ReLU-masked gradient g of a
  // BN output and the GEMM row operand is dz = abn[m] g + abn[M + m] z + abn[2M + m] with z = az (the BN
  // input, A's layout) -- bn_bwd_apply's formula; zero outside the image.  Null: A as is.
  const bf16_t* az; const float* abn;
};

// 16-B LDS-DMA: lane l's bytes land at lds + 16*l.  (Wrapped in a __device__ function: used
// directly inside a kernel template the builtin makes the host pass drop the kernel's launch stub.)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// nk images ([rows][BK] bf16, 16-B chunks): conflict-free ds_read_b128 fragment reads for any
// 16 consecutive rows (tools/lds_banks.py)
template <int BK>
__device__ __forceinline__ int swz_nk(int row, int chunk) {
  if constexpr (BK == 32) return chunk ^ ((row >> 1) & 3);
  else return chunk ^ (row & 7);
}

// kk images ([pixel rows][channels] bf16, RB bytes per row) read with ds_read_b64_tr_b16
template <int RB>
__device__ __forceinline__ int swz_kk(int r) {
  if constexpr (RB == 64) return ((r >> 3) & 1) * 2;
  else if constexpr (RB == 128) return (((r >> 1) & 1) * 2) ^ (((r >> 3) & 1) * 4);
  else if constexpr (RB == 256 || RB == 512) return ((r & 1) * 2) ^ (((r >> 1) & 1) * 4) ^ (((r >> 3) & 1) * 8);
  else return 0;
}

// 8 consecutive k (pixel rows 8g..8g+7 of a [32][RB] image) for the 16 columns starting at col0
template <int RB>
__device__ __forceinline__ bf16x8_t tr_frag(const char* img, int col0, int lane, int roff = 0) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = col0 + 4 * p;
  const int ch = col >> 3, hb = (col & 7) * 2;
  const int r0 = roff + 8 * g + q, r1 = r0 + 4;
  const char* a0 = img + r0 * RB + ((ch ^ swz_kk<RB>(r0)) << 4) + hb;
  const char* a1 = img + r1 * RB + ((ch ^ swz_kk<RB>(r1)) << 4) + hb;
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, a0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, a1));
  typedef __attribute__((ext_vector_type(8))) short s16x8_t;
  s16x8_t v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

