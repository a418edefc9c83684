// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of distributedpytorch_amd.
// Every launcher is extern "C", takes raw device pointers + a hipStream_t, and returns hipError_t.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DPA_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;                                     // raw bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;      // MFMA 16x16x32 A/B fragment
typedef __attribute__((ext_vector_type(4))) short s16x4_t;        // ds_read_b64_tr_b16 result
typedef __attribute__((ext_vector_type(4))) float f32x4_t;        // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16_t;      // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

static __device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}
// round-to-nearest-even f32 -> bf16 (NaN-preserving cast; hipcc lowers to v_cvt_pk_bf16_f32)
static __device__ __forceinline__ unsigned short f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&b);
}
// two f32 -> one bf16 pair, round-to-nearest-even: ONE v_cvt_pk_bf16_f32 (two scalar casts compile to two
// of them plus a v_or_b32_sdwa -- three VALU per pair in every epilogue and loader transform)
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
static __device__ __forceinline__ unsigned int pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(unsigned int, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
static __device__ __forceinline__ float lo_bf(unsigned int u) { return __uint_as_float(u << 16); }
static __device__ __forceinline__ float hi_bf(unsigned int u) { return __uint_as_float(u & 0xffff0000u); }

// Segmentation-head backward per pixel (torch formulas: BCE backward (p - t) / max(p(1-p), 1e-12),
// sigmoid backward g p (1-p)), from the loss's partial-sum gradient dS = (d0, d1, d2):
//   dz = (d0 (p-t) / max(s, 1e-12) + d1 [t==1] + d2) s,   s = p (1-p)
// written without the division: s / max(s, 1e-12) is 1 unless the sigmoid saturated.
static __device__ __forceinline__ float head_dz(float p, float t, float one, float d0, float d1, float d2) {
  const float s = (1.f - p) * p;
  const float rs = s >= 1e-12f ? 1.f : s * 1e12f;
  return d0 * (p - t) * rs + (d1 * one + d2) * s;
}
// ReLU as one integer max on the f32 bits (negative floats are negative ints): no NaN-quieting
// v_max_f32 in front of the v_max_f32 that fmaxf(v, 0) costs on MFMA results
static __device__ __forceinline__ float relu_f(float v) { return __int_as_float(max(__float_as_int(v), 0)); }

// Packed bf16 pairs of NON-NEGATIVE values (post-ReLU) order like unsigned 16-bit integers, so
// 2x2 max-pool windows reduce two channels per instruction (v_pk_max_u16 / v_pk_sub_u16).
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2_t;
static __device__ __forceinline__ unsigned pk_max16(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, a), __builtin_bit_cast(u16x2_t, b)));
}
// bit 15 / 31 set where the half of b exceeds the half of a (halves in [0, 0x7fff])
static __device__ __forceinline__ unsigned pk_gt16(unsigned b, unsigned a) {
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(u16x2_t, a) - __builtin_bit_cast(u16x2_t, b)) & 0x80008000u;
}
// bit 15 / 31 set where the half is non-zero
static __device__ __forceinline__ unsigned pk_nz16(unsigned a) {
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(u16x2_t, a) + u16x2_t{0x7fff, 0x7fff}) & 0x80008000u;
}

// sigmoid with the hardware reciprocal (1 ulp) instead of an IEEE division
static __device__ __forceinline__ float fast_sigmoid(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum for 256-thread blocks; `red` must hold >= 4 floats of LDS. Result valid in all threads.
static __device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// Bijective XCD-aware remap (MI355X: 8 XCDs, hardware deals blocks round-robin): consecutive
// *logical* ids land on the same XCD, so neighbouring tiles share that XCD's L2.
static __device__ __forceinline__ int xcd_remap(int hw, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = hw & 7, slot = hw >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

static inline int dpa_grid(long long n, int block, int cap = 2048) {
  long long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}
