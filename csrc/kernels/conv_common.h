// Shared device helpers for the NHWC bf16 implicit-GEMM conv kernels (gfx950).
//
// MFMA operand maps used throughout (wave64, cdna_hip_programming.md §3):
//   v_mfma_f32_16x16x16_bf16 : lane l supplies A[m=l&15][k=4(l>>4)+j] and
//                              B[k=4(l>>4)+j][n=l&15], j=0..3 (4 bf16 each)
//   v_mfma_f32_16x16x32_bf16 : same with k=8(l>>4)+j, j=0..7 (8 bf16 each)
//   D (both)                 : lane l holds D[m=4(l>>4)+i][n=l&15], i=0..3
// Forward / dgrad compute D^T = W^T X^T so that n = pixel and each lane ends
// up with 4 consecutive output channels of one pixel (one 8-byte NHWC store,
// 4 lanes cover a 32-byte pixel, 16 pixels per wave-instruction).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {
namespace conv {

typedef unsigned short bf16_t;
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// Two floats -> packed bf16 pair (lo in bits 0-15): ONE v_cvt_pk_bf16_f32
// (RNE).  Packing two f2bf results by hand costs two converts plus
// and/shift/or, the compiler does not merge them.
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{lo, hi}, bf2v));
}
// Same instruction as an opaque asm statement: used where the vector-convert
// form changes the compiler's unrolling of the surrounding tile loops (the
// residual-operand register arrays of res_conv_fwd/bwd then went to scratch).
__device__ __forceinline__ uint32_t pack_bf16x2_asm(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
// ReLU on two packed bf16 (sign bit set -> 0).
__device__ __forceinline__ uint32_t relu2(uint32_t v) {
  const uint32_t s = (v >> 15) & 0x00010001u;
  return v & ~(s * 0xFFFFu);
}
__device__ __forceinline__ uint4 relu8(uint4 v) {
  v.x = relu2(v.x); v.y = relu2(v.y); v.z = relu2(v.z); v.w = relu2(v.w);
  return v;
}

__device__ __forceinline__ f4 mfma16(s4 a, s4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma32(bf8 a, bf8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Transposed LDS read (ds_read_b64_tr_b16): per 16-lane group, lane 4q+p
// supplies the address of row q, columns 4p..4p+3 of a 4x16 bf16 block;
// lane i receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ s4 lds_tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)((__attribute__((address_space(3))) char*)(
          (__attribute__((address_space(3))) void*)(p))));
}

// Loads rows [r_begin, r_begin+rows) x cols [-1, W] of image n (NHWC bf16,
// C channels) into LDS as [rows][W+2][C], zero outside the image; optional
// ReLU on load.  16-byte chunks, block-cooperative.
template <int C, bool RELU>
__device__ __forceinline__ void load_halo_tile(
    const bf16_t* __restrict__ src, int n, int H, int W, int r_begin,
    int rows, bf16_t* lds) {
  constexpr int CH = C / 8;
  const int Wp = W + 2;
  const int total = rows * Wp * CH;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int part = e % CH;
    const int pix = e / CH;
    const int rr = pix / Wp;
    const int cc = pix - rr * Wp;
    const int r = r_begin + rr, c = cc - 1;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r >= 0 && r < H && c >= 0 && c < W) {
      v = *reinterpret_cast<const uint4*>(
          src + ((static_cast<int64_t>(n) * H + r) * W + c) * C + part * 8);
      if (RELU) v = relu8(v);
    }
    *reinterpret_cast<uint4*>(lds + pix * C + part * 8) = v;
  }
}

// uint8 frame variant (C=3), byte granularity (the frame rows are 3*W bytes).
__device__ __forceinline__ void load_halo_tile_u8(
    const uint8_t* __restrict__ src, int n, int H, int W, int r_begin,
    int rows, uint8_t* lds) {
  const int Wp = W + 2;
  const int total = rows * Wp * 3;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int ch = e % 3;
    const int pix = e / 3;
    const int rr = pix / Wp;
    const int cc = pix - rr * Wp;
    const int r = r_begin + rr, c = cc - 1;
    uint8_t v = 0;
    if (r >= 0 && r < H && c >= 0 && c < W)
      v = src[((static_cast<int64_t>(n) * H + r) * W + c) * 3 + ch];
    lds[e] = v;
  }
}

// Weights fp32 [3][3][CIN][COUT] (TF HWIO) -> LDS bf16.
//   FWD layout  [tap][COUT][CIN]  (A = W^T: rows co, k = ci)
//   DGRAD layout[tap][CIN][COUT]  (A = W  : rows ci, k = co)
template <int CIN, int COUT, bool FWD>
__device__ __forceinline__ void load_weights(const float* __restrict__ w,
                                             float scale, bf16_t* lds) {
  const int total = 9 * CIN * COUT;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int co = e % COUT;
    const int ci = (e / COUT) % CIN;
    const int tap = e / (COUT * CIN);
    const bf16_t v = f2bf(w[e] * scale);
    if (FWD)
      lds[(tap * COUT + co) * CIN + ci] = v;
    else
      lds[(tap * CIN + ci) * COUT + co] = v;
  }
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

}  // namespace conv
}  // namespace sa
