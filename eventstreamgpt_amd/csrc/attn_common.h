// Device helpers shared by the bf16 MFMA attention backward kernels (attention_bwd.hip: the fused dQ/dK/dV kernel;
// attention_bwd2.hip: the split dK/dV and dQ kernels): MFMA wrapper, fragment conversions, transposed LDS reads,
// the swizzled LDS image layout and the 16-B column stores. v_mfma_f32_32x32x16_bf16 maps: lane l = (r = l&31,
// h = l>>5); A[row r][k = 8h+j], B[k = 8h+j][col r]; C reg i = row (i&3) + 8(i>>2) + 4h, col r.
#pragma once
#include "common.h"

namespace esgpt {
namespace attnb {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));


__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.f;
  return z;
}

__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)p);
}

__device__ __forceinline__ bf16x8 join(bf16x4 lo, bf16x4 hi) {
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// Accumulator registers 8s..8s+7 -> bf16 operand fragment (permuted k order).
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
  return f;
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// Stores the 32 accumulator-row values of one lane's column (x[i] = row acc_row(i, h)) as bf16 into
// dst[0 .. 31] with 16-B stores: register groups g and g+1 are joined across the half-waves with
// v_permlane32_swap (lanes 0-31 end up with rows 8g..8g+7, lanes 32-63 with rows 8g+8..8g+15). N = 16: rows 0..15.
template <int N = 32>
__device__ __forceinline__ void store_col32(__bf16* dst, const f32x16& x, int h) {
#pragma unroll
  for (int g = 0; g < N / 8; g += 2) {
    uint32_t a0 = pack2(x[4 * g], x[4 * g + 1]), a1 = pack2(x[4 * g + 2], x[4 * g + 3]);
    uint32_t b0 = pack2(x[4 * g + 4], x[4 * g + 5]), b1 = pack2(x[4 * g + 6], x[4 * g + 7]);
    const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    *reinterpret_cast<uint4*>(dst + 8 * g + 8 * h) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  }
}

// LDS images with W bf16 columns per row, unpadded, 16-B chunks XOR-swizzled per row so that BOTH access kinds
// are bank-conflict free: 16-B row reads (ds_read_b128: lane r reads row r, one chunk; 16-lane groups
// {0-3,12-15,20-27} / {4-11,16-19,28-31}) and transposed reads (ds_read_b64_tr_b16: a 32-lane half reads 4
// consecutive rows x 32 columns), plus 8-B stores of 16 consecutive rows at one column.
//   W = 32  (64-B rows):  chunk ^ ((row >> 2) & 3)
//   W = 64  (128-B rows): chunk ^ g(row >> 1),  g(m) = ((m & 1) << 2) | ((m >> 1) & 3)
//   W = 128 (256-B rows): chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))
// off(row, col) is an element offset; col % 4 == 0 (8-B accesses stay inside one chunk).
template <int W>
struct Img {
  __device__ __forceinline__ static int off(int row, int col) {
    int sw;
    if (W == 32) sw = (row >> 2) & 3;
    else if (W == 64) sw = (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
    else sw = ((row & 3) << 2) | ((row >> 2) & 3);
    return row * W + (((col >> 3) ^ sw) << 3) + (col & 7);
  }
};

// Workgroup b -> (item, bh) with the (batch, head)s of one XCD kept together and items (chain rank 0 = longest)
// dealt in rank order on every XCD; nbh % 8 == 0 (else the plain round-robin order).
__device__ __forceinline__ void deal(int b, int G, int nbh, int& rank, int& bh) {
  (void)G;
  if ((nbh & 7) == 0) {
    const int x = b & 7, slot = b >> 3, per = nbh >> 3;
    rank = slot / per;
    bh = x + 8 * (slot % per);
  } else {
    rank = b / nbh;
    bh = b % nbh;
  }
}

// Dropout in the backward: none, regenerated from the counter hash, or the forward's keep bits.
enum : int { DROP_NONE = 0, DROP_HASH = 1, DROP_BITS = 2 };

}  // namespace attnb
}  // namespace esgpt
