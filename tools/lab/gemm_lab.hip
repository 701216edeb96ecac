// GEMM staging experiments (tools only, never loaded by the product): forward projections C = A·Bᵀ + bias with
// LDS-DMA (buffer_load ... lds) operand staging into XOR-swizzled 128-B-row images, several tile / wave / buffer
// geometries, timed against the product's register-staged gemm_kernel by tools/lab/gemm_lab.py.
#include "../../eventstreamgpt_amd/csrc/common.h"

using namespace esgpt;

namespace lab {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt left at their maxima), n < 64
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define W_(k) case k: __builtin_amdgcn_s_waitcnt(((k) & 15) | (((k) >> 4) << 14) | (7 << 4) | (15 << 8)); break;
    W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
    W_(16) W_(18) W_(20) W_(24) W_(28) W_(32) W_(36) W_(40) W_(48)
#undef W_
    default: __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8)); break;
  }
}

template <int WM, int WN, int FM, int FN, int NB>
__device__ __forceinline__ void gemm_glds_body(const uint16_t* __restrict__ A_, const uint16_t* __restrict__ B_,
                                                          const float* __restrict__ bias, uint16_t* __restrict__ C_,
                                                          int M, int N, int K, int lda, int ldb, int ldc) {
  const __bf16* A = reinterpret_cast<const __bf16*>(A_);
  const __bf16* B = reinterpret_cast<const __bf16*>(B_);
  __bf16* C = reinterpret_cast<__bf16*>(C_);
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;
  constexpr int ROWB = 128;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW, P = PA + PB;
  static_assert(PA * 8 * NW == BM && PB * 8 * NW == BN, "rows per wave");
  constexpr int EPI = BM * (BN + 8) * 2;
  constexpr int LDS = NB * STAGE > EPI ? NB * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const int lin = xcd_linear(blockIdx.x, gridDim.x);
  const int tn = N / BN;
  const int bx = lin % tn, by = lin / tn;
  const int m0 = by * BM, n0 = bx * BN;
  const int nk = K / 64;

  int voA[PA], voB[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = 8 * (wave + NW * i) + (lane >> 3), lg = (lane & 7) ^ ((row >> 1) & 7);
    voA[i] = ((m0 + row) * lda + lg * 8) * 2;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = 8 * (wave + NW * i) + (lane >> 3), lg = (lane & 7) ^ ((row >> 1) & 7);
    voB[i] = ((n0 + row) * ldb + lg * 8) * 2;
  }
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(B), (short)0, 0x7fffffff, 0x00020000);

  auto issue = [&](int kt, int buf) {
    char* sA = smem + buf * STAGE;
    char* sB = sA + BM * ROWB;
    const int so = kt * 128;
#pragma unroll
    for (int i = 0; i < PA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(sA + 8 * (wave + NW * i) * ROWB), 16, voA[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < PB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void*)(sB + 8 * (wave + NW * i) * ROWB), 16, voB[i], so, 0, 0);
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int sw = (r >> 1) & 7;
  auto compute = [&](int buf) {
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + BM * ROWB;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cb = ((2 * t + h) ^ sw) * 16;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * 32 * FM + 32 * i + r) * ROWB + cb);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sB + (wn * 32 * FN + 32 * j + r) * ROWB + cb);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NB - 2, nk - 1 - kt);
    wait_vm(ahead * P);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NB - 1 < nk) issue(kt + NB - 1, (kt + NB - 1) % NB);
    compute(kt % NB);
  }

  // epilogue: bias, bf16, fragment-order LDS writes, row-major 16-B stores
  const int lrow0 = wm * 32 * FM + r;
  const int lcol0 = wn * 32 * FN;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int LDB = BN + 8;
  __bf16* tb = reinterpret_cast<__bf16*>(smem);
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = lcol0 + 32 * j + 8 * g + 4 * h;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (bias) bv = *reinterpret_cast<const float4*>(bias + n0 + c);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const uint2 d = make_uint2(pack2(acc[i][j][4 * g] + bv.x, acc[i][j][4 * g + 1] + bv.y),
                                   pack2(acc[i][j][4 * g + 2] + bv.z, acc[i][j][4 * g + 3] + bv.w));
        *reinterpret_cast<uint2*>(tb + (lrow0 + 32 * i) * LDB + c) = d;
      }
    }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < BM * BN / 8 / NT; ++q) {
    const int ch = threadIdx.x + NT * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
    *reinterpret_cast<uint4*>(C + (int64_t)(m0 + tr) * ldc + n0 + tc) = *reinterpret_cast<const uint4*>(tb + tr * LDB + tc);
  }
}

template <int WM, int WN, int FM, int FN, int NB>
__global__ __launch_bounds__(64 * WM * WN) void gemm_glds(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                          const float* __restrict__ bias, uint16_t* __restrict__ C,
                                                          int M, int N, int K, int lda, int ldb, int ldc) {
  gemm_glds_body<WM, WN, FM, FN, NB>(A, B, bias, C, M, N, K, lda, ldb, ldc);
}

template <int WM, int WN, int FM, int FN, int NB>
int launch(const void* A, const void* B, const float* bias, void* C, int M, int N, int K, hipStream_t st) {
  constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;
  if (M % BM || N % BN || K % 64) return -1;
  gemm_glds<WM, WN, FM, FN, NB><<<dim3((M / BM) * (N / BN)), 64 * WM * WN, 0, st>>>(
      (const uint16_t*)A, (const uint16_t*)B, bias, (uint16_t*)C, M, N, K, K, K, N);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}  // namespace lab
using namespace lab;

extern "C" int lab_fwd(int v, const void* A, const void* B, const float* bias, void* C, int M, int N, int K, void* s) {
  hipStream_t st = (hipStream_t)s;
  switch (v) {
    case 0: return launch<2, 2, 2, 2, 2>(A, B, bias, C, M, N, K, st);  // 128x128, 4 waves, 2 buffers
    case 1: return launch<2, 2, 2, 2, 3>(A, B, bias, C, M, N, K, st);  // 128x128, 3 buffers
    case 2: return launch<2, 2, 2, 2, 4>(A, B, bias, C, M, N, K, st);  // 128x128, 4 buffers
    case 3: return launch<2, 2, 1, 1, 2>(A, B, bias, C, M, N, K, st);  // 64x64, 2 buffers
    case 4: return launch<2, 2, 1, 1, 4>(A, B, bias, C, M, N, K, st);  // 64x64, 4 buffers
    case 5: return launch<2, 2, 2, 1, 3>(A, B, bias, C, M, N, K, st);  // 128x64, 3 buffers
    case 6: return launch<4, 2, 1, 2, 2>(A, B, bias, C, M, N, K, st);  // 128x128, 8 waves (32x64 each)
    case 7: return launch<4, 2, 1, 2, 3>(A, B, bias, C, M, N, K, st);  // 128x128, 8 waves, 3 buffers
    case 8: return launch<4, 2, 2, 2, 2>(A, B, bias, C, M, N, K, st);  // 256x128, 8 waves
    case 9: return launch<2, 2, 2, 1, 2>(A, B, bias, C, M, N, K, st);  // 128x64, 2 buffers
    case 10: return launch<2, 2, 1, 2, 3>(A, B, bias, C, M, N, K, st); // 64x128, 3 buffers
    case 11: return launch<2, 4, 2, 1, 2>(A, B, bias, C, M, N, K, st); // 128x128, 8 waves (64x32 each)
    default: return -3;
  }
}
