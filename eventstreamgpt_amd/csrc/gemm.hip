// bf16 MFMA tile GEMM for the training step's projections (the InnerAttention q/k/v/out projections, the InnerMLP
// c_fc/c_proj and the generative heads: transformer.py:133-163, 378-391; generative_layers.py) on gfx950.
//
//   C[M, N] = A · B (+ bias[n]),   bf16 operands, f32 accumulation, C bf16 or f32.
//
// The step's shapes are skinny: M = B·L tokens (8192 for the C2 workload) with N, K in {256 … 1232}, and the
// weight gradients are [out, in] products with K = tokens. Library kernels pick 64x64 tiles with no K split for
// the latter (64 workgroups on a 256-CU part); here the decomposition is chosen for the chip: 128x128 / 128x64 /
// 64x64 tiles, and split-K into f32 slabs plus a fixed-order reduce (deterministic) when there are too few tiles.
//
// Operand layouts (both supported for either operand, so fwd, dX and dW need no transposed copies):
//   A "K-contig": A[m][k] = a[m*lda + k]   LDS image [rows][BK + 8], fragments by 16-B row reads
//   A "M-contig": A[m][k] = a[k*lda + m]   LDS image [BK][160], fragments by ds_read_b64_tr_b16 (hardware
//                                          transpose; row stride = 16 dwords mod 64 -> conflict-free reads)
//   B likewise with n in place of m ("K-contig": B[k][n] = b[n*ldb + k], "N-contig": B[k][n] = b[k*ldb + n]).
// MFMA v_mfma_f32_32x32x16_bf16; 4 waves as 2x2, each wave (BM/2)x(BN/2); register-staged global->LDS with the
// next k-tile's loads in flight during the current tile's MFMAs.
#include <algorithm>

#include "common.h"

using namespace esgpt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int BK = 64;
constexpr int KC_LD = BK + 8;  // K-contig image row stride (elements)
constexpr int THREADS = 256;
constexpr int NS = 3;          // register stages: NS-1 k-tiles in flight while one is written to LDS

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.f;
  return z;
}

// One operand's tile: R rows (m or n) x BK k. Loads are branch-free (addresses clamped into the operand, the
// out-of-range chunks zeroed when written to LDS) so that the compiler keeps counted vmcnt waits across stages.
template <bool KC, int R>
struct Tile {
  // M/N-contig image row stride: 4 consecutive k-rows must start 16 or 48 dwords apart (mod 64) so that a
  // 32-lane half of a transposed read (4 rows x 32 columns) touches every bank once.
  static constexpr int MN_LD = (R == 64) ? 96 : 160;
  static constexpr int kElems = KC ? R * KC_LD : BK * MN_LD;
  static constexpr int kChunks = R * BK / 8 / THREADS;  // 16-B chunks per thread

  __device__ __forceinline__ static void coords(int i, int& a, int& b) {
    const int c = threadIdx.x + THREADS * i;
    if (KC) {
      a = c >> 3;          // row
      b = (c & 7) * 8;     // k
    } else {
      a = c / (R / 8);     // k-row
      b = (c % (R / 8)) * 8;  // column
    }
  }

  __device__ __forceinline__ static void load(bf16x8 (&reg)[kChunks], const __bf16* __restrict__ g, int64_t ld,
                                              int row0, int rows, int k0, int kend) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      if (KC) {
        const int row = min(row0 + a, rows - 1), k = min(k0 + b, kend - 8);
        reg[i] = *reinterpret_cast<const bf16x8*>(g + (int64_t)row * ld + k);
      } else {
        const int k = min(k0 + a, kend - 1), col = min(row0 + b, rows - 8);
        reg[i] = *reinterpret_cast<const bf16x8*>(g + (int64_t)k * ld + col);
      }
    }
  }

  __device__ __forceinline__ static void store(__bf16* s, const bf16x8 (&reg)[kChunks], int row0, int rows, int k0,
                                               int kend) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      if (KC) {
        const bool ok = row0 + a < rows && k0 + b < kend;
        *reinterpret_cast<bf16x8*>(s + a * KC_LD + b) = ok ? reg[i] : zero8();
      } else {
        const bool ok = k0 + a < kend && row0 + b < rows;
        *reinterpret_cast<bf16x8*>(s + a * MN_LD + b) = ok ? reg[i] : zero8();
      }
    }
  }

  // MFMA operand fragment for rows sub0 .. sub0+31 of the tile and k-step t (k = 16t .. 16t+15):
  // lane (r = l&31, h = l>>5) gets row sub0 + r, k = 16t + 8h + j, j = 0..7.
  __device__ __forceinline__ static bf16x8 frag(const __bf16* s, int sub0, int t) {
    const int l = threadIdx.x & 63;
    if (KC) {
      const int r = l & 31, h = l >> 5;
      return *reinterpret_cast<const bf16x8*>(s + (sub0 + r) * KC_LD + 16 * t + 8 * h);
    } else {
      // ds_read_b64_tr_b16: in each 16-lane group, lane 4q+p addresses k-row (base + q), columns 4p .. 4p+3;
      // lane i of the group receives column i of the 4 rows.
      const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
      const int col = sub0 + (g & 1) * 16 + 4 * p;
      const int kr = 16 * t + 8 * (g >> 1) + q;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s + kr * MN_LD + col));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s + (kr + 4) * MN_LD + col));
      bf16x8 f;
      f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
      f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
      return f;
    }
  }
};

// C = A·B (+ bias) for one BMxBN tile over k in [z*kchunk, min(K, (z+1)*kchunk)).
// OUT_F32: C f32 (accumulate: C += …); else bf16. Split-K callers pass C = slab z (ldc = N) and no bias.
// Pipeline: NS register stages (loads for k-tile i+NS-1 are issued before k-tile i is written to LDS) and two LDS
// buffers (one barrier per k-tile: a buffer is rewritten only after every wave passed the next barrier).
template <bool AKC, bool BKC, int WM, int WN, bool OUT_F32>
__global__ __launch_bounds__(THREADS) void gemm_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                       const __bf16* __restrict__ B, int64_t ldb, int M, int N,
                                                       int K, int kchunk, const float* __restrict__ bias,
                                                       void* __restrict__ Cv, int64_t ldc, int64_t slab_stride,
                                                       int accumulate) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  using TA = Tile<AKC, BM>;
  using TB = Tile<BKC, BN>;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * (TA::kElems + TB::kElems)];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  bf16x8 ra[NS][TA::kChunks], rb[NS][TB::kChunks];
  // Consumes k-tile `i` from register stage `st`: write to LDS buffer i&1, one barrier, MFMAs.
  auto consume = [&](int st, int i) {
    __bf16* sA = smem + (i & 1) * (TA::kElems + TB::kElems);
    __bf16* sB = sA + TA::kElems;
    TA::store(sA, ra[st], m0, M, kb + i * BK, ke);
    TB::store(sB, rb[st], n0, N, kb + i * BK, ke);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < BK / 16; ++t) {
      bf16x8 af[WM], bfr[WN];
#pragma unroll
      for (int ii = 0; ii < WM; ++ii) af[ii] = TA::frag(sA, wm * 32 * WM + 32 * ii, t);
#pragma unroll
      for (int j = 0; j < WN; ++j) bfr[j] = TB::frag(sB, wn * 32 * WN + 32 * j, t);
#pragma unroll
      for (int ii = 0; ii < WM; ++ii)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[ii][j] = mfma(af[ii], bfr[j], acc[ii][j]);
    }
  };
  // Loads are unconditional (clamped addresses; tiles past the end are zeroed at the LDS write), so the stage
  // registers are never merged across branches and the compiler keeps the vmcnt waits counted.
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) {
    TA::load(ra[st], A, lda, m0, M, kb + st * BK, ke);
    TB::load(rb[st], B, ldb, n0, N, kb + st * BK, ke);
  }
  int i0 = 0;
  for (; i0 + NS <= nk; i0 += NS) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      TA::load(ra[(st + NS - 1) % NS], A, lda, m0, M, kb + (i0 + st + NS - 1) * BK, ke);
      TB::load(rb[(st + NS - 1) % NS], B, ldb, n0, N, kb + (i0 + st + NS - 1) * BK, ke);
      consume(st, i0 + st);
    }
  }
  // tail: fewer than NS k-tiles left, already resident in stages 0 .. nk-i0-1
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (i0 + st < nk) consume(st, i0 + st);

  // Epilogue: register e of tile (i, j) holds row (e&3) + 8(e>>2) + 4h, column r.
  char* Cb = reinterpret_cast<char*>(Cv) + (int64_t)blockIdx.z * slab_stride * (OUT_F32 ? 4 : 2);
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int col = n0 + wn * 32 * WN + 32 * j + r;
    const bool cok = col < N;
    const float bc = (bias && cok) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * 32 * WM + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (!cok || row >= M) continue;
        const float v = acc[i][j][e] + bc;
        if (OUT_F32) {
          float* c = reinterpret_cast<float*>(Cb) + (int64_t)row * ldc + col;
          *c = accumulate ? *c + v : v;
        } else {
          reinterpret_cast<__bf16*>(Cb)[(int64_t)row * ldc + col] = (__bf16)v;
        }
      }
  }
}

// out[m, n] (=, or += when accumulate) sum_z slab[z, m, n] + bias[n]; fixed summation order.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                            const float* __restrict__ bias, void* __restrict__ C,
                                                            int64_t ldc, int out_bf16, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int64_t row = i / N, col = i % N;
  float s = bias ? bias[col] : 0.f;
  for (int z = 0; z < splits; ++z) s += slab[(int64_t)z * M * N + i];
  if (out_bf16) {
    reinterpret_cast<__bf16*>(C)[row * ldc + col] = (__bf16)s;
  } else {
    float* c = reinterpret_cast<float*>(C) + row * ldc + col;
    *c = accumulate ? *c + s : s;
  }
}

struct Plan {
  int wm, wn, splits, kchunk;
};

Plan plan(int64_t M, int64_t N, int64_t K) {
  constexpr int64_t kTarget = 240;  // workgroups wanted (256 CUs, one resident tile each is already MFMA-bound)
  Plan p{2, 2, 1, (int)(cdiv(K, BK) * BK)};
  if (K == 0) return p;
  if (cdiv(M, 128) * cdiv(N, 128) >= kTarget) return p;
  if (cdiv(M, 128) * cdiv(N, 64) >= kTarget) {
    p.wn = 1;
    return p;
  }
  p.wm = p.wn = 1;
  const int64_t tiles = cdiv(M, 64) * cdiv(N, 64);
  if (tiles >= kTarget) return p;
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(kTarget / tiles, K / 256));
  const int64_t kchunk = cdiv(cdiv(K, splits), BK) * BK;
  p.splits = (int)cdiv(K, kchunk);
  p.kchunk = (int)kchunk;
  return p;
}

template <bool AKC, bool BKC, bool F32>
void launch(const Plan& p, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M, int N, int K,
            const float* bias, void* C, int64_t ldc, int64_t slab_stride, int accumulate, hipStream_t st) {
  const int BM = 64 * p.wm, BN = 64 * p.wn;
  dim3 grid((unsigned)cdiv(N, BN), (unsigned)cdiv(M, BM), (unsigned)p.splits);
  if (p.wm == 2 && p.wn == 2)
    gemm_kernel<AKC, BKC, 2, 2, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, C, ldc,
                                                                slab_stride, accumulate);
  else if (p.wm == 2)
    gemm_kernel<AKC, BKC, 2, 1, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, C, ldc,
                                                                slab_stride, accumulate);
  else
    gemm_kernel<AKC, BKC, 1, 1, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, C, ldc,
                                                                slab_stride, accumulate);
}

template <bool F32>
void launch_any(bool akc, bool bkc, const Plan& p, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M,
                int N, int K, const float* bias, void* C, int64_t ldc, int64_t slab_stride, int accumulate,
                hipStream_t st) {
  if (akc && bkc) launch<true, true, F32>(p, A, lda, B, ldb, M, N, K, bias, C, ldc, slab_stride, accumulate, st);
  else if (akc) launch<true, false, F32>(p, A, lda, B, ldb, M, N, K, bias, C, ldc, slab_stride, accumulate, st);
  else if (bkc) launch<false, true, F32>(p, A, lda, B, ldb, M, N, K, bias, C, ldc, slab_stride, accumulate, st);
  else launch<false, false, F32>(p, A, lda, B, ldb, M, N, K, bias, C, ldc, slab_stride, accumulate, st);
}

}  // namespace

extern "C" {

size_t esgpt_gemm_workspace(int64_t M, int64_t N, int64_t K) {
  const Plan p = plan(M, N, K);
  return p.splits > 1 ? sizeof(float) * (size_t)p.splits * M * N : 0;
}

int esgpt_gemm_bf16(int a_layout, const void* A, int64_t lda, int b_layout, const void* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, void* C, int64_t ldc, int c_dtype, int accumulate,
                    void* workspace, size_t workspace_bytes, void* stream) {
  ESGPT_REQUIRE(A && B && C && M >= 0 && N >= 0 && K >= 0);
  ESGPT_REQUIRE(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31));
  ESGPT_REQUIRE(c_dtype == ESGPT_F32 || (c_dtype == ESGPT_BF16 && !accumulate));
  const bool akc = a_layout == ESGPT_GEMM_K_CONTIG, bkc = b_layout == ESGPT_GEMM_K_CONTIG;
  ESGPT_REQUIRE(akc || a_layout == ESGPT_GEMM_MN_CONTIG);
  ESGPT_REQUIRE(bkc || b_layout == ESGPT_GEMM_MN_CONTIG);
  // 16-B vector loads: the contiguous extent and every row start must be 8-element aligned.
  ESGPT_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0);
  ESGPT_REQUIRE((akc || M % 8 == 0) && (bkc || N % 8 == 0));
  ESGPT_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0);
  if (M == 0 || N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const Plan p = plan(M, N, K);  // K == 0: one split, the k-loop is empty and C = bias (or C += bias)
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* b = reinterpret_cast<const __bf16*>(B);
  const bool f32 = c_dtype == ESGPT_F32;
  if (p.splits > 1) {
    ESGPT_REQUIRE(workspace && workspace_bytes >= sizeof(float) * (size_t)p.splits * M * N);
    float* slab = reinterpret_cast<float*>(workspace);
    launch_any<true>(akc, bkc, p, a, lda, b, ldb, M, N, K, nullptr, slab, N, M * N, 0, st);
    splitk_reduce_kernel<<<(unsigned)cdiv(M * N, 256), 256, 0, st>>>(slab, p.splits, (int)M, (int)N, bias, C, ldc,
                                                                      f32 ? 0 : 1, accumulate);
  } else if (f32) {
    launch_any<true>(akc, bkc, p, a, lda, b, ldb, M, N, K, bias, C, ldc, 0, accumulate, st);
  } else {
    launch_any<false>(akc, bkc, p, a, lda, b, ldb, M, N, K, bias, C, ldc, 0, 0, st);
  }
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
