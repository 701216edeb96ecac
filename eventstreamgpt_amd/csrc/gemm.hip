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
#include <cstdio>
#include <cstdlib>

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

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
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

// XCD-aware tile order: the hardware deals consecutive workgroup ids round-robin over the 8 XCDs (each with its
// own L2), so id -> (xcd = id % 8, slot = id / 8) is remapped (bijectively) to a linear tile index that gives every
// XCD a contiguous run of tiles. The n-tile index runs fastest, so the tiles of one XCD share A row-blocks in L2.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg >> 3, rr = nwg & 7, xcd = id & 7, slot = id >> 3;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
}

// C = alpha · (A·B) (+ bias) for one BMxBN tile over k in [z*kchunk, min(K, (z+1)*kchunk)).
// OUT_F32: C f32 (accumulate: C += …); else bf16. Split-K callers pass C = slab z (ldc = N) and no bias.
// Pipeline: NS register stages (loads for k-tile i+NS-1 are issued before k-tile i is written to LDS) and two LDS
// buffers (one barrier per k-tile: a buffer is rewritten only after every wave passed the next barrier).
// The MFMAs compute the tile transposed (A-operand = B fragment, B-operand = A fragment), so that a lane owns one
// output ROW m and its registers hold columns n = (e&3) + 8(e>>2) + 4h: four consecutive columns per register
// group. The epilogue then stores 16 B per lane (f32: one group; bf16: two groups joined across the half-waves
// with v_permlane32_swap), 8x fewer store instructions than one 2-byte store per element.
template <bool AKC, bool BKC, int WM, int WN, bool OUT_F32>
__global__ __launch_bounds__(THREADS) void gemm_kernel(const __bf16* __restrict__ A, int64_t lda,
                                                       const __bf16* __restrict__ B, int64_t ldb, int M, int N,
                                                       int K, int kchunk, const float* __restrict__ bias,
                                                       const float* __restrict__ alpha, void* __restrict__ Cv,
                                                       int64_t ldc, int64_t slab_stride, int accumulate) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  using TA = Tile<AKC, BM>;
  using TB = Tile<BKC, BN>;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * (TA::kElems + TB::kElems)];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int tn = gridDim.x, tm = gridDim.y;
  const int nwg = tn * tm * gridDim.z;
  const int lin = xcd_remap(blockIdx.x + tn * (blockIdx.y + tm * blockIdx.z), nwg);
  const int bx = lin % tn, by = (lin / tn) % tm, bz = lin / (tn * tm);
  const int m0 = by * BM, n0 = bx * BN;
  const int kb = bz * kchunk, ke = min(K, kb + kchunk);
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
        for (int j = 0; j < WN; ++j) acc[ii][j] = mfma(bfr[j], af[ii], acc[ii][j]);
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

  // Epilogue. Lane: row m0 + wm*32*WM + 32i + r; register group g of tile (i, j): columns
  // n0 + wn*32*WN + 32j + 8g + 4h + {0..3}. N is a multiple of 8 (bf16) / 4 (f32): a group is in or out whole.
  const float al = alpha ? *alpha : 1.f;
  char* Cb = reinterpret_cast<char*>(Cv) + (int64_t)bz * slab_stride * (OUT_F32 ? 4 : 2);
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    const int row = m0 + wm * 32 * WM + 32 * i + r;
    const bool rok = row < M;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int cb = n0 + wn * 32 * WN + 32 * j;
      float v[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb + 8 * g + 4 * h;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bias && c < N) bv = *reinterpret_cast<const float4*>(bias + c);
        v[4 * g + 0] = acc[i][j][4 * g + 0] * al + bv.x;
        v[4 * g + 1] = acc[i][j][4 * g + 1] * al + bv.y;
        v[4 * g + 2] = acc[i][j][4 * g + 2] * al + bv.z;
        v[4 * g + 3] = acc[i][j][4 * g + 3] * al + bv.w;
      }
      if (OUT_F32) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = cb + 8 * g + 4 * h;
          if (!rok || c >= N) continue;
          float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(Cb) + (int64_t)row * ldc + c);
          float4 w = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
          if (accumulate) {
            const float4 o = *p;
            w.x += o.x; w.y += o.y; w.z += o.z; w.w += o.w;
          }
          *p = w;
        }
      } else {
        uint32_t d[4][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          d[g][0] = pack_bf16x2(v[4 * g], v[4 * g + 1]);
          d[g][1] = pack_bf16x2(v[4 * g + 2], v[4 * g + 3]);
        }
#pragma unroll
        for (int g = 0; g < 4; g += 2) {
          // lanes 0-31: columns 8g..8g+7 (own group g | upper half's group g);
          // lanes 32-63: columns 8g+8..8g+15 (lower half's group g+1 | own group g+1)
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const auto sw = __builtin_amdgcn_permlane32_swap(d[g][w], d[g + 1][w], false, false);
            d[g][w] = sw[0];
            d[g + 1][w] = sw[1];
          }
          const int c = cb + 8 * g + 8 * h;
          if (rok && c < N)
            *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(Cb) + (int64_t)row * ldc + c) =
                make_uint4(d[g][0], d[g][1], d[g + 1][0], d[g + 1][1]);
        }
      }
    }
  }
}

// out[m, n] (=, or += when accumulate) sum_z slab[z, m, n] + bias[n]; fixed summation order; 4 columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                            const float* __restrict__ bias, void* __restrict__ C,
                                                            int64_t ldc, int out_bf16, int accumulate) {
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= (int64_t)M * N) return;
  const int64_t row = i4 / N, col = i4 % N;
  float4 s = bias ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < splits; ++z) {
    const float4 x = *reinterpret_cast<const float4*>(slab + (int64_t)z * M * N + i4);
    s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
  }
  if (out_bf16) {
    *reinterpret_cast<uint2*>(reinterpret_cast<__bf16*>(C) + row * ldc + col) =
        make_uint2(pack_bf16x2(s.x, s.y), pack_bf16x2(s.z, s.w));
  } else {
    float4* c = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + row * ldc + col);
    if (accumulate) {
      const float4 o = *c;
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    *c = s;
  }
}

struct Plan {
  int wm, wn, splits, kchunk;
};

Plan plan(int64_t M, int64_t N, int64_t K) {
  constexpr int64_t kTarget = 240;  // workgroups wanted (256 CUs, one resident tile each is already MFMA-bound)
  Plan p{2, 2, 1, (int)(cdiv(K, BK) * BK)};
  if (K == 0) return p;
  if (const char* e = getenv("ESGPT_GEMM_PLAN")) {  // tuning hook: "wm,wn,splits"
    int wm = 2, wn = 2, sp = 1;
    if (sscanf(e, "%d,%d,%d", &wm, &wn, &sp) == 3 && wm >= 1 && wm <= 2 && wn >= 1 && wn <= 2 && sp >= 1) {
      p.wm = wm;
      p.wn = wn;
      const int64_t kchunk = cdiv(cdiv(K, sp), BK) * BK;
      p.splits = (int)cdiv(K, kchunk);
      p.kchunk = (int)kchunk;
      return p;
    }
  }
  // Measured on MI355X at the C2 step's shapes (tools/gemm_sweep.py): 64x64 tiles beat 128x64 / 128x128 for the
  // short-K (256, 1024) projections — more resident workgroups per CU hide the load/store latency that dominates
  // at these sizes. Long-K (dW, K = tokens) products with few tiles split K to about two workgroups per CU.
  p.wm = p.wn = 1;
  const int64_t tiles = cdiv(M, 64) * cdiv(N, 64);
  if (tiles >= kTarget) return p;
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(2 * kTarget / tiles, K / 512));
  const int64_t kchunk = cdiv(cdiv(K, splits), BK) * BK;
  p.splits = (int)cdiv(K, kchunk);
  p.kchunk = (int)kchunk;
  return p;
}

template <bool AKC, bool BKC, bool F32>
void launch(const Plan& p, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M, int N, int K,
            const float* bias, const float* alpha, void* C, int64_t ldc, int64_t slab_stride, int accumulate,
            hipStream_t st) {
  const int BM = 64 * p.wm, BN = 64 * p.wn;
  dim3 grid((unsigned)cdiv(N, BN), (unsigned)cdiv(M, BM), (unsigned)p.splits);
  if (p.wm == 2 && p.wn == 2)
    gemm_kernel<AKC, BKC, 2, 2, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, alpha, C,
                                                                ldc, slab_stride, accumulate);
  else if (p.wm == 2)
    gemm_kernel<AKC, BKC, 2, 1, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, alpha, C,
                                                                ldc, slab_stride, accumulate);
  else
    gemm_kernel<AKC, BKC, 1, 1, F32><<<grid, THREADS, 0, st>>>(A, lda, B, ldb, M, N, K, p.kchunk, bias, alpha, C,
                                                                ldc, slab_stride, accumulate);
}

template <bool F32>
void launch_any(bool akc, bool bkc, const Plan& p, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M,
                int N, int K, const float* bias, const float* alpha, void* C, int64_t ldc, int64_t slab_stride,
                int accumulate, hipStream_t st) {
  if (akc && bkc) launch<true, true, F32>(p, A, lda, B, ldb, M, N, K, bias, alpha, C, ldc, slab_stride, accumulate, st);
  else if (akc) launch<true, false, F32>(p, A, lda, B, ldb, M, N, K, bias, alpha, C, ldc, slab_stride, accumulate, st);
  else if (bkc) launch<false, true, F32>(p, A, lda, B, ldb, M, N, K, bias, alpha, C, ldc, slab_stride, accumulate, st);
  else launch<false, false, F32>(p, A, lda, B, ldb, M, N, K, bias, alpha, C, ldc, slab_stride, accumulate, st);
}

}  // namespace

extern "C" {

size_t esgpt_gemm_workspace(int64_t M, int64_t N, int64_t K) {
  const Plan p = plan(M, N, K);
  return p.splits > 1 ? sizeof(float) * (size_t)p.splits * M * N : 0;
}

int esgpt_gemm_bf16(int a_layout, const void* A, int64_t lda, int b_layout, const void* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, const float* alpha, void* C, int64_t ldc, int c_dtype,
                    int accumulate, void* workspace, size_t workspace_bytes, void* stream) {
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
  // 16-B epilogue stores: whole 8-column (bf16) / 4-column (f32) groups, 16-B aligned rows.
  const int cgrp = c_dtype == ESGPT_F32 ? 4 : 8;
  ESGPT_REQUIRE(N % cgrp == 0 && ldc % cgrp == 0 && ((uintptr_t)C % 16) == 0);
  ESGPT_REQUIRE(bias == nullptr || ((uintptr_t)bias % 16) == 0);
  if (M == 0 || N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const Plan p = plan(M, N, K);  // K == 0: one split, the k-loop is empty and C = bias (or C += bias)
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* b = reinterpret_cast<const __bf16*>(B);
  const bool f32 = c_dtype == ESGPT_F32;
  if (p.splits > 1) {
    ESGPT_REQUIRE(workspace && workspace_bytes >= sizeof(float) * (size_t)p.splits * M * N);
    float* slab = reinterpret_cast<float*>(workspace);
    launch_any<true>(akc, bkc, p, a, lda, b, ldb, M, N, K, nullptr, alpha, slab, N, M * N, 0, st);
    splitk_reduce_kernel<<<(unsigned)cdiv(M * N / 4, 256), 256, 0, st>>>(slab, p.splits, (int)M, (int)N, bias, C, ldc,
                                                                      f32 ? 0 : 1, accumulate);
  } else if (f32) {
    launch_any<true>(akc, bkc, p, a, lda, b, ldb, M, N, K, bias, alpha, C, ldc, 0, accumulate, st);
  } else {
    launch_any<false>(akc, bkc, p, a, lda, b, ldb, M, N, K, bias, alpha, C, ldc, 0, 0, st);
  }
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
