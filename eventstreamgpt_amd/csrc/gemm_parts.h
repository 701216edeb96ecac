// Device-side pieces shared by the projection GEMM kernels (gemm.hip: tile GEMM, grouped backward, slab reduce;
// tools/lab/gemm_stream.hip: the streamed-tile persistent GEMM, tools build): bf16 / f32 operand tiles, LDS-DMA tiles, the problem
// descriptor and small helpers. Included by those two translation units only.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace esgpt {
namespace gk {

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
      a = c >> 3;             // row
      b = (c & 7) * 8;        // k
    } else {
      a = c / (R / 8);        // k-row
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

  // Fast path (whole tiles, operand < 2 GiB): per-lane byte offsets within a k-tile computed once; each k-tile
  // is one uniform (SGPR) offset on buffer loads — no per-chunk address math, clamps or zero selects.
  __device__ __forceinline__ static void lane_offsets(int (&vo)[kChunks], int64_t ld, int row0) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      vo[i] = KC ? (int)(((int64_t)(row0 + a) * ld + b) * 2) : (int)(((int64_t)a * ld + row0 + b) * 2);
    }
  }
  __device__ __forceinline__ static int k_offset(int k0, int64_t ld) { return KC ? k0 * 2 : (int)(k0 * ld * 2); }
  __device__ __forceinline__ static void load_fast(bf16x8 (&reg)[kChunks], __amdgpu_buffer_rsrc_t rs,
                                                   const int (&vo)[kChunks], int so) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i)
      reg[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vo[i], so, 0));
  }
  __device__ __forceinline__ static void store_fast(__bf16* s, const bf16x8 (&reg)[kChunks]) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      *reinterpret_cast<bf16x8*>(s + a * (KC ? KC_LD : MN_LD) + b) = reg[i];
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

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left at their maxima), N < 64
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// LDS-DMA operand staging of whole tiles (buffer_load … lds): one 1-KiB wave-instruction writes its 64 lanes' 16-B
// pieces lane-linearly into LDS, so the images carry no padding; their 16-B chunks are XOR-swizzled per image row to
// keep the fragment reads bank-conflict free, the swizzle applied to each lane's SOURCE address (the destination
// stays linear: cdna_hip_programming.md rule 21). No VGPR round trip, no ds_write pass, no per-chunk address math in
// the k-loop (one uniform soffset per k-tile).
//   K-contig image  [R rows][64 k] (128-B rows):     chunk ^ ((row >> 1) & 7)   — ds_read_b128 fragments: each
//                                                    16-lane group reads 16 distinct rows ≡ (row & 15) → 16 bank quads
//   M/N-contig image [64 k-rows][R columns]:  R = 64:  chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))
//                                             R = 128: chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))
//                                            — ds_read_b64_tr_b16 fragments: a 32-lane half reads 4 consecutive
//                                              k-rows x 32 columns, spread over all 64 banks
template <bool KC, int R>
struct GTile {
  static constexpr int kElems = R * BK;                 // bf16 elements of one k-tile image
  static constexpr int CPR = KC ? BK / 8 : R / 8;       // 16-B chunks per image row
  static constexpr int RPI = 64 / CPR;                  // image rows per 1-KiB instruction
  static constexpr int kInstr = kElems * 2 / 1024 / 4;  // instructions per wave and k-tile (4 waves)
  static_assert(kInstr >= 1 && kInstr * 4 * 512 == kElems, "tile rows");

  __device__ __forceinline__ static int sw(int row) {
    if (KC) return (row >> 1) & 7;
    if (R == 64) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
    return ((row & 3) << 2) | ((row >> 2) & 3);
  }
  __device__ __forceinline__ static int off(int row, int col) {  // element offset, col % 4 == 0
    return row * (KC ? BK : R) + (((col >> 3) ^ sw(row)) << 3) + (col & 7);
  }
  // Out-of-range pieces (rows / columns past the operand's m or n extent, k past the split's end) read zeros: their
  // voffset is set beyond the buffer's num_records (buffer loads return 0 out of range), so edge tiles take the same
  // loop — no register-staged fallback, no clamps. Every piece is a whole 16-B chunk (K, and M / N of an M/N-contig
  // operand, are multiples of 8).
  static constexpr int kOOB = (int)0x80000000u;
  __device__ __forceinline__ static void coords(int i, int& row, int& lg) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    row = (wave + 4 * i) * RPI + lane / CPR;
    lg = (lane % CPR) ^ sw(row);
  }
  // per-lane source byte offsets of this wave's instructions (row0 = the tile's first m / n, nrows its extent)
  __device__ __forceinline__ static void lane_src(int (&vo)[kInstr], int64_t ld, int row0, int nrows) {
#pragma unroll
    for (int i = 0; i < kInstr; ++i) {
      int row, lg;
      coords(i, row, lg);
      if (KC) vo[i] = row0 + row < nrows ? (int)(((int64_t)(row0 + row) * ld + lg * 8) * 2) : kOOB;
      else vo[i] = row0 + lg * 8 < nrows ? (int)(((int64_t)row * ld + row0 + lg * 8) * 2) : kOOB;
    }
  }
  __device__ __forceinline__ static int k_soff(int k0, int64_t ld) { return KC ? k0 * 2 : (int)(k0 * ld * 2); }
  // one k-tile into `img`; kvalid < BK: the split's last, partial k-tile (its pieces past kvalid read zeros)
  __device__ __forceinline__ static void issue(__amdgpu_buffer_rsrc_t rs, const int (&vo)[kInstr], int so,
                                               __bf16* img, int kvalid) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kInstr; ++i) {
      int v = vo[i];
      if (kvalid < BK) {
        int row, lg;
        coords(i, row, lg);
        if ((KC ? lg * 8 : row) >= kvalid) v = kOOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wave + 4 * i) * 512), 16, v, so, 0, 0);
    }
  }
  // the same fragment as Tile<KC, R>::frag, from the swizzled image. The transposed reads are inline asm: hipcc
  // (ROCm 7.2) cannot tell the ds_read_tr16_b64 builtin apart from the LDS-DMA writes in flight and drains every
  // one of them (vmcnt(0)) before it, which serialises the k-loop; the asm form is ordered by the loop's own counted
  // vmcnt + barrier, and its results are waited for explicitly (frag_wait) before the MFMAs read them.
  __device__ __forceinline__ static bf16x8 frag(const __bf16* s, int sub0, int t) {
    const int l = threadIdx.x & 63;
    if (KC) {
      const int r = l & 31, h = l >> 5;
      return *reinterpret_cast<const bf16x8*>(s + off(sub0 + r, 16 * t + 8 * h));
    } else {
      const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
      const int col = sub0 + (g & 1) * 16 + 4 * p;
      const int kr = 16 * t + 8 * (g >> 1) + q;
      bf16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"((uint32_t)(uintptr_t)(lds_bf16x4*)(s + off(kr, col)))
                   : "memory");
      asm volatile("ds_read_b64_tr_b16 %0, %1"
                   : "=v"(hi) : "v"((uint32_t)(uintptr_t)(lds_bf16x4*)(s + off(kr + 4, col))) : "memory");
      bf16x8 f;
      f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
      f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
      return f;
    }
  }
};

// Waits for the inline-asm fragment reads (the compiler does not count them) before their registers are used; the
// sched_barrier keeps hipcc from hoisting an MFMA above the wait (cdna_hip_programming.md rule 18).
__device__ __forceinline__ void frag_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ---- f32 operands (the reference-precision step: scripts/pretrain.py trains in f32) ----
// v_mfma_f32_32x32x2_f32: lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]; the product is exact f32
// (bitwise a k-ordered fmaf chain, one rounding per product: cdna_hip_programming.md §3), at the f32 vector rate.
// k-stage BKF = 32; each image row holds its k in the order (0, 2, …, 30, 1, 3, …, 31), so a lane half h (k ≡ h mod 2)
// reads its next four k-steps as one 16-B read. Register-staged (the images are permuted / transposed on the LDS
// write); loads branch-free with clamped addresses, out-of-range chunks zeroed on the LDS write.
constexpr int BKF = 32;
constexpr int FLD = BKF + 4;  // image row pitch (floats): the 16-lane groups of a 16-B fragment read hit 16 bank quads
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool KC, int R>
struct FTile {
  static constexpr int kFloats = R * FLD;
  static constexpr int kChunks = R * BKF / 4 / THREADS;  // 16-B chunks per thread and k-stage
  static_assert(kChunks >= 1 && kChunks * 4 * THREADS == R * BKF, "f32 tile rows");
  __device__ __forceinline__ static int pos(int k) { return (k & 1) * (BKF / 2) + (k >> 1); }
  __device__ __forceinline__ static void coords(int i, int& a, int& b) {
    const int c = threadIdx.x + THREADS * i;
    if (KC) {
      a = c / (BKF / 4);       // row
      b = (c % (BKF / 4)) * 4;  // k
    } else {
      a = c % BKF;             // k-row (consecutive lanes walk k: the transposing LDS writes are conflict-free)
      b = (c / BKF) * 4;       // column
    }
  }
  __device__ __forceinline__ static void load(float4 (&reg)[kChunks], const float* __restrict__ g, int64_t ld,
                                              int row0, int rows, int k0, int kend) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      if (KC) {
        const int row = min(row0 + a, rows - 1), k = min(k0 + b, kend - 4);
        reg[i] = *reinterpret_cast<const float4*>(g + (int64_t)row * ld + k);
      } else {
        const int k = min(k0 + a, kend - 1), col = min(row0 + b, rows - 4);
        reg[i] = *reinterpret_cast<const float4*>(g + (int64_t)k * ld + col);
      }
    }
  }
  __device__ __forceinline__ static void store(float* s, const float4 (&reg)[kChunks], int row0, int rows, int k0,
                                               int kend) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      int a, b;
      coords(i, a, b);
      float4 v = reg[i];
      if (KC) {
        if (!(row0 + a < rows && k0 + b < kend)) v = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float2*>(s + a * FLD + (b >> 1)) = make_float2(v.x, v.z);
        *reinterpret_cast<float2*>(s + a * FLD + BKF / 2 + (b >> 1)) = make_float2(v.y, v.w);
      } else {
        if (!(k0 + a < kend && row0 + b < rows)) v = make_float4(0.f, 0.f, 0.f, 0.f);
        const int q = pos(a);
        s[(b + 0) * FLD + q] = v.x;
        s[(b + 1) * FLD + q] = v.y;
        s[(b + 2) * FLD + q] = v.z;
        s[(b + 3) * FLD + q] = v.w;
      }
    }
  }
  // k-steps 4q .. 4q+3 of rows sub0 .. sub0+31: element j = A[sub0 + (l&31)][2(4q + j) + (l>>5)]
  __device__ __forceinline__ static f32x4 frag(const float* s, int sub0, int q) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const f32x4*>(s + (sub0 + (l & 31)) * FLD + (l >> 5) * (BKF / 2) + 4 * q);
  }
};

// XCD-aware order: the hardware deals consecutive workgroup ids round-robin over the 8 XCDs (each with its own
// L2), so id -> (xcd = id % 8, slot = id / 8) is remapped (bijectively) to a linear index that gives every XCD a
// contiguous run. The split index runs fastest (the slabs of a tile are written and reduced on one XCD), then
// the n-tile (the tiles of one XCD share A row-blocks in L2).
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg >> 3, rr = nwg & 7, xcd = id & 7, slot = id >> 3;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
}

enum : int { EPI_STORE = 0, EPI_BIAS_ACT = 1, EPI_ACT_GRAD = 2 };

// One GEMM problem of a (possibly grouped) launch.
struct Prob {
  const __bf16* A;
  const __bf16* B;
  int64_t lda, ldb;
  int M, N, K;
  int tm, tn, splits, kchunk;  // tile grid and split-K
  int wg0;                     // grouped launch: first workgroup id of this problem
  void* C;
  int64_t ldc;
  int out_f32, accumulate;
  const float* bias;   // [N] f32 (or null)
  const float* alpha;  // device scalar (or null = 1)
  int epi, act;        // epilogue kind; activation (0 erf-GELU, 1 tanh-GELU, 2 ReLU)
  const __bf16* aux;   // EPI_ACT_GRAD: pre-activation [M][ld_aux]
  __bf16* aux_out;     // EPI_BIAS_ACT: pre-activation output [M][ld_aux]
  int64_t ld_aux;
  float* rowsum;       // optional [M] f32: alpha · Σ_k A[m][k] (the bias gradient of a dW product)
  float* slab;         // split-K: f32 [splits][tiles][64 x 64] fragment order (+ [splits][M] row sums)
  int* counters;       // split-K, in-launch reduction: one zeroed ticket per tile (left zeroed)
  int ext_reduce;      // split-K: slabs summed by slab_reduce_kernel (a second launch) instead of in-launch
  int fast;            // A and B each < 2 GiB: whole tiles take the buffer-load fast path
  int fm, fn;          // tile = (64·fm) x (64·fn): each of the 4 waves holds fm x fn 32x32 fragments
  const float* rs_extra;  // optional [rs_extra_n][M] f32 rows added into rowsum before alpha
  int rs_extra_n;
  int xmap;  // grouped backward workgroup order: 0 = xcd_remap runs; 1 (dW) / 2 (dX) = split-major (pair_lin)
  int rps;   // xmap 2: dX row blocks per dW split chunk
  int dbg;   // tools build only (ESGPT_GEMM_DBG): bit 0 = skip the bf16 output stores, bit 1 = skip the MFMA k-steps,
             // bit 2 / 3 = grouped backward without its dW / dX workgroups
  const uint8_t* row_tiles;  // optional, one byte per 64 rows of M (esgpt_gemm_row_tiles): 0 = every row of the block
                             // is a padded event's — a tile covering only such blocks skips its k loop
};

// True when the tile's rows [m0, m0 + BM) all lie in 64-row blocks the row-tile mask marks padded.
__device__ __forceinline__ bool rows_skipped(const Prob& p, int m0, int BM) {
  if (p.row_tiles == nullptr) return false;
  const int b0 = m0 >> 6, b1 = min(m0 + BM, p.M) - 1;
  for (int b = b0; b <= (b1 >> 6); ++b)
    if (p.row_tiles[b]) return false;
  return true;
}

// Split-major order of a projection backward (xmap): workgroup id -> XCD x = id % 8 (the dispatcher's round robin),
// slot = id / 8. XCD x takes the dW splits s ≡ x (mod 8) — every tile of each — and the dX row blocks of the same
// token chunks, so one token chunk's dY rows (and X rows) are fetched from HBM once, by one XCD, and shared in its
// L2 by the dW split and the dX tiles that read them (the contiguous-run order had every XCD read all of X and both
// products read dY separately: 3.6x the algorithmic bytes at C2's c_fc). Needs dW splits % 8 == 0 and equal chunks.
__device__ __forceinline__ int pair_lin(const Prob& p, int id) {
  const int x = id & 7, slot = id >> 3;
  if (p.xmap == 1) {  // dW: slot -> (k, tile), split = x + 8k
    const int ntile = p.tm * p.tn;
    const int k = slot / ntile, t = slot - k * ntile;
    return t * p.splits + x + 8 * k;
  }
  const int per = p.rps * p.tn;  // dX tiles per token chunk
  const int k = slot / per, rem = slot - k * per;
  const int by = (x + 8 * k) * p.rps + rem / p.tn, bx = rem % p.tn;
  return by * p.tn + bx;  // dX is never split
}

// Σ_b extra[b][m] (fixed order) of the optional row-sum addend.
__device__ __forceinline__ float rowsum_extra(const Prob& p, int m) {
  float a = 0.f;
  for (int b = 0; b < p.rs_extra_n; ++b) a += p.rs_extra[(int64_t)b * p.M + m];
  return a;
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// gemm_big.hip: launches the large-tile kernel (256 x bn tiles, 8 waves, LDS-DMA ring) for a bf16-output, unsplit
// product with A K-contiguous (false: not applicable, caller launches)
bool launch_big(Prob p, bool akc, bool bkc, int bn, hipStream_t st);
// gemm_big.hip, tools build only: the weight-gradient form on the large-tile kernel (split-K slabs + a reduction
// launch; measured slower than the grouped tile-GEMM backward in the C3 step)
struct BigDw {
  int tm, bn, nwv, splits, kchunk;
  size_t slab_bytes;
};
BigDw big_dw_plan(int64_t T, int64_t in, int64_t out);
bool launch_big_dw(Prob p, hipStream_t st);

// tools/lab/gemm_stream.hip (tools build only): launches the streamed-tile kernel for p when enabled and applicable (false: caller launches)
bool launch_stream(const Prob& p, bool bkc, hipStream_t st);

}  // namespace gk
}  // namespace esgpt
