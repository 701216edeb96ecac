// bf16 MFMA tile GEMM for the training step's projections (the InnerAttention q/k/v/out projections, the InnerMLP
// c_fc/c_proj and the generative heads: transformer.py:133-163, 378-391; generative_layers.py) on gfx950.
//
//   C[M, N] = alpha · A · B (+ bias[n]) (+ epilogue),   bf16 operands, f32 accumulation, C bf16 or f32.
//
// The step's shapes are skinny: M = B·L tokens (8192 for the C2 workload) with N, K in {256 … 1624}, and the
// weight gradients are [out, in] products with K = tokens. Tiles are (64·fm) x (64·fn), 4 waves of fm x fn 32x32
// fragments; 64x64 measured best at these sizes (more resident workgroups hide the load / store latency that
// dominates at K = 256; 128x128 forward / dX tiles were 10-100 % slower), 128x128 for the largest weight gradients. Products with few tiles or
// a long K split K into f32 slabs that the LAST-arriving workgroup of each tile sums in a fixed order (agent-scope
// release / acquire ticket, cdna_hip_programming.md's in-launch split-K recipe; deterministic, no second launch).
// Epilogues fuse what the step needs around a GEMM: bias + activation (c_fc: stores the pre-activation too), the
// activation gradient (c_proj's dX), a device-side alpha (the incoming loss gradient) and the bias gradient
// Σ_k A[m][k] as one extra MFMA against a ones operand. A projection's whole backward (dX = dY·W, dW = dYᵀ·X,
// db = Σ dY) is ONE grouped launch.
//
// Operand layouts (both supported for either operand, so fwd, dX and dW need no transposed copies):
//   A "K-contig": A[m][k] = a[m*lda + k]   LDS image [rows][BK + 8], fragments by 16-B row reads
//   A "M-contig": A[m][k] = a[k*lda + m]   LDS image [BK][96], fragments by ds_read_b64_tr_b16 (hardware
//                                          transpose; row stride = 48 dwords -> conflict-free reads)
//   B likewise with n in place of m ("K-contig": B[k][n] = b[n*ldb + k], "N-contig": B[k][n] = b[k*ldb + n]).
// MFMA v_mfma_f32_32x32x16_bf16; register-staged global->LDS with NS-1 k-tiles in flight during the MFMAs.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_parts.h"

using namespace esgpt;
using namespace esgpt::gk;

namespace {



// One (64·FM)x(64·FN) output tile of problem p (4 waves as 2x2, each wave FM x FN fragments of 32x32);
// `lin` = the tile's index within the problem. The MFMAs compute each fragment transposed (A-operand = B fragment,
// B-operand = A fragment) so that a lane owns one output ROW m and its registers hold columns
// n = (e&3) + 8(e>>2) + 4h: the epilogue stores 16 B per lane. LDS of one tile's staging: two buffers x (A image +
// B image), sized for the operand layouts (the K-contig images are smaller: the 64x64 forward kernel fits 4
// workgroups per CU instead of 3). Also holds the epilogue's C tile (f32: BM x (BN + 4) floats) and the split-K
// reducer flag.
template <bool AKC, bool BKC, int FM, int FN, int NB = 2, int NBG = 0, bool F32 = false>
constexpr int lds_elems() {
  constexpr int st = (NBG > 0 || F32) ? 0 : NB * (Tile<AKC, 64 * FM>::kElems + Tile<BKC, 64 * FN>::kElems);
  constexpr int gl = NBG * (GTile<AKC, 64 * FM>::kElems + GTile<BKC, 64 * FN>::kElems);
  constexpr int f32 = F32 ? 2 * 2 * (FTile<AKC, 64 * FM>::kFloats + FTile<BKC, 64 * FN>::kFloats) : 0;
  constexpr int epi = 64 * FM * (64 * FN + 4) * 2;  // f32 C tile in bf16 elements
  return std::max(std::max(std::max(st, gl), f32), epi);
}

// NB = LDS staging buffers: 2 (one barrier per k-tile) or 1 (two barriers per k-tile, half the LDS: the 64x64
// forward then keeps 8 workgroups per CU resident instead of 4 — every tile of a C2 projection in flight at once).
// NBG > 0: whole tiles are staged by LDS-DMA (GTile) through NBG buffers instead — NBG - 1 k-tiles in flight while
// one is consumed, one raw barrier per k-tile; edge tiles keep the register-staged loop.
// F32: f32 operands through v_mfma_f32_32x32x2_f32 (FTile), f32 outputs.
template <bool AKC, bool BKC, int NS_, int FM, int FN, int NB = 2, int NBG = 0, bool F32 = false>
__device__ __forceinline__ void gemm_tile(const Prob& p, int lin, __bf16* smem) {
  constexpr int NS = NS_, BM = 64 * FM, BN = 64 * FN, F = FM * FN;
  constexpr bool kRowSum = !(AKC && BKC);  // compiled out of the forward (K-contig x K-contig) instantiation
  using TA = Tile<AKC, BM>;
  using TB = Tile<BKC, BN>;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int bz = lin % p.splits, tile = lin / p.splits;
  const int bx = tile % p.tn, by = tile / p.tn;
  const int M = p.M, N = p.N;
  const int m0 = by * BM, n0 = bx * BN;
  const int kb = bz * p.kchunk, ke = min(p.K, kb + p.kchunk);
  // rows of padded events only (row-tile mask): no k loop — the epilogue stores act(0·alpha + bias), or zeros
  const int nk = (ke > kb && !rows_skipped(p, m0, BM)) ? (ke - kb + BK - 1) / BK : 0;
  const __bf16* __restrict__ A = p.A;
  const __bf16* __restrict__ B = p.B;
  const bool want_rs = kRowSum && p.rowsum != nullptr && bx == 0 && wn == 0;  // wave-uniform

  f32x16 acc[FM][FN], racc[FM];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      racc[i][e] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j][e] = 0.f;
    }
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;

  bf16x8 ra[NS][TA::kChunks], rb[NS][TB::kChunks];
  // the k loop in four compiled forms: whole tile or edge tile x with or without the bias-gradient MFMA (both
  // conditions workgroup- / wave-uniform, decided once)
  auto mainloop = [&](auto fast_c, auto rs_c) {
    constexpr bool FAST = decltype(fast_c)::value, RS = decltype(rs_c)::value;
    int voA[TA::kChunks], voB[TB::kChunks];
    __amdgpu_buffer_rsrc_t rsA, rsB;
    if constexpr (FAST) {
      TA::lane_offsets(voA, p.lda, m0);
      TB::lane_offsets(voB, p.ldb, n0);
      rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
      rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(B), (short)0, 0x7fffffff, 0x00020000);
    }
    const int klast = ke - BK;  // FAST: prefetches past the range re-read the last k-tile (never consumed)
    auto load = [&](int st, int i) {
      const int k0 = kb + i * BK;
      if constexpr (FAST) {
        const int kk = min(k0, klast);
        TA::load_fast(ra[st], rsA, voA, TA::k_offset(kk, p.lda));
        TB::load_fast(rb[st], rsB, voB, TB::k_offset(kk, p.ldb));
      } else {
        TA::load(ra[st], A, p.lda, m0, M, k0, ke);
        TB::load(rb[st], B, p.ldb, n0, N, k0, ke);
      }
    };
    auto consume = [&](int st, int i) {
      if constexpr (NB == 1) {
        if (i > 0) __syncthreads();  // every wave is done reading the previous k-tile
      }
      __bf16* sA = smem + (NB == 2 ? (i & 1) : 0) * (TA::kElems + TB::kElems);
      __bf16* sB = sA + TA::kElems;
      if constexpr (FAST) {
        TA::store_fast(sA, ra[st]);
        TB::store_fast(sB, rb[st]);
      } else {
        TA::store(sA, ra[st], m0, M, kb + i * BK, ke);
        TB::store(sB, rb[st], n0, N, kb + i * BK, ke);
      }
      __syncthreads();
      if (p.dbg & 2) return;  // tools build (ESGPT_GEMM_DBG bit 1): operand staging only, no fragment reads / MFMAs
#pragma unroll
      for (int t = 0; t < BK / 16; ++t) {
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = TA::frag(sA, wm * 32 * FM + 32 * i, t);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = TB::frag(sB, wn * 32 * FN + 32 * j, t);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma(bfr[j], af[i], acc[i][j]);
          if constexpr (RS) racc[i] = mfma(ones, af[i], racc[i]);
        }
      }
    };
#pragma unroll
    for (int st = 0; st < NS - 1; ++st) load(st, st);
    int i0 = 0;
    for (; i0 + NS <= nk; i0 += NS) {
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        load((st + NS - 1) % NS, i0 + st + NS - 1);
        consume(st, i0 + st);
      }
    }
#pragma unroll
    for (int st = 0; st < NS - 1; ++st)
      if (i0 + st < nk) consume(st, i0 + st);
  };
  // LDS-DMA form of the whole-tile k loop: NBG buffers, k-tile i+NBG-1 issued right after the barrier that retires
  // k-tile i (every wave is then done reading buffer (i-1) % NBG, which it overwrites), so NBG-1 k-tiles stream in
  // while one is consumed. The counted vmcnt before each barrier leaves the younger k-tiles in flight (an LDS-DMA is
  // ordered for a ds_read only by its issuing wave's vmcnt plus a barrier: MI355X_MICROARCH.md item 7); raw
  // s_barrier, as __syncthreads() would drain every DMA in flight (vmcnt(0)).
  auto mainloop_glds = [&](auto rs_c) {
    constexpr bool RS = decltype(rs_c)::value;
    using GA = GTile<AKC, BM>;
    using GB = GTile<BKC, BN>;
    constexpr int P = GA::kInstr + GB::kInstr, STAGE = GA::kElems + GB::kElems;
    constexpr int NBq = NBG > 1 ? NBG : 2;
    int voA[GA::kInstr], voB[GB::kInstr];
    GA::lane_src(voA, p.lda, m0, M);
    GB::lane_src(voB, p.ldb, n0, N);
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(B), (short)0, 0x7fffffff, 0x00020000);
    auto issue = [&](int i, int buf) {
      const int k0 = kb + i * BK, kv = ke - k0;
      __bf16* sA = smem + buf * STAGE;
      GA::issue(rsA, voA, GA::k_soff(k0, p.lda), sA, kv);
      GB::issue(rsB, voB, GB::k_soff(k0, p.ldb), sA + GA::kElems, kv);
    };
#pragma unroll
    for (int st = 0; st < NBq - 1; ++st)
      if (st < nk) issue(st, st);
    for (int i = 0; i < nk; ++i) {
      const int ahead = min(NBq - 2, nk - 1 - i);  // k-tiles allowed in flight once k-tile i has landed
      if (NBq >= 4 && ahead >= 2) vm_wait<(NBq >= 4 ? 2 * P : 0)>();
      else if (NBq >= 3 && ahead >= 1) vm_wait<(NBq >= 3 ? P : 0)>();
      else vm_wait<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (i + NBq - 1 < nk) issue(i + NBq - 1, (i + NBq - 1) % NBq);
      const __bf16* sA = smem + (i % NBq) * STAGE;
      const __bf16* sB = sA + GA::kElems;
      // fragments of k-step t + 1 are read while the MFMAs of k-step t run
      bf16x8 af[2][FM], bfr[2][FN];
      auto read = [&](int t, int b) {
#pragma unroll
        for (int ii = 0; ii < FM; ++ii) af[b][ii] = GA::frag(sA, wm * 32 * FM + 32 * ii, t);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[b][j] = GB::frag(sB, wn * 32 * FN + 32 * j, t);
      };
      read(0, 0);
#pragma unroll
      for (int t = 0; t < BK / 16; ++t) {
        if constexpr (!(AKC && BKC)) frag_wait();
        if (t + 1 < BK / 16) read(t + 1, (t + 1) & 1);
#pragma unroll
        for (int ii = 0; ii < FM; ++ii) {
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[ii][j] = mfma(bfr[t & 1][j], af[t & 1][ii], acc[ii][j]);
          if constexpr (RS) racc[ii] = mfma(ones, af[t & 1][ii], racc[ii]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // f32 operands: two LDS buffers (one barrier per k-stage), the next stage's loads in flight during the MFMAs
  auto mainloop_f32 = [&](auto rs_c) {
    constexpr bool RS = decltype(rs_c)::value;
    using FA = FTile<AKC, BM>;
    using FB = FTile<BKC, BN>;
    float* sm = reinterpret_cast<float*>(smem);
    const float* Af = reinterpret_cast<const float*>(A);
    const float* Bf = reinterpret_cast<const float*>(B);
    const int nkf = (ke > kb && !rows_skipped(p, m0, BM)) ? (ke - kb + BKF - 1) / BKF : 0;
    float4 ra[FA::kChunks], rb[FB::kChunks];
    if (nkf > 0) {
      FA::load(ra, Af, p.lda, m0, M, kb, ke);
      FB::load(rb, Bf, p.ldb, n0, N, kb, ke);
    }
    for (int i = 0; i < nkf; ++i) {
      float* sA = sm + (i & 1) * (FA::kFloats + FB::kFloats);
      float* sB = sA + FA::kFloats;
      FA::store(sA, ra, m0, M, kb + i * BKF, ke);
      FB::store(sB, rb, n0, N, kb + i * BKF, ke);
      __syncthreads();
      if (i + 1 < nkf) {
        FA::load(ra, Af, p.lda, m0, M, kb + (i + 1) * BKF, ke);
        FB::load(rb, Bf, p.ldb, n0, N, kb + (i + 1) * BKF, ke);
      }
#pragma unroll
      for (int q = 0; q < BKF / 8; ++q) {
        f32x4 af[FM], bfr[FN];
#pragma unroll
        for (int ii = 0; ii < FM; ++ii) af[ii] = FA::frag(sA, wm * 32 * FM + 32 * ii, q);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = FB::frag(sB, wn * 32 * FN + 32 * j, q);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int ii = 0; ii < FM; ++ii) {
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(bfr[j][t], af[ii][t], acc[ii][j], 0, 0, 0);
            if constexpr (RS) racc[ii] = __builtin_amdgcn_mfma_f32_32x32x2f32(1.f, af[ii][t], racc[ii], 0, 0, 0);
          }
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if constexpr (F32) {
    if (want_rs) mainloop_f32(T_{});
    else mainloop_f32(F_{});
  } else if constexpr (NBG > 0) {  // every tile (the host takes this form only for operands below 2 GiB: p.fast)
    if (want_rs) mainloop_glds(T_{});
    else mainloop_glds(F_{});
  } else {
    const bool fast = p.fast && m0 + BM <= M && n0 + BN <= N && nk > 0 && (ke - kb) % BK == 0;
    if (fast) {
      if (want_rs) mainloop(T_{}, T_{});
      else mainloop(T_{}, F_{});
    } else {
      if (want_rs) mainloop(F_{}, T_{});
      else mainloop(F_{}, F_{});
    }
  }

  // this lane's output row of fragment row i, and the first column of fragment column j (within the tile)
  auto lrow = [&](int i) { return wm * 32 * FM + 32 * i + r; };
  auto lcol = [&](int j) { return wn * 32 * FN + 32 * j; };

  // ---- split-K: slab, ticket, the last arriver reduces in z order ----
  // Hand-off in its write-through form (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms): every slab
  // store is an sc1 (write-through) store, every storing wave drains it (vmcnt(0)) before the workgroup barrier and
  // one agent-scope ticket add; the workgroup whose add comes last reads every slab with sc1 loads. No L2
  // write-back fence: with the grouped dX product streaming its output through the same L2s, buffer_wbl2 per
  // workgroup serialised on the dirty lines of the whole XCD. Slabs are lane-linear (fragment order: tile, wave,
  // fragment, register group, lane): each wave-instruction writes / reads 1 KiB contiguously — whole lines, no
  // partial-line write-through.
  const int ntile = p.tm * p.tn;
  auto slab_idx = [&](int z, int f, int g) {  // float index of this lane's 4 values
    return 4 * (((((z * ntile + tile) * 4 + wave) * F + f) * 4 + g) * 64 + lane);
  };
  const int rs_base = p.splits * ntile * BM * BN;  // row-sum slabs follow the tile slabs
  if (p.splits > 1 && p.ext_reduce) {
    // slabs only (plain stores: the kernel boundary orders them before slab_reduce_kernel)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(p.slab + slab_idx(bz, i * FN + j, g)) =
              make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
    if (want_rs && h == 0)
#pragma unroll
      for (int i = 0; i < FM; ++i)
        if (m0 + lrow(i) < M) p.slab[rs_base + (int64_t)bz * M + m0 + lrow(i)] = racc[i][0];
    return;
  }
  if (p.splits > 1) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(p.slab, (short)0, 0x7fffffff, 0x00020000);
    constexpr int kSC1 = 16;  // cache policy: sc1
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const u32x4 w = {__float_as_uint(acc[i][j][4 * g]), __float_as_uint(acc[i][j][4 * g + 1]),
                           __float_as_uint(acc[i][j][4 * g + 2]), __float_as_uint(acc[i][j][4 * g + 3])};
          __builtin_amdgcn_raw_buffer_store_b128(w, rs, 4 * slab_idx(bz, i * FN + j, g), 0, kSC1);
        }
    if (want_rs && h == 0)
#pragma unroll
      for (int i = 0; i < FM; ++i)
        if (m0 + lrow(i) < M)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(racc[i][0]), rs,
                                                4 * (rs_base + bz * M + m0 + lrow(i)), 0, kSC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's slab stores have drained (and the LDS tiles are no longer read)
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0) {
      const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == p.splits - 1;
      if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        racc[i][e] = 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j][e] = 0.f;
      }
    }
    // slabs in batches of kRB: every load of a batch in flight before the (z-ordered, deterministic) adds — one
    // memory round trip per batch instead of one per slab
    constexpr int kRB = F >= 4 ? 1 : 4 / F;
    for (int z0 = 0; z0 < p.splits; z0 += kRB) {
      u32x4 x[kRB][F][4];
      float rv[kRB][FM];
#pragma unroll
      for (int u = 0; u < kRB; ++u) {
        const int z = min(z0 + u, p.splits - 1);
#pragma unroll
        for (int f = 0; f < F; ++f)
#pragma unroll
          for (int g = 0; g < 4; ++g) x[u][f][g] = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * slab_idx(z, f, g), 0, kSC1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
          rv[u][i] = (want_rs && m0 + lrow(i) < M) ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                                          rs, 4 * (rs_base + z * M + m0 + lrow(i)), 0, kSC1))
                                                    : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kRB; ++u) {
        if (z0 + u >= p.splits) break;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              acc[i][j][4 * g] += __uint_as_float(x[u][i * FN + j][g][0]);
              acc[i][j][4 * g + 1] += __uint_as_float(x[u][i * FN + j][g][1]);
              acc[i][j][4 * g + 2] += __uint_as_float(x[u][i * FN + j][g][2]);
              acc[i][j][4 * g + 3] += __uint_as_float(x[u][i * FN + j][g][3]);
            }
          racc[i][0] += rv[u][i];
        }
      }
    }
  }

  // ---- epilogue: lane = row, register group g = columns lcol(j) + 8g + 4h + {0..3} ----
  const float al = p.alpha ? *p.alpha : 1.f;
  if (want_rs && h == 0)
#pragma unroll
    for (int i = 0; i < FM; ++i)
      if (m0 + lrow(i) < M) p.rowsum[m0 + lrow(i)] = (racc[i][0] + rowsum_extra(p, m0 + lrow(i))) * al;
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = n0 + lcol(j) + 8 * g + 4 * h;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias && c < N) bv = *reinterpret_cast<const float4*>(p.bias + c);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc[i][j][4 * g + 0] = acc[i][j][4 * g + 0] * al + bv.x;
        acc[i][j][4 * g + 1] = acc[i][j][4 * g + 1] * al + bv.y;
        acc[i][j][4 * g + 2] = acc[i][j][4 * g + 2] * al + bv.z;
        acc[i][j][4 * g + 3] = acc[i][j][4 * g + 3] * al + bv.w;
      }
    }
  // The tile goes out through LDS (the staging buffers are free once every wave is past its last fragment read):
  // written in fragment order, stored row-major with 16-B chunks, each wave-instruction covering whole 128-B lines
  // instead of 32-B pieces of 32 rows.
  __syncthreads();
  if (p.out_f32) {
    // f32 operands (F32): the activation-gradient epilogue reads an f32 pre-activation
    if (F32 && p.epi == EPI_ACT_GRAD) {
      const float* aux = reinterpret_cast<const float*>(p.aux);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = m0 + lrow(i);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int c = n0 + lcol(j) + 8 * g + 4 * h;
            if (row < M && c < N) {
              const float4 f = *reinterpret_cast<const float4*>(aux + (int64_t)row * p.ld_aux + c);
              acc[i][j][4 * g + 0] *= act_factor(f.x, p.act);
              acc[i][j][4 * g + 1] *= act_factor(f.y, p.act);
              acc[i][j][4 * g + 2] *= act_factor(f.z, p.act);
              acc[i][j][4 * g + 3] *= act_factor(f.w, p.act);
            }
          }
      }
    }
    constexpr int kLd = BN + 4;  // f32 row pitch (floats): 16-B aligned, conflict-free fragment writes
    float* t = reinterpret_cast<float*>(smem);
    // one f32 tile out: fragment-order LDS writes, barrier, row-major 16-B chunk stores (+= when accumulating)
    auto store_f32 = [&](float* dst, int64_t ld, bool accum) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(t + lrow(i) * kLd + lcol(j) + 8 * g + 4 * h) =
                make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < BM * BN / 4 / THREADS; ++q) {
        const int ch = threadIdx.x + THREADS * q, tr = ch / (BN / 4), tc = (ch % (BN / 4)) * 4;
        const int gr = m0 + tr, gc = n0 + tc;
        if (gr >= M || gc >= N) continue;
        float4 w = *reinterpret_cast<const float4*>(t + tr * kLd + tc);
        float4* o4 = reinterpret_cast<float4*>(dst + (int64_t)gr * ld + gc);
        if (accum) {
          const float4 o = *o4;
          w.x += o.x;
          w.y += o.y;
          w.z += o.z;
          w.w += o.w;
        }
        *o4 = w;
      }
    };
    if (F32 && p.epi == EPI_BIAS_ACT) {  // the f32 pre-activation (or its act' under ESGPT_ACT_DERIV), then act
      if (p.act & ESGPT_ACT_DERIV) {
        f32x16 yv[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              float y, g;
              act_fwd_grad(acc[i][j][e], p.act & 7, y, g);
              yv[i][j][e] = y;
              acc[i][j][e] = g;
            }
        store_f32(reinterpret_cast<float*>(p.aux_out), p.ld_aux, false);
        __syncthreads();  // the LDS tile is rewritten below
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = yv[i][j];
      } else {
        store_f32(reinterpret_cast<float*>(p.aux_out), p.ld_aux, false);
        __syncthreads();  // the LDS tile is rewritten below
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = act_fwd(acc[i][j][e], p.act);
      }
    }
    store_f32(reinterpret_cast<float*>(p.C), p.ldc, p.accumulate != 0);
    return;
  }
  if (p.epi == EPI_ACT_GRAD) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = m0 + lrow(i);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = n0 + lcol(j) + 8 * g + 4 * h;
          if (row < M && c < N) {
            const uint2 f = *reinterpret_cast<const uint2*>(p.aux + (int64_t)row * p.ld_aux + c);
            acc[i][j][4 * g + 0] *= act_factor(bf16_lo(f.x), p.act);
            acc[i][j][4 * g + 1] *= act_factor(bf16_hi(f.x), p.act);
            acc[i][j][4 * g + 2] *= act_factor(bf16_lo(f.y), p.act);
            acc[i][j][4 * g + 3] *= act_factor(bf16_hi(f.y), p.act);
          }
        }
    }
  }
  constexpr int kLdB = BN + 8;  // bf16 row pitch (elements): conflict-free 8-B fragment writes
  __bf16* tb = smem;
  // one bf16 tile out: fragment-order LDS writes, barrier, row-major 16-B chunk stores
  auto store_tile = [&](const uint32_t (&d)[FM][FN][4][2], __bf16* dst, int64_t ld) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<uint2*>(tb + lrow(i) * kLdB + lcol(j) + 8 * g + 4 * h) = make_uint2(d[i][j][g][0], d[i][j][g][1]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BM * BN / 8 / THREADS; ++q) {
      const int ch = threadIdx.x + THREADS * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
      const int gr = m0 + tr, gc = n0 + tc;
      if (gr < M && gc < N && !(p.dbg & 1))
        *reinterpret_cast<uint4*>(dst + (int64_t)gr * ld + gc) = *reinterpret_cast<const uint4*>(tb + tr * kLdB + tc);
    }
  };
  uint32_t d[FM][FN][4][2];
  if (p.epi == EPI_BIAS_ACT) {
    // store the pre-activation (bf16: the value the activation and its gradient see), then activate it
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          d[i][j][g][0] = pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
          d[i][j][g][1] = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          if (p.act & ESGPT_ACT_DERIV) {  // act and act' of the bf16 pre-activation; act' is what gets stored
            float gd[4], yd[4];
            act_fwd_grad(bf16_lo(d[i][j][g][0]), p.act & 7, yd[0], gd[0]);
            act_fwd_grad(bf16_hi(d[i][j][g][0]), p.act & 7, yd[1], gd[1]);
            act_fwd_grad(bf16_lo(d[i][j][g][1]), p.act & 7, yd[2], gd[2]);
            act_fwd_grad(bf16_hi(d[i][j][g][1]), p.act & 7, yd[3], gd[3]);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = yd[e];
            d[i][j][g][0] = pack_bf16x2(gd[0], gd[1]);
            d[i][j][g][1] = pack_bf16x2(gd[2], gd[3]);
          } else {
            acc[i][j][4 * g + 0] = act_fwd(bf16_lo(d[i][j][g][0]), p.act);
            acc[i][j][4 * g + 1] = act_fwd(bf16_hi(d[i][j][g][0]), p.act);
            acc[i][j][4 * g + 2] = act_fwd(bf16_lo(d[i][j][g][1]), p.act);
            acc[i][j][4 * g + 3] = act_fwd(bf16_hi(d[i][j][g][1]), p.act);
          }
        }
    store_tile(d, p.aux_out, p.ld_aux);
    __syncthreads();  // the LDS tile is rewritten below
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        d[i][j][g][0] = pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
        d[i][j][g][1] = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
      }
  store_tile(d, reinterpret_cast<__bf16*>(p.C), p.ldc);
}

template <bool AKC, bool BKC, int NS_, int FM, int FN, int NB = 2, int NBG = 0, bool F32 = false>
__global__ __launch_bounds__(THREADS) void gemm_kernel(Prob p) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[lds_elems<AKC, BKC, FM, FN, NB, NBG, F32>()];
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  gemm_tile<AKC, BKC, NS_, FM, FN, NB, NBG, F32>(p, lin, smem);
}

// The same tiles walked by a persistent grid (gridDim.x a multiple of 8 and at most the tile count): workgroup b
// takes ids b, b + grid, … — all on b's XCD — mapped by xcd_remap over the whole tile range, so each XCD still walks
// a contiguous run of tiles. (Tools-build experiment, ESGPT_GEMM_PERSIST = workgroups per CU.)
template <bool AKC, bool BKC, int NS_, int FM, int FN, int NB = 2>
__global__ __launch_bounds__(THREADS) void gemm_persist_kernel(Prob p, int ntiles) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[lds_elems<AKC, BKC, FM, FN, NB>()];
  for (int id = blockIdx.x; id < ntiles; id += gridDim.x) {
    gemm_tile<AKC, BKC, NS_, FM, FN, NB>(p, xcd_remap(id, ntiles), smem);
    __syncthreads();  // the LDS images / epilogue tile are rewritten by the next tile
  }
}

// Forward LDS staging buffers (1 or 2; ESGPT_GEMM_FWD_NB tuning hook, read once).
int fwd_buffers() {
  static int nb = 0;
  if (nb == 0) {
    const char* e = tuning_env("ESGPT_GEMM_FWD_NB");
    nb = (e && atoi(e) == 2) ? 2 : 1;
  }
  return nb;
}

// LDS-DMA staging buffers of the whole-tile k loops (0 = register staging; ESGPT_GEMM_FWD_GLDS /
// ESGPT_GEMM_BWD_GLDS tuning hooks, read once). Measured at the C2 shapes (tools/glds_check.sh,
// tools/glds_bwd_sweep.sh, profiles/r04_glds_*.log): in isolation the forward projections gain 3-12 % from two
// LDS-DMA buffers (qkv 10.3 -> 9.1-9.4 us, head 20.0 -> 17.7-19.0 us; three buffers lose), but inside the training
// step register staging is faster on every bench config (tools/env_sweep.sh, ESGPT_GEMM_FWD_GLDS=0: C2 1.695 ->
// 1.651 ms, C3 11.52 -> 11.38, C4 6.65 -> 6.59, C5 3.95 -> 3.89; profiles/r05b_fwd_glds_sweep.log), so the forward
// keeps register staging by default too; the grouped backward loses 4-6 % with either depth (627 -> 659 / 671 us
// per step's set) and at every dX / dW tile size.
int fwd_glds() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_GEMM_FWD_GLDS");
    v = e ? std::min(3, std::max(0, atoi(e))) : 0;
    if (v == 1) v = 2;
  }
  return v;
}
int bwd_glds() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_GEMM_BWD_GLDS");
    v = e ? std::min(3, std::max(0, atoi(e))) : 0;
    if (v == 1) v = 2;
  }
  return v;
}

// Forward register-stage depth (2 or 3; ESGPT_GEMM_FWD_NS tuning hook, read once).
int fwd_stages() {
  static int ns = 0;
  if (ns == 0) {
    const char* e = tuning_env("ESGPT_GEMM_FWD_NS");
    ns = e ? std::min(5, std::max(2, atoi(e))) : 3;
  }
  return ns;
}

// A projection's backward in one launch: problem 0 = dX (A = dY K-contig, B = W N-contig), problem 1 = dW (A = dYᵀ
// M-contig, B = X N-contig, + the bias gradient). The dW workgroups (the long K = tokens chains) take the first
// p0.wg0 workgroup ids, so the dispatcher deals them round-robin over all 8 XCDs first and the short dX tiles
// fill in behind them; each problem keeps its own XCD-aware order within its id range.
// Register stages of the backward products: 2 for the 4-fragment tiles (3 would leave 1 wave per SIMD).
template <int FM, int FN>
constexpr int bwd_stages() {
  return FM * FN >= 4 ? 2 : NS;
}

template <int XM, int XN, int WM, int WN, int NBG = 0, bool F32 = false>
__global__ __launch_bounds__(THREADS) void gemm_bwd_pair_kernel(Prob p0, Prob p1) {
  constexpr int kLds =
      std::max(lds_elems<false, false, WM, WN, 2, NBG, F32>(), lds_elems<true, false, XM, XN, 2, NBG, F32>());
  __shared__ __attribute__((aligned(16))) __bf16 smem[kLds];
  const int id = blockIdx.x, n1 = p0.wg0;
  if (id < n1) {
    if (p1.dbg & 4) return;  // tools build: the dX product alone
    gemm_tile<false, false, bwd_stages<WM, WN>(), WM, WN, 2, NBG, F32>(
        p1, p1.xmap ? pair_lin(p1, id) : xcd_remap(id, n1), smem);
  } else {
    if (p0.dbg & 8) return;  // tools build: the dW product alone
    gemm_tile<true, false, bwd_stages<XM, XN>(), XM, XN, 2, NBG, F32>(
        p0, p0.xmap ? pair_lin(p0, id - n1) : xcd_remap(id - n1, gridDim.x - n1), smem);
  }
}

// Split-K reduction as its own launch (large slab sets: one last-arriving workgroup reading every slab of its tile
// is a serial memory-latency chain on one CU; here every CU takes a share). f32 output, plain store epilogue (the
// weight-gradient products): thread = one 16-B fragment chunk (tile, wave, fragment, register group, lane) of the
// output, summing its splits in z order (deterministic), then alpha, bias, accumulate, and the 4 columns stored;
// threads past the tiles sum the row-sum slabs into p.rowsum.
__global__ __launch_bounds__(256) void slab_reduce_kernel(Prob p) {
  const int F = p.fm * p.fn, BM = 64 * p.fm, BN = 64 * p.fn;
  const int64_t ntile = (int64_t)p.tm * p.tn, nch = ntile * BM * BN / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float al = p.alpha ? *p.alpha : 1.f;
  if (t < nch) {
    const int lane = (int)(t & 63), g = (int)((t >> 6) & 3);
    const int64_t wf = t >> 8;  // (tile, wave, fragment)
    const int f = (int)(wf % F), wave = (int)((wf / F) & 3);
    const int64_t tile = wf / F / 4;
    const int bx = (int)(tile % p.tn), by = (int)(tile / p.tn);
    const int row = by * BM + (wave >> 1) * 32 * p.fm + (f / p.fn) * 32 + (lane & 31);
    const int col = bx * BN + (wave & 1) * 32 * p.fn + (f % p.fn) * 32 + 8 * g + 4 * (lane >> 5);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int kU = 8;
    for (int z0 = 0; z0 < p.splits; z0 += kU) {
      float4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int z = min(z0 + u, p.splits - 1);
        v[u] = *reinterpret_cast<const float4*>(p.slab + ((int64_t)z * nch + t) * 4);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (z0 + u >= p.splits) break;
        a.x += v[u].x;
        a.y += v[u].y;
        a.z += v[u].z;
        a.w += v[u].w;
      }
    }
    if (row < p.M && col < p.N) {
      float4* q = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + (int64_t)row * p.ldc + col);
      float4 w = make_float4(a.x * al, a.y * al, a.z * al, a.w * al);
      if (p.bias) {
        const float4 b = *reinterpret_cast<const float4*>(p.bias + col);
        w.x += b.x;
        w.y += b.y;
        w.z += b.z;
        w.w += b.w;
      }
      if (p.accumulate) {
        const float4 o = *q;
        w.x += o.x;
        w.y += o.y;
        w.z += o.z;
        w.w += o.w;
      }
      *q = w;
    }
  } else if (p.rowsum && t - nch < p.M) {
    const int64_t m = t - nch;
    const float* rs = p.slab + (int64_t)p.splits * nch * 4;
    float a = 0.f;
    for (int z = 0; z < p.splits; ++z) a += rs[(int64_t)z * p.M + m];
    p.rowsum[m] = (a + rowsum_extra(p, (int)m)) * al;
  }
}

void launch_slab_reduce(const Prob& p, hipStream_t st) {
  const int64_t n = (int64_t)p.tm * p.tn * 64 * p.fm * 64 * p.fn / 4 + (p.rowsum ? p.M : 0);
  slab_reduce_kernel<<<(unsigned)cdiv(n, 256), 256, 0, st>>>(p);
}

// Slab sets above this many splits are reduced by slab_reduce_kernel (f32 outputs without an epilogue); smaller
// ones by the tile's last-arriving workgroup (ESGPT_GEMM_INLAUNCH_SPLITS tuning hook, read once; measured at C2:
// in-launch for the grouped backward pairs (8 splits) is 0.09 ms per step faster than the separate launch).
int in_launch_splits() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_GEMM_INLAUNCH_SPLITS");
    v = e ? std::max(1, atoi(e)) : 32;
  }
  return v;
}

constexpr int64_t kMaxChunk = 1024;
constexpr int64_t kTarget = 480;  // about two resident 64x64 tiles per CU

// Tile shape of a product: (64·fm) x (64·fn). Larger tiles read each operand fewer times through L2 (the 64x64
// tile's k-loop is bound by the L2 -> CU rate at ≈32 B per MFMA-cycle) but put fewer workgroups on the chip.
struct TileCfg {
  int fm, fn;
};

// ESGPT_GEMM_TILE_FWD / _DX / _DW = "<fm><fn>" (e.g. "22"): tuning hooks, read once; only compiled shapes accepted.
TileCfg env_tile(const char* name, TileCfg def, const int* allowed, int n_allowed) {
  const char* e = tuning_env(name);
  if (!e) return def;
  const int code = atoi(e);
  for (int i = 0; i < n_allowed; ++i)
    if (allowed[i] == code) return TileCfg{code / 10, code % 10};
  return def;
}
constexpr int kFwdTiles[] = {11, 21, 12, 22};
constexpr int kDxTiles[] = {11, 21, 22};
constexpr int kDwTiles[] = {11, 22};

// Forward tiles: 128x64 for the plain-store products with K <= 256 and at least 512 output columns (tools/fwd_sweep.sh,
// C2 shapes: qkv 11.2 -> 10.2 us, head 20.3 -> 19.2 us), 64x64 otherwise (out_proj and c_fc with its activation
// epilogue are 5-13 % slower at 128x64, c_proj at K = 1024 equal).
// Wide products (K and N >= 512, e.g. C3's d = 512 / 2048 layers) on 128x128 tiles: four times the MFMAs per
// operand tile load where the 64x64 tile's per-tile overhead dominates (C3 step, tools/tile_sweep_cfg.sh C3: every
// forward on 128x128 12.69 -> 12.50 ms, every dX 12.69 -> 11.76 ms; at d = 256 (C2, C4) 64x64 stays best).
TileCfg fwd_tile(int64_t M, int64_t N, int64_t K, bool act) {
  static const TileCfg forced = env_tile("ESGPT_GEMM_TILE_FWD", TileCfg{0, 0}, kFwdTiles, 4);
  if (forced.fm) return forced;
  if (!act && K <= 256 && N >= 512 && M >= 128) return TileCfg{2, 1};
  return (K >= 512 && N >= 512 && M >= 4096) ? TileCfg{2, 2} : TileCfg{1, 1};
}
TileCfg dx_tile(int64_t T, int64_t in, int64_t out) {
  static const TileCfg forced = env_tile("ESGPT_GEMM_TILE_DX", TileCfg{0, 0}, kDxTiles, 3);
  if (forced.fm) return forced;
  if (in >= 512 && out >= 512 && T >= 4096) return TileCfg{2, 2};
  return T >= 16384 ? TileCfg{2, 1} : TileCfg{1, 1};  // long token runs (C4's dependency graph, C5): 128x64
}
// dW [out, in] over K = T tokens: 128x128 tiles once the 64x64 plan (at its minimum split count, one split per
// kMaxChunk of tokens) would put more than three workgroups per CU on the chip — their f32 slab traffic then costs
// more than the fewer workgroups (C2: the generative head's [1624, 256] 45 -> 37 us; c_fc's [1024, 256] stays
// 64x64: 24 vs 27 us).
TileCfg dw_tile(int64_t T, int64_t in, int64_t out) {
  static const TileCfg forced = env_tile("ESGPT_GEMM_TILE_DW", TileCfg{0, 0}, kDwTiles, 2);
  if (forced.fm) return forced;
  const int64_t wg = cdiv(out, 64) * cdiv(in, 64) * std::max<int64_t>(1, T / kMaxChunk);
  return wg > 3 * 256 ? TileCfg{2, 2} : TileCfg{1, 1};
}

// activation codes: 0 erf-GELU, 1 tanh-GELU, 2 ReLU, optionally | ESGPT_ACT_DERIV
bool act_ok(int act) { return act >= 0 && (act & ~ESGPT_ACT_DERIV) <= 2; }

int64_t n_tiles(int64_t M, int64_t N, TileCfg c) { return cdiv(M, 64 * c.fm) * cdiv(N, 64 * c.fn); }

// Large-tile kernel (gemm_big.hip) for a bf16-output product: 256 or 128 output columns per 256-row tile, 0 = the
// tile GEMM. Product rule (measured in the C3 training step, same box, profiles/r06_c3_big_ab.log): the plain-store
// forward projections of wide layers (M >= 4096 tokens, K and N >= 512, no activation epilogue: C3's qkv, out_proj
// and c_proj) on 256 x 128 tiles — 42 vs 50 us per launch in step; c_fc with its activation epilogue (two outputs of
// 64 MB each) stays on the tile GEMM, whose 2-3 resident workgroups per CU overlap one tile's epilogue with another's
// k-loop (80 vs 110 us); the backward (large-tile dX + split-K dW + slab reduction) lost to the grouped tile-GEMM
// backward (about 440 vs 390 us per layer) and exists in the tools build only (ESGPT_GEMM_BIG = 0 / 128 / 256 forces
// every eligible product there, fwd / dX / dW).
int big_fwd_cols(int64_t M, int64_t N, int64_t K, bool act) {
  static const int forced = [] {
    const char* e = tuning_env("ESGPT_GEMM_BIG");
    return e ? atoi(e) : -1;
  }();
  if (forced == 0 || forced == 128 || forced == 256) return forced;
  return (!act && M >= 4096 && K >= 512 && N >= 512) ? 128 : 0;
}
#ifdef ESGPT_TUNING_HOOKS
// tools build: the large-tile backward (dX + split-K dW) when ESGPT_GEMM_BIG forces it
int big_cols(int64_t M, int64_t N, int64_t K) {
  const int f = big_fwd_cols(M, N, K, false);
  return (f == 128 || f == 256) && tuning_env("ESGPT_GEMM_BIG") ? f : 0;
}
#else
int big_cols(int64_t, int64_t, int64_t) { return 0; }
#endif

struct Plan {
  int splits, kchunk;
};

// Split-K: enough workgroups for `target` (<= 0: never split), and no workgroup walks more than kMaxChunk of K
// (a long K is one long serial chain: 8192 tokens = 128 k-tiles), never below 256 of K per split.

Plan plan(int64_t M, int64_t N, int64_t K, int64_t target, TileCfg c) {
  Plan p{1, (int)(cdiv(K, BK) * BK)};
  if (K == 0 || target <= 0) return p;
  int64_t splits = 1;
  if (const char* e = tuning_env("ESGPT_GEMM_SPLITS")) {  // tuning hook
    splits = std::max<int64_t>(1, atoi(e));
  } else {
    const int64_t tiles = n_tiles(M, N, c);
    if (tiles < target) splits = cdiv(target, tiles);
    splits = std::max<int64_t>(splits, K / kMaxChunk);
    splits = std::min<int64_t>(splits, std::max<int64_t>(1, K / 256));
  }
  const int64_t kchunk = cdiv(cdiv(K, splits), BK) * BK;
  p.splits = (int)cdiv(K, kchunk);
  p.kchunk = (int)kchunk;
  return p;
}

// Row-tile mask of the next launches on this host thread (esgpt_gemm_row_tiles): applied to products whose M is
// token rows — the forward projections and the dX half of the grouped backward.
static thread_local const uint8_t* g_row_tiles = nullptr;

Prob make_prob(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K, void* C,
               int64_t ldc, int out_f32, int accumulate, const float* bias, const float* alpha, int64_t target,
               TileCfg c) {
  Prob p{};
  p.A = reinterpret_cast<const __bf16*>(A);
  p.B = reinterpret_cast<const __bf16*>(B);
  p.lda = lda;
  p.ldb = ldb;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.fm = c.fm;
  p.fn = c.fn;
  p.tm = (int)cdiv(M, 64 * c.fm);
  p.tn = (int)cdiv(N, 64 * c.fn);
  const Plan pl = plan(M, N, K, target, c);
  p.splits = pl.splits;
  p.kchunk = pl.kchunk;
  p.C = C;
  p.ldc = ldc;
  p.out_f32 = out_f32;
  p.accumulate = accumulate;
  p.bias = bias;
  p.alpha = alpha;
  // operand extents in bytes (K-contig: rows x ld; M/N-contig: K rows x ld) within the 32-bit buffer offsets
  const int64_t lim = (int64_t)1 << 31;
  p.fast = (std::max(M, K) * lda * 2 < lim && std::max(N, K) * ldb * 2 < lim) ? 1 : 0;
  return p;
}

// Split-K slabs: [splits][tiles][BM x BN] f32 in fragment order, then [splits][M] row sums.
size_t slab_bytes(int64_t splits, int64_t M, int64_t N, TileCfg c) {
  return splits > 1 ? sizeof(float) * ((size_t)splits * n_tiles(M, N, c) * 64 * c.fm * 64 * c.fn + (size_t)splits * M)
                    : 0;
}

int n_wg(const Prob& p) { return p.tm * p.tn * p.splits; }

// Shared argument checks of a bf16 product with a 16-B epilogue (K > 0: an empty reduction is the caller's case).
bool shapes_ok(bool akc, bool bkc, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N,
               int64_t K, const void* C, int64_t ldc, bool f32) {
  if (!(A && B && C && M >= 0 && N >= 0 && K > 0)) return false;
  if (!(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31))) return false;
  // K is the chunked (16-B) dimension only of a K-contig operand; an M/N-contig operand takes any K (k = its row)
  if (!((K % 8 == 0 || !(akc || bkc)) && lda % 8 == 0 && ldb % 8 == 0)) return false;
  if (!((akc || M % 8 == 0) && (bkc || N % 8 == 0))) return false;
  if (((uintptr_t)A % 16) || ((uintptr_t)B % 16) || ((uintptr_t)C % 16)) return false;
  const int cgrp = f32 ? 4 : 8;
  return N % cgrp == 0 && ldc % cgrp == 0;
}

// The same checks for f32 operands and an f32 output (16-B chunks of 4 elements).
bool shapes_ok_f32(bool akc, bool bkc, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N,
                   int64_t K, const void* C, int64_t ldc) {
  if (!(A && B && C && M >= 0 && N >= 0 && K > 0)) return false;
  if (!(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31))) return false;
  if (!((K % 4 == 0 || !(akc || bkc)) && lda % 4 == 0 && ldb % 4 == 0)) return false;
  if (!((akc || M % 4 == 0) && (bkc || N % 4 == 0))) return false;
  if (((uintptr_t)A % 16) || ((uintptr_t)B % 16) || ((uintptr_t)C % 16)) return false;
  return N % 4 == 0 && ldc % 4 == 0;
}

// Workgroups of the dX product (what the grouped launch already puts on the chip): the dW split targets the rest.
int64_t dw_target(bool has_dx, int64_t T, int64_t in, int64_t out, bool f32 = false) {
  static int64_t tgt = -1;
  if (tgt < 0) {
    const char* e = tuning_env("ESGPT_GEMM_DW_TARGET");  // tuning hook: fixed dW item target (0 = the default rule)
    tgt = e ? std::max(0, atoi(e)) : 0;
  }
  if (tgt > 0) return tgt;
  const TileCfg xt = f32 ? TileCfg{1, 1} : dx_tile(T, in, out);
  return has_dx ? std::max<int64_t>(64, kTarget - n_tiles(T, in, xt)) : kTarget;
}

template <int FM, int FN>
void launch_fwd(const Prob& p, hipStream_t st) {
#ifdef ESGPT_TUNING_HOOKS
  if (esgpt::gk::launch_stream(p, true, st)) return;  // tools/lab/gemm_stream.hip (tools build only)
#endif
  const dim3 grid((unsigned)n_wg(p));
  static const int persist = [] {
    const char* e = tuning_env("ESGPT_GEMM_PERSIST");
    return e ? atoi(e) : 0;
  }();
  if (persist > 0 && FM == 1 && FN == 1) {
    const int nt = n_wg(p);
    const int g = std::min(nt, 256 * persist) & ~7;
    if (g >= 8 && nt % 8 == 0) {
      gemm_persist_kernel<true, true, 3, FM, FN, 1><<<dim3((unsigned)g), THREADS, 0, st>>>(p, nt);
      return;
    }
  }
  if (fwd_glds() == 2 && p.fast) {
    gemm_kernel<true, true, 3, FM, FN, 1, 2><<<grid, THREADS, 0, st>>>(p);
    return;
  }
#ifdef ESGPT_TUNING_HOOKS
  if (fwd_glds() == 3 && p.fast) {
    gemm_kernel<true, true, 3, FM, FN, 1, 3><<<grid, THREADS, 0, st>>>(p);
    return;
  }
#endif
  if (fwd_stages() == 2) gemm_kernel<true, true, 2, FM, FN><<<grid, THREADS, 0, st>>>(p);
#ifdef ESGPT_TUNING_HOOKS
  else if (fwd_stages() == 4) gemm_kernel<true, true, 4, FM, FN, 1><<<grid, THREADS, 0, st>>>(p);
  else if (fwd_stages() == 5) gemm_kernel<true, true, 5, FM, FN, 1><<<grid, THREADS, 0, st>>>(p);
#endif
  else if (fwd_buffers() == 1) gemm_kernel<true, true, 3, FM, FN, 1><<<grid, THREADS, 0, st>>>(p);
  else gemm_kernel<true, true, 3, FM, FN><<<grid, THREADS, 0, st>>>(p);
}

template <int XM, int XN, int NBG>
void launch_pair_g(const Prob& p0, const Prob& p1, hipStream_t st) {
  const dim3 grid((unsigned)(n_wg(p0) + n_wg(p1)));
  if (p1.fm == 2) gemm_bwd_pair_kernel<XM, XN, 2, 2, NBG><<<grid, THREADS, 0, st>>>(p0, p1);
  else gemm_bwd_pair_kernel<XM, XN, 1, 1, NBG><<<grid, THREADS, 0, st>>>(p0, p1);
}
template <int XM, int XN>
void launch_pair_x(const Prob& p0, const Prob& p1, hipStream_t st) {
  switch (p0.fast && p1.fast ? bwd_glds() : 0) {
#ifdef ESGPT_TUNING_HOOKS
    case 2: launch_pair_g<XM, XN, 2>(p0, p1, st); break;
    case 3: launch_pair_g<XM, XN, 3>(p0, p1, st); break;
#endif
    default: launch_pair_g<XM, XN, 0>(p0, p1, st); break;
  }
}

void launch_pair(const Prob& p0, const Prob& p1, hipStream_t st) {
  switch (p0.fm * 10 + p0.fn) {
    case 21: launch_pair_x<2, 1>(p0, p1, st); break;
    case 22: launch_pair_x<2, 2>(p0, p1, st); break;
    default: launch_pair_x<1, 1>(p0, p1, st); break;
  }
}

template <int XM, int XN>
void launch_dx_only(const Prob& p0, hipStream_t st) {
  gemm_kernel<true, false, bwd_stages<XM, XN>(), XM, XN><<<dim3((unsigned)n_wg(p0)), THREADS, 0, st>>>(p0);
}

// The backward of one projection. st_dw == nullptr: dX and dW (+ db) in ONE grouped launch on st. Otherwise
// split: dX on st, dW (+ db, its split-K workspace and counters) on st_dw after it waits for the work queued on st
// so far — the weight gradient leaves the critical path of backward and runs beside the next layers' kernels. Both
// forms use the same tiles and split plan (the dW target counts the dX tiles either way): bitwise equal results.
// f32: every operand and dx in f32 (the reference-precision step), 64x64 f32-MFMA tiles.
int linear_bwd_impl(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T, int64_t in,
                    int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre, void* dx, int64_t lddx,
                    float* dw, float* db, void* workspace, size_t workspace_bytes, int32_t* counters,
                    const float* db_extra, int64_t n_extra, hipStream_t st, hipStream_t st_dw, bool f32 = false) {
  ESGPT_REQUIRE(T >= 0 && in >= 0 && out >= 0);
  ESGPT_REQUIRE(n_extra >= 0 && n_extra < (1 << 20) &&
                (n_extra == 0 || (db_extra != nullptr && db != nullptr && T > 0)));
  if (in == 0 || out == 0) return ESGPT_OK;
  ESGPT_REQUIRE(dw != nullptr);
  const bool has_dx = dx != nullptr;
  hipStream_t sw = st_dw ? st_dw : st;
  if (st_dw && esgpt_stream_wait(st_dw, st) != ESGPT_OK) return ESGPT_ERR_LAUNCH;
  if (T == 0) {  // empty batch (the operands may be empty allocations): zero weight / bias gradients
    if (zero_async(dw, sizeof(float) * out * in, sw) != hipSuccess) return ESGPT_ERR_LAUNCH;
    if (db && zero_async(db, sizeof(float) * out, sw) != hipSuccess) return ESGPT_ERR_LAUNCH;
    return ESGPT_OK;
  }
  if (f32) {
    ESGPT_REQUIRE(shapes_ok_f32(false, false, dy, lddy, x, ldx, out, in, T, dw, in));
    if (has_dx) ESGPT_REQUIRE(shapes_ok_f32(true, false, dy, lddy, w, in, T, in, out, dx, lddx));
    ESGPT_REQUIRE(act < 0 || (pre != nullptr && act_ok(act) && has_dx && ldpre % 4 == 0 && ((uintptr_t)pre % 16) == 0));
  } else {
    ESGPT_REQUIRE(shapes_ok(false, false, dy, lddy, x, ldx, out, in, T, dw, in, true));
    if (has_dx) ESGPT_REQUIRE(shapes_ok(true, false, dy, lddy, w, in, T, in, out, dx, lddx, false));
    ESGPT_REQUIRE(act < 0 || (pre != nullptr && act_ok(act) && has_dx && ldpre % 4 == 0 && ((uintptr_t)pre % 8) == 0));
  }
#ifdef ESGPT_TUNING_HOOKS
  // tools build (ESGPT_GEMM_BIG): wide products: dX and dW (+ db) on the large-tile kernel, each its own launch (+ dW's slab reduction)
  if (!f32 && !st_dw && big_cols(T, in, out)) {
    const BigDw plan_w = big_dw_plan(T, in, out);
    ESGPT_REQUIRE(workspace && workspace_bytes >= plan_w.slab_bytes && plan_w.slab_bytes < (1ull << 31));
    Prob pw = make_prob(dy, lddy, x, ldx, out, in, T, dw, in, 1, 0, nullptr, alpha, 0, TileCfg{4, 4});
    pw.rowsum = db;
    pw.rs_extra = n_extra ? db_extra : nullptr;
    pw.rs_extra_n = (int)n_extra;
    pw.slab = reinterpret_cast<float*>(workspace);
    if (has_dx) {
      Prob px = make_prob(dy, lddy, w, in, T, in, out, dx, lddx, 0, 0, nullptr, alpha, 0, TileCfg{4, 4});
      if (act >= 0) {
        px.epi = EPI_ACT_GRAD;
        px.act = act;
        px.aux = reinterpret_cast<const __bf16*>(pre);
        px.ld_aux = ldpre;
      }
      if (px.fast && pw.fast && g_row_tiles == nullptr) {
        launch_big(px, true, false, big_cols(T, in, out), st);
        launch_big_dw(pw, st);
        ESGPT_LAUNCH_CHECK();
        return ESGPT_OK;
      }
    } else if (pw.fast) {
      launch_big_dw(pw, st);
      ESGPT_LAUNCH_CHECK();
      return ESGPT_OK;
    }
    return ESGPT_ERR_UNSUPPORTED;  // operands past 2 GiB or a row-tile mask: not for these shapes
  }
#endif
  Prob p0{};
  if (has_dx) {
    p0 = make_prob(dy, lddy, w, in, T, in, out, dx, lddx, f32 ? 1 : 0, 0, nullptr, alpha, 0,
                   f32 ? TileCfg{1, 1} : dx_tile(T, in, out));
    p0.row_tiles = g_row_tiles;  // dX rows are token rows (dW's M is the output feature: never masked)
    if (act >= 0) {
      p0.epi = EPI_ACT_GRAD;
      p0.act = act;
      p0.aux = reinterpret_cast<const __bf16*>(pre);
      p0.ld_aux = ldpre;
    }
  }
  const TileCfg wc = f32 ? TileCfg{1, 1} : dw_tile(T, in, out);
  Prob p1 = make_prob(dy, lddy, x, ldx, out, in, T, dw, in, 1, 0, nullptr, alpha, dw_target(has_dx, T, in, out, f32),
                      wc);
  p1.rowsum = db;
  p1.rs_extra = n_extra ? db_extra : nullptr;
  p1.rs_extra_n = (int)n_extra;
  if (p1.splits > 1) {
    p1.ext_reduce = p1.splits > in_launch_splits();
    ESGPT_REQUIRE(workspace && workspace_bytes >= slab_bytes(p1.splits, out, in, wc) &&
                  (p1.ext_reduce || counters));
    ESGPT_REQUIRE(slab_bytes(p1.splits, out, in, wc) < (1ull << 31));  // 32-bit buffer offsets
    p1.slab = reinterpret_cast<float*>(workspace);
    p1.counters = counters;
  }
  if (const char* e = tuning_env("ESGPT_GEMM_DBG")) p0.dbg = p1.dbg = atoi(e);
  if (has_dx && !st_dw) {
    p0.wg0 = n_wg(p1);
    // split-major XCD order when the token chunks line up: every dW split a full chunk, splits a multiple of the 8
    // XCDs, each chunk a whole number of dX row blocks
    const int bm_dx = 64 * p0.fm;
    if (p1.splits % 8 == 0 && (int64_t)p1.splits * p1.kchunk == T && p1.kchunk % bm_dx == 0 && p0.splits == 1 &&
        p0.tm * bm_dx == T) {
      p1.xmap = 1;
      p0.xmap = 2;
      p0.rps = p1.kchunk / bm_dx;
    }
    if (f32)
      gemm_bwd_pair_kernel<1, 1, 1, 1, 0, true><<<dim3((unsigned)(n_wg(p0) + n_wg(p1))), THREADS, 0, st>>>(p0, p1);
    else
      launch_pair(p0, p1, st);
  } else if (f32) {
    if (has_dx) gemm_kernel<true, false, NS, 1, 1, 2, 0, true><<<dim3((unsigned)n_wg(p0)), THREADS, 0, st>>>(p0);
    gemm_kernel<false, false, NS, 1, 1, 2, 0, true><<<dim3((unsigned)n_wg(p1)), THREADS, 0, sw>>>(p1);
  } else {
    if (has_dx) {
      switch (p0.fm * 10 + p0.fn) {
        case 21: launch_dx_only<2, 1>(p0, st); break;
        case 22: launch_dx_only<2, 2>(p0, st); break;
        default: launch_dx_only<1, 1>(p0, st); break;
      }
    }
    if (wc.fm == 2)
      gemm_kernel<false, false, bwd_stages<2, 2>(), 2, 2><<<dim3((unsigned)n_wg(p1)), THREADS, 0, sw>>>(p1);
    else
      gemm_kernel<false, false, NS, 1, 1><<<dim3((unsigned)n_wg(p1)), THREADS, 0, sw>>>(p1);
  }
  if (p1.ext_reduce) launch_slab_reduce(p1, sw);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // namespace

extern "C" {

int esgpt_gemm_row_tiles(const uint8_t* tiles) {
  static int use = -1;  // tools build: ESGPT_ROW_TILES_IGNORE=1 drops the mask (A/B of the in-kernel check)
  if (use < 0) {
    const char* e = tuning_env("ESGPT_ROW_TILES_IGNORE");
    use = (e && e[0] == '1') ? 0 : 1;
  }
  g_row_tiles = use ? tiles : nullptr;
  return ESGPT_OK;
}

size_t esgpt_gemm_workspace(int64_t M, int64_t N, int64_t K) {
  return slab_bytes(plan(M, N, K, kTarget, TileCfg{1, 1}).splits, M, N, TileCfg{1, 1});
}

int64_t esgpt_gemm_counters(int64_t M, int64_t N) { return cdiv(M, 64) * cdiv(N, 64); }

int esgpt_gemm_bf16(int a_layout, const void* A, int64_t lda, int b_layout, const void* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, const float* alpha, void* C, int64_t ldc, int c_dtype,
                    int accumulate, void* workspace, size_t workspace_bytes, int32_t* counters, void* stream) {
  ESGPT_REQUIRE(c_dtype == ESGPT_F32 || (c_dtype == ESGPT_BF16 && !accumulate));
  const bool akc = a_layout == ESGPT_GEMM_K_CONTIG, bkc = b_layout == ESGPT_GEMM_K_CONTIG;
  ESGPT_REQUIRE(akc || a_layout == ESGPT_GEMM_MN_CONTIG);
  ESGPT_REQUIRE(bkc || b_layout == ESGPT_GEMM_MN_CONTIG);
  const bool f32 = c_dtype == ESGPT_F32;
  ESGPT_REQUIRE(shapes_ok(akc, bkc, A, lda, B, ldb, M, N, K, C, ldc, f32));
  ESGPT_REQUIRE(bias == nullptr || ((uintptr_t)bias % 16) == 0);
  if (M == 0 || N == 0) return ESGPT_OK;
  // the forward projections (K-contig x K-contig, bf16 out, no split): the forward kernel configuration of
  // esgpt_linear_fwd (tile / stages / LDS buffers)
  const bool fwd_form = akc && bkc && !f32 && !accumulate && alpha == nullptr;
  const TileCfg tc = fwd_form ? fwd_tile(M, N, K, false) : TileCfg{1, 1};
  Prob p = make_prob(A, lda, B, ldb, M, N, K, C, ldc, f32 ? 1 : 0, accumulate, bias, alpha, kTarget, tc);
  p.row_tiles = g_row_tiles;
  // bf16-output products with A K-contiguous (the forward and input-gradient forms) on the large-tile kernel, which
  // never splits K
  const int big = akc && !f32 && !accumulate ? (bkc ? big_fwd_cols(M, N, K, false) : big_cols(M, N, K)) : 0;
  if (big) {
    Prob q = make_prob(A, lda, B, ldb, M, N, K, C, ldc, 0, 0, bias, alpha, 0, tc);
    q.row_tiles = g_row_tiles;
    if (launch_big(q, true, bkc, big, as_stream(stream))) {
      ESGPT_LAUNCH_CHECK();
      return ESGPT_OK;
    }
  }
  if (fwd_form && p.splits == 1) {
    if (const char* e = tuning_env("ESGPT_GEMM_DBG")) p.dbg = atoi(e);
    hipStream_t st = as_stream(stream);
    switch (tc.fm * 10 + tc.fn) {
      case 21: launch_fwd<2, 1>(p, st); break;
      case 12: launch_fwd<1, 2>(p, st); break;
      case 22: launch_fwd<2, 2>(p, st); break;
      default: launch_fwd<1, 1>(p, st); break;
    }
    ESGPT_LAUNCH_CHECK();
    return ESGPT_OK;
  }
  if (tc.fm != 1 || tc.fn != 1) p = make_prob(A, lda, B, ldb, M, N, K, C, ldc, 0, accumulate, bias, alpha, kTarget,
                                                TileCfg{1, 1});
  p.row_tiles = g_row_tiles;
  if (p.splits > 1) {
    p.ext_reduce = f32 && p.splits > in_launch_splits();
    ESGPT_REQUIRE(workspace && workspace_bytes >= slab_bytes(p.splits, M, N, tc) && (p.ext_reduce || counters));
    ESGPT_REQUIRE(slab_bytes(p.splits, M, N, tc) < (1ull << 31));  // 32-bit buffer offsets
    p.slab = reinterpret_cast<float*>(workspace);
    p.counters = counters;
  }
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)n_wg(p));
  if (akc && bkc) gemm_kernel<true, true, NS, 1, 1><<<grid, THREADS, 0, st>>>(p);
  else if (akc) gemm_kernel<true, false, NS, 1, 1><<<grid, THREADS, 0, st>>>(p);
  else if (bkc) gemm_kernel<false, true, NS, 1, 1><<<grid, THREADS, 0, st>>>(p);
  else gemm_kernel<false, false, NS, 1, 1><<<grid, THREADS, 0, st>>>(p);
  if (p.ext_reduce) launch_slab_reduce(p, st);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_linear_fwd(const void* x, int64_t ldx, const void* w, int64_t T, int64_t in, int64_t out,
                     const float* bias, int act, void* pre, void* y, int64_t ldy, void* stream) {
  ESGPT_REQUIRE(shapes_ok(true, true, x, ldx, w, in, T, out, in, y, ldy, false));
  ESGPT_REQUIRE(act < 0 || (pre != nullptr && act_ok(act)));
  ESGPT_REQUIRE(bias == nullptr || ((uintptr_t)bias % 16) == 0);
  ESGPT_REQUIRE(pre == nullptr || ((uintptr_t)pre % 16) == 0);
  if (T == 0 || out == 0) return ESGPT_OK;
  const TileCfg tc = fwd_tile(T, out, in, act >= 0);
  Prob p = make_prob(x, ldx, w, in, T, out, in, y, ldy, 0, 0, bias, nullptr, 0, tc);  // never split
  p.row_tiles = g_row_tiles;
  if (act >= 0) {
    p.epi = EPI_BIAS_ACT;
    p.act = act;
    p.aux_out = reinterpret_cast<__bf16*>(pre);
    p.ld_aux = ldy;
  }
  if (const char* e = tuning_env("ESGPT_GEMM_DBG")) p.dbg = atoi(e);
  hipStream_t st = as_stream(stream);
  if (const int bn = big_fwd_cols(T, out, in, act >= 0))
    if (launch_big(p, true, true, bn, st)) {
      ESGPT_LAUNCH_CHECK();
      return ESGPT_OK;
    }
  switch (tc.fm * 10 + tc.fn) {
    case 21: launch_fwd<2, 1>(p, st); break;
    case 12: launch_fwd<1, 2>(p, st); break;
    case 22: launch_fwd<2, 2>(p, st); break;
    default: launch_fwd<1, 1>(p, st); break;
  }
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

size_t esgpt_linear_bwd_workspace(int64_t T, int64_t in, int64_t out, int has_dx) {
  const TileCfg wc = dw_tile(T, in, out);
  const size_t tile = slab_bytes(plan(out, in, T, dw_target(has_dx != 0, T, in, out), wc).splits, out, in, wc);
  // (tools build, ESGPT_GEMM_BIG: the large-tile dW's split-K slabs; the split-stream form takes the tile kernel)
#ifdef ESGPT_TUNING_HOOKS
  return big_cols(T, in, out) ? std::max(tile, big_dw_plan(T, in, out).slab_bytes) : tile;
#else
  return tile;
#endif
}

int esgpt_linear_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T, int64_t in,
                     int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre, void* dx,
                     int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes, int32_t* counters,
                     void* stream) {
  return esgpt_linear_bwd_ex(dy, lddy, x, ldx, w, T, in, out, alpha, act, pre, ldpre, dx, lddx, dw, db, workspace,
                             workspace_bytes, counters, nullptr, 0, stream);
}

int esgpt_linear_bwd_ex(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T,
                        int64_t in, int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre,
                        void* dx, int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                        int32_t* counters, const float* db_extra, int64_t n_extra, void* stream) {
  return linear_bwd_impl(dy, lddy, x, ldx, w, T, in, out, alpha, act, pre, ldpre, dx, lddx, dw, db, workspace,
                         workspace_bytes, counters, db_extra, n_extra, as_stream(stream), nullptr);
}

size_t esgpt_linear_bwd_f32_workspace(int64_t T, int64_t in, int64_t out, int has_dx) {
  return slab_bytes(plan(out, in, T, dw_target(has_dx != 0, T, in, out, true), TileCfg{1, 1}).splits, out, in,
                    TileCfg{1, 1});
}

int esgpt_linear_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* w, int64_t T,
                         int64_t in, int64_t out, const float* alpha, int act, const float* pre, int64_t ldpre,
                         float* dx, int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                         int32_t* counters, const float* db_extra, int64_t n_extra, void* stream) {
  return linear_bwd_impl(dy, lddy, x, ldx, w, T, in, out, alpha, act, pre, ldpre, dx, lddx, dw, db, workspace,
                         workspace_bytes, counters, db_extra, n_extra, as_stream(stream), nullptr, true);
}

int esgpt_linear_fwd_f32(const float* x, int64_t ldx, const float* w, int64_t T, int64_t in, int64_t out,
                         const float* bias, int act, float* pre, float* y, int64_t ldy, void* stream) {
  ESGPT_REQUIRE(shapes_ok_f32(true, true, x, ldx, w, in, T, out, in, y, ldy));
  ESGPT_REQUIRE(act < 0 || (pre != nullptr && act_ok(act)));
  ESGPT_REQUIRE(bias == nullptr || ((uintptr_t)bias % 16) == 0);
  ESGPT_REQUIRE(pre == nullptr || ((uintptr_t)pre % 16) == 0);
  if (T == 0 || out == 0) return ESGPT_OK;
  Prob p = make_prob(x, ldx, w, in, T, out, in, y, ldy, 1, 0, bias, nullptr, 0, TileCfg{1, 1});  // never split
  p.row_tiles = g_row_tiles;
  if (act >= 0) {
    p.epi = EPI_BIAS_ACT;
    p.act = act;
    p.aux_out = reinterpret_cast<__bf16*>(pre);
    p.ld_aux = ldy;
  }
  gemm_kernel<true, true, NS, 1, 1, 2, 0, true><<<dim3((unsigned)n_wg(p)), THREADS, 0, as_stream(stream)>>>(p);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_gemm_f32(int a_layout, const float* A, int64_t lda, int b_layout, const float* B, int64_t ldb, int64_t M,
                   int64_t N, int64_t K, const float* bias, const float* alpha, float* C, int64_t ldc, int accumulate,
                   void* workspace, size_t workspace_bytes, int32_t* counters, void* stream) {
  const bool akc = a_layout == ESGPT_GEMM_K_CONTIG, bkc = b_layout == ESGPT_GEMM_K_CONTIG;
  ESGPT_REQUIRE(akc || a_layout == ESGPT_GEMM_MN_CONTIG);
  ESGPT_REQUIRE(bkc || b_layout == ESGPT_GEMM_MN_CONTIG);
  ESGPT_REQUIRE(shapes_ok_f32(akc, bkc, A, lda, B, ldb, M, N, K, C, ldc));
  ESGPT_REQUIRE(bias == nullptr || ((uintptr_t)bias % 16) == 0);
  if (M == 0 || N == 0) return ESGPT_OK;
  Prob p = make_prob(A, lda, B, ldb, M, N, K, C, ldc, 1, accumulate, bias, alpha, kTarget, TileCfg{1, 1});
  p.row_tiles = g_row_tiles;
  if (p.splits > 1) {
    p.ext_reduce = p.splits > in_launch_splits();
    ESGPT_REQUIRE(workspace && workspace_bytes >= slab_bytes(p.splits, M, N, TileCfg{1, 1}) &&
                  (p.ext_reduce || counters));
    ESGPT_REQUIRE(slab_bytes(p.splits, M, N, TileCfg{1, 1}) < (1ull << 31));
    p.slab = reinterpret_cast<float*>(workspace);
    p.counters = counters;
  }
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)n_wg(p));
  if (akc && bkc) gemm_kernel<true, true, NS, 1, 1, 2, 0, true><<<grid, THREADS, 0, st>>>(p);
  else if (akc) gemm_kernel<true, false, NS, 1, 1, 2, 0, true><<<grid, THREADS, 0, st>>>(p);
  else if (bkc) gemm_kernel<false, true, NS, 1, 1, 2, 0, true><<<grid, THREADS, 0, st>>>(p);
  else gemm_kernel<false, false, NS, 1, 1, 2, 0, true><<<grid, THREADS, 0, st>>>(p);
  if (p.ext_reduce) launch_slab_reduce(p, st);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_linear_bwd_split(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T,
                           int64_t in, int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre,
                           void* dx, int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                           int32_t* counters, const float* db_extra, int64_t n_extra, void* stream,
                           void* stream_dw) {
  ESGPT_REQUIRE(stream_dw != nullptr && stream_dw != stream);
  return linear_bwd_impl(dy, lddy, x, ldx, w, T, in, out, alpha, act, pre, ldpre, dx, lddx, dw, db, workspace,
                         workspace_bytes, counters, db_extra, n_extra, as_stream(stream), as_stream(stream_dw));
}

}  // extern "C"
