// Large-tile bf16 MFMA GEMM for the wide projections (transformer.py:133-163, 378-391 at d >= 512: C3's q/k/v,
// out_proj, c_fc, c_proj and their input gradients; the tile GEMM of gemm.hip keeps the narrow C2 shapes).
//
//   C[M, N] = alpha · A · B (+ bias[n]) (+ epilogue),   bf16 operands, f32 accumulation, C bf16.
//
// Why a second kernel: the 64x64 / 128x128 tiles of gemm.hip re-read every operand row through L2 once per output
// tile column and run 4 waves of 1-4 fragments each, so at M = 16,384, K = 512-2,048 the k-loop is bound by operand
// staging, not by the matrix cores (0.17 of the bf16 peak). Here one 512-thread workgroup (8 waves,
// one per CU: two waves per SIMD) owns a 256 x BN output tile:
//   * waves as 2 (M) x 4 (N) for BN = 256 (each 128 x 64: 4 x 2 accumulators of v_mfma_f32_32x32x16_bf16 = 128
//     accumulator registers), 4 x 2 for BN = 128 (64 x 64: 2 x 2);
//   * operands staged by LDS-DMA (buffer_load ... lds, 16 B per lane straight into LDS, no VGPR round trip) in a
//     ring of NSLOT stages of 32 k each (A 256 x 32 + B BN x 32 bf16); NSLOT - 2 stages stay in flight while one is
//     consumed — counted vmcnt waits and raw s_barrier (a __syncthreads() would drain every DMA in flight,
//     cdna_hip_programming.md §5 "Pipelining across barriers");
//   * fragment reads as inline ds_read_b128 (K-contiguous images) / ds_read_b64_tr_b16 (M/N-contiguous images:
//     hardware transpose) with counted lgkmcnt waits: the next k-step's fragments are read under the current MFMAs;
//   * XOR-swizzled images (the swizzle applied to each lane's DMA SOURCE address, the destination stays
//     lane-linear: rule 21) so both fragment reads are bank-conflict free:
//       K-contig [R rows][32 k], 64-B rows:  16-B chunk c of row q at c ^ ((q >> 2) & 3)
//       M/N-contig [32 k-rows][R cols]:       16-B chunk c of k-row q at c ^ (4 (q & 3));
//   * XCD-aware tile order (each XCD walks a contiguous run: the A row blocks and B column blocks of a run share an
//     L2);
//   * the epilogue (alpha, bias, activation with its pre-activation output, or the activation gradient of c_proj's
//     input gradient) through LDS: fragment-order writes, then row-major 16-B stores covering whole 128-B lines.
// The swapped-operand MFMA form makes each lane own one output ROW (its registers hold 4 consecutive columns per
// register group), as in gemm.hip.
#include <algorithm>
#include <cstdio>

#include "common.h"
#include "gemm_parts.h"

using namespace esgpt;
using namespace esgpt::gk;

namespace {

constexpr int SK = 32;  // k per stage

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ bf16x8 ds_b128(const __bf16* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ u32x2 ds_tr(const __bf16* p) {
  u32x2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
// s_waitcnt lgkmcnt(N) (vmcnt / expcnt left at their maxima), then a scheduling fence: the MFMAs that read the
// waited registers must not be hoisted above it (cdna_hip_programming.md rule 18)
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt((N << 8) | (7 << 4) | 0xF | (3 << 14));
  __builtin_amdgcn_sched_barrier(0);
}

// One operand's stage image: R rows (m or n) x SK k, filled by LDS-DMA (NWV waves).
template <bool KC, int R, int NWV>
struct BTile {
  static constexpr int kElems = R * SK;
  static constexpr int kInstr = kElems * 2 / 1024 / NWV;  // 1-KiB DMA instructions per wave and stage
  static constexpr int CPR = KC ? SK / 8 : R / 8;       // 16-B chunks per image row
  static constexpr int RPI = 64 / CPR;                  // image rows per instruction
  static constexpr int kReads = KC ? 1 : 2;             // LDS read instructions per fragment
  static_assert(kInstr >= 1 && kInstr * NWV * 512 == kElems, "tile rows");
  static constexpr int kOOB = (int)0x80000000u;

  __device__ __forceinline__ static int sw(int row) { return KC ? ((row >> 2) & 3) : 4 * (row & 3); }
  __device__ __forceinline__ static int off(int row, int col) {  // element offset, col % 4 == 0
    return row * (KC ? SK : R) + (((col >> 3) ^ sw(row)) << 3) + (col & 7);
  }
  __device__ __forceinline__ static void coords(int i, int& row, int& lg) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    row = (wave + NWV * i) * RPI + lane / CPR;
    lg = (lane % CPR) ^ sw(row);
  }
  // per-lane source byte offsets (row0 = the tile's first m / n, nrows = the operand's m / n extent); rows / columns
  // past the extent read zeros (offset past the buffer's range)
  __device__ __forceinline__ static void lane_src(int (&vo)[kInstr], int64_t ld, int row0, int nrows) {
#pragma unroll
    for (int i = 0; i < kInstr; ++i) {
      int row, lg;
      coords(i, row, lg);
      if (KC) vo[i] = row0 + row < nrows ? (int)(((int64_t)(row0 + row) * ld + lg * 8) * 2) : kOOB;
      else vo[i] = row0 + lg * 8 < nrows ? (int)(((int64_t)row * ld + row0 + lg * 8) * 2) : kOOB;
    }
  }
  __device__ __forceinline__ static int soff(int k0, int64_t ld) { return KC ? k0 * 2 : (int)(k0 * ld * 2); }
  // one stage into img; kvalid < SK: the last, partial stage (its pieces past kvalid read zeros)
  __device__ __forceinline__ static void issue(__amdgpu_buffer_rsrc_t rs, const int (&vo)[kInstr], int so,
                                               __bf16* img, int kvalid) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kInstr; ++i) {
      int v = vo[i];
      if (kvalid < SK) {
        int row, lg;
        coords(i, row, lg);
        if ((KC ? lg * 8 : row) >= kvalid) v = kOOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wave + NWV * i) * 512), 16, v, so, 0, 0);
    }
  }
  // MFMA operand fragment of rows sub0 .. sub0 + 31, k-step t (k = 16t .. 16t + 15): lane (r, h) gets row sub0 + r,
  // k = 16t + 8h + j
  __device__ __forceinline__ static bf16x8 frag(const __bf16* s, int sub0, int t) {
    const int l = threadIdx.x & 63;
    if (KC) {
      return ds_b128(s + off(sub0 + (l & 31), 16 * t + 8 * (l >> 5)));
    } else {
      // ds_read_b64_tr_b16: in each 16-lane group lane 4q + p addresses k-row (base + q), columns 4p .. 4p + 3;
      // lane i of the group receives column i of the 4 rows
      const int g = l >> 4, w = l & 15, q = w >> 2, p = w & 3;
      const int col = sub0 + (g & 1) * 16 + 4 * p;
      const int kr = 16 * t + 8 * (g >> 1) + q;
      const u32x2 lo = ds_tr(s + off(kr, col)), hi = ds_tr(s + off(kr + 4, col));
      const u32x4 f = {lo[0], lo[1], hi[0], hi[1]};
      return __builtin_bit_cast(bf16x8, f);
    }
  }
};

// Tile order: consecutive tile ids (one XCD's contiguous run, xcd_remap) walk groups of kGroupM row blocks column
// by column, so the ~32 tiles an XCD works on at once span about kGroupM row blocks x 32 / kGroupM column blocks:
// per 32-k stage the XCD's L2 takes in both operands' slices of those blocks instead of one row block and every
// column block (the whole B operand per row block, re-streamed from beyond L2 by every XCD).
constexpr int kGroupM = 8;
__device__ __forceinline__ void group_tile(int t, int tm, int tn, int& by, int& bx) {
  const int per = kGroupM * tn, g = t / per, first = g * kGroupM, gs = min(tm - first, kGroupM);
  const int in = t - g * per;
  by = first + in % gs;
  bx = in / gs;
}

// Tile TM x BN on NWV waves (8: two per SIMD, one workgroup per CU; 4: one per SIMD, 2-3 workgroups per CU). Wave
// grid WM x WN: 8 waves as 2 x 4 (4 x 2 for the 256 x 128 tile), 4 waves as 2 x 2.
template <bool AKC, bool BKC, int TM, int BN, int NWV, int NSLOT>
struct BigCfg {
  static constexpr int BT = 64 * NWV;
  using TA = BTile<AKC, TM, NWV>;
  using TB = BTile<BKC, BN, NWV>;
  static constexpr int WN = NWV == 8 ? ((TM == 256 && BN == 128) ? 2 : 4) : 2, WM = NWV / WN;  // wave grid
  static constexpr int FM = TM / 32 / WM, FN = BN / 32 / WN;  // fragments per wave
  static_assert(FM >= 1 && FN >= 1 && FM * 32 * WM == TM && FN * 32 * WN == BN, "wave grid");
  static constexpr int STAGE = TA::kElems + TB::kElems;         // bf16 elements per ring slot
  static constexpr int P = TA::kInstr + TB::kInstr;             // DMA instructions per wave and stage
  static constexpr int RING = NSLOT * STAGE;
  static constexpr int EPI = (TM > 128 ? 128 : TM) * (BN + 4) * 2;  // bf16 elements of an f32 C tile (half)
  static constexpr int LDS = RING > EPI ? RING : EPI;           // bf16 elements
  static constexpr int NR = FM * TA::kReads + FN * TB::kReads;  // LDS read instructions per k-step
  static_assert(NSLOT >= 3 && NSLOT <= 6 && (NSLOT - 1) * P < 64, "ring");
  static_assert(NR < 16, "lgkmcnt");
};

// DW: the weight-gradient form (A and B M/N-contiguous, K = tokens split over p.splits workgroups of p.kchunk
// tokens each): the f32 partial tile goes to a slab in fragment order (every wave-instruction a contiguous 1 KiB)
// and the bias gradient's row sums (one extra MFMA against a ones operand per k-step, spread over the waves of the
// tile's first column block) to the row-sum slab; big_slab_reduce_kernel sums the slabs.
template <bool AKC, bool BKC, int TM, int BN, int NWV, int NSLOT, bool DW = false>
__global__ __launch_bounds__(64 * NWV) void gemm_big_kernel(Prob p) {
  using C = BigCfg<AKC, BKC, TM, BN, NWV, NSLOT>;
  constexpr int BT = C::BT;
  using TA = typename C::TA;
  using TB = typename C::TB;
  constexpr int FM = C::FM, FN = C::FN, WN = C::WN, P = C::P, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(16))) __bf16 smem[C::LDS];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int bz = DW ? lin % p.splits : 0, tile = DW ? lin / p.splits : lin;
  int bx, by;
  group_tile(tile, p.tm, p.tn, by, bx);
  const int M = p.M, N = p.N;
  const int m0 = by * TM, n0 = bx * BN;
  const int kb = DW ? bz * p.kchunk : 0, ke = DW ? min(p.K, kb + p.kchunk) : p.K;
  const int ns = ke > kb ? (ke - kb + SK - 1) / SK : 0;
  const bool want_rs = DW && p.rowsum != nullptr && bx == 0;  // workgroup-uniform

  static_assert(!DW || FM <= WN, "row sums: at most one fragment row per wave");
  f32x16 acc[FM][FN], racc;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    racc[e] = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j][e] = 0.f;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;

  int voA[TA::kInstr], voB[TB::kInstr];
  TA::lane_src(voA, p.lda, m0, M);
  TB::lane_src(voB, p.ldb, n0, N);
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(p.A), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(p.B), (short)0, 0x7fffffff, 0x00020000);
  auto issue = [&](int s) {
    const int k0 = kb + s * SK, kv = ke - k0;
    __bf16* img = smem + (s % NSLOT) * STAGE;
    TA::issue(rsA, voA, TA::soff(k0, p.lda), img, kv);
    TB::issue(rsB, voB, TB::soff(k0, p.ldb), img + TA::kElems, kv);
  };

  // Ring schedule (NSLOT slots, one stage of 32 k each; stage s in slot s % NSLOT):
  //   prologue: issue stages 0 .. NSLOT-1; wait for stage 0; barrier; read k-step 0 of stage 0
  //   stage i:  MFMAs of k-step 0 | read k-step 1, wait for it | wait for stage i+1's DMA (NSLOT-2 younger stages
  //             stay in flight); barrier; issue stage i+NSLOT into the slot of stage i (every wave has finished
  //             reading it); read k-step 0 of stage i+1 | MFMAs of k-step 1 — the barrier, the DMA issue and the
  //             next stage's first reads are covered by the MFMAs in flight on either side.
  auto wait_younger = [&](int younger) {  // stage s has landed once at most `younger` younger stages are outstanding
    if (NSLOT >= 6 && younger >= 5) vm_wait<(NSLOT >= 6 ? 5 * P : 0)>();
    else if (NSLOT >= 5 && younger >= 4) vm_wait<(NSLOT >= 5 ? 4 * P : 0)>();
    else if (younger >= 3) vm_wait<3 * P>();
    else if (younger == 2) vm_wait<2 * P>();
    else if (younger == 1) vm_wait<P>();
    else vm_wait<0>();
  };
  bf16x8 af0[FM], bf0[FN], af1[FM], bf1[FN];
  auto read = [&](const __bf16* sA, int t, bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
    for (int a = 0; a < FM; ++a) af[a] = TA::frag(sA, wm * 32 * FM + 32 * a, t);
#pragma unroll
    for (int b = 0; b < FN; ++b) bfr[b] = TB::frag(sA + TA::kElems, wn * 32 * FN + 32 * b, t);
  };
  auto mainloop = [&](auto rs_c) {
    constexpr bool RS = decltype(rs_c)::value;
    auto mma = [&](const bf16x8 (&af)[FM], const bf16x8 (&bfr)[FN]) {
#pragma unroll
      for (int a = 0; a < FM; ++a) {
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = mfma(bfr[b], af[a], acc[a][b]);
        if constexpr (RS)
          if (a == wn) racc = mfma(ones, af[a], racc);  // wave-uniform: fragment row a on wave column a
      }
    };
    const int pro = min(NSLOT, ns);
#pragma unroll
    for (int s = 0; s < NSLOT; ++s)
      if (s < ns) issue(s);
    wait_younger(pro - 1);
    __builtin_amdgcn_s_barrier();
    read(smem, 0, af0, bf0);
    for (int i = 0; i < ns; ++i) {
      const __bf16* sA = smem + (i % NSLOT) * STAGE;
      lgkm_wait<0>();
      mma(af0, bf0);
      read(sA, 1, af1, bf1);
      lgkm_wait<0>();
      if (i + 1 < ns) {
        wait_younger(min(NSLOT - 2, ns - 2 - i));
        __builtin_amdgcn_s_barrier();
        if (i + NSLOT < ns) issue(i + NSLOT);
        read(smem + ((i + 1) % NSLOT) * STAGE, 0, af0, bf0);
      }
      mma(af1, bf1);
    }
  };
  if (want_rs) mainloop(std::true_type{});
  else mainloop(std::false_type{});
  if constexpr (DW) {
    // f32 partial tile -> slab (fragment order: split, tile, wave, fragment, register group, lane; plain stores:
    // the kernel boundary orders them before big_slab_reduce_kernel); row sums -> [splits][M]
    const int ntile = p.tm * p.tn;
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int64_t idx = 4 * (((((int64_t)bz * ntile + tile) * NWV + wave) * (FM * FN) + a * FN + b) * 4 + g) * 64 +
                              4 * lane;
          *reinterpret_cast<float4*>(p.slab + idx) =
              make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2], acc[a][b][4 * g + 3]);
        }
    if (want_rs && h == 0 && wn < FM) {  // fragment row a = wn
      const int row = m0 + wm * 32 * FM + 32 * wn + r;
      if (row < M) p.slab[(int64_t)p.splits * ntile * TM * BN + (int64_t)bz * M + row] = racc[0];
    }
    return;
  }
  vm_wait<0>();
  __syncthreads();  // the ring is free: the epilogue reuses it

  // ---- epilogue: lane = row lrow(a), register group g = columns lcol(b) + 8g + 4h + {0..3} ----
  // alpha · acc goes to LDS as f32 in fragment order (in row halves where the f32 tile exceeds the LDS), then every
  // thread takes 8 consecutive columns of a row: + bias, the activation (storing the bf16 pre-activation and its
  // activation) or the activation gradient (the pre-activation read as one coalesced 16-B chunk), one rounding to
  // bf16, one 16-B store — whole 128-B lines per 8 lanes.
  auto lrow = [&](int a) { return wm * 32 * FM + 32 * a + r; };
  auto lcol = [&](int b) { return wn * 32 * FN + 32 * b; };
  const float al = p.alpha ? *p.alpha : 1.f;
  constexpr int kLd = BN + 4;                                     // f32 row pitch
  constexpr int ROWS_PASS = (TM * kLd * 4 <= C::LDS * 2) ? TM : TM / 2;
  constexpr int NPASS = TM / ROWS_PASS;
  static_assert(ROWS_PASS * kLd * 4 <= C::LDS * 2, "f32 epilogue tile");
  float* tf = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass) __syncthreads();  // the previous half's row-major reads are done
    const int rlo = pass * ROWS_PASS;
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const int lr = lrow(a) - rlo;  // wave-uniform range test (a wave's rows lie in one half)
      if (lr >= 0 && lr < ROWS_PASS)
#pragma unroll
        for (int b = 0; b < FN; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(tf + lr * kLd + lcol(b) + 8 * g + 4 * h) =
                make_float4(acc[a][b][4 * g] * al, acc[a][b][4 * g + 1] * al, acc[a][b][4 * g + 2] * al,
                            acc[a][b][4 * g + 3] * al);
    }
    __syncthreads();
    // every global operand of the pass (bias, pre-activation) loaded up front: the chunks' loads are independent,
    // so one memory round trip per pass instead of one per chunk
    // (in groups of 4 chunks: the other half's accumulators are still live in the two-pass form)
    constexpr int NQ = ROWS_PASS * BN / 8 / BT, QG = NQ < 4 ? NQ : 4;
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += QG) {
    float4 bias_v[QG][2];
    uint4 aux_v[QG];
#pragma unroll
    for (int qq = 0; qq < QG; ++qq) {
      const int q = q0 + qq;
      const int ch = threadIdx.x + BT * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
      const int gr = min(m0 + rlo + tr, M - 1), gc = min(n0 + tc, N - 8);
      bias_v[qq][0] = bias_v[qq][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) {
        bias_v[qq][0] = *reinterpret_cast<const float4*>(p.bias + gc);
        bias_v[qq][1] = *reinterpret_cast<const float4*>(p.bias + gc + 4);
      }
      if (p.epi == EPI_ACT_GRAD) aux_v[qq] = *reinterpret_cast<const uint4*>(p.aux + (int64_t)gr * p.ld_aux + gc);
    }
#pragma unroll
    for (int qq = 0; qq < QG; ++qq) {
      const int q = q0 + qq;
      const int ch = threadIdx.x + BT * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
      const int gr = m0 + rlo + tr, gc = n0 + tc;
      if (gr >= M || gc >= N) continue;
      const float4 v0 = *reinterpret_cast<const float4*>(tf + tr * kLd + tc);
      const float4 v1 = *reinterpret_cast<const float4*>(tf + tr * kLd + tc + 4);
      float v[8] = {v0.x + bias_v[qq][0].x, v0.y + bias_v[qq][0].y, v0.z + bias_v[qq][0].z, v0.w + bias_v[qq][0].w,
                    v1.x + bias_v[qq][1].x, v1.y + bias_v[qq][1].y, v1.z + bias_v[qq][1].z, v1.w + bias_v[qq][1].w};
      uint32_t o[4];
      if (p.epi == EPI_ACT_GRAD) {
        const uint32_t fw[4] = {aux_v[qq].x, aux_v[qq].y, aux_v[qq].z, aux_v[qq].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] *= act_factor(bf16_lo(fw[e]), p.act);
          v[2 * e + 1] *= act_factor(bf16_hi(fw[e]), p.act);
        }
      } else if (p.epi == EPI_BIAS_ACT) {  // the pre-activation (bf16: the value the activation and its gradient
                                          // see), then its activation
        if (p.act & ESGPT_ACT_DERIV) {  // act and act' of the bf16 pre-activation; act' is what gets stored
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
            float g0, g1;
            act_fwd_grad(bf16_lo(o[e]), p.act & 7, v[2 * e], g0);
            act_fwd_grad(bf16_hi(o[e]), p.act & 7, v[2 * e + 1], g1);
            o[e] = pack_bf16x2(g0, g1);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
            v[2 * e] = act_fwd(bf16_lo(o[e]), p.act);
            v[2 * e + 1] = act_fwd(bf16_hi(o[e]), p.act);
          }
        }
        *reinterpret_cast<uint4*>(p.aux_out + (int64_t)gr * p.ld_aux + gc) = make_uint4(o[0], o[1], o[2], o[3]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
      *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(p.C) + (int64_t)gr * p.ldc + gc) =
          make_uint4(o[0], o[1], o[2], o[3]);
    }
    }
  }
}

#ifdef ESGPT_TUNING_HOOKS
// Split-K reduction of the weight-gradient form: thread = one 16-B chunk of the fragment-order slab (tile, wave,
// fragment, register group, lane), summing its splits in split order (deterministic), then alpha, stored as 4
// columns of dW; threads past the tiles sum the row-sum slabs into the bias gradient (+ the optional extra rows).
template <int TM, int BN, int NWV>
__global__ __launch_bounds__(256) void big_slab_reduce_kernel(Prob p) {
  using C = BigCfg<false, false, TM, BN, NWV, 4>;
  constexpr int WN = C::WN, FM = C::FM, FN = C::FN, F = FM * FN;
  const int64_t ntile = (int64_t)p.tm * p.tn, nch = ntile * TM * BN / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float al = p.alpha ? *p.alpha : 1.f;
  if (t < nch) {
    const int lane = (int)(t & 63), g = (int)((t >> 6) & 3);
    const int64_t wf = t >> 8;  // (tile, wave, fragment)
    const int f = (int)(wf % F), wave = (int)((wf / F) % NWV);
    const int64_t tile = wf / F / NWV;
    int bx, by;
    group_tile((int)tile, p.tm, p.tn, by, bx);
    const int wm = wave / WN, wn = wave % WN, a = f / FN, b = f % FN;
    const int row = by * TM + wm * 32 * FM + 32 * a + (lane & 31);
    const int col = bx * BN + wn * 32 * FN + 32 * b + 8 * g + 4 * (lane >> 5);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
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
        s.x += v[u].x;
        s.y += v[u].y;
        s.z += v[u].z;
        s.w += v[u].w;
      }
    }
    if (row < p.M && col < p.N)
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + (int64_t)row * p.ldc + col) =
          make_float4(s.x * al, s.y * al, s.z * al, s.w * al);
  } else if (p.rowsum && t - nch < p.M) {
    const int64_t m = t - nch;
    const float* rs = p.slab + (int64_t)p.splits * nch * 4;
    float a = 0.f;
    for (int z = 0; z < p.splits; ++z) a += rs[(int64_t)z * p.M + m];
    p.rowsum[m] = (a + rowsum_extra(p, (int)m)) * al;
  }
}

#endif

template <bool AKC, bool BKC, int TM, int BN, int NWV, int NSLOT>
void launch_t(const Prob& p, hipStream_t st) {
  gemm_big_kernel<AKC, BKC, TM, BN, NWV, NSLOT><<<dim3((unsigned)(p.tm * p.tn)), 64 * NWV, 0, st>>>(p);
}

}  // namespace

namespace esgpt {
namespace gk {

// Large-tile form of a bf16-output, unsplit product (the forward projections: A and B K-contiguous; the input
// gradients: B M/N-contiguous). bn = 256 or 128 output columns per tile; p's tile grid is set here.
#ifdef ESGPT_TUNING_HOOKS
// tools build: a tile configuration "TM,BN,NWV" from the environment (0 = not set), read once per variable
struct BigTile {
  int tm, bn, nwv;
};
static BigTile env_tile_big(const char* name) {
  BigTile t{0, 0, 0};
  if (const char* e = tuning_env(name)) sscanf(e, "%d,%d,%d", &t.tm, &t.bn, &t.nwv);
  return t;
}
// the configurations compiled into the tools build
template <bool AKC, bool BKC, bool DW = false>
static bool launch_cfg(const Prob& p, BigTile t, unsigned grid, hipStream_t st) {
#define ESGPT_BIG_CFG(TM_, BN_, NW_)                                                              \
  if (t.tm == TM_ && t.bn == BN_ && t.nwv == NW_) {                                              \
    gemm_big_kernel<AKC, BKC, TM_, BN_, NW_, 4, DW><<<grid, 64 * NW_, 0, st>>>(p);                \
    return true;                                                                                 \
  }
  ESGPT_BIG_CFG(256, 256, 8)
  ESGPT_BIG_CFG(256, 128, 8)
  ESGPT_BIG_CFG(128, 128, 8)
  ESGPT_BIG_CFG(128, 256, 8)
  ESGPT_BIG_CFG(128, 128, 4)
  ESGPT_BIG_CFG(64, 128, 4)
  ESGPT_BIG_CFG(64, 64, 4)
#undef ESGPT_BIG_CFG
  return false;
}
#endif

bool launch_big(Prob p, bool akc, bool bkc, int bn, hipStream_t st) {
  if (!akc || p.out_f32 || p.splits != 1 || !p.fast || p.row_tiles || p.accumulate) return false;
  if (bn != 256 && bn != 128) return false;
  int tm = 256;
#ifdef ESGPT_TUNING_HOOKS
  static const BigTile forced = env_tile_big("ESGPT_GEMM_BIG_TILE");  // e.g. "64,128,4"
  if (forced.tm) {
    tm = forced.tm;
    bn = forced.bn;
  }
#endif
  p.fm = tm / 64;
  p.fn = bn / 64;
  p.tm = (int)cdiv(p.M, tm);
  p.tn = (int)cdiv(p.N, bn);
#ifdef ESGPT_TUNING_HOOKS
  if (forced.tm) {
    const unsigned grid = (unsigned)(p.tm * p.tn);
    return bkc ? launch_cfg<true, true>(p, forced, grid, st) : launch_cfg<true, false>(p, forced, grid, st);
  }
#endif
  if (bkc) {
    if (bn == 256) launch_t<true, true, 256, 256, 8, 4>(p, st);
    else launch_t<true, true, 256, 128, 8, 4>(p, st);
    return true;
  }
#ifdef ESGPT_TUNING_HOOKS  // the input-gradient form (B M/N-contiguous): tools build only (measured slower in step)
  if (bn == 256) launch_t<true, false, 256, 256, 8, 4>(p, st);
  else launch_t<true, false, 256, 128, 8, 4>(p, st);
  return true;
#else
  return false;
#endif
}

#ifdef ESGPT_TUNING_HOOKS
// The weight-gradient plan: tile (256 x 256 when that grid has at least 8 tiles, else 256 x 128; ESGPT_GEMM_BIG_DWTILE
// forces "TM,BN,NWV"), split count (about one workgroup per CU, every split at least kMinChunk tokens: fewer splits,
// less slab traffic) and the slab bytes.
constexpr int kMinChunk = 1024;
BigDw big_dw_plan(int64_t T, int64_t in, int64_t out) {
  static const BigTile forced = env_tile_big("ESGPT_GEMM_BIG_DWTILE");
  BigDw d{};
  d.tm = forced.tm ? forced.tm : 256;
  d.nwv = forced.tm ? forced.nwv : 8;
  d.bn = forced.tm ? forced.bn : (cdiv(out, 256) * cdiv(in, 256) >= 8 ? 256 : 128);
  const int64_t tiles = cdiv(out, d.tm) * cdiv(in, d.bn);
  static const int forced_chunk = [] {  // tools build: ESGPT_GEMM_BIG_DWCHUNK = minimum tokens per split
    const char* e = tuning_env("ESGPT_GEMM_BIG_DWCHUNK");
    return e ? atoi(e) : 0;
  }();
  // few tiles (a square-ish [out, in] of 512 x 512): chunks down to half the usual length
  const int64_t min_chunk =
      forced_chunk > 0 ? forced_chunk : (tiles * (T / kMinChunk) < 256 ? kMinChunk / 2 : kMinChunk);
  const int64_t target = forced.nwv == 4 ? 768 : 256;  // 4-wave workgroups: about three per CU
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(cdiv(target, tiles), T / min_chunk));
  const int64_t chunk = std::max<int64_t>(SK, cdiv(cdiv(T, splits), SK) * SK);
  d.splits = (int)std::max<int64_t>(1, cdiv(T, chunk));
  d.kchunk = (int)chunk;
  d.slab_bytes = sizeof(float) * ((size_t)d.splits * tiles * d.tm * d.bn + (size_t)d.splits * out);
  return d;
}

// dW [out, in] (+ db) = alpha · dYᵀ · X over T tokens on the large-tile kernel: the split workgroups, then the slab
// reduction. p: the dW product (A = dY M-contiguous, B = X N-contiguous, f32 C, slab = workspace of
// big_dw_plan(...).slab_bytes).
bool launch_big_dw(Prob p, hipStream_t st) {
  if (!p.fast || p.accumulate || p.slab == nullptr) return false;
  const BigDw d = big_dw_plan(p.K, p.N, p.M);
  p.fm = d.tm / 64;
  p.fn = d.bn / 64;
  p.tm = (int)cdiv(p.M, d.tm);
  p.tn = (int)cdiv(p.N, d.bn);
  p.splits = d.splits;
  p.kchunk = d.kchunk;
  const unsigned grid = (unsigned)((int64_t)p.tm * p.tn * p.splits);
  const int64_t nred = (int64_t)p.tm * p.tn * d.tm * d.bn / 4 + (p.rowsum ? p.M : 0);
  const BigTile t{d.tm, d.bn, d.nwv};
  if (!launch_cfg<false, false, true>(p, t, grid, st)) return false;
  const unsigned rg = (unsigned)cdiv(nred, 256);
#define ESGPT_BIG_RED(TM_, BN_, NW_) \
  if (d.tm == TM_ && d.bn == BN_ && d.nwv == NW_) big_slab_reduce_kernel<TM_, BN_, NW_><<<rg, 256, 0, st>>>(p);
  ESGPT_BIG_RED(256, 256, 8)
  ESGPT_BIG_RED(256, 128, 8)
  ESGPT_BIG_RED(128, 128, 8)
  ESGPT_BIG_RED(128, 256, 8)
  ESGPT_BIG_RED(128, 128, 4)
  ESGPT_BIG_RED(64, 128, 4)
  ESGPT_BIG_RED(64, 64, 4)
#undef ESGPT_BIG_RED
  return true;
}

#endif

}  // namespace gk
}  // namespace esgpt
