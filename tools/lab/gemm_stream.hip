// Streamed-tile persistent GEMM for the projections (bf16): see the kernel comment below. Measured and rejected
// (round 5, profiles/r05_gemm_stream_ab.log); built into the tools build only (csrc/Makefile TUNING=1), launched by
// gemm.hip (esgpt::gk::launch_stream) for the forward projections and the input-gradient products.
#include "gemm_parts.h"

namespace esgpt {
namespace gk {
#ifdef ESGPT_TUNING_HOOKS
namespace {

// ---- Streamed-tile GEMM: a persistent grid whose LDS-DMA ring runs across tile boundaries ----
// C2's projections have K = 256 (four 64-deep k-tiles) or 1024 and 8192 rows: a 64x64-tile launch re-reads every
// operand row through L2 once per output tile (qkv forward: 100 MB of tile operands for 12.6 MB of output) and each
// short-lived workgroup pays a full load latency in its prologue and its store tail in the epilogue. Here each
// workgroup (one per CU) walks a list of 128x128 (or 64·FM x 64·FN) output tiles with ONE continuous pipeline of
// (tile, k-tile) steps: NST LDS stages filled by buffer_load … lds, the DMA of step s + NST - 1 — possibly the next
// tile's first k-tiles — issued right after the barrier that retires step s, so the next tile's operands stream in
// while the current tile finishes and while its epilogue stores drain. Tiles are dealt per XCD in contiguous runs
// (the workgroups of one XCD work on neighbouring tiles at once: the A row block and the B tiles they share are
// fetched into that XCD's L2 once). A is K-contig (activations / dY rows); B K-contig (forward: W [N][K]) or
// N-contig (input gradient: W [K][N]). Epilogues as gemm_tile's (bias, activation with the pre-activation stored,
// activation gradient, device alpha), through a C tile in LDS beside the ring; bf16 output.
// Waits: a wave's VMEM ops (DMA pieces, epilogue loads and stores) retire in issue order; the wait for step s
// leaves the DMA steps issued after it in flight (vmcnt(P·ahead), P pieces per step). Epilogue stores issued after
// step s's DMA are not counted, so that wait also retires them: a store batch drains under the next tile's first
// k-tile. The epilogue's operand loads are issued before the step's DMA and carry no divergent control flow, so
// the compiler's own waits for them leave the ring in flight.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Epilogue LDS accesses as inline asm: hipcc cannot tell the C tile / bias rows apart from the ring the DMA is still
// filling and would drain every DMA in flight (vmcnt(0)) before each plain LDS access; these are ordered by explicit
// lgkmcnt waits and the workgroup barriers instead.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void lds_write_b64(void* p, uint32_t lo, uint32_t hi) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(make_uint2(lo, hi)) : "memory");
}
__device__ __forceinline__ u32x4_t lds_read_b128(const void* p) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ void lgkm_wait0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool BKC, int FM, int FN, int NST>
struct StreamCfg {
  using GA = GTile<true, 64 * FM>;
  using GB = GTile<BKC, 64 * FN>;
  static constexpr int BM = 64 * FM, BN = 64 * FN;
  static constexpr int STAGE = GA::kElems + GB::kElems;  // bf16 elements of one ring stage
  static constexpr int P = GA::kInstr + GB::kInstr;      // DMA instructions per wave and step
  static constexpr int CLD = BN + 8;                     // C tile pitch (bf16 elements)
  static constexpr int CEL = BM * CLD;
  static constexpr int ES = BM * BN / 8 / THREADS;       // 16-B stores per thread for one output tile
  static constexpr int LDS = NST * STAGE + CEL + 2 * BN * 2;  // + the bias rows of two tiles (f32)
};

template <bool BKC, int FM, int FN, int NST>
__global__ __launch_bounds__(THREADS, 1) void gemm_stream_kernel(Prob p) {
  using S = StreamCfg<BKC, FM, FN, NST>;
  using GA = typename S::GA;
  using GB = typename S::GB;
  constexpr int BM = S::BM, BN = S::BN, P = S::P;
  __shared__ __attribute__((aligned(16))) __bf16 smem[S::LDS];
  __bf16* const ctile = smem + NST * S::STAGE;
  float* const sbias = reinterpret_cast<float*>(ctile + S::CEL);  // [2][BN]: tile parity

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = p.M, N = p.N;
  const int ntile = p.tm * p.tn;
  // this workgroup's tiles: XCD x = blockIdx % 8 owns the contiguous run [lo, hi) of the tile order (n-tile
  // fastest); its workgroups take every nsl-th tile of the run
  const int G = gridDim.x, x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nsl = (G - x + 7) >> 3;
  const int lo = (int)(((int64_t)ntile * x) >> 3), hi = (int)(((int64_t)ntile * (x + 1)) >> 3);
  const int nmine = slot < hi - lo ? (hi - lo - slot + nsl - 1) / nsl : 0;
  const int nk = (p.K + BK - 1) / BK;
  const int nsteps = nmine * nk;
  if (nsteps == 0) return;

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(p.A), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(p.B), (short)0, 0x7fffffff, 0x00020000);
  // output stores are buffer stores whose out-of-range pieces (edge tiles) carry an offset past num_records and are
  // dropped: every lane issues the same number of stores, so the counted waits hold on edge tiles too
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsP =
      __builtin_amdgcn_make_buffer_rsrc(p.aux_out ? (void*)p.aux_out : p.C, (short)0, 0x7fffffff, 0x00020000);
  // the bias row of a tile rides with the tile's last k-tile as one 4-B DMA piece per 64 columns (waves 0 .. BN/64 - 1;
  // columns past N read 0: num_records = 4·N); the epilogue reads it from LDS after the barrier that retires that step
  const __amdgpu_buffer_rsrc_t rsBias = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.bias ? p.bias : reinterpret_cast<const float*>(p.A)), (short)0, p.bias ? 4 * N : 0,
      0x00020000);
  auto tile_of = [&](int i) { return lo + slot + i * nsl; };

  // issue cursor: step `is` = (tile it, k-tile ik); lane source offsets of tile it
  int is = 0, it = 0, ik = 0;
  int voA[GA::kInstr], voB[GB::kInstr];
  auto set_src = [&](int i) {
    const int t = tile_of(i);
    GA::lane_src(voA, p.lda, (t / p.tn) * BM, M);
    GB::lane_src(voB, p.ldb, (t % p.tn) * BN, N);
  };
  set_src(0);
  auto issue_next = [&]() {
    __bf16* sA = smem + (is % NST) * S::STAGE;
    const int k0 = ik * BK;
    GA::issue(rsA, voA, GA::k_soff(k0, p.lda), sA, p.K - k0);
    GB::issue(rsB, voB, GB::k_soff(k0, p.ldb), sA + GA::kElems, p.K - k0);
    if (ik == nk - 1 && p.bias && wave < BN / 64) {
      const int n0 = (tile_of(it) % p.tn) * BN;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsBias, (lds_void*)(sbias + (it & 1) * BN + 64 * wave), 4,
                                               (n0 + 64 * wave + lane) * 4, 0, 0, 0);
    }
    ++is;
    if (++ik == nk) {
      ik = 0;
      if (++it < nmine) set_src(it);
    }
  };
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (is < nsteps) issue_next();

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const float al = p.alpha ? *p.alpha : 1.f;
  int ct = 0, ck = 0;   // compute cursor: tile index, k-tile
  for (int s = 0; s < nsteps; ++s) {
    // retire step s: the younger DMA steps and the store batches issued after its DMA stay in flight
    const int ahead = is - (s + 1);  // NST - 2 except in the last steps
    if (NST >= 4 && ahead >= 2) vm_wait<(NST >= 4 ? 2 * P : 0)>();
    else if (NST >= 3 && ahead >= 1) vm_wait<(NST >= 3 ? P : 0)>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool last_k = ck + 1 == nk;
    if (is < nsteps) issue_next();  // into the stage every wave finished reading at step s - 1
    const __bf16* sA = smem + (s % NST) * S::STAGE;
    const __bf16* sB = sA + GA::kElems;
#pragma unroll
    for (int t = 0; t < BK / 16; ++t) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = GA::frag(sA, wm * 32 * FM + 32 * i, t);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = GB::frag(sB, wn * 32 * FN + 32 * j, t);
      if constexpr (!BKC) frag_wait();
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma(bfr[j], af[i], acc[i][j]);
    }
    if (!last_k) {
      ++ck;
      continue;
    }
    // ---- epilogue of tile ct: lane = output row, register group g = columns lcol(j) + 8g + 4h + {0..3} ----
    ck = 0;
    const int tl = tile_of(ct);
    const int m0 = (tl / p.tn) * BM, n0 = (tl % p.tn) * BN;
    const float* bt = sbias + (ct & 1) * BN;
    ++ct;
    auto lrow = [&](int i) { return wm * 32 * FM + 32 * i + r; };
    auto lcol = [&](int j) { return wn * 32 * FN + 32 * j; };
    u32x4_t bw[FN][4];
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) bw[j][g] = lds_read_b128(bt + lcol(j) + 8 * g + 4 * h);
      lgkm_wait0();
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) bw[j][g] = u32x4_t{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = acc[i][j][4 * g + e] * al + __uint_as_float(bw[j][g][e]);
        }
      }
    // one bf16 tile out: fragment-order LDS writes into the C tile, barrier, row-major 16-B chunk stores. The C tile
    // was last read by the previous epilogue's stores, before at least one barrier of a later step.
    auto store_tile = [&](const uint32_t (&d)[FM][FN][4][2], __amdgpu_buffer_rsrc_t rs, int64_t ld) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            lds_write_b64(ctile + lrow(i) * S::CLD + lcol(j) + 8 * g + 4 * h, d[i][j][g][0], d[i][j][g][1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      u32x4_t v[S::ES];
#pragma unroll
      for (int q = 0; q < S::ES; ++q) {
        const int ch = threadIdx.x + THREADS * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
        v[q] = lds_read_b128(ctile + tr * S::CLD + tc);
      }
      lgkm_wait0();
#pragma unroll
      for (int q = 0; q < S::ES; ++q) {
        const int ch = threadIdx.x + THREADS * q, tr = ch / (BN / 8), tc = (ch % (BN / 8)) * 8;
        const int gr = m0 + tr, gc = n0 + tc;
        const int off = (gr < M && gc < N) ? (int)(((int64_t)gr * ld + gc) * 2) : (int)0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 0);
      }
    };
    uint32_t d[FM][FN][4][2];
    if (p.epi == EPI_BIAS_ACT) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            d[i][j][g][0] = pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
            d[i][j][g][1] = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
            acc[i][j][4 * g + 0] = act_fwd(bf16_lo(d[i][j][g][0]), p.act);
            acc[i][j][4 * g + 1] = act_fwd(bf16_hi(d[i][j][g][0]), p.act);
            acc[i][j][4 * g + 2] = act_fwd(bf16_lo(d[i][j][g][1]), p.act);
            acc[i][j][4 * g + 3] = act_fwd(bf16_hi(d[i][j][g][1]), p.act);
          }
      store_tile(d, rsP, p.ld_aux);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave has read the C tile before it is rewritten
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
    store_tile(d, rsC, p.ldc);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  }
}


// Streamed-tile forward (gemm_stream_kernel): ESGPT_GEMM_STREAM tuning hook, read once — "0" off, "<fm><fn><nst>"
// forces a compiled configuration (e.g. "223"); unset: the default rule below.
int stream_mode() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_GEMM_STREAM");
    v = e ? std::max(0, atoi(e)) : 0;
  }
  return v;
}

int n_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount
                                                                                                 : 256;
    if (n < 8) n = 8;
  }
  return n;
}

template <bool BKC, int FM, int FN, int NST>
void launch_stream_cfg(Prob p, hipStream_t st) {
  p.fm = FM;
  p.fn = FN;
  p.tm = (int)cdiv(p.M, 64 * FM);
  p.tn = (int)cdiv(p.N, 64 * FN);
  p.splits = 1;
  const int64_t ntile = (int64_t)p.tm * p.tn;
  const int g = (int)std::max<int64_t>(8, std::min<int64_t>(ntile, n_cus()));
  gemm_stream_kernel<BKC, FM, FN, NST><<<dim3((unsigned)g), THREADS, 0, st>>>(p);
}

// bf16 output, A K-contig, whole-K (never split), operands and output addressable by 32-bit buffer offsets
template <bool BKC>
bool launch_stream_t(const Prob& p, hipStream_t st) {
  static_assert(StreamCfg<BKC, 2, 2, 3>::LDS * 2 <= 160 * 1024 * 2, "LDS");
  const int mode = stream_mode();
  if (mode == 0 || !p.fast || p.out_f32 || p.splits != 1 || p.accumulate || p.rowsum || p.epi == EPI_ACT_GRAD)
    return false;
  if (p.K <= BK) return false;  // the bias rows are double-buffered: a tile spans at least two k-tiles
  if ((int64_t)std::max(p.M, 1) * p.ldc * 2 >= ((int64_t)1 << 31)) return false;
  if (p.epi == EPI_BIAS_ACT && (int64_t)std::max(p.M, 1) * p.ld_aux * 2 >= ((int64_t)1 << 31)) return false;
  switch (mode) {
    case 223: launch_stream_cfg<BKC, 2, 2, 3>(p, st); return true;
    case 222: launch_stream_cfg<BKC, 2, 2, 2>(p, st); return true;
    case 214: launch_stream_cfg<BKC, 2, 1, 4>(p, st); return true;
    case 213: launch_stream_cfg<BKC, 2, 1, 3>(p, st); return true;
    case 124: launch_stream_cfg<BKC, 1, 2, 4>(p, st); return true;
    case 114: launch_stream_cfg<BKC, 1, 1, 4>(p, st); return true;
    default: launch_stream_cfg<BKC, 2, 2, 3>(p, st); return true;
  }
}

}  // namespace
#endif

// Measured at C2's forward shapes against the tile GEMM (tools/stream_ab.sh, profiles/r05_gemm_stream_ab.log): 1.4-1.7x
// SLOWER in every configuration (qkv 9.2 -> 14.2-19.7 us, c_fc 20.7 -> 33.5-42.9 us). One workgroup per CU keeps
// 64-96 KB of operands in flight through the ring, where eight resident 64x64 tile workgroups keep ~256 KB in flight
// in registers: at these K the operand fetch is latency-bound and the bytes in flight, not the bytes moved, set the
// rate. Kept in the tools build only (ESGPT_GEMM_STREAM); the product libraries never launch it.
bool launch_stream(const Prob& p, bool bkc, hipStream_t st) {
#ifdef ESGPT_TUNING_HOOKS
  return bkc ? launch_stream_t<true>(p, st) : launch_stream_t<false>(p, st);
#else
  (void)p;
  (void)bkc;
  (void)st;
  return false;
#endif
}

}  // namespace gk
}  // namespace esgpt
