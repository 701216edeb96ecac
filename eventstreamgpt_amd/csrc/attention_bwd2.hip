// bf16 MFMA attention backward in two kernels for gfx950 (InnerSelfAttention._attn, transformer.py:171-217):
// dK / dV key-block-major (attn_bwd_dkv_kernel) and dQ query-block-major (attn_bwd_dq_kernel), with no partial sums
// in memory. The fused kernel of attention_bwd.hip owns every key of a (batch, head) in one workgroup only up to 256
// keys; past that its dQ becomes one f32 partial per key block over every later query row, summed by a second pass
// (840 MB at B=4 H=8 L=4096, 6.3x the algorithmic bytes). Here each output is written once, by the one workgroup
// that owns it: the dK / dV workgroup sweeps the query tiles that see its keys (S and dP recomputed, dVᵀ += dOᵀ·(P∘Z),
// dKᵀ += Qᵀ·dS, as the fused kernel), and the dQ workgroup sweeps the key tiles its queries see (S and dP recomputed
// once more, dQᵀ += Kᵀ·dSᵀ). Deterministic, no atomics, no workspace; the extra S / dP products cost 2/5 more MFMA
// work than the fused kernel at large L, where that kernel is bound by its partial-sum traffic instead.
// Scheduling: causal chains differ in length by up to Lq / 64 tiles; the workgroups of each XCD are dealt longest
// chain first (the first key blocks / last query blocks), the (batch, head)s of one XCD sharing its L2.
// Fragment maps: attn_common.h. Dropout: the forward's keep bits (word (bh·Lq + q)·nw + key/32, bit key%32), or the
// counter hash regenerated; P is the undropped softmax probability, dS = P∘(Z∘dP − δ), δ = rowsum(dO∘O).
#include <algorithm>
#include <cstdlib>

#include "attn_common.h"
#include "common.h"

using namespace esgpt;
using namespace esgpt::attnb;

namespace {

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ bool allowed(int key, int qpos, int window) {
  return key <= qpos && (window == 0 || qpos - key < window);
}

// ---------------------------------------------------------------------------------------------------------------
// dK / dV: one workgroup = NWK waves = 32·NWK keys of one (batch, head); wave w owns keys 32w .. 32w+31 (K, V
// fragments in registers, dKᵀ / dVᵀ accumulators in registers). Per query tile (QT queries): Q and dO staged in LDS,
// lse / δ / keep words per query row; per wave and 32-query slice S = Q·Kᵀ − lse, dP = dO·Vᵀ − δ (key on the lane),
// then dVᵀ += dOᵀ·(P∘Z), dKᵀ += Qᵀ·dS from the accumulators as B operands (no LDS round trip).
template <int HD, int NWK, int DM>
struct DkvCfg {
  static constexpr int HDP = HD < 32 ? 32 : HD;
  // 32-query tiles at hd 128, and at hd 64 with the forward's keep bits (at 64 that instance spilled at two
  // workgroups per CU)
  static constexpr int QT = (HD == 128 || (HD == 64 && DM == DROP_BITS)) ? 32 : 64;
  static constexpr int KBW = 32 * NWK;
  static constexpr int THREADS = 64 * NWK;
  static constexpr int NKW = NWK;                             // keep words per query row of the key block
  static constexpr int NCH = QT * HD / 8;                     // 16-B chunks of a Q / dO tile
  static constexpr int CPT = (NCH + THREADS - 1) / THREADS;  // per thread
  static constexpr int LDS_BYTES = 2 * (2 * QT * HDP) + 4 * QT * NKW + 8 * QT;
};

template <int HD, int DM, int NWK>
__global__ __launch_bounds__(64 * NWK, HD == 128 ? 1 : 2) void attn_bwd_dkv_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v, int64_t ld_in,
    int64_t tq, const __bf16* __restrict__ o, int64_t ld_o, const __bf16* __restrict__ dout, int64_t ld_do,
    const float* __restrict__ lse, const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask,
    __bf16* __restrict__ dk, __bf16* __restrict__ dv, int64_t ld_d, int H, int nbh, int Lq, int Lk, int window,
    float drop_p, const uint64_t* __restrict__ seed, const uint32_t* __restrict__ keep, int nw) {
  using C = DkvCfg<HD, NWK, DM>;
  constexpr int QT = C::QT, HDP = C::HDP, NKW = C::NKW, KBW = C::KBW, NT = C::THREADS, CPT = C::CPT;
  constexpr bool DROP = DM != DROP_NONE, bits = DM == DROP_BITS;
  using IQ = Img<HDP>;
  __shared__ __attribute__((aligned(16))) char smem_raw[C::LDS_BYTES];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  __bf16* sQ = reinterpret_cast<__bf16*>(smem_raw);
  __bf16* sD = sQ + QT * HDP;
  uint32_t* sZ = reinterpret_cast<uint32_t*>(sD + QT * HDP);  // [word][query]
  float* sL = reinterpret_cast<float*>(sZ + NKW * QT);
  float* sDl = sL + QT;

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;  // transposed-read lane roles
  int kblk, bh;
  deal(blockIdx.x, gridDim.x, nbh, kblk, bh);  // rank 0 = key block 0 = the longest causal chain
  const int b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const bool idx32 = (uint64_t)nbh * (uint64_t)Lq * (uint64_t)Lk <= 0xffffffffull;
  const int off = Lk - Lq;
  const int kb0 = kblk * KBW;
  const int kw0 = kb0 + 32 * wave;  // this wave's first key
  const int key = kw0 + r;
  const bool kvalid = key < Lk && (kmask == nullptr || kmask[(int64_t)b * Lk + key] != 0);

  bf16x8 kf[HD / 16], vf[HD / 16];
  {
    const int kk = min(key, Lk - 1);
    const __bf16* krow = k + ((int64_t)b * Lk + kk) * ld_in + hh * HD;
    const __bf16* vrow = v + ((int64_t)b * Lk + kk) * ld_in + hh * HD;
#pragma unroll
    for (int t = 0; t < HD / 16; ++t) {
      kf[t] = key < Lk ? *reinterpret_cast<const bf16x8*>(krow + 16 * t + 8 * h) : zero8();
      vf[t] = key < Lk ? *reinterpret_cast<const bf16x8*>(vrow + 16 * t + 8 * h) : zero8();
    }
  }
  f32x16 dka[HDP / 32], dva[HDP / 32];
#pragma unroll
  for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dka[dt][i] = dva[dt][i] = 0.f;
  if (HD < HDP) {  // hd = 16: image columns 16..31 stay zero (staging writes columns 0..15 only)
    for (int row = tid; row < 2 * QT; row += NT) {
      __bf16* img = row < QT ? sQ : sD;
      const int rr = row < QT ? row : row - QT;
      *reinterpret_cast<bf16x8*>(img + IQ::off(rr, HD)) = zero8();
      *reinterpret_cast<bf16x8*>(img + IQ::off(rr, HD + 8)) = zero8();
    }
  }

  const int kbend = min(Lk, kb0 + KBW) - 1;
  const int qlo = max(0, kb0 - off);
  const int qhi = window ? min(Lq - 1, kbend + window - 1 - off) : Lq - 1;

  // query-tile prefetch: CPT 16-B chunks of Q, dO and O per thread, the row's lse / validity for the chunk-0
  // thread and one keep word per thread; issued one tile ahead, written to LDS at the top of the tile
  const bool zstager = bits && tid < QT * NKW;
  const int zw = tid / QT, zrow = tid % QT;
  bf16x8 pq[CPT], pd[CPT], po[CPT];
  float pl[CPT];
  uint32_t pz = 0;
  auto prefetch = [&](int q0) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ch = tid + NT * c, srow = ch / (HD / 8), sc8 = ch % (HD / 8);
      const int qi = q0 + srow;
      const bool in = ch < C::NCH && qi < Lq;
      pq[c] = pd[c] = po[c] = zero8();
      pl[c] = INFINITY;
      if (in) {
        pq[c] = *reinterpret_cast<const bf16x8*>(q + ((int64_t)b * tq + qi) * ld_in + hh * HD + sc8 * 8);
        pd[c] = *reinterpret_cast<const bf16x8*>(dout + ((int64_t)b * Lq + qi) * ld_do + hh * HD + sc8 * 8);
        po[c] = *reinterpret_cast<const bf16x8*>(o + ((int64_t)b * Lq + qi) * ld_o + hh * HD + sc8 * 8);
        if (sc8 == 0 && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0)) pl[c] = lse[(int64_t)bh * Lq + qi];
      }
    }
    const int zq = q0 + zrow, zc = (kb0 >> 5) + zw;
    pz = (zstager && zq < Lq && zc < nw) ? keep[((int64_t)bh * Lq + zq) * nw + zc] : 0u;
  };
  const int qt0 = (qlo / QT) * QT;
  if (qt0 <= qhi) prefetch(qt0);

  for (int q0 = qt0; q0 <= qhi; q0 += QT) {
    __syncthreads();  // the previous tile's reads of sQ / sD / sZ / sL are done
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ch = tid + NT * c, srow = ch / (HD / 8), sc8 = ch % (HD / 8);
      if (ch < C::NCH) {
        *reinterpret_cast<bf16x8*>(sQ + IQ::off(srow, sc8 * 8)) = pq[c];
        *reinterpret_cast<bf16x8*>(sD + IQ::off(srow, sc8 * 8)) = pd[c];
      }
      float dl = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) dl = fmaf((float)pd[c][j], (float)po[c][j], dl);
      // δ: sum over the HD/8 consecutive threads of the row (rows never straddle a wave)
#pragma unroll
      for (int o2 = 1; o2 < HD / 8; o2 <<= 1) dl += __shfl_xor(dl, o2, 64);
      if (ch < C::NCH && sc8 == 0) {
        sL[srow] = pl[c];  // +inf for invalid / missing queries: P = exp(S - inf) = 0 for the row
        sDl[srow] = pl[c] == INFINITY ? 0.f : dl;
      }
    }
    if (zstager) sZ[tid] = pz;
    __syncthreads();
    if (q0 + QT <= qhi) prefetch(q0 + QT);  // in flight during this tile's MFMAs

#pragma unroll 1
    for (int qs = 0; qs < QT / 32; ++qs) {
      const int qa = q0 + 32 * qs;
      const int qpos_lo = qa + off, qpos_hi = min(qa + 31, Lq - 1) + off;
      const bool any = qa < Lq && qpos_hi >= kw0 && kw0 < Lk && (window == 0 || qpos_lo - (kw0 + 31) < window);
      if (!any) continue;  // wave-uniform
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = 32 * qs + acc_row(i, h);
        s[i] = -sL[row];
        dp[i] = -sDl[row];
      }
#pragma unroll
      for (int t = 0; t < HD / 16; ++t) {
        const bf16x8 qa8 = *reinterpret_cast<const bf16x8*>(sQ + IQ::off(32 * qs + r, 16 * t + 8 * h));
        const bf16x8 da8 = *reinterpret_cast<const bf16x8*>(sD + IQ::off(32 * qs + r, 16 * t + 8 * h));
        s = mfma(qa8, kf[t], s);
        dp = mfma(da8, vf[t], dp);
      }
      const bool full = __ballot(kvalid) == ~0ull && qpos_lo >= kw0 + 31 && (window == 0 || qpos_hi - kw0 < window);
      float zk[16];
      const uint32_t* zrow_w = sZ + wave * QT + 32 * qs;
      uint32_t zbits = 0;  // DROP_BITS: this lane's keep bit of each of its 16 rows (bit i <-> register i)
      if (bits) {
        // rows acc_row(i, h) = 4h + {0..3, 8..11, 16..19, 24..27}: four 16-B groups of keep words, folded into one
        // 16-bit mask at once (the words do not stay live across the element loop)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const uint4 w4 = *reinterpret_cast<const uint4*>(zrow_w + 8 * gq + 4 * h);
          zbits |= ((w4.x >> r) & 1u) << (4 * gq) | ((w4.y >> r) & 1u) << (4 * gq + 1) |
                   ((w4.z >> r) & 1u) << (4 * gq + 2) | ((w4.w >> r) & 1u) << (4 * gq + 3);
        }
      } else if (DROP && idx32) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          zk[i] = dropout_mult_32(dr, ((uint32_t)bh * (uint32_t)Lq + (uint32_t)(qa + acc_row(i, h))) * (uint32_t)Lk +
                                          (uint32_t)key);
      } else if (DROP) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          zk[i] = dropout_mult(dr, ((uint64_t)bh * (uint64_t)Lq + (uint64_t)(qa + acc_row(i, h))) * (uint64_t)Lk +
                                       (uint64_t)key);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = 32 * qs + acc_row(i, h);
        const int qpos = q0 + ql + off;
        const float e = __builtin_amdgcn_exp2f(s[i] * kLog2e);
        const bool ok = full | (kvalid & (key <= qpos) & ((window == 0) | (qpos - key < window)));
        const float p = ok ? e : 0.f;
        if (DROP) {
          const float z = bits ? (((zbits >> i) & 1u) ? dr.scale : 0.f) : zk[i];
          const float dl = sDl[ql];
          s[i] = p * z;                          // P∘Z (feeds dV)
          dp[i] = p * (z * (dp[i] + dl) - dl);   // dS
        } else {
          s[i] = p;
          dp[i] = p * dp[i];
        }
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pf = acc_frag(s, ss);
        const bf16x8 dsf = acc_frag(dp, ss);
        const int row0 = 32 * qs + 16 * ss + 4 * (g >> 1) + q4;
#pragma unroll
        for (int dt = 0; dt < HDP / 32; ++dt) {
          const int col = 32 * dt + 16 * (g & 1) + 4 * p4;
          const bf16x8 dof = join(tr_read(sD + IQ::off(row0, col)), tr_read(sD + IQ::off(row0 + 8, col)));
          dva[dt] = mfma(dof, pf, dva[dt]);
          const bf16x8 qf = join(tr_read(sQ + IQ::off(row0, col)), tr_read(sQ + IQ::off(row0 + 8, col)));
          dka[dt] = mfma(qf, dsf, dka[dt]);
        }
      }
    }
  }
  if (key < Lk) {
    __bf16* ko = dk + ((int64_t)b * Lk + key) * ld_d + hh * HD;
    __bf16* vo = dv + ((int64_t)b * Lk + key) * ld_d + hh * HD;
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt) {
      store_col32<HD < 32 ? HD : 32>(ko + 32 * dt, dka[dt], h);
      store_col32<HD < 32 ? HD : 32>(vo + 32 * dt, dva[dt], h);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// dQ: one 256-thread workgroup (4 waves) per 64-query block of one (batch, head), as the forward kernel: wave w owns
// queries 32·(w&1) .. +31 of the block (the query on the MFMA lane: Q and dO fragments, lse, δ in registers) and the
// 64-key tiles of parity w>>1; K and V tiles are staged in LDS in pairs (next pair prefetched into registers). Per
// tile: Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ (key in the accumulator rows), P, dS, then dQᵀ += Kᵀ·dSᵀ with dS straight from the
// accumulator registers (K read transposed, in the permuted key order). The two key parities' dQᵀ are summed
// through LDS at the end.
template <int HD>
struct DqCfg {
  static constexpr int HDP = HD < 32 ? 32 : HD;
  static constexpr int ROWS = 64;
  static constexpr int NLD = 2 * ROWS * (HD / 8) / 256;  // 16-B chunks per thread and tensor for a pair of tiles
  static constexpr int IMG = 2 * ROWS * HDP;             // bf16 elements of a pair of K (or V) tiles
  static constexpr int MERGE = 2 * (HDP / 32) * 16 * 64 * 2;  // bf16 elements holding the f32 merge state
};

template <int HD, int DM>
__global__ __launch_bounds__(256, HD == 128 ? 1 : 2) void attn_bwd_dq_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v, int64_t ld_in,
    int64_t tq, const __bf16* __restrict__ o, int64_t ld_o, const __bf16* __restrict__ dout, int64_t ld_do,
    const float* __restrict__ lse, const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask,
    __bf16* __restrict__ dq, int64_t ld_d, int H, int nbh, int Lq, int Lk, int window, float drop_p,
    const uint64_t* __restrict__ seed, const uint32_t* __restrict__ keep, int nw) {
  using C = DqCfg<HD>;
  constexpr int HDP = C::HDP, ROWS = C::ROWS, NLD = C::NLD, CH = HD / 8;
  constexpr bool DROP = DM != DROP_NONE, bits = DM == DROP_BITS;
  static_assert(NLD >= 1 && NLD * 256 == 2 * ROWS * CH, "tile pair staging");
  static_assert(C::MERGE <= C::IMG, "merge state in the K images");
  using IK = Img<HDP>;
  __shared__ __attribute__((aligned(16))) __bf16 sK[C::IMG];
  __shared__ __attribute__((aligned(16))) __bf16 sV[C::IMG];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int qh = wave & 1, kp = wave >> 1;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int nqb = (Lq + ROWS - 1) / ROWS;
  int rank, bh;
  deal(blockIdx.x, gridDim.x, nbh, rank, bh);
  const int qb = nqb - 1 - rank;  // rank 0 = the last query block = the longest causal chain
  const int b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const bool idx32 = (uint64_t)nbh * (uint64_t)Lq * (uint64_t)Lk <= 0xffffffffull;
  const int off = Lk - Lq;
  const int qb0 = qb * ROWS;
  const int qi = qb0 + qh * 32 + r;
  const bool qin = qi < Lq;
  const bool qvalid = qin && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0);
  const int qpos = qi + off;
  const int qlo_w = qb0 + qh * 32 + off;
  const int qhi_w = min(qb0 + qh * 32 + 31, Lq - 1) + off;

  // this lane's query: Q and dO fragments (B operands), δ = rowsum(dO∘O), lse in the log2 domain (+inf: no row)
  bf16x8 qf[HD / 16], df[HD / 16];
  float dl = 0.f;
  {
    const int qc = min(qi, Lq - 1);
    const __bf16* qrow = q + ((int64_t)b * tq + qc) * ld_in + hh * HD;
    const __bf16* drow = dout + ((int64_t)b * Lq + qc) * ld_do + hh * HD;
    const __bf16* orow = o + ((int64_t)b * Lq + qc) * ld_o + hh * HD;
#pragma unroll
    for (int t = 0; t < HD / 16; ++t) {
      qf[t] = qin ? *reinterpret_cast<const bf16x8*>(qrow + 16 * t + 8 * h) : zero8();
      df[t] = qin ? *reinterpret_cast<const bf16x8*>(drow + 16 * t + 8 * h) : zero8();
      const bf16x8 of = qin ? *reinterpret_cast<const bf16x8*>(orow + 16 * t + 8 * h) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) dl = fmaf((float)df[t][j], (float)of[j], dl);
    }
  }
  dl += __shfl_xor(dl, 32, 64);
  const float lq = qvalid ? lse[(int64_t)bh * Lq + qi] * kLog2e : INFINITY;
  if (!qvalid) dl = 0.f;

  f32x16 dqa[HDP / 32];
#pragma unroll
  for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqa[dt][i] = 0.f;

  const int qhi = min(Lq, qb0 + ROWS) - 1;
  const int kmax = min(Lk - 1, qhi + off);
  const int kmin = window ? max(0, qb0 + off - window + 1) : 0;
  const __bf16* kbase = k + (int64_t)b * Lk * ld_in + hh * HD;
  const __bf16* vbase = v + (int64_t)b * Lk * ld_in + hh * HD;
  const uint8_t* kmb = kmask ? kmask + (int64_t)b * Lk : nullptr;
  const uint32_t* kwrow = (bits && qin) ? keep + ((int64_t)bh * Lq + qi) * nw : nullptr;

  // pair of tiles (keys kt .. kt+127) -> registers by buffer loads whose range ends after row kmax (rows past it read
  // as zeros, no per-load branch; esgpt_attn_mfma_supported bounds Lk·ld_in·2 below 2^31)
  bf16x8 rk[NLD], rv[NLD];
  uint32_t zw[2] = {0u, 0u};  // keep words of this wave's tile (two 32-key groups), prefetched with the pair
  const int rec = (kmax + 1) * (int)ld_in * 2;
  const __amdgpu_buffer_rsrc_t rsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(kbase), (short)0, rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(vbase), (short)0, rec, 0x00020000);
  auto load_pair = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + 256 * i, row = c / CH, c8 = c % CH;
      const int vo = (kt + row) * (int)ld_in * 2 + c8 * 16;
      rk[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsk, vo, 0, 0));
      rv[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsv, vo, 0, 0));
    }
    if (bits) {
      const int w0 = (kt + ROWS * kp) >> 5;
#pragma unroll
      for (int c = 0; c < 2; ++c) zw[c] = (kwrow != nullptr && w0 + c < nw) ? kwrow[w0 + c] : 0u;
    }
  };
  auto key_ok = [&](int kt) {
    const int key = kt + ROWS * kp + lane;
    return key <= kmax && (kmb == nullptr || kmb[key] != 0);
  };

  int kt = (kmin / ROWS) * ROWS;
  load_pair(kt);
  bool kok = key_ok(kt);
  for (; kt <= kmax; kt += 2 * ROWS) {
    const int t0 = kt + ROWS * kp;
    const uint64_t kbits = __ballot(kok);
    uint32_t zc[2] = {zw[0], zw[1]};
    __syncthreads();  // the previous pair's LDS reads are done
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + 256 * i, row = c / CH, c8 = c % CH;
      *reinterpret_cast<bf16x8*>(sK + IK::off(row, c8 * 8)) = rk[i];
      *reinterpret_cast<bf16x8*>(sV + IK::off(row, c8 * 8)) = rv[i];
    }
    if (HD < HDP) {  // hd = 16: image columns 16..31 zero
      for (int row = tid; row < 2 * ROWS; row += 256) {
        *reinterpret_cast<bf16x8*>(sK + IK::off(row, HD)) = zero8();
        *reinterpret_cast<bf16x8*>(sK + IK::off(row, HD + 8)) = zero8();
        *reinterpret_cast<bf16x8*>(sV + IK::off(row, HD)) = zero8();
        *reinterpret_cast<bf16x8*>(sV + IK::off(row, HD + 8)) = zero8();
      }
    }
    __syncthreads();
    if (kt + 2 * ROWS <= kmax) {
      load_pair(kt + 2 * ROWS);
      kok = key_ok(kt + 2 * ROWS);
    }
    if (!kbits) continue;  // fully padded (or absent) key tile
    const int rb = ROWS * kp;  // this wave's tile rows in the pair images

    const bool full = kbits == ~0ull && t0 + ROWS - 1 <= qlo_w && (window == 0 || qhi_w - t0 < window);
    // this lane's visible keys of the tile as one word (valid-key ballot ∩ causal limit ∩ window), the half-wave's
    // 4-row offset shifted out: each score's test is one bit at a compile-time position
    uint64_t okm = ~0ull;
    if (!full) {
      const int rel = qpos - t0;
      uint64_t am = kbits & (rel >= 63 ? ~0ull : (rel < 0 ? 0ull : ((2ull << rel) - 1ull)));
      if (window) {
        const int lo = rel - window + 1;
        am &= lo <= 0 ? ~0ull : (lo > 63 ? 0ull : ~((1ull << lo) - 1ull));
      }
      okm = am >> (4 * h);
    }
    // the two 32-key halves one after the other (half the live accumulators)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = 0.f;
        dp[i] = -dl;
      }
#pragma unroll
      for (int t = 0; t < HD / 16; ++t) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(sK + IK::off(rb + 32 * c + r, 16 * t + 8 * h));
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(sV + IK::off(rb + 32 * c + r, 16 * t + 8 * h));
        s = mfma(a, qf[t], s);
        dp = mfma(av, df[t], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kr = 32 * c + acc_row(i, h);
        const float e = __builtin_amdgcn_exp2f(fmaf(s[i], kLog2e, -lq));  // exp2(-inf) = 0: no row
        const bool ok = ((uint32_t)(okm >> (32 * c)) >> ((i & 3) + 8 * (i >> 2))) & 1u;
        const float p = ok ? e : 0.f;
        if (DROP) {
          float z;
          if (bits) {
            z = ((zc[c] >> acc_row(i, h)) & 1u) ? dr.scale : 0.f;
          } else if (idx32) {
            z = dropout_mult_32(dr, ((uint32_t)bh * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk + (uint32_t)(t0 + kr));
          } else {
            z = dropout_mult(dr, ((uint64_t)bh * (uint64_t)Lq + (uint64_t)qi) * (uint64_t)Lk + (uint64_t)(t0 + kr));
          }
          dp[i] = p * (z * (dp[i] + dl) - dl);
        } else {
          dp[i] = p * dp[i];
        }
      }
      // dQᵀ[d][q] += Kᵀ[d][key] · dSᵀ[key][q]: K read transposed in the accumulator's permuted key order
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 dsf = acc_frag(dp, ss);
        const int row0 = rb + 32 * c + 16 * ss + 4 * (g >> 1) + q4;
#pragma unroll
        for (int dt = 0; dt < HDP / 32; ++dt) {
          const int col = 32 * dt + 16 * (g & 1) + 4 * p4;
          const bf16x8 kfr = join(tr_read(sK + IK::off(row0, col)), tr_read(sK + IK::off(row0 + 8, col)));
          dqa[dt] = mfma(kfr, dsf, dqa[dt]);
        }
      }
    }
  }

  // ---- sum the two key parities of each query half (the odd-parity wave hands its dQᵀ over in LDS) ----
  __syncthreads();
  float* cO = reinterpret_cast<float*>(sK);  // [qh][HDP/32][16][64]
  if (kp == 1) {
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) cO[((qh * (HDP / 32) + dt) * 16 + i) * 64 + lane] = dqa[dt][i];
  }
  __syncthreads();
  if (kp == 1 || !qin) return;
  __bf16* qo = dq + ((int64_t)b * tq + qi) * ld_d + hh * HD;
#pragma unroll
  for (int dt = 0; dt < HDP / 32; ++dt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) dqa[dt][i] += cO[((qh * (HDP / 32) + dt) * 16 + i) * 64 + lane];
    store_col32<HD < 32 ? HD : 32>(qo + 32 * dt, dqa[dt], h);
  }
}

template <int HD, int NWK>
int launch2(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o, int64_t ld_o,
            const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask, const uint8_t* qmask, void* dq,
            void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t window,
            float drop_p, const uint64_t* seed, const uint32_t* keep, hipStream_t st) {
  const int nbh = (int)(B * H), nw = (int)cdiv(Lk, 32);
  const dim3 ga((unsigned)(cdiv(Lk, 32 * NWK) * nbh)), gq((unsigned)(cdiv(Lq, 64) * nbh));
#define ESGPT_BWD2(DM_)                                                                                             \
  do {                                                                                                              \
    attn_bwd_dkv_kernel<HD, DM_, NWK><<<ga, 64 * NWK, 0, st>>>(                                                     \
        (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, ld_in, tq, (const __bf16*)o, ld_o, (const __bf16*)dout, \
        ld_do, lse, kmask, qmask, (__bf16*)dk, (__bf16*)dv, ld_d, (int)H, nbh, (int)Lq, (int)Lk, (int)window, drop_p,  \
        seed, keep, nw);                                                                                            \
    attn_bwd_dq_kernel<HD, DM_><<<gq, 256, 0, st>>>(                                                                \
        (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, ld_in, tq, (const __bf16*)o, ld_o, (const __bf16*)dout, \
        ld_do, lse, kmask, qmask, (__bf16*)dq, ld_d, (int)H, nbh, (int)Lq, (int)Lk, (int)window, drop_p, seed, keep, \
        nw);                                                                                                        \
  } while (0)
  if (!(drop_p > 0.f)) ESGPT_BWD2(DROP_NONE);
  else if (keep) ESGPT_BWD2(DROP_BITS);
  else ESGPT_BWD2(DROP_HASH);
#undef ESGPT_BWD2
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

}  // namespace

// The split backward (dK / dV kernel + dQ kernel) for the bf16 MFMA path; same arguments and semantics as the fused
// kernel (attention_bwd.hip), no workspace. keys_per_wg: 32 x the dK / dV workgroup's waves (64 or 128).
int esgpt_attn_bwd_mfma_split(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                              int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                              const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                              int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                              const uint32_t* keep, int keys_per_wg, hipStream_t st) {
#ifdef ESGPT_TUNING_HOOKS
#define ESGPT_BWD2_HD(HD_)                                                                                           \
  return keys_per_wg == 64                                                                                           \
             ? launch2<HD_, 2>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, \
                               Lk, window, drop_p, seed, keep, st)                                                     \
             : launch2<HD_, 4>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, \
                               Lk, window, drop_p, seed, keep, st)
  if (hd == 16) ESGPT_BWD2_HD(16);
  if (hd == 32) ESGPT_BWD2_HD(32);
  if (hd == 64) ESGPT_BWD2_HD(64);
  ESGPT_BWD2_HD(128);
#else
  // the product takes the split form at hd = 16 / 64 / 128 with 128 keys per dK / dV workgroup (split2_keys); the
  // hd = 32 and 64-key forms (measured slower) exist in the tools build only
  (void)keys_per_wg;
#define ESGPT_BWD2_HD(HD_)                                                                                           \
  return launch2<HD_, 4>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, Lk,  \
                         window, drop_p, seed, keep, st)
  if (hd == 16) ESGPT_BWD2_HD(16);
  if (hd == 64) ESGPT_BWD2_HD(64);
  if (hd == 128) ESGPT_BWD2_HD(128);
  return ESGPT_ERR_UNSUPPORTED;
#endif
#undef ESGPT_BWD2_HD
}
