// bf16 MFMA attention backward for gfx950 (InnerSelfAttention._attn, transformer.py:171-217): ONE kernel computes
// dQ, dK and dV with no atomics when a (batch, head) has at most 256 keys (every C1/C2/C4 sequence), and adds dQ with
// f32 atomics into a workspace otherwise (one conversion pass at the end).
//
// Work decomposition: one 512-thread workgroup = 8 waves = 256 keys of one (batch, head); wave w owns keys
// 32w .. 32w+31 of the block (K, V fragments in registers, dKᵀ / dVᵀ accumulators in registers). The workgroup
// sweeps the query tiles that can see its keys (causal / local window bounds), QT queries at a time:
//   stage Q, dO (row-major LDS images) and the per-query constants lse, δ = rowsum(dO∘O) (δ computed here from
//   dO and O: no separate pass, no δ buffer);
//   per wave and 32-query slice:   S  = Q·Kᵀ − lse      (accumulator initialised to −lse: P = exp(S) directly)
//                                  dP = dO·Vᵀ − δ       (initialised to −δ)
//                                  (key on the MFMA lane: both accumulators are the B operands of the next two)
//                                  dVᵀ += dOᵀ·(P∘Z),  dKᵀ += Qᵀ·dS,  dS = P∘(Z∘dP̃ − δ)   (Z = dropout keep/scale)
//   dS crosses LDS once ([key][q] image, 8-byte stores), then dQ = dS·K for the tile over all 256 keys, one 32x32
//   output tile per wave (K image [key][d] read transposed).
// Fragment conventions (v_mfma_f32_32x32x16_bf16): lane l = (r = l&31, h = l>>5); A[row r][k = 8h+j],
// B[k = 8h+j][col r]; C reg i = row (i&3) + 8(i>>2) + 4h, col r. An accumulator used as a B operand supplies k-step
// s element j = row 16s + 8(j>>2) + 4h + (j&3) (permuted); the A operand is then read in that order.
// hd = 16 (C1): S and dP are one K = 16 step; the Q / dO / K images are 32 columns wide with columns 16..31 zero, so
// dVᵀ / dKᵀ / dQ run as 32-wide tiles whose rows 16..31 come out zero and are not stored.
// Roofline: MFMA-bound at large L; algorithmic FLOPs 8·H·hd·T (T = allowed (q, k) pairs; recompute not counted).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "attn_common.h"

using namespace esgpt;
using namespace esgpt::attnb;

int esgpt_attn_bwd_mfma_split(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                              int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                              const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                              int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                              const uint32_t* keep, int keys_per_wg, hipStream_t st);

namespace {

#ifdef ESGPT_STAMPS
__device__ uint64_t g_stamps[64];
#define STAMP(i)                                                                              \
  do {                                                                                        \
    if (blockIdx.x == 40 && threadIdx.x == 0) g_stamps[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(i)
#endif

constexpr int KB = 256;      // keys per workgroup
constexpr int NW = 8;        // waves
constexpr int THREADS = 64 * NW;

template <int HD>
struct Cfg {
  static constexpr int HDP = HD < 32 ? 32 : HD;   // image / accumulator width (hd = 16: zero-padded to 32)
  static constexpr int QT = HD == 128 ? 32 : 64;  // queries per tile
  static constexpr int NKW = KB / 32;             // keep-bit words per query row of the key block
  // K image, Q and dO images, dS image, keep words, lse and δ
  static constexpr int LDS_BYTES = 2 * (KB * HDP + 2 * QT * HDP + KB * QT) + 4 * QT * NKW + 8 * QT;
};


// Query tile j (counted from the first tile that can see the key block) of split s out of S: S = 1 takes every
// tile; S = 2 deals the tiles zig-zag (s = 0: 0, 3, 4, 7, 8, …; s = 1: 1, 2, 5, 6, …), so that under a causal mask
// (tile cost growing with its index) both splits get the same dQ work.
__device__ __forceinline__ int split_tile(int it, int s, int S) {
  if (S == 1) return it;
  return 4 * (it >> 1) + ((it & 1) ? 3 - s : s);
}

// nsplit > 1: the query tiles of a key block are split (zig-zag) over two workgroups that add their partial dKᵀ / dVᵀ
// through write-through slabs (xcnt / xbuf). DM = DROP_BITS: the forward's dropout keep bits, word
// keep[(bh*Lq + q)*nw + key/32], bit key%32, staged in LDS with each query tile; DROP_HASH: the keep mask is
// regenerated from the counter hash (the same bits, twice the per-tile VALU work at L = 256).
template <int HD, int DM>
__global__ __launch_bounds__(THREADS) void attn_bwd_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v, int64_t ld_in,
    int64_t tq, const __bf16* __restrict__ o, int64_t ld_o, const __bf16* __restrict__ dout, int64_t ld_do,
    const float* __restrict__ lse, const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask,
    __bf16* __restrict__ dq, __bf16* __restrict__ dk, __bf16* __restrict__ dv, int64_t ld_d,
    float* __restrict__ dq32, int H, int Lq, int Lk, int window, float drop_p, const uint64_t* __restrict__ seed,
    const uint32_t* __restrict__ keep, int nw, int nsplit, int32_t* __restrict__ xcnt, float* __restrict__ xbuf,
    int64_t dq_slab, int order) {
  using C = Cfg<HD>;
  constexpr int QT = C::QT, HDP = C::HDP, NKW = C::NKW;
  constexpr bool DROP = DM != DROP_NONE, bits = DM == DROP_BITS;
  using IQ = Img<HDP>;  // Q, dO, K images: [row][HDP]
  using IS = Img<QT>;   // dS image: [key][QT]
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  __bf16* sK = reinterpret_cast<__bf16*>(smem_raw);
  __bf16* sQ = sK + KB * HDP;
  __bf16* sD = sQ + QT * HDP;
  __bf16* sS = sD + QT * HDP;
  uint32_t* sZ = reinterpret_cast<uint32_t*>(sS + KB * QT);  // [word][query]
  float* sL = reinterpret_cast<float*>(sZ + NKW * QT);
  float* sDl = sL + QT;

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;  // transposed-read lane roles
  const int nxb = ((Lk + KB - 1) / KB) * nsplit;       // workgroups per (batch, head)
  // order 0: XCD-contiguous runs per (batch, head); order 1: the (batch, head)s of one XCD kept together and their
  // key blocks dealt longest causal chain (first block) first, the two halves of a split block adjacent
  int bh, item;
  if (order == 1) {
    deal(blockIdx.x, gridDim.x, (int)(gridDim.x / nxb), item, bh);
  } else {
    const int lin = xcd_linear(blockIdx.x, gridDim.x);  // the key-block halves of one (batch, head) share an XCD
    bh = lin / nxb;
    item = lin % nxb;
  }
  const int b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const bool idx32 = (uint64_t)(gridDim.x / nxb) * (uint64_t)Lq * (uint64_t)Lk <= 0xffffffffull;  // B·H = grid / nxb
  const int off = Lk - Lq;
  const int kblk = item / nsplit;
  const int split = item % nsplit, S = nsplit;  // this workgroup's share of the query tiles
  const int kb0 = kblk * KB;
  const int kw0 = kb0 + 32 * wave;  // this wave's first key
  const int key = kw0 + r;
  const bool kvalid = key < Lk && (kmask == nullptr || kmask[(int64_t)b * Lk + key] != 0);
  STAMP(0);

  // ---- prologue loads, all issued before any is consumed (one memory round trip): own keys' K / V fragments (B
  // operands of S and dP) and the K image of the whole key block (dQ = dS·K; rows clamped, zeroed when written) ----
  bf16x8 kf[HD / 16], vf[HD / 16];
  constexpr int KCH = KB * HD / 8;                       // 16-B chunks of the K image
  constexpr int KIMG = (KCH + THREADS - 1) / THREADS;  // per thread
  bf16x8 kimg[KIMG];
  {
    const int kk = min(key, Lk - 1);
    const __bf16* krow = k + ((int64_t)b * Lk + kk) * ld_in + hh * HD;
    const __bf16* vrow = v + ((int64_t)b * Lk + kk) * ld_in + hh * HD;
#pragma unroll
    for (int t = 0; t < HD / 16; ++t) {
      kf[t] = *reinterpret_cast<const bf16x8*>(krow + 16 * t + 8 * h);
      vf[t] = *reinterpret_cast<const bf16x8*>(vrow + 16 * t + 8 * h);
    }
#pragma unroll
    for (int i = 0; i < KIMG; ++i) {
      const int c = min(tid + THREADS * i, KCH - 1), row = c / (HD / 8), c8 = c % (HD / 8);
      const int kr = min(kb0 + row, Lk - 1);
      kimg[i] = *reinterpret_cast<const bf16x8*>(k + ((int64_t)b * Lk + kr) * ld_in + hh * HD + c8 * 8);
    }
  }

  f32x16 dka[HDP / 32], dva[HDP / 32];
#pragma unroll
  for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dka[dt][i] = dva[dt][i] = 0.f;
  if (HD < HDP) {  // hd = 16: image columns 16..31 of K, Q and dO stay zero (staging writes columns 0..15 only)
    for (int row = tid; row < KB + 2 * QT; row += THREADS) {
      __bf16* img = row < KB ? sK : row < KB + QT ? sQ : sD;
      const int rr = row < KB ? row : row < KB + QT ? row - KB : row - KB - QT;
      *reinterpret_cast<bf16x8*>(img + IQ::off(rr, HD)) = zero8();
      *reinterpret_cast<bf16x8*>(img + IQ::off(rr, HD + 8)) = zero8();
    }
  }

  const int kbend = min(Lk, kb0 + KB) - 1;  // last key of the block
  const int qlo = max(0, kb0 - off);
  const int qhi = window ? min(Lq - 1, kbend + window - 1 - off) : Lq - 1;
  const bool direct = dq32 == nullptr;  // this workgroup holds every key of the (batch, head)
  // otherwise this key block's partial dQ goes to its own f32 slab (plain stores, summed in dq_convert_kernel)
  float* dq_part = direct ? nullptr : dq32 + (int64_t)kblk * dq_slab;
  auto tile_q0 = [&](int it, int s) { return (qlo / QT + split_tile(it, s, S)) * QT; };

  // Query-tile prefetch: one 16-B chunk of Q, dO and O per thread (QT*HD/8 <= THREADS chunks per tile), the row's
  // lse / validity for the chunk-0 thread and one keep word per thread. Issued one tile ahead, written to LDS at the
  // top of the tile.
  constexpr int NCHUNK = QT * HD / 8;
  const bool stager = tid < NCHUNK;  // whole waves (NCHUNK is a multiple of 64)
  const int srow = tid / (HD / 8), sc8 = tid % (HD / 8);
  const bool zstager = bits && tid < QT * NKW;
  const int zw = tid / QT, zrow = tid % QT;  // keep word zw of query row zrow (LDS image [word][query])
  bf16x8 pq = zero8(), pd = zero8(), po = zero8();
  float pl = INFINITY;
  uint32_t pz = 0;
  auto prefetch = [&](int q0) {
    const int qi = q0 + srow;
    const bool in = stager && qi < Lq;
    pq = pd = po = zero8();
    pl = INFINITY;
    if (in) {
      pq = *reinterpret_cast<const bf16x8*>(q + ((int64_t)b * tq + qi) * ld_in + hh * HD + sc8 * 8);
      pd = *reinterpret_cast<const bf16x8*>(dout + ((int64_t)b * Lq + qi) * ld_do + hh * HD + sc8 * 8);
      po = *reinterpret_cast<const bf16x8*>(o + ((int64_t)b * Lq + qi) * ld_o + hh * HD + sc8 * 8);
      if (sc8 == 0 && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0)) pl = lse[(int64_t)bh * Lq + qi];
    }
    const int zq = q0 + zrow, zc = (kb0 >> 5) + zw;
    pz = (zstager && zq < Lq && zc < nw) ? keep[((int64_t)bh * Lq + zq) * nw + zc] : 0u;
  };
  int q0 = tile_q0(0, split);
  if (q0 <= qhi) prefetch(q0);
  if (key >= Lk) {
#pragma unroll
    for (int t = 0; t < HD / 16; ++t) kf[t] = vf[t] = zero8();
  }
#pragma unroll
  for (int i = 0; i < KIMG; ++i) {
    const int c = tid + THREADS * i, row = c / (HD / 8), c8 = c % (HD / 8);
    if (c < KCH) *reinterpret_cast<bf16x8*>(sK + IQ::off(row, c8 * 8)) = kb0 + row < Lk ? kimg[i] : zero8();
  }
  STAMP(1);

  for (int it = 0;; ++it) {
    q0 = tile_q0(it, split);
    if (q0 > qhi) break;
    __syncthreads();  // the previous tile's reads of sQ / sD / sS / sZ are done
    STAMP(2 + 6 * it);
    if (stager) {
      *reinterpret_cast<bf16x8*>(sQ + IQ::off(srow, sc8 * 8)) = pq;
      *reinterpret_cast<bf16x8*>(sD + IQ::off(srow, sc8 * 8)) = pd;
      float dl = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) dl = fmaf((float)pd[j], (float)po[j], dl);
      // δ: sum over the HD/8 consecutive threads of the row (rows never straddle a wave)
#pragma unroll
      for (int o2 = 1; o2 < HD / 8; o2 <<= 1) dl += __shfl_xor(dl, o2, 64);
      if (sc8 == 0) {
        sL[srow] = pl;  // +inf for invalid / missing queries: P = exp(S - inf) = 0 for the row
        sDl[srow] = pl == INFINITY ? 0.f : dl;
      }
    }
    if (zstager) sZ[tid] = pz;
    __syncthreads();
    STAMP(3 + 6 * it);
    {
      const int qn = tile_q0(it + 1, split);
      if (qn <= qhi) prefetch(qn);  // in flight during this tile's MFMAs
    }

    // ---- per wave: S, dP, dV, dK for its 32 keys over the tile's queries (slices not interleaved: register
    // pressure) ----
#pragma unroll 1
    for (int qs = 0; qs < QT / 32; ++qs) {
      const int qa = q0 + 32 * qs;  // first query of the slice
      const int qpos_lo = qa + off, qpos_hi = min(qa + 31, Lq - 1) + off;
      const bool any = qa < Lq && qpos_hi >= kw0 && kw0 < Lk && (window == 0 || qpos_lo - (kw0 + 31) < window);
      f32x16 s, dp;
      if (any) {
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
        constexpr float kLog2e = 1.4426950408889634f;
        // fully visible slice: every key of the wave valid and inside the causal / local band of every query
        const bool full = __ballot(kvalid) == ~0ull && qpos_lo >= kw0 + 31 && (window == 0 || qpos_hi - kw0 < window);
        float zk[16];  // dropout multipliers of this lane's (query row, key) elements (DROP_HASH)
        const uint32_t* zrow_w = sZ + wave * QT + 32 * qs;  // DROP_BITS: this wave's keep words of the slice's rows
        if (bits) {
        } else if (DROP && idx32) {  // 32-bit element indices (wave-uniform): the same hashes without 64-bit math
          if ((Lk & 1) == 0 && (kw0 & 1) == 0) {
            const int odd = key & 1;
            const uint32_t base = ((uint32_t)bh * (uint32_t)Lq + (uint32_t)q0) * (uint32_t)Lk + (uint32_t)(key - odd);
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
              const uint32_t e = base + (uint32_t)(32 * qs + acc_row(i + odd, h)) * (uint32_t)Lk;
              const uint32_t mine = mix32((e >> 1) ^ dr.key);
              const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
              const uint32_t ha = odd ? other : mine, hb = odd ? mine : other;
              const uint32_t ua = odd ? (ha >> 16) : (ha & 0xffffu), ub = odd ? (hb >> 16) : (hb & 0xffffu);
              zk[i] = ua >= dr.thresh ? dr.scale : 0.f;
              zk[i + 1] = ub >= dr.thresh ? dr.scale : 0.f;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              zk[i] = dropout_mult_32(dr, ((uint32_t)bh * (uint32_t)Lq + (uint32_t)(q0 + 32 * qs + acc_row(i, h))) *
                                              (uint32_t)Lk + (uint32_t)key);
          }
        } else if (DROP) {
          if ((Lk & 1) == 0 && (kw0 & 1) == 0) {
            // lanes r, r^1 hold keys 2j, 2j+1 (one hash pair) of the same query rows: for each pair of rows the
            // even lane hashes the first row, the odd lane the second, and they swap hashes (one hash per element
            // pair instead of per element)
            const int odd = key & 1;
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
              const int ql = 32 * qs + acc_row(i + odd, h);
              const uint64_t e = ((uint64_t)bh * (uint64_t)Lq + (uint64_t)(q0 + ql)) * (uint64_t)Lk + (uint64_t)(key - odd);
              const uint32_t mine = dropout_hash(dr.key, e >> 1);
              const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
              const uint32_t ha = odd ? other : mine, hb = odd ? mine : other;
              const uint32_t ua = odd ? (ha >> 16) : (ha & 0xffffu), ub = odd ? (hb >> 16) : (hb & 0xffffu);
              zk[i] = ua >= dr.thresh ? dr.scale : 0.f;
              zk[i + 1] = ub >= dr.thresh ? dr.scale : 0.f;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              zk[i] = dropout_mult(dr, ((uint64_t)bh * (uint64_t)Lq + (uint64_t)(q0 + 32 * qs + acc_row(i, h))) *
                                           (uint64_t)Lk + (uint64_t)key);
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int ql = 32 * qs + acc_row(i, h);
          const int qpos = q0 + ql + off;
          const float e = __builtin_amdgcn_exp2f(s[i] * kLog2e);
          const bool ok = full | (kvalid & (key <= qpos) & ((window == 0) | (qpos - key < window)));
          const float p = ok ? e : 0.f;
          if (DROP) {
            const float z = bits ? (((zrow_w[ql - 32 * qs] >> r) & 1u) ? dr.scale : 0.f) : zk[i];
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
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) dp[i] = 0.f;
      }
      // dS -> LDS [key][q] (4 consecutive queries per register group: one 8-byte store each)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (__bf16)dp[4 * gg + j];
        *reinterpret_cast<bf16x4*>(sS + IS::off(32 * wave + r, 32 * qs + 8 * gg + 4 * h)) = w;
      }
    }
    STAMP(4 + 6 * it);
    __syncthreads();
    STAMP(5 + 6 * it);

    // ---- dQ[q][d] = Σ_key dS[q][key] · K[key][d] for the tile: one 32x32 output tile per wave ----
    constexpr int NT = (QT / 32) * (HDP / 32);
    if (wave < NT) {
      const int qsub = wave % (QT / 32), dsub = wave / (QT / 32);
      const int qpos_max = min(q0 + QT - 1, Lq - 1) + off;
      const int nkeys = min(min(kbend, qpos_max) - kb0 + 1, KB);  // keys past the causal bound contribute 0
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      if (direct) {
        // dQᵀ[d][q] = Kᵀ·dSᵀ: the query on the lane, 16-B row stores of the bf16 result
        for (int t = 0; t < (nkeys + 15) / 16; ++t) {
          const int kr = 16 * t + 8 * (g >> 1) + q4;
          const int qc = 32 * qsub + 16 * (g & 1) + 4 * p4, dc = 32 * dsub + 16 * (g & 1) + 4 * p4;
          const bf16x8 af = join(tr_read(sS + IS::off(kr, qc)), tr_read(sS + IS::off(kr + 4, qc)));
          const bf16x8 bf = join(tr_read(sK + IQ::off(kr, dc)), tr_read(sK + IQ::off(kr + 4, dc)));
          acc = mfma(bf, af, acc);
        }
        const int qi = q0 + 32 * qsub + r;
        STAMP(6 + 6 * it);
        if (qi < Lq) store_col32<HD < 32 ? HD : 32>(dq + ((int64_t)b * tq + qi) * ld_d + hh * HD + 32 * dsub, acc, h);
        STAMP(7 + 6 * it);
      } else {
        // dQ[q][d] = dS·K: the head dim on the lane, so that each store instruction writes two 128-B rows of the
        // key block's partial (no atomics: the slabs are summed per row in key-block order, deterministic)
        for (int t = 0; t < (nkeys + 15) / 16; ++t) {
          const int kr = 16 * t + 8 * (g >> 1) + q4;
          const int qc = 32 * qsub + 16 * (g & 1) + 4 * p4, dc = 32 * dsub + 16 * (g & 1) + 4 * p4;
          const bf16x8 af = join(tr_read(sS + IS::off(kr, qc)), tr_read(sS + IS::off(kr + 4, qc)));
          const bf16x8 bf = join(tr_read(sK + IQ::off(kr, dc)), tr_read(sK + IQ::off(kr + 4, dc)));
          acc = mfma(af, bf, acc);
        }
        const int d = 32 * dsub + r;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qi = q0 + 32 * qsub + acc_row(i, h);
          if (qi < Lq && d < HD) dq_part[((int64_t)bh * Lq + qi) * HD + d] = acc[i];
        }
      }
    }
  }

  STAMP(40);
  // ---- the key block's two query-split workgroups hold partial dKᵀ / dVᵀ: exchange and add ----
  // The first to finish publishes its partial (write-through sc1 stores, drained, then an sc1 flag); the second
  // polls the flag (relaxed sc1 loads + s_sleep), reads the partial with sc1 loads, adds it in registers and stores
  // the bf16 result. Two-term f32 sums commute, so the result does not depend on which one finishes first.
  if (nsplit > 1) {
    const int64_t id = (int64_t)bh * (nxb / nsplit) + kblk;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int kSC1 = 16;  // buffer cache policy: sc1 (write-through stores, L1-bypassing loads)
    // [dk | dv] f32 slab of this pair, [wave][dt][i/4][lane] x 16 B (coalesced per store / load instruction)
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(xbuf + id * (2 * KB * HDP), (short)0, 2 * KB * HDP * 4, 0x00020000);
    int* flag = reinterpret_cast<int*>(smem_raw);
    __syncthreads();  // every wave is done with the LDS images
    if (tid == 0) *flag = __hip_atomic_fetch_add(xcnt + 2 * id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool first = *flag == 0;
    if (first) {
#pragma unroll
      for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const int e = 4 * (((wave * (HDP / 32) + dt) * 4 + i / 4) * 64 + lane);  // float index, 16-B granules
          const u32x4 k4 = {__float_as_uint(dka[dt][i]), __float_as_uint(dka[dt][i + 1]),
                            __float_as_uint(dka[dt][i + 2]), __float_as_uint(dka[dt][i + 3])};
          const u32x4 v4 = {__float_as_uint(dva[dt][i]), __float_as_uint(dva[dt][i + 1]),
                            __float_as_uint(dva[dt][i + 2]), __float_as_uint(dva[dt][i + 3])};
          __builtin_amdgcn_raw_buffer_store_b128(k4, xr, 4 * e, 0, kSC1);
          __builtin_amdgcn_raw_buffer_store_b128(v4, xr, 4 * (KB * HDP + e), 0, kSC1);
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(xcnt + 2 * id + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(xcnt + 2 * id + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(xcnt + 2 * id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // leave the pair zeroed
      __hip_atomic_store(xcnt + 2 * id + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        const int e = 4 * (((wave * (HDP / 32) + dt) * 4 + i / 4) * 64 + lane);
        const u32x4 k4 = __builtin_amdgcn_raw_buffer_load_b128(xr, 4 * e, 0, kSC1);
        const u32x4 v4 = __builtin_amdgcn_raw_buffer_load_b128(xr, 4 * (KB * HDP + e), 0, kSC1);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          dka[dt][i + c] += __uint_as_float(k4[c]);
          dva[dt][i + c] += __uint_as_float(v4[c]);
        }
      }
  }
  // ---- dK, dV (every key belongs to exactly one workgroup): 16-B row stores ----
  if (key < Lk) {
    __bf16* ko = dk + ((int64_t)b * Lk + key) * ld_d + hh * HD;
    __bf16* vo = dv + ((int64_t)b * Lk + key) * ld_d + hh * HD;
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt) {
      store_col32<HD < 32 ? HD : 32>(ko + 32 * dt, dka[dt], h);
      store_col32<HD < 32 ? HD : 32>(vo + 32 * dt, dva[dt], h);
    }
  }
  STAMP(41);
}

// dq (bf16, rows strided by tq) <- Σ_kb dq32[kb] (f32 [nkb][B*H, Lq, HD]) over the key blocks whose workgroups wrote
// the row's query tile (the tiles [qlo, qhi] of attn_bwd_kernel), in key-block order.
template <int HD>
__global__ __launch_bounds__(256) void dq_convert_kernel(const float* __restrict__ dq32, __bf16* __restrict__ dq,
                                                         int64_t ld_d, int64_t tq, int H, int Lq, int Lk, int window,
                                                         int64_t n4) {
  constexpr int QT = Cfg<HD>::QT;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t e = 4 * i;
  const int d = (int)(e % HD);
  const int64_t rowi = e / HD;  // (bh, qi)
  const int qi = (int)(rowi % Lq);
  const int64_t bh = rowi / Lq;
  const int b = (int)(bh / H), hh = (int)(bh % H);
  const int off = Lk - Lq, nkb = (Lk + KB - 1) / KB, tile = qi / QT;
  float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kb = 0; kb < nkb; ++kb) {
    const int kb0 = kb * KB, kbend = min(Lk, kb0 + KB) - 1;
    const int qlo = max(0, kb0 - off), qhi = window ? min(Lq - 1, kbend + window - 1 - off) : Lq - 1;
    if (qlo > qhi || tile < qlo / QT || tile > qhi / QT) continue;
    const float4 v = *reinterpret_cast<const float4*>(dq32 + (int64_t)kb * n4 * 4 + e);
    x.x += v.x, x.y += v.y, x.z += v.z, x.w += v.w;
  }
  bf16x4 w;
  w[0] = (__bf16)x.x; w[1] = (__bf16)x.y; w[2] = (__bf16)x.z; w[3] = (__bf16)x.w;
  *reinterpret_cast<bf16x4*>(dq + ((int64_t)b * tq + qi) * ld_d + hh * HD + d) = w;
}

template <int HD, int DM>
int set_lds_attr() {
  return hipFuncSetAttribute((const void*)attn_bwd_kernel<HD, DM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             Cfg<HD>::LDS_BYTES) == hipSuccess
             ? 0
             : 1;
}

// The split backward (attention_bwd2.hip: dK / dV kernel + dQ kernel, no partial sums) for more than one key block
// of the fused kernel, where that kernel's per-key-block f32 dQ partials dominate its traffic. ESGPT_ATTN_BWD_SPLIT2
// tuning hook (read once): 0 = never, 1 = always, 64 / 128 = always with that many keys per dK / dV workgroup.
constexpr int64_t kSplit64MinLk = 2048;
int split2_keys(int64_t Lk, int64_t hd, bool drop) {
  static const int forced = [] {
    const char* e = tuning_env("ESGPT_ATTN_BWD_SPLIT2");
    return e ? atoi(e) : -1;
  }();
  if (forced == 0) return 0;
  if (forced == 64 || forced == 128) return forced;
  if (forced == 1) return 128;
  // measured (tools/attn_split_ab.py, profiles/r05_attn_split_ab.log): faster past one key block at hd = 16 and 128
  // (L = 520 local-40: 20.0 -> 15.6 us; L = 600: 161.6 -> 118.9 us). hd = 64: round 6's split kernels (dQ: buffer-load
  // staging, one allowed-key word per lane and tile; dK / dV: keep bits folded into a 16-bit lane mask, 32-query tiles
  // with keep bits) win in isolation (tools/attn_split2_ab.sh, profiles/r06_attn_split2_ab3.log: C5 133 -> 109 us,
  // L = 4096 479 -> 430 us), but inside the C3 / C5 training steps (dropout, keep bits) they lose: C5 3.767 vs 3.845
  // ms/step, C3 10.79 vs 10.86 alternating on one box (profiles/r06_split_step_ab.log; in-step per layer the split
  // pair takes 76.7 + 41.3 us against the fused kernel's 93.8 + 9.8, profiles/r06_c5_*_bwd_kernel_stats.csv). So at
  // hd 64 the split form runs only without dropout past kSplit64MinLk keys (the long-sequence case, where the fused
  // kernel's per-key-block dQ partials reach 925 MB at L = 4096: 300 MB with the split pair).
  // hd = 128: always (the fused kernel's 512-thread workgroups cap it at 256 registers, where its hd-128 instances
  // spilled 464-572 B per lane to scratch; the split kernels run one wave per SIMD at hd 128 and do not spill)
  return ((Lk > KB && hd == 16) || (Lk >= kSplit64MinLk && hd == 64 && !drop) || hd == 128) ? 128 : 0;
}

template <int HD>
int launch(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o, int64_t ld_o,
           const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask, const uint8_t* qmask, void* dq,
           void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t window,
           float drop_p, const uint64_t* seed, const uint32_t* keep, float* dq32, int32_t* counters, hipStream_t st) {
  if (const int kpw = split2_keys(Lk, HD, drop_p > 0.f))
    return esgpt_attn_bwd_mfma_split(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H,
                                     Lq, Lk, HD, window, drop_p, seed, keep, kpw, st);
  constexpr int lds = Cfg<HD>::LDS_BYTES;
  static bool attr = false;
  if (!attr) {
    if (set_lds_attr<HD, DROP_NONE>() || set_lds_attr<HD, DROP_HASH>() || set_lds_attr<HD, DROP_BITS>())
      return ESGPT_ERR_LAUNCH;
    attr = true;
  }
  const int nkb = (int)cdiv(Lk, KB);
  float* acc = nkb > 1 ? dq32 : nullptr;
  // Two workgroups per key block (the zig-zag query-tile split, partial dKᵀ / dVᵀ exchanged through write-through
  // slabs: 2 x 128 KB per pair at hd = 64) only where the parallelism pays for that exchange: no more key-block
  // workgroups than CUs, or a causal chain of at least 16 query tiles for the first key block. Measured
  // (tools/attn_bench.py, dropout 0.1): C2 (128 key blocks) 29.5 vs 30.2 us split / not; C3 L=512 H=8 global
  // (512 blocks) 161 vs 130 us, local-32 121 vs 81 us; L=4096 B=4 H=8 (512 blocks, 64-tile chains) 574 vs 819 us.
  // C5 (L = 1024, 256 blocks: one per CU) measured 134 vs 123 us in isolation before the longest-chain-first order;
  // with it, the C5 step is 3.4 % faster split (4.065 -> 3.926 ms, profiles/r05b_c5_sweep.log), hence "no more
  // than". (ESGPT_ATTN_BWD_NSPLIT=1 / 2: forced — tuning hook, read once.)
  static const int forced_split = [] {
    const char* e = tuning_env("ESGPT_ATTN_BWD_NSPLIT");
    return e ? atoi(e) : 0;
  }();
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int64_t chain = window > 0 ? std::min<int64_t>(Lq, KB + window) : Lq;  // queries seen by one key block
  const bool want_split = forced_split ? forced_split == 2 : (nkb * B * H <= n_cu || chain >= 1024);
  const int nsplit = (counters && Lq > Cfg<HD>::QT && want_split) ? 2 : 1;
  const int64_t slab = B * H * Lq * HD;  // one f32 dQ partial per key block (nkb > 1)
  static const int order = [] {  // workgroup order: ESGPT_ATTN_ORDER tuning hook, read once
    const char* e = tuning_env("ESGPT_ATTN_ORDER");
    return e ? atoi(e) : 1;  // longest chain first: profiles/r05_attn_order_ab.log
  }();
  float* xbuf = dq32 + (nkb > 1 ? (size_t)(nkb * slab) : 0);
  const dim3 grid((unsigned)(nkb * nsplit * B * H));  // 1-D: XCD-aware order in the kernel
  const int nw = (int)cdiv(Lk, 32);
#define ESGPT_ATTN_BWD_LAUNCH(DM_)                                                                                 \
  attn_bwd_kernel<HD, DM_><<<grid, THREADS, lds, st>>>(                                                           \
      (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, ld_in, tq, (const __bf16*)o, ld_o, (const __bf16*)dout, \
      ld_do, lse, kmask, qmask, (__bf16*)dq, (__bf16*)dk, (__bf16*)dv, ld_d, acc, (int)H, (int)Lq, (int)Lk,         \
      (int)window, drop_p, seed, keep, nw, nsplit, counters, xbuf, slab, order)
  if (!(drop_p > 0.f)) ESGPT_ATTN_BWD_LAUNCH(DROP_NONE);
  else if (keep) ESGPT_ATTN_BWD_LAUNCH(DROP_BITS);
  else ESGPT_ATTN_BWD_LAUNCH(DROP_HASH);
#undef ESGPT_ATTN_BWD_LAUNCH
  if (acc) {
    const int64_t n4 = B * H * Lq * HD / 4;
    dq_convert_kernel<HD><<<(unsigned)cdiv(n4, 256), 256, 0, st>>>(acc, (__bf16*)dq, ld_d, tq, (int)H, (int)Lq,
                                                                   (int)Lk, (int)window, n4);
  }
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

}  // namespace

#ifdef ESGPT_STAMPS
extern "C" int esgpt_debug_stamps(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(uint64_t) * 64) == hipSuccess ? 0 : 1;
}
#endif

// f32 dQ partials, one per key block (more than one key block) + the dK / dV exchange slabs of the query-split pairs.
size_t esgpt_attn_bwd_mfma_workspace(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd) {
  if (split2_keys(Lk, hd, true)) return 0;  // the split backward needs none (asked as with dropout: the fused
                                             // kernel's workspace whenever either may run)
  const size_t dq = Lk > KB ? sizeof(float) * (size_t)(cdiv(Lk, KB) * B * H * Lq * hd) : 0;
  const int64_t hdp = hd < 32 ? 32 : hd;  // exchange slabs hold the padded accumulator tiles
  return dq + sizeof(float) * (size_t)(B * H * cdiv(Lk, KB)) * 2 * KB * hdp;
}

int64_t esgpt_attn_bwd_mfma_counters(int64_t B, int64_t H, int64_t Lk) { return 2 * B * H * cdiv(Lk, KB); }

int esgpt_attn_bwd_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                        int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                        const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                        const uint32_t* keep, float* dq32, int32_t* counters, hipStream_t st) {
  if (hd == 16)
    return launch<16>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, Lk,
                      window, drop_p, seed, keep, dq32, counters, st);
  if (hd == 32)
    return launch<32>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, Lk,
                      window, drop_p, seed, keep, dq32, counters, st);
  if (hd == 64)
    return launch<64>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, Lk,
                      window, drop_p, seed, keep, dq32, counters, st);
#ifdef ESGPT_TUNING_HOOKS
  return launch<128>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H, Lq, Lk,
                     window, drop_p, seed, keep, dq32, counters, st);
#else
  // hd = 128 always takes the split backward (split2_keys); the fused hd-128 kernel is built in the tools build only
  return esgpt_attn_bwd_mfma_split(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, dq, dk, dv, ld_d, B, H,
                                   Lq, Lk, 128, window, drop_p, seed, keep, 128, st);
#endif
}
