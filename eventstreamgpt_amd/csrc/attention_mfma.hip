// bf16 MFMA flash attention forward for gfx950 (InnerSelfAttention._attn, transformer.py:171-217), hd in {16, 32,
// 64, 128}; the fused backward (dQ, dK, dV in one kernel) is attention_bwd.hip. hd = 16 (C1: hidden 64 over 4 heads)
// is exactly one K = 16 step of S = K·Qᵀ; its P·V product runs on a 32-wide V image whose columns 16..31 stay zero.
//
// v_mfma_f32_32x32x16_bf16 with the query on the MFMA lane, so the per-row softmax statistics are lane-local (no
// cross-lane row reductions beyond one xor-32 exchange):
//   Sᵀ[key][q] = K·Qᵀ  (A = K rows from LDS, B = Q fragments in registers)
//   Oᵀ[d][q]  += Vᵀ·Pᵀ (A = Vᵀ tile in LDS read in the permuted key order, B = P straight from the Sᵀ accumulator
//                       registers converted to bf16 — no LDS round trip for P)
// Fragment maps (gfx950, 32x32x16 bf16): lane l = (r = l&31, h = l>>5); A[row r][k = 8h+j], B[k = 8h+j][col r];
// C/D reg i holds row (i&3) + 8(i>>2) + 4h, col r. An accumulator used as the next B operand supplies, for k-step s,
// element j of half h = row 16s + 8(j>>2) + 4h + (j&3); the A operand is read from LDS in that same key order.
//
// Work decomposition (forward): one 256-thread workgroup per 64-query block of one (batch, head), two waves per
// query half splitting its key tiles by parity; K/V tiles of 64 rows are staged in LDS in pairs. Causal /
// local-window / fully-padded key tiles are skipped.
// Roofline: MFMA-bound at large L (algorithmic FLOPs: fwd 4*H*hd*T, bwd 8*H*hd*T, T = allowed (q,k) pairs).
#include <type_traits>

#include "attn_common.h"
#include "common.h"

using namespace esgpt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ROWS = 64;   // rows per workgroup block and per staged tile
constexpr int THREADS = 256;  // forward workgroup: 4 waves

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// Stores one lane's 32 accumulator-row values (x[i] = row acc_row(i, h)) as bf16 into dst[0 .. N-1] (N = 32, or 16
// for hd = 16: rows 0..15 only) with 16-B stores, joining register groups g, g+1 across the half-waves with
// v_permlane32_swap.
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

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.f;
  return z;
}

// Accumulator registers 8s..8s+7 -> bf16 operand fragment (permuted k order, see header).
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
  return f;
}

// A-operand fragment from a transposed LDS tile T[row][col] (row stride `ld` elements), for the 32-column
// sub-block starting at c0 and k-step s: cols c0 + 16s + 4h + {0..3} and c0 + 16s + 8 + 4h + {0..3}.
__device__ __forceinline__ bf16x8 perm_frag(const __bf16* T, int ld, int row, int c0, int s, int h) {
  const __bf16* p = T + row * ld + c0 + 16 * s + 4 * h;
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 8);
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

__device__ __forceinline__ bool allowed(int key, int qpos, int window) {
  return key <= qpos && (window == 0 || qpos - key < window);
}

// Maximum of a lane's 32 scores as four independent max chains joined at the end (depth 6 instead of a 32-deep chain;
// the compiler forms v_max3_f32). Not inline asm: the compiler does not insert the MFMA-result -> VALU wait states in
// front of an asm statement that reads an accumulator (measured: intermittently wrong maxima at hd 16, where the
// max follows a single MFMA).
__device__ __forceinline__ float max3_f32(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
// Masks a lane's 32 scores of one 64-key tile without branches: the lane's allowed keys as one 64-bit word (the tile's
// valid-key ballot, the causal limit key <= qpos, the local window qpos - key < window, the query's validity), then
// one bit test per element at a compile-time position (the half-wave's 4-row offset is shifted out first).
__device__ __forceinline__ void mask_tile(f32x16 (&s)[2], uint64_t kbits, bool qvalid, int rel, int window, int h) {
  // rel = qpos - t0: key t0 + j is causally visible iff j <= rel, inside the window iff j > rel - window
  uint64_t am = qvalid ? kbits : 0ull;
  am &= rel >= 63 ? ~0ull : (rel < 0 ? 0ull : ((2ull << rel) - 1ull));
  if (window) {
    const int lo = rel - window + 1;  // smallest visible j
    am &= lo <= 0 ? ~0ull : (lo > 63 ? 0ull : ~((1ull << lo) - 1ull));
  }
  const uint64_t okm = am >> (4 * h);
  const uint32_t w0 = (uint32_t)okm, w1 = (uint32_t)(okm >> 32);
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pos = (i & 3) + 8 * (i >> 2);  // acc_row(i, 0)
      const uint32_t w = c ? w1 : w0;
      s[c][i] = ((w >> pos) & 1u) ? s[c][i] : -INFINITY;
    }
}

__device__ __forceinline__ float row_max32(const f32x16 (&s)[2]) {
  float a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = k >> 1, i0 = 8 * (k & 1);
    float x = max3_f32(s[c][i0], s[c][i0 + 1], s[c][i0 + 2]);
    x = max3_f32(x, s[c][i0 + 3], s[c][i0 + 4]);
    x = max3_f32(x, s[c][i0 + 5], s[c][i0 + 6]);
    a[k] = max3_f32(x, s[c][i0 + 7], s[c][i0 + 7]);
  }
  return max3_f32(max3_f32(a[0], a[1], a[2]), a[3], a[3]);
}

// Dropout element counter, identical to the generic kernels': (bh * Lq + q) * Lk + key.
__device__ __forceinline__ uint64_t elem_index(int bh, int Lq, int Lk, int qi, int kj) {
  return ((uint64_t)bh * (uint64_t)Lq + (uint64_t)qi) * (uint64_t)Lk + (uint64_t)kj;
}

// ------------------------------------------------------------------------------------------------------------
// V image row stride for ds_read_b64_tr_b16 (elements): 4 consecutive rows must land 16 dwords apart (mod 64)
// so that a 32-lane half reading 4 rows x 32 columns touches all 64 banks once.
template <int HD>
struct VImg {
  static constexpr int LD = (HD <= 32) ? 32 : 160;
};

__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)p);
}

// ------------------------------------------------------------------------------------------------------------
// Forward. One 256-thread workgroup (4 waves) per 64-query block of one (batch, head): wave w owns queries
// 32·(w&1) .. +31 of the block and the 64-key tiles of parity w>>1 (tiles t, t+128, … and t+64, t+192, …), so two
// waves walk the causal key range of each query half in parallel (half the serial chain of a 2-wave block) and
// merge their online-softmax states (max, sum, O) through LDS at the end. K is staged row-major (A operand of
// Sᵀ = K·Qᵀ by 16-B row reads); V row-major too, read as the transposed A operand of Oᵀ += Vᵀ·Pᵀ with
// ds_read_b64_tr_b16 (no transposing LDS writes). The next pair of K/V tiles is prefetched into registers while the
// current pair is consumed. Key validity is a 64-bit ballot per tile; tiles that are fully valid and fully inside the
// causal / local band skip the per-element masks. Softmax in the exp2 domain (v_exp_f32).
// IDX64: some element counter of the launch exceeds 32 bits (the dropout hash then runs on 64-bit counters); a
// template parameter, so each instance carries one hash path (with both, the hd-64 dropout instance spilled).
template <int HD, bool DROP, bool IDX64 = false>
__global__ __launch_bounds__(THREADS, HD == 128 ? 1 : 2) void attn_fwd_mfma_kernel(const __bf16* __restrict__ q,
                                                               const __bf16* __restrict__ k,
                                                               const __bf16* __restrict__ v, int64_t ld_in, int64_t tq,
                                                               __bf16* __restrict__ o, int64_t ld_o,
                                                               float* __restrict__ lse,
                                                               const uint8_t* __restrict__ kmask,
                                                               const uint8_t* __restrict__ qmask, int H, int Lq,
                                                               int Lk, int window, float drop_p,
                                                               const uint64_t* __restrict__ seed,
                                                               uint32_t* __restrict__ keep, int nw, int order) {
  constexpr int HDP = HD < 32 ? 32 : HD;           // output (P·V) width: hd = 16 runs one 32-wide tile
  constexpr int NP = HD + 8, VLD = VImg<HD>::LD;
  constexpr int CH = HD / 8;                        // 16-B chunks per row
  constexpr int NLD = 2 * ROWS * CH / THREADS;      // chunks per thread and tensor for a pair of tiles
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  // [2 tiles][ROWS][NP] K and [2 tiles][ROWS][VLD] V images; the K image doubles as the merge buffer at the end
  constexpr int kMergeElems = 2 * (2 * (HDP / 32) * 16 * 64 + 4 * 64);  // bf16 elements holding the f32 merge state
  constexpr int kSK = 2 * ROWS * NP > kMergeElems ? 2 * ROWS * NP : kMergeElems;
  __shared__ __attribute__((aligned(16))) __bf16 sK[kSK];
  __shared__ __attribute__((aligned(16))) __bf16 sV[2 * ROWS * VLD];
  static_assert(NLD >= 1, "tile pair staging");

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int qh = wave & 1, kp = wave >> 1;
  const int nqb = (Lq + ROWS - 1) / ROWS;
  // order 0: XCD-contiguous runs, query blocks ascending per (batch, head); order 1: the (batch, head)s of one XCD
  // kept together and their query blocks dealt longest causal chain (last block) first
  int bh, qbi;
  if (order == 1) {
    int rank;
    esgpt::attnb::deal(blockIdx.x, gridDim.x, (int)(gridDim.x / nqb), rank, bh);
    qbi = nqb - 1 - rank;
  } else {
    const int lin = xcd_linear(blockIdx.x, gridDim.x);  // the query blocks of one (batch, head) share an XCD
    bh = lin / nqb;
    qbi = lin % nqb;
  }
  const int b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  constexpr bool idx32 = !IDX64;
  const int off = Lk - Lq;
  const int qb = qbi * ROWS;
  const int qi = qb + qh * 32 + r;
  const bool qin = qi < Lq;
  const bool qvalid = qin && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0);
  const int qpos = qi + off;
  const int qlo_w = qb + qh * 32 + off;                      // smallest query position of this wave
  const int qhi_w = min(qb + qh * 32 + 31, Lq - 1) + off;    // largest
  const __bf16* myK = sK + kp * ROWS * NP;
  const __bf16* myV = sV + kp * ROWS * VLD;

  bf16x8 qf[HD / 16];
  const __bf16* qrow = q + ((int64_t)b * tq + qi) * ld_in + hh * HD;
#pragma unroll
  for (int t = 0; t < HD / 16; ++t)
    qf[t] = qin ? *reinterpret_cast<const bf16x8*>(qrow + 16 * t + 8 * h) : zero8();

  if (HD < HDP) {  // hd = 16: V image columns 16..31 are zeros for the whole kernel (never staged over)
    for (int i = tid; i < 2 * ROWS; i += THREADS)
      *reinterpret_cast<bf16x8*>(sV + i * VLD + HD) = zero8(), *reinterpret_cast<bf16x8*>(sV + i * VLD + HD + 8) = zero8();
  }
  f32x16 oacc[HDP / 32];
#pragma unroll
  for (int dt = 0; dt < HDP / 32; ++dt) oacc[dt] = zero16();
  float m = -INFINITY, l = 0.f;  // running max (log2 domain) and normaliser

  const int qhi = min(Lq, qb + ROWS) - 1;
  const int kmax = min(Lk - 1, qhi + off);
  const int kmin = window ? max(0, qb + off - window + 1) : 0;
  const __bf16* kbase = k + (int64_t)b * Lk * ld_in + hh * HD;
  const __bf16* vbase = v + (int64_t)b * Lk * ld_in + hh * HD;
  const uint8_t* kmb = kmask ? kmask + (int64_t)b * Lk : nullptr;

  // pair of tiles (keys kt .. kt+127) -> registers by buffer loads whose range ends after row kmax: rows past it (never
  // visible to this block) read as zeros with no branch (esgpt_attn_mfma_supported: Lk·ld_in·2 < 2^31)
  bf16x8 rk[NLD], rv[NLD];
  const int rec = (kmax + 1) * (int)ld_in * 2;
  const __amdgpu_buffer_rsrc_t rsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(kbase), (short)0, rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(vbase), (short)0, rec, 0x00020000);
  auto load_pair = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + THREADS * i, row = c / CH, c8 = c % CH;
      const int vo = (kt + row) * (int)ld_in * 2 + c8 * 16;
      rk[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsk, vo, 0, 0));
      rv[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsv, vo, 0, 0));
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
    const int t0 = kt + ROWS * kp;          // this wave's tile
    const uint64_t kbits = __ballot(kok);   // 0 when the tile lies past kmax
    __syncthreads();                        // the previous pair's LDS reads are done
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + THREADS * i, row = c / CH, c8 = c % CH;
      *reinterpret_cast<bf16x8*>(sK + row * NP + c8 * 8) = rk[i];
      *reinterpret_cast<bf16x8*>(sV + row * VLD + c8 * 8) = rv[i];
    }
    __syncthreads();
    if (kt + 2 * ROWS <= kmax) {
      load_pair(kt + 2 * ROWS);
      kok = key_ok(kt + 2 * ROWS);
    }
    if (!kbits) continue;  // fully padded (or absent) key tile

    // one instance per FULL (tiles inside the causal / local band with every key valid skip the masks): a mask
    // applied under a runtime branch made the compiler copy all 32 scores on the unmasked path
    const bool full = kbits == ~0ull && t0 + ROWS - 1 <= qlo_w && (window == 0 || qhi_w - t0 < window);
    auto tile = [&](auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    f32x16 s[2] = {zero16(), zero16()};
#pragma unroll
    for (int t = 0; t < HD / 16; ++t)  // the two score chains interleaved (no back-to-back dependent MFMAs)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(myK + (32 * c + r) * NP + 16 * t + 8 * h);
        s[c] = mfma(a, qf[t], s[c]);
      }
    // row maximum of the raw scores (the log2(e) scaling is monotonic: max(s)·log2e = max(s·log2e) bit for bit),
    // then p = exp2(s·log2e − m) as one FMA per element (in the log2 domain: m = running max · log2e)
    if (!FULL) mask_tile(s, kbits, qvalid, qpos - t0, window, h);
    float mt = row_max32(s);
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * kLog2e;
    const float mnew = fmaxf(m, mt);
    const float alpha = (mnew == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
    const float msub = (mnew == -INFINITY) ? 0.f : mnew;
    float rsp[4] = {0.f, 0.f, 0.f, 0.f};  // four partial sums: no 32-deep add chain
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[c][i], kLog2e, -msub));  // exp2(-inf) = 0
        rsp[i & 3] += p;  // normaliser over undropped probabilities
        s[c][i] = p;
      }
    float rs = (rsp[0] + rsp[1]) + (rsp[2] + rsp[3]);
    if (DROP) {
      uint32_t kw[2] = {0u, 0u};  // keep bits of this lane's keys, at their key position within the 32-key group
      // registers (i, i+1), i even, hold consecutive keys: one hash per pair when the pair is aligned
      if constexpr (idx32) {  // every element index of the launch fits 32 bits
        const uint32_t rowbase = ((uint32_t)bh * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk;
        const bool aligned = (rowbase & 1) == 0;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            const uint32_t e = rowbase + (uint32_t)(t0 + 32 * c + acc_row(i, h));
            float m0, m1;
            if (aligned) {
              dropout_mult2_32(dr, e, m0, m1);
            } else {
              m0 = dropout_mult_32(dr, e);
              m1 = dropout_mult_32(dr, e + 1);
            }
            s[c][i] *= m0;
            s[c][i + 1] *= m1;
            kw[c] |= (m0 != 0.f ? 1u : 0u) << acc_row(i, h);
            kw[c] |= (m1 != 0.f ? 1u : 0u) << acc_row(i + 1, h);
          }
      } else {
        const uint64_t rowbase = ((uint64_t)bh * (uint64_t)Lq + (uint64_t)qi) * (uint64_t)Lk;
        const bool aligned = (rowbase & 1) == 0;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            const uint64_t e = rowbase + (uint64_t)(t0 + 32 * c + acc_row(i, h));
            float m0, m1;
            if (aligned) {
              dropout_mult2(dr, e, m0, m1);
            } else {
              m0 = dropout_mult(dr, e);
              m1 = dropout_mult(dr, e + 1);
            }
            s[c][i] *= m0;
            s[c][i + 1] *= m1;
            kw[c] |= (m0 != 0.f ? 1u : 0u) << acc_row(i, h);
            kw[c] |= (m1 != 0.f ? 1u : 0u) << acc_row(i + 1, h);
          }
      }
      if (keep != nullptr) {  // the backward reads these words instead of re-hashing: word (query, key / 32)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t w = kw[c] | (uint32_t)__shfl_xor((int)kw[c], 32, 64);
          const int wi = (t0 >> 5) + c;
          if (h == 0 && qin && wi < nw) keep[((int64_t)bh * Lq + qi) * nw + wi] = w;
        }
      }
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mnew;
    if (__ballot(alpha != 1.f))  // no lane's maximum moved (most tiles past the first): the O rescale is a no-op
#pragma unroll
      for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    // Vᵀ fragment by transposed reads: lane group g (16 lanes) reads keys 16ss + 4(g>>1) + {0..3} (+8) of
    // columns 32dt + 16(g&1) + {0..15}; the lane receives its column r, in the accumulator's permuted key order.
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pf = acc_frag(s[c], ss);
        const int row0 = 32 * c + 16 * ss + 4 * (g >> 1) + q4;
#pragma unroll
        for (int dt = 0; dt < HDP / 32; ++dt) {
          const __bf16* vp = myV + row0 * VLD + 32 * dt + 16 * (g & 1) + 4 * p4;
          const bf16x4 lo = tr_read(vp), hi = tr_read(vp + 8 * VLD);
          bf16x8 vf;
          vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
          vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
          oacc[dt] = mfma(vf, pf, oacc[dt]);
        }
      }
    };
    if (full) tile(std::true_type{});
    else tile(std::false_type{});
  }

  // ---- merge the two key parities of each query half (the odd-parity wave hands its state over in LDS) ----
  __syncthreads();  // every wave is done with the K / V images
  float* cO = reinterpret_cast<float*>(sK);   // [qh][HDP/32][16][64]
  float* cM = cO + 2 * (HDP / 32) * 16 * 64;  // [qh][64]
  float* cL = cM + 2 * 64;
  if (kp == 1) {
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) cO[((qh * (HDP / 32) + dt) * 16 + i) * 64 + lane] = oacc[dt][i];
    cM[qh * 64 + lane] = m;
    cL[qh * 64 + lane] = l;
  }
  __syncthreads();
  if (kp == 1) return;
  {
    const float m1 = cM[qh * 64 + lane], l1 = cL[qh * 64 + lane];
    const float mm = fmaxf(m, m1);
    const float a0 = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m - mm);
    const float a1 = (m1 == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m1 - mm);
    l = l * a0 + l1 * a1;
    m = mm;
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        oacc[dt][i] = oacc[dt][i] * a0 + cO[((qh * (HDP / 32) + dt) * 16 + i) * 64 + lane] * a1;
  }

  // the query's row, mask and validity recomputed here rather than kept live across the key loop (an opaque copy of
  // the thread id the compiler cannot fold into the pre-loop values: at 2 waves per SIMD the hd-64 dropout instance
  // otherwise spilled two of them to scratch)
  int tid2;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid2) : "v"(tid));
  const int qi_e = qb + qh * 32 + (tid2 & 31);
  const bool qin_e = qi_e < Lq;
  const bool qvalid_e = qin_e && (qmask == nullptr || qmask[(int64_t)b * Lq + qi_e] != 0);
  const bool ok = qvalid_e && l > 0.f;
  const float inv = ok ? 1.f / l : 0.f;
  if (qin_e) {
    __bf16* orow = o + ((int64_t)b * Lq + qi_e) * ld_o + hh * HD;
#pragma unroll
    for (int dt = 0; dt < HDP / 32; ++dt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= inv;
      store_col32<HD < 32 ? HD : 32>(orow + 32 * dt, oacc[dt], (tid2 >> 5) & 1);
    }
    if ((tid2 & 32) == 0) lse[(int64_t)bh * Lq + qi_e] = ok ? m * kLn2 + logf(l) : 0.f;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Forward, wide form (long sequences): one workgroup of NW waves per QB = 32·NU·NW-query block of one (batch, head);
// every wave owns NU 32-query slices and walks ALL of the block's 64-key tiles itself, so each K / V tile staged in
// LDS feeds NW waves (the parity form above: 2 per tile), and with NU = 2 every K / V fragment a wave reads from LDS
// feeds two MFMAs (two query slices). At long L the parity form is bound by the per-CU L2 -> LDS stream (≈128 B/clk
// per CU for the K / V pairs at the MFMA rate, against the ≈30-35 the CU sustains), which the wider reuse divides by
// NW / 2. K / V tiles are double-buffered in XOR-swizzled LDS images (attnb::Img: conflict-free 16-B row reads for K,
// ds_read_b64_tr_b16 for Vᵀ); tile j+2's global loads are issued right after the barrier that publishes tile j+1 and
// are written to LDS after tile j's compute: one barrier per tile. Tiles past a wave's causal range (or before its
// window) are skipped by that wave. Same softmax, dropout hash / keep words and outputs as the parity form.
template <int HD, bool DROP, bool IDX64, int NW, int NU>
__global__ __launch_bounds__(64 * NW, NW >= 8 || NU > 1 ? 1 : (DROP ? 2 : 3)) void attn_fwd_wide_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v, int64_t ld_in,
    int64_t tq, __bf16* __restrict__ o, int64_t ld_o, float* __restrict__ lse, const uint8_t* __restrict__ kmask,
    const uint8_t* __restrict__ qmask, int H, int Lq, int Lk, int window, float drop_p,
    const uint64_t* __restrict__ seed, uint32_t* __restrict__ keep, int nw, int order) {
  static_assert(HD == 32 || HD == 64 || HD == 128, "wide forward head dims");
  using Im = esgpt::attnb::Img<HD>;
  constexpr int T = 64 * NW, QW = 32 * NU, QB = QW * NW;
  constexpr int CH = HD / 8;                          // 16-B chunks per row
  constexpr int NLD = (ROWS * CH + T - 1) / T;        // chunks per thread and tensor for one tile
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  __shared__ __attribute__((aligned(16))) __bf16 sK[2][ROWS * HD];
  __shared__ __attribute__((aligned(16))) __bf16 sV[2][ROWS * HD];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int nqb = (Lq + QB - 1) / QB;
  int bh, qbi;
  if (order == 1) {
    int rank;
    esgpt::attnb::deal(blockIdx.x, gridDim.x, (int)(gridDim.x / nqb), rank, bh);
    qbi = nqb - 1 - rank;
  } else {
    const int lin = xcd_linear(blockIdx.x, gridDim.x);
    bh = lin / nqb;
    qbi = lin % nqb;
  }
  const int b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  constexpr bool idx32 = !IDX64;
  const int off = Lk - Lq;
  const int qb = qbi * QB;
  const int qw = qb + QW * wave;                              // this wave's first query
  const bool wave_any = qw < Lq;
  const int qlo_w = qw + off;                                 // smallest query position of this wave
  const int qhi_w = min(qw + QW - 1, Lq - 1) + off;           // largest

  bf16x8 qf[NU][HD / 16];
  f32x16 oacc[NU][HD / 32];
  float m[NU], l[NU];  // running max (log2 domain) and normaliser per query slice
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int qi = qw + 32 * u + r;
    const __bf16* qrow = q + ((int64_t)b * tq + qi) * ld_in + hh * HD;
#pragma unroll
    for (int t = 0; t < HD / 16; ++t)
      qf[u][t] = qi < Lq ? *reinterpret_cast<const bf16x8*>(qrow + 16 * t + 8 * h) : zero8();
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt) oacc[u][dt] = zero16();
    m[u] = -INFINITY;
    l[u] = 0.f;
  }

  const int qhi = min(Lq, qb + QB) - 1;
  const int kmax = min(Lk - 1, qhi + off);
  const int kmin = window ? max(0, qb + off - window + 1) : 0;
  const __bf16* kbase = k + (int64_t)b * Lk * ld_in + hh * HD;
  const __bf16* vbase = v + (int64_t)b * Lk * ld_in + hh * HD;
  const uint8_t* kmb = kmask ? kmask + (int64_t)b * Lk : nullptr;

  bf16x8 rk[NLD], rv[NLD];
  const int rec = (kmax + 1) * (int)ld_in * 2;  // buffer range ends after row kmax: later rows read as zeros
  const __amdgpu_buffer_rsrc_t rsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(kbase), (short)0, rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsv = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(vbase), (short)0, rec, 0x00020000);
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + T * i, row = c / CH, c8 = c % CH;
      const int vo = (NLD * T == ROWS * CH || c < ROWS * CH) ? (kt + row) * (int)ld_in * 2 + c8 * 16 : rec;
      rk[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsk, vo, 0, 0));
      rv[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsv, vo, 0, 0));
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int c = tid + T * i, row = c / CH, c8 = c % CH;
      if (NLD * T == ROWS * CH || c < ROWS * CH) {
        const int e = Im::off(row, 8 * c8);
        *reinterpret_cast<bf16x8*>(&sK[buf][e]) = rk[i];
        *reinterpret_cast<bf16x8*>(&sV[buf][e]) = rv[i];
      }
    }
  };
  auto key_ok = [&](int kt) {
    const int key = kt + lane;
    return key <= kmax && (kmb == nullptr || kmb[key] != 0);
  };

  const int kt0 = (kmin / ROWS) * ROWS;
  load_tile(kt0);
  bool kok = key_ok(kt0), kok_n = false;
  store_tile(0);
  __syncthreads();
  if (kt0 + ROWS <= kmax) {
    load_tile(kt0 + ROWS);
    kok_n = key_ok(kt0 + ROWS);
  }
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  int buf = 0;
  for (int kt = kt0; kt <= kmax; kt += ROWS) {
    const uint64_t kbits = __ballot(kok);
    const bool act = wave_any && kbits != 0 && kt <= qhi_w && (window == 0 || qlo_w - (kt + ROWS - 1) < window);
    const __bf16* tK = sK[buf];
    const __bf16* tV = sV[buf];
    const bool full = kbits == ~0ull && kt + ROWS - 1 <= qlo_w && (window == 0 || qhi_w - kt < window);
    auto tile = [&](auto full_c) {  // one instance per FULL (see the parity form)
      constexpr bool FULL = decltype(full_c)::value;
      f32x16 s[NU][2];
#pragma unroll
      for (int u = 0; u < NU; ++u) s[u][0] = s[u][1] = zero16();
#pragma unroll
      for (int t = 0; t < HD / 16; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(tK + Im::off(32 * c + r, 16 * t + 8 * h));
#pragma unroll
          for (int u = 0; u < NU; ++u) s[u][c] = mfma(a, qf[u][t], s[u][c]);
        }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int qi = qw + 32 * u + r;
        const bool qin = qi < Lq;
        if (!FULL) {
          const bool qvalid = qin && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0);
          mask_tile(s[u], kbits, qvalid, qi + off - kt, window, h);
        }
        float mt = row_max32(s[u]);
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * kLog2e;
        const float mnew = fmaxf(m[u], mt);
        const float alpha = (mnew == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m[u] - mnew);
        const float msub = (mnew == -INFINITY) ? 0.f : mnew;
        float rsp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[u][c][i], kLog2e, -msub));
            rsp[i & 3] += p;
            s[u][c][i] = p;
          }
        float rs = (rsp[0] + rsp[1]) + (rsp[2] + rsp[3]);
        if (DROP) {
          uint32_t kw[2] = {0u, 0u};
          if constexpr (idx32) {
            const uint32_t rowbase = ((uint32_t)bh * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk;
            const bool aligned = (rowbase & 1) == 0;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int i = 0; i < 16; i += 2) {
                const uint32_t e = rowbase + (uint32_t)(kt + 32 * c + acc_row(i, h));
                float m0, m1;
                if (aligned) {
                  dropout_mult2_32(dr, e, m0, m1);
                } else {
                  m0 = dropout_mult_32(dr, e);
                  m1 = dropout_mult_32(dr, e + 1);
                }
                s[u][c][i] *= m0;
                s[u][c][i + 1] *= m1;
                kw[c] |= (m0 != 0.f ? 1u : 0u) << acc_row(i, h);
                kw[c] |= (m1 != 0.f ? 1u : 0u) << acc_row(i + 1, h);
              }
          } else {
            const uint64_t rowbase = ((uint64_t)bh * (uint64_t)Lq + (uint64_t)qi) * (uint64_t)Lk;
            const bool aligned = (rowbase & 1) == 0;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int i = 0; i < 16; i += 2) {
                const uint64_t e = rowbase + (uint64_t)(kt + 32 * c + acc_row(i, h));
                float m0, m1;
                if (aligned) {
                  dropout_mult2(dr, e, m0, m1);
                } else {
                  m0 = dropout_mult(dr, e);
                  m1 = dropout_mult(dr, e + 1);
                }
                s[u][c][i] *= m0;
                s[u][c][i + 1] *= m1;
                kw[c] |= (m0 != 0.f ? 1u : 0u) << acc_row(i, h);
                kw[c] |= (m1 != 0.f ? 1u : 0u) << acc_row(i + 1, h);
              }
          }
          if (keep != nullptr) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const uint32_t w = kw[c] | (uint32_t)__shfl_xor((int)kw[c], 32, 64);
              const int wi = (kt >> 5) + c;
              if (h == 0 && qin && wi < nw) keep[((int64_t)bh * Lq + qi) * nw + wi] = w;
            }
          }
        }
        rs += __shfl_xor(rs, 32, 64);
        l[u] = l[u] * alpha + rs;
        m[u] = mnew;
        if (__ballot(alpha != 1.f))
#pragma unroll
          for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) oacc[u][dt][i] *= alpha;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          bf16x8 pf[NU];
#pragma unroll
          for (int u = 0; u < NU; ++u) pf[u] = acc_frag(s[u][c], ss);
          const int row0 = 32 * c + 16 * ss + 4 * (g >> 1) + q4;
#pragma unroll
          for (int dt = 0; dt < HD / 32; ++dt) {
            const int col = 32 * dt + 16 * (g & 1) + 4 * p4;
            const bf16x4 lo = tr_read(tV + Im::off(row0, col)), hi = tr_read(tV + Im::off(row0 + 8, col));
            bf16x8 vf;
            vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
            vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
#pragma unroll
            for (int u = 0; u < NU; ++u) oacc[u][dt] = mfma(vf, pf[u], oacc[u][dt]);
          }
        }
    };
    if (act) {
      if (full) tile(std::true_type{});
      else tile(std::false_type{});
    }
    if (kt + ROWS <= kmax) store_tile(buf ^ 1);  // tile kt + 64 (its buffer was last read before the previous barrier)
    __syncthreads();
    kok = kok_n;
    if (kt + 2 * ROWS <= kmax) {
      load_tile(kt + 2 * ROWS);
      kok_n = key_ok(kt + 2 * ROWS);
    }
    buf ^= 1;
  }

  int tid2;  // an opaque copy of the thread id (see the parity form's epilogue)
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid2) : "v"(tid));
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int qi_e = qb + QW * (tid2 >> 6) + 32 * u + (tid2 & 31);
    const bool qin_e = qi_e < Lq;
    const bool qvalid_e = qin_e && (qmask == nullptr || qmask[(int64_t)b * Lq + qi_e] != 0);
    const bool ok = qvalid_e && l[u] > 0.f;
    const float inv = ok ? 1.f / l[u] : 0.f;
    if (qin_e) {
      __bf16* orow = o + ((int64_t)b * Lq + qi_e) * ld_o + hh * HD;
#pragma unroll
      for (int dt = 0; dt < HD / 32; ++dt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[u][dt][i] *= inv;
        store_col32<32>(orow + 32 * dt, oacc[u][dt], (tid2 >> 5) & 1);
      }
      if ((tid2 & 32) == 0) lse[(int64_t)bh * Lq + qi_e] = ok ? m[u] * kLn2 + logf(l[u]) : 0.f;
    }
  }
}

}  // namespace

bool esgpt_attn_mfma_supported(int64_t hd, int64_t Lq, int64_t Lk, int64_t tq, int64_t ld_in, int64_t ld_o) {
  if (!(hd == 16 || hd == 32 || hd == 64 || hd == 128)) return false;
  if (Lk < 16 || Lq > (1 << 30)) return false;  // short dependency-graph sequences use the generic kernel
  // the forward's buffer loads address a batch element's K / V rows with 32-bit byte offsets
  return (ld_in % 8 == 0) && (ld_o % 8 == 0) && (tq >= Lq) && Lk * ld_in < (int64_t(1) << 30);
}

// Workgroup order (ESGPT_ATTN_ORDER tuning hook, read once; see attn_fwd_mfma_kernel)
static int attn_order() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_ATTN_ORDER");
    v = e ? atoi(e) : 1;  // measured (tools/attn_order_ab.sh, profiles/r05_attn_order_ab.log): order 1 wins everywhere
  }
  return v;
}

// Waves per workgroup of the wide forward (0: the parity form). Rule (tools/attn_wide_time.sh,
// profiles/r06_attn_wide_ab.log): hd 64 with Lq >= kWideMinLq and at least kWideMinBlocks 128-query blocks (four
// per CU) take 4 waves (C3: 52.4 -> 49.4 us, B=4 L=4096 H=8: 142 -> 114 us); fewer blocks keep the parity form (C5,
// 1024 blocks of 64 queries: 45.4 vs 49.9 us; C2: 10.9 vs 15.5 us). ESGPT_ATTN_FWD_NW (tools builds) forces 0 / 4 / 8.
constexpr int64_t kWideMinLq = 512, kWideMinBlocks = 1024;
// Query slices per wave of the 4-wave wide forward (ESGPT_ATTN_FWD_NU tools hook: 1 or 2; 2 halves the LDS reads
// per MFMA but needs ~350-440 registers, one wave per SIMD: L=4096 144 -> 257 us, C3 63 -> 93 us same box,
// profiles/r06_attn_nu_ab.log — tools build only).
static int fwd_wide_nu() {
  static int v = -1;
  if (v < 0) {
    const char* e = tuning_env("ESGPT_ATTN_FWD_NU");
    v = (e && atoi(e) == 2) ? 2 : 1;
  }
  return v;
}

static int fwd_wide_nw(int64_t B, int64_t H, int64_t Lq, int64_t hd) {
  static int forced = -2;
  if (forced == -2) {
    const char* e = tuning_env("ESGPT_ATTN_FWD_NW");
    forced = e ? atoi(e) : -1;
    if (forced != -1 && forced != 0 && forced != 4 && forced != 8) forced = -1;
  }
  if (hd != 64) return 0;  // hd 128: the wide form's registers spill (the parity form stays)
  if (forced >= 0) return forced;
  return Lq >= kWideMinLq && cdiv(Lq, 128) * B * H >= kWideMinBlocks ? 4 : 0;
}

template <int HD, int NW, int NU>
static void launch_wide(int64_t B, int64_t H, hipStream_t st, const void* q, const void* k, const void* v,
                        int64_t ld_in, int64_t tq, void* o, int64_t ld_o, float* lse, const uint8_t* kmask,
                        const uint8_t* qmask, int64_t Lq, int64_t Lk, int64_t window, float drop_p,
                        const uint64_t* seed, uint32_t* keep) {
  const int nw = (int)cdiv(Lk, 32);
  const dim3 grid((unsigned)(cdiv(Lq, 32 * NU * NW) * B * H));
  const bool idx64 = (uint64_t)(B * H) * (uint64_t)Lq * (uint64_t)Lk > 0xffffffffull;
#define ESGPT_WIDE(DROP, I64)                                                                                        \
  attn_fwd_wide_kernel<HD, DROP, I64, NW, NU><<<grid, dim3(64 * NW), 0, st>>>(                                             \
      (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, ld_in, tq, (__bf16*)o, ld_o, lse, kmask, qmask, (int)H,  \
      (int)Lq, (int)Lk, (int)window, drop_p, seed, DROP ? keep : nullptr, nw, attn_order())
  if (drop_p > 0.f && idx64) ESGPT_WIDE(true, true);
  else if (drop_p > 0.f) ESGPT_WIDE(true, false);
  else ESGPT_WIDE(false, false);
#undef ESGPT_WIDE
}

template <int HD>
static void launch_fwd(dim3 grid, hipStream_t st, const void* q, const void* k, const void* v, int64_t ld_in,
                       int64_t tq, void* o, int64_t ld_o, float* lse, const uint8_t* kmask, const uint8_t* qmask,
                       int64_t H, int64_t Lq, int64_t Lk, int64_t window, float drop_p, const uint64_t* seed,
                       uint32_t* keep) {
  const int nw = (int)cdiv(Lk, 32);
  // B·H·Lq·Lk element counters: 32-bit hash path when they all fit (B·H = grid / query blocks)
  const bool idx64 = (uint64_t)(grid.x / cdiv(Lq, ROWS)) * (uint64_t)Lq * (uint64_t)Lk > 0xffffffffull;
  if (drop_p > 0.f && idx64)
    attn_fwd_mfma_kernel<HD, true, true><<<grid, dim3(THREADS), 0, st>>>((const __bf16*)q, (const __bf16*)k,
                                                                          (const __bf16*)v, ld_in, tq, (__bf16*)o, ld_o,
                                                                          lse, kmask, qmask, (int)H, (int)Lq, (int)Lk,
                                                                          (int)window, drop_p, seed, keep, nw,
                                                                          attn_order());
  else if (drop_p > 0.f)
    attn_fwd_mfma_kernel<HD, true><<<grid, dim3(THREADS), 0, st>>>((const __bf16*)q, (const __bf16*)k,
                                                                    (const __bf16*)v, ld_in, tq, (__bf16*)o, ld_o,
                                                                    lse, kmask, qmask, (int)H, (int)Lq, (int)Lk,
                                                                    (int)window, drop_p, seed, keep, nw,
                                                                    attn_order());
  else
  attn_fwd_mfma_kernel<HD, false><<<grid, dim3(THREADS), 0, st>>>((const __bf16*)q, (const __bf16*)k, (const __bf16*)v,
                                                           ld_in, tq, (__bf16*)o, ld_o, lse, kmask, qmask, (int)H,
                                                           (int)Lq, (int)Lk, (int)window, drop_p, seed, nullptr, nw,
                                                           attn_order());
}

int esgpt_attn_fwd_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                        float* lse, const uint8_t* kmask, const uint8_t* qmask, int64_t B, int64_t H, int64_t Lq,
                        int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed, uint32_t* keep,
                        hipStream_t st) {
  dim3 grid((unsigned)(cdiv(Lq, ROWS) * B * H));  // 1-D: XCD-aware (query block, batch-head) order in the kernel
  const int nwv = fwd_wide_nw(B, H, Lq, hd), nu = nwv ? fwd_wide_nu() : 1;
  if (nwv == 8)
    launch_wide<64, 8, 1>(B, H, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, Lq, Lk, window, drop_p, seed, keep);
#ifdef ESGPT_TUNING_HOOKS
  else if (nwv == 4 && nu == 2)  // measured slower everywhere (one wave per SIMD at ~350-440 registers)
    launch_wide<64, 4, 2>(B, H, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, Lq, Lk, window, drop_p, seed, keep);
#endif
  else if (nwv == 4)
    launch_wide<64, 4, 1>(B, H, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, Lq, Lk, window, drop_p, seed, keep);
  else if (hd == 16)
    launch_fwd<16>(grid, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, H, Lq, Lk, window, drop_p, seed, keep);
  else if (hd == 32)
    launch_fwd<32>(grid, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, H, Lq, Lk, window, drop_p, seed, keep);
  else if (hd == 64)
    launch_fwd<64>(grid, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, H, Lq, Lk, window, drop_p, seed, keep);
  else
    launch_fwd<128>(grid, st, q, k, v, ld_in, tq, o, ld_o, lse, kmask, qmask, H, Lq, Lk, window, drop_p, seed, keep);
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}
