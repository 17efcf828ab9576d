// K5 at the reference's precision: the fused classifier-head linear + cross-entropy of ce.hip on
// SPLIT-bf16 operands, for the fp32 training mode (north_star: forward/loss within 1e-4 of fp32).
//
// Replaces trainer.py:131-154 (logits = h·Wᵀ + b over all n items ‖ the pad column,
// F.cross_entropy(ignore_index = n), forward and backward) like ce.hip, but every fp32 operand x is
// carried as two bf16 values
//     x = hi + lo + ε,   hi = RNE_bf16(x),  lo = RNE_bf16(x − hi),   |ε| ≤ 2^-17·|x|
// and every product as three bf16 MFMAs accumulated in fp32:
//     a·b ≈ a_hi·b_hi + a_lo·b_hi + a_hi·b_lo          (dropped: a_lo·b_lo, ≤ 2^-16·|ab|)
// so each term of a dot product is exact to ≈3·2^-17 relative — the per-term error of an fp32 MFMA
// chain is 2^-24, the CPU reference's accumulation-order noise at K = 256 is of order 1e-6 — at 3/16 of
// the cost of the fp32-input MFMA (v_mfma_f32_32x32x2_f32 runs at 1/16 of the bf16 rate; gfx950 has no
// xf32).  Logits are never materialised over all rows; with LGS the forward stores the valid rows' logits for
// ce3_dwl_kernel (the stored-logits dW sweep, below).
//
// Operands live as [rows][2·D] bf16 images "hi ‖ lo" (c2dsr_f32_split_bf16).  One kernel template, two
// roles (the ce.hip fwd_u / dw pair with the tile height halved so the stationary hi AND lo fragments
// fit next to the accumulators):
//   MODE 0 (forward + U): stationary = H rows (lane ↔ row r), swept = W rows (the columns c of S):
//     Sᵀ = W·Hᵀ, v = S·log2e + b2_c, lazy running max m, p = 2^(v − m), z += p, Uᵀ += Wᵀ·Pᵀ
//     → part_m [split][M], part_s [split][M], Up [split][M][D]   (combined by ce_rows / dh_from_u)
//   MODE 1 (dW): stationary = W rows (lane ↔ column c), swept = H rows r:
//     S = H·W_cᵀ, E = 2^(S·log2e + cr_r + b2_c) (cr = log2 rw − lse2), db += E, dWᵀ += Hᵀ·E
//     → dbp [split][n], dWp [split][n][D]
// v_mfma_f32_16x16x32_bf16 throughout: on this chip the 16x16x32 shape holds a ≈14 % higher clock under
// full matrix load than 32x32x16 at equal cycles per flop (tools/peak/mfma_peak.hip: 2147 vs 1887 TFLOP/s
// sustained; measured here 2.2 vs 1.84 GHz inside this kernel).  Per wave: 32 stationary rows as two
// 16-row blocks sb (lane ↔ row 16sb + l%16), their hi / lo k-slices (128 registers) pinned to AGPRs as
// MFMA B operands; per 32-row swept tile: 96 MFMAs for S, 96 for the second product, whose accumulator
// (Uᵀ / dWᵀ, 128 registers) is also AGPR-resident.  The swept image (32 rows × 2D bf16 = 32 KiB at
// D = 256) streams through four LDS buffers by saddr LDS-DMA (tile t+3 issued during the second product
// of tile t), read row-wise (ds_read_b128) for S and transposed (ds_read_b64_tr_b16) for the second
// product, whose B operand is S's accumulator itself (P split into hi/lo in registers).  The epilogue
// of S(t) runs in the MFMA shadow of S(t+1).
#include "img.h"

#include <utility>

// tuning knobs (tools/ce3_micro.py; the defaults are the shipped configuration)
#ifndef CE3_DS
#define CE3_DS 2
#endif
#ifndef CE3_DT
#define CE3_DT 2
#endif
#ifndef CE3B_DS  // the plain-bf16 instantiation (one MFMA per fragment: the reads run further ahead)
#define CE3B_DS 2
#endif
#ifndef CE3B_DT
#define CE3B_DT 2
#endif
#ifndef CE3B_ILV
#define CE3B_ILV 1
#endif
#ifndef CE3_NW  // waves per workgroup (4: one per SIMD; 8: two per SIMD, one stationary block each)
#define CE3_NW 4
#endif
#ifndef CE3B_NW
#define CE3B_NW 4
#endif
#ifndef CE3_PRIO
#define CE3_PRIO 0
#endif
#ifndef CE3_DQ
#define CE3_DQ 2
#endif
#ifndef CE3B_DQ
#define CE3B_DQ 4
#endif
// the plain-bf16 instantiation's geometry: stationary 16-row blocks per wave and swept rows per LDS tile.  Measured in
// round 6 (tools/ce3b_micro.py + CE3_STAMP, MB head b): 3 blocks × 32-row tiles — each LDS fragment read feeding 3
// MFMAs instead of 2; the 3-block accumulators (192 AGPRs) and stationary fragments (96 VGPRs) fit one wave's 512
// registers, 4 blocks would not (256 AGPRs of accumulators alone) — ran 5–35 % SLOWER than 2 × 64 (fwd_u 1282 vs
// 1213 µs, dw 1317 vs 979 µs at one row split): per tile and wave the second product took 31 cycles per MFMA
// (1500 / 48) against 29 (1869 / 64), the S phase 26 against 23.6, and the per-tile fixed cost (rescale, DMA wait,
// barrier, loop top) 583 cycles now paid per 32 rows.  The default stays 2 × 64.
#ifndef CE3B_SBW
#define CE3B_SBW 2
#endif
#ifndef CE3_LGW0  // diagnostic: the forward's logits stores drained at the DMA wait (vmcnt(0))
#define CE3_LGW0 0
#endif
#ifndef CE3_LGE  // the forward's logits stores in the S phase's epilogue steps (else at the end of the second product)
#define CE3_LGE 1
#endif
#ifndef CE3B_T3
#define CE3B_T3 64
#endif

namespace {

using namespace c2img;

#ifdef CE3_STAMP  // diagnostic build only: per-phase cycle sums of the tile loop (tools/ce3_micro.py prints them)
__device__ unsigned long long ce3_stamp_acc[8];
#define STAMP(i)                                                   \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const unsigned now_ = (unsigned)__builtin_amdgcn_s_memtime();  \
    st_acc[i] += now_ - st_prev;                                   \
    st_prev = now_;                                                \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

constexpr int T3 = 32;  // swept rows per LDS tile

// the two half-waves hold the two halves of a row's columns: combine them with one v_permlane32_swap (no LDS
// round trip): swap(x, x) returns (lower half broadcast, upper half broadcast)
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------------------------------------------------------- fragment layout
// Swept tiles of 32 rows as two 16-row blocks cb.  Sᵀ block
// (cb, sb): lane holds swept rows 16cb + 4g + i (g = lane/16, i < 4) of stationary row 16sb + l%16, so a
// lane's 8 values of one sb ARE the B operand of the second product with the reduction index permuted
// k = 8g + j ↔ swept row (j < 4 ? 4g + j : 16 + 4g + j − 4); the A operand (Xwᵀ, rows = columns e of
// the image) is read transposed in the same order: two ds_read_b64_tr_b16, rows 4g.. and 16 + 4g...
// Image swizzle: img.h swz16.
__device__ __forceinline__ float quad_max(float x) {  // over lanes l, l^16, l^32, l^48
  x = half_max(x);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float quad_sum(float x) {
  x = half_sum(x);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// global accesses by hand (saddr form: a wave-uniform base in SGPRs, a 32-bit per-lane offset, an immediate): the
// logits store of the forward and the logits loads of ce3_dwl_kernel, which run among the tile's LDS-DMA pieces — the
// compiler's wait-count pass does not see those (asm), so a compiler-visible load would get a wait that also drains
// the younger DMA pieces; the loads are waited for by hand (dma_wait_keep) and their registers re-defined there
// (CE3_LGNT bit 0: the stores non-temporal, bit 1: the loads — streamed once, kept out of the L2 the operand tiles
// are shared through)
#ifndef CE3_LGNT
#define CE3_LGNT 1
#endif
// stored-logits layout: 16 × 16 blocks of 1 KiB; GRP column blocks grouped — block (c16, h16) at
// ((c16 / GRP)·HB + h16)·GRP + c16 % GRP (GRP = 1: column-block-major; 8: a row block's 8 column blocks side by side,
// so a forward tile's 8 row blocks × 2 column blocks fall in one 64 KiB run)
#ifndef CE3_LGG  // measured: GRP = 8 writes at the same rate as 1 (forward 3,117 µs both, MB head b; dW within 1 %)
#define CE3_LGG 1
#endif
constexpr int LGG = CE3_LGG;
__device__ __forceinline__ long lg_blk(int c16, int h16, int hb) {
  return ((long)(c16 / LGG) * hb + h16) * LGG + c16 % LGG;
}
template <int IMM>
__device__ __forceinline__ void gst1(const void* sbase, unsigned voff, float v) {
  if constexpr (CE3_LGNT & 1)
    asm volatile("global_store_dword %0, %1, %2 offset:%3 nt" ::"v"(voff), "v"(v), "s"(sbase), "n"(IMM));
  else
    asm volatile("global_store_dword %0, %1, %2 offset:%3" ::"v"(voff), "v"(v), "s"(sbase), "n"(IMM));
}
#ifndef CE3_LGNOST  // diagnostic: the forward's logits transposed but not stored
#define CE3_LGNOST 0
#endif
template <int IMM>
__device__ __forceinline__ void gst4(const void* sbase, unsigned voff, const f32x4& v) {
  if constexpr (CE3_LGNOST)
    asm volatile("" ::"v"(voff), "v"(v), "s"(sbase));
  else if constexpr (CE3_LGNT & 1)
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 nt" ::"v"(voff), "v"(v), "s"(sbase), "n"(IMM));
  else
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3" ::"v"(voff), "v"(v), "s"(sbase), "n"(IMM));
}
// 4 × 4 transpose across the lanes of a quad (lane & 3) and a lane's 4 values: out[j] of lane b = in[b] of lane j
// (two rounds of 2 × 2 swaps, one DPP quad permutation each)
__device__ __forceinline__ f32x4 quad_transpose(const f32x4& x) {
  const int lane = (int)(threadIdx.x & 3);
  f32x4 y, z;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float t = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x[r ^ 1]), 0xB1, 0xF, 0xF, false));
    y[r] = ((r & 1) == (lane & 1)) ? x[r] : t;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float t = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y[r ^ 2]), 0x4E, 0xF, 0xF, false));
    z[r] = ((r & 2) == (lane & 2)) ? y[r] : t;
  }
  return z;
}
template <int IMM>
__device__ __forceinline__ void gld4(f32x4& v, const void* sbase, unsigned voff) {
  if constexpr (CE3_LGNT & 2)
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3 nt" : "=v"(v) : "v"(voff), "s"(sbase), "n"(IMM));
  else
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(v) : "v"(voff), "s"(sbase), "n"(IMM));
}

#ifndef CE3_BI  // compiler-visible MFMAs in both roles (CE3_BI0: MODE 0 only, CE3_BI1: MODE 1 only)
#define CE3_BI 0
#endif
#ifndef CE3_BI0
#define CE3_BI0 CE3_BI
#endif
#ifndef CE3_BI1
#define CE3_BI1 CE3_BI
#endif
#ifndef CE3_BIS0  // the S phase only (MODE 0 / MODE 1), and the second-product phase only
#define CE3_BIS0 0
#endif
#ifndef CE3_BIS1
#define CE3_BIS1 0
#endif
#ifndef CE3_BIU0  // default: the second product on builtin MFMAs (fwd_u 2676 → 2590 µs, dw −1 % at MB head-b shapes)
#define CE3_BIU0 1
#endif
#ifndef CE3_BIU1
#define CE3_BIU1 1
#endif
#ifndef CE3_VN
#define CE3_VN 5
#endif
#ifndef CE3_P1  // the second product with the probabilities as one bf16 term (2 MFMAs instead of 3; measured option)
#define CE3_P1 0
#endif
// Two forms of one split product step, acc (+)= a_hi·b_hi + a_lo·b_hi + a_hi·b_lo, chosen per kernel role:
//  * asm: ONE asm statement for the three MFMAs on one accumulator (separate statements get an s_nop between
//    dependent MFMAs from the hazard pass).  S product: the stationary b_hi / b_lo pinned to AGPRs (128 registers
//    that would otherwise be re-staged into VGPRs every tile), acc in VGPRs (read by the VALU only after s_nop
//    padding).  Second product: the long-lived accumulator pinned to AGPRs (the compiler otherwise stages it
//    through VGPRs around the rescale branch); VALU readers of acc run after mfma_drain().
//  * builtin (BI): compiler-visible MFMAs (exact hazard padding), so the scheduler places the step's LDS reads and
//    VALU work between dependent MFMAs (sched_group_barrier pattern in the tile loop, step_pattern).
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0)
template <bool BI>
__device__ __forceinline__ void split3_s0(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                          const bf16x8& bl) {
  if constexpr (BI) {
    acc = MF(ah, bh, (f32x4{0.f, 0.f, 0.f, 0.f}));
    acc = MF(al, bh, acc);
    acc = MF(ah, bl, acc);
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, 0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
        : "=&v"(acc)
        : "v"(ah), "v"(al), "a"(bh), "a"(bl));
  }
}
template <bool BI>
__device__ __forceinline__ void split3_s(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bl) {
  if constexpr (BI) {
    acc = MF(ah, bh, acc);
    acc = MF(al, bh, acc);
    acc = MF(ah, bl, acc);
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
        : "+v"(acc)
        : "v"(ah), "v"(al), "a"(bh), "a"(bl));
  }
}
// second product: acc += a_hi·b_hi + a_hi·b_lo + a_lo·b_hi
template <bool BI>
__device__ __forceinline__ void split3_u(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bl) {
  if constexpr (BI) {
    acc = MF(ah, bh, acc);
    acc = MF(ah, bl, acc);
    acc = MF(al, bh, acc);
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0"
        : "+a"(acc)
        : "v"(ah), "v"(al), "v"(bh), "v"(bl));
  }
}
// second product with the B operand (the probabilities) as ONE bf16 term (CE3_P1, measured option, not the default):
// acc += a_hi·b + a_lo·b
template <bool BI>
__device__ __forceinline__ void split2_u(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& b) {
  if constexpr (BI) {
    acc = MF(ah, b, acc);
    acc = MF(al, b, acc);
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0"
        : "+a"(acc)
        : "v"(ah), "v"(al), "v"(b));
  }
}
#undef MF

// plain-bf16 products (the bf16 training mode): one MFMA, accumulator in AGPRs; the stationary operand in AGPRs
// (BA) or, when the accumulators leave no room there (3 stationary blocks), in VGPRs
template <bool BA = true>
__device__ __forceinline__ void mf1_s0(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (BA)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
template <bool BA = true>
__device__ __forceinline__ void mf1_s(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (BA)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mf1_u(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// scheduling hint for one tile-loop step of the builtin form: per MFMA, one LDS read and up to VN VALU instructions
template <int NMF, int VN, bool BI>
__device__ __forceinline__ void step_pattern() {
  if constexpr (BI) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      ((__builtin_amdgcn_sched_group_barrier(0x008, 1, 0), __builtin_amdgcn_sched_group_barrier(0x100, 1, 0),
        __builtin_amdgcn_sched_group_barrier(0x002, VN, 0), (void)I),
       ...);
    }(std::make_integer_sequence<int, NMF>{});
  }
}

// swept rows per LDS tile: 32 for split images (2D columns: 32 KiB at D = 256), CE3B_T3 for plain bf16 (D columns)
template <bool SPLIT>
constexpr int tile_rows() { return SPLIT ? 32 : CE3B_T3; }
// 16-row stationary blocks per wave, and stationary rows per workgroup (the row block of the launch grid)
template <bool SPLIT, int NW>
constexpr int stat_blocks() { return SPLIT || NW != 4 ? 8 / NW : CE3B_SBW; }
template <bool SPLIT, int NW>
constexpr int row_block() { return 16 * NW * stat_blocks<SPLIT, NW>(); }
constexpr int ROW_BLOCK_MAX = 16 * 4 * (CE3B_SBW > 2 ? CE3B_SBW : 2);

// NW: waves per workgroup — 4 (one per SIMD, two 16-row stationary blocks each) or 8 (two per SIMD, one block each:
// half the registers, so one wave's LDS waits, epilogue VALU and barrier run under its partner's MFMAs).  The
// workgroup covers the same 128 stationary rows either way and every accumulation order is the same.
// LGS (MODE 0, split images): also store every tile's logits v = S·log2e + b2 into lg (ce3_dwl_kernel's layout, below)
template <int D, int MODE, bool SPLIT, int NW = 4, bool LGS = false>
__global__ __launch_bounds__(64 * NW, 1) void ce3_kernel(const bf16* __restrict__ Xs, const bf16* __restrict__ Xw,
                                                      const float* __restrict__ svec, const float* __restrict__ wvec,
                                                      int n_s, int n_w, int per_split, float* __restrict__ part_m,
                                                      float* __restrict__ part_s, float* __restrict__ outp,
                                                      int accum, int sk_nwg, float* __restrict__ slot_w,
                                                      float* __restrict__ slot_b, float* __restrict__ lg, int lg_hb) {
  constexpr int T3 = tile_rows<SPLIT>();
  constexpr int CB = T3 / 16;                      // 16-row swept blocks per tile
  constexpr int UK = T3 / 32;                      // 32-row k-steps of the second product per e-block
  constexpr int KS = D / 32;                       // k-steps of the S product
  constexpr int NSS = KS * CB;                     // S-phase steps: (ks, cb)
  constexpr int NE = D / 16;                       // 16-column e-blocks of the second product
  constexpr int NUS = NE * UK;                     // second-product steps: (u, e-block)
  constexpr int D2 = SPLIT ? 2 * D : D;            // image columns (hi ‖ lo, or bf16)
  constexpr int IMG = T3 * D2 * 2;                 // bytes per image
  constexpr int HT = T3 * 256;                     // bytes per 128-column half-tile
  constexpr int SBW = stat_blocks<SPLIT, NW>();     // 16-row stationary blocks per wave
  constexpr int RB = row_block<SPLIT, NW>();       // stationary rows per workgroup
  constexpr bool BA = SPLIT || SBW <= 2;           // stationary fragments in AGPRs (else VGPRs: the accumulators fill them)
  constexpr int NDMA = (T3 / 4) * (D2 / 128) / NW;  // LDS-DMA wave-instructions per wave per tile
  constexpr int NB = 4;
  constexpr int DS = SPLIT ? CE3_DS : CE3B_DS, DT = SPLIT ? CE3_DT : CE3B_DT;
  constexpr int NEL = 4 * SBW * CB;                // S values per lane per tile (SBW stationary blocks × CB)
  constexpr float TAU = 8.f;
  static_assert((NW == 4 || NW == 8) && NDMA * NW == (T3 / 4) * (D2 / 128) && NEL % 8 == 0 && DS <= NUS &&
                    DT <= NSS, "tile / wave split");
  // one LDS-DMA wave-instruction of tile t+3 every DQ second-product steps, from the first (DQ = 1: the whole
  // tile at the start of the phase, the longest time to land before the barrier that publishes it)
  constexpr int DQ = SPLIT ? CE3_DQ : CE3B_DQ;
  // builtin MFMA form per role and phase (S: the first product, U: the second); ILV (asm form): the step's VALU work
  // between its stationary blocks' products — the builtin form is scheduled by step_pattern instead
  constexpr bool BIS = SPLIT && (MODE == 0 ? CE3_BI0 || CE3_BIS0 : CE3_BI1 || CE3_BIS1);
  constexpr bool BIU = SPLIT && (MODE == 0 ? CE3_BI0 || CE3_BIU0 : CE3_BI1 || CE3_BIU1);
  constexpr bool ILVS = SPLIT ? !BIS : CE3B_ILV, ILVU = SPLIT ? !BIU : CE3B_ILV;
  static_assert(DQ >= 1 && DQ * NDMA <= NUS, "DMA spacing");
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float wv[NB][NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, g = lane >> 4;
  // XCD-aware work map: block b runs on XCD b % 8; the (split, row block) pairs, split-major, are dealt to the XCDs in
  // contiguous ranges, so each split's swept slice streams through the L2 of one or two XCDs instead of all eight
  const int nrb = (n_s + RB - 1) / RB, nb = (int)gridDim.x;
  // stream-K (MODE 1, sk_nwg workgroups, one per CU): the (row block, swept tile) units in row-block-major order are
  // dealt to the workgroups in equal contiguous ranges, one launch round with no partial last round; a workgroup walks
  // its range as segments (≤ one per row block it touches).  A row block swept whole by one workgroup is added onto the
  // gradient directly; a split one leaves a partial in its workgroup's slot 0 (its first segment) or 1 (its last),
  // summed in workgroup order by ce3_sk_combine_kernel.
  const long skT = (n_w + T3 - 1) / T3, skU = (long)nrb * skT;
  long sk_u = sk_nwg ? (long)blockIdx.x * skU / sk_nwg : 0;
  const long sk_u1 = sk_nwg ? ((long)blockIdx.x + 1) * skU / sk_nwg : 0;
  for (int seg = 0;; ++seg) {
  int split, rblk, w_beg, w_end, slot = -1;
  if (sk_nwg) {
    if (sk_u >= sk_u1) break;  // uniform over the workgroup
    rblk = (int)(sk_u / skT);
    const long t0 = sk_u % skT, t1 = min(skT, t0 + (sk_u1 - sk_u));
    split = 0;
    w_beg = (int)(t0 * T3);
    w_end = min(n_w, (int)(t1 * T3));
    if (t0 != 0 || t1 != skT) slot = seg == 0 ? 0 : 1;
    sk_u += t1 - t0;
  } else {
    if (seg) break;
    const int pidx = nb % 8 == 0 ? (int)(blockIdx.x & 7) * (nb >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    split = pidx / nrb;
    rblk = pidx % nrb;
    w_beg = split * per_split;
    w_end = min(n_w, w_beg + per_split);
  }
  const int s0 = rblk * RB + w * 16 * SBW + l16;  // stationary rows s0 + 16·sb, sb < SBW
  const int ntiles = w_end > w_beg ? (w_end - w_beg + T3 - 1) / T3 : 0;
  f32x4 dacc[NE][SBW];
  float mrow[SBW], zrow[SBW];
#pragma unroll
  for (int sb = 0; sb < SBW; ++sb) {
#pragma unroll
    for (int e = 0; e < NE; ++e) dacc[e][sb] = f32x4{0.f, 0.f, 0.f, 0.f};
    mrow[sb] = -INFINITY;
    zrow[sb] = 0.f;
  }
  if (ntiles > 0) {
    const int w_last = w_beg + (ntiles - 1) * T3;
    const int ib = (int)lds_addr(img[0]);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + NW * i;
      constexpr int GROUPS = T3 / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz16(row);
      dvoff[i] = (unsigned)((row * D2 + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * HT + rg * 1024));
    }
    auto dma = [&](int tt) {
      const int r0 = min(w_beg + tt * T3, w_last);
      const int buf = tt % NB;
      const bf16* base = Xw + (long)r0 * D2;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma4(wvec + r0 + lane, wv[buf][w]);
    };
    // per-lane image offsets: row fragments (row l16 of block cb, k-chunk 4c + g) and transposed
    // fragments (rows 4g + (l16>>2) and +16, columns 16v + 4(lane&3)..)
    int roff0[4], toff0[8];
    {
      const int fr = swz16(l16);
#pragma unroll
      for (int c = 0; c < 4; ++c) roff0[c] = l16 * 256 + 16 * ((4 * c + g) ^ fr);
      const int trow = 4 * g + (l16 >> 2), p = lane & 3, ft = swz16(trow);
#pragma unroll
      for (int v = 0; v < 8; ++v) toff0[v] = trow * 256 + 16 * ((2 * v + (p >> 1)) ^ ft) + 8 * (p & 1);
    }
    bf16x8 fh[SBW][KS], fl[SBW][KS];
#pragma unroll
    for (int sb = 0; sb < SBW; ++sb) {
      const long sr = min(s0 + 16 * sb, n_s - 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fh[sb][ks] = *(const bf16x8*)(Xs + sr * D2 + ks * 32 + 8 * g);
        if constexpr (SPLIT) fl[sb][ks] = *(const bf16x8*)(Xs + sr * D2 + D + ks * 32 + 8 * g);
      }
    }
    float b2s[SBW];
#pragma unroll
    for (int sb = 0; sb < SBW; ++sb) b2s[sb] = MODE == 1 ? svec[min(s0 + 16 * sb, n_s - 1)] : 0.f;
    // LGS: tile tt's logits (the epilogue's v, before the running max is subtracted) into the 16 × 16 blocks
    // [column block][row block] of lg: element (row 16sb + l16, column 16cb + 4g + r) of this wave's 32 rows.  Tile
    // t+1's are stored at the end of the second product of tile t: at the DMA wait of the next S phase they are the
    // youngest vector-memory operations but the loop top's row-constant DMA, and stay in flight
    const int lg_h0 = __builtin_amdgcn_readfirstlane((rblk * RB + w * 16 * SBW) >> 4);
    const unsigned lg_lo = (unsigned)((((l16 >> 2) * 16 + 4 * g) * 4 + (l16 & 3)) * 4);
    constexpr bool LGW = LGS && MODE == 0 && SPLIT;
    constexpr int NST = LGW ? NEL : 0;  // stores per tile
    auto lg_store = [&](int tt, const f32x4(&v)[SBW * CB]) {
      if constexpr (LGW && !CE3_LGE) {
        const int cw = (w_beg + tt * T3) >> 4;
        [&]<int... C>(std::integer_sequence<int, C...>) {
          (
              [&] {
                constexpr int cb = C / (4 * SBW), sb = (C / 4) % SBW, r = C % 4;
                const float* base = lg + lg_blk(cw + cb, lg_h0, lg_hb) * 256;
                gst1<sb * 1024 * LGG + r * 16>(base, lg_lo, v[cb * SBW + sb][r]);
              }(),
              ...);
        }(std::make_integer_sequence<int, NST>{});
      }
    };
    // CE3_LGE: tile t's logits stored in the epilogue steps of iteration t instead, each 16 × 16 block (elements
    // 4j .. 4j+3 of the lane, j = sb·CB + cb) in the step that exponentiates its first element: the quad's 4 × 4
    // transpose gives each lane the block's 16-byte chunk 16·(l16/4) + 4g + l16%4 (rows 4·(l16/4) .., column 4g +
    // l16%4), one dwordx4 store per block and wave
    const unsigned lg_lo4 = (unsigned)((16 * (l16 >> 2) + 4 * g + (l16 & 3)) * 16);
    unsigned lg_lo4s[SBW];  // + the stationary block's row-block offset (past the immediate's range when LGG > 1)
#pragma unroll
    for (int sb = 0; sb < SBW; ++sb) lg_lo4s[sb] = lg_lo4 + (unsigned)(sb * LGG * 1024);
    auto lg_put = [&]<int IB, int IE>(const float* const(&lgp)[CB], const f32x4(&v)[SBW * CB]) {
      if constexpr (LGW && CE3_LGE) {
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (
              [&] {
                constexpr int i = IB + I, sb = i / (4 * CB), cb = (i >> 2) % CB;
                if constexpr (i % 4 == 0) gst4<0>(lgp[cb], lg_lo4s[sb], quad_transpose(v[cb * SBW + sb]));
              }(),
              ...);
        }(std::make_integer_sequence<int, IE - IB>{});
      }
    };
    dma(0);
    dma(1);
    dma(2);
    vm_drain();
    dma_wait();
    __syncthreads();
    struct Offs {
      int r[4];
      int t[8];
    };
    auto offs_rows = [&](int b, Offs& o) {
#pragma unroll
      for (int c = 0; c < 4; ++c) o.r[c] = roff0[c] + ib + b * IMG;
    };
    auto offs_tr = [&](int b, Offs& o) {
#pragma unroll
      for (int v = 0; v < 8; ++v) o.t[v] = toff0[v] + ib + b * IMG;
    };
    // row fragment of image column block kx (32 columns; hi: ks, lo: KS + ks) and swept-row block C
    auto rfrag = [&]<int KX, int C>(const Offs& o) {
      return lds_ld128<(KX >> 2) * HT + C * 16 * 256>(o.r[KX & 3]);
    };
    // transposed fragment of image columns 16·EX .. +15 (hi: EX, lo: D/16 + EX), swept rows 32U ..
    auto tfrag = [&]<int EX, int U>(const Offs& o) {
      constexpr int IMM = (EX >> 3) * HT + U * 32 * 256;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (lds_bf16x4*)(size_t)(lds_base(o.t[EX & 7]) + IMM));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (lds_bf16x4*)(size_t)(lds_base(o.t[EX & 7]) + IMM + 16 * 256));
      bf16x8 v;
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
      return v;
    };
    // S-phase step k ↔ (ks = k / CB, cb = k % CB); second-product step k ↔ (u = k / NE, e-block k % NE)
    auto s_frags = [&]<int K>(const Offs& o, bf16x8(&f)[2]) {
      f[0] = rfrag.template operator()<K / CB, K % CB>(o);
      if constexpr (SPLIT) f[1] = rfrag.template operator()<KS + K / CB, K % CB>(o);
    };
    auto u_frags = [&]<int K>(const Offs& o, bf16x8(&f)[2]) {
      f[0] = tfrag.template operator()<K % NE, K / NE>(o);
      if constexpr (SPLIT) f[1] = tfrag.template operator()<NE + K % NE, K / NE>(o);
    };
    auto s_prod = [&]<int KSI>(f32x4& acc, const bf16x8(&a)[2], int sb) {
      if constexpr (SPLIT) {
        if constexpr (KSI == 0)
          split3_s0<BIS>(acc, a[0], a[1], fh[sb][KSI], fl[sb][KSI]);
        else
          split3_s<BIS>(acc, a[0], a[1], fh[sb][KSI], fl[sb][KSI]);
      } else {
        if constexpr (KSI == 0)
          mf1_s0<BA>(acc, a[0], fh[sb][KSI]);
        else
          mf1_s<BA>(acc, a[0], fh[sb][KSI]);
      }
    };
    // the per-swept-row constants of this lane's rows 16cb + 4g + i
    auto wconst = [&](int b, f32x4(&c4)[CB]) {
      const int bo = (int)lds_addr(wv[b][w]) + 16 * g;
      [&]<int... C>(std::integer_sequence<int, C...>) {
        ((c4[C] = lds_ld<f32x4, 64 * C>(bo)), ...);
      }(std::make_integer_sequence<int, CB>{});
    };
    // epilogue element i (0 .. NEL-1) ↔ (sb = i / 4CB, cb = (i / 4) % CB, r = i % 4) = accumulator (cb·SBW + sb)[r];
    // the second product's B fragment (u, sb) packs elements of cb = 2u, 2u + 1 (8-element chunk sb·UK + u).
    // Step k of a phase with NST steps handles elements [⌈k·NEL/NST⌉, ⌈(k+1)·NEL/NST⌉)
    f32x4 sc[SBW * CB];
    {
      Offs oS;
      offs_rows(0, oS);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int cb = K % CB;
              bf16x8 a[2];
              s_frags.template operator()<K>(oS, a);
#pragma unroll
              for (int sb = 0; sb < SBW; ++sb) s_prod.template operator()<K / CB>(sc[cb * SBW + sb], a, sb);
            }(),
            ...);
      }(std::make_integer_sequence<int, NSS>{});
    }
    mfma_drain();
    float mnext[SBW];
    {
      f32x4 c4[CB];
      wconst(0, c4);
      float tm[SBW];
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb) tm[sb] = mnext[sb] = -INFINITY;
#pragma unroll
      for (int i = 0; i < NEL; ++i) {
        const int sb = i / (4 * CB), cb = (i >> 2) % CB, r = i & 3;
        float v = fmaf(sc[cb * SBW + sb][r], LOG2E, c4[cb][r]);
        if constexpr (MODE == 1) v += b2s[sb];
        sc[cb * SBW + sb][r] = v;
        tm[sb] = fmaxf(tm[sb], v);
      }
      if constexpr (MODE == 0) {
#pragma unroll
        for (int sb = 0; sb < SBW; ++sb) mnext[sb] = quad_max(tm[sb]);
      }
    }
    if constexpr (!CE3_LGE) lg_store(0, sc);
    bf16x8 fa[DS + 2][2];
    bf16x8 tf[DT + 2][2];
    {
      Offs oS;
      offs_rows(1 % NB, oS);
      [&]<int... P>(std::integer_sequence<int, P...>) {
        (s_frags.template operator()<P>(oS, fa[P]), ...);
      }(std::make_integer_sequence<int, DS>{});
    }
#ifdef CE3_STAMP
    unsigned st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = (unsigned)__builtin_amdgcn_s_memtime();
#endif
    // CE3_PRIO (8 waves): static priority for the second-dispatched half, the arbitration loser of each SIMD pair
    if constexpr (NW == 8 && CE3_PRIO) {
      if (w >= 4) __builtin_amdgcn_s_setprio(1);
    }
    for (int t = 0; t < ntiles; ++t) {
      STAMP(5);
      const int bh = t % NB, bs = (t + 1) % NB;
      const int rn = min(w_beg + (t + 3) * T3, w_last);
      const bf16* nsrc = Xw + (long)rn * D2;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      dma4(wvec + rn + lane, wv[(t + 3) % NB][w]);
      float msub[SBW];
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb) msub[sb] = 0.f;
      if constexpr (MODE == 0) {
#pragma unroll
        for (int sb = 0; sb < SBW; ++sb) {
          const bool need = mnext[sb] > mrow[sb] + TAU;
          if (__builtin_amdgcn_ballot_w64(need)) [[unlikely]] {
            const float f = need ? ex2(mrow[sb] - mnext[sb]) : 1.f;
            mfma_drain();
#pragma unroll
            for (int e = 0; e < NE; ++e) {
              // (re)defined here, so the copies to VGPRs for the multiply cannot be hoisted above the branch
              asm volatile("" : "+a"(dacc[e][sb]) : "v"(f));
              dacc[e][sb] *= f;
              asm volatile("" : "+a"(dacc[e][sb]));  // back to AGPRs inside the branch
            }
            zrow[sb] *= f;
            mrow[sb] = need ? mnext[sb] : mrow[sb];
          }
          // keep the accumulators in AGPRs across the branch (else they are staged through VGPRs every tile)
#pragma unroll
          for (int e = 0; e < NE; ++e) asm volatile("" : "+a"(dacc[e][sb]));
          msub[sb] = mrow[sb] == -INFINITY ? 0.f : mrow[sb];
        }
      }
      STAMP(0);
      const float* lgp[CB];
      if constexpr (LGW && CE3_LGE) {
        const int cw = (w_beg + t * T3) >> 4;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) lgp[cb] = lg + lg_blk(cw + cb, lg_h0, lg_hb) * 256;
      }
      Offs oS, oH;
      offs_rows(bs, oS);
      offs_tr(bh, oH);
      // ---- S(t+1) ∥ epilogue(t)
      f32x4 sn[SBW * CB];
      bf16x8 xh[UK][SBW], xl[UK][SBW];
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int k = K, cb = k % CB;
              // the two rings run DS / DT steps ahead, each across the phase boundary
              if constexpr (k + DS < NSS) s_frags.template operator()<k + DS>(oS, fa[(k + DS) % (DS + 2)]);
              if constexpr (k + DT >= NSS) u_frags.template operator()<k + DT - NSS>(oH, tf[k + DT - NSS]);
              // ILV: the step's VALU work between its two stationary blocks' products (each MFMA's shadow
              // covers half of it; in-order issue otherwise stalls it behind the second MFMA)
              s_prod.template operator()<k / CB>(sn[cb * SBW], fa[k % (DS + 2)], 0);
              if constexpr (ILVS || SBW == 1) {
                __builtin_amdgcn_sched_barrier(0);
              } else {
#pragma unroll
                for (int sb = 1; sb < SBW; ++sb) s_prod.template operator()<k / CB>(sn[cb * SBW + sb], fa[k % (DS + 2)], sb);
              }
              constexpr int ib = (k * NEL + NSS - 1) / NSS, ie = ((k + 1) * NEL + NSS - 1) / NSS;
              lg_put.template operator()<ib, ie>(lgp, sc);
#pragma unroll
              for (int i = ib; i < ie; ++i) {
                const int sb = i / (4 * CB), cb2 = (i >> 2) % CB, r = i & 3;
                const float pv = ex2(sc[cb2 * SBW + sb][r] - msub[sb]);
                sc[cb2 * SBW + sb][r] = pv;
                zrow[sb] += pv;
              }
              // the 8-element chunks this step completes (ib < 8(c+1) <= ie: with NEL / NSS not an integer — 3
              // stationary blocks — a step's range can straddle a chunk end)
              [&]<int... C>(std::integer_sequence<int, C...>) {
                (
                    [&] {
                      constexpr int c = C, sb = c / UK, u = c % UK;
                      if constexpr (ib < 8 * (c + 1) && 8 * (c + 1) <= ie) {
                        bf16x8 h, l;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                          const float x = sc[(2 * u + (j >> 2)) * SBW + sb][j & 3];
                          h[j] = (bf16)x;
                          if constexpr (SPLIT && !CE3_P1) l[j] = (bf16)(x - (float)h[j]);
                        }
                        xh[u][sb] = h;
                        if constexpr (SPLIT && !CE3_P1) xl[u][sb] = l;
                      }
                    }(),
                    ...);
              }(std::make_integer_sequence<int, NEL / 8>{});
              if constexpr (ILVS && SBW >= 2) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int sb = 1; sb < SBW; ++sb) s_prod.template operator()<k / CB>(sn[cb * SBW + sb], fa[k % (DS + 2)], sb);
              }
              step_pattern<SPLIT ? 3 * SBW : SBW, CE3_VN, BIS>();
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NSS>{});
      STAMP(1);
      // the second product's B fragments are redefined here: their VALU conversions cannot sink past this point
      // to just before an asm MFMA that reads them (no hazard padding is inserted for asm operands)
#pragma unroll
      for (int u = 0; u < UK; ++u) {
#pragma unroll
        for (int sb = 0; sb < SBW; ++sb) {
          asm volatile("" : "+v"(xh[u][sb]));
          if constexpr (SPLIT && !CE3_P1) asm volatile("" : "+v"(xl[u][sb]));
        }
      }
      asm volatile("s_nop 7" ::: "memory");  // S(t+1)'s last results before the prep's VALU reads
      // tile t+2's image (DMA'd during the previous second product); LGS: the logits stores that followed it and the
      // row-constant DMA of the loop top, younger, stay in flight
      if constexpr (LGW && !CE3_LGW0)
        dma_wait_keep<(CE3_LGE ? NST / 4 : NST) + 1>();
      else
        dma_wait();
      STAMP(2);
      __syncthreads();
      STAMP(3);
      // ---- second product (t) ∥ prep of S(t+1) ∥ DMA of tile t+3
      Offs oN;
      offs_rows((t + 2) % NB, oN);
      f32x4 c4n[CB];
      wconst(bs, c4n);
      float tm[SBW];
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb) tm[sb] = -INFINITY;
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        (
            [&] {
              constexpr int k = Q, q = k % NE, u = k / NE;
              if constexpr (k + DT < NUS) u_frags.template operator()<k + DT>(oH, tf[(k + DT) % (DT + 2)]);
              if constexpr (k + DS >= NUS) s_frags.template operator()<k + DS - NUS>(oN, fa[k + DS - NUS]);
              const bf16x8(&tq)[2] = tf[k % (DT + 2)];
              auto u_prod = [&](int sb) {
                if constexpr (SPLIT && CE3_P1)
                  split2_u<BIU>(dacc[q][sb], tq[0], tq[1], xh[u][sb]);
                else if constexpr (SPLIT)
                  split3_u<BIU>(dacc[q][sb], tq[0], tq[1], xh[u][sb], xl[u][sb]);
                else
                  mf1_u(dacc[q][sb], tq[0], xh[u][sb]);
              };
              u_prod(0);
              if constexpr (ILVU || SBW == 1) {
                __builtin_amdgcn_sched_barrier(0);
              } else {
#pragma unroll
                for (int sb = 1; sb < SBW; ++sb) u_prod(sb);
              }
              if constexpr (k % DQ == DQ - 1 && k / DQ < NDMA)
                dma16_s<k == DQ - 1>(nsrc, dvoff[k / DQ], ddst[k / DQ] + nbuf);
              constexpr int ib = (k * NEL + NUS - 1) / NUS, ie = ((k + 1) * NEL + NUS - 1) / NUS;
#pragma unroll
              for (int i = ib; i < ie; ++i) {
                const int sb = i / (4 * CB), cb = (i >> 2) % CB, r = i & 3;
                float v = fmaf(sn[cb * SBW + sb][r], LOG2E, c4n[cb][r]);
                if constexpr (MODE == 1) v += b2s[sb];
                sn[cb * SBW + sb][r] = v;
                tm[sb] = fmaxf(tm[sb], v);
              }
              if constexpr (ILVU && SBW >= 2) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int sb = 1; sb < SBW; ++sb) u_prod(sb);
              }
              step_pattern<SPLIT ? (CE3_P1 ? 2 : 3) * SBW : SBW, CE3_VN, BIU>();
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NUS>{});
      if constexpr (MODE == 0) {
#pragma unroll
        for (int sb = 0; sb < SBW; ++sb) mnext[sb] = quad_max(tm[sb]);
      }
      if (LGW && !CE3_LGE && t + 1 < ntiles) lg_store(t + 1, sn);
#pragma unroll
      for (int i = 0; i < SBW * CB; ++i) sc[i] = sn[i];
      STAMP(4);
    }
#ifdef CE3_STAMP
    if (lane == 0) {
      for (int i = 0; i < 6; ++i) atomicAdd(&ce3_stamp_acc[i], (unsigned long long)st_acc[i]);
      atomicAdd(&ce3_stamp_acc[6], (unsigned long long)ntiles);
    }
#endif
  }
  mfma_drain();
#pragma unroll
  for (int sb = 0; sb < SBW; ++sb) {
    const float ztot = quad_sum(zrow[sb]);
    const int s = s0 + 16 * sb;
    if (s < n_s && slot >= 0) {  // stream-K partial of a split row block
      const long so = (long)(2 * blockIdx.x + slot) * RB + (s - rblk * RB);
      if (g == 0) slot_b[so] = ztot;
      float* out = slot_w + so * D + 4 * g;
#pragma unroll
      for (int e = 0; e < NE; ++e) *(f32x4*)(out + 16 * e) = dacc[e][sb];
    } else if (s < n_s) {
      const bool acc = accum || sk_nwg;
      if (g == 0) {
        if constexpr (MODE == 0) part_m[(long)split * n_s + s] = mrow[sb];
        // accum (MODE 1, one split or a whole stream-K row block: this workgroup owns its columns): add onto the
        // epoch-long gradient directly
        part_s[(long)split * n_s + s] = acc ? part_s[s] + ztot : ztot;
      }
      float* out = outp + ((long)split * n_s + s) * D + 4 * g;
      if (acc) {
#pragma unroll
        for (int e = 0; e < NE; ++e) *(f32x4*)(out + 16 * e) = *(const f32x4*)(out + 16 * e) + dacc[e][sb];
      } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) *(f32x4*)(out + 16 * e) = dacc[e][sb];
      }
    }
  }
  if (sk_nwg) {  // the next segment's prologue refills the LDS images: every wave past this one's reads and DMAs
    vm_drain();
    __syncthreads();
  }
  }  // segments
}

// ce3_dwl_kernel knobs measured at MB head b (tools/ce3_lg_micro.py, one box): fragment reads 2 / 3 / 4 steps ahead
// 1,837 / 1,842 / 1,862 µs, the compiler's own schedule instead of the step pattern 1,857 µs — all within 1 %
#ifndef CE3L_DT  // ce3_dwl_kernel: transposed fragment reads issued this many steps ahead
#define CE3L_DT 2
#endif
#ifndef CE3L_PAT  // ce3_dwl_kernel: the sched_group_barrier step pattern (0: the compiler's own schedule)
#define CE3L_PAT 1
#endif
#ifndef CE3L_PF  // ce3_dwl_kernel: tiles of logits loaded ahead (register sets; the tile loop is unrolled by it); 3
#define CE3L_PF 2  // measured within 1.5 % of 2 (MB head b 1,808 vs 1,835 µs, head a 1,013 vs 1,022)
#endif
#ifndef CE3L_NW  // ce3_dwl_kernel at d = 256: 4 waves (one per SIMD) or 8 (two per SIMD splitting the e-blocks; measured
#define CE3L_NW 4  // slower: MB head b 1,966 vs 1,798 µs, head a 1,108 vs 999 — the logits loads and E twice per SIMD)
#endif
#ifndef CE3L_X  // diagnostic builds of ce3_dwl_kernel (timing only): bit 0 no logits loads, bit 1 no per-tile H DMA
#define CE3L_X 0
#endif
// ---------------------------------------------------------------- dW from the forward's logits
// The forward (ce3_kernel MODE 0 with LGS) stores v = S·log2e + b2_c of every (row r < ⌈M/128⌉·128, column c <
// ⌈n/32⌉·32) — the logits in log2 units, fp32 — as 16 × 16 blocks, column-block-major: block (c/16, r/16) at
// lg + ((c/16)·HB + r/16)·256 (HB = ⌈M/128⌉·8 row blocks), element (r, c) of a block at ((r%16)/4·16 + c%16)·4 + r%4.
// In this kernel's accumulator layout (lane ↔ column c%16 and row group (r%16)/4) a lane's four rows r%4 of a block
// are one float4 at lane·16 bytes.  The dW sweep then needs no S product: per swept 32-row H tile
//     E = 2^(v + cr_r)  (cr = log2 rw − lse2, −inf past M),   db += E,   dWᵀ += Hᵀ·E
// — 96 MFMAs per tile instead of 192, the logits read once from HBM (M·n·4 bytes) instead of recomputed.  Same
// work map, outputs and stream-K slots as ce3_kernel MODE 1.  Per wave and tile, in issue order: the logits and row
// constants of tile t+2 (NL loads, two register sets alternating by tile parity: the loop is unrolled by two so no
// register of a load in flight is ever copied), then — spread over the second product of tile t — the LDS-DMA pieces
// of tile t+3's H image (NDMA).  The second product of tile t runs on the B operand built from tile t's logits during
// tile t−1 (E, z and the hi / lo split in the MFMA shadow); tile t+1's logits (loaded at the top of tile t−1) are
// waited for at the top of tile t with NDMA + NL younger operations left in flight, tile t+1's image at its end with
// 2·(NL + NDMA).
// NWD = 8 (D = 256): two waves per SIMD, the pair on one SIMD sharing its 32 columns and splitting the 16 e-blocks of
// the second product (each computes the tile's E itself), so one wave's waits and VALU run under the other's MFMAs
template <int D, int SBW, int NWD = 4>
__global__ __launch_bounds__(64 * NWD, 1) void ce3_dwl_kernel(const bf16* __restrict__ Xw, const float* __restrict__ lg,
                                                         int lg_hb, int lg_cw, const float* __restrict__ crow, int n_s,
                                                         int n_w, int per_split, float* __restrict__ part_s,
                                                         float* __restrict__ outp, int accum, int sk_nwg,
                                                         float* __restrict__ slot_w, float* __restrict__ slot_b) {
  constexpr int NW = NWD, T3 = 32, CB = 2, NE = D / 16, D2 = 2 * D, IMG = T3 * D2 * 2, HT = T3 * 256, NB = 4;
  constexpr int EH = NW / 4, NES = NE / EH;          // e-block halves (waves per SIMD), e-blocks per wave = steps
  constexpr int RB = 16 * 4 * SBW;
  constexpr int NDMA = (T3 / 4) * (D2 / 128) / NW;  // LDS-DMA wave-instructions per wave per tile
  constexpr int NL = SBW * CB + CB;                  // logits blocks + row-constant float4s per wave per tile
  constexpr int DT = CE3L_DT, DQ = NES / NDMA;
  constexpr int NEL = 4 * SBW * CB;                  // E values per lane per tile
  static_assert((NW == 4 || (NW == 8 && NES == 8)) && DQ >= 1 && DQ * NDMA == NES && NEL % 8 == 0 &&
                    2 * (NL + NDMA) < 64, "tile / wave split");
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, g = lane >> 4;
  const int cw = w & 3, eh = w >> 2;  // column group, e-block half
  const int nrb = (n_s + RB - 1) / RB, nb = (int)gridDim.x;
  const long skT = (n_w + T3 - 1) / T3, skU = (long)nrb * skT;
  long sk_u = sk_nwg ? (long)blockIdx.x * skU / sk_nwg : 0;
  const long sk_u1 = sk_nwg ? ((long)blockIdx.x + 1) * skU / sk_nwg : 0;
  for (int seg = 0;; ++seg) {
  int split, rblk, w_beg, w_end, slot = -1;
  if (sk_nwg) {
    if (sk_u >= sk_u1) break;  // uniform over the workgroup
    rblk = (int)(sk_u / skT);
    const long t0 = sk_u % skT, t1 = min(skT, t0 + (sk_u1 - sk_u));
    split = 0;
    w_beg = (int)(t0 * T3);
    w_end = min(n_w, (int)(t1 * T3));
    if (t0 != 0 || t1 != skT) slot = seg == 0 ? 0 : 1;
    sk_u += t1 - t0;
  } else {
    if (seg) break;
    const int pidx = nb % 8 == 0 ? (int)(blockIdx.x & 7) * (nb >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    split = pidx / nrb;
    rblk = pidx % nrb;
    w_beg = split * per_split;
    w_end = min(n_w, w_beg + per_split);
  }
  const int s0 = rblk * RB + cw * 16 * SBW + l16;  // stationary columns s0 + 16·sb
  const int ntiles = w_end > w_beg ? (w_end - w_beg + T3 - 1) / T3 : 0;
  f32x4 dacc[NES][SBW];
  float zrow[SBW];
#pragma unroll
  for (int sb = 0; sb < SBW; ++sb) {
#pragma unroll
    for (int e = 0; e < NES; ++e) dacc[e][sb] = f32x4{0.f, 0.f, 0.f, 0.f};
    zrow[sb] = 0.f;
  }
  if (ntiles > 0) {
    const int w_last = w_beg + (ntiles - 1) * T3;
    const int ib = (int)lds_addr(img[0]);
    const int ebo = eh * HT;  // this wave's e-blocks: image columns 128·eh .. (hi) and D + 128·eh .. (lo)
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + NW * i;
      constexpr int GROUPS = T3 / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz16(row);
      dvoff[i] = (unsigned)((row * D2 + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * HT + rg * 1024));
    }
    int toff0[8];
    {
      const int trow = 4 * g + (l16 >> 2), p = lane & 3, ft = swz16(trow);
#pragma unroll
      for (int v = 0; v < 8; ++v) toff0[v] = trow * 256 + 16 * ((2 * v + (p >> 1)) ^ ft) + 8 * (p & 1);
    }
    // this wave's logits column blocks (clamped to the written ones: columns past ⌈n/32⌉·32 only feed discarded
    // outputs), one wave-uniform base each
    const float* lgb[SBW];
#pragma unroll
    for (int sb = 0; sb < SBW; ++sb) {
      const int c16 = __builtin_amdgcn_readfirstlane(min(((rblk * RB + cw * 16 * SBW) >> 4) + sb, lg_cw - 1));
      lgb[sb] = lg + lg_blk(c16, 0, lg_hb) * 256;
    }
    struct LSet {
      f32x4 v[SBW][CB];  // logits: block (sb, cb), rows 16cb + 4g + i of column s0 + 16sb
      f32x4 c[CB];       // row constants cr of rows 16cb + 4g + i
    };
    auto ld_logits = [&](int tt, LSet& x) {
      if constexpr (CE3L_X & 1) {  // diagnostic: no logits traffic
#pragma unroll
        for (int sb = 0; sb < SBW; ++sb) x.v[sb][0] = x.v[sb][1] = f32x4{-1.f, -1.f, -1.f, -1.f};
        x.c[0] = x.c[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        return;
      }
      const int r0 = min(w_beg + tt * T3, w_last);
      const unsigned vo = (unsigned)(lane * 16 + r0 * 64 * LGG), vc = (unsigned)((r0 + 4 * g) * 4);
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb) {
        gld4<0>(x.v[sb][0], lgb[sb], vo);
        if constexpr (LGG * 1024 < 4096)
          gld4<LGG * 1024>(x.v[sb][1], lgb[sb], vo);
        else
          gld4<0>(x.v[sb][1], lgb[sb], vo + LGG * 1024);
      }
      gld4<0>(x.c[0], crow, vc);
      gld4<64>(x.c[1], crow, vc);
    };
    auto landed = [&](LSet& x) {  // after the wait: the set's registers are (re)defined here
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) asm volatile("" : "+v"(x.v[sb][cb]));
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) asm volatile("" : "+v"(x.c[cb]));
    };
    auto dma = [&](int tt) {
      const int r0 = min(w_beg + tt * T3, w_last);
      const bf16* base = Xw + (long)r0 * D2;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + (tt % NB) * IMG);
    };
    struct XSet {
      bf16x8 h[SBW], l[SBW];  // the second product's B operand (hi / lo) per stationary block
    };
    // E element i (0 .. NEL-1) ↔ (sb = i / 4CB, cb = (i / 4) % CB, r = i % 4); B fragment sb packs cb = 0, 1
    auto e_elems = [&]<int IB, int IE>(const LSet& x, float(&ev)[NEL], float zm) {
#pragma unroll
      for (int i = IB; i < IE; ++i) {
        const int sb = i / (4 * CB), cb = (i >> 2) % CB, r = i & 3;
        const float e = ex2(x.v[sb][cb][r] + x.c[cb][r]);
        ev[i] = e;
        zrow[sb] = fmaf(e, zm, zrow[sb]);
      }
    };
    auto pack = [&]<int SB>(const float(&ev)[NEL], XSet& xs) {
      bf16x8 h, l;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = ev[SB * 4 * CB + j];
        h[j] = (bf16)x;
        l[j] = (bf16)(x - (float)h[j]);
      }
      xs.h[SB] = h;
      xs.l[SB] = l;
    };
    auto tfrag = [&]<int EX>(int bbase) {
      constexpr int IMM = (EX >> 3) * HT;
      const int o = toff0[EX & 7] + bbase;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(size_t)(lds_base(o) + IMM));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(size_t)(lds_base(o) + IMM + 16 * 256));
      bf16x8 v;
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
      return v;
    };
    constexpr int U = CE3L_PF;  // logits register sets = tiles loaded ahead (the loop is unrolled by U)
    static_assert(U == 2 || U == 3, "logits prefetch depth");
    LSet L[U];
    XSet X[U];
    ld_logits(0, L[0]);
    dma(0);
    ld_logits(1, L[1]);
    dma(1);
    if constexpr (U == 3) ld_logits(2, L[2]);
    dma(2);
    vm_drain();
    dma_wait();
#pragma unroll
    for (int u = 0; u < U; ++u) landed(L[u]);
    __syncthreads();
    {
      float ev[NEL];
      e_elems.template operator()<0, NEL>(L[0], ev, 1.f);
      [&]<int... S>(std::integer_sequence<int, S...>) {
        (pack.template operator()<S>(ev, X[0]), ...);
      }(std::make_integer_sequence<int, SBW>{});
    }
    // tile t (P = t mod U): loads of tile t+U into L[P]; the second product on X[P] ∥ tile t+1's E into X[P+1] from
    // L[P+1] (mod U) ∥ the DMA of tile t+3.  Step k: e-block eh·NES + k (image columns of the hi half at offset ebo, the lo
    // half NE e-blocks further)
    bf16x8 tf[DT + 2][2];
    auto tile = [&]<int P>(int t) {
      constexpr int PN = (P + 1) % U;
      ld_logits(t + U, L[P]);
      dma_wait_keep<(U - 1) * (NDMA + NL)>();
      landed(L[PN]);
      const int bh = ib + (t % NB) * IMG + ebo;
      const int rn = min(w_beg + (t + 3) * T3, w_last);
      const bf16* nsrc = Xw + (long)rn * D2;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      const float zm = t + 1 < ntiles ? 1.f : 0.f;  // the E of a tile past the end (clamped loads) counts nowhere
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        ((tf[Q][0] = tfrag.template operator()<Q>(bh), tf[Q][1] = tfrag.template operator()<NE + Q>(bh)), ...);
      }(std::make_integer_sequence<int, DT>{});
      float ev[NEL];
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int k = K;
              if constexpr (k + DT < NES) {
                tf[(k + DT) % (DT + 2)][0] = tfrag.template operator()<k + DT>(bh);
                tf[(k + DT) % (DT + 2)][1] = tfrag.template operator()<NE + k + DT>(bh);
              }
              const bf16x8(&tq)[2] = tf[k % (DT + 2)];
#pragma unroll
              for (int sb = 0; sb < SBW; ++sb) split3_u<true>(dacc[k][sb], tq[0], tq[1], X[P].h[sb], X[P].l[sb]);
              if constexpr (k % DQ == DQ - 1 && !(CE3L_X & 2))
                dma16_s<k == DQ - 1>(nsrc, dvoff[k / DQ], ddst[k / DQ] + nbuf);
              constexpr int i0 = (k * NEL + NES - 1) / NES, i1 = ((k + 1) * NEL + NES - 1) / NES;
              e_elems.template operator()<i0, i1>(L[PN], ev, zm);
              [&]<int... S>(std::integer_sequence<int, S...>) {
                (
                    [&] {
                      if constexpr (i0 < 8 * (S + 1) && 8 * (S + 1) <= i1) pack.template operator()<S>(ev, X[PN]);
                    }(),
                    ...);
              }(std::make_integer_sequence<int, SBW>{});
              step_pattern<3 * SBW, CE3_VN, (bool)CE3L_PAT>();
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NES>{});
#pragma unroll
      for (int sb = 0; sb < SBW; ++sb) {
        asm volatile("" : "+v"(X[PN].h[sb]));
        asm volatile("" : "+v"(X[PN].l[sb]));
      }
      dma_wait_keep<2 * (NDMA + NL)>();
      __syncthreads();
    };
    for (int t = 0; t < ntiles; t += U) {
      tile.template operator()<0>(t);
      if (t + 1 < ntiles) tile.template operator()<1>(t + 1);
      if constexpr (U == 3)
        if (t + 2 < ntiles) tile.template operator()<2 % U>(t + 2);
    }
    // the loads past the end (clamped) land before their registers — live until here — or the LDS are reused
    vm_drain();
#pragma unroll
    for (int u = 0; u < U; ++u) landed(L[u]);
  }
  mfma_drain();
#pragma unroll
  for (int sb = 0; sb < SBW; ++sb) {
    const float ztot = quad_sum(zrow[sb]);
    const int s = s0 + 16 * sb;
    const int eo = 16 * NES * eh;  // this wave's columns of dW
    if (s < n_s && slot >= 0) {  // stream-K partial of a split row block
      const long so = (long)(2 * blockIdx.x + slot) * RB + (s - rblk * RB);
      if (g == 0 && eh == 0) slot_b[so] = ztot;
      float* out = slot_w + so * D + eo + 4 * g;
#pragma unroll
      for (int e = 0; e < NES; ++e) *(f32x4*)(out + 16 * e) = dacc[e][sb];
    } else if (s < n_s) {
      const bool acc = accum || sk_nwg;
      if (g == 0 && eh == 0) part_s[(long)split * n_s + s] = acc ? part_s[s] + ztot : ztot;
      float* out = outp + ((long)split * n_s + s) * D + eo + 4 * g;
      if (acc) {
#pragma unroll
        for (int e = 0; e < NES; ++e) *(f32x4*)(out + 16 * e) = *(const f32x4*)(out + 16 * e) + dacc[e][sb];
      } else {
#pragma unroll
        for (int e = 0; e < NES; ++e) *(f32x4*)(out + 16 * e) = dacc[e][sb];
      }
    }
  }
  if (sk_nwg) {  // the next segment's prologue refills the LDS images: every wave past this one's reads and DMAs
    vm_drain();
    __syncthreads();
  }
  }  // segments
}

// stream-K partials of the split row blocks (ce3_kernel MODE 1): gW[rb] += Σ_w slot(w, rb), w ascending over the
// workgroups whose unit ranges overlap row block rb (a block swept whole by one workgroup was written directly).
// Blocks (row block, 16-row group): thread → (row, float4 column) — 16 rows per block, not the whole row block: the
// per-element loop over the contributing workgroups is a chain of dependent adds, and one block per row block
// (66 / 90 blocks at the Entertainment-Education heads) left the combine latency-bound at 118 µs.
__device__ __forceinline__ int sk_wg_of(long u, long U, int nwg) {
  int w = (int)((u * nwg) / U);
  while (w + 1 < nwg && ((long)(w + 1) * U) / nwg <= u) ++w;
  while (w > 0 && ((long)w * U) / nwg > u) --w;
  return w;
}
__global__ __launch_bounds__(256) void ce3_sk_combine_kernel(const float* __restrict__ slot_w,
                                                             const float* __restrict__ slot_b, int n, int D, long T,
                                                             int nwg, int RB, float* __restrict__ gW,
                                                             float* __restrict__ gb) {
  const int rb = blockIdx.x, r0 = blockIdx.y * 16;
  const long U = (long)((n + RB - 1) / RB) * T;
  const long ub = (long)rb * T, ue = ub + T - 1;
  const int wa = sk_wg_of(ub, U, nwg), wz = sk_wg_of(ue, U, nwg);
  if (wa == wz) return;  // uniform
  const int C4 = D / 4;
  for (int i = threadIdx.x; i < 16 * (C4 + 1); i += 256) {
    const int r = r0 + i / (C4 + 1), c = i % (C4 + 1);  // c == C4: the bias column
    const long row = (long)rb * RB + r;
    if (row >= n) continue;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    float b = 0.f;
    for (int w = wa; w <= wz; ++w) {
      const long wu0 = ((long)w * U) / nwg;
      if (wu0 == ((long)(w + 1) * U) / nwg) continue;  // an empty range (fewer units than workgroups)
      const int sl = wu0 >= ub ? 0 : 1;
      const long so = (long)(2 * w + sl) * RB + r;
      if (c < C4) a = a + *(const float4*)(slot_w + so * D + 4 * c);
      else b += slot_b[so];
    }
    if (c < C4) {
      float4* o = (float4*)(gW + row * D + 4 * c);
      *o = *o + a;
    } else {
      gb[row] += b;
    }
  }
}

// out[r] = [RNE(x[r]) ‖ RNE(x[r] − RNE(x[r]))] for r < rows; zero rows up to rows_out.  4 values per thread.
__global__ void split_bf16_kernel(const float* __restrict__ x, long rows, int D, long rows_out,
                                  bf16* __restrict__ out) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= rows_out * D) return;
  const long r = i / D;
  const int k = (int)(i % D);
  const float4 v = r < rows ? *(const float4*)(x + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  bf16x4 h, l;
  h[0] = (bf16)v.x;
  h[1] = (bf16)v.y;
  h[2] = (bf16)v.z;
  h[3] = (bf16)v.w;
  l[0] = (bf16)(v.x - (float)h[0]);
  l[1] = (bf16)(v.y - (float)h[1]);
  l[2] = (bf16)(v.z - (float)h[2]);
  l[3] = (bf16)(v.w - (float)h[3]);
  *(bf16x4*)(out + r * 2 * D + k) = h;
  *(bf16x4*)(out + r * 2 * D + D + k) = l;
}

int per_split3(int total, int nsplit, int t3) {
  const int tiles = c2::ceil_div(total, t3);
  return c2::ceil_div(tiles, nsplit) * t3;
}

int g_ncu3 = 0;
int num_cus3() {
  if (!g_ncu3) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    g_ncu3 = v > 0 ? v : 256;
  }
  return g_ncu3;
}

// stream-K slots: two [RB][D] fp32 partials (+ two [RB] bias partials) per workgroup, RB up to ROW_BLOCK_MAX (one
// workspace size serves both instantiations)
size_t sk_slot_floats(int nwg, int D) { return (size_t)2 * nwg * ROW_BLOCK_MAX * D; }
size_t sk_ws_bytes(int nwg, int D) { return (sk_slot_floats(nwg, D) + (size_t)2 * nwg * ROW_BLOCK_MAX) * 4; }

// the logits layout of ce3_dwl_kernel: 16-row blocks per 16-column block (the forward's row blocks, whole), and
// 16-column blocks written (whole 32-column tiles)
inline int lg_row_blocks(int M) { return c2::ceil_div(M, 128) * 8; }
inline int lg_col_blocks(int n) { return c2::ceil_div(c2::ceil_div(n, 32) * 2, LGG) * LGG; }

template <int MODE, bool SPLIT>
int launch3(const void* Xs, const void* Xw, const float* svec, const float* wvec, int n_s, int n_w, int D, int nsplit,
            float* pm, float* ps, float* out, hipStream_t st, int sk_nwg = 0, float* slot_w = nullptr,
            float* slot_b = nullptr, float* lg = nullptr) {
  // MODE 1 with nsplit == 0: one split, accumulated straight onto out / ps (the gradient buffers); sk_nwg > 0:
  // stream-K over sk_nwg workgroups (MODE 1; whole row blocks accumulated, partials into the slots)
  const int accum = MODE == 1 && nsplit == 0;
  if (accum) nsplit = 1;
  if (nsplit < 1 || (sk_nwg && (MODE != 1 || !slot_w || !slot_b))) return (int)hipErrorInvalidValue;
  const int per = per_split3(n_w, nsplit, tile_rows<SPLIT>());
  // (row block, split) pairs: ce3_kernel's XCD-aware map; stream-K: one workgroup per CU
  constexpr int NW = SPLIT ? CE3_NW : CE3B_NW;
  constexpr int RB = row_block<SPLIT, NW>();
  const dim3 grid(sk_nwg ? sk_nwg : c2::ceil_div(n_s, RB) * nsplit);
  const int hb = lg_row_blocks(n_s);
  if (lg && !(MODE == 0 && SPLIT && NW == 4)) return (int)hipErrorInvalidValue;
  if (D == 128 && lg)
    ce3_kernel<128, MODE, SPLIT, NW, true><<<grid, 64 * NW, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s,
                                                                      n_w, per, pm, ps, out, accum, sk_nwg, slot_w,
                                                                      slot_b, lg, hb);
  else if (D == 256 && lg)
    ce3_kernel<256, MODE, SPLIT, NW, true><<<grid, 64 * NW, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s,
                                                                      n_w, per, pm, ps, out, accum, sk_nwg, slot_w,
                                                                      slot_b, lg, hb);
  else if (D == 128)
    ce3_kernel<128, MODE, SPLIT, NW><<<grid, 64 * NW, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s, n_w,
                                                                per, pm, ps, out, accum, sk_nwg, slot_w, slot_b,
                                                                nullptr, 0);
  else if (D == 256)
    ce3_kernel<256, MODE, SPLIT, NW><<<grid, 64 * NW, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s, n_w,
                                                                per, pm, ps, out, accum, sk_nwg, slot_w, slot_b,
                                                                nullptr, 0);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  if (sk_nwg) {
    const long T = (n_w + tile_rows<SPLIT>() - 1) / tile_rows<SPLIT>();
    ce3_sk_combine_kernel<<<dim3(c2::ceil_div(n_s, RB), RB / 16), 256, 0, st>>>(slot_w, slot_b, n_s, D, T, sk_nwg, RB,
                                                                                out, ps);
    C2_CHECK_LAUNCH();
  }
  return 0;
}

// the dW sweep from stored logits (ce3_dwl_kernel): n_s = n stationary W columns, n_w = M swept H rows; nsplit as
// launch3 (0: one split added onto out / ps), sk_nwg > 0: stream-K with its combine
#ifndef CE3L_SBW  // stationary 16-column blocks per wave of the dW-from-logits sweep
#define CE3L_SBW 2
#endif
constexpr int DWL_SBW = CE3L_SBW;
int launch_dwl(const void* Hx, const float* lg, int lg_hb, int lg_cw, const float* crow, int n, int M, int D,
               int nsplit, float* ps, float* out, hipStream_t st, int sk_nwg = 0, float* slot_w = nullptr,
               float* slot_b = nullptr) {
  const int accum = nsplit == 0;
  if (accum) nsplit = 1;
  if (nsplit < 1 || !lg || lg_cw < 1 || lg_hb < c2::ceil_div(M, 16) || (sk_nwg && (!slot_w || !slot_b)))
    return (int)hipErrorInvalidValue;
  constexpr int RB = 64 * DWL_SBW;
  const int per = per_split3(M, nsplit, 32);
  const dim3 grid(sk_nwg ? sk_nwg : c2::ceil_div(n, RB) * nsplit);
  if (D == 128)
    ce3_dwl_kernel<128, DWL_SBW><<<grid, 256, 0, st>>>((const bf16*)Hx, lg, lg_hb, lg_cw, crow, n, M, per, ps, out,
                                                       accum, sk_nwg, slot_w, slot_b);
  else if (D == 256)
    ce3_dwl_kernel<256, DWL_SBW, CE3L_NW><<<grid, 64 * CE3L_NW, 0, st>>>((const bf16*)Hx, lg, lg_hb, lg_cw, crow, n, M,
                                                                         per, ps, out, accum, sk_nwg, slot_w, slot_b);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  if (sk_nwg) {
    const long T = (M + 31) / 32;
    ce3_sk_combine_kernel<<<dim3(c2::ceil_div(n, RB), RB / 16), 256, 0, st>>>(slot_w, slot_b, n, D, T, sk_nwg, RB, out,
                                                                            ps);
    C2_CHECK_LAUNCH();
  }
  return 0;
}

template <bool SPLIT>
int dw_sk(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, const float* crow, float* gW,
          float* gb, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n == 0) return 0;
  const int nwg = num_cus3();
  if (!gW || !gb || !ws || ws_bytes < sk_ws_bytes(nwg, D)) return (int)hipErrorInvalidValue;
  float* sw = (float*)ws;
  return launch3<1, SPLIT>(Wx, Hx, bias2, crow, n, M, D, 1, nullptr, gb, gW, st, nwg, sw, sw + sk_slot_floats(nwg, D));
}

}  // namespace

extern "C" int c2dsr_ce_rows(const float* part_m, const float* part_s, int n_split, int M, const float* padlogit,
                             const int64_t* tgt, int n, const float* H, const float* W, const float* bias, int D,
                             float* lse, float* lse2, float* loss_row, void* stream);

C2_API int c2dsr_ce3_supported(int D) { return D == 128 || D == 256; }

// the sweep geometry of an instantiation (split = 1: the fp32 mode's split-bf16 kernels, 0: the bf16 mode's), for the
// host's split plans (losshead.py): what = 0 → stationary rows per workgroup (the launch's row block), 1 → swept rows
// per LDS tile
C2_API int c2dsr_ce3_geometry(int split, int what) {
  if (what == 0) return split ? row_block<true, CE3_NW>() : row_block<false, CE3B_NW>();
  if (what == 1) return split ? tile_rows<true>() : tile_rows<false>();
  return -1;
}

C2_API int c2dsr_f32_split_bf16(const float* x, long rows, int D, long rows_out, void* out, void* stream) {
  if (rows_out == 0) return 0;
  if (D % 4 || rows > rows_out) return (int)hipErrorInvalidValue;
  split_bf16_kernel<<<c2::ceil_div(rows_out * D / 4, 256), 256, 0, (hipStream_t)stream>>>(x, rows, D, rows_out,
                                                                                         (bf16*)out);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_ce3_fused_fwd_u(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_split,
                                 float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                                 const float* H, const float* W, const float* bias, float* lse, float* lse2,
                                 float* loss_row, void* stream) {
  if (M == 0) return 0;
  const int e = launch3<0, true>(Hx, Wx, nullptr, bias2, M, n, D, n_split, part_m, part_s, Up, (hipStream_t)stream);
  if (e) return e;
  return c2dsr_ce_rows(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse, lse2, loss_row, stream);
}

C2_API int c2dsr_ce3_fused_dw(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_rsplit,
                              const float* crow, float* dWp, float* dbp, void* stream) {
  if (n == 0) return 0;
  return launch3<1, true>(Wx, Hx, bias2, crow, n, M, D, n_rsplit, nullptr, dbp, dWp, (hipStream_t)stream);
}

C2_API size_t c2dsr_ce3_dw_sk_workspace(int D) { return sk_ws_bytes(num_cus3(), D); }

C2_API int c2dsr_ce3_logits_group(int what) { return what == 0 ? LGG : -1; }

C2_API size_t c2dsr_ce3_logits_floats(int M, int n) {
  return M > 0 && n > 0 ? (size_t)lg_col_blocks(n) * lg_row_blocks(M) * 256 : 0;
}

C2_API int c2dsr_ce3_fused_fwd_u_lg(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D,
                                    int n_split, float* part_m, float* part_s, float* Up, const float* padlogit,
                                    const int64_t* tgt, const float* H, const float* W, const float* bias, float* lse,
                                    float* lse2, float* loss_row, float* lg, void* stream) {
  if (M == 0) return 0;
  if (!lg) return (int)hipErrorInvalidValue;
  const int e = launch3<0, true>(Hx, Wx, nullptr, bias2, M, n, D, n_split, part_m, part_s, Up, (hipStream_t)stream, 0,
                                 nullptr, nullptr, lg);
  if (e) return e;
  return c2dsr_ce_rows(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse, lse2, loss_row, stream);
}

C2_API int c2dsr_ce3_fused_dw_lg(const void* Hx, const float* lg, int M, int n_lg, int col0, int n, int D,
                                 int n_rsplit, const float* crow, float* dWp, float* dbp, void* stream) {
  if (n == 0) return 0;
  if (col0 < 0 || col0 % (16 * (LGG > 2 ? LGG : 2)) || col0 + n > n_lg) return (int)hipErrorInvalidValue;
  const int hb = lg_row_blocks(M);
  return launch_dwl(Hx, lg + (size_t)(col0 / 16) * hb * 256, hb, lg_col_blocks(n_lg) - col0 / 16, crow, n, M, D,
                    n_rsplit, dbp, dWp, (hipStream_t)stream);
}

C2_API int c2dsr_ce3_fused_dw_lg_sk(const void* Hx, const float* lg, int M, int n, int D, const float* crow,
                                    float* gW, float* gb, void* ws, size_t ws_bytes, void* stream) {
  if (n == 0) return 0;
  const int nwg = num_cus3();
  if (!gW || !gb || !ws || ws_bytes < sk_ws_bytes(nwg, D)) return (int)hipErrorInvalidValue;
  float* sw = (float*)ws;
  return launch_dwl(Hx, lg, lg_row_blocks(M), lg_col_blocks(n), crow, n, M, D, 1, gb, gW, (hipStream_t)stream, nwg, sw,
                    sw + sk_slot_floats(nwg, D));
}

C2_API int c2dsr_ce3_fused_dw_sk(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D,
                                 const float* crow, float* gW, float* gb, void* ws, size_t ws_bytes, void* stream) {
  return dw_sk<true>(Hx, Wx, bias2, M, n, D, crow, gW, gb, ws, ws_bytes, (hipStream_t)stream);
}

// The same pair on plain bf16 images [rows][D] (the bf16 mode; drop-in for ce.hip's c2dsr_ce_fused_fwd_u /
// c2dsr_ce_fused_dw, same arguments and outputs): 64-row swept tiles, one MFMA per product.  Images hold whole
// 64-row tiles (zero rows past the end); crow carries a 64-value tail.
C2_API int c2dsr_ce3b_fused_fwd_u(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                                  float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                                  const float* H, const float* W, const float* bias, float* lse, float* lse2,
                                  float* loss_row, void* stream) {
  if (M == 0) return 0;
  const int e = launch3<0, false>(Hb, Wb, nullptr, bias2, M, n, D, n_split, part_m, part_s, Up, (hipStream_t)stream);
  if (e) return e;
  return c2dsr_ce_rows(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse, lse2, loss_row, stream);
}

C2_API int c2dsr_ce3b_fused_dw(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_rsplit,
                               const float* crow, float* dWp, float* dbp, void* stream) {
  if (n == 0) return 0;
  return launch3<1, false>(Wb, Hb, bias2, crow, n, M, D, n_rsplit, nullptr, dbp, dWp, (hipStream_t)stream);
}

C2_API int c2dsr_ce3b_fused_dw_sk(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D,
                                  const float* crow, float* gW, float* gb, void* ws, size_t ws_bytes, void* stream) {
  return dw_sk<false>(Hb, Wb, bias2, M, n, D, crow, gW, gb, ws, ws_bytes, (hipStream_t)stream);
}

#ifdef CE3_STAMP
C2_API int c2dsr_ce3_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(ce3_stamp_acc), sizeof(ce3_stamp_acc));
  if (e == hipSuccess && reset) {
    static const unsigned long long z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(ce3_stamp_acc), z, sizeof(z));
  }
  return (int)e;
}
#endif
