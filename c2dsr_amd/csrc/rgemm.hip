// Row-streaming GEMMs for the sequence-encoder projections at d = 256 (bf16 MFMA, fp32
// accumulate, fp32 activations in HBM):
//
//   rg:  C[M, N] = alpha·A[M, K]·B[N, K]ᵀ + beta·C + bias  (+ relu·dropout epilogue)
//        forward  y = x·Wᵀ   (B = W in bf16)          K = d_in
//        backward dx = dy·W  (B = Wᵀ in bf16)         K = d_out
//   wg:  dW[N, D] += Σ_t dY[t, N]ᵀ·X[t, D]            (split over t, fixed-order combine)
//
// Replaces the nn.Linear addmm / mm calls of TransformerEncoderLayer (in_proj, out_proj,
// linear1, linear2; models/encoders.py:23-27 → torch/nn/modules/transformer.py) at the
// shapes where M = B·L ≫ N, K.  These are HBM-bound (every activation byte is read once
// per product), so the design streams the long operand straight into MFMA registers:
//  * rg: persistent and B-stationary: each wave holds its B columns (all K, bf16) in
//    registers for the whole launch, so B never moves again (an LDS-tiled version was bound
//    by the LDS fill rate of re-loaded B tiles); A streams through a double-buffered LDS
//    image with row-contiguous loads two chunks ahead.
//  * wg: both operands are t-major; 64-row stages of dY and X are converted to bf16 into
//    two images and read TRANSPOSED (ds_read_b64_tr_b16), the t permutation being common
//    to both operands.
#include "img.h"

namespace {
using namespace c2img;
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Epi2 {
  float alpha, beta;
  const float* bias;
  int relu;
  c2::Drop drop;
  int64_t row_base;
  const float* aux;  // AUX epilogues: [M][ldc] fp32 read at the output positions
  float aux_scale;
  const int* rowmap;  // dropout row index = row_base + (rowmap ? rowmap[row] : row)
  const int* auxmap;  // AUX_ACC_MAP: aux row of output row r = auxmap[r] (< 0: none, aux reads 0)
  // guarded ReLU (rg3 GUARD, c2dsr_rgemm_x3_relu_guard): a pre-activation within the split product's error bound
  // of zero is flagged for an exact recompute: |v| <= tau·‖a_r‖·‖w_c‖  ⇔  v² <= gtau2·‖a_r‖²·wn2[c]
  const float* wn2;      // [N] squared norms of the weight rows (output columns)
  unsigned char* gflag;  // [M][N/4]: bit e of byte (r, q) ↔ element (r, 4q + e) (zero on entry; the fix clears)
  float gtau2;
};

// epilogues that read a second [M, N] tensor at the output positions (prefetched one tile ahead):
//   AUX_ACC:  C = alpha·A·Bᵀ + bias + aux             (aux may be C itself: C += A·Bᵀ)
//   AUX_MASK: C = aux > 0 ? (alpha·A·Bᵀ + bias)·s : 0  (backward of drop(relu(.)) given its output aux)
//   AUX_ACC_MAP: C = alpha·A·Bᵀ + bias + aux[auxmap[r]]  (aux holds a compacted subset of the rows; the
//                map of the tile after next is loaded with the aux values of the next one)
enum { AUX_NONE = 0, AUX_ACC = 1, AUX_MASK = 2, AUX_ACC_MAP = 3 };

__device__ __forceinline__ bf16x8 cvt8(float4 a, float4 b) {
  bf16x8 r;
  r[0] = (bf16)a.x; r[1] = (bf16)a.y; r[2] = (bf16)a.z; r[3] = (bf16)a.w;
  r[4] = (bf16)b.x; r[5] = (bf16)b.y; r[6] = (bf16)b.z; r[7] = (bf16)b.w;
  return r;
}

// LDS image of a 32-row A chunk [32][256] bf16: two half-tiles of [32][128] (256-byte rows,
// XOR-swizzled 16-byte chunks as in img.h: conflict-free row fragments).
__device__ __forceinline__ int aoff(int row, int k) { return (k >> 7) * (32 * 256) + swz(row, (k & 127) >> 3) + 2 * (k & 7); }

// buffer descriptor over [base, base + bytes); every input made provably wave-uniform
// (readfirstlane) so the buffer ops need no waterfall loop (cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_bytes(const void* base, long bytes) {
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL));
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, nb, 0x00020000);
}

// B-stationary, persistent.  Each wave keeps CT 32-column tiles of B (all K, bf16) in registers
// for the whole launch; the workgroup (4 waves = 128·CT columns) walks 32-row tiles of A in
// 256-wide k-chunks: 256 threads load a [32][256] fp32 chunk with row-contiguous float4 buffer
// loads two chunks ahead, convert it to bf16 into a double-buffered LDS image, and every wave
// multiplies the image's row fragments with its B registers.  The loop body is branch-free
// (rows past M read 0 / are not stored through the buffer descriptors; the last tile is
// repeated to fill a pair) so the compiler's wait counts stay exact and the prefetch lives.
// Block b runs on XCD b % 8; the G column groups of an XCD walk the same rows in the same
// order, so the G passes over A share its L2.
// AB16: A is bf16 in HBM (the attention backward's dqkv, c2dsr_rgemm_aux_b16a): the same [32][256] chunk
// lands as 8-byte loads and is staged without conversion — half the bytes of the fp32 stream, identical
// products (the fp32 path rounds A to bf16 the same way, RNE).
// X3 (fp32 mode, c2dsr_rgemm_x3): split-bf16 operands — B is the image [N][2K] = hi ‖ lo (ldb = 2K) held in
// registers as two fragment sets, each A chunk is staged as hi = RNE(a) and lo = RNE(a − hi) in two LDS
// images, and every k-step runs three MFMAs (a_hi·b_hi + a_lo·b_hi + a_hi·b_lo; see ce3.hip for the error
// bound: ≈3·2^-17 relative per product term, fp32 accumulation).
template <int KCH, int CT, bool EPI, int AUX = AUX_NONE, bool AB16 = false, bool X3 = false>
__global__ __launch_bounds__(256) void rg_kernel(int M, int N, int K, const void* __restrict__ A, long lda,
                                                 const bf16* __restrict__ B, long ldb, float* C,
                                                 long ldc, Epi2 ep, int G) {
  static_assert(!(AB16 && X3), "split operands take fp32 A");
  constexpr int AIMG = 32 * 256 * 2;  // bytes of one [32][256] bf16 image (X3: lo image right after hi)
  __shared__ __attribute__((aligned(16))) char aimg[2][(X3 ? 2 : 1) * AIMG];
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nslots = gridDim.x >> 3;
  const int nwalk = nslots / G;
  const int g = slot % G, walker = slot / G;
  if (walker >= nwalk) return;  // uniform
  const int RT = (M + 31) >> 5;
  const int rt0 = xcd + 8 * walker, rts = 8 * nwalk;
  const int ntile = rt0 < RT ? (RT - 1 - rt0) / rts + 1 : 0;
  if (ntile == 0) return;  // uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ncol0 = g * (128 * CT) + w * (32 * CT);  // this wave's first column
  // ---- B fragments → registers (once): lane (j = l&31, kh) holds B[col j][16ks + 8kh .. +7]
  bf16x8 bq[CT][KCH * 16];
  bf16x8 bl[X3 ? CT : 1][X3 ? KCH * 16 : 1];  // X3: the lo fragments
  float bcol[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = min(ncol0 + ct * 32 + (lane & 31), N - 1);
#pragma unroll
    for (int ks = 0; ks < KCH * 16; ++ks) {
      if (!X3 && ldb == 0)  // fragment-ordered bf16 image (b16_frag_index): one coalesced 1 KiB piece per load
        bq[ct][ks] = *(const bf16x8*)(B + (((long)(min(ncol0 + ct * 32, N - 1) >> 5) * (K / 16) + ks) * 64 + lane) * 8);
      else
        bq[ct][ks] = *(const bf16x8*)(B + (long)col * ldb + ks * 16 + 8 * (lane >> 5));
      if constexpr (X3) bl[ct][ks] = *(const bf16x8*)(B + (long)col * ldb + K + ks * 16 + 8 * (lane >> 5));
    }
    bcol[ct] = ep.bias ? ep.bias[col] : 0.f;
  }
  // land every loop-invariant register operand here, where the compiler sees the wait
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
    for (int ks = 0; ks < KCH * 16; ++ks) {
      pin(bq[ct][ks]);
      if constexpr (X3) pin(bl[ct][ks]);
    }
    pin(bcol[ct]);
  }
  vm_drain();
  constexpr int AEB = AB16 ? 2 : 4;  // bytes per A element
  const auto asrc = rsrc_bytes(A, (long)M * lda * AEB);  // rows >= M read 0
  const auto csrc = rsrc_bytes(C, (long)M * ldc * 4);  // stores to rows >= M are dropped
  const auto xsrc = rsrc_bytes(AUX != AUX_NONE ? ep.aux : C, (long)M * ldc * 4);  // rows >= M read 0
  // aux values of this wave's outputs for the current tile, loaded one tile ahead
  float xa[AUX != AUX_NONE ? CT : 1][16];
  int xm[AUX == AUX_ACC_MAP ? 16 : 1];  // AUX_ACC_MAP: aux rows of the tile aux_load reads next
  const auto map_load = [&](int tile) {
    if constexpr (AUX == AUX_ACC_MAP) {
      const int r0 = (rt0 + tile * rts) * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = r0 + creg(r, lane);
        xm[r] = rr < M ? ep.auxmap[rr] : -1;
      }
    }
  };
  const auto aux_load = [&](int tile) {
    if constexpr (AUX != AUX_NONE) {
      const int r0 = (rt0 + tile * rts) * 32;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int col = ncol0 + 32 * ct + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int off;
          if constexpr (AUX == AUX_ACC_MAP)
            off = (col < N && xm[r] >= 0) ? (xm[r] * (int)ldc + col) * 4 : 0x7fffffff;
          else
            off = col < N ? ((r0 + creg(r, lane)) * (int)ldc + col) * 4 : 0x7fffffff;
          xa[ct][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xsrc, off, 0, 0));
        }
      }
      map_load(min(tile + 1, ntile - 1));
    }
  };
  map_load(0);
  aux_load(0);
  // chunk c = (tile c / KCH (clamped to the last), k-chunk c % KCH); thread t loads float4
  // t + 256u, u < 8: row (t >> 6) + 4u, columns 4·lane .. +3
  const int ldab = (int)lda * AEB;
  const int lrow = threadIdx.x >> 6;
  // AB16: P[u].xy carry the 4 bf16 values (8 bytes) of the same row / columns
#define RG_LOAD(c, P)                                                                                          \
  {                                                                                                            \
    const int tile_ = min((c) / KCH, ntile - 1), kc_ = (c) % KCH;                                              \
    const int vo_ = ((rt0 + tile_ * rts) * 32 + lrow) * ldab + (kc_ * 256 + 4 * lane) * AEB;                   \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                                            \
      if constexpr (AB16) {                                                                                    \
        const f32x2 h_ = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(asrc, vo_ + u * 4 * ldab, 0, 0)); \
        P[u].x = h_[0];                                                                                        \
        P[u].y = h_[1];                                                                                        \
      } else {                                                                                                 \
        P[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(asrc, vo_ + u * 4 * ldab, 0, 0)); \
      }                                                                                                        \
    }                                                                                                          \
  }
#define RG_STAGE(P, im)                                                                                        \
  {                                                                                                            \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                                            \
      bf16x4 v_;                                                                                               \
      if constexpr (AB16) {                                                                                    \
        f32x2 g_;                                                                                              \
        g_[0] = P[u].x;                                                                                        \
        g_[1] = P[u].y;                                                                                        \
        v_ = __builtin_bit_cast(bf16x4, g_);                                                                   \
      } else {                                                                                                 \
        v_[0] = (bf16)P[u].x; v_[1] = (bf16)P[u].y; v_[2] = (bf16)P[u].z; v_[3] = (bf16)P[u].w;                \
      }                                                                                                        \
      *(bf16x4*)((im) + aoff(lrow + 4 * u, 4 * lane)) = v_;                                                   \
      if constexpr (X3) {                                                                                      \
        bf16x4 l_;                                                                                             \
        l_[0] = (bf16)(P[u].x - (float)v_[0]); l_[1] = (bf16)(P[u].y - (float)v_[1]);                          \
        l_[2] = (bf16)(P[u].z - (float)v_[2]); l_[3] = (bf16)(P[u].w - (float)v_[3]);                          \
        *(bf16x4*)((im) + AIMG + aoff(lrow + 4 * u, 4 * lane)) = l_;                                           \
      }                                                                                                        \
    }                                                                                                          \
  }
  f32x16 acc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
  // step c (k-chunk KC, compile-time): R (free) is refilled with chunk c+2; S holds chunk c+1,
  // staged after the multiply.  Written out per chunk so R/S alternate without copies.
#define RG_STEP(c, KC, R, S)                                                                                   \
  {                                                                                                            \
    RG_LOAD((c) + 2, R)                                                                                        \
    const char* im_ = aimg[(c) & 1];                                                                           \
    _Pragma("unroll") for (int ks = 0; ks < 16; ++ks) {                                                        \
      const bf16x8 af_ = *(const bf16x8*)(im_ + aoff(lane & 31, ks * 16 + 8 * (lane >> 5)));                   \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) acc[ct] =                                              \
          __builtin_amdgcn_mfma_f32_32x32x16_bf16(af_, bq[ct][(KC) * 16 + ks], acc[ct], 0, 0, 0);              \
      if constexpr (X3) {                                                                                      \
        const bf16x8 al_ = *(const bf16x8*)(im_ + AIMG + aoff(lane & 31, ks * 16 + 8 * (lane >> 5)));          \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                                    \
          acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al_, bq[ct][(KC) * 16 + ks], acc[ct], 0, 0, 0);    \
          acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af_, bl[ct][(KC) * 16 + ks], acc[ct], 0, 0, 0);    \
        }                                                                                                      \
      }                                                                                                        \
    }                                                                                                          \
    if constexpr ((KC) == KCH - 1) epilogue(min((c) / KCH, ntile - 1), (c) / KCH < ntile);                    \
    RG_STAGE(S, aimg[((c) + 1) & 1])                                                                           \
    __syncthreads();                                                                                           \
  }
  // live = false: the repeated last tile of an odd count (its stores are dropped, so an in-place
  // AUX_ACC never adds twice)
  const auto epilogue = [&](int tile, bool live) {
    const int r0 = (rt0 + tile * rts) * 32;
    // lane holds C[r0 + creg(r)][ncol0 + 32ct + (lane&31)]
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int col = ncol0 + 32 * ct + (lane & 31);
      // drop(relu) multipliers of this column tile's 16 registers, in one of three kernel-uniform modes:
      // no dropout; pairs — lanes l and l^1 hold the same rows at columns 2m, 2m+1, one element pair, one
      // hash (N even): each lane hashes 8 of the 16 rows (even lane rows 0-7, odd lane 8-15) and takes the
      // partner's 8; per element (N odd)
      float dm[EPI ? 16 : 1];
      if constexpr (EPI) {
        if (!ep.drop.active()) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dm[r] = 1.f;
        } else if ((N & 1) == 0) {
          const int par = lane & 1;
          uint32_t hown[8], hpar[8];
          int rows_[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) rows_[j] = r0 + creg(j + 8 * par, lane);
          if (ep.rowmap) {
#pragma unroll
            for (int j = 0; j < 8; ++j) rows_[j] = ep.rowmap[min(rows_[j], M - 1)];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j)
            hown[j] = c2::pair_hash(((uint64_t)(ep.row_base + rows_[j]) * N + (col & ~1)) >> 1, ep.drop.k0,
                                    ep.drop.k1);
#pragma unroll
          for (int j = 0; j < 8; ++j) hpar[j] = __shfl_xor(hown[j], 1, 64);
          const uint32_t sh = 16 * (col & 1);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t h = ((r >> 3) == par) ? hown[r & 7] : hpar[r & 7];
            dm[r] = ((h >> sh) & 0xffffu) >= ep.drop.thr ? ep.drop.scale : 0.f;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = r0 + creg(r, lane);
            const int rg_ = ep.rowmap ? ep.rowmap[min(rr, M - 1)] : rr;
            dm[r] = ep.drop.mul((uint64_t)(ep.row_base + rg_) * N + col);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = r0 + creg(r, lane);
        float v = fmaf(ep.alpha, acc[ct][r], bcol[ct]);
        if constexpr (EPI) v = fmaxf(v, 0.f) * dm[r];
        if constexpr (AUX == AUX_ACC || AUX == AUX_ACC_MAP) v += xa[ct][r];
        if constexpr (AUX == AUX_MASK) v = xa[ct][r] > 0.f ? v * ep.aux_scale : 0.f;
        const int off = (col < N && live) ? (rr * (int)ldc + col) * 4 : 0x7fffffff;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), csrc, off, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
    }
    aux_load(min(tile + 1, ntile - 1));  // the next tile's aux values, in flight under its MFMAs
  };
  float4 Pa[8], Pb[8];
  RG_LOAD(0, Pa)
  RG_LOAD(1, Pb)
  RG_STAGE(Pa, aimg[0])
  __syncthreads();
  const int npair = (ntile + 1) >> 1;
  for (int i = 0; i < npair; ++i) {
    const int c0 = i * 2 * KCH;
    if constexpr (KCH == 1) {
      RG_STEP(c0, 0, Pa, Pb)
      RG_STEP(c0 + 1, 0, Pb, Pa)
    } else if constexpr (KCH == 2) {
      RG_STEP(c0, 0, Pa, Pb)
      RG_STEP(c0 + 1, 1, Pb, Pa)
      RG_STEP(c0 + 2, 0, Pa, Pb)
      RG_STEP(c0 + 3, 1, Pb, Pa)
    } else {
      RG_STEP(c0, 0, Pa, Pb)
      RG_STEP(c0 + 1, 1, Pb, Pa)
      RG_STEP(c0 + 2, 2, Pa, Pb)
      RG_STEP(c0 + 3, 0, Pb, Pa)
      RG_STEP(c0 + 4, 1, Pa, Pb)
      RG_STEP(c0 + 5, 2, Pb, Pa)
    }
  }
#undef RG_STEP
#undef RG_STAGE
#undef RG_LOAD
}

// ---------------------------------------------------------------------------------------------
// rg3: the split-bf16 (fp32 mode) row-streaming GEMM on v_mfma_f32_16x16x32_bf16, computed transposed:
// Cᵀ tile = B·Aᵀ, so a lane's accumulator holds 4 CONSECUTIVE columns of one output row (float4 stores,
// a float4 epilogue: bias, relu·dropout pairs, aux) instead of 16 rows of one column (16 scalar stores per
// lane per tile: the old epilogue was store-issue-bound).  B (the split weight image, hi ‖ lo) is the MFMA
// A operand, pinned to AGPRs for the launch: 64 columns × K = 256 (or 32 × 512) hi + lo = 256 registers per
// lane; the workgroup covers 256 / KCH columns, so at N = 256 / K = 256 every A row is read from HBM once
// and converted once.  A streams as before: [32][256] fp32 chunks loaded two ahead in registers, split into
// hi / lo images (img.h swz16 layout; the conversion of chunk c+1 interleaved with chunk c's MFMAs), read as
// the MFMA B operand (lane ↔ row l%16, k 8·(l/16)..).  Per 32-row chunk and wave: 2 row blocks × NCB column
// blocks × 8 k-steps × 3 MFMAs (a_hi·b_hi + a_hi·b_lo + a_lo·b_hi).
// Rows past M read 0 and are not stored (buffer descriptors); N % 4 == 0, ldc % 4 == 0.
// Fragment order of a split weight image (c2dsr_to_split_bf16_frag_multi → c2dsr_rgemm_x3f): the values one rg3
// wave loads for (16-column block cb, k-step ks, hi / lo) are one contiguous 1 KiB piece — lane g·16 + l16 holds
// column 16cb + l16, k = 32ks + 8g .. +7 — so each weight load is one coalesced 1 KiB read instead of 16 row
// segments of 64 B.  Piece (cb, ks, hl) = cb·(2K/32) + 2ks + hl.
__host__ __device__ __forceinline__ long split_frag_index(int col, int k, int hl, int K) {
  const long piece = (long)(col >> 4) * (K / 16) + 2 * (k >> 5) + hl;
  return (piece * 64 + ((k >> 3) & 3) * 16 + (col & 15)) * 8 + (k & 7);
}
// The same for a bf16 weight image and rg_kernel (the bf16 mode: 32x32 fragments, lane (j = l % 32, kh = l / 32)
// holds column 32ct + j, k = 16ks + 8kh .. +7): piece (32-column block, k-step of 16) = one 1 KiB wave load.
__host__ __device__ __forceinline__ long b16_frag_index(int col, int k, int K) {
  const long piece = (long)(col >> 5) * (K / 16) + (k >> 4);
  return (piece * 64 + ((k >> 3) & 1) * 32 + (col & 31)) * 8 + (k & 7);
}
__device__ __forceinline__ void x3_0(f32x4& acc, const bf16x8& wh, const bf16x8& wl, const bf16x8& ah,
                                     const bf16x8& al) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %1, %3, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
      : "=&v"(acc)
      : "a"(wh), "a"(wl), "v"(ah), "v"(al));
}
__device__ __forceinline__ void x3_acc(f32x4& acc, const bf16x8& wh, const bf16x8& wl, const bf16x8& ah,
                                       const bf16x8& al) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
      : "+v"(acc)
      : "a"(wh), "a"(wl), "v"(ah), "v"(al));
}

#ifndef RG3_GUARD_NW  // waves per workgroup of the guarded instance (at 4 its unrolled three-set loop spills 39 registers, at 8 five)
#define RG3_GUARD_NW 8
#endif
#ifndef RG3_NW
#define RG3_NW 8  // waves per workgroup of the split-bf16 row-streaming GEMM (8: 2 per SIMD, measured 5-13% over 4 at N=256)
#endif
#ifdef RG3_STAMP  // diagnostic build only: per-phase cycle sums of the rg3 chunk loop (tools/rg_micro.py prints them)
__device__ unsigned long long rg3_stamp_acc[8];
#define RSTAMP(i)                                                  \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const unsigned now_ = (unsigned)__builtin_amdgcn_s_memtime();  \
    st_acc[i] += now_ - st_prev;                                   \
    st_prev = now_;                                                \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)
#else
#define RSTAMP(i) \
  do {            \
  } while (0)
#endif

// GUARD (EPI, K = 256 only; the ReLU producer linear1 in the fp32 mode): a pre-activation v = a·w + b whose split
// product error could move it across zero — |a·w − split(a·w)| ≤ 3·2^-18·Σ|a_k w_k| ≤ 3·2^-18·‖a‖‖w‖, guarded at
// 2^-15·‖a‖‖w‖ — is listed (r·N + c) and recomputed exactly by guard_fix_kernel: the ReLU's sign decisions, which
// select the dy·x terms of the weight gradient, are those of an fp32 product (tools/fp32_diag.py).  ‖a_r‖² is summed
// while a chunk is staged (a wave holds whole rows at K = 256), ‖w_c‖² comes from the caller (ep.wn2).
// NW: waves per workgroup — 4 (one per SIMD, 64 columns × K hi + lo = 256 AGPRs each) or 8 (two per SIMD, half the
// columns each: one wave's staging / epilogue / barrier waits run under the other's MFMAs).  The workgroup covers the
// same 256 / KCH columns either way; every output element's accumulation order is the same.
template <int KCH, bool EPI, int AUX, bool GUARD = false, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void rg3_kernel(int M, int N, const float* __restrict__ A, long lda,
                                                         const bf16* __restrict__ B, long ldb, float* C, long ldc,
                                                         Epi2 ep, int G) {
  static_assert(!GUARD || (EPI && KCH == 1 && AUX == AUX_NONE), "guarded ReLU: the K = 256 relu·dropout epilogue");
  static_assert(NW == 4 || NW == 8, "rg3 waves");
  constexpr int K = 256 * KCH;
  constexpr int NCB = 16 / NW / KCH;  // 16-column blocks per wave
  constexpr int CW = 16 * NCB;      // columns per wave
  constexpr int WGC = NW * CW;      // columns per workgroup
  constexpr int SPU = 32 / NW;      // rows of a chunk each thread stages (float4 per thread per chunk)
  constexpr int RA = NW == 4 ? 3 : 2;  // chunks loaded ahead (register sets): 3 at one wave per SIMD, 2 at two
  constexpr int IMGB = 32 * 256 * 2;  // bytes of one [32][256] bf16 image
  constexpr int NST = 16;           // MFMA steps per chunk: (k-step ks, row block rb)
  __shared__ __attribute__((aligned(16))) char aimg[2][2 * IMGB];  // [buffer][hi | lo]
  __shared__ float rn2s[2][GUARD ? 32 : 1];  // GUARD: ‖a_r‖² of the chunk's 32 rows, per image buffer
  __shared__ __attribute__((aligned(16))) float wn2s[GUARD ? 256 : 1];  // GUARD: ‖w_c‖² of the workgroup's columns
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nslots = gridDim.x >> 3;
  const int nwalk = nslots / G;
  const int gcol = slot % G, walker = slot / G;
  if (walker >= nwalk) return;  // uniform
  const int RT = (M + 31) >> 5;
  const int rt0 = xcd + 8 * walker, rts = 8 * nwalk;
  const int ntile = rt0 < RT ? (RT - 1 - rt0) / rts + 1 : 0;
  if (ntile == 0) return;  // uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, g = lane >> 4;
#ifdef RG3_STAMP
  unsigned st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = (unsigned)__builtin_amdgcn_s_memtime();
#endif
  const int ncol0 = gcol * WGC + w * CW;
  bf16x8 wh[NCB][8 * KCH], wl[NCB][8 * KCH];  // the weight columns' hi / lo fragments (AGPRs)
  f32x4 bias4[NCB];
  const auto asrc = rsrc_bytes(A, (long)M * lda * 4);   // rows >= M read 0
  const auto csrc = rsrc_bytes(C, (long)M * ldc * 4);   // stores to rows >= M are dropped
  const auto fsrc = rsrc_bytes(GUARD ? (void*)ep.gflag : (void*)C, GUARD ? (long)M * (N >> 2) : 0);
  const auto xsrc = rsrc_bytes(AUX != AUX_NONE ? ep.aux : C, (long)M * ldc * 4);  // rows >= M read 0
  // per-lane image offsets: row l16 (+16 rb), chunk 4c + g of the 128-column half-tile
  int roff[4];
  {
    const int sw = swz16(l16);
#pragma unroll
    for (int c = 0; c < 4; ++c) roff[c] = (int)lds_addr(aimg[0]) + l16 * 256 + 16 * ((4 * c + g) ^ sw);
  }
  // staging: thread t converts the float4 of row lrow + NW·u (u < SPU), columns 4·lane .. +3 of a chunk
  const int lrow = threadIdx.x >> 6;
  int soff[SPU];
#pragma unroll
  for (int u = 0; u < SPU; ++u) {
    const int row = lrow + NW * u, k = 4 * lane;
    soff[u] = (int)lds_addr(aimg[0]) + (k >> 7) * (32 * 256) + row * 256 + 16 * (((k & 127) >> 3) ^ swz16(row)) +
              2 * (k & 7);
  }
  const int ldab = (int)lda * 4;
  auto load = [&](int c, float4 (&P)[SPU]) {
    const int tile = min(c / KCH, ntile - 1), kc = c % KCH;
    const int vo = ((rt0 + tile * rts) * 32 + lrow) * ldab + (kc * 256 + 4 * lane) * 4;
#pragma unroll
    for (int u = 0; u < SPU; ++u)
      P[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(asrc, vo + u * NW * ldab, 0, 0));
  };
  typedef __attribute__((address_space(3))) bf16x4 lds4;
  auto stage1 = [&](const float4& v, int u, int buf) {
    bf16x4 h, l;
    h[0] = (bf16)v.x; h[1] = (bf16)v.y; h[2] = (bf16)v.z; h[3] = (bf16)v.w;
    l[0] = (bf16)(v.x - (float)h[0]); l[1] = (bf16)(v.y - (float)h[1]);
    l[2] = (bf16)(v.z - (float)h[2]); l[3] = (bf16)(v.w - (float)h[3]);
    *(lds4*)(size_t)lds_base(soff[u] + buf * 2 * IMGB) = h;
    *(lds4*)(size_t)lds_base(soff[u] + buf * 2 * IMGB + IMGB) = l;
    if constexpr (GUARD) {  // ‖row lrow + 4u‖²: the row is this wave's 64 lanes × 4 (K = 256)
      float x = fmaf(v.w, v.w, fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x)));
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xf, 0xf, false));   // quad_perm 2,3,0,1
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x124, 0xf, 0xf, false));  // row_ror 4
      x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xf, 0xf, false));  // row_ror 8
      const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
      x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
      const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
      x = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
      if (lane == 0) rn2s[buf][lrow + NW * u] = x;
    }
  };
  // aux / row maps of the current tile (loaded at its first chunk, used by its epilogue)
  f32x4 aux4[AUX != AUX_NONE ? 2 : 1][AUX != AUX_NONE ? NCB : 1];
  int amap[2], dmap[2];
  auto tile_rows = [&](int tile, int rb) { return (rt0 + tile * rts) * 32 + 16 * rb + l16; };
  auto pre_tile = [&](int tile) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int row = tile_rows(tile, rb);
      if constexpr (AUX == AUX_ACC_MAP) amap[rb] = row < M ? ep.auxmap[row] : -1;
      if constexpr (EPI) dmap[rb] = ep.rowmap ? ep.rowmap[min(row, M - 1)] : row;
    }
    if constexpr (AUX != AUX_NONE) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int row = tile_rows(tile, rb);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int col = ncol0 + 16 * cb + 4 * g;
          int off;
          if constexpr (AUX == AUX_ACC_MAP)
            off = (col < N && amap[rb] >= 0) ? (amap[rb] * (int)ldc + col) * 4 : 0x7ffffff0;
          else
            off = col < N ? (row * (int)ldc + col) * 4 : 0x7ffffff0;
          aux4[rb][cb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrc, off, 0, 0));
        }
      }
    }
  };
  f32x4 acc[2][NCB];
  auto epilogue = [&](int tile, bool live, int buf) {
    mfma_drain();
    unsigned gmask = 0;  // GUARD: bit (rb·NCB + cb)·4 + i ↔ element (rb, cb, i) of this lane needs the exact product
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int row = tile_rows(tile, rb);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = ncol0 + 16 * cb + 4 * g;
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaf(ep.alpha, acc[rb][cb][i], bias4[cb][i]);
        if constexpr (GUARD) {
          const float rr = rn2s[buf][16 * rb + l16] * ep.gtau2;
          const f32x4 wq = *(const f32x4*)&wn2s[16 * cb + w * CW + 4 * g];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            gmask |= (unsigned)(live && row < M && col + i < N && v[i] * v[i] <= rr * wq[i]) << ((rb * NCB + cb) * 4 + i);
        }
        if constexpr (EPI) {
          const float4 dm = ep.drop.mul4((uint64_t)(ep.row_base + dmap[rb]) * N + col);
          v[0] = fmaxf(v[0], 0.f) * dm.x;
          v[1] = fmaxf(v[1], 0.f) * dm.y;
          v[2] = fmaxf(v[2], 0.f) * dm.z;
          v[3] = fmaxf(v[3], 0.f) * dm.w;
        }
        if constexpr (AUX == AUX_ACC || AUX == AUX_ACC_MAP) v += aux4[rb][cb];
        if constexpr (AUX == AUX_MASK) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = aux4[rb][cb][i] > 0.f ? v[i] * ep.aux_scale : 0.f;
        }
        const int off = (col < N && live) ? (row * (int)ldc + col) * 4 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), csrc, off, 0, 0);
      }
    }
    if constexpr (GUARD) {
      // the lane's 4-column groups with a guarded element: one flag byte each (a group belongs to one lane),
      // branch-free — unflagged groups store out of range
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const unsigned f = (gmask >> ((rb * NCB + cb) * 4)) & 0xfu;
          const int off = f ? tile_rows(tile, rb) * (N >> 2) + ((ncol0 + 16 * cb + 4 * g) >> 2) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b8((unsigned char)f, fsrc, off, 0, 0);
        }
      }
    }
  };
  float4 Pa[SPU], Pb[SPU], Pc[RA == 3 ? SPU : 1];
  load(0, Pa);
  load(1, Pb);
  if constexpr (RA == 3) load(2, Pc);
  // the weight fragments are fetched (L2) while the first A chunks are in flight (HBM)
  // B (split image) fragments → AGPRs: column ncol0 + 16cb + l16, k = 32ks + 8g
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const long col = min(ncol0 + 16 * cb + l16, N - 1);
#pragma unroll
    for (int ks = 0; ks < 8 * KCH; ++ks) {
#ifdef RG3_X_NOW  // timing experiment only (wrong results): no weight fetch, the prologue's cost without it
      wh[cb][ks] = wl[cb][ks] = bf16x8{} + (bf16)(0.001f * (col + ks));
#else
      if (ldb == 0) {  // fragment-ordered image (split_frag_index): one coalesced 1 KiB piece per load
        const long f = ((long)(min(ncol0 + 16 * cb, N - 1) >> 4) * (K / 16) + 2 * ks) * 64 + lane;
        wh[cb][ks] = *(const bf16x8*)(B + f * 8);
        wl[cb][ks] = *(const bf16x8*)(B + (f + 64) * 8);
      } else {
        wh[cb][ks] = *(const bf16x8*)(B + col * ldb + ks * 32 + 8 * g);
        wl[cb][ks] = *(const bf16x8*)(B + col * ldb + K + ks * 32 + 8 * g);
      }
#endif
    }
    const int c4 = min(ncol0 + 16 * cb + 4 * g, N - 4);
    bias4[cb] = ep.bias ? *(const f32x4*)(ep.bias + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (GUARD) {
    if ((int)threadIdx.x < WGC) wn2s[threadIdx.x] = ep.wn2[min(gcol * WGC + (int)threadIdx.x, N - 1)];
  }
  vm_drain();
#pragma unroll
  for (int u = 0; u < SPU; ++u) stage1(Pa[u], u, 0);
  pre_tile(0);
  __syncthreads();
  RSTAMP(0);
  // chunk c (k-chunk KC): MFMAs on image c&1 ∥ split of chunk c+1 (registers S) into image (c+1)&1; R is
  // refilled with chunk c+3 first (three register sets: a staged chunk was loaded two steps earlier)
  auto step = [&]<int KC>(int c, float4 (&R)[SPU], float4 (&S)[SPU]) {
    load(c + RA, R);
    const int buf = c & 1, nb = (c + 1) & 1;
    const int tile = c / KCH;
    bf16x8 fr[4][2];
    auto rd = [&]<int ST>() {
      constexpr int ks = ST >> 1, rb = ST & 1;
      constexpr int IMM = (ks >> 2) * (32 * 256) + rb * 16 * 256;
      fr[ST & 3][0] = lds_ld128<IMM>(roff[ks & 3] + buf * 2 * IMGB);
      fr[ST & 3][1] = lds_ld128<IMM + IMGB>(roff[ks & 3] + buf * 2 * IMGB);
    };
    rd.template operator()<0>();
    rd.template operator()<1>();
    [&]<int... SS>(std::integer_sequence<int, SS...>) {
      (
          [&] {
            constexpr int st = SS, ks = st >> 1, rb = st & 1;
            if constexpr (st + 2 < NST) rd.template operator()<st + 2>();
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
              if constexpr (KC == 0 && ks == 0)
                x3_0(acc[rb][cb], wh[cb][KC * 8 + ks], wl[cb][KC * 8 + ks], fr[st & 3][0], fr[st & 3][1]);
              else
                x3_acc(acc[rb][cb], wh[cb][KC * 8 + ks], wl[cb][KC * 8 + ks], fr[st & 3][0], fr[st & 3][1]);
            }
            if constexpr (st % (NST / SPU) == NST / SPU - 1) stage1(S[st / (NST / SPU)], st / (NST / SPU), nb);
            __builtin_amdgcn_sched_barrier(0);
          }(),
          ...);
    }(std::make_integer_sequence<int, NST>{});
    RSTAMP(1);
    if constexpr (KC == KCH - 1) {
      epilogue(min(tile, ntile - 1), tile < ntile, buf);
      pre_tile(min(tile + 1, ntile - 1));
    }
    RSTAMP(2);
    __syncthreads();
    RSTAMP(3);
  };
  const int nchunk = ntile * KCH;
  if constexpr (RA == 2) {
    for (int c0 = 0; c0 < nchunk; c0 += 2) {  // register sets and k-chunks both rotate with period 2
      step.template operator()<0>(c0, Pa, Pb);
      if (c0 + 1 >= nchunk) break;
      step.template operator()<1 % KCH>(c0 + 1, Pb, Pa);
    }
  } else
  for (int c0 = 0; c0 < nchunk; c0 += 6) {  // register sets rotate with period 3, k-chunks with period KCH
    step.template operator()<0>(c0, Pa, Pb);
    if (c0 + 1 >= nchunk) break;
    step.template operator()<1 % KCH>(c0 + 1, Pb, Pc);
    if (c0 + 2 >= nchunk) break;
    step.template operator()<0>(c0 + 2, Pc, Pa);
    if (c0 + 3 >= nchunk) break;
    step.template operator()<1 % KCH>(c0 + 3, Pa, Pb);
    if (c0 + 4 >= nchunk) break;
    step.template operator()<0>(c0 + 4, Pb, Pc);
    if (c0 + 5 >= nchunk) break;
    step.template operator()<1 % KCH>(c0 + 5, Pc, Pa);
  }
#ifdef RG3_STAMP
  if (lane == 0) {
    for (int i = 0; i < 4; ++i) atomicAdd(&rg3_stamp_acc[i], (unsigned long long)st_acc[i]);
    atomicAdd(&rg3_stamp_acc[6], (unsigned long long)nchunk);
    atomicAdd(&rg3_stamp_acc[7], 1ull);
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// wg: dW[N, 256] partials = Σ_{t in split} dY[t, N]ᵀ·X[t, 256], both operands t-major (fp32).
// Workgroup = 4 waves = a 128-row slice of N × all 256 columns (wave: 64 × 128, 2×4 MFMA tiles);
// 32-row chunks of dY (32×128) and X (32×256) are converted to bf16 into LDS images and both
// operands are read TRANSPOSED (ds_read_b64_tr_b16): the reduction runs over the image rows (t)
// in the same permuted order for A and B.  Loads run two chunks ahead in registers, the loop
// body is branch-free (rows past T read 0 through the buffer descriptors).
// part[split][N][256] (fixed-order combine: c2dsr_sum_parts).

// transposed fragment from a [32][ncols] image (half-tiles of [32][128], stride 8 KB)
__device__ __forceinline__ bf16x8 tr32(const char* img, int rr0, int kb0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (32 * 256);
  const char* a0 = img + base + swz(row, ch) + 8 * (p & 1);
  const char* a1 = img + base + swz(row + 8, ch) + 8 * (p & 1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// YB16: dY is bf16 in HBM (the attention backward's dqkv): 8-byte loads, no conversion; the bias
// column sums add the same bf16 values.
// Segments (c2dsr_wgemm_multi): the row sets of several products into the same dW (one weight used by several
// encoder passes) walked as one virtual row range; segment k occupies virtual rows [vbeg[k], vbeg[k+1]) (its
// T[k] rows padded to a multiple of 32, so no 32-row chunk straddles two segments or a split end).
constexpr int WG_MAXSEG = 4;
#ifndef WG_AHEAD
#define WG_AHEAD 2  // chunks loaded ahead (3: three register sets — spills at 4 waves, 2.5x slower)
#endif
#ifndef WG_NW_X3
#define WG_NW_X3 8  // waves per workgroup of the split-bf16 weight gradient (4 → 8: T = 57k, N = 256: 50.8 → 43.3 µs)
#endif
#ifndef WG_AH_X3
#define WG_AH_X3 WG_AHEAD
#endif
struct WSeg {
  const void* dY[WG_MAXSEG];
  const float* X[WG_MAXSEG];
  int ldy[WG_MAXSEG], ldx[WG_MAXSEG], T[WG_MAXSEG];
  int vbeg[WG_MAXSEG + 1];
  int nseg;
};
template <typename V>
__device__ __forceinline__ V wg_pick(const V (&a)[WG_MAXSEG], int k) {  // uniform k: no dynamic indexing
  return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

// X3 (fp32 mode, c2dsr_wgemm_x3): both chunks staged as split-bf16 hi and lo images, three MFMAs per step
// (y_hi·x_hi + y_lo·x_hi + y_hi·x_lo, fp32 accumulation; the bias column sums stay exact fp32).
// NW: waves per workgroup — 4 (wave tile 64 n × 128 i) or 8 (32 n × 128 i: two waves per SIMD, so one wave's
// staging and barrier waits run under the other's MFMAs); AH: chunks loaded ahead in registers (2 or 3).  The
// accumulation order of every dW element is the same for all (NW, AH); the bias column sums (db) are not: each
// thread's partial covers NYU rows and red_b combines NT/32 partials, so db's bits depend on NW (deterministic for
// a given NW).
template <bool YB16, bool X3 = false, int NW = 4, int AH = WG_AHEAD>
__global__ __launch_bounds__(64 * NW) void wg_kernel(int N, WSeg sg, float* __restrict__ part,
                                                     float* __restrict__ part_b, int NTL, int rows_per_split) {
  static_assert(!(YB16 && X3), "split operands take fp32 dY");
  static_assert((NW == 4 || NW == 8) && (AH == 2 || AH == 3), "wg shape");
  constexpr int NT = 64 * NW;       // threads
  constexpr int NYU = 1024 / NT;    // dY float4 per thread per chunk (32 rows × 128 columns)
  constexpr int NXU = 2048 / NT;    // X float4 per thread per chunk (32 rows × 256 columns)
  constexpr int NA = 8 / NW;        // 32-row n tiles per wave
  const int T = sg.vbeg[WG_MAXSEG];  // virtual rows (entries past nseg repeat the total)
  constexpr int YIMG = 32 * 128 * 2, XIMG = 32 * 256 * 2;  // bytes per image (X3: lo image after hi)
  __shared__ __attribute__((aligned(16))) float4 red_b[NT / 32][32];
  __shared__ __attribute__((aligned(16))) char yimg[2][(X3 ? 2 : 1) * YIMG];
  __shared__ __attribute__((aligned(16))) char ximg[2][(X3 ? 2 : 1) * XIMG];
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nslots = gridDim.x >> 3;
  const int per_x = nslots / NTL;  // splits per XCD
  const int nt = slot % NTL, sl = slot / NTL;
  if (sl >= per_x) return;  // uniform
  const int split = xcd + 8 * sl;
  const int t_beg = split * rows_per_split;
  const int t_end = min(T, t_beg + rows_per_split);
  const int nchunk = t_end > t_beg ? (t_end - t_beg + 31) >> 5 : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n_base = nt * 128;
  constexpr int YEB = YB16 ? 2 : 4;
  const int lrow = threadIdx.x >> 6;  // 0..NW-1
  // chunk c: thread t loads dY rows lrow + 4u (u < 8) → 1 float4 (cols 4·(lane&31) of the 128) per
  // half-wave pair... simpler: dY chunk 32×128 floats = 1024 float4 = 4 per thread, X 2048 = 8 per thread.
  // The chunk's segment (uniform): rows past its T read 0 through the descriptors.
#define WG_LOAD(c, PY, PX)                                                                                    \
  {                                                                                                           \
    const int tv_ = t_beg + min(c, nchunk - 1) * 32;                                                          \
    int k_ = 0;                                                                                               \
    _Pragma("unroll") for (int kk = 1; kk < WG_MAXSEG; ++kk) k_ = (kk < sg.nseg && tv_ >= sg.vbeg[kk]) ? kk : k_; \
    const int t0_ = tv_ - (k_ == 0 ? sg.vbeg[0] : k_ == 1 ? sg.vbeg[1] : k_ == 2 ? sg.vbeg[2] : sg.vbeg[3]);  \
    const int ly_ = wg_pick(sg.ldy, k_), lx_ = wg_pick(sg.ldx, k_), tk_ = wg_pick(sg.T, k_);                 \
    const int ldyb = ly_ * YEB, ldxb = lx_ * 4;                                                               \
    const auto ysrc = rsrc_bytes(wg_pick(sg.dY, k_), (long)tk_ * ly_ * YEB);                                  \
    const auto xsrc = rsrc_bytes(wg_pick(sg.X, k_), (long)tk_ * lx_ * 4);                                     \
    _Pragma("unroll") for (int u = 0; u < NYU; ++u) {                                                         \
      const int q_ = threadIdx.x + NT * u; /* 0..1023: row q_>>5, float4 q_&31 */                            \
      const int yo_ = (t0_ + (q_ >> 5)) * ldyb + (n_base + 4 * (q_ & 31)) * YEB;                              \
      if constexpr (YB16) {                                                                                   \
        const auto h_ = __builtin_amdgcn_raw_buffer_load_b64(ysrc, yo_, 0, 0);                                \
        const bf16x4 b_ = __builtin_bit_cast(bf16x4, h_);                                                     \
        PY[u] = make_float4((float)b_[0], (float)b_[1], (float)b_[2], (float)b_[3]);                          \
      } else {                                                                                                \
        PY[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ysrc, yo_, 0, 0));           \
      }                                                                                                       \
    }                                                                                                         \
    _Pragma("unroll") for (int u = 0; u < NXU; ++u) {                                                         \
      PX[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(                              \
                                             xsrc, (t0_ + lrow + NW * u) * ldxb + 16 * lane, 0, 0));          \
    }                                                                                                         \
  }
#define WG_PUT(im, LOFF, row, col, v4)                                                                        \
  {                                                                                                           \
    bf16x4 b_;                                                                                                \
    b_[0] = (bf16)(v4).x; b_[1] = (bf16)(v4).y; b_[2] = (bf16)(v4).z; b_[3] = (bf16)(v4).w;                   \
    const int o_ = ((col) >> 7) * (32 * 256) + swz(row, ((col) & 127) >> 3) + 2 * ((col) & 7);               \
    *(bf16x4*)((im) + o_) = b_;                                                                               \
    if constexpr (X3) {                                                                                       \
      bf16x4 l_;                                                                                              \
      l_[0] = (bf16)((v4).x - (float)b_[0]); l_[1] = (bf16)((v4).y - (float)b_[1]);                           \
      l_[2] = (bf16)((v4).z - (float)b_[2]); l_[3] = (bf16)((v4).w - (float)b_[3]);                           \
      *(bf16x4*)((im) + (LOFF) + o_) = l_;                                                                    \
    }                                                                                                         \
  }
// staging chunk cc also adds its dY rows into the column sums (the bias gradient): this thread
// always holds columns n_base + 4·(tid & 31) of rows (tid >> 5) + 8u; clamped re-loads past the
// last chunk are weighted 0
#define WG_STAGE(PY, PX, b, cc)                                                                               \
  {                                                                                                           \
    const float on_ = (cc) < nchunk ? 1.f : 0.f;                                                              \
    _Pragma("unroll") for (int u = 0; u < NYU; ++u) {                                                         \
      const int q_ = threadIdx.x + NT * u;                                                                    \
      WG_PUT(yimg[b], YIMG, q_ >> 5, 4 * (q_ & 31), PY[u])                                                    \
      csum.x = fmaf(on_, PY[u].x, csum.x);                                                                    \
      csum.y = fmaf(on_, PY[u].y, csum.y);                                                                    \
      csum.z = fmaf(on_, PY[u].z, csum.z);                                                                    \
      csum.w = fmaf(on_, PY[u].w, csum.w);                                                                    \
    }                                                                                                         \
    _Pragma("unroll") for (int u = 0; u < NXU; ++u) WG_PUT(ximg[b], XIMG, lrow + NW * u, 4 * lane, PX[u])     \
  }
  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);
  f32x16 acc[NA][4];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
  const int wn = (w >> 1) * 32 * NA, wi = (w & 1) * 128;  // this wave's 32·NA n-rows and 128 i-columns
#define WG_STEP(c, RY, RX, SY, SX)                                                                            \
  {                                                                                                           \
    WG_LOAD((c) + AH, RY, RX)                                                                                 \
    const char* yi_ = yimg[(c) & 1];                                                                          \
    const char* xi_ = ximg[(c) & 1];                                                                          \
    _Pragma("unroll") for (int kst = 0; kst < 2; ++kst) {                                                     \
      bf16x8 fa_[NA], fb_[4];                                                                                 \
      _Pragma("unroll") for (int a = 0; a < NA; ++a) fa_[a] = tr32(yi_, 16 * kst, wn + 32 * a, lane);         \
      _Pragma("unroll") for (int b = 0; b < 4; ++b) fb_[b] = tr32(xi_, 16 * kst, wi + 32 * b, lane);          \
      _Pragma("unroll") for (int a = 0; a < NA; ++a) _Pragma("unroll") for (int b = 0; b < 4; ++b) acc[a][b] = \
          __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa_[a], fb_[b], acc[a][b], 0, 0, 0);                        \
      if constexpr (X3) {                                                                                     \
        bf16x8 fal_[NA], fbl_[4];                                                                             \
        _Pragma("unroll") for (int a = 0; a < NA; ++a) fal_[a] = tr32(yi_ + YIMG, 16 * kst, wn + 32 * a, lane); \
        _Pragma("unroll") for (int b = 0; b < 4; ++b) fbl_[b] = tr32(xi_ + XIMG, 16 * kst, wi + 32 * b, lane); \
        _Pragma("unroll") for (int a = 0; a < NA; ++a) _Pragma("unroll") for (int b = 0; b < 4; ++b) {       \
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fal_[a], fb_[b], acc[a][b], 0, 0, 0);           \
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa_[a], fbl_[b], acc[a][b], 0, 0, 0);           \
        }                                                                                                     \
      }                                                                                                       \
    }                                                                                                         \
    WG_STAGE(SY, SX, ((c) + 1) & 1, (c) + 1)                                                                  \
    __syncthreads();                                                                                          \
  }
  if (nchunk > 0) {
    if constexpr (AH == 2) {
    float4 Ya[NYU], Xa[NXU], Yb[NYU], Xb[NXU];
    WG_LOAD(0, Ya, Xa)
    WG_LOAD(1, Yb, Xb)
    WG_STAGE(Ya, Xa, 0, 0)
    __syncthreads();
    for (int c = 0; c < nchunk; c += 2) {
      WG_STEP(c, Ya, Xa, Yb, Xb)
      if (c + 1 >= nchunk) break;
      WG_STEP(c + 1, Yb, Xb, Ya, Xa)
    }
    } else {
    // three register sets: chunk c+3 is loaded at step c, so the staging of chunk c+1 (end of step c) waits on a
    // load issued two steps earlier
    float4 Ya[NYU], Xa[NXU], Yb[NYU], Xb[NXU], Yc[NYU], Xc[NXU];
    WG_LOAD(0, Ya, Xa)
    WG_LOAD(1, Yb, Xb)
    WG_LOAD(2, Yc, Xc)
    WG_STAGE(Ya, Xa, 0, 0)
    __syncthreads();
    for (int c = 0; c < nchunk; c += 3) {
      WG_STEP(c, Ya, Xa, Yb, Xb)
      if (c + 1 >= nchunk) break;
      WG_STEP(c + 1, Yb, Xb, Yc, Xc)
      if (c + 2 >= nchunk) break;
      WG_STEP(c + 2, Yc, Xc, Ya, Xa)
    }
    }
  }
#undef WG_STEP
#undef WG_STAGE
#undef WG_PUT
#undef WG_LOAD
  // column sums: the NT/32 threads of a column group (tid >> 5) combined in a fixed order
  if (part_b) {
    red_b[threadIdx.x >> 5][threadIdx.x & 31] = csum;
    __syncthreads();
    if (threadIdx.x < 32) {
      float4 t = red_b[0][threadIdx.x];
#pragma unroll
      for (int j = 1; j < NT / 32; ++j) t = make_float4(t.x + red_b[j][threadIdx.x].x, t.y + red_b[j][threadIdx.x].y,
                                                  t.z + red_b[j][threadIdx.x].z, t.w + red_b[j][threadIdx.x].w);
      const int n0 = n_base + 4 * threadIdx.x;
      if (n0 < N) *(float4*)(part_b + (long)split * N + n0) = t;
    }
  }
  // D[n][i]: lane holds (row n = wn + 32a + creg(r), col i = wi + 32b + (lane&31))
  float* out = part + (long)split * N * 256;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n_base + wn + 32 * a + creg(r, lane);
        if (n < N) out[(long)n * 256 + wi + 32 * b + (lane & 31)] = acc[a][b][r];
      }
}

// out[i] = beta·out[i] + Σ_s part[s][i]  (fixed order, float4): 8 lanes per float4 output, lane j
// summing the splits s ≡ j (mod 8), then a fixed xor tree over the 8 lanes.  blk: this range's block.
__device__ __forceinline__ void sum_parts_body(const float* __restrict__ part, int nparts, long n, float beta,
                                               float* __restrict__ out, long blk) {
  const long g = blk * blockDim.x + threadIdx.x;
  const long i = (g >> 3) * 4;
  const int j = (int)(g & 7);
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n)
    for (int s = j; s < nparts; s += 8) {
      const float4 v = *(const float4*)(part + (long)s * n + i);
      t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
    }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    t.x += __shfl_xor(t.x, m, 64);
    t.y += __shfl_xor(t.y, m, 64);
    t.z += __shfl_xor(t.z, m, 64);
    t.w += __shfl_xor(t.w, m, 64);
  }
  if (i >= n || j) return;
  float4 o = beta == 0.f ? make_float4(0.f, 0.f, 0.f, 0.f) : *(const float4*)(out + i);
  *(float4*)(out + i) = make_float4(beta * o.x + t.x, beta * o.y + t.y, beta * o.z + t.z, beta * o.w + t.w);
}

// the weight and bias partial sums of one wgemm in one launch: blocks [0, blocks_a) sum range a, the rest
// range b (each block entirely in one range)
__global__ void sum_parts_kernel2(const float* __restrict__ part_a, long n_a, float* __restrict__ out_a,
                                  const float* __restrict__ part_b, long n_b, float* __restrict__ out_b,
                                  int nparts, float beta, long blocks_a) {
  if ((long)blockIdx.x < blocks_a)
    sum_parts_body(part_a, nparts, n_a, beta, out_a, blockIdx.x);
  else
    sum_parts_body(part_b, nparts, n_b, beta, out_b, blockIdx.x - blocks_a);
}

// fp32 [R][Cc] (row stride lds) → bf16, optionally transposed (out [Cc][R])
__global__ void to_bf16_kernel(const float* __restrict__ x, int R, int Cc, long ldx, int trans, bf16* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)R * Cc) return;
  const int r = (int)(i / Cc), c = (int)(i % Cc);
  const bf16 v = (bf16)x[(long)r * ldx + c];
  if (trans)
    y[(long)c * R + r] = v;
  else
    y[i] = v;
}

// ‖W[c]‖² for the guarded ReLU (W fp32 [N][K], K = 256): one wave per row, fixed-order butterfly
__global__ void row_norm2_kernel(const float* __restrict__ W, int N, int K, float* __restrict__ out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= N) return;
  float s = 0.f;
  for (int k = 4 * lane; k < K; k += 256) {
    const float4 w = *(const float4*)(W + (long)c * K + k);
    s = fmaf(w.w, w.w, fmaf(w.z, w.z, fmaf(w.y, w.y, fmaf(w.x, w.x, s))));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) out[c] = s;
}

// the exact recompute of the flagged elements (rg3 GUARD): C[r][c] = drop(relu(alpha·Σ_k A[r][k]·W[c][k] + b[c])),
// each dot product one fp32 FMA chain in k order — the order of a k-sequential fp32 GEMM, so a pre-activation within
// fp32 rounding of zero gets that GEMM's sign (tools/linear1_emu.py: a float64-exact product misses the reference's C2
// step by 1.2e-4 on linear1's weight gradient through one such tie; this order matches it).  One wave per 64 flag bytes
// (a byte = a 4-column group of one row: flagged bytes are rare, so each wave sees one at most, usually); per flagged
// byte the wave stages the row of A and the 4 weight rows in LDS with coalesced loads and lanes 0..3 run the chains of
// the group's 4 columns from there.  The flags are cleared.
__global__ __launch_bounds__(256) void guard_fix_kernel(const float* __restrict__ A, long lda,
                                                        const float* __restrict__ W, int M, int N, Epi2 ep,
                                                        float* __restrict__ C, long ldc) {
  __shared__ float4 st[4][5][64];  // per wave: A row, 4 weight rows (K = 256)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nq = N >> 2;
  const long fi = (long)blockIdx.x * 256 + threadIdx.x;
  const bool in = fi < (long)M * nq;
  const unsigned f = in ? ep.gflag[fi] : 0u;
  if (f) ep.gflag[fi] = 0;
  for (unsigned long long m = __builtin_amdgcn_ballot_w64(f != 0); m; m &= m - 1) {  // wave-uniform
    const int src = __builtin_ctzll(m);
    const long fl = fi - lane + src;
    const unsigned fs = (unsigned)__builtin_amdgcn_readlane((int)f, src);
    const int r = (int)(fl / nq), c0 = (int)(fl % nq) * 4;
    st[wv][0][lane] = *(const float4*)(A + (long)r * lda + 4 * lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) st[wv][1 + e][lane] = *(const float4*)(W + (long)(c0 + e) * 256 + 4 * lane);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS stores have landed
    if (lane < 4 && ((fs >> lane) & 1u)) {
      float sum = 0.f;
#pragma unroll 16
      for (int k = 0; k < 64; ++k) {
        const float4 a = st[wv][0][k], w = st[wv][1 + lane][k];
        sum = fmaf(a.w, w.w, fmaf(a.z, w.z, fmaf(a.y, w.y, fmaf(a.x, w.x, sum))));
      }
      const int c = c0 + lane, dr = ep.rowmap ? ep.rowmap[r] : r;
      const float v = fmaf(ep.alpha, sum, ep.bias ? ep.bias[c] : 0.f);
      C[(long)r * ldc + c] = fmaxf(v, 0.f) * ep.drop.mul((uint64_t)(ep.row_base + dr) * N + c);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace

// 1 when c2dsr_rgemm takes (M, N, K): K ∈ {256, 512, 768} (the encoder projections at d = 256)
C2_API int c2dsr_rgemm_supported(int M, int N, int K) {
  return M > 0 && N > 0 && (K == 256 || K == 512 || K == 768) && (long)M * K * 4 < (1L << 31) && (long)M * N * 4 < (1L << 31);
}

// C[M,N] = alpha·A[M,K]·B[N,K]ᵀ + bias[N]  (beta must be 0; epilogue 1: relu then dropout(p), index
// (row_base+row)·N + col).  A fp32 (row stride lda, 16-byte aligned rows), B bf16 [N][ldb].
C2_API int c2dsr_rgemm_aux(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                           float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                           int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                           float aux_scale, void* stream);

C2_API int c2dsr_rgemm(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                       float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                       int64_t row_base, const int* rowmap, void* stream) {
  return c2dsr_rgemm_aux(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, bias, epilogue, k0, k1, p, row_base, rowmap, 0,
                         nullptr, nullptr, 0.f, stream);
}

// ... with an aux epilogue: aux_mode 1: C = alpha·A·Bᵀ + bias + aux (aux == C: accumulate in
// place); 2: C = aux > 0 ? (alpha·A·Bᵀ + bias)·aux_scale : 0 (aux [M][ldc]); 3: C = alpha·A·Bᵀ + bias
// + aux[auxmap[r]] (auxmap [M], entries < 0 add nothing; aux holds the mapped rows only).
static int rgemm_impl(int M, int N, int K, const void* A, bool ab16, int lda, const void* B, int ldb, float* C,
                      int ldc, float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1,
                      float p, int64_t row_base, const int* rowmap, int aux_mode, const float* aux,
                      const int* auxmap, float aux_scale, void* stream, bool x3 = false, bool frag = false) {
  if (!c2dsr_rgemm_supported(M, N, K) || lda % 4 || ldb % 8 || beta != 0.f) return (int)hipErrorInvalidValue;
  if (x3 && (ab16 || (K != 256 && K != 512) || (frag ? ldb != 0 || N % 4 || ldc % 4 : ldb < 2 * K)))
    return (int)hipErrorInvalidValue;
  if (ab16 && (epilogue || aux_mode == AUX_MASK || (K != 768 && aux_mode == AUX_ACC_MAP) ||
               (K == 512 && aux_mode != AUX_NONE)))
    return (int)hipErrorInvalidValue;
  if (aux_mode < 0 || aux_mode > 3 || (aux_mode && (!aux || epilogue))) return (int)hipErrorInvalidValue;
  if ((aux_mode == AUX_ACC_MAP) != (auxmap != nullptr) || (aux_mode == AUX_ACC_MAP && aux == C))
    return (int)hipErrorInvalidValue;
  Epi2 ep{alpha, beta, bias, epilogue == 1, c2::make_drop(k0, k1, epilogue == 1 ? p : 0.f), row_base, aux,
          aux_scale, rowmap, auxmap, nullptr, nullptr, 0.f};
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  hipStream_t s = (hipStream_t)stream;
  const int CT = K == 256 && !x3 ? 2 : 1;
  const int G = c2::ceil_div(N, 128 * CT);
  // persistent grid: exactly the workgroups that are resident at once (occupancy of the variant)
  static int per_cu[48] = {0};
  auto launch = [&](void (*kern)(int, int, int, const void*, long, const bf16*, long, float*, long, Epi2, int),
                    int slot) -> int {
    if (!per_cu[slot]) {
      int n = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kern, 256, 0);
      per_cu[slot] = n > 0 ? n : 1;
    }
    const int blocks = (ncu * per_cu[slot] / 8) * 8;
    if (blocks / 8 < G) return (int)hipErrorInvalidValue;
    kern<<<blocks, 256, 0, s>>>(M, N, K, A, lda, (const bf16*)B, ldb, C, ldc, ep, G);
    return 0;
  };
  int rc;
  const bool e = epilogue == 1;
  if (x3 && N % 4 == 0 && ldc % 4 == 0) {  // split-bf16 operands (fp32 mode): rg3 (16x16x32, transposed tiles)
    const int G3 = c2::ceil_div(N, K == 256 ? 256 : 128);
    auto launch3 = [&](void (*kern)(int, int, const float*, long, const bf16*, long, float*, long, Epi2, int),
                       int slot) -> int {
      if (!per_cu[slot]) {
        int n = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kern, 64 * RG3_NW, 0);
        per_cu[slot] = n > 0 ? n : 1;
      }
      const int blocks = (ncu * per_cu[slot] / 8) * 8;
      if (blocks / 8 < G3) return (int)hipErrorInvalidValue;
      kern<<<blocks, 64 * RG3_NW, 0, s>>>(M, N, (const float*)A, lda, (const bf16*)B, ldb, C, ldc, ep, G3);
      return 0;
    };
    const bool k1 = K == 256;
#define RG3(E, X) (k1 ? launch3(rg3_kernel<1, E, X, false, RG3_NW>, 31 + 2 * (X) + (E ? 8 : 0)) \
                      : launch3(rg3_kernel<2, E, X, false, RG3_NW>, 32 + 2 * (X) + (E ? 8 : 0)))
    if (e && aux_mode == AUX_NONE)
      rc = RG3(true, AUX_NONE);
    else if (aux_mode == AUX_ACC)
      rc = RG3(false, AUX_ACC);
    else if (aux_mode == AUX_ACC_MAP)
      rc = RG3(false, AUX_ACC_MAP);
    else if (aux_mode == AUX_MASK)
      rc = RG3(false, AUX_MASK);
    else
      rc = RG3(false, AUX_NONE);
#undef RG3
  } else if (x3) {  // split-bf16 operands, N or ldc not a multiple of 4: one 32-column tile per wave
    const bool k1 = K == 256;
    if (aux_mode == AUX_ACC)
      rc = k1 ? launch(rg_kernel<1, 1, false, AUX_ACC, false, true>, 21) : launch(rg_kernel<2, 1, false, AUX_ACC, false, true>, 22);
    else if (aux_mode == AUX_ACC_MAP)
      rc = k1 ? launch(rg_kernel<1, 1, false, AUX_ACC_MAP, false, true>, 23)
              : launch(rg_kernel<2, 1, false, AUX_ACC_MAP, false, true>, 24);
    else if (aux_mode == AUX_MASK)
      rc = k1 ? launch(rg_kernel<1, 1, false, AUX_MASK, false, true>, 25) : launch(rg_kernel<2, 1, false, AUX_MASK, false, true>, 26);
    else if (e)
      rc = k1 ? launch(rg_kernel<1, 1, true, AUX_NONE, false, true>, 27) : launch(rg_kernel<2, 1, true, AUX_NONE, false, true>, 28);
    else
      rc = k1 ? launch(rg_kernel<1, 1, false, AUX_NONE, false, true>, 29) : launch(rg_kernel<2, 1, false, AUX_NONE, false, true>, 30);
  } else if (ab16 && K == 256) {  // the row-subset attention's bf16 dq (+ the parked LN gradient)
    rc = aux_mode == AUX_ACC ? launch(rg_kernel<1, 2, false, AUX_ACC, true>, 18)
                             : launch(rg_kernel<1, 2, false, AUX_NONE, true>, 19);
  } else if (ab16 && K == 512) {  // ... and its bf16 dkv
    rc = launch(rg_kernel<2, 1, false, AUX_NONE, true>, 20);
  } else if (ab16) {  // K = 768: the in_proj backward over the attention's bf16 dqkv
    if (aux_mode == AUX_ACC)
      rc = launch(rg_kernel<3, 1, false, AUX_ACC, true>, 15);
    else if (aux_mode == AUX_ACC_MAP)
      rc = launch(rg_kernel<3, 1, false, AUX_ACC_MAP, true>, 16);
    else
      rc = launch(rg_kernel<3, 1, false, AUX_NONE, true>, 17);
  } else if (aux_mode == AUX_ACC) {
    if (K == 256)
      rc = launch(rg_kernel<1, 2, false, AUX_ACC>, 6);
    else if (K == 512)
      rc = launch(rg_kernel<2, 1, false, AUX_ACC>, 7);
    else
      rc = launch(rg_kernel<3, 1, false, AUX_ACC>, 8);
  } else if (aux_mode == AUX_ACC_MAP) {
    if (K == 256)
      rc = launch(rg_kernel<1, 2, false, AUX_ACC_MAP>, 12);
    else if (K == 512)
      rc = launch(rg_kernel<2, 1, false, AUX_ACC_MAP>, 13);
    else
      rc = launch(rg_kernel<3, 1, false, AUX_ACC_MAP>, 14);
  } else if (aux_mode == AUX_MASK) {
    if (K == 256)
      rc = launch(rg_kernel<1, 2, false, AUX_MASK>, 9);
    else if (K == 512)
      rc = launch(rg_kernel<2, 1, false, AUX_MASK>, 10);
    else
      rc = launch(rg_kernel<3, 1, false, AUX_MASK>, 11);
  } else if (K == 256)
    rc = e ? launch(rg_kernel<1, 2, true>, 0) : launch(rg_kernel<1, 2, false>, 1);
  else if (K == 512)
    rc = e ? launch(rg_kernel<2, 1, true>, 2) : launch(rg_kernel<2, 1, false>, 3);
  else
    rc = e ? launch(rg_kernel<3, 1, true>, 4) : launch(rg_kernel<3, 1, false>, 5);
  if (rc) return rc;
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_rgemm_aux(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                           float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                           int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                           float aux_scale, void* stream) {
  return rgemm_impl(M, N, K, A, false, lda, B, ldb, C, ldc, alpha, beta, bias, epilogue, k0, k1, p, row_base, rowmap,
                    aux_mode, aux, auxmap, aux_scale, stream);
}

// fp32 mode: split-bf16 products (B = the split image [N][2K] = hi ‖ lo, ldb >= 2K; K = 256 or 512)
#ifdef RG3_STAMP
C2_API int c2dsr_rg3_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rg3_stamp_acc), sizeof(rg3_stamp_acc));
  if (e == hipSuccess && reset) {
    static const unsigned long long z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(rg3_stamp_acc), z, sizeof(z));
  }
  return (int)e;
}
#endif
// workspace of c2dsr_rgemm_x3_relu_guard: ‖W[c]‖² [N], then the element flags [M][N/4] (zero on entry; every call
// leaves them zero again, so a workspace zeroed once serves all later calls of the same or smaller M·N)
C2_API size_t c2dsr_rgemm_guard_workspace(int M, int N) {
  return (((size_t)N * 4 + 255) & ~(size_t)255) + (((size_t)M * (N / 4) + 15) & ~(size_t)15);
}

// linear1 of the fp32 mode (models/encoders.py:23-27 → TransformerEncoderLayer linear1 + relu + dropout):
// C = drop(relu(A·Wᵀ + bias)) on split-bf16 products (B = the split image of W, K = 256), every pre-activation within
// the split error bound of zero recomputed exactly from the fp32 A and W in k order (rg3 GUARD flags it,
// guard_fix_kernel recomputes and clears)
C2_API int c2dsr_rgemm_x3_relu_guard(int M, int N, int K, const float* A, int lda, const void* B, int ldb,
                                     const float* W, const float* wn2_in, float* C, int ldc, const float* bias,
                                     uint32_t k0, uint32_t k1, float p, int64_t row_base, const int* rowmap,
                                     void* workspace, size_t ws_bytes, void* stream) {
  // ldb == 0: B is the fragment-ordered split image (c2dsr_to_split_bf16_frag_multi)
  if (M <= 0 || K != 256 || N % 4 || ldc % 4 || lda % 4 || (ldb != 0 && ldb < 2 * K) || ldb % 8 || !W ||
      !c2dsr_rgemm_supported(M, N, K) || ws_bytes < c2dsr_rgemm_guard_workspace(M, N))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* wn2 = (float*)ws;
  unsigned char* flags = (unsigned char*)(ws + (((size_t)N * 4 + 255) & ~(size_t)255));
  if (!wn2_in) row_norm2_kernel<<<c2::ceil_div(N, 4), 256, 0, s>>>(W, N, K, wn2);
  Epi2 ep{1.f, 0.f, bias, 1, c2::make_drop(k0, k1, p), row_base, nullptr, 0.f, rowmap, nullptr,
          wn2_in ? wn2_in : wn2, flags, 0x1p-30f};  // tau = 2^-15
  static int ncu = 0, per_cu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)rg3_kernel<1, true, AUX_NONE, true, RG3_GUARD_NW>,
                                                       64 * RG3_GUARD_NW, 0);
    per_cu = n > 0 ? n : 1;
  }
  const int G3 = c2::ceil_div(N, 256);
  const int blocks = (ncu * per_cu / 8) * 8;
  if (blocks / 8 < G3) return (int)hipErrorInvalidValue;
  rg3_kernel<1, true, AUX_NONE, true, RG3_GUARD_NW><<<blocks, 64 * RG3_GUARD_NW, 0, s>>>(M, N, A, lda, (const bf16*)B,
                                                                                         ldb, C, ldc, ep, G3);
  guard_fix_kernel<<<c2::ceil_div((long)M * (N / 4), 256), 256, 0, s>>>(A, lda, W, M, N, ep, C, ldc);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_rgemm_x3_supported(int M, int N, int K) {
  return c2dsr_rgemm_supported(M, N, K) && (K == 256 || K == 512);
}
C2_API int c2dsr_rgemm_x3(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                          float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                          int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                          float aux_scale, void* stream) {
  if (ldb == 0) return (int)hipErrorInvalidValue;  // 0 selects the fragment-ordered image (c2dsr_rgemm_x3f)
  return rgemm_impl(M, N, K, A, false, lda, B, ldb, C, ldc, alpha, beta, bias, epilogue, k0, k1, p, row_base, rowmap,
                    aux_mode, aux, auxmap, aux_scale, stream, true);
}
C2_API int c2dsr_rgemm_x3f(int M, int N, int K, const float* A, int lda, const void* B, float* C, int ldc, float alpha,
                           float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                           int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                           float aux_scale, void* stream) {
  return rgemm_impl(M, N, K, A, false, lda, B, 0, C, ldc, alpha, beta, bias, epilogue, k0, k1, p, row_base, rowmap,
                    aux_mode, aux, auxmap, aux_scale, stream, true, true);
}

// the same with A bf16 (K = 768, no epilogue, aux modes 0 / 1 / 3)
C2_API int c2dsr_rgemm_aux_b16a(int M, int N, int K, const void* A, int lda, const void* B, int ldb, float* C, int ldc,
                                float alpha, float beta, const float* bias, int aux_mode, const float* aux,
                                const int* auxmap, void* stream) {
  return rgemm_impl(M, N, K, A, true, lda, B, ldb, C, ldc, alpha, beta, bias, 0, 0, 0, 0.f, 0, nullptr, aux_mode, aux,
                    auxmap, 0.f, stream);
}

// dW[N][256] (+)= Σ_t dY[t][N]ᵀ·X[t][256] (N % 128 == 0) and, when db is given, db[N] (+)= Σ_t dY[t][N]
// (the bias gradient, from the same dY chunks): split over t into `splits` partial slices
// part[splits][N][256] + [splits][N] (c2dsr_wgemm_workspace bytes), combined in a fixed order with
// beta (0 or 1).
static int wg_splits(int N) {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (ncu <= 0) ncu = 256;
  const int NTL = N / 128;
  return (ncu / 8 / NTL) * 8;  // per XCD: ncu/8 slots / NTL n-tiles
}
C2_API int c2dsr_wgemm_supported(int T, int N, int D) {
  return T > 0 && D == 256 && N % 128 == 0 && N <= 32 * 128 && (long)T * N * 4 < (1L << 31) && (long)T * D * 4 < (1L << 31);
}
C2_API size_t c2dsr_wgemm_workspace(int N) { return (size_t)wg_splits(N) * N * 257 * 4; }
static int wgemm_segs(const WSeg& sg, int N, int D, bool yb16, float beta, float* dW, float* db, void* part,
                      void* stream, bool x3 = false) {
  const int T = sg.vbeg[WG_MAXSEG];
  if (T == 0) return 0;
  if (!c2dsr_wgemm_supported(T, N, D)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int NTL = N / 128;
  const int splits = wg_splits(N);
  if (splits < 8) return (int)hipErrorInvalidValue;
  const int rows = c2::ceil_div(c2::ceil_div(T, splits), 32) * 32;
  const int blocks = splits * NTL;  // = 8 XCDs x (splits/8) x NTL
  const long n = (long)N * 256;
  float* part_b = db ? (float*)part + (long)splits * n : nullptr;
  if (x3 && yb16) return (int)hipErrorInvalidValue;
  if (x3)
    wg_kernel<false, true, WG_NW_X3, WG_AH_X3><<<blocks, 64 * WG_NW_X3, 0, s>>>(N, sg, (float*)part, part_b, NTL,
                                                                                rows);
  else if (yb16)
    wg_kernel<true><<<blocks, 256, 0, s>>>(N, sg, (float*)part, part_b, NTL, rows);
  else
    wg_kernel<false><<<blocks, 256, 0, s>>>(N, sg, (float*)part, part_b, NTL, rows);
  const long blocks_a = c2::ceil_div(n / 4 * 8, 256), blocks_b = db ? c2::ceil_div((long)N / 4 * 8, 256) : 0;
  sum_parts_kernel2<<<blocks_a + blocks_b, 256, 0, s>>>((const float*)part, n, dW, part_b, N, db, splits, beta,
                                                        blocks_a);
  C2_CHECK_LAUNCH();
  return 0;
}

static int wgemm_impl(int T, int N, int D, const void* dY, bool yb16, int ldy, const float* X, int ldx, float beta,
                      float* dW, float* db, void* part, void* stream, bool x3 = false) {
  if (!c2dsr_wgemm_supported(T, N, D) || ldy % 4 || ldx % 4) return (int)hipErrorInvalidValue;
  WSeg sg{};
  sg.nseg = 1;
  sg.dY[0] = dY;
  sg.X[0] = X;
  sg.ldy[0] = ldy;
  sg.ldx[0] = ldx;
  sg.T[0] = T;
  sg.vbeg[0] = 0;
  for (int k = 1; k <= WG_MAXSEG; ++k) sg.vbeg[k] = c2::ceil_div(T, 32) * 32;
  return wgemm_segs(sg, N, D, yb16, beta, dW, db, part, stream, x3);
}

// dW[N, D] = beta·dW + Σ_k dY_kᵀ·X_k (and db = beta·db + Σ_k Σ_t dY_k[t]) over up to 4 row sets in ONE product
// (the weight of a module that several encoder passes used): seg = HOST array of nseg records of five int64
// (dY, ldy, X, ldx, T); dY fp32 (yb16 = 0) or bf16 (1); the same deterministic split partials as c2dsr_wgemm
static int wgemm_multi_impl(const int64_t* seg, int nseg, int N, int D, int yb16, float beta, float* dW, float* db,
                            void* part, void* stream, bool x3) {
  if (nseg < 1 || nseg > WG_MAXSEG) return (int)hipErrorInvalidValue;
  WSeg sg{};
  sg.nseg = nseg;
  sg.vbeg[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    const int64_t* r = seg + 5 * k;
    sg.dY[k] = (const void*)(intptr_t)r[0];
    sg.ldy[k] = (int)r[1];
    sg.X[k] = (const float*)(intptr_t)r[2];
    sg.ldx[k] = (int)r[3];
    sg.T[k] = (int)r[4];
    if (sg.T[k] < 0 || sg.ldy[k] % 4 || sg.ldx[k] % 4) return (int)hipErrorInvalidValue;
    sg.vbeg[k + 1] = sg.vbeg[k] + c2::ceil_div(sg.T[k], 32) * 32;
  }
  for (int k = nseg + 1; k <= WG_MAXSEG; ++k) sg.vbeg[k] = sg.vbeg[nseg];
  return wgemm_segs(sg, N, D, yb16 != 0, beta, dW, db, part, stream, x3);
}
C2_API int c2dsr_wgemm_multi(const int64_t* seg, int nseg, int N, int D, int yb16, float beta, float* dW, float* db,
                             void* part, void* stream) {
  return wgemm_multi_impl(seg, nseg, N, D, yb16, beta, dW, db, part, stream, false);
}
// fp32 mode: split-bf16 products (dY fp32)
C2_API int c2dsr_wgemm_x3_multi(const int64_t* seg, int nseg, int N, int D, float beta, float* dW, float* db,
                                void* part, void* stream) {
  return wgemm_multi_impl(seg, nseg, N, D, 0, beta, dW, db, part, stream, true);
}
C2_API int c2dsr_wgemm_x3(int T, int N, int D, const float* dY, int ldy, const float* X, int ldx, float beta, float* dW,
                          float* db, void* part, void* stream) {
  return wgemm_impl(T, N, D, dY, false, ldy, X, ldx, beta, dW, db, part, stream, true);
}

C2_API int c2dsr_wgemm(int T, int N, int D, const float* dY, int ldy, const float* X, int ldx, float beta, float* dW,
                       float* db, void* part, void* stream) {
  return wgemm_impl(T, N, D, dY, false, ldy, X, ldx, beta, dW, db, part, stream);
}
// dY bf16
C2_API int c2dsr_wgemm_b16y(int T, int N, int D, const void* dY, int ldy, const float* X, int ldx, float beta,
                            float* dW, float* db, void* part, void* stream) {
  return wgemm_impl(T, N, D, dY, true, ldy, X, ldx, beta, dW, db, part, stream);
}

// y = bf16(x) for x fp32 [R][Cc] (row stride ldx); trans: y is [Cc][R]
namespace {
constexpr int MULTI_MAX = 64;
struct MultiBf16 {
  const float* x[MULTI_MAX];
  bf16* y[MULTI_MAX];
  int R[MULTI_MAX], C[MULTI_MAX], ld[MULTI_MAX], tr[MULTI_MAX];
  int bstart[MULTI_MAX + 1];  // first block of each matrix (256 elements per block)
  int count;
};
// every matrix of the list in one launch: block b converts 256 elements of the matrix whose block range holds
// it (block-uniform lookup: scalar reads of the argument block)
// SPLIT: y = hi ‖ lo (row r of y: [hi(row) | lo(row)], width 2·C, or transposed [C][2R])
// FRAG (SPLIT only): the same values in rg3's fragment order (split_frag_index)
template <bool SPLIT = false, bool FRAG = false>
__global__ __launch_bounds__(256) void to_bf16_multi_kernel(MultiBf16 m) {
  const int b = blockIdx.x;
  int lo = 0, hi = m.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (m.bstart[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const long e = (long)(b - m.bstart[lo]) * 256 + threadIdx.x;
  const int Cc = m.C[lo], R = m.R[lo];
  if (e >= (long)R * Cc) return;
  const int r = (int)(e / Cc), c = (int)(e % Cc);
  const float x = m.x[lo][(long)r * m.ld[lo] + c];
  const bf16 v = (bf16)x;
  if constexpr (SPLIT) {
    const bf16 l = (bf16)(x - (float)v);
    const int RR = m.tr[lo] ? Cc : R, CC = m.tr[lo] ? R : Cc;  // output rows / columns
    const int orow = m.tr[lo] ? c : r, ocol = m.tr[lo] ? r : c;
    (void)RR;
    if constexpr (FRAG) {
      m.y[lo][split_frag_index(orow, ocol, 0, CC)] = v;
      m.y[lo][split_frag_index(orow, ocol, 1, CC)] = l;
    } else {
      m.y[lo][(long)orow * 2 * CC + ocol] = v;
      m.y[lo][(long)orow * 2 * CC + CC + ocol] = l;
    }
  } else if constexpr (FRAG) {  // rg_kernel's fragment order (b16_frag_index)
    const int CC = m.tr[lo] ? R : Cc;
    m.y[lo][b16_frag_index(m.tr[lo] ? c : r, m.tr[lo] ? r : c, CC)] = v;
  } else if (m.tr[lo]) {
    m.y[lo][(long)c * R + r] = v;
  } else {
    m.y[lo][e] = v;
  }
}
}  // namespace

// c2dsr_to_bf16 over a list of matrices in one launch: desc = HOST array of count (<= 64) records of six
// int64 (x, y, R, Cc, ldx, trans) with the meaning of c2dsr_to_bf16's arguments
static int to_bf16_multi_impl(const int64_t* desc, int count, void* stream, bool split, bool frag = false) {
  if (count < 0 || count > MULTI_MAX) return (int)hipErrorInvalidValue;
  if (count == 0) return 0;
  MultiBf16 m;
  m.count = count;
  m.bstart[0] = 0;
  for (int k = 0; k < count; ++k) {
    const int64_t* d = desc + 6 * k;
    m.x[k] = (const float*)(intptr_t)d[0];
    m.y[k] = (bf16*)(intptr_t)d[1];
    m.R[k] = (int)d[2];
    m.C[k] = (int)d[3];
    m.ld[k] = (int)d[4];
    m.tr[k] = (int)d[5];
    if (m.R[k] < 0 || m.C[k] < 0 || (long)m.R[k] * m.C[k] > (1l << 30)) return (int)hipErrorInvalidValue;
    m.bstart[k + 1] = m.bstart[k] + (int)c2::ceil_div((long)m.R[k] * m.C[k], 256);
  }
  if (m.bstart[count] == 0) return 0;
  for (int k = count + 1; k <= MULTI_MAX; ++k) m.bstart[k] = m.bstart[count];
  if (frag && split) {
    for (int k = 0; k < count; ++k)  // rg3's fragment order: K (the image's reduction width) 256 or 512
      if ((m.tr[k] ? m.R[k] : m.C[k]) % 256 || (m.tr[k] ? m.R[k] : m.C[k]) > 512) return (int)hipErrorInvalidValue;
    to_bf16_multi_kernel<true, true><<<m.bstart[count], 256, 0, (hipStream_t)stream>>>(m);
  } else if (frag) {
    for (int k = 0; k < count; ++k)  // rg_kernel's fragment order: K 256, 512 or 768
      if ((m.tr[k] ? m.R[k] : m.C[k]) % 256 || (m.tr[k] ? m.R[k] : m.C[k]) > 768) return (int)hipErrorInvalidValue;
    to_bf16_multi_kernel<false, true><<<m.bstart[count], 256, 0, (hipStream_t)stream>>>(m);
  } else if (split)
    to_bf16_multi_kernel<true><<<m.bstart[count], 256, 0, (hipStream_t)stream>>>(m);
  else
    to_bf16_multi_kernel<false><<<m.bstart[count], 256, 0, (hipStream_t)stream>>>(m);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_to_bf16_multi(const int64_t* desc, int count, void* stream) {
  return to_bf16_multi_impl(desc, count, stream, false);
}
// the split-bf16 images (y = [R][2·Cc] hi ‖ lo, or [Cc][2·R] transposed) of a list of matrices in one launch
C2_API int c2dsr_to_split_bf16_multi(const int64_t* desc, int count, void* stream) {
  return to_bf16_multi_impl(desc, count, stream, true);
}
// bf16 images in rg_kernel's fragment order (c2dsr_rgemm* with ldb = 0): ⌈N'/32⌉·32 × K' bf16 per matrix
C2_API int c2dsr_to_bf16_frag_multi(const int64_t* desc, int count, void* stream) {
  return to_bf16_multi_impl(desc, count, stream, false, true);
}
// the same values in rg3's fragment order (c2dsr_rgemm_x3f's B): ⌈N'/16⌉·16 × 2K' bf16 per matrix, N' / K' = the
// output rows / columns (Cc / R when transposed); rows past N' are not written
C2_API int c2dsr_to_split_bf16_frag_multi(const int64_t* desc, int count, void* stream) {
  return to_bf16_multi_impl(desc, count, stream, true, true);
}

// ‖W[r]‖² of a list of fp32 matrices (the guarded linear1's threshold, ops.WEIGHTS 'norm2'), one launch: one wave per
// row, lane l sums elements l, l + 64, … in order, then a fixed butterfly — deterministic.  Rows per block: 4.
namespace {
struct MultiNorm {
  const float* x[MULTI_MAX];
  float* y[MULTI_MAX];
  int R[MULTI_MAX], C[MULTI_MAX], ld[MULTI_MAX];
  int bstart[MULTI_MAX + 1];  // first block of each matrix
  int count;
};
__global__ __launch_bounds__(256) void row_sqnorm_multi_kernel(MultiNorm m) {
  const int b = blockIdx.x;
  int lo = 0, hi = m.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (m.bstart[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int r = (b - m.bstart[lo]) * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= m.R[lo]) return;
  const float* xr = m.x[lo] + (long)r * m.ld[lo];
  float s = 0.f;
  for (int c = lane; c < m.C[lo]; c += 64) s = fmaf(xr[c], xr[c], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) m.y[lo][r] = s;
}
}  // namespace

// desc: HOST array of count (<= 64) records of six int64 (x, y, R, Cc, ldx, 0): y[r] = Σ_c x[r·ldx + c]² (fp32 [R])
C2_API int c2dsr_row_sqnorm_multi(const int64_t* desc, int count, void* stream) {
  if (count < 0 || count > MULTI_MAX) return (int)hipErrorInvalidValue;
  if (count == 0) return 0;
  MultiNorm m;
  m.count = count;
  m.bstart[0] = 0;
  for (int k = 0; k < count; ++k) {
    const int64_t* d = desc + 6 * k;
    m.x[k] = (const float*)(intptr_t)d[0];
    m.y[k] = (float*)(intptr_t)d[1];
    m.R[k] = (int)d[2];
    m.C[k] = (int)d[3];
    m.ld[k] = (int)d[4];
    if (m.R[k] < 0 || m.C[k] < 0 || d[5] != 0 || m.ld[k] < m.C[k]) return (int)hipErrorInvalidValue;
    m.bstart[k + 1] = m.bstart[k] + c2::ceil_div(m.R[k], 4);
  }
  if (m.bstart[count] == 0) return 0;
  for (int k = count + 1; k <= MULTI_MAX; ++k) m.bstart[k] = m.bstart[count];
  row_sqnorm_multi_kernel<<<m.bstart[count], 256, 0, (hipStream_t)stream>>>(m);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_to_bf16(const float* x, int R, int Cc, int ldx, int trans, void* y, void* stream) {
  const long n = (long)R * Cc;
  if (n == 0) return 0;
  to_bf16_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(x, R, Cc, ldx, trans, (bf16*)y);
  C2_CHECK_LAUNCH();
  return 0;
}
