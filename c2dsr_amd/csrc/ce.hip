// K5: fused classifier-head linear + cross-entropy (the one real dense contraction of
// the path), bf16 MFMA with fp32 accumulation, logits never materialised.
//
// Replaces trainer.py:131-154: logits = h·Wᵀ + b (classifier_a/b, C2DSR.py:36-44) over
// all n items, concatenated with the pad column, F.cross_entropy(ignore_index = n)
// forward and backward.  Rows are the stacked [share ; specific] heads that share W
// (M = 2·B·R), K = D = d_latent.
//
//   lse kernel  (S^T = W·Hᵀ): per row tile, online log-sum-exp over a column range
//   dH kernel   (S^T again):   P'ᵀ = (softmax - onehot)·w_r, dHᵀ += Wᵀ·P'ᵀ
//   dW kernel   (S = H·Wᵀ):    P'  likewise,                 dWᵀ += Hᵀ·P',  db += Σ_r P'
// The accumulator of the first product is fed straight back as the B operand of the
// second (gfx950 32x32 C/D layout = B layout up to a k permutation), and the other
// operand is read TRANSPOSED from the same LDS image with ds_read_b64_tr_b16: one
// XOR-swizzled image per tile serves both the row reads (ds_read_b128) and the
// transposed reads, conflict-free (cdna_hip_programming.md §5.5 T10, image (b)).
// Each lane keeps its rows' (or columns') operand fragments in registers for the
// whole sweep; the swept operand is double-buffered through LDS with register-staged
// prefetch.  Work is split over column (lse, dH) or row (dW) ranges for occupancy and
// the partials are combined in a fixed order (deterministic).
#include "img.h"

#include <utility>

// tuning knobs (measured with tools/ce_micro.py; the defaults are the shipped configuration)
#ifndef CE_FWDU_DS
#define CE_FWDU_DS 3
#endif
#ifndef CE_FWDU_DT
#define CE_FWDU_DT 3
#endif
#ifndef CE_DW_DS
#define CE_DW_DS 3
#endif
#ifndef CE_DW_DT
#define CE_DW_DT 3
#endif

namespace {

using namespace c2img;

// ---------------------------------------------------------------- forward: partial LSE
// grid (ceil(M/256), n_split); 8 waves x 32 rows, two waves per SIMD (one wave's exp/max
// epilogue runs in the other's MFMA shadow).  part_m/part_s [n_split][M]: log2-domain running
// max and sum of 2^(s·log2e) over the split's columns.  bias2 = bias·log2e, -inf past n.
// W tiles stream through three LDS images: tile t+2's pieces (four per wave, saddr LDS-DMA)
// are issued between the k-steps of tile t and land during tile t+1.  Wb holds ⌈n/64⌉·64
// rows (zero padding past n).
template <int D>
__global__ __launch_bounds__(512, 1) void ce_lse_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                        const float* __restrict__ bias2, int M, int n,
                                                        int cols_per_split, float* __restrict__ part_m,
                                                        float* __restrict__ part_s) {
  constexpr int KS = D / 16;
  constexpr int NW = 8;
  constexpr int NB = 3;
  constexpr int DS = 3;
  constexpr int IMG = TILE * D * 2;
  constexpr int NDMA = (TILE / 4) * (D / 128) / NW;  // pieces per wave per tile
  static_assert(NDMA >= 1 && (KS / NDMA) >= 1, "tile / wave split");
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float b2s[NB][NW][TILE];  // [buffer][wave]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * 256 + w * 32 + (lane & 31);
  const int c_beg = blockIdx.y * cols_per_split;
  const int c_end = min(n, c_beg + cols_per_split);
  const int ntiles = c_end > c_beg ? (c_end - c_beg + TILE - 1) / TILE : 0;
  float mrun = -INFINITY, srun = 0.f;
  if (ntiles > 0) {
    const int c_last = c_beg + (ntiles - 1) * TILE;
    const ImgOffsets o0 = img_offsets(lane);
    const int ib = (int)lds_addr(img[0]);
    const int bb = (int)lds_addr(b2s[0][w]) + 16 * (lane >> 5);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + NW * i;
      constexpr int GROUPS = TILE / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz_f(row);
      dvoff[i] = (unsigned)((row * D + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * (TILE * 256) + rg * 1024));
    }
    auto dma = [&](int tt) {  // tile tt (clamped to the last) → buffer tt % NB
      const int c0 = min(c_beg + tt * TILE, c_last);
      const int buf = tt % NB;
      const bf16* base = Wb + (long)c0 * D;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma4(bias2 + c0 + lane, b2s[buf][w]);
    };
    bf16x8 hf[KS];
    const int rc = min(M - 1, r);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hf[ks] = *(const bf16x8*)(Hb + (long)rc * D + ks * 16 + 8 * (lane >> 5));
    dma(0);
    dma(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) pin(hf[ks]);
    vm_drain();
    dma_wait();
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      const int bc = t % NB;
      const int cn = min(c_beg + (t + 2) * TILE, c_last);
      const bf16* nsrc = Wb + (long)cn * D;
      const unsigned nbuf = ((t + 2) % NB) * IMG;
      dma4(bias2 + cn + lane, b2s[(t + 2) % NB][w]);
      ImgOffsets oS;
      {
        const int add = ib + bc * IMG;
#pragma unroll
        for (int k = 0; k < 8; ++k) oS.roff[k] = o0.roff[k] + add;
      }
      f32x16 acc[2];
      bf16x8 fa[DS + 2][2];
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((fa[P][0] = row_frag_c<TILE, 0, P, 0>(oS), fa[P][1] = row_frag_c<TILE, 32, P, 0>(oS)), ...);
      }(std::make_integer_sequence<int, DS>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              if constexpr (ks + DS < KS) {
                fa[(ks + DS) % (DS + 2)][0] = row_frag_c<TILE, 0, ks + DS, 0>(oS);
                fa[(ks + DS) % (DS + 2)][1] = row_frag_c<TILE, 32, ks + DS, 0>(oS);
              }
              if constexpr (ks % (KS / NDMA) == 1 % (KS / NDMA) && ks / (KS / NDMA) < NDMA)
                dma16_s<ks / (KS / NDMA) == 0>(nsrc, dvoff[ks / (KS / NDMA)], ddst[ks / (KS / NDMA)] + nbuf);
              if constexpr (ks == 0) {
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], hf[0], f32x16{}, 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][1], hf[0], f32x16{}, 0, 0, 0);
              } else {
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][0], hf[ks], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][1], hf[ks], acc[1], 0, 0, 0);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
      f32x4 b4[2][4];  // bias·log2e of this lane's 32 columns (4 runs of 4)
      {
        const int bo = bb + bc * (NW * TILE * 4);
        [&]<int... J>(std::integer_sequence<int, J...>) {
          ((b4[J >> 2][J & 3] = lds_ld<f32x4, 128 * (J >> 2) + 32 * (J & 3)>(bo)), ...);
        }(std::make_integer_sequence<int, 8>{});
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = fmaf(acc[cb][i], LOG2E, b4[cb][i >> 2][i & 3]);
          acc[cb][i] = v;
          tmax = fmaxf(tmax, v);
        }
      const float mnew = fmaxf(mrun, tmax);
      float sm = (mrun == -INFINITY) ? 0.f : srun * ex2(mrun - mnew);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sm += ex2(acc[cb][i] - mnew);
      mrun = mnew;
      srun = sm;
      dma_wait_keep<NDMA + 1>();  // tile t+1 has landed; tile t+2 may still be in flight
      __syncthreads();
    }
  }
  const float m2 = __shfl_xor(mrun, 32, 64), s2 = __shfl_xor(srun, 32, 64);
  const float mm = fmaxf(mrun, m2);
  const float sm = (mrun == -INFINITY ? 0.f : srun * ex2(mrun - mm)) + (m2 == -INFINITY ? 0.f : s2 * ex2(m2 - mm));
  if (lane < 32 && r < M) {
    part_m[(long)blockIdx.y * M + r] = mm;
    part_s[(long)blockIdx.y * M + r] = sm;
  }
}

// per row: lse over the splits and the pad column, target logit (fp32), loss.  One wave per row.
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ part_m,
                                                      const float* __restrict__ part_s, int n_split, int M,
                                                      const float* __restrict__ padlogit,
                                                      const int64_t* __restrict__ tgt, int n,
                                                      const float* __restrict__ H, const float* __restrict__ W,
                                                      const float* __restrict__ bias, int D,
                                                      float* __restrict__ lse_out, float* __restrict__ lse2_out,
                                                      float* __restrict__ loss_row) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  const long t = tgt[r];
  float dot = 0.f;
  if (t >= 0 && t < n)
    for (int k = lane; k < D; k += 64) dot += H[r * D + k] * W[t * D + k];
  dot = c2::wave_sum(dot);
  // the splits' partials one per lane (loads in parallel), combined by wave reductions (fixed order)
  float pm = -INFINITY, ps = 0.f;
  for (int s = lane; s < n_split; s += 64) {
    const float m = part_m[(long)s * M + r], z = part_s[(long)s * M + r];
    const float mx = fmaxf(pm, m);
    ps = (pm == -INFINITY ? 0.f : ps * exp2f(pm - mx)) + (m == -INFINITY ? 0.f : z * exp2f(m - mx));
    pm = mx;
  }
  const float mm = c2::wave_max(pm);
  const float ss = c2::wave_sum(pm == -INFINITY ? 0.f : ps * exp2f(pm - mm));
  if (lane == 0) {
    const float lse_items = (mm + log2f(ss)) / LOG2E;
    const float pl = padlogit[r];
    const float hi = fmaxf(lse_items, pl);
    const float lse = hi + logf(expf(lse_items - hi) + expf(pl - hi));
    lse_out[r] = lse;
    lse2_out[r] = lse * LOG2E;
    loss_row[r] = (t != n) ? lse - (t < n ? dot + bias[t] : pl) : 0.f;
  }
}

// ---------------------------------------------------------------- backward: dH
// grid (ceil(M/128), n_split); 4 waves x 32 rows, one wave per SIMD (512 registers); sweeps the
// split's columns 64 at a time, software-pipelined over three W images:
//   step t:  [ S(t+1) = W_{t+1}·Hᵀ on the matrix cores  ∥  epilogue of S(t) on the VALU ]
//            dHᵀ += W_tᵀ·P'ᵀ(t);  tile t+3 lands while tile t+2 waits
// The epilogue is P'ᵀ[c][r] = 2^(s·log2e + b2[c] + cr[r]) with cr = log2(w_r) - lse2_r (the row
// weight folded into the exponent; w = 0 → -inf → 0; from c2dsr_ce_row_weights); the one-hot part of (softmax - onehot)
// is the exact per-row correction -w_r·W[t_r] applied by c2dsr_ce_dh_combine.  Every LDS fragment
// read is an asm ds_read at a precomputed per-lane offset, issued ahead of its MFMA with a counted
// wait; all MFMAs are asm (fixed order), the dHᵀ accumulators live in AGPRs; a sched_barrier
// between chunks keeps each epilogue slice in its MFMA gap.
// Wb holds ⌈n/64⌉·64 rows (zero padding past n); bias2 is -inf past n.
// dHp [n_split][M][D] fp32 partials.
__device__ __forceinline__ void mfma_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v0(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(acc) : "v"(a), "v"(b));
}

template <int D>
__global__ __launch_bounds__(256, 1) void ce_dh_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                       const float* __restrict__ bias2, int M, int n,
                                                       int cols_per_split, const float* __restrict__ crow,
                                                       float* __restrict__ dHp) {
  constexpr int KS = D / 16;
  constexpr int KB = D / 32;
  constexpr int NQ = KB * 4;
  constexpr int DS = 3;                          // S-phase row fragments ahead
  constexpr int DT = 3;                          // dH-phase transposed fragments ahead
  constexpr int EPK = 16 / KS;                   // epilogue elements per S k-step (per column block)
  constexpr int IMG = TILE * D * 2;              // bytes per image
  constexpr int NDMA = (TILE / 4) * (D / 128) / 4;  // DMA wave-instructions per wave per tile
  constexpr int NB = 4;                              // W images: S(t+1), dH(t), tile t+2 landed, t+3 landing
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float b2s[NB][4][TILE];  // [buffer][wave] (each wave its own copy)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int rc = min(r, M - 1);
  const int c_beg = blockIdx.y * cols_per_split;
  const int c_end = min(n, c_beg + cols_per_split);
  const int ntiles = c_end > c_beg ? (c_end - c_beg + TILE - 1) / TILE : 0;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  if (ntiles > 0) {
    const int c_last = c_beg + (ntiles - 1) * TILE;
    // ---- per-lane constants
    const ImgOffsets o0 = img_offsets(lane);
    const int ib = (int)lds_addr(img[0]);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + 4 * i;
      constexpr int GROUPS = TILE / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz_f(row);
      dvoff[i] = (unsigned)((row * D + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * (TILE * 256) + rg * 1024));
    }
    auto dma = [&](int tt) {  // tile tt (clamped to the last) → buffer tt % NB
      const int c0 = min(c_beg + tt * TILE, c_last);
      const int buf = tt % NB;
      const bf16* base = Wb + (long)c0 * D;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma4(bias2 + c0 + lane, b2s[buf][w]);
    };
    bf16x8 hf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hf[ks] = *(const bf16x8*)(Hb + (long)rc * D + ks * 16 + 8 * (lane >> 5));
    float cr = r < M ? crow[rc] : -INFINITY;
    dma(0);
    dma(1);
    dma(2);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) pin(hf[ks]);
    pin(cr);
    vm_drain();
    dma_wait();
    __syncthreads();

    // offsets into buffer b of the 16 per-lane fragment bases
    auto offs = [&](int b, int (&ro)[8], int (&to)[4][2]) {
      const int add = ib + b * IMG;
#pragma unroll
      for (int c = 0; c < 8; ++c) ro[c] = o0.roff[c] + add;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        to[v][0] = o0.troff[v][0] + add;
        to[v][1] = o0.troff[v][1] + add;
      }
    };
    // ---- S(0) (not overlapped)
    f32x16 sc[2];
    {
      int ro[8], to[4][2];
      offs(0, ro, to);
      ImgOffsets oS;
#pragma unroll
      for (int c = 0; c < 8; ++c) oS.roff[c] = ro[c];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 f0 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256);
        const bf16x8 f1 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256 + 32 * 256);
        if (ks == 0) {
          sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, hf[0], f32x16{}, 0, 0, 0);
          sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, hf[0], f32x16{}, 0, 0, 0);
        } else {
          sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, hf[ks], sc[0], 0, 0, 0);
          sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, hf[ks], sc[1], 0, 0, 0);
        }
      }
    }
    for (int t = 0; t < ntiles; ++t) {
      const int bh = t % NB, bs = (t + 1) % NB;
      // tile t+3 → the buffer tile t-1 used (every wave passed the barrier after its dH); its pieces
      // are issued in the dH phase (MFMA-bound, issue slots to spare), one per four dH steps, and
      // land during the next step
      const int cn = min(c_beg + (t + 3) * TILE, c_last);
      const bf16* nsrc = Wb + (long)cn * D;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      dma4(bias2 + cn + lane, b2s[(t + 3) % NB][w]);
      ImgOffsets oS, oH;
      {
        int ro[8], to[4][2];
        offs(bs, ro, to);
#pragma unroll
        for (int c = 0; c < 8; ++c) oS.roff[c] = ro[c];
        offs(bh, ro, to);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          oH.troff[v][0] = to[v][0];
          oH.troff[v][1] = to[v][1];
        }
      }
      f32x4 b4[2][4];
      {
        const int bo = (int)lds_addr(b2s[bh][w]) + 16 * (lane >> 5);
        [&]<int... J>(std::integer_sequence<int, J...>) {
          ((b4[J >> 2][J & 3] = lds_ld<f32x4, 128 * (J >> 2) + 32 * (J & 3)>(bo)), ...);
        }(std::make_integer_sequence<int, 8>{});
      }
      // ---- S(t+1) ∥ epilogue(t): k-step ks runs 2 MFMAs, issues the reads DS steps ahead, and
      // computes EPK elements of each column block of S(t)
      f32x16 sn[2];
      bf16x8 fa[DS + 2][2];  // ring one longer than the lookahead: a slot is rewritten two MFMAs after its read
      bf16x8 x[2][2];
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((fa[P][0] = row_frag_c<TILE, 0, P, 0>(oS), fa[P][1] = row_frag_c<TILE, 32, P, 0>(oS)), ...);
      }(std::make_integer_sequence<int, DS>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              if constexpr (ks + DS < KS) {
                fa[(ks + DS) % (DS + 2)][0] = row_frag_c<TILE, 0, ks + DS, 0>(oS);
                fa[(ks + DS) % (DS + 2)][1] = row_frag_c<TILE, 32, ks + DS, 0>(oS);
              }
              if constexpr (ks == 0) {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], hf[0], f32x16{}, 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][1], hf[0], f32x16{}, 0, 0, 0);
              } else {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][0], hf[ks], sn[0], 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][1], hf[ks], sn[1], 0, 0, 0);
              }
              // epilogue slice: elements [ks·EPK, ks·EPK + EPK) of both column blocks
#pragma unroll
              for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int e = 0; e < EPK; ++e) {
                  const int i = ks * EPK + e;
                  sc[cb][i] = ex2(fmaf(sc[cb][i], LOG2E, ((const float*)&b4[cb][i >> 2])[i & 3]) + cr);
                }
              if constexpr ((ks * EPK + EPK) % 8 == 0) {
                constexpr int st = (ks * EPK) / 8;
                x[0][st] = acc_frag(sc[0], st);
                x[1][st] = acc_frag(sc[1], st);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
      // ---- dHᵀ[k][r] += Σ_c W[c][k] P'ᵀ[c][r], q = (kb, cb, st)
      bf16x8 tf[DT + 2];
      // U step q: output k-block U_KB(q), column quarter U_J(q) (16 columns: block U_J >> 1, half U_J & 1)
#define U_KB(q) ((q) >> 2)
#define U_J(q) ((q) & 3)
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((tf[P] = tr_frag_c<TILE, U_J(P) * 16, U_KB(P) * 32, 0>(oH)), ...);
      }(std::make_integer_sequence<int, DT>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        (
            [&] {
              constexpr int q = Q;
              if constexpr (q + DT < NQ) {
                constexpr int q1 = q + DT;
                tf[q1 % (DT + 2)] = tr_frag_c<TILE, U_J(q1) * 16, U_KB(q1) * 32, 0>(oH);
              }
              dacc[U_KB(q)] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[q % (DT + 2)], x[U_J(q) >> 1][U_J(q) & 1],
                                                                     dacc[U_KB(q)], 0, 0, 0);
              if constexpr (q % 4 == 1 && q / 4 < NDMA) dma16_s<q == 1>(nsrc, dvoff[q / 4], ddst[q / 4] + nbuf);
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NQ>{});
      // S(t+1) becomes the next step's S(t): its MFMAs have long retired (the dH chain ran since)
      sc[0] = sn[0];
      sc[1] = sn[1];
      dma_wait_keep<NDMA + 1>();  // tile t+2 has landed; tile t+3 may still be in flight
      __syncthreads();
    }
  }
  if (r < M) {
    float* out = dHp + ((long)blockIdx.y * M + r) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
  }
}

// ---------------------------------------------------------------- forward with dH: online LSE + U
// The forward of the training step already has the only thing the input gradient needs besides lse:
//   dH_r = rw_r · (Σ_c softmax_rc·W_c − W_{t_r}),   softmax_rc = 2^(s_rc·log2e + b2_c − lse2_r)
// so it is accumulated here, flash-attention style (W is both the "keys" and the "values"), and the
// backward has no dH sweep at all: 4·M·n·D MFMA flops for lse + dH instead of 2 + 4 in two kernels.
// Same block shape and software pipeline as ce_dh_kernel (grid (ceil(M/128), n_split), 4 waves × 32
// rows, one wave per SIMD, four W images):
//   step t:  [ S(t+1) = W_{t+1}·Hᵀ ∥ epilogue of S(t): p = 2^(v − m), z += p, pack ]
//            [ Uᵀ += W_tᵀ·Pᵀ(t)   ∥ DMA of tile t+3 ∥ v = S(t+1)·log2e + b2 and its row max ]
// m is the row's running max (log2 domain), raised LAZILY: only when a tile's max exceeds it by more
// than TAU does the wave rescale its accumulators (p ≤ 2^TAU otherwise; m never exceeds the true max,
// so no term underflows against a stale m).  Each lane holds one row r (the Sᵀ / Uᵀ column), its two
// half-waves different columns c / different k: the row max is combined across lane^32.
// Outputs per split s: part_m[s][r] = m, part_s[s][r] = Σ_c 2^(v_rc − m), Up[s][r][:] = Σ_c 2^(v_rc − m)·W_c
// (combined by ce_rows_kernel and ce_dh_from_u_kernel).
template <int D>
__global__ __launch_bounds__(256, 1) void ce_fwdu_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                         const float* __restrict__ bias2, int M, int n,
                                                         int cols_per_split, float* __restrict__ part_m,
                                                         float* __restrict__ part_s, float* __restrict__ Up) {
  constexpr int KS = D / 16;
  constexpr int KB = D / 32;
  constexpr int NQ = KB * 4;
  constexpr int DS = CE_FWDU_DS;  // LDS fragment prefetch depth, S phase
  constexpr int DT = CE_FWDU_DT;  // LDS fragment prefetch depth, U phase
  constexpr int EPK = 16 / KS;
  constexpr int MPK = 32 / NQ;                       // max-prep elements per U step
  constexpr int IMG = TILE * D * 2;
  constexpr int NDMA = (TILE / 4) * (D / 128) / 4;
  constexpr int NB = 4;
  constexpr float TAU = 8.f;  // lazy-max threshold (p ≤ 2^TAU)
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float b2s[NB][4][TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int rc = min(r, M - 1);
  const int c_beg = blockIdx.y * cols_per_split;
  const int c_end = min(n, c_beg + cols_per_split);
  const int ntiles = c_end > c_beg ? (c_end - c_beg + TILE - 1) / TILE : 0;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  float mrow = -INFINITY, zrow = 0.f;
  if (ntiles > 0) {
    const int c_last = c_beg + (ntiles - 1) * TILE;
    const ImgOffsets o0 = img_offsets(lane);
    const int ib = (int)lds_addr(img[0]);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + 4 * i;
      constexpr int GROUPS = TILE / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz_f(row);
      dvoff[i] = (unsigned)((row * D + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * (TILE * 256) + rg * 1024));
    }
    auto dma = [&](int tt) {
      const int c0 = min(c_beg + tt * TILE, c_last);
      const int buf = tt % NB;
      const bf16* base = Wb + (long)c0 * D;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma4(bias2 + c0 + lane, b2s[buf][w]);
    };
    bf16x8 hf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hf[ks] = *(const bf16x8*)(Hb + (long)rc * D + ks * 16 + 8 * (lane >> 5));
    dma(0);
    dma(1);
    dma(2);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) pin(hf[ks]);
    vm_drain();
    dma_wait();
    __syncthreads();
    auto offs = [&](int b, int (&ro)[8], int (&to)[4][2]) {
      const int add = ib + b * IMG;
#pragma unroll
      for (int c = 0; c < 8; ++c) ro[c] = o0.roff[c] + add;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        to[v][0] = o0.troff[v][0] + add;
        to[v][1] = o0.troff[v][1] + add;
      }
    };
    // bias·log2e of this lane's 32 columns of tile buffer b (4 runs of 4 per column block)
    auto bias4 = [&](int b, f32x4 (&b4)[2][4]) {
      const int bo = (int)lds_addr(b2s[b][w]) + 16 * (lane >> 5);
      [&]<int... J>(std::integer_sequence<int, J...>) {
        ((b4[J >> 2][J & 3] = lds_ld<f32x4, 128 * (J >> 2) + 32 * (J & 3)>(bo)), ...);
      }(std::make_integer_sequence<int, 8>{});
    };
    // ---- S(0) and its max (not overlapped)
    f32x16 sc[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 f0 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256);
      const bf16x8 f1 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256 + 32 * 256);
      if (ks == 0) {
        sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, hf[0], f32x16{}, 0, 0, 0);
        sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, hf[0], f32x16{}, 0, 0, 0);
      } else {
        sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, hf[ks], sc[0], 0, 0, 0);
        sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, hf[ks], sc[1], 0, 0, 0);
      }
    }
    float mnext;
    {
      f32x4 b4[2][4];
      bias4(0, b4);
      float tm = -INFINITY;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sc[cb][i] = fmaf(sc[cb][i], LOG2E, ((const float*)&b4[cb][i >> 2])[i & 3]);
          tm = fmaxf(tm, sc[cb][i]);
        }
      mnext = fmaxf(tm, __shfl_xor(tm, 32, 64));
    }
    for (int t = 0; t < ntiles; ++t) {
      const int bh = t % NB, bs = (t + 1) % NB;
      const int cn = min(c_beg + (t + 3) * TILE, c_last);
      const bf16* nsrc = Wb + (long)cn * D;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      dma4(bias2 + cn + lane, b2s[(t + 3) % NB][w]);
      // lazy rescale: the row's max moved up by more than TAU (always on the first tile)
      {
        const bool need = mnext > mrow + TAU;
        if (__builtin_amdgcn_ballot_w64(need)) {
          const float f = need ? ex2(mrow - mnext) : 1.f;  // mrow = -inf → 0
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) dacc[kb][i] *= f;
          zrow *= f;
          mrow = need ? mnext : mrow;
        }
      }
      const float msub = mrow == -INFINITY ? 0.f : mrow;  // all of S(t) is -inf then: p = 0
      ImgOffsets oS, oH;
      {
        int ro[8], to[4][2];
        offs(bs, ro, to);
#pragma unroll
        for (int c = 0; c < 8; ++c) oS.roff[c] = ro[c];
        offs(bh, ro, to);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          oH.troff[v][0] = to[v][0];
          oH.troff[v][1] = to[v][1];
        }
      }
      // ---- S(t+1) ∥ epilogue(t)
      f32x16 sn[2];
      bf16x8 x[2][2];
      bf16x8 fa[DS + 2][2];
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((fa[P][0] = row_frag_c<TILE, 0, P, 0>(oS), fa[P][1] = row_frag_c<TILE, 32, P, 0>(oS)), ...);
      }(std::make_integer_sequence<int, DS>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              if constexpr (ks + DS < KS) {
                fa[(ks + DS) % (DS + 2)][0] = row_frag_c<TILE, 0, ks + DS, 0>(oS);
                fa[(ks + DS) % (DS + 2)][1] = row_frag_c<TILE, 32, ks + DS, 0>(oS);
              }
              if constexpr (ks == 0) {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], hf[0], f32x16{}, 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][1], hf[0], f32x16{}, 0, 0, 0);
              } else {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][0], hf[ks], sn[0], 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][1], hf[ks], sn[1], 0, 0, 0);
              }
#pragma unroll
              for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int e = 0; e < EPK; ++e) {
                  const int i = ks * EPK + e;
                  const float pv = ex2(sc[cb][i] - msub);
                  sc[cb][i] = pv;
                  zrow += pv;
                }
              if constexpr ((ks * EPK + EPK) % 8 == 0) {
                constexpr int st = (ks * EPK) / 8;
                x[0][st] = acc_frag(sc[0], st);
                x[1][st] = acc_frag(sc[1], st);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
      // ---- Uᵀ[k][r] += Σ_c W[c][k] Pᵀ[c][r]  ∥  v = S(t+1)·log2e + b2 and its max
      f32x4 b4n[2][4];
      bias4(bs, b4n);
      float tm = -INFINITY;
      bf16x8 tf[DT + 2];
      // U step q: output k-block U_KB(q), column quarter U_J(q) (16 columns: block U_J >> 1, half U_J & 1)
#define U_KB(q) ((q) >> 2)
#define U_J(q) ((q) & 3)
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((tf[P] = tr_frag_c<TILE, U_J(P) * 16, U_KB(P) * 32, 0>(oH)), ...);
      }(std::make_integer_sequence<int, DT>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        (
            [&] {
              constexpr int q = Q;
              if constexpr (q + DT < NQ) {
                constexpr int q1 = q + DT;
                tf[q1 % (DT + 2)] = tr_frag_c<TILE, U_J(q1) * 16, U_KB(q1) * 32, 0>(oH);
              }
              dacc[U_KB(q)] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[q % (DT + 2)], x[U_J(q) >> 1][U_J(q) & 1],
                                                                     dacc[U_KB(q)], 0, 0, 0);
              if constexpr (q % 4 == 1 && q / 4 < NDMA) dma16_s<q == 1>(nsrc, dvoff[q / 4], ddst[q / 4] + nbuf);
#pragma unroll
              for (int e = 0; e < MPK; ++e) {
                const int el = q * MPK + e;
                const int cb = el >> 4, i = el & 15;
                const float v = fmaf(sn[cb][i], LOG2E, ((const float*)&b4n[cb][i >> 2])[i & 3]);
                sn[cb][i] = v;
                tm = fmaxf(tm, v);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NQ>{});
#undef U_KB
#undef U_J
      mnext = fmaxf(tm, __shfl_xor(tm, 32, 64));
      sc[0] = sn[0];
      sc[1] = sn[1];
      dma_wait_keep<NDMA + 1>();
      __syncthreads();
    }
  }
  const float ztot = zrow + __shfl_xor(zrow, 32, 64);
  if (r < M) {
    if (lane < 32) {
      part_m[(long)blockIdx.y * M + r] = mrow;
      part_s[(long)blockIdx.y * M + r] = ztot;
    }
    float* out = Up + ((long)blockIdx.y * M + r) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
  }
}

// dH[r] = rw_r · (Σ_s 2^(pm[s][r] − lse2_r)·Up[s][r] − W[t_r])   (t_r outside [0, n): no one-hot term;
// fixed split order)
__global__ void ce_dh_from_u_kernel(const float* __restrict__ Up, const float* __restrict__ pm, int ns, int M, int D,
                                    const float* __restrict__ lse2, const int* __restrict__ t32,
                                    const float* __restrict__ rw, const float* __restrict__ W, int n,
                                    float* __restrict__ dH) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= (long)M * D) return;
  const int r = (int)(i / D), k = (int)(i % D);
  const float l2 = lse2[r];
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  // every split's running max, then every split's slab loaded before the first add (one round trip each instead
  // of ns dependent pairs); added in split order as before.  ns <= DHU_MAX (losshead.split_count caps it at 16).
  constexpr int DHU_MAX = 16;
  float mm[DHU_MAX];
#pragma unroll
  for (int s = 0; s < DHU_MAX; ++s) mm[s] = s < ns ? pm[(long)s * M + r] : -INFINITY;
  float4 u[DHU_MAX];
#pragma unroll
  for (int s = 0; s < DHU_MAX; ++s)
    u[s] = mm[s] != -INFINITY ? *(const float4*)(Up + ((long)s * M) * D + i) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int s = 0; s < DHU_MAX; ++s)
    if (mm[s] != -INFINITY) t = c2::fma4(exp2f(mm[s] - l2), u[s], t);
  const float w = rw[r];
  const int tg = t32[r];
  if (tg >= 0 && tg < n) t = c2::fma4(-1.f, *(const float4*)(W + (long)tg * D + k), t);
  *(float4*)(dH + i) = make_float4(t.x * w, t.y * w, t.z * w, t.w * w);
}

// dH[r] = Σ_s dHp[s][r] - (0 <= t_r < n ? w_r·W[t_r] : 0)   (the one-hot part of P'; fixed order)
__global__ void ce_dh_combine_kernel(const float* __restrict__ dHp, int ns, int M, int D,
                                     const int* __restrict__ t32, const float* __restrict__ rw,
                                     const float* __restrict__ W, int n, float* __restrict__ dH) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= (long)M * D) return;
  const int r = (int)(i / D), k = (int)(i % D);
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < ns; ++s) t = c2::operator+(t, *(const float4*)(dHp + (long)s * M * D + i));
  const int tg = t32[r];
  if (tg >= 0 && tg < n) t = c2::fma4(-rw[r], *(const float4*)(W + (long)tg * D + k), t);
  *(float4*)(dH + i) = t;
}

// ---------------------------------------------------------------- backward: dW, db
// grid (ceil(n/128), n_rsplit); 4 waves x 32 columns, one wave per SIMD; sweeps the split's rows
// 64 at a time over three H images — the dH kernel with the roles of H and W exchanged:
//   step t:  [ S(t+1) = H_{t+1}·W_cᵀ on the matrix cores  ∥  epilogue of S(t), first 24 of 32 ]
//            [ dWᵀ += H_tᵀ·P'(t)                          ∥  epilogue of S(t), last 8        ]
// P'[r][c] = 2^(s·log2e + cr_r + b2_c) with cr = log2(w_r) - lse2_r (c2dsr_ce_row_weights), db[c] = Σ_r P'[r][c];
// the one-hot part of (softmax - onehot)·w is applied afterwards by c2dsr_ce_onehot_dw.  The dWᵀ MFMAs run column-block-major (x[0][0] first), so the last
// epilogue slice overlaps the first 24 of them.
// Hb holds ⌈M/64⌉·64 rows (zero padding past M); crow is padded likewise with -inf.  dWp [n_rsplit][n][D], dbp [n_rsplit][n] fp32 partials.
template <int D>
__global__ __launch_bounds__(256, 1) void ce_dw_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                       const float* __restrict__ bias2, int M, int n,
                                                       int rows_per_split, const float* __restrict__ crow,
                                                       float* __restrict__ dWp,
                                                       float* __restrict__ dbp) {
  constexpr int KS = D / 16;
  constexpr int KB = D / 32;
  constexpr int NQ = KB * 4;
  constexpr int DS = CE_DW_DS;
  constexpr int DT = CE_DW_DT;
  constexpr int IMG = TILE * D * 2;
  constexpr int NDMA = (TILE / 4) * (D / 128) / 4;
  constexpr int NB = 4;  // H images: S(t+1), dW(t), tile t+2 landed, t+3 landing
  static_assert(KS >= 8, "the epilogue schedule assumes at least 8 S k-steps");
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float rv[NB][4][TILE];  // [buffer][wave][row] crow
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int cc = min(c, n - 1);
  const int r_beg = blockIdx.y * rows_per_split;
  const int r_end = min(M, r_beg + rows_per_split);
  const int ntiles = r_end > r_beg ? (r_end - r_beg + TILE - 1) / TILE : 0;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  float db = 0.f;
  if (ntiles > 0) {
    const int r_last = r_beg + (ntiles - 1) * TILE;
    const ImgOffsets o0 = img_offsets(lane);
    const int ib = (int)lds_addr(img[0]);
    const int rvb = (int)lds_addr(rv[0][w]) + 16 * (lane >> 5);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + 4 * i;
      constexpr int GROUPS = TILE / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz_f(row);
      dvoff[i] = (unsigned)((row * D + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * (TILE * 256) + rg * 1024));
    }
    auto dma_rows = [&](int r0, int buf) { dma4(crow + r0 + lane, rv[buf][w]); };  // each wave its own copy
    auto dma = [&](int tt) {  // tile tt (clamped to the last) → buffer tt % NB
      const int r0 = min(r_beg + tt * TILE, r_last);
      const int buf = tt % NB;
      const bf16* base = Hb + (long)r0 * D;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma_rows(r0, buf);
    };
    bf16x8 wf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[ks] = *(const bf16x8*)(Wb + (long)cc * D + ks * 16 + 8 * (lane >> 5));
    float b2 = bias2[c];  // -inf past n: those columns contribute 0
    dma(0);
    dma(1);
    dma(2);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) pin(wf[ks]);
    pin(b2);
    vm_drain();
    dma_wait();
    __syncthreads();
    auto offs = [&](int b, int (&ro)[8], int (&to)[4][2]) {
      const int add = ib + b * IMG;
#pragma unroll
      for (int k = 0; k < 8; ++k) ro[k] = o0.roff[k] + add;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        to[v][0] = o0.troff[v][0] + add;
        to[v][1] = o0.troff[v][1] + add;
      }
    };
    // ---- S(0) (not overlapped)
    f32x16 sc[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 f0 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256);
      const bf16x8 f1 = *(const bf16x8*)(img[0] + o0.roff[ks & 7] + (ks >> 3) * TILE * 256 + 32 * 256);
      if (ks == 0) {
        sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, wf[0], f32x16{}, 0, 0, 0);
        sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, wf[0], f32x16{}, 0, 0, 0);
      } else {
        sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, wf[ks], sc[0], 0, 0, 0);
        sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, wf[ks], sc[1], 0, 0, 0);
      }
    }
    for (int t = 0; t < ntiles; ++t) {
      const int bh = t % NB, bs = (t + 1) % NB;
      const int rn = min(r_beg + (t + 3) * TILE, r_last);  // tile t+3: pieces in the dWᵀ phase
      const bf16* nsrc = Hb + (long)rn * D;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      dma_rows(rn, (t + 3) % NB);
      ImgOffsets oS, oH;
      {
        int ro[8], to[4][2];
        offs(bs, ro, to);
#pragma unroll
        for (int k = 0; k < 8; ++k) oS.roff[k] = ro[k];
        offs(bh, ro, to);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          oH.troff[v][0] = to[v][0];
          oH.troff[v][1] = to[v][1];
        }
      }
      // per-row constants of this lane's 32 rows: element i of column block cb is row cb·32 + creg(i)
      f32x4 cr4[2][4];
      {
        const int rvo = rvb + bh * (4 * TILE * 4);  // [NB][4][TILE]; row r4 = cb·32 + 8·j4 + 4·(lane >> 5)
        [&]<int... J>(std::integer_sequence<int, J...>) {
          ((cr4[J >> 2][J & 3] = lds_ld<f32x4, 128 * (J >> 2) + 32 * (J & 3)>(rvo)), ...);
        }(std::make_integer_sequence<int, 8>{});
      }
      bf16x8 x[2][2];
#define C2_DW_EPI(cb, i)                                                                                    \
  {                                                                                                         \
    const float ev = ex2(fmaf(sc[cb][i], LOG2E, ((const float*)&cr4[cb][(i) >> 2])[(i) & 3]) + b2);         \
    sc[cb][i] = ev;                                                                                         \
    db += ev;                                                                                               \
  }
// the 32 epilogue elements in the order the dWᵀ MFMAs need them (e → block e/16, element e%16) are
// spread over U = 2·KS + 2·KB issue units: two per S k-step (2 MFMAs), one per dWᵀ step q < 2·KB;
// x[cb][st] is packed right after its last element, before its first use at q = (2cb + st)·KB
#define C2_DW_EPI_UNITS(u0, u1)                                                   \
  {                                                                               \
    constexpr int U = 2 * KS + 2 * KB;                                            \
    constexpr int e0 = (32 * (u0) + U - 1) / U, e1 = (32 * (u1) + U - 1) / U;     \
    _Pragma("unroll") for (int e = e0; e < e1; ++e) C2_DW_EPI(e >> 4, e & 15)     \
    _Pragma("unroll") for (int cs = 0; cs < 4; ++cs) if (8 * cs + 7 >= e0 && 8 * cs + 7 < e1) \
      x[cs >> 1][cs & 1] = acc_frag(sc[cs >> 1], cs & 1);                         \
  }
      // ---- S(t+1) ∥ epilogue(t)
      f32x16 sn[2];
      bf16x8 fa[DS + 2][2];
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((fa[P][0] = row_frag_c<TILE, 0, P, 0>(oS), fa[P][1] = row_frag_c<TILE, 32, P, 0>(oS)), ...);
      }(std::make_integer_sequence<int, DS>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              if constexpr (ks + DS < KS) {
                fa[(ks + DS) % (DS + 2)][0] = row_frag_c<TILE, 0, ks + DS, 0>(oS);
                fa[(ks + DS) % (DS + 2)][1] = row_frag_c<TILE, 32, ks + DS, 0>(oS);
              }
              if constexpr (ks == 0) {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][0], wf[0], f32x16{}, 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][1], wf[0], f32x16{}, 0, 0, 0);
              } else {
                sn[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][0], wf[ks], sn[0], 0, 0, 0);
                sn[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (DS + 2)][1], wf[ks], sn[1], 0, 0, 0);
              }
              C2_DW_EPI_UNITS(2 * ks, 2 * ks + 2)
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
      // ---- dWᵀ[k][c] += Σ_r H[r][k] P'[r][c], q = (cb, st, kb): x[cb][st] is used from q = 16cb + 8st on
      bf16x8 tf[DT + 2];
#define C2_DW_TF(q1) tr_frag_c<TILE, (((q1) / KB) >> 1) * 32 + 16 * (((q1) / KB) & 1), ((q1) % KB) * 32, 0>(oH)
      [&]<int... P>(std::integer_sequence<int, P...>) { ((tf[P] = C2_DW_TF(P)), ...); }(std::make_integer_sequence<int, DT>{});
      __builtin_amdgcn_sched_barrier(0);
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        (
            [&] {
              constexpr int q = Q;
              constexpr int cs = q / KB, kb = q % KB;
              if constexpr (q + DT < NQ) tf[(q + DT) % (DT + 2)] = C2_DW_TF(q + DT);
              dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[q % (DT + 2)], x[cs >> 1][cs & 1], dacc[kb], 0, 0, 0);
              if constexpr (q < 2 * KB) C2_DW_EPI_UNITS(2 * KS + q, 2 * KS + q + 1)
              if constexpr (q % 4 == 3 && q / 4 < NDMA) dma16_s<q == 3>(nsrc, dvoff[q / 4], ddst[q / 4] + nbuf);
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NQ>{});
#undef C2_DW_TF
#undef C2_DW_EPI_UNITS
#undef C2_DW_EPI
      sc[0] = sn[0];
      sc[1] = sn[1];
      dma_wait_keep<NDMA + 1>();  // tile t+2 has landed; tile t+3 (pieces + row vector) may be in flight
      __syncthreads();
    }
  }
  db += __shfl_xor(db, 32, 64);
  if (c < n) {
    if (lane < 32) dbp[(long)blockIdx.y * n + c] = db;
    float* out = dWp + ((long)blockIdx.y * n + c) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
  }
}

// out[i] = beta*out[i] + Σ_s part[s][i]   (fixed order); float4 per thread (n % 4 == 0 and 16-byte aligned
// buffers; otherwise one element per thread)
template <bool V4>
__global__ void sum_parts_kernel(const float* __restrict__ part, int nparts, long n, float beta,
                                 float* __restrict__ out) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * (V4 ? 4 : 1);
  if (i >= n) return;
  if constexpr (V4) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < nparts; ++s) {
      const float4 v = *(const float4*)(part + (long)s * n + i);
      t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
    }
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (beta != 0.f) {
      const float4 w = *(const float4*)(out + i);
      o = make_float4(beta * w.x, beta * w.y, beta * w.z, beta * w.w);
    }
    *(float4*)(out + i) = make_float4(o.x + t.x, o.y + t.y, o.z + t.z, o.w + t.w);
  } else {
    float t = 0.f;
    for (int s = 0; s < nparts; ++s) t += part[(long)s * n + i];
    out[i] = (beta == 0.f ? 0.f : beta * out[i]) + t;
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, long n, bf16* __restrict__ y) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 3 < n) {
    const float4 v = *(const float4*)(x + i);
    y[i] = (bf16)v.x;
    y[i + 1] = (bf16)v.y;
    y[i + 2] = (bf16)v.z;
    y[i + 3] = (bf16)v.w;
  } else {
    for (long j = i; j < n; ++j) y[j] = (bf16)x[j];
  }
}

// bias2[c] = bias[c]·log2e for c < n, -inf up to n_pad
__global__ void bias2_kernel(const float* __restrict__ bias, int n, int n_pad, float* __restrict__ b2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n_pad) b2[c] = c < n ? bias[c] * LOG2E : -INFINITY;
}

// per row r < M_pad: rw = valid ? gscale*lam*coef[r >= split] : 0; t32 = target (-1 past M);
// crow = log2(rw) - lse2 (-inf where rw = 0 and past M); dpad = exp(pl - lse)·rw (the pad column of the softmax; its target is ignored)
__global__ void ce_roww_kernel(const int64_t* __restrict__ tgt, int M, int M_pad, int ignore,
                               const float* __restrict__ coef, int split, const float* __restrict__ gscale,
                               float lam, const float* __restrict__ pl, const float* __restrict__ lse,
                               float* __restrict__ rw, int* __restrict__ t32, const float* __restrict__ lse2,
                               float* __restrict__ crow, float* __restrict__ dpad) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M_pad) return;
  if (r >= M) {
    rw[r] = 0.f;
    t32[r] = -1;
    crow[r] = -INFINITY;
    return;
  }
  const long t = tgt[r];
  const float w = t != ignore ? gscale[0] * lam * coef[r >= split ? 1 : 0] : 0.f;
  rw[r] = w;
  t32[r] = (int)t;
  crow[r] = w > 0.f ? __log2f(w) - lse2[r] : -INFINITY;
  dpad[r] = expf(pl[r] - lse[r]) * w;
}

// self-test of the transposed fragment addressing: image row = rr, col = k holds rr*256+k (int16)
__global__ void selftest_tr_kernel(int rr0, int kb0, short* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char img[TILE * 256 * 2];
  for (int q = threadIdx.x; q < TILE * 256; q += blockDim.x) {
    const int row = q / 256, k = q % 256;
    *(short*)(img + img_off(row, k)) = (short)(row * 256 + k);
  }
  __syncthreads();
  const int lane = threadIdx.x;
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (TILE * 256);
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + base + swz(row, ch) + 8 * (p & 1)));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + base + swz(row + 8, ch) + 8 * (p & 1)));
  for (int j = 0; j < 4; ++j) {
    out[lane * 8 + j] = lo[j];
    out[lane * 8 + 4 + j] = hi[j];
  }
  // row fragment check (rows rr0.., k-slice kb0..)
  const bf16x8 rf = row_frag(img, rr0, kb0, lane);
  const short* rs = (const short*)&rf;
  for (int j = 0; j < 8; ++j) out[512 + lane * 8 + j] = rs[j];
}

int per_split(int total, int nsplit, int gran) {
  int tiles = c2::ceil_div(total, gran);
  return c2::ceil_div(tiles, nsplit) * gran;
}

}  // namespace

C2_API int c2dsr_ce_supported(int D) { return D == 128 || D == 256; }

C2_API int c2dsr_f32_to_bf16(const float* x, long n, void* y, void* stream) {
  if (n == 0) return 0;
  f32_to_bf16_kernel<<<c2::ceil_div((n + 3) / 4, 256), 256, 0, (hipStream_t)stream>>>(x, n, (bf16*)y);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_ce_bias2(const float* bias, int n, int n_pad, float* bias2, void* stream) {
  bias2_kernel<<<c2::ceil_div(n_pad, 256), 256, 0, (hipStream_t)stream>>>(bias, n, n_pad, bias2);
  C2_CHECK_LAUNCH();
  return 0;
}

// forward: part_m/part_s [n_split][M] → (with pad logits, targets, fp32 H/W/bias for the target
// logit) lse, lse2 (= lse·log2e), loss_row [M].
C2_API int c2dsr_ce_fused_fwd(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                              float* part_m, float* part_s, const float* padlogit, const int64_t* tgt,
                              const float* H, const float* W, const float* bias, float* lse, float* lse2,
                              float* loss_row, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  const int per = per_split(n, n_split, TILE);
  dim3 grid(c2::ceil_div(M, 256), n_split);
  if (D == 128)
    ce_lse_kernel<128><<<grid, 512, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, part_m, part_s);
  else if (D == 256)
    ce_lse_kernel<256><<<grid, 512, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, part_m, part_s);
  else
    return (int)hipErrorInvalidValue;
  ce_rows_kernel<<<c2::ceil_div(M, 4), 256, 0, s>>>(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse,
                                                    lse2, loss_row);
  C2_CHECK_LAUNCH();
  return 0;
}

// forward + the softmax part of dH: part_m/part_s [n_split][M] (log2-domain max, sum) and Up [n_split][M][D]
// → (with pad logits, targets, fp32 H/W/bias for the target logit) lse, lse2, loss_row [M]
C2_API int c2dsr_ce_fused_fwd_u(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D,
                                int n_split, float* part_m, float* part_s, float* Up, const float* padlogit,
                                const int64_t* tgt, const float* H, const float* W, const float* bias, float* lse,
                                float* lse2, float* loss_row, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  const int per = per_split(n, n_split, TILE);
  dim3 grid(c2::ceil_div(M, 128), n_split);
  if (D == 128)
    ce_fwdu_kernel<128><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, part_m, part_s, Up);
  else if (D == 256)
    ce_fwdu_kernel<256><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, part_m, part_s, Up);
  else
    return (int)hipErrorInvalidValue;
  ce_rows_kernel<<<c2::ceil_div(M, 4), 256, 0, s>>>(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse,
                                                    lse2, loss_row);
  C2_CHECK_LAUNCH();
  return 0;
}

// per row: lse over the splits' (max, sum) partials and the pad column, target logit, loss (see ce_rows_kernel)
C2_API int c2dsr_ce_rows(const float* part_m, const float* part_s, int n_split, int M, const float* padlogit,
                         const int64_t* tgt, int n, const float* H, const float* W, const float* bias, int D,
                         float* lse, float* lse2, float* loss_row, void* stream) {
  if (M == 0) return 0;
  ce_rows_kernel<<<c2::ceil_div(M, 4), 256, 0, (hipStream_t)stream>>>(part_m, part_s, n_split, M, padlogit, tgt, n, H,
                                                                     W, bias, D, lse, lse2, loss_row);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_ce_dh_from_u(const float* Up, const float* part_m, int ns, int M, int D, const float* lse2,
                              const int* t32, const float* rw, const float* W, int n, float* dH, void* stream) {
  if (M == 0) return 0;
  if (D % 4 || ns < 1 || ns > 16) return (int)hipErrorInvalidValue;  // the kernel holds at most 16 splits
  ce_dh_from_u_kernel<<<c2::ceil_div((long)M * D / 4, 256), 256, 0, (hipStream_t)stream>>>(Up, part_m, ns, M, D, lse2,
                                                                                          t32, rw, W, n, dH);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_ce_row_weights(const int64_t* tgt, int M, int M_pad, int ignore, const float* coef, int split,
                                const float* gscale, float lam, const float* padlogit, const float* lse, float* rw,
                                int* t32, const float* lse2, float* crow, float* dpad, void* stream) {
  if (M_pad == 0) return 0;
  ce_roww_kernel<<<c2::ceil_div(M_pad, 256), 256, 0, (hipStream_t)stream>>>(tgt, M, M_pad, ignore, coef, split,
                                                                             gscale, lam, padlogit, lse, rw, t32,
                                                                             lse2, crow, dpad);
  C2_CHECK_LAUNCH();
  return 0;
}

// dHp[s][r] = Σ_{c in split s} P'[r][c] W[c]  (combine with c2dsr_sum_parts)
C2_API int c2dsr_ce_fused_dh(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                             const float* crow, float* dHp, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  const int per = per_split(n, n_split, TILE);
  dim3 grid(c2::ceil_div(M, 128), n_split);
  if (D == 128)
    ce_dh_kernel<128><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, crow, dHp);
  else if (D == 256)
    ce_dh_kernel<256><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, crow, dHp);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  return 0;
}

// dWp[s][c] = Σ_{r in split s} P'[r][c] H[r];  dbp[s][c] = Σ_r P'[r][c]  (softmax part; combine with
// c2dsr_sum_parts, then c2dsr_ce_onehot_dw)
C2_API int c2dsr_ce_fused_dw(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_rsplit,
                             const float* crow, float* dWp, float* dbp, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  const int per = per_split(M, n_rsplit, TILE);
  dim3 grid(c2::ceil_div(n, 128), n_rsplit);
  if (D == 128)
    ce_dw_kernel<128><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, crow, dWp,
                                           dbp);
  else if (D == 256)
    ce_dw_kernel<256><<<grid, 256, 0, s>>>((const bf16*)Hb, (const bf16*)Wb, bias2, M, n, per, crow, dWp,
                                           dbp);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  return 0;
}

// dH = Σ_s dHp[s] - w_r·W[t_r]  (the one-hot part of P' for rows with an item target)
C2_API int c2dsr_ce_dh_combine(const float* dHp, int ns, int M, int D, const int* t32, const float* rw, const float* W,
                               int n, float* dH, void* stream) {
  if (M == 0) return 0;
  if (D % 4) return (int)hipErrorInvalidValue;
  ce_dh_combine_kernel<<<c2::ceil_div((long)M * D / 4, 256), 256, 0, (hipStream_t)stream>>>(dHp, ns, M, D, t32, rw, W,
                                                                                            n, dH);
  C2_CHECK_LAUNCH();
  return 0;
}

// out[i] = beta*out[i] + Σ_s part[s][i]  (fixed order) — combines the split partials
C2_API int c2dsr_sum_parts(const float* part, int nparts, long n, float beta, float* out, void* stream) {
  if (n == 0) return 0;
  const bool v4 = n % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)out & 15) == 0;
  if (v4)
    sum_parts_kernel<true><<<c2::ceil_div(n / 4, 256), 256, 0, (hipStream_t)stream>>>(part, nparts, n, beta, out);
  else
    sum_parts_kernel<false><<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(part, nparts, n, beta, out);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_selftest_tr(int rr0, int kb0, short* out, void* stream) {
  selftest_tr_kernel<<<1, 64, 0, (hipStream_t)stream>>>(rr0, kb0, out);
  C2_CHECK_LAUNCH();
  return 0;
}
