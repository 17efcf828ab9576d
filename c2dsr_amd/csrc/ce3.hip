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
// xf32).  Logits are never materialised.
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
// Per 32-row tile and wave (32 stationary rows): 48 MFMAs for S, 48 for the second product; the swept
// image (32 rows × 2D bf16 = 32 KiB at D = 256) streams through four LDS buffers by saddr LDS-DMA
// (tile t+3 issued during the second product of tile t), read row-wise (ds_read_b128) for S and
// transposed (ds_read_b64_tr_b16) for the second product, whose B operand is S's accumulator itself
// (P split into hi/lo in registers).  The epilogue of S(t) runs in the MFMA shadow of S(t+1).
#include "img.h"

#include <utility>

// tuning knobs (tools/ce3_micro.py; the defaults are the shipped configuration)
#ifndef CE3_DS
#define CE3_DS 2
#endif
#ifndef CE3_DT
#define CE3_DT 2
#endif

namespace {

using namespace c2img;

constexpr int T3 = 32;  // swept rows per LDS tile

// lo part of a B-operand fragment: element j = a[8s+j] − hi[j], rounded
__device__ __forceinline__ bf16x8 lo_frag(const f32x16& a, int s, const bf16x8& hi) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)(a[8 * s + j] - (float)hi[j]);
  return r;
}

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

template <int D, int MODE>
__global__ __launch_bounds__(256, 1) void ce3_kernel(const bf16* __restrict__ Xs, const bf16* __restrict__ Xw,
                                                     const float* __restrict__ svec, const float* __restrict__ wvec,
                                                     int n_s, int n_w, int per_split, float* __restrict__ part_m,
                                                     float* __restrict__ part_s, float* __restrict__ outp) {
  constexpr int KS = D / 16;                       // k-steps of a product
  constexpr int KB = D / 32;                       // 32-wide output k-blocks of the second product
  constexpr int NQ = 2 * KB;                       // second-product steps: (k-block, 16-row half of the tile)
  constexpr int D2 = 2 * D;                        // hi ‖ lo
  constexpr int IMG = T3 * D2 * 2;                 // bytes per image
  constexpr int NDMA = (T3 / 4) * (D2 / 128) / 4;  // LDS-DMA wave-instructions per wave per tile
  constexpr int NB = 4;                            // images: S(t+1), second product(t), t+2 landed, t+3 landing
  constexpr int DS = CE3_DS, DT = CE3_DT;          // LDS fragment prefetch depth (steps ahead)
  constexpr int EPK = 16 / KS;                     // epilogue elements per S k-step
  constexpr int MPK = 16 / NQ;                     // prep elements per second-product step
  constexpr float TAU = 8.f;                       // lazy-max threshold (p ≤ 2^TAU)
  static_assert(KS * EPK == 16 && NQ * MPK == 16 && NQ % NDMA == 0, "tile / wave split");
  constexpr int QD = NQ / NDMA;                    // second-product steps per DMA piece
  __shared__ __attribute__((aligned(16))) char img[NB][IMG];
  __shared__ __attribute__((aligned(16))) float wv[NB][4][64];  // [buffer][wave]: the tile's per-row constants
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int sc_ = min(s, n_s - 1);
  const int w_beg = blockIdx.y * per_split;
  const int w_end = min(n_w, w_beg + per_split);
  const int ntiles = w_end > w_beg ? (w_end - w_beg + T3 - 1) / T3 : 0;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  float mrow = -INFINITY, zrow = 0.f;  // MODE 0: running max (log2 domain) and sum; MODE 1: zrow = db
  if (ntiles > 0) {
    const int w_last = w_beg + (ntiles - 1) * T3;
    const ImgOffsets o0 = img_offsets(lane);
    const int ib = (int)lds_addr(img[0]);
    unsigned dvoff[NDMA], ddst[NDMA];
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = w + 4 * i;
      constexpr int GROUPS = T3 / 4;
      const int half = q / GROUPS, rg = q % GROUPS;
      const int row = rg * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ swz_f(row);
      dvoff[i] = (unsigned)((row * D2 + half * 128 + lch * 8) * 2);
      ddst[i] = __builtin_amdgcn_readfirstlane((unsigned)(ib + half * (T3 * 256) + rg * 1024));
    }
    auto dma = [&](int tt) {  // tile tt (clamped to the last) → buffer tt % NB
      const int r0 = min(w_beg + tt * T3, w_last);
      const int buf = tt % NB;
      const bf16* base = Xw + (long)r0 * D2;
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma16_s(base, dvoff[i], ddst[i] + buf * IMG);
      dma4(wvec + r0 + lane, wv[buf][w]);
    };
    bf16x8 fh[KS], fl[KS];  // the lane's stationary row: hi and lo k-slices (B operands)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      fh[ks] = *(const bf16x8*)(Xs + (long)sc_ * D2 + ks * 16 + 8 * (lane >> 5));
      fl[ks] = *(const bf16x8*)(Xs + (long)sc_ * D2 + D + ks * 16 + 8 * (lane >> 5));
    }
    const float b2s = MODE == 1 ? svec[s] : 0.f;  // MODE 1: the lane column's bias·log2e (-inf past n)
    dma(0);
    dma(1);
    dma(2);
    vm_drain();
    dma_wait();
    __syncthreads();
    auto offs_rows = [&](int b, ImgOffsets& o) {
      const int add = ib + b * IMG;
#pragma unroll
      for (int c = 0; c < 8; ++c) o.roff[c] = o0.roff[c] + add;
    };
    auto offs_tr = [&](int b, ImgOffsets& o) {
      const int add = ib + b * IMG;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        o.troff[v][0] = o0.troff[v][0] + add;
        o.troff[v][1] = o0.troff[v][1] + add;
      }
    };
    // the per-swept-row constants of this lane's 16 accumulator rows (row creg(i, lane) = (i&3) + 8(i>>2) + 4h)
    auto wconst = [&](int b, f32x4 (&c4)[4]) {
      const int bo = (int)lds_addr(wv[b][w]) + 16 * (lane >> 5);
      [&]<int... J>(std::integer_sequence<int, J...>) {
        ((c4[J] = lds_ld<f32x4, 32 * J>(bo)), ...);
      }(std::make_integer_sequence<int, 4>{});
    };
    // ---- S(0) and its prep (not overlapped)
    f32x16 sc;
    {
      ImgOffsets oS;
      offs_rows(0, oS);
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              const bf16x8 ah = row_frag_c<T3, 0, ks, 0>(oS);
              const bf16x8 al = row_frag_c<T3, 0, KS + ks, 0>(oS);
              if constexpr (ks == 0)
                sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fh[0], f32x16{}, 0, 0, 0);
              else
                sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fh[ks], sc, 0, 0, 0);
              sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, fh[ks], sc, 0, 0, 0);
              sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fl[ks], sc, 0, 0, 0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
    }
    float mnext = -INFINITY;
    {
      f32x4 c4[4];
      wconst(0, c4);
      float tm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = fmaf(sc[i], LOG2E, ((const float*)&c4[i >> 2])[i & 3]) + b2s;
        sc[i] = v;
        tm = fmaxf(tm, v);
      }
      if constexpr (MODE == 0) mnext = half_max(tm);
    }
    // fragment rings carried across the phase boundaries: the first DS row fragments of the next S phase are
    // read during the last steps of the second product, the first DT transposed fragments of the second
    // product during the last S steps — no LDS-latency bubble at either boundary
    bf16x8 fa[DS + 2][2];
    bf16x8 tf[DT + 2][2];
    {
      ImgOffsets oS;
      offs_rows(1 % NB, oS);  // S(1) reads tile 1 (landed in the prologue)
      [&]<int... P>(std::integer_sequence<int, P...>) {
        ((fa[P][0] = row_frag_c<T3, 0, P, 0>(oS), fa[P][1] = row_frag_c<T3, 0, KS + P, 0>(oS)), ...);
      }(std::make_integer_sequence<int, DS>{});
    }
    for (int t = 0; t < ntiles; ++t) {
      const int bh = t % NB, bs = (t + 1) % NB;
      const int rn = min(w_beg + (t + 3) * T3, w_last);
      const bf16* nsrc = Xw + (long)rn * D2;
      const unsigned nbuf = ((t + 3) % NB) * IMG;
      dma4(wvec + rn + lane, wv[(t + 3) % NB][w]);
      float msub = 0.f;
      if constexpr (MODE == 0) {
        // lazy rescale: the row's max moved up by more than TAU (always on the first tile with a finite max)
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
        msub = mrow == -INFINITY ? 0.f : mrow;  // all of S(t) is -inf then: p = 0
      }
      ImgOffsets oS, oH;
      offs_rows(bs, oS);
      offs_tr(bh, oH);
      // ---- S(t+1) ∥ epilogue(t): p = 2^(v − msub), packed into the hi / lo B fragments; the last DT steps
      //      read the second product's first transposed fragments (tile t)
      f32x16 sn;
      bf16x8 xh[2], xl[2];
      [&]<int... K>(std::integer_sequence<int, K...>) {
        (
            [&] {
              constexpr int ks = K;
              if constexpr (ks + DS < KS) {
                fa[(ks + DS) % (DS + 2)][0] = row_frag_c<T3, 0, ks + DS, 0>(oS);
                fa[(ks + DS) % (DS + 2)][1] = row_frag_c<T3, 0, KS + ks + DS, 0>(oS);
              } else {
                constexpr int q1 = ks + DS - KS;  // 0 .. DS-1 → the second product's fragments q1 < DT
                if constexpr (q1 < DT) {
                  tf[q1][0] = tr_frag_c<T3, (q1 & 1) * 16, (q1 >> 1) * 32, 0>(oH);
                  tf[q1][1] = tr_frag_c<T3, (q1 & 1) * 16, D + (q1 >> 1) * 32, 0>(oH);
                }
              }
              const bf16x8& ah = fa[ks % (DS + 2)][0];
              const bf16x8& al = fa[ks % (DS + 2)][1];
              if constexpr (ks == 0)
                sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fh[0], f32x16{}, 0, 0, 0);
              else
                sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fh[ks], sn, 0, 0, 0);
              sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, fh[ks], sn, 0, 0, 0);
              sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, fl[ks], sn, 0, 0, 0);
#pragma unroll
              for (int e = 0; e < EPK; ++e) {
                const int i = ks * EPK + e;
                const float pv = ex2(sc[i] - msub);
                sc[i] = pv;
                zrow += pv;
              }
              if constexpr ((ks * EPK + EPK) % 8 == 0) {
                constexpr int st = (ks * EPK) / 8;
                xh[st] = acc_frag(sc, st);
                xl[st] = lo_frag(sc, st, xh[st]);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, KS>{});
      // ---- tile t+2 (issued during the previous second product) has landed for every wave, and every wave
      //      is past its reads of buffer (t+3) % NB (the previous second product): publish / reuse
      dma_wait();
      __syncthreads();
      // ---- second product (t) ∥ prep of S(t+1) ∥ DMA of tile t+3; the last DS steps read the first row
      //      fragments of S(t+2) (tile t+2, landed above)
      //      Oᵀ[k][s] += Σ_{c in tile} X_w[c][k]·P[c][s],  q = (kb = q >> 1, half st = q & 1)
      ImgOffsets oN;
      offs_rows((t + 2) % NB, oN);
      f32x4 c4n[4];
      wconst(bs, c4n);
      float tm = -INFINITY;
      [&]<int... Q>(std::integer_sequence<int, Q...>) {
        (
            [&] {
              constexpr int q = Q;
              constexpr int kb = q >> 1, st = q & 1;
              if constexpr (q + DT < NQ) {
                constexpr int q1 = q + DT;
                tf[q1 % (DT + 2)][0] = tr_frag_c<T3, (q1 & 1) * 16, (q1 >> 1) * 32, 0>(oH);
                tf[q1 % (DT + 2)][1] = tr_frag_c<T3, (q1 & 1) * 16, D + (q1 >> 1) * 32, 0>(oH);
              } else {
                constexpr int k1 = q + DT - NQ;  // S(t+2)'s fragments k1 < DS
                if constexpr (k1 < DS) {
                  fa[k1][0] = row_frag_c<T3, 0, k1, 0>(oN);
                  fa[k1][1] = row_frag_c<T3, 0, KS + k1, 0>(oN);
                }
              }
              const bf16x8& th = tf[q % (DT + 2)][0];
              const bf16x8& tl = tf[q % (DT + 2)][1];
              dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, xh[st], dacc[kb], 0, 0, 0);
              dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, xl[st], dacc[kb], 0, 0, 0);
              dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, xh[st], dacc[kb], 0, 0, 0);
              if constexpr (q % QD == QD - 1)
                dma16_s<q == QD - 1>(nsrc, dvoff[q / QD], ddst[q / QD] + nbuf);
#pragma unroll
              for (int e = 0; e < MPK; ++e) {
                const int i = q * MPK + e;
                const float v = fmaf(sn[i], LOG2E, ((const float*)&c4n[i >> 2])[i & 3]) + b2s;
                sn[i] = v;
                tm = fmaxf(tm, v);
              }
              __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
      }(std::make_integer_sequence<int, NQ>{});
      if constexpr (MODE == 0) mnext = half_max(tm);
      sc = sn;
    }
  }
  const float ztot = half_sum(zrow);
  if (s < n_s) {
    if (lane < 32) {
      if constexpr (MODE == 0) part_m[(long)blockIdx.y * n_s + s] = mrow;
      part_s[(long)blockIdx.y * n_s + s] = ztot;
    }
    float* out = outp + ((long)blockIdx.y * n_s + s) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
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

int per_split3(int total, int nsplit) {
  const int tiles = c2::ceil_div(total, T3);
  return c2::ceil_div(tiles, nsplit) * T3;
}

template <int MODE>
int launch3(const void* Xs, const void* Xw, const float* svec, const float* wvec, int n_s, int n_w, int D, int nsplit,
            float* pm, float* ps, float* out, hipStream_t st) {
  const int per = per_split3(n_w, nsplit);
  dim3 grid(c2::ceil_div(n_s, 128), nsplit);
  if (D == 128)
    ce3_kernel<128, MODE><<<grid, 256, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s, n_w, per, pm, ps,
                                                out);
  else if (D == 256)
    ce3_kernel<256, MODE><<<grid, 256, 0, st>>>((const bf16*)Xs, (const bf16*)Xw, svec, wvec, n_s, n_w, per, pm, ps,
                                                out);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int c2dsr_ce_rows(const float* part_m, const float* part_s, int n_split, int M, const float* padlogit,
                             const int64_t* tgt, int n, const float* H, const float* W, const float* bias, int D,
                             float* lse, float* lse2, float* loss_row, void* stream);

C2_API int c2dsr_ce3_supported(int D) { return D == 128 || D == 256; }

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
  const int e = launch3<0>(Hx, Wx, nullptr, bias2, M, n, D, n_split, part_m, part_s, Up, (hipStream_t)stream);
  if (e) return e;
  return c2dsr_ce_rows(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse, lse2, loss_row, stream);
}

C2_API int c2dsr_ce3_fused_dw(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_rsplit,
                              const float* crow, float* dWp, float* dbp, void* stream) {
  if (n == 0) return 0;
  return launch3<1>(Wx, Hx, bias2, crow, n, M, D, n_rsplit, nullptr, dbp, dWp, (hipStream_t)stream);
}
