// MFMA operand images in LDS shared by the gfx950 kernels (fused CE, row GEMMs):
// XOR-swizzled bf16 tiles read row-wise (ds_read_b128) and transposed
// (ds_read_b64_tr_b16), LDS-DMA loaders with hand-placed waits, register pinning.
#pragma once
#include "common.h"

namespace c2img {

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float LOG2E = 1.4426950408889634f;
constexpr int TILE = 64;  // rows of the swept operand per LDS tile

// ---------------------------------------------------------------- LDS image
// A [TILE][D] bf16 tile is stored as D/128 half-tiles of [TILE][128] bf16 (256-byte
// rows); 16-byte chunk `ch` of row `row` sits at swz(row, ch).
__device__ __forceinline__ int swz(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
// byte offset of element (row, k) (k multiple of 8 for a 16-byte read)
template <int TR = TILE>
__device__ __forceinline__ int img_off(int row, int k) { return (k >> 7) * (TR * 256) + swz(row, (k & 127) >> 3) + 2 * (k & 7); }

// A-operand fragment for v_mfma_f32_32x32x16_bf16 whose rows are TILE rows r0..r0+31 and
// whose k-slice is k0..k0+15 (k0 multiple of 16): lane (i = l&31, h = l>>5) gets (row r0+i, k0+8h..+7).
template <int TR = TILE>
__device__ __forceinline__ bf16x8 row_frag(const char* img, int r0, int k0, int lane) {
  const int row = r0 + (lane & 31), k = k0 + 8 * (lane >> 5);
  return *(const bf16x8*)(img + img_off<TR>(row, k));
}

// Transposed fragment: the MFMA operand whose row index is the image's k (kb0..kb0+31 ↔ lane&31)
// and whose reduction index runs over image rows in the permuted order of an accumulator
// fed back as B: element j of lane half h ↔ image row rr0 + 8*(j>>2) + 4*h + (j&3).
template <int TR = TILE>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int rr0, int kb0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);  // this 16-lane group's 16 image columns
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (TR * 256);
  const char* a0 = img + base + swz(row, ch) + 8 * (p & 1);
  const char* a1 = img + base + swz(row + 8, ch) + 8 * (p & 1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// accumulator registers 8s..8s+7 → bf16 B operand of k-step s
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

typedef __attribute__((address_space(3))) char lds_char;

// One LDS-DMA wave-instruction: each lane copies `bytes` (4 or 16) from its global address to
// LDS[m0 + lane*bytes].  Issued from inline asm so the compiler's wait-count pass does not
// conservatively drain it before every later LDS read (it cannot prove the prefetch buffer
// disjoint from the one being read); the kernels wait for it by hand (dma_wait) before the
// barrier that publishes the buffer.  m0 is written here and nowhere else in these kernels.
__device__ __forceinline__ void dma16(const void* g, char* lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(g) : "memory");
}
__device__ __forceinline__ void dma4(const void* g, void* lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(g) : "memory");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// wait until at most N vector-memory operations (the newest N; vmcnt retires in order) are outstanding
template <int N>
__device__ __forceinline__ void dma_wait_keep() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// vmcnt(0) the compiler can see (its wait-count state then knows the register operands
// loaded before the tile loop have landed, and emits no waits for them inside the loop)
// pin a register operand here: its load must be issued (and have landed) before this point
__device__ __forceinline__ void pin(bf16x8& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(int& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void vm_drain() {
  __builtin_amdgcn_sched_barrier(0);  // keep the preceding loads above the wait
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA tile loader: rows g0..g0+TILE-1 of a row-major bf16 [nrows][D] matrix into the
// swizzled image, no staging registers.  One wave-instruction fills 1 KiB = 4 image rows of
// one half-tile; lane l writes physical chunk l&15 of row l>>4, so its SOURCE is the logical
// chunk (l&15) ^ swizzle(row).  Rows past the end are clamped to the last row (finite data;
// callers zero their contribution).
template <int D, int NW = 4, int TR = TILE>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ X, long nrows, long g0, char* img) {
  constexpr int GROUPS = TR / 4;               // 4-row groups per half-tile
  constexpr int INSTR = GROUPS * (D / 128);    // wave-instructions per tile
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = w; q < INSTR; q += NW) {
    const int half = q / GROUPS, rg = q % GROUPS;
    const int row = rg * 4 + (lane >> 4);
    const int lch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
    long gr = g0 + row;
    gr = gr < nrows ? gr : nrows - 1;
    dma16(X + gr * D + half * 128 + lch * 8, img + half * (TR * 256) + rg * 1024);
  }
}

// ---------------------------------------------------------------- asm LDS reads (manual wait)
// Issued from inline asm so their order and distance ahead of the consuming MFMA are ours:
// hipcc neither hoists nor sinks them and emits no wait for them.  The consumer must first
// call lds_wait<N>(v) — "at most N LDS operations issued after v's read still outstanding"
// (lgkmcnt completes in order) — which also makes v opaque until the wait has passed.
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(size_t)(const lds_char*)p; }
__device__ __forceinline__ void lds_rd128(bf16x8& v, const char* p) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
}
__device__ __forceinline__ void lds_rd_tr(bf16x4& v, const char* p) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lds_wait2(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
// row fragment (see row_frag) by one asm read
template <int TR = TILE>
__device__ __forceinline__ void row_frag_asm(bf16x8& v, const char* img, int r0, int k0, int lane) {
  const int row = r0 + (lane & 31), k = k0 + 8 * (lane >> 5);
  lds_rd128(v, img + img_off<TR>(row, k));
}
// transposed fragment (see tr_frag) by two asm reads
template <int TR = TILE>
__device__ __forceinline__ void tr_frag_asm(bf16x8& v, const char* img, int rr0, int kb0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (TR * 256);
  bf16x4 lo, hi;
  lds_rd_tr(lo, img + base + swz(row, ch) + 8 * (p & 1));
  lds_rd_tr(hi, img + base + swz(row + 8, ch) + 8 * (p & 1));
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
}

// acc += A·B (v_mfma_f32_32x32x16_bf16) with the accumulator pinned to AGPRs ("+a"): a long-lived
// accumulator then stays in the AGPR file across loop iterations instead of being copied between
// VGPRs and AGPRs every trip.  No wait states inside (an s_nop between MFMAs costs 17-43 cycles):
// call mfma_operand_fence() once after VALU-writing an A/B operand and before the chain that reads
// it; a consumer of acc outside MFMA chains must be preceded by mfma_drain().
__device__ __forceinline__ void mfma_agpr(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_operand_fence() { asm volatile("s_nop 1" ::: "memory"); }
// the same, preceded (inside the statement) by `s_waitcnt lgkmcnt(N)` for asm-read operands: a
// separate wait statement that names the operand makes hipcc see a fresh VGPR write and pad the
// MFMA with s_nop (17-43 cycles each between MFMAs)
template <int N>
__device__ __forceinline__ void mfma_agpr_w(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%3)\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b), "n"(N));
}
template <int N>
__device__ __forceinline__ void mfma_v_w(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%3)\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b), "n"(N));
}
template <int N>
__device__ __forceinline__ void mfma_v0_w(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%3)\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(acc) : "v"(a), "v"(b), "n"(N));
}
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }

// ---------------------------------------------------------------- precomputed-offset image access
// Per-lane LDS byte offsets (relative to an image base) for the fragment reads of a [TR][256]
// image, computed once per kernel: every later read is `ds_read … offset:IMM` on one of them.
//   row fragments (row_frag(img, r0, 16ks, lane)): roff[ks & 7] + (ks >> 3)·TR·256 + r0·256
//   transposed (tr_frag(img, rr0, kb0, lane), kb0 % 32 == 0, rr0 % 16 == 0): two reads at
//   troff[(kb0 & 127) / 32][j] + rr0·256 + (kb0 >> 7)·TR·256, j = 0, 1
struct ImgOffsets {
  int roff[8];
  int troff[4][2];
};
__device__ __forceinline__ int swz_f(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ ImgOffsets img_offsets(int lane) {
  ImgOffsets o;
  const int row = lane & 31, h = lane >> 5;
#pragma unroll
  for (int c = 0; c < 8; ++c) o.roff[c] = row * 256 + 16 * ((2 * c + h) ^ swz_f(row));
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int ch = 4 * v + 2 * (g & 1) + (p >> 1);
    const int r0 = 4 * h + q, r1 = r0 + 8;
    o.troff[v][0] = r0 * 256 + 16 * (ch ^ swz_f(r0)) + 8 * (p & 1);
    o.troff[v][1] = r1 * 256 + 16 * (ch ^ swz_f(r1)) + 8 * (p & 1);
  }
  return o;
}
template <int IMM>
__device__ __forceinline__ void lds_rd128_o(bf16x8& v, int off) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(off), "n"(IMM));
}
template <int IMM>
__device__ __forceinline__ void lds_rdtr_o(bf16x4& v, int off) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(off), "n"(IMM));
}
// row fragment: image base (LDS byte address) folded into the offsets by the caller
template <int TR, int R0, int KS, int BUF>
__device__ __forceinline__ void row_frag_o(bf16x8& v, const ImgOffsets& o) {
  lds_rd128_o<BUF + (KS >> 3) * TR * 256 + R0 * 256>(v, o.roff[KS & 7]);
}
template <int TR, int RR0, int KB0, int BUF>
__device__ __forceinline__ void tr_frag_o(bf16x8& v, const ImgOffsets& o) {
  bf16x4 lo, hi;
  lds_rdtr_o<BUF + RR0 * 256 + (KB0 >> 7) * TR * 256>(lo, o.troff[(KB0 & 127) / 32][0]);
  lds_rdtr_o<BUF + RR0 * 256 + (KB0 >> 7) * TR * 256>(hi, o.troff[(KB0 & 127) / 32][1]);
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
}
// Compiler-visible LDS fragment loads at a per-lane offset (an LDS byte address) + IMM: hipcc
// counts them (exact lgkmcnt waits, no hazard pads); keep them DEPTH steps ahead with
// __builtin_amdgcn_sched_barrier(0) between steps so the scheduler cannot sink them to their use.
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;
// An LDS byte address with a provably clear sign bit: only then does the backend fold a
// constant into the ds_read offset field instead of materialising one address per read.
__device__ __forceinline__ unsigned lds_base(int off) { return (unsigned)off & 0x3ffffu; }
// typed LDS load at a sign-bit-clear byte address + IMM (the constant folds into the offset field)
template <typename T, int IMM>
__device__ __forceinline__ T lds_ld(int off) {
  typedef __attribute__((address_space(3))) T lds_T;
  return *(const lds_T*)(size_t)(lds_base(off) + IMM);
}
template <int IMM>
__device__ __forceinline__ bf16x8 lds_ld128(int off) {
  return *(const lds_bf16x8*)(size_t)(lds_base(off) + IMM);
}
template <int TR, int R0, int KS, int BUF>
__device__ __forceinline__ bf16x8 row_frag_c(const ImgOffsets& o) {
  return lds_ld128<BUF + (KS >> 3) * TR * 256 + R0 * 256>(o.roff[KS & 7]);
}
template <int TR, int RR0, int KB0, int BUF>
__device__ __forceinline__ bf16x8 tr_frag_c(const ImgOffsets& o) {
  constexpr int IMM = BUF + RR0 * 256 + (KB0 >> 7) * TR * 256;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)(size_t)(lds_base(o.troff[(KB0 & 127) / 32][0]) + IMM));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)(size_t)(lds_base(o.troff[(KB0 & 127) / 32][1]) + IMM));
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

// LDS-DMA with a scalar global base and a per-lane 32-bit byte offset (saddr form).  The M0 write →
// LDS-DMA pair needs one wait state (s_nop 0).  hipcc may produce sbase with v_readfirstlane (a VALU
// SGPR write, 5 wait states before a VMEM reads it): the first piece after sbase changes opens
// with s_nop 4 (FRESH), later pieces of the same base are far enough behind it.
template <bool FRESH = true>
__device__ __forceinline__ void dma16_s(const void* sbase, unsigned voff, unsigned lds_dst) {
  if constexpr (FRESH)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:0"
                 ::"s"(lds_dst), "v"(voff), "s"(sbase) : "memory");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:0"
                 ::"s"(lds_dst), "v"(voff), "s"(sbase) : "memory");
}

// 64 consecutive 4-byte values (a padded per-row / per-column constant array) → LDS, by wave `wv`
__device__ __forceinline__ void dma_vec64(const void* __restrict__ src, void* dst, int wv) {
  if ((threadIdx.x >> 6) == wv) dma4((const char*)src + 4 * (threadIdx.x & 63), dst);
}

// XOR swizzle of the 16-byte chunks of a 256-byte image row for the 16x16x32 operand layouts (ce3.hip,
// rgemm.hip rg3): chunk ch of row r sits at r·256 + 16·(ch ^ swz16(r)), swz16(r) = ((r&3)<<2) | h((r>>2)&3),
// h = [0,2,3,1] — conflict-free for row fragments (lane ↔ row l%16, chunk 4c + l/16: each LDS cycle's 16 lanes
// are 16 distinct rows of two adjacent chunk groups) and for transposed fragments (rows 4g + (l%16)/4, two
// chunks per 16-column block).
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | ((0x78 >> (2 * ((row >> 2) & 3))) & 3); }

__device__ __forceinline__ int creg(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// raw v_exp_f32 (2^x; no denormal range handling — results below 2^-126 flush to 0)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

}  // namespace c2img
