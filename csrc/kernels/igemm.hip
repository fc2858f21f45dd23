// Implicit-GEMM engine on gfx950 bf16 MFMA (v_mfma_f32_32x32x16_bf16).
//
// One templated main loop serves every matmul-shaped op of the training step:
//   conv fwd   Y[p][co]   = sum_k im2col(X)[p][k] * W[co][k]          (A: KC gather, B: KC)
//   conv dgrad dX[q][ci]  = sum_k col(dY)[q][k] * W^T[k][ci]          (A: KC gather, B: MC)
//   conv wgrad dW[co][kk] = sum_p dY[p][co]^T * im2col(X)[p][kk]      (A: MC,        B: MC gather)
//   linear fwd/dgrad/wgrad (plain matrices in the three layouts)
// Activations are NHWC so the channel axis is the contiguous one: every operand is
// either K-contiguous ("KC": tile stored [mn][k], read with ds_read_b128) or
// MN-contiguous ("MC": tile stored [k][mn], read transposed with ds_read_b64_tr_b16).
//
// Block: 256 threads = 4 waves, each wave owns a 64x64 output sub-tile (2x2 MFMA
// 32x32 tiles); block tile BMxBN in {128x128, 256x64, 64x256} so narrow layers (64
// channels) do not waste half the MFMA work.  K-step 64, register-staged
// double-buffered LDS, one barrier per K-tile, XOR-swizzled LDS images
// (conflict-free b128 row reads and tr_b16 column reads), bijective XCD remap +
// grouped tile order for L2 reuse.  All index decompositions use precomputed
// multiply-shift division (FastDiv) instead of runtime integer division.
//
// Strided dgrad: output rows are ordered by stride-parity class (all pixels with
// hi%S==ph, wi%S==pw together) so a block belongs to ONE class, and every K-tile (one
// filter tap when Co%64==0) whose tap cannot reach that class is skipped: no MFMA
// work is spent on the structurally-zero taps of a stride-2 transpose conv.
//
// Epilogues: bf16 store through an LDS-staged 16 B/lane write (+ fused per-channel BN
// sum / sum-of-squares, spread over NSTAT copies to avoid same-address atomic
// contention), fp32 atomic add (split-K weight gradients), fp32 store (+bias).
#include "common.h"
#include "convgeom.h"
#include <stdlib.h>
#include <map>
#include <mutex>
#include <vector>
#include <algorithm>
#include <cstdio>

namespace igemm {

constexpr int BK = 64, NTHR = 256;


// ---------------------------------------------------------------- LDS images
// KC image: [rows][64 k] bf16, 128 B rows, 16 B chunk c of row r stored at
// chunk c ^ ((r>>1)&7): the 16-lane groups of ds_read_b128 hit 16 distinct slots.
__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// MC image: [64 k][R mn] bf16 (R*2-byte rows); each 32-lane half of a tr_b16 read
// (4 k-rows x 64 B) covers 16 distinct 16 B slots of the 256 B bank row.
template <int R>
__device__ __forceinline__ int mc_off(int k, int c) {
  if (R == 64) return k * 128 + ((c ^ (((k >> 1) & 1) << 2)) << 4);
  return k * (R * 2) + ((c ^ ((k & 3) << 2)) << 4);
}

// write a loader's R/32 register chunks into its LDS image
template <class L, int R>
__device__ __forceinline__ void store_stage(char* lds, int tid, const uint4 (&v)[R / 32]) {
#pragma unroll
  for (int i = 0; i < R / 32; ++i) *reinterpret_cast<uint4*>(lds + L::lds_off(i, tid)) = v[i];
}

// fragment of a 32-row (KC) / 32-col (MC) sub-tile for k-step s (16 deep)
template <bool KC, int R>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int base, int s, int lane) {
  if (KC) {
    const int r = base + (lane & 31), c = 2 * s + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(lds + kc_off(r, c));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m0 = base + 16 * (g & 1), k0 = 16 * s + 8 * (g >> 1);
    const int col = m0 + 4 * p;
    const int a0 = mc_off<R>(k0 + q, col >> 3) + (col & 7) * 2;
    const int a1 = mc_off<R>(k0 + 4 + q, col >> 3) + (col & 7) * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// ---------------------------------------------------------------- buffer loads
// Every operand load is a branch-free raw buffer load: the per-thread 32-bit voffset is
// precomputed (relative to a wave-uniform base that moves per block / K-tile), and a
// load that must read zero (padding tap, row past M, K tail) gets voffset OOB, past
// num_records, so the hardware returns 0.  No exec-mask branches around loads means the
// compiler sees a fixed number of loads per K-tile and can wait with counted vmcnt
// instead of draining all of them, which is what lets loads stay in flight across the
// MFMA phase (two tiles deep with PF=2).
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr unsigned OOB = 0x80000000u;
__device__ __forceinline__ Rsrc rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ uint4 bload(Rsrc r, unsigned voff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
// LDS-DMA (buffer_load ... lds): 16 B per lane straight into LDS, lane-linear from the
// wave-uniform destination `dst` (no VGPR round trip and no ds_write); an OOB voffset
// writes zeros.  The KC images below are filled this way by the DMA main loop (PF = 3):
// lane l of wave w, copy i, lands in image row w*8 + (l>>3) + 32i at slot l&7, so the
// XOR swizzle moves to the source side - the lane fetches logical chunk (l&7) ^ swz(row),
// and swz(row) = (tid>>4)&7 for every copy i.
__device__ __forceinline__ void dma16(Rsrc rs, char* dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ int dma_chunk(int tid) { return (tid & 7) ^ ((tid >> 4) & 7); }
__device__ __forceinline__ char* dma_dst(char* img, int tid) {
  return img + __builtin_amdgcn_readfirstlane(tid >> 6) * 1024;
}
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// ---------------------------------------------------------------- loaders
// Thread -> 16 B chunk mapping (chunk i of R/32 per thread), unless a loader overrides
// lds_off: KC tile of R rows: row (t>>3)+32i, chunk t&7 (8 k per chunk); MC tile of R
// cols: chunk t%(R/8) (8 mn), k-row t/(R/8) + (256/(R/8))i.  Loaders take the K-tile
// index kt (k0 = kt*BK).

template <int R>
struct MatKC {  // [rows][K] row-major, ld elements per row
  static constexpr bool KC = true;
  const bf16* p; int ld, rows, K;
  struct St { unsigned off[R / 32]; int m0; };
  __device__ static int lds_off(int i, int tid) { return kc_off((tid >> 3) + 32 * i, tid & 7); }
  __device__ void init(St& st, int m0, int tid) const {
    st.m0 = m0;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int r = (tid >> 3) + 32 * i;
      st.off[i] = m0 + r < rows ? (unsigned)(r * ld + (tid & 7) * 8) * 2u : OOB;
    }
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int k0 = kt * BK;
    const Rsrc rs = rsrc(p + (size_t)st.m0 * ld + k0);
    const bool kv = (tid & 7) * 8 < K - k0;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bload(rs, kv ? st.off[i] : OOB);
  }
  static constexpr bool DMA = true;
  __device__ void dma(const St& st, int kt, int tid, char* img) const {
    const int k0 = kt * BK, ch = dma_chunk(tid);
    const Rsrc rs = rsrc(p + (size_t)st.m0 * ld + k0);
    const bool kv = ch * 8 < K - k0;
    const unsigned delta = (unsigned)((ch - (tid & 7)) * 16);
    char* dst = dma_dst(img, tid);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) dma16(rs, dst + i * 4096, kv && st.off[i] != OOB ? st.off[i] + delta : OOB);
  }
};

template <int R>
struct MatMC {  // [K][cols] row-major, ld elements per row
  static constexpr bool KC = false;
  const bf16* p; int ld, K, cols;
  struct St { unsigned off[R / 32]; int n0; };
  __device__ static int kr(int i, int tid) { return tid / (R / 8) + (NTHR / (R / 8)) * i; }
  __device__ static int lds_off(int i, int tid) { return mc_off<R>(kr(i, tid), tid % (R / 8)); }
  __device__ void init(St& st, int n0, int tid) const {
    st.n0 = n0;
    const int c = (tid % (R / 8)) * 8;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) st.off[i] = n0 + c < cols ? (unsigned)(kr(i, tid) * ld + c) * 2u : OOB;
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int k0 = kt * BK;
    const Rsrc rs = rsrc(p + (size_t)k0 * ld + st.n0);
    const int left = K - k0;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bload(rs, kr(i, tid) < left ? st.off[i] : OOB);
  }
  // LDS-DMA: copy i of wave w covers k-rows kr(i, tid) lane-linearly (1 KiB = 8 / 4 / 2
  // k-rows of 64 / 128 / 256 columns), so lane l lands in slot tid % (R/8) of its k-row
  // and fetches the logical chunk that mc_off puts there (the XOR is an involution).
  // Correct (GPU tests) but measured slower than the register-staged copy on the weight
  // gradients (ResNet-50 wgrads 5.25 -> 5.43 ms, BERT-base -3.5 %), so not enabled.
  static constexpr bool DMA = false;
  __device__ void dma(const St& st, int kt, int tid, char* img) const {
    const int k0 = kt * BK, left = K - k0;
    const int slot = tid % (R / 8), k = tid / (R / 8);
    const int ch = R == 64 ? slot ^ (((k >> 1) & 1) << 2) : slot ^ ((k & 3) << 2);
    const bool cv = st.n0 + ch * 8 < cols;
    const Rsrc rs = rsrc(p + (size_t)k0 * ld + st.n0);
    char* dst = dma_dst(img, tid);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int r = kr(i, tid);
      dma16(rs, dst + i * 4096, cv && r < left ? (unsigned)(r * ld + ch * 8) * 2u : OOB);
    }
  }
};

// MatMC that also sums every column over the K rows it stages (A operand of a dense
// weight gradient dW = dY^T X: the column sums of dY are the bias gradient).  The sums are
// taken from the staged registers (after the loads landed, only for real K-tiles) and
// flushed by the N-tile-0 blocks with one fp32 atomic per column per wave.
template <int R>
struct MatMCSum {
  static constexpr bool KC = false, SUM = true;
  const bf16* p; int ld, K, cols; float* colsum;
  struct St { typename MatMC<R>::St b; float s[8]; };
  __device__ MatMC<R> base() const { return MatMC<R>{p, ld, K, cols}; }
  __device__ static int lds_off(int i, int tid) { return MatMC<R>::lds_off(i, tid); }
  __device__ void init(St& st, int n0, int tid) const {
    base().init(st.b, n0, tid);
#pragma unroll
    for (int e = 0; e < 8; ++e) st.s[e] = 0.f;
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const { base().load(st.b, kt, tid, v); }
  __device__ void accum(St& st, const uint4 (&v)[R / 32]) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) st.s[e] += f[e];
    }
  }
  // the 4 waves' partial sums of a column are combined in a fixed order through LDS and
  // added with ONE atomic per column per block (with one K-split that single add onto
  // the zeroed gradient is exact, so deterministic mode gets reproducible bias grads)
  __device__ void finish(St& st, bool owner, int tid, char* lds) const {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int o = R / 8; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) st.s[e] += __shfl_xor(st.s[e], o, 64);
    float* red = reinterpret_cast<float*>(lds);   // [NTHR/64 waves][R/8 lanes][8]
    if (owner && lane < R / 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(wave * (R / 8) + lane) * 8 + e] = st.s[e];
    }
    __syncthreads();
    const int c = st.b.n0 + 8 * lane;
    if (owner && wave == 0 && lane < R / 8 && c < cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < NTHR / 64; ++w) a += red[(w * (R / 8) + lane) * 8 + e];
        atomicAdd(colsum + c + e, a);
      }
    }
    __syncthreads();   // the epilogue reuses the LDS
  }
};
template <class L, class = void> struct HasSum { static constexpr bool value = false; };
template <class L> struct HasSum<L, decltype((void)L::SUM)> { static constexpr bool value = L::SUM; };


// conv fwd A operand: rows = output pixels (n, ho, wo), k = (r, s, ci), ci fastest.
// Row offsets are relative to the block's first row; the tap offset is per chunk.
template <int R>
struct ConvFwdA {
  static constexpr bool KC = true;
  const bf16* x; ConvGeom g; int M, K;
  struct St { unsigned off[R / 32], msk[R / 32]; long long b0; };
  __device__ static int lds_off(int i, int tid) { return kc_off((tid >> 3) + 32 * i, tid & 7); }
  __device__ long long rowoff(int m, int& hb, int& wb) const {
    unsigned t, wo, n, ho;
    g.fWo.divmod((unsigned)m, t, wo);
    g.fHo.divmod(t, n, ho);
    hb = (int)ho * g.stride - g.pad;
    wb = (int)wo * g.stride - g.padw;
    return (((long long)n * g.H + hb) * g.W + wb) * g.C;
  }
  __device__ void init(St& st, int m0, int tid) const {
    int hb, wb;
    st.b0 = rowoff(m0, hb, wb);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      const bool ok = m < M;
      const long long o = rowoff(ok ? m : m0, hb, wb);
      st.off[i] = (unsigned)(o - st.b0) * 2u;
      unsigned mk = 0;
      for (int r = 0; r < g.KH; ++r) mk |= ((unsigned)(hb + r * g.dil) < (unsigned)g.H) ? (1u << r) : 0u;
      for (int s = 0; s < g.KW; ++s) mk |= ((unsigned)(wb + s * g.dil) < (unsigned)g.W) ? (1u << (16 + s)) : 0u;
      st.msk[i] = ok ? mk : 0u;
    }
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int k0 = kt * BK, k = k0 + (tid & 7) * 8;
    unsigned rs_, cc, rr, ss;
    if (g.C % BK == 0) {  // whole K-tile = one tap (uniform decomposition)
      g.fC.divmod((unsigned)k0, rs_, cc);
      cc += (unsigned)(k - k0);
    } else {
      g.fC.divmod((unsigned)k, rs_, cc);
    }
    g.fKW.divmod(rs_, rr, ss);
    const unsigned P = k < K ? tap_pat((int)rr, (int)ss) : NO_TAP;
    const unsigned toff = (unsigned)(((int)rr * g.dil * g.W + (int)ss * g.dil) * g.C + (int)cc) * 2u;
    const Rsrc rsr = rsrc(x + st.b0);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bload(rsr, (st.msk[i] & P) == P ? st.off[i] + toff : OOB);
  }
  static constexpr bool DMA = true;
  __device__ void dma(const St& st, int kt, int tid, char* img) const {
    const int k0 = kt * BK, k = k0 + dma_chunk(tid) * 8;
    unsigned rs_, cc, rr, ss;
    if (g.C % BK == 0) {
      g.fC.divmod((unsigned)k0, rs_, cc);
      cc += (unsigned)(k - k0);
    } else {
      g.fC.divmod((unsigned)k, rs_, cc);
    }
    g.fKW.divmod(rs_, rr, ss);
    const unsigned P = k < K ? tap_pat((int)rr, (int)ss) : NO_TAP;
    const unsigned toff = (unsigned)(((int)rr * g.dil * g.W + (int)ss * g.dil) * g.C + (int)cc) * 2u;
    const Rsrc rsr = rsrc(x + st.b0);
    char* dst = dma_dst(img, tid);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) dma16(rsr, dst + i * 4096, (st.msk[i] & P) == P ? st.off[i] + toff : OOB);
  }
};


template <int R>
struct ConvDgradA {  // rows = class pixels, k = (a, b, co)
  static constexpr bool KC = true;
  const bf16* dy; ConvGeom g; int M, K; DgradClass cl;
  struct St { unsigned off[R / 32], msk[R / 32]; long long b0; };
  __device__ static int lds_off(int i, int tid) { return kc_off((tid >> 3) + 32 * i, tid & 7); }
  __device__ long long rowoff(int m, int& i, int& j) const {
    int n;
    cl.decode(m, n, i, j);
    return (((long long)n * g.Ho + i) * g.Wo + j) * g.Co;
  }
  __device__ void init(St& st, int m0, int tid) const {
    int i0, j0;
    st.b0 = rowoff(m0, i0, j0) + cl.tmin;
#pragma unroll
    for (int u = 0; u < R / 32; ++u) {
      const int m = m0 + (tid >> 3) + 32 * u;
      const bool ok = m < M;
      int i, j;
      const long long o = rowoff(ok ? m : m0, i, j);
      st.off[u] = (unsigned)(o + cl.tmin - st.b0) * 2u;
      unsigned mk = 0;
      for (int a = 0; a < cl.nr; ++a) mk |= ((unsigned)(i + cl.dh0 - a * cl.dhs) < (unsigned)g.Ho) ? (1u << a) : 0u;
      for (int b = 0; b < cl.ns; ++b) mk |= ((unsigned)(j + cl.dw0 - b * cl.dws) < (unsigned)g.Wo) ? (1u << (16 + b)) : 0u;
      st.msk[u] = ok ? mk : 0u;
    }
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    int a, b, co0;
    cl.tap(kt, a, b, co0);
    const int co = co0 + (tid & 7) * 8;
    const unsigned P = co < g.Co ? tap_pat(a, b) : NO_TAP;
    const long long toff = ((long long)(cl.dh0 - a * cl.dhs) * g.Wo + (cl.dw0 - b * cl.dws)) * g.Co + co - cl.tmin;
    const unsigned t2 = (unsigned)toff * 2u;
    const Rsrc rsr = rsrc(dy + st.b0);
#pragma unroll
    for (int u = 0; u < R / 32; ++u) v[u] = bload(rsr, (st.msk[u] & P) == P ? st.off[u] + t2 : OOB);
  }
  static constexpr bool DMA = true;
  __device__ void dma(const St& st, int kt, int tid, char* img) const {
    int a, b, co0;
    cl.tap(kt, a, b, co0);
    const int co = co0 + dma_chunk(tid) * 8;
    const unsigned P = co < g.Co ? tap_pat(a, b) : NO_TAP;
    const long long toff = ((long long)(cl.dh0 - a * cl.dhs) * g.Wo + (cl.dw0 - b * cl.dws)) * g.Co + co - cl.tmin;
    const unsigned t2 = (unsigned)toff * 2u;
    const Rsrc rsr = rsrc(dy + st.b0);
    char* dst = dma_dst(img, tid);
#pragma unroll
    for (int u = 0; u < R / 32; ++u) dma16(rsr, dst + u * 4096, (st.msk[u] & P) == P ? st.off[u] + t2 : OOB);
  }
};

// conv dgrad B operand: k = (a, b, co) rows, cols = ci; W stored [co][r][s][ci]
template <int R>
struct ConvDgradB {
  static constexpr bool KC = false;
  const bf16* w; ConvGeom g; DgradClass cl;
  struct St { unsigned off[R / 32]; int n0; };
  __device__ static int kr(int i, int tid) { return tid / (R / 8) + (NTHR / (R / 8)) * i; }
  __device__ static int lds_off(int i, int tid) { return mc_off<R>(kr(i, tid), tid % (R / 8)); }
  __device__ void init(St& st, int n0, int tid) const {
    st.n0 = n0;
    const int c = (tid % (R / 8)) * 8;
    const int T = g.KH * g.KW;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) st.off[i] = n0 + c < g.C ? (unsigned)(kr(i, tid) * T * g.C + c) * 2u : OOB;
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    int a, b, co0;
    cl.tap(kt, a, b, co0);
    const int r = cl.r0 + a * cl.rstep, s = cl.s0 + b * cl.sstep;
    const Rsrc rsr = rsrc(w + (((size_t)co0 * g.KH + r) * g.KW + s) * g.C + st.n0);
    const int left = g.Co - co0;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bload(rsr, kr(i, tid) < left ? st.off[i] : OOB);
  }
};

// conv dgrad B operand from the transposed, flipped filter wt[C][KH][KW][Co]
// (wtrans.hip): rows = ci, k = (a, b, co) as in ConvDgradB, but K-contiguous - the tap
// (r, s) of W is tap (KH-1-r, KW-1-s) of wt, and its Co channels are one contiguous run.
template <int R>
struct ConvDgradBT {
  static constexpr bool KC = true;
  const bf16* wt; ConvGeom g; DgradClass cl;
  struct St { unsigned off[R / 32]; int n0; };
  __device__ static int lds_off(int i, int tid) { return kc_off((tid >> 3) + 32 * i, tid & 7); }
  __device__ void init(St& st, int n0, int tid) const {
    st.n0 = n0;
    const int rl = g.KH * g.KW * g.Co;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int r = (tid >> 3) + 32 * i;
      st.off[i] = n0 + r < g.C ? (unsigned)(r * rl + (tid & 7) * 8) * 2u : OOB;
    }
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    int a, b, co0;
    cl.tap(kt, a, b, co0);
    const int r = cl.r0 + a * cl.rstep, s = cl.s0 + b * cl.sstep;
    const int tf = (g.KH - 1 - r) * g.KW + (g.KW - 1 - s);
    const Rsrc rs = rsrc(wt + (size_t)st.n0 * g.KH * g.KW * g.Co + (size_t)tf * g.Co + co0);
    const bool kv = co0 + (tid & 7) * 8 < g.Co;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bload(rs, kv ? st.off[i] : OOB);
  }
  static constexpr bool DMA = true;
  __device__ void dma(const St& st, int kt, int tid, char* img) const {
    int a, b, co0;
    cl.tap(kt, a, b, co0);
    const int r = cl.r0 + a * cl.rstep, s = cl.s0 + b * cl.sstep;
    const int tf = (g.KH - 1 - r) * g.KW + (g.KW - 1 - s);
    const Rsrc rs = rsrc(wt + (size_t)st.n0 * g.KH * g.KW * g.Co + (size_t)tf * g.Co + co0);
    const int ch = dma_chunk(tid);
    const bool kv = co0 + ch * 8 < g.Co;
    const unsigned delta = (unsigned)((ch - (tid & 7)) * 16);
    char* dst = dma_dst(img, tid);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) dma16(rs, dst + i * 4096, kv && st.off[i] != OOB ? st.off[i] + delta : OOB);
  }
};

// conv wgrad B operand: k = output pixel p rows, cols = kk = (r, s, ci).  Thread t loads
// pixels (t>>3) and (t>>3)+32 of the K-tile and column chunks (t&7)+8c (c < R/64): two
// pixel decompositions per thread and K-tile, shared by its column chunks.
template <int R>
struct ConvWgradB {
  static constexpr bool KC = false;
  static constexpr int NC = R / 64;
  const bf16* x; ConvGeom g; int P, KK;
  struct St { unsigned coff[NC]; int rd[NC], sd[NC]; unsigned ci[NC]; };
  __device__ static int lds_off(int i, int tid) {
    return mc_off<R>((tid >> 3) + 32 * (i & 1), (tid & 7) + 8 * (i >> 1));
  }
  __device__ void init(St& st, int n0, int tid) const {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int kk = n0 + ((tid & 7) + 8 * c) * 8;
      unsigned rs_, ci, r, s;
      g.fC.divmod((unsigned)(kk < KK ? kk : 0), rs_, ci);
      g.fKW.divmod(rs_, r, s);
      st.ci[c] = ci;
      st.coff[c] = (unsigned)(((int)r * g.dil * g.W + (int)s * g.dil) * g.C + (int)ci) * 2u;
      st.rd[c] = kk < KK ? (int)r * g.dil : (1 << 28);   // an invalid column never passes the bounds test
      st.sd[c] = (int)s * g.dil;
    }
  }
  __device__ void load(const St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int p0 = kt * BK;
    unsigned t, w0, n0, h0;
    g.fWo.divmod((unsigned)p0, t, w0);
    g.fHo.divmod(t, n0, h0);
    const long long b0 = (((long long)n0 * g.H + (int)h0 * g.stride - g.pad) * g.W + (int)w0 * g.stride - g.padw) * g.C;
    const Rsrc rsr = rsrc(x + b0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kr = (tid >> 3) + 32 * j;
      unsigned cw, wo, ch, ho;
      g.fWo.divmod(w0 + (unsigned)kr, cw, wo);
      g.fHo.divmod(h0 + cw, ch, ho);
      const int hb = p0 + kr < P ? (int)ho * g.stride - g.pad : -(1 << 29);
      const int wb = (int)wo * g.stride - g.padw;
      const unsigned rel = (unsigned)((((int)ch * g.H + ((int)ho - (int)h0) * g.stride) * g.W +
                                       ((int)wo - (int)w0) * g.stride) * g.C) * 2u;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bool ok = (unsigned)(hb + st.rd[c]) < (unsigned)g.H && (unsigned)(wb + st.sd[c]) < (unsigned)g.W;
        v[2 * c + j] = bload(rsr, ok ? rel + st.coff[c] : OOB);
      }
    }
  }
};

// ---------------------------------------------------------------- BN-apply operand transform
// A conv whose input is the output z = relu(y*sc + sh) of a BatchNorm can read the pre-BN
// tensor y instead: the transform is applied per channel while the staged registers go to
// LDS (after the loads landed), and chunks that stand for padding taps / rows past M /
// k past K stay zero (the transform of a zero is not zero).  Forward: units 2 and 3 of a
// bottleneck read y1 / y2, so z1 / z2 are never written; backward: the weight gradients
// of those convs re-apply it to their activation operand.
struct BnIn { const float* sc; const float* sh; };
template <class L, class = void> struct HasXform { static constexpr bool value = false; };
template <class L> struct HasXform<L, decltype((void)L::XF)> { static constexpr bool value = L::XF; };
// loaders that can fill their KC image by LDS-DMA (no register transform)
template <class L, class = void> struct HasDma { static constexpr bool value = false; };
template <class L> struct HasDma<L, decltype((void)L::DMA)> {
  static constexpr bool value = L::DMA && !HasXform<L>::value && !HasSum<L>::value;
};

__device__ __forceinline__ uint4 bn_relu8(uint4 v, const float* a, const float* b, bool ok) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e] * a[e] + b[e], 0.f);
  const uint4 r = pack8(f);
  return ok ? r : make_uint4(0u, 0u, 0u, 0u);
}

// plain [rows][K] activation (1x1 conv A operand): channel = k
template <int R>
struct MatKCBn : MatKC<R> {
  static constexpr bool XF = true;
  BnIn bn;
  __device__ void xform(const typename MatKC<R>::St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int c0 = kt * BK + (tid & 7) * 8;
    const bool kv = c0 < this->K;
    float a[8], b[8];
    ldg8f(bn.sc + (kv ? c0 : 0), a);
    ldg8f(bn.sh + (kv ? c0 : 0), b);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bn_relu8(v[i], a, b, kv && st.off[i] != OOB);
  }
};

// implicit-GEMM conv forward A operand: channel = ci of the chunk's tap
template <int R>
struct ConvFwdABn : ConvFwdA<R> {
  static constexpr bool XF = true;
  BnIn bn;
  __device__ void xform(const typename ConvFwdA<R>::St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const ConvGeom& g = this->g;
    const int k0 = kt * BK, k = k0 + (tid & 7) * 8;
    unsigned rs_, cc, rr, ss;
    if (g.C % BK == 0) {
      g.fC.divmod((unsigned)k0, rs_, cc);
      cc += (unsigned)(k - k0);
    } else {
      g.fC.divmod((unsigned)k, rs_, cc);
    }
    g.fKW.divmod(rs_, rr, ss);
    const bool kv = k < this->K;
    const unsigned P = kv ? tap_pat((int)rr, (int)ss) : NO_TAP;
    float a[8], b[8];
    ldg8f(bn.sc + (kv ? cc : 0), a);
    ldg8f(bn.sh + (kv ? cc : 0), b);
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bn_relu8(v[i], a, b, (st.msk[i] & P) == P);
  }
};

// 1x1 weight-gradient B operand x [P][C] (k = pixel rows, columns = channels)
template <int R>
struct MatMCBn : MatMC<R> {
  static constexpr bool XF = true;
  BnIn bn;
  __device__ void xform(const typename MatMC<R>::St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    const int c0 = st.n0 + (tid % (R / 8)) * 8;
    const bool cv = c0 < this->cols;
    float a[8], b[8];
    ldg8f(bn.sc + (cv ? c0 : 0), a);
    ldg8f(bn.sh + (cv ? c0 : 0), b);
    const int left = this->K - kt * BK;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) v[i] = bn_relu8(v[i], a, b, cv && MatMC<R>::kr(i, tid) < left);
  }
};

// gathered weight-gradient B operand (3x3 ...): same bounds test as ConvWgradB::load
template <int R>
struct ConvWgradBBn : ConvWgradB<R> {
  static constexpr bool XF = true;
  BnIn bn;
  __device__ void xform(const typename ConvWgradB<R>::St& st, int kt, int tid, uint4 (&v)[R / 32]) const {
    constexpr int NC = ConvWgradB<R>::NC;
    const ConvGeom& g = this->g;
    const int p0 = kt * BK;
    unsigned t, w0, n0, h0;
    g.fWo.divmod((unsigned)p0, t, w0);
    g.fHo.divmod(t, n0, h0);
    int hb[2], wb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kr = (tid >> 3) + 32 * j;
      unsigned cw, wo, ch, ho;
      g.fWo.divmod(w0 + (unsigned)kr, cw, wo);
      g.fHo.divmod(h0 + cw, ch, ho);
      hb[j] = p0 + kr < this->P ? (int)ho * g.stride - g.pad : -(1 << 29);
      wb[j] = (int)wo * g.stride - g.padw;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float a[8], b[8];
      ldg8f(bn.sc + st.ci[c], a);
      ldg8f(bn.sh + st.ci[c], b);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = (unsigned)(hb[j] + st.rd[c]) < (unsigned)g.H && (unsigned)(wb[j] + st.sd[c]) < (unsigned)g.W;
        v[2 * c + j] = bn_relu8(v[2 * c + j], a, b, ok);
      }
    }
  }
};

// ---------------------------------------------------------------- epilogues
// acc[i][j][reg] of wave (wm, wn) holds C[m][n] with
//   m = wm*64 + 32i + (reg&3) + 8(reg>>2) + 4(lane>>5),  n = wn*64 + 32j + (lane&31)

struct IdentityRows {
  __device__ __forceinline__ size_t operator()(int m) const { return (size_t)m; }
};
struct ClassRows {  // dgrad class row (n, i, j) -> NHWC pixel (n, i*S+ph, j*S+pw)
  DgradClass c; int H, W;
  __device__ __forceinline__ size_t operator()(int m) const {
    int n, i, j;
    c.decode(m, n, i, j);
    return ((size_t)n * H + i * c.S + c.ph) * W + j * c.S + c.pw;
  }
};

// BatchNorm-backward reduction fused into the epilogue of the dgrad that produces the
// final gradient dU of a BN's output (the branch-point sum is already in via addend):
//   dU <- dU * [mask > 0]   (ReLU of the BN being differentiated; mask = its output z)
//   sums_k[slot][0][c] += sum dU,  sums_k[slot][1][c] += sum dU*(y_k - mean_k)
// for up to two BNs sharing the same dU (a block's last BN and its downsample BN).  The
// masked dU is what gets stored, so the elementwise BN-backward pass needs neither z
// nor a separate residual-gradient copy.
// Without a mask tensor the ReLU mask can be recomputed from the pre-BN values the
// reduction reads anyway: [y0*msc0 + msh0 (+ y1*msc1 + msh1) > 0] with the forward's
// (scale, shift) -- exactly the forward's z > 0 -- so z is not read at all.
struct BnBwdEpi {
  const bf16* mask = nullptr;
  const bf16* y0 = nullptr; const float* mean0 = nullptr; float* sums0 = nullptr;
  const bf16* y1 = nullptr; const float* mean1 = nullptr; float* sums1 = nullptr;
  const float* msc0 = nullptr; const float* msh0 = nullptr;
  const float* msc1 = nullptr; const float* msh1 = nullptr;
  int ncopy = NSTAT;   // copies of sums0/sums1 (g_mlc_ncopy at launch)
};

// Dense-layer activation of 8 consecutive outputs.  act & 3: 0 none, 1 exact-erf GELU with
// the pre-activation u stored to `pre`, 2 GELU with its DERIVATIVE gelu'(u) stored to `pre`
// instead (the forward has erf(u) at hand, so the backward then only multiplies: no erf /
// exp in the input-gradient epilogue, which cost BERT-base's FFN dgrad ~40 % of its time).
// erf(x) given e = exp(-x*x) (Abramowitz-Stegun 7.1.26, |error| <= 1.5e-7): one reciprocal
// and five FMAs, and the exponential is the one gelu'(u) = cdf + u*phi(u) needs anyway
// (phi(u) = exp(-u*u/2)/sqrt(2 pi), x = u/sqrt(2)).  The device-library erff costs ~3x more
// VALU, which the GELU epilogue of BERT's FFN1 (512 tiles, one round on 256 CUs) pays in
// full after the main loop.  The error is ~1e-6 after fp32 rounding, far under a bf16 ulp.
__device__ __forceinline__ float erf_from_exp(float x, float e) {
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * fabsf(x));
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  return copysignf(1.f - p * e, x);
}

__device__ __forceinline__ void dense_act8(float (&a)[8], int act, bf16* pre) {
  const int mode = act & 3;
  if (mode == 3) {   // ReLU (generic engine: conv / linear + bias + ReLU)
    if (pre) *reinterpret_cast<uint4*>(pre) = pack8(a);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = fmaxf(a[e], 0.f);
    return;
  }
  if (mode == 2) {
    float d[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float u = a[e];
      const float ex = __expf(-0.5f * u * u);
      const float cdf = 0.5f * (1.f + erf_from_exp(u * 0.70710678118654752f, ex));
      d[e] = cdf + u * 0.3989422804014327f * ex;
      a[e] = u * cdf;
    }
    if (pre) *reinterpret_cast<uint4*>(pre) = pack8(d);
    return;
  }
  if (pre) *reinterpret_cast<uint4*>(pre) = pack8(a);
  if (mode == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      a[e] = 0.5f * a[e] * (1.f + erf_from_exp(a[e] * 0.70710678118654752f, __expf(-0.5f * a[e] * a[e])));
  }
}
// backward of the activation: a *= gelu'(z) for z the stored pre-activation, or a *= z when
// z already holds the derivative (act & 4, written by dense_act8 mode 2); act 3: ReLU mask
__device__ __forceinline__ void dense_dact8(float (&a)[8], int act, uint4 zv) {
  float z[8];
  unpack8(zv, z);
  if (act & 4) {
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] *= z[e];
    return;
  }
  if ((act & 3) == 3) {   // ReLU: z is the pre-activation or the output, either gives the mask
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float ex = __expf(-0.5f * z[e] * z[e]);
    const float cdf = 0.5f * (1.f + erf_from_exp(z[e] * 0.70710678118654752f, ex));
    a[e] *= cdf + z[e] * 0.3989422804014327f * ex;
  }
}

template <class RowMap = IdentityRows, bool kDense = false>
struct EpiBF16 {  // bf16 [M][ld] store (+ addend), optional per-column sum / sum of squares
  bf16* out; int ld; float* sum; float* sumsq; RowMap rowmap; const bf16* addend = nullptr;
  BnBwdEpi bn = {};
  // dense-layer extras: out = act(acc + bias) (pre-activation, or with act 2 the
  // activation's derivative, stored to preact), or out = acc * act'(dact) for the backward
  // of an activation (act 1/2 = exact-erf GELU; act 4: dact holds the derivative)
  const float* bias = nullptr; int act = 0; bf16* preact = nullptr; const bf16* dact = nullptr;
  int ncopy = NSTAT;   // copies of sum / sumsq (g_mlc_ncopy at launch)
  // the persistent kernel runs this epilogue while the next tile's LDS-DMA copies are in
  // flight: its barriers must then be raw s_barriers (a full barrier would wait vmcnt(0))
  bool raw_sync = false;
  __device__ __forceinline__ void esync() const {
    if (raw_sync) lds_barrier();
    else __syncthreads();
  }
  template <int BM, int BN, int MI, int NI>
  __device__ void apply(f32x16 (&acc)[MI][NI], char* lds, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int tid) const {
    if (sum) {
      // copy slot spreads the per-channel atomics of different blocks over NSTAT rows
      const int slot = (int)((unsigned)((m0 / 64) + wm) % (unsigned)ncopy);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) { const float v = acc[i][j][r]; s1 += v; s2 += v * v; }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        const int n = n0 + wn * 32 * NI + 32 * j + lane;
        if (lane < 32 && n < N) {
          atomicAdd(sum + (size_t)slot * N + n, s1);
          atomicAdd(sumsq + (size_t)slot * N + n, s2);
        }
      }
    }
    // stage the BMxBN tile through LDS as bf16 rows of (BN+8)*2 B, then 16 B/lane stores
    constexpr int RS = (BN + 8) * 2;
    esync();
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm * 32 * MI + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int n = wn * 32 * NI + 32 * j + (lane & 31);
          *reinterpret_cast<bf16*>(lds + m * RS + n * 2) = (bf16)acc[i][j][r];
        }
    esync();
    constexpr int CPR = BN / 8;              // 16 B chunks per row
    constexpr int RPI = NTHR / CPR;          // rows per iteration
    // three-wide tiles: CPR does not divide the block (12 / 24 / 36 chunks per row), so
    // the last NTHR % CPR threads idle and the last iteration is partial
    constexpr bool EXACT = RPI * CPR == NTHR && BM % RPI == 0;
    const bool tok = EXACT || tid < RPI * CPR;
    const int c = tid % CPR;
    const int nc = n0 + c * 8;
    const bool red = !kDense && bn.y0 != nullptr;
    float mu0[8], mu1[8], s1[8], s2[8], t2[8], ma0[8], mb0[8], ma1[8], mb1[8];
    const bool aff = red && !bn.mask && bn.msc0, aff1 = aff && bn.msc1;
    if (red) {
      // per-column constants: vector loads from a clamped (always valid) column, under
      // wave-uniform pointer tests only; columns past N are never stored
      const int ncl = nc < N ? nc : 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] = 0.f; s2[e] = 0.f; t2[e] = 0.f;
        mu1[e] = 0.f; ma0[e] = 0.f; mb0[e] = 0.f; ma1[e] = 0.f; mb1[e] = 0.f;
      }
      ldg8f(bn.mean0 + ncl, mu0);
      if (bn.y1) ldg8f(bn.mean1 + ncl, mu1);
      if (aff) { ldg8f(bn.msc0 + ncl, ma0); ldg8f(bn.msh0 + ncl, mb0); }
      if (aff1) { ldg8f(bn.msc1 + ncl, ma1); ldg8f(bn.msh1 + ncl, mb1); }
    }
    const bool dense = kDense && (bias || act || dact);
    float bz[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bz[e] = 0.f;
    if (kDense && bias) ldg8f(bias + (nc < N ? nc : 0), bz);
    constexpr int ITERS = (BM + RPI - 1) / RPI;
    if (!addend && !red && !dense) {  // plain store (forward convs / GEMMs)
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int row = tid / CPR + RPI * it;
        const int m = m0 + row;
        if ((EXACT || (tok && row < BM)) && m < M && nc < N)
          *reinterpret_cast<uint4*>(out + rowmap(m) * ld + nc) =
              *reinterpret_cast<const uint4*>(lds + row * RS + c * 16);
      }
      return;
    }
    // rows are processed U at a time: every global load of a chunk (addend, mask, y) is
    // issued before the chunk's stores, so the loads overlap instead of serialising
    // behind stores the compiler must assume alias them (out may alias addend)
    constexpr int UMAX = kDense ? 4 : 8;   // conv epilogues: every row's loads in flight at once
    constexpr int U = ITERS < UMAX ? ITERS : UMAX;
    const bool has_add = addend != nullptr, has_mask = red && bn.mask, has_y1 = red && bn.y1;
#pragma unroll 1
    for (int it0 = 0; it0 < ITERS; it0 += U) {
      constexpr int UB = kDense ? 1 : U;   // BN-reduction operands (conv dgrad only)
      constexpr int UD = kDense ? U : 1;   // activation-derivative operand (dense only)
      uint4 vv[U], aa[U], zz[UB], p0[UB], p1[UB], du[UD];
      size_t off[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int row = tid / CPR + RPI * (it0 + u);
        const bool rin = EXACT || (tok && row < BM);
        if (!rin) row = 0;                          // idle thread / past the tile: read row 0, no store
        const int m = m0 + row;
        ok[u] = rin && m < M && nc < N;
        off[u] = ok[u] ? rowmap(m) * ld + nc : 0;   // rows/cols outside: element 0 (valid)
        vv[u] = *reinterpret_cast<const uint4*>(lds + row * RS + c * 16);
        const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
        // unconditional per lane (the store is what ok[u] guards), uniform per pointer
        aa[u] = has_add ? ldg16(addend + off[u]) : zero;
        if constexpr (!kDense) {
          zz[u] = has_mask ? ldg16(bn.mask + off[u]) : zero;
          p0[u] = red ? ldg16(bn.y0 + off[u]) : zero;
          p1[u] = has_y1 ? ldg16(bn.y1 + off[u]) : zero;
        }
        if constexpr (kDense) du[u] = dact ? ldg16(dact + off[u]) : zero;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        uint4 v = vv[u];
        if (has_add || red || dense) {
          float a[8];
          unpack8(v, a);
          if constexpr (kDense) {
          if (bias) {
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += bz[e];
          }
          dense_act8(a, act, preact ? preact + off[u] : nullptr);
          if (dact) dense_dact8(a, act, du[u]);
          }
          if (has_add) {  // fused residual-gradient sum (dx of a branch point)
            float b[8];
            unpack8(aa[u], b);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += b[e];
          }
          if constexpr (!kDense) {
            if (has_mask) {
              float z[8];
              unpack8(zz[u], z);
#pragma unroll
              for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
            } else if (aff) {  // z > 0 recomputed from the pre-BN value(s)
              float y[8], q[8];
              unpack8(p0[u], y);
#pragma unroll
              for (int e = 0; e < 8; ++e) q[e] = y[e] * ma0[e] + mb0[e];
              if (aff1) {
                unpack8(p1[u], y);
#pragma unroll
                for (int e = 0; e < 8; ++e) q[e] += y[e] * ma1[e] + mb1[e];
              }
#pragma unroll
              for (int e = 0; e < 8; ++e) a[e] = q[e] > 0.f ? a[e] : 0.f;
            }
          }
          v = pack8(a);
          if constexpr (!kDense) if (red) {
            unpack8(v, a);  // reduce exactly the bf16 values that are stored
            float y[8];
            unpack8(p0[u], y);
#pragma unroll
            for (int e = 0; e < 8; ++e) { s1[e] += a[e]; s2[e] += a[e] * (y[e] - mu0[e]); }
            if (has_y1) {
              unpack8(p1[u], y);
#pragma unroll
              for (int e = 0; e < 8; ++e) t2[e] += a[e] * (y[e] - mu1[e]);
            }
          }
        }
        *reinterpret_cast<uint4*>(out + off[u]) = v;
      }
    }
    if (red) {
      // combine the RPI threads that own the same 8 columns, then one atomic per
      // column and quantity into this block's copy slot
      float* rb = reinterpret_cast<float*>(lds);     // [NTHR][24]
      esync();
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        rb[tid * 24 + e] = s1[e];
        rb[tid * 24 + 8 + e] = s2[e];
        rb[tid * 24 + 16 + e] = t2[e];
      }
      esync();
      if (tid < BN) {
        const int col = tid, cc = col >> 3, e = col & 7, n = n0 + col;
        float a = 0.f, b = 0.f, d = 0.f;
        for (int r = 0; r < RPI; ++r) {
          const float* q = rb + (cc + CPR * r) * 24;
          a += q[e]; b += q[8 + e]; d += q[16 + e];
        }
        if (n < N) {
          const int slot = (int)((unsigned)(m0 / BM) % (unsigned)bn.ncopy);
          float* d0 = bn.sums0 + (size_t)slot * 2 * N;
          atomicAdd(d0 + n, a);
          atomicAdd(d0 + N + n, b);
          if (bn.y1) {
            float* d1 = bn.sums1 + (size_t)slot * 2 * N;
            atomicAdd(d1 + n, a);
            atomicAdd(d1 + N + n, d);
          }
        }
      }
    }
  }
};

struct EpiF32Slab {  // split-K partial tile -> slab blockIdx.z of ws ([splits][M][ld] fp32, plain stores)
  float* ws; int ld; size_t slab;
  template <int BM, int BN, int MI, int NI>
  __device__ void apply(f32x16 (&acc)[MI][NI], char*, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int) const {
    float* out = ws + (size_t)blockIdx.z * slab;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * 32 * NI + 32 * j + (lane & 31);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 32 * MI + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) out[(size_t)m * ld + n] = acc[i][j][r];
        }
      }
  }
};


// Dense-layer finish of 8 consecutive columns from split-K slabs (shared by the fused
// epilogue below and dense_finalize_kernel): sum `splits` fp32 slabs at element offset
// `src`, then bias / GELU (pre-activation to preact) / GELU' (from dact) / + addend.
struct DenseFinish {
  bf16* C; int ldc; const float* bias; int act; bf16* preact; const bf16* addend; const bf16* dact;
  __device__ __forceinline__ void run(const float* ws, size_t slab, int splits, size_t src, int m, int c) const {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const float* base = ws + src;
    v4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 2 <= splits; k += 2) {      // both slabs' loads in flight together
      const v4 p0 = *reinterpret_cast<const v4*>(base + k * slab);
      const v4 q0 = *reinterpret_cast<const v4*>(base + k * slab + 4);
      const v4 p1 = *reinterpret_cast<const v4*>(base + (k + 1) * slab);
      const v4 q1 = *reinterpret_cast<const v4*>(base + (k + 1) * slab + 4);
      lo += p0 + p1;
      hi += q0 + q1;
    }
    if (k < splits) {
      lo += *reinterpret_cast<const v4*>(base + k * slab);
      hi += *reinterpret_cast<const v4*>(base + k * slab + 4);
    }
    float a[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const size_t o = (size_t)m * ldc + c;
    if (bias) {
      float bz[8];
      ldg8f(bias + c, bz);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += bz[e];
    }
    dense_act8(a, act, preact ? preact + o : nullptr);
    if (dact) dense_dact8(a, act, ldg16(dact + o));
    if (addend) {
      float b[8];
      unpack8(ldg16(addend + o), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    *reinterpret_cast<uint4*>(C + o) = pack8(a);
  }
};

// Split-K with the reduction inside the launch (cdna_hip_programming.md, projection GEMM
// item 2): every split writes its fp32 partial tile to slab blockIdx.z of ws with plain
// stores, publishes it (vmcnt drain, agent-scope release, drain again) and takes a ticket
// from the tile's counter; the split that draws the last ticket acquires, resets the
// counter and sums all slabs of the tile into the final output - fp32 (+= when
// accumulating; weight gradients) or the dense bf16 epilogue.  Correct for any placement
// of a tile's splits over XCDs; saves the separate reduce/finalize launch and its boundary.
// cnt: one zeroed counter per tile (grid.x), left zeroed; launches sharing it must be
// stream-ordered.
struct EpiSlabFused {
  float* ws; int ld; size_t slab; unsigned* cnt;
  int dense;                 // 0: fp32 out[M][ld] (+)= sum; 1: DenseFinish (ld == N)
  float* outf; int accumulate;
  DenseFinish fin;
  template <int BM, int BN, int MI, int NI>
  __device__ void apply(f32x16 (&acc)[MI][NI], char* lds, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int tid) const {
    float* part = ws + (size_t)blockIdx.z * slab;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * 32 * NI + 32 * j + (lane & 31);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 32 * MI + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) part[(size_t)m * ld + n] = acc[i][j][r];
        }
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == gridDim.z - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    const int splits = gridDim.z;
    if (dense) {
      constexpr int G = BN / 8;
      for (int q = tid; q < BM * G; q += NTHR) {
        const int m = m0 + q / G, c = n0 + (q % G) * 8;
        if (m < M && c < N) fin.run(ws, slab, splits, (size_t)m * ld + c, m, c);
      }
    } else {
      typedef float v4 __attribute__((ext_vector_type(4)));
      constexpr int G = BN / 4;
      for (int q = tid; q < BM * G; q += NTHR) {
        const int m = m0 + q / G, c = n0 + (q % G) * 4;
        if (m >= M || c >= N) continue;
        const size_t o = (size_t)m * ld + c;
        v4 a = accumulate ? *reinterpret_cast<const v4*>(outf + o) : (v4){0.f, 0.f, 0.f, 0.f};
        v4 b = {0.f, 0.f, 0.f, 0.f};
        int k = 0;
        for (; k + 2 <= splits; k += 2) {
          a += *reinterpret_cast<const v4*>(ws + k * slab + o);
          b += *reinterpret_cast<const v4*>(ws + (k + 1) * slab + o);
        }
        if (k < splits) a += *reinterpret_cast<const v4*>(ws + k * slab + o);
        *reinterpret_cast<v4*>(outf + o) = a + b;
      }
    }
  }
};

struct EpiF32Atomic {  // fp32 [M][ld] += (split-K partial sums)
  float* out; int ld;
  template <int BM, int BN, int MI, int NI>
  __device__ void apply(f32x16 (&acc)[MI][NI], char*, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int) const {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * 32 * NI + 32 * j + (lane & 31);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 32 * MI + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) atomicAdd(out + (size_t)m * ld + n, acc[i][j][r]);
        }
      }
  }
};

struct EpiF32 {  // fp32 [M][ld] = acc (+ bias[n]) (+= if accumulate)
  float* out; int ld; const float* bias; int accumulate;
  template <int BM, int BN, int MI, int NI>
  __device__ void apply(f32x16 (&acc)[MI][NI], char*, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int) const {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * 32 * NI + 32 * j + (lane & 31);
        if (n >= N) continue;
        const float b = bias ? bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 32 * MI + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) {
            float* o = out + (size_t)m * ld + n;
            *o = (accumulate ? *o : 0.f) + acc[i][j][r] + b;
          }
        }
      }
  }
};

// ---------------------------------------------------------------- main loop
// PF = 1: the next K-tile's loads are issued before the MFMAs of the current one.
// PF = 2: two register sets, loads issued two K-tiles ahead (the last tiles' prefetches
// are clamped to the final tile, so every iteration issues the same loads and the
// compiler can wait for the older set with a counted vmcnt).  The body is unrolled twice
// so each set's role is static (no runtime-indexed register arrays).
// Block tile -> per-wave tile (MI x NI MFMA 32x32 sub-tiles, 4 waves) and occupancy.  The
// 64x64 wave tile (2x2) reads one LDS fragment per MFMA; the 128x64 wave tile of the
// 256x128 / 128x256 blocks reads 0.75 and halves the global->LDS bytes per MFMA, at one
// block per CU (96 KB of double-buffered LDS).
// Three-wide dense tiles (128 x 96 / 192 / 288, both operands K-contiguous only): sized so
// that a 4096-token dense layer's output is exactly 256 or 512 tiles - one or two per CU,
// no partial last round - where 128x128 leaves 768/2304/3072-wide outputs at 192, 576 and
// 768 tiles.  128x96: 4x1 waves of 32x96; 128x192: 2x2 waves of 64x96 (80 KB of LDS, two
// blocks fill the 160 KB); 128x288: 4x1 waves of 32x288 at one block per CU.
template <int BM, int BN> struct TileCfg {
  static constexpr bool WIDE3 = BM == 128 && (BN == 96 || BN == 192 || BN == 288);
  static constexpr bool BIG = !WIDE3 && BM * BN > 128 * 128;
  // 128x64 (dense GEMMs with a 768-wide output): 2x2 waves of 64x32 (MI = 2, NI = 1)
  static constexpr bool NARROW = BM == 128 && BN == 64;
  static constexpr int MI = WIDE3 ? (BN == 192 ? 2 : 1) : (BIG && BM > BN) ? 4 : 2;
  static constexpr int NI = WIDE3 ? (BN == 192 ? 3 : BN / 32) : NARROW ? 1 : (BIG && BN > BM) ? 4 : 2;
  static constexpr int OCC = WIDE3 ? (BN == 288 ? 1 : 2) : BIG ? 1 : 2;
};

template <int BM, int BN, class LA, class LB, class EPI, int PF>
__global__ void __launch_bounds__(NTHR, (TileCfg<BM, BN>::OCC))
gemm_kernel(const LA la, const LB lb, const EPI epi, int M, int N, int K, int ktiles_per_split) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int MI = TileCfg<BM, BN>::MI, NI = TileCfg<BM, BN>::NI;
  constexpr int WN = BN / (32 * NI);
  // PF = 0: one LDS stage (single-K-tile GEMMs: 1x1 convs over 64 channels), sized only
  // for the tile and the epilogue's staging image, so 4 blocks fit a CU instead of 2
  constexpr int EPI_BYTES = BM * (BN + 8) * 2;
  constexpr int SMEM = PF == 0 ? (STAGE > EPI_BYTES ? STAGE : EPI_BYTES) : 2 * STAGE;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // tile id: XCD remap, then grouped (8 M-tiles per group) order for L2 reuse
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  constexpr int GM = 8;
  const int group = id / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsize = min(tiles_m - first_m, GM);
  const int in_g = id % (GM * tiles_n);
  const int tm = first_m + in_g % gsize, tn = in_g / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int ktiles = (K + BK - 1) / BK;
  const int kt0 = blockIdx.z * ktiles_per_split;
  const int nt = min(ktiles, kt0 + ktiles_per_split) - kt0;

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  typename LA::St sa;
  typename LB::St sb;
  la.init(sa, m0, tid);
  lb.init(sb, n0, tid);
  auto mfma_tile = [&](const char* As, const char* Bs) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = read_frag<LA::KC, BM>(As, wm * 32 * MI + 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = read_frag<LB::KC, BN>(Bs, wn * 32 * NI + 32 * j, s, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  // real: the tile is inside this split (PF=2 re-stages the clamped last tile); kt: the
  // K-tile the registers hold (for operand transforms)
  auto stage = [&](char* buf, uint4 (&ra)[BM / 32], uint4 (&rb)[BN / 32], int kt, bool real) {
    if constexpr (HasXform<LA>::value) la.xform(sa, kt, tid, ra);
    if constexpr (HasXform<LB>::value) lb.xform(sb, kt, tid, rb);
    store_stage<LA, BM>(buf, tid, ra);
    store_stage<LB, BN>(buf + A_BYTES, tid, rb);
    if constexpr (HasSum<LA>::value) {
      if (real) la.accum(sa, ra);
    }
  };
  if (nt > 0) {
    if constexpr (PF == 0) {
      for (int t = 0; t < nt; ++t) {
        uint4 ra[BM / 32], rb[BN / 32];
        la.load(sa, kt0 + t, tid, ra);
        lb.load(sb, kt0 + t, tid, rb);
        if (t > 0) __syncthreads();          // previous tile's fragment reads are done
        stage(smem, ra, rb, kt0 + t, true);
        __syncthreads();
        mfma_tile(smem, smem + A_BYTES);
      }
      __syncthreads();                       // the epilogue reuses the LDS
    } else if constexpr (PF == 3) {
      // LDS-DMA double buffer: tile t+1 streams global -> LDS (no VGPRs, no ds_write)
      // while tile t is multiplied; each thread issues NDMA copies per tile, so
      // vmcnt(NDMA) after issuing t+1 means this wave's copies of t have landed
      constexpr int NDMA = BM / 32 + BN / 32;
      la.dma(sa, kt0, tid, smem);
      lb.dma(sb, kt0, tid, smem + A_BYTES);
      for (int t = 0; t < nt; ++t) {
        char* cur = smem + (t & 1) * STAGE;
        if (t + 1 < nt) {
          char* nxt = smem + ((t + 1) & 1) * STAGE;
          la.dma(sa, kt0 + t + 1, tid, nxt);
          lb.dma(sb, kt0 + t + 1, tid, nxt + A_BYTES);
          vmwait<NDMA>();
        } else {
          vmwait<0>();
        }
        // raw s_barrier, not __syncthreads(): its fence would wait for vmcnt(0), i.e. for
        // tile t+1's copies too, and serialise the DMA with the MFMAs
        lds_barrier();                       // every wave's copies of tile t landed
        mfma_tile(cur, cur + A_BYTES);
        lds_barrier();                       // tile t's buffer is free for tile t+2
      }
      __syncthreads();                       // the epilogue reuses the LDS
    } else if constexpr (PF == 1) {
      uint4 ra[BM / 32], rb[BN / 32];
      la.load(sa, kt0, tid, ra);
      lb.load(sb, kt0, tid, rb);
      stage(smem, ra, rb, kt0, true);
      __syncthreads();
      for (int t = 0; t < nt; ++t) {
        const char* cur = smem + (t & 1) * STAGE;
        const bool more = t + 1 < nt;
        if (more) {  // issue next tile's global loads before the MFMAs
          la.load(sa, kt0 + t + 1, tid, ra);
          lb.load(sb, kt0 + t + 1, tid, rb);
        }
        mfma_tile(cur, cur + A_BYTES);
        if (more) stage(smem + ((t + 1) & 1) * STAGE, ra, rb, kt0 + t + 1, true);
        __syncthreads();
      }
    } else {
      const int last = kt0 + nt - 1;
      uint4 a0[BM / 32], b0[BN / 32], a1[BM / 32], b1[BN / 32];
      la.load(sa, kt0, tid, a0);
      lb.load(sb, kt0, tid, b0);
      la.load(sa, min(kt0 + 1, last), tid, a1);
      lb.load(sb, min(kt0 + 1, last), tid, b1);
      stage(smem, a0, b0, kt0, true);
      __syncthreads();
      for (int t = 0;; t += 2) {
        // compute t from buffer 0; set 1 (tile t+1) in flight; set 0 free
        la.load(sa, min(kt0 + t + 2, last), tid, a0);
        lb.load(sb, min(kt0 + t + 2, last), tid, b0);
        mfma_tile(smem, smem + A_BYTES);
        stage(smem + STAGE, a1, b1, min(kt0 + t + 1, last), t + 1 < nt);
        __syncthreads();
        if (t + 1 >= nt) break;
        // compute t+1 from buffer 1; set 0 (tile t+2) in flight; set 1 free
        la.load(sa, min(kt0 + t + 3, last), tid, a1);
        lb.load(sb, min(kt0 + t + 3, last), tid, b1);
        mfma_tile(smem + STAGE, smem + STAGE + A_BYTES);
        stage(smem, a0, b0, min(kt0 + t + 2, last), t + 2 < nt);
        __syncthreads();
        if (t + 2 >= nt) break;
      }
    }
  }
  if constexpr (HasSum<LA>::value) la.finish(sa, tn == 0, tid, smem);
  epi.template apply<BM, BN, MI, NI>(acc, smem, m0, n0, M, N, wm, wn, lane, tid);
}

// Persistent variant of the LDS-DMA main loop for short-K GEMMs (1x1 convs over <= a few
// hundred channels: 1-8 K-tiles per output tile).  The non-persistent kernel pays, per
// output tile, a cold prologue (first DMA round trip with nothing to overlap) and an
// epilogue (LDS staging + stores) with nothing in flight; with only 1-4 K-tiles that is
// most of a tile's life (the channel-expanding ResNet 1x1 convs ran at 1.7-4.5 TB/s,
// profiles/round6/roofline_resnet50_b512.txt).  Here one block per CU walks a sequence of
// tiles and the DMA ring runs ACROSS tile boundaries: the copies of the next tile's first
// K-tiles are in flight while this tile's last MFMAs and its epilogue run.
//   * NBUF operand stages in a ring + a separate epilogue staging region, so the epilogue
//     never waits for the ring;
//   * the epilogue's barriers are raw s_barriers (EpiBF16::raw_sync), never a full
//     __syncthreads() that would drain vmcnt;
//   * tiles are split into 8 contiguous ranges of the grouped tile order, one per XCD
//     (blockIdx.x % 8), whose blocks stride through it: the tiles one XCD holds at a time
//     are neighbours, so the A rows / B columns they share stay in that XCD's L2.
template <class E> struct IsEpiBF16 { static constexpr bool value = false; };
template <class RM, bool D> struct IsEpiBF16<EpiBF16<RM, D>> { static constexpr bool value = true; };

template <int BM, int BN, class LA, class LB, class EPI, int NBUF>
__global__ void __launch_bounds__(NTHR, 1)
gemm_persist_kernel(const LA la, const LB lb, EPI epi, int M, int N, int K) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int MI = TileCfg<BM, BN>::MI, NI = TileCfg<BM, BN>::NI;
  constexpr int WN = BN / (32 * NI);
  constexpr int EPI_BYTES = BM * (BN + 8) * 2;
  constexpr int NDMA = BM / 32 + BN / 32;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE + EPI_BYTES];
  char* const elds = smem + NBUF * STAGE;
  epi.raw_sync = true;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int nt = (K + BK - 1) / BK;
  // this XCD's contiguous range of tile ids and this block's stride through it
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int gx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int t_begin = xcd * q8 + (xcd < r8 ? xcd : r8);
  const int t_count = q8 + (xcd < r8 ? 1 : 0);
  const int mine = loc < t_count ? (t_count - loc + gx - 1) / gx : 0;
  const int Q = mine * nt;                  // (tile, K-tile) work items of this block
  auto tile_mn = [&](int j, int& m0, int& n0) {
    const int id = t_begin + loc + j * gx;
    constexpr int GM = 8;
    const int group = id / (GM * tiles_n);
    const int first_m = group * GM;
    const int gsize = min(tiles_m - first_m, GM);
    const int in_g = id % (GM * tiles_n);
    m0 = (first_m + in_g % gsize) * BM;
    n0 = (in_g / gsize) * BN;
  };
  typename LA::St sa;
  typename LB::St sb;
  int issue_tile = -1;
  auto issue = [&](int q) {
    const int j = q / nt, t = q - j * nt;
    if (j != issue_tile) {
      int m0, n0;
      tile_mn(j, m0, n0);
      la.init(sa, m0, tid);
      lb.init(sb, n0, tid);
      issue_tile = j;
    }
    char* buf = smem + (q % NBUF) * STAGE;
    la.dma(sa, t, tid, buf);
    lb.dma(sb, t, tid, buf + A_BYTES);
  };
  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int q = 0; q < NBUF - 1 && q < Q; ++q) issue(q);
  int cm0 = 0, cn0 = 0;
  if (Q > 0) tile_mn(0, cm0, cn0);
  for (int q = 0; q < Q; ++q) {
    if (q + NBUF - 1 < Q) {
      issue(q + NBUF - 1);
      vmwait<(NBUF - 1) * NDMA>();           // this wave's copies of item q landed
    } else {
      vmwait<0>();
    }
    lds_barrier();                           // every wave's copies of item q landed
    const char* cur = smem + (q % NBUF) * STAGE;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = read_frag<LA::KC, BM>(cur, wm * 32 * MI + 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = read_frag<LB::KC, BN>(cur + A_BYTES, wn * 32 * NI + 32 * j, s, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if ((q + 1) % nt == 0) {                 // the tile's last K-tile: epilogue, next tile
      epi.template apply<BM, BN, MI, NI>(acc, elds, cm0, cn0, M, N, wm, wn, lane, tid);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      if (q + 1 < Q) tile_mn((q + 1) / nt, cm0, cn0);
    }
    lds_barrier();                           // stage q % NBUF is free for item q + NBUF
  }
}

// K-tile prefetch depth of the main loop (1 = next tile, 2 = two tiles ahead, used for the
// 128x128 tile when a split has at least 4 K-tiles); mlc_gemm_config switches it for A/B
// measurements
static int g_prefetch = 2;
// split-K weight gradients: grow the split until tiles*splits reaches this many blocks.
// Plain-matrix operands (1x1 convs, dense layers) prefer fewer splits: their K loop is
// cheap, so the fp32 atomic traffic of extra splits costs more than the lost occupancy
// (measured on every ResNet-50 wgrad shape: 256 vs 768 blocks saves 10-30 %); gathered
// operands (3x3 / 7x7 convs) want more occupancy.  Re-tuned on the whole step once the
// weight gradients ran beside the LDS-DMA forward / dgrad GEMMs: gathered 768 -> 384 and
// plain (1x1 conv) 256 -> 128 gave ResNet-50 +1.5 %, U-Net +3.6 % (profiles/round2_ab/split_retune).
// Round 5 (atomic wgrads on ResNet-50, unjoined chains on the segmentation engines): gathered
// 384 -> 256 gives U-Net / LinkNet / FPN +2.1-2.5 %, DeepLab +1.7 %, U-Net-ResNeXt-50 +1.1 %,
// ResNet-50 neutral (profiles/round5/split_target_256_ab.txt).
static int g_split_target = 256;
// single-LDS-stage variant for single-K-tile splits (A/B knob 5)
static int g_single_stage = 1;
// ... and for splits of up to this many K-tiles (A/B knob 13, MLC_SINGLE_STAGE_KT): one LDS
// stage fits 4 blocks per CU instead of 2, which hides the load / store latency of short-K
// GEMMs (ResNet's channel-expanding 1x1 convs) across blocks instead of within one
static int g_single_stage_kt = 1;
static int g_split_target_mat = 128;
// dense-layer weight gradients (mlc_linear_wgrad_bias, mlc_gemm_f32out), A/B knob 9.
// Round 2 kept 256 (128 lost 3 %); once the bf16 dgrads stopped splitting (knob 12 = 0)
// 128 became the better point: BERT-base 5041/5096 vs 5021/4991 seq/s at 256, 64 lost
// 2 % (profiles/round3/session2/wgrad_split_ab.txt).  Since round 5 the weight gradients
// run as one unjoined side chain (native_bert.py) and 256 is the better point again:
// 5720/5731 vs 5643/5658 seq/s, 192 and 320 lose (profiles/round5/bert_wgrad_join_ab.txt)
static int g_split_target_dense = 256;
// bf16-output dense GEMMs on the 128x128 path (BERT's input gradients with MN-contiguous
// weights) split K until tiles * splits reaches this (A/B knob 12, MLC_DENSE_SPLIT_TARGET;
// 0 never splits).  Default 0 since round 3: unsplit 192-tile dgrads with the epilogue in
// the GEMM beat split-K 2 + slab finalize by 4.3 % on the BERT-base step (5041/5058 vs
// 4853/4821 seq/s, profiles/round3/session2/dense_split_ab.txt); 768 lost 4.5 %.
static int g_dense_bf16_split_target = 0;
// LDS-DMA main loop (PF = 3) for GEMMs whose two operands both have an enabled DMA copy
// (the K-contiguous MatKC / ConvFwdA: forward convs, stride-1 dgrads, dense forward):
// A/B knob 8; -1: read MLC_GEMM_DMA on first use (default 1: ResNet-50 +1.2 %, U-Net
// +3.2 %, BERT +0.8 %, profiles/round2_ab/gemm_dma)
static int g_gemm_dma = -1;
// persistent short-K kernel (gemm_persist_kernel): 0 off, 1 for epilogues without global
// loads (forward convs + BN statistics), 2 also epilogues that load (residual addend, BN
// backward operands, bias); MLC_GEMM_PERSIST, read on first use.  g_persist_kt: most
// K-tiles per output tile it takes (MLC_GEMM_PERSIST_KT); g_persist_nbuf: ring depth 2 / 3.
static int g_persist = -1;
static int g_persist_kt = 8;
static int g_persist_nbuf = 3;
static int g_num_cus = 0;

template <class EPI>
static bool epi_loads(const EPI& e) {
  if constexpr (IsEpiBF16<EPI>::value) return e.addend || e.bn.y0 || e.dact || e.bias || e.preact;
  return true;
}

template <int BM, int BN, class LA, class LB, class EPI>
static hipError_t launch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K,
                         int splits, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  if constexpr (BM == 128 && BN == 128 && HasDma<LA>::value && HasDma<LB>::value && IsEpiBF16<EPI>::value) {
    if (g_persist < 0) {
      const char* e = getenv("MLC_GEMM_PERSIST");
      g_persist = e ? atoi(e) : 0;
      if (const char* k = getenv("MLC_GEMM_PERSIST_KT")) g_persist_kt = atoi(k);
      if (const char* b = getenv("MLC_GEMM_PERSIST_NBUF")) g_persist_nbuf = atoi(b);
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (g_num_cus <= 0) g_num_cus = 256;
    }
    if (g_persist && splits <= 1 && ktiles >= 1 && ktiles <= g_persist_kt && tiles >= 2 * g_num_cus &&
        (g_persist >= 2 || !epi_loads(epi))) {
      const int grid = g_num_cus;            // one block per CU (the LDS ring + staging region)
      if (g_persist_nbuf == 2)
        hipLaunchKernelGGL((gemm_persist_kernel<BM, BN, LA, LB, EPI, 2>), dim3(grid), dim3(NTHR), 0, st, la, lb, epi,
                           M, N, K);
      else
        hipLaunchKernelGGL((gemm_persist_kernel<BM, BN, LA, LB, EPI, 3>), dim3(grid), dim3(NTHR), 0, st, la, lb, epi,
                           M, N, K);
      return hipGetLastError();
    }
  }
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles > 0 ? ktiles : 1;
  const int per = ktiles > 0 ? (ktiles + splits - 1) / splits : 0;
  splits = per > 0 ? (ktiles + per - 1) / per : 1;
  dim3 grid(tiles, 1, splits);
  if (per <= (g_single_stage_kt > 1 ? g_single_stage_kt : 1) && g_single_stage) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 0>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
    return hipGetLastError();
  }
  if constexpr (HasDma<LA>::value && HasDma<LB>::value) {
    if (g_gemm_dma < 0) {
      const char* e = getenv("MLC_GEMM_DMA");
      g_gemm_dma = e ? atoi(e) : 1;
    }
    if (g_gemm_dma && per >= 2) {
      hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 3>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
      return hipGetLastError();
    }
  }
  // the second register set only fits the square (and the 128x64) tile without spilling
  if constexpr (BM == BN || TileCfg<BM, BN>::NARROW) {
    if (g_prefetch >= 2 && per >= 4) {
      hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 2>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 1>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
  return hipGetLastError();
}

// tile shape: 0 = 128x128, 1 = 256x64 (narrow N), 2 = 64x256 (narrow M), 3 = 256x128,
// 4 = 128x256 (wide-wave tiles, used when they still give every CU a block)
static int g_big_tiles = 0;
static int g_big_min_blocks = 240;
// split-K reduction inside the GEMM launch (EpiSlabFused) instead of a separate
// reduce / finalize kernel, for GEMMs whose slabs of one tile (splits x BM x BN fp32) the
// reducing block can read in at most this many KB (A/B knob 6; 0 = never).  The reducer
// reads them alone, so many splits (weight gradients, up to 16+) stay on the separate pass.
static int g_splitk_fused = 0;
// 128x64 tiles instead of split-K for narrow dense outputs (A/B knob 7); -1: read
// MLC_DENSE_NARROW on first use (default 0: measured neutral on BERT-base)
static int g_dense_narrow = -1;
// three-wide tile (5: 128x96, 6: 128x192, 7: 128x288) for a dense GEMM whose operands are
// both K-contiguous; 0 keeps the 128x128 / split-K path.  MLC_DENSE_TILE forces a tile
// (A/B; MLC_DENSE_SPLIT a split-K factor with it); unset: picked by pick_dense_tile's model.
static int g_dense_tile = -2, g_dense_split = 1;
static int pick_dense_tile(int M, int N, int K, int& split) {
  if (g_dense_tile == -2) {
    const char* e = getenv("MLC_DENSE_TILE");
    g_dense_tile = e ? atoi(e) : -1;
    const char* s = getenv("MLC_DENSE_SPLIT");
    g_dense_split = s ? atoi(s) : 1;
  }
  split = g_dense_split > 1 ? g_dense_split : 1;
  if (g_dense_tile >= 0) return g_dense_tile;
  // Model from scripts/bench_dense_tiles.py on BERT-base (M = 4096 tokens, graph-timed):
  // a three-wide tile pays when it turns the output into 256-640 tiles (one or two per CU,
  // 128x128 leaves a partial last round): 2304/3072-wide outputs on 128x192 (-9 / -12 %),
  // 768-wide on 128x96 (-33 % at K = 768), split-K 2 on top from K >= 2560 (-6 %).  The
  // 128x288 tile (one block per CU) lost on every shape.
  split = 1;
  const long tm = (M + 127) / 128;
  const long t192 = tm * ((N + 191) / 192), t96 = tm * ((N + 95) / 96);
  if (t192 >= 256 && t192 <= 640) return 6;
  if (t96 >= 128 && t96 <= 640) {
    if (K >= 2560 && t96 <= 256) split = 2;
    return 5;
  }
  return 0;
}
constexpr int kSplitCounters = 1 << 16;          // tiles per eager stream region
constexpr long kCapturedCounters = 1L << 21;      // per device, handed out once per captured launch
// Tile counters for EpiSlabFused.  A counter is persistent state: every launch leaves its
// tiles' counters zeroed, so two launches that count on the SAME counters at the same
// time (a main-stream dgrad beside a side-stream weight gradient inside one graph, or an
// eager launch on another stream beside a graph replay) make one split take a foreign
// ticket.  The tile then finalizes early (partial sums) or never, and its counter is left
// non-zero, so every later launch that uses it computes garbage: the "NaN within ~10 graph
// replays once eager kernels ran on the NULL stream" of round 4 (docs/architecture.md).
// Hence no two launches that can overlap share counters:
//   * eager launches get one region per stream (launches on one stream are ordered);
//   * a launch being captured gets a region of its own from a per-device pool, tagged with
//     the capture's owner id (mlc_counters_owner, set by the Python capture scope).  When
//     the owning graph is dropped its regions go back to the pool (mlc_counters_release):
//     every launch leaves its counters zeroed, and a later capture starts after a device
//     synchronize, so a recycled region is never counted on by two live graphs.
// Everything is allocated (zeroed) outside capture; nullptr -> the caller falls back to
// the separate reduction kernel, which needs no counters (logged once per device).
struct CounterRegion {
  long off, len;
  int owner;
};
struct CounterPool {
  std::mutex mu;
  unsigned* captured = nullptr;
  long captured_used = 0;
  std::vector<CounterRegion> live;          // owned regions of captured launches
  std::vector<std::pair<long, long>> free;  // released (off, len), first fit
  bool warned = false;
  std::map<hipStream_t, unsigned*> eager;
};
static CounterPool g_counter_pools[16];
static int g_counter_owner = 0;             // owner id of captures in progress (0: none)

static unsigned* alloc_zeroed_counters(long n, hipStream_t st) {
  unsigned* p = nullptr;
  if (hipMalloc(&p, n * sizeof(unsigned)) != hipSuccess) return nullptr;
  // zeroed on the stream that first uses the region (stream order covers that use); no
  // device-wide synchronize, which would invalidate a capture running on another stream
  if (hipMemsetAsync(p, 0, n * sizeof(unsigned), st) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}
static long take_captured(CounterPool& P, long n) {
  for (size_t i = 0; i < P.free.size(); ++i) {
    if (P.free[i].second >= n) {
      const long off = P.free[i].first;
      P.free[i].first += n;
      P.free[i].second -= n;
      if (P.free[i].second == 0) P.free.erase(P.free.begin() + i);
      return off;
    }
  }
  if (P.captured_used + n > kCapturedCounters) return -1;
  const long off = P.captured_used;
  P.captured_used += n;
  return off;
}
static unsigned* split_counters(hipStream_t st, long tiles, int splits, int bm, int bn) {
  if (tiles > kSplitCounters || (long)splits * bm * bn * 4 > (long)g_splitk_fused * 1024) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  CounterPool& P = g_counter_pools[dev];
  std::lock_guard<std::mutex> lk(P.mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
  if (cs != hipStreamCaptureStatusNone) {
    const long n = (tiles + 63) & ~63L;      // keep regions on separate 256-B lines
    const long off = P.captured ? take_captured(P, n) : -1;
    if (off < 0) {
      if (!P.warned) {
        fprintf(stderr, "[mlcomp] split-K counter pool of device %d exhausted (%ld of %ld in use): captured "
                        "split-K GEMMs fall back to the separate reduction pass\n", dev, P.captured_used,
                kCapturedCounters);
        P.warned = true;
      }
      return nullptr;
    }
    P.live.push_back({off, n, g_counter_owner});
    return P.captured + off;
  }
  if (!P.captured) P.captured = alloc_zeroed_counters(kCapturedCounters, st);  // ready for a later capture
  auto it = P.eager.find(st);
  if (it != P.eager.end()) return it->second;
  unsigned* r = alloc_zeroed_counters(kSplitCounters, st);
  if (r) P.eager[st] = r;
  return r;
}

// Owner id for the captured counter regions handed out from now on (0: unowned, kept for
// the life of the process).  Called by the capture scope around a graph capture.
MLC_EXPORT void mlc_counters_owner(int owner) { g_counter_owner = owner; }

// Return every captured region of ``owner`` (a dropped graph) to the device's pool; the
// number of counters freed.
MLC_EXPORT long mlc_counters_release(int owner) {
  if (owner == 0) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  CounterPool& P = g_counter_pools[dev];
  std::lock_guard<std::mutex> lk(P.mu);
  long freed = 0;
  for (size_t i = 0; i < P.live.size();) {
    if (P.live[i].owner == owner) {
      P.free.push_back({P.live[i].off, P.live[i].len});
      freed += P.live[i].len;
      P.live[i] = P.live.back();
      P.live.pop_back();
    } else {
      ++i;
    }
  }
  // coalesce neighbours, then give a free tail back to the bump pointer
  std::sort(P.free.begin(), P.free.end());
  std::vector<std::pair<long, long>> merged;
  for (auto& f : P.free) {
    if (!merged.empty() && merged.back().first + merged.back().second == f.first) merged.back().second += f.second;
    else merged.push_back(f);
  }
  if (!merged.empty() && merged.back().first + merged.back().second == P.captured_used) {
    P.captured_used = merged.back().first;
    merged.pop_back();
  }
  P.free.swap(merged);
  return freed;
}

// Counters of the device's captured pool in use (bump pointer minus released holes).
MLC_EXPORT long mlc_counters_in_use() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  CounterPool& P = g_counter_pools[dev];
  std::lock_guard<std::mutex> lk(P.mu);
  long holes = 0;
  for (auto& f : P.free) holes += f.second;
  return P.captured_used - holes;
}
static inline int tile_bm(int tile) { return tile == 1 || tile == 3 ? 256 : tile == 2 ? 64 : 128; }
static inline int tile_bn(int tile) { return tile == 1 ? 64 : tile == 2 || tile == 4 ? 256 : 128; }
static int pick_tile(int M, int N) {
  if (N <= 64 && M > 64) return 1;
  if (M <= 64 && N > 64) return 2;
  if (g_big_tiles) {
    const long t3 = (long)((M + 255) / 256) * ((N + 127) / 128);
    const long t4 = (long)((M + 127) / 128) * ((N + 255) / 256);
    if (M >= N && t3 >= g_big_min_blocks) return 3;
    if (N > M && t4 >= g_big_min_blocks) return 4;
  }
  return 0;
}

// pick a split-K factor so a small-output / long-K GEMM still fills 256 CUs
static int auto_splits(int M, int N, int K, int tile, int target = g_split_target) {
  const int BMv = tile_bm(tile);
  const int BNv = tile_bn(tile);
  const int tiles = ((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv);
  const int ktiles = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < target && ktiles / (s * 2) >= 4) s *= 2;
  return s;
}

}  // namespace igemm

using namespace igemm;
using namespace igemm_host;




// dispatch one GEMM over the three tile shapes; MK(R) builds the loaders for R rows
#define MLC_TILE_DISPATCH(TILE, M, N, K, SPLITS, ST, EPI, MKA, MKB)                              \
  do {                                                                                         \
    if ((TILE) == 1) return launch<256, 64>(MKA(256), MKB(64), EPI, M, N, K, SPLITS, ST);      \
    if ((TILE) == 2) return launch<64, 256>(MKA(64), MKB(256), EPI, M, N, K, SPLITS, ST);      \
    if ((TILE) == 3) return launch<256, 128>(MKA(256), MKB(128), EPI, M, N, K, SPLITS, ST);    \
    if ((TILE) == 4) return launch<128, 256>(MKA(128), MKB(256), EPI, M, N, K, SPLITS, ST);    \
    return launch<128, 128>(MKA(128), MKB(128), EPI, M, N, K, SPLITS, ST);                     \
  } while (0)

MLC_EXPORT int mlc_bn_stat_copies() { return NSTAT; }

MLC_EXPORT int mlc_gemm_config(int prefetch) {
  const int old = igemm::g_prefetch;
  if (prefetch == 1 || prefetch == 2) igemm::g_prefetch = prefetch;
  return old;
}

// tuning knobs for A/B measurements: key 0 = prefetch depth (1, 2), key 1 / 2 = split-K
// block target of gathered / plain-matrix weight-gradient GEMMs, ..., 10 / 11 = three-wide
// dense tile (-1 auto, 0 off, 5-7) / its split-K factor; returns the previous value
// (-1: bad key)
MLC_EXPORT int mlc_gemm_get_set(int key, int value) {
  int* k = key == 0 ? &igemm::g_prefetch : key == 1 ? &igemm::g_split_target
          : key == 2 ? &igemm::g_split_target_mat : key == 3 ? &igemm::g_big_tiles
          : key == 4 ? &igemm::g_big_min_blocks : key == 5 ? &igemm::g_single_stage
          : key == 6 ? &igemm::g_splitk_fused : key == 7 ? &igemm::g_dense_narrow
          : key == 8 ? &igemm::g_gemm_dma : key == 9 ? &igemm::g_split_target_dense
          : key == 10 ? &igemm::g_dense_tile : key == 11 ? &igemm::g_dense_split
          : key == 12 ? &igemm::g_dense_bf16_split_target : key == 13 ? &igemm::g_single_stage_kt
          : key == 14 ? &igemm::g_persist : key == 15 ? &igemm::g_persist_nbuf : key == 16 ? &igemm::g_persist_kt
          : nullptr;
  if (!k) return -1;
  if (key == 14 && igemm::g_persist < 0) {   // resolve the env defaults (CU count) first
    const char* e = getenv("MLC_GEMM_PERSIST");
    igemm::g_persist = e ? atoi(e) : 0;
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&igemm::g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (igemm::g_num_cus <= 0) igemm::g_num_cus = 256;
  }
  if (key == 10 || key == 11) {   // resolve the env defaults before the first override
    int sp = 1;
    (void)igemm::pick_dense_tile(4096, 768, 768, sp);
  }
  const int old = *k;
  if (key == 10) {                // -1 = auto (pick_dense_tile's model), 0 = off, 5-7 = forced
    if (value >= -1) *k = value;
    return old;
  }
  if (value >= 0 && (value > 0 || key == 3 || key == 5 || key == 6 || key == 7 || key == 8 || key == 12)) *k = value;
  return old;
}

// y[N,Ho,Wo,Co] = conv(x[N,H,W,C], w[Co,KH,KW,C]).  If sum/sumsq are given they must
// hold NSTAT*Co fp32 (zeroed by the caller); per-channel partial sums of y and y^2 are
// accumulated into them (reduce over the NSTAT copies to get the BN statistics).
// Requires C % 8 == 0 and Co % 8 == 0.
// in_sc/in_sh (optional, [C] fp32): x is the PRE-BatchNorm tensor of a ReLU BN and the
// conv reads relu(x * in_sc + in_sh) (BnIn transform in the A loader; zero padding stays
// zero), so the BN output never has to be written.
// y rows of stride ldy >= Co (ldy > Co: y is a channel slice of wider rows - a DenseNet layer's
// new features written straight into its block's concat buffer)
static int conv_fwd_impl(const bf16* x, const bf16* w, bf16* y, int ldy, float* sum, float* sumsq,
                         int N, int H, int W, int C, int Co, int KH, int KW, int stride,
                         int pad, int dil, int Ho, int Wo, const float* in_sc, const float* in_sh,
                         hipStream_t st) {
  if (C % 8 || Co % 8 || ldy < Co || ldy % 8 || KH > 15 || KW > 16 || ((in_sc == nullptr) != (in_sh == nullptr)))
    return -1;
  const int M = N * Ho * Wo, K = KH * KW * C;
  const int tile = pick_tile(M, Co);
  EpiBF16<> epi{y, ldy, sum, sumsq, IdentityRows{}};
  epi.ncopy = g_mlc_ncopy;
  if (sum && g_mlc_det && (M + 63) / 64 > g_mlc_ncopy) return -2;   // one copy per 64-row group
  const BnIn bn{in_sc, in_sh};
#define MKB(R) (MatKC<R>{w, K, Co, K})
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    if (in_sc) {
#define MKA(R) (MatKCBn<R>{{x, C, M, K}, bn})
      MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
    }
#define MKA(R) (MatKC<R>{x, C, M, K})
    MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  if (in_sc) {
#define MKA(R) (ConvFwdABn<R>{{x, g, M, K}, bn})
    MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
#define MKA(R) (ConvFwdA<R>{x, g, M, K})
  MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
#undef MKB
}

MLC_EXPORT int mlc_conv_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq,
                            int N, int H, int W, int C, int Co, int KH, int KW, int stride,
                            int pad, int dil, int Ho, int Wo, const float* in_sc, const float* in_sh,
                            hipStream_t st) {
  return conv_fwd_impl(x, w, y, Co, sum, sumsq, N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo, in_sc, in_sh, st);
}

MLC_EXPORT int mlc_conv_fwd_ld(const bf16* x, const bf16* w, bf16* y, int ldy, int N, int H, int W, int C, int Co,
                               int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, hipStream_t st) {
  return conv_fwd_impl(x, w, y, ldy, nullptr, nullptr, N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo, nullptr,
                       nullptr, st);
}

// dx[N,H,W,C] = conv_transpose(dy[N,Ho,Wo,Co], w) (+ addend, same layout as dx; may
// alias dx) -- the addend fuses the gradient sum at a residual branch point.
// bn_y0 != null additionally fuses the backward reduction of the BatchNorm(s) whose
// output gradient dx is (see BnBwdEpi): dx is stored masked by bn_mask > 0 (or by the
// mask recomputed from bn_y0/bn_y1 with bn_msc/bn_msh) and the partial sums go to
// bn_sums{0,1}[NSTAT][2][C] (zeroed by the caller).
// A strided conv runs one GEMM per stride-parity class of dx (only the filter taps that
// reach the class are in its K loop; a class no tap reaches gets K = 0), so every dx row
// is written by a GEMM epilogue and no structurally-zero products are computed.
// sum/sumsq (optional): per-column BN forward statistics of dx, as in mlc_conv_fwd - the
// transposed-conv forward (mlc_conv_tr_fwd) is this GEMM with a BatchNorm after it.
static int conv_dgrad_impl(const bf16* dy, const bf16* w, bf16* dx, const bf16* addend, int N,
                           int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                           int dil, int Ho, int Wo, const bf16* bn_mask, const bf16* bn_y0,
                           const float* bn_mean0, float* bn_sums0, const bf16* bn_y1,
                           const float* bn_mean1, float* bn_sums1, const float* bn_msc0,
                           const float* bn_msh0, const float* bn_msc1, const float* bn_msh1,
                           float* sum, float* sumsq, hipStream_t st) {
  if (C % 8 || Co % 8 || KH > 15 || KW > 16 || stride < 1 || ((sum == nullptr) != (sumsq == nullptr))) return -1;
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  BnBwdEpi bn{bn_mask, bn_y0, bn_mean0, bn_sums0, bn_y1, bn_mean1, bn_sums1,
              bn_msc0, bn_msh0, bn_msc1, bn_msh1, g_mlc_ncopy};
  if (bn_y0 && g_mlc_det && ((long)N * H * W + 63) / 64 > g_mlc_ncopy) return -2;
  if (bn_msc0 && (!bn_msh0 || !bn_y0 || (bn_msc1 && (!bn_msh1 || !bn_y1)))) return -1;
  if (bn_y0 && (!bn_mean0 || !bn_sums0 || (bn_y1 && (!bn_mean1 || !bn_sums1)))) return -1;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    const DgradClass cl = mkclass(1, 0, 0, H, W, Ho, Wo, Co, 1, 1, 0, dil);
    const int M = N * H * W, K = cl.ncb * BK;
    if (sum && g_mlc_det && (M + 63) / 64 > g_mlc_ncopy) return -2;
    const int tile = pick_tile(M, C);
    EpiBF16<> epi{dx, C, sum, sumsq, IdentityRows{}, addend, bn};
    epi.ncopy = g_mlc_ncopy;
#define MKA(R) (MatKC<R>{dy, Co, M, Co})
#define MKB(R) (ConvDgradB<R>{w, g, cl})
    MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
  hipError_t err = hipSuccess;
  // the parity-class GEMMs run one after another on the stream, so in deterministic mode
  // the statistics stay reproducible as long as each launch has a copy per 64-row group
  for (int ph = 0; ph < stride && ph < H; ++ph)
    for (int pw = 0; pw < stride && pw < W; ++pw) {
      const DgradClass cl = mkclass(stride, ph, pw, H, W, Ho, Wo, Co, KH, KW, pad, dil);
      if (cl.nr > 15 || cl.ns > 16) return -1;
      const int M = N * cl.Hc * cl.Wc, K = cl.nr * cl.ns * cl.ncb * BK;
      if (M <= 0) continue;
      if (sum && g_mlc_det && (M + 63) / 64 > g_mlc_ncopy) return -2;
      const int tile = pick_tile(M, C);
#define MKA(R) (ConvDgradA<R>{dy, g, M, K, cl})
      if (stride == 1) {
        EpiBF16<> epi{dx, C, sum, sumsq, IdentityRows{}, addend, bn};
        epi.ncopy = g_mlc_ncopy;
        err = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB); }();
      } else {
        EpiBF16<ClassRows> epi{dx, C, sum, sumsq, ClassRows{cl, H, W}, addend, bn};
        epi.ncopy = g_mlc_ncopy;
        err = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB); }();
      }
#undef MKA
      if (err != hipSuccess) return err;
    }
  return err;
#undef MKB
}

MLC_EXPORT int mlc_conv_dgrad(const bf16* dy, const bf16* w, bf16* dx, const bf16* addend, int N,
                              int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                              int dil, int Ho, int Wo, const bf16* bn_mask, const bf16* bn_y0,
                              const float* bn_mean0, float* bn_sums0, const bf16* bn_y1,
                              const float* bn_mean1, float* bn_sums1, const float* bn_msc0,
                              const float* bn_msh0, const float* bn_msc1, const float* bn_msh1,
                              hipStream_t st) {
  return conv_dgrad_impl(dy, w, dx, addend, N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo, bn_mask, bn_y0,
                         bn_mean0, bn_sums0, bn_y1, bn_mean1, bn_sums1, bn_msc0, bn_msh0, bn_msc1, bn_msh1,
                         nullptr, nullptr, st);
}

// Transposed convolution (nn.ConvTranspose2d, no bias): y[N, Ho, Wo, Cout] from
// x[N, Hi, Wi, Cin] and w[Cin][KH][KW][Cout] (the ConvTranspose2d weight [Cin, Cout, KH, KW]
// with its taps moved before the output channels).  It is the input gradient of the conv
// y -> x with that filter, so it runs the dgrad's parity-class GEMMs (a 4x4 / stride-2
// LinkNet up-conv: 4 classes of 2x2 taps, no structurally-zero products), with the
// following BatchNorm's sum / sum-of-squares in the epilogue as in mlc_conv_fwd.
// The input gradient of this op is mlc_conv_fwd of dy over the same w, its weight
// gradient mlc_conv_wgrad with the roles of x and y swapped.
MLC_EXPORT int mlc_conv_tr_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq, int N, int Hi,
                               int Wi, int Cin, int Cout, int KH, int KW, int stride, int pad, int dil, int Ho,
                               int Wo, hipStream_t st) {
  int pad_h, pad_w;
  unpack_pad(pad, pad_h, pad_w);
  if (Hi != (Ho + 2 * pad_h - dil * (KH - 1) - 1) / stride + 1 || Wi != (Wo + 2 * pad_w - dil * (KW - 1) - 1) / stride + 1)
    return -1;
  return conv_dgrad_impl(x, w, y, nullptr, N, Ho, Wo, Cout, Cin, KH, KW, stride, pad, dil, Hi, Wi, nullptr,
                         nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                         nullptr, sum, sumsq, st);
}

// dgrad from the transposed, flipped filter wt[C][KH][KW][Co] (wtrans.hip), same
// arguments and epilogue (addend, fused BN-backward reduction) as mlc_conv_dgrad.  The
// filter operand is then K-contiguous (ds_read_b128) instead of ConvDgradB's transposed
// LDS reads.  A stride-1 conv's dgrad IS a forward conv of dy over wt with pad' =
// dil*(K-1) - pad, so it runs on the forward loaders; strided convs keep the parity-class
// GEMMs with the ConvDgradBT filter loader.
MLC_EXPORT int mlc_conv_dgrad_t(const bf16* dy, const bf16* wt, bf16* dx, const bf16* addend, int N,
                                int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                                int dil, int Ho, int Wo, const bf16* bn_mask, const bf16* bn_y0,
                                const float* bn_mean0, float* bn_sums0, const bf16* bn_y1,
                                const float* bn_mean1, float* bn_sums1, const float* bn_msc0,
                                const float* bn_msh0, const float* bn_msc1, const float* bn_msh1,
                                hipStream_t st) {
  if (C % 8 || Co % 8 || KH > 15 || KW > 16 || stride < 1) return -1;
  if (bn_msc0 && (!bn_msh0 || !bn_y0 || (bn_msc1 && (!bn_msh1 || !bn_y1)))) return -1;
  if (bn_y0 && (!bn_mean0 || !bn_sums0 || (bn_y1 && (!bn_mean1 || !bn_sums1)))) return -1;
  BnBwdEpi bn{bn_mask, bn_y0, bn_mean0, bn_sums0, bn_y1, bn_mean1, bn_sums1,
              bn_msc0, bn_msh0, bn_msc1, bn_msh1, g_mlc_ncopy};
  if (bn_y0 && g_mlc_det && ((long)N * H * W + 63) / 64 > g_mlc_ncopy) return -2;
  int pad_h, pad_w;
  unpack_pad(pad, pad_h, pad_w);
  const int ph = dil * (KH - 1) - pad_h, pw = dil * (KW - 1) - pad_w;
  if (stride == 1 && ph >= 0 && pw >= 0) {
    if (Ho != H + 2 * pad_h - dil * (KH - 1) || Wo != W + 2 * pad_w - dil * (KW - 1)) return -1;
    const int M = N * H * W, K = KH * KW * Co;
    const int tile = pick_tile(M, C);
    EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}, addend, bn};
#define MKB(R) (MatKC<R>{wt, K, C, K})
    if (KH == 1 && KW == 1) {
#define MKA(R) (MatKC<R>{dy, Co, M, Co})
      MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
#undef MKA
    }
    // geometry of the equivalent forward conv: input dy [N, Ho, Wo, Co], output [N, H, W, C]
    const ConvGeom gf = mkgeom(N, Ho, Wo, Co, C, KH, KW, 1, pack_pad(ph, pw), dil, H, W);
#define MKA(R) (ConvFwdA<R>{dy, gf, M, K})
    MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
#undef MKA
#undef MKB
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  hipError_t err = hipSuccess;
  for (int qh = 0; qh < stride && qh < H; ++qh)
    for (int qw = 0; qw < stride && qw < W; ++qw) {
      const DgradClass cl = mkclass(stride, qh, qw, H, W, Ho, Wo, Co, KH, KW, pad, dil);
      if (cl.nr > 15 || cl.ns > 16) return -1;
      const int M = N * cl.Hc * cl.Wc, K = cl.nr * cl.ns * cl.ncb * BK;
      if (M <= 0) continue;
      const int tile = pick_tile(M, C);
#define MKA(R) (ConvDgradA<R>{dy, g, M, K, cl})
#define MKB(R) (ConvDgradBT<R>{wt, g, cl})
      if (stride == 1) {
        EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}, addend, bn};
        err = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB); }();
      } else {
        EpiBF16<ClassRows> epi{dx, C, nullptr, nullptr, ClassRows{cl, H, W}, addend, bn};
        err = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB); }();
      }
#undef MKA
#undef MKB
      if (err != hipSuccess) return err;
    }
  return err;
}

// dw[Co, KH*KW*C] (fp32) = sum_p dy[p][co] * im2col(x)[p][kk]; zeroes dw first unless
// accumulate != 0.  splits <= 0 picks a split-K factor automatically.
namespace {
// out[i] (+)= sum over splits of ws[s][i]  (float4 per thread)
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, long n4, int splits,
                     long slab4, int accumulate) {
  // ext-vector loads (HIP's float4 struct loads were not batched by hipcc)
  typedef float v4 __attribute__((ext_vector_type(4)));
  const v4* w4 = reinterpret_cast<const v4*>(ws);
  v4* o4 = reinterpret_cast<v4*>(out);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    v4 a = accumulate ? o4[i] : (v4){0.f, 0.f, 0.f, 0.f};
    v4 b = {0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 4 <= splits; k += 4) {  // four independent loads in flight
      const v4 u0 = w4[(k + 0) * slab4 + i], u1 = w4[(k + 1) * slab4 + i];
      const v4 u2 = w4[(k + 2) * slab4 + i], u3 = w4[(k + 3) * slab4 + i];
      a += u0 + u1;
      b += u2 + u3;
    }
    for (; k < splits; ++k) a += w4[k * slab4 + i];
    o4[i] = a + b;
  }
}
}  // namespace

// dw[Co, KH*KW*C] (fp32) = sum_p dy[p][co] * im2col(x)[p][kk]; written, or added to dw
// when accumulate != 0.  splits <= 0 picks a split-K factor automatically.  With a
// workspace (ws_floats >= splits*Co*KK) the split-K partial tiles go to fp32 slabs with
// plain stores and one reduction pass sums them into dw; without, they are added into dw
// with fp32 atomics (memory-side, ~1.3 TB/s: the slab round trip is ~4x cheaper).
// in_sc/in_sh: as in mlc_conv_fwd - x is pre-BN and the conv's input is relu(x*sc + sh).
MLC_EXPORT int mlc_conv_wgrad_native(const bf16* dy, const bf16* x, float* dw, int N, int H, int W,
                              int C, int Co, int KH, int KW, int stride, int pad, int dil,
                              int Ho, int Wo, int splits, int accumulate, float* ws, long ws_floats,
                              const float* in_sc, const float* in_sh, hipStream_t st) {
  if (C % 8 || Co % 8 || ((in_sc == nullptr) != (in_sh == nullptr))) return -1;
  const BnIn bn{in_sc, in_sh};
  const int P = N * Ho * Wo, KK = KH * KW * C;
  const int tile = pick_tile(Co, KK);
  const bool plain = KH == 1 && KW == 1 && stride == 1 && pad == 0;
  const size_t slab = (size_t)Co * KK;
  // slabs pay when the partial sums are large (>= 8 MB: atomics ~1.3 TB/s vs two plain
  // passes ~5 TB/s each) and the reduction has enough elements to fill the chip
  bool use_slab = false;
  if (g_mlc_det) {
    splits = 1;   // one contribution per dw element: exact, order-free
  } else if (splits <= 0) {
    const int ss = auto_splits(Co, KK, P, tile, g_split_target);
    use_slab = ws && slab >= (1u << 18) && (double)ss * slab * 4 >= 8e6 && (long)(ss * slab) <= ws_floats;
    splits = use_slab ? ss : auto_splits(Co, KK, P, tile, plain ? g_split_target_mat : g_split_target);
  } else {
    use_slab = ws && (long)(splits * slab) <= ws_floats;
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
#define MKA(R) (MatMC<R>{dy, Co, P, Co})
  if (use_slab) {
    {  // the launch rounds splits so that no split is empty: size the reduction to it
      const int ktiles = (P + BK - 1) / BK;
      const int per = (ktiles + splits - 1) / splits;
      splits = (ktiles + per - 1) / per;
    }
    const int BMv = tile_bm(tile), BNv = tile_bn(tile);
    if (unsigned* cnt = split_counters(st, (long)((Co + BMv - 1) / BMv) * ((KK + BNv - 1) / BNv), splits, BMv, BNv)) {
      EpiSlabFused epi{ws, KK, slab, cnt, 0, dw, accumulate, {}};
      if (in_sc) {
#define MKB(R) (MatMCBn<R>{{x, C, P, C}, bn})
        if (plain) MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
#define MKB(R) (ConvWgradBBn<R>{{x, g, P, KK}, bn})
        MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
      }
#define MKB(R) (MatMC<R>{x, C, P, C})
      if (plain) MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
#define MKB(R) (ConvWgradB<R>{x, g, P, KK})
      MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
    }
    EpiF32Slab epi{ws, KK, slab};
    hipError_t e;
    if (in_sc) {
#define MKB(R) (MatMCBn<R>{{x, C, P, C}, bn})
      if (plain) e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
#define MKB(R) (ConvWgradBBn<R>{{x, g, P, KK}, bn})
      else e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
    } else {
#define MKB(R) (MatMC<R>{x, C, P, C})
      if (plain) e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
#define MKB(R) (ConvWgradB<R>{x, g, P, KK})
      else e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
    }
    if (e != hipSuccess) return e;
    const long n4 = (long)slab / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, dw, n4, splits,
                       (long)slab / 4, accumulate);
    return hipGetLastError();
  }
  if (!accumulate) mlc_zero_f32(dw, (long)slab, st);
  EpiF32Atomic epi{dw, KK};
  if (in_sc) {
    if (plain) {
#define MKB(R) (MatMCBn<R>{{x, C, P, C}, bn})
      MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
    }
#define MKB(R) (ConvWgradBBn<R>{{x, g, P, KK}, bn})
    MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
  }
  if (plain) {
#define MKB(R) (MatMC<R>{x, C, P, C})
    MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
  }
#define MKB(R) (ConvWgradB<R>{x, g, P, KK})
  MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
#undef MKA
}

// Conv forward with a dense epilogue: y = act(conv(x, w) + bias) (act 0 / 3 = ReLU; the
// GELU codes of the dense layers apply too) - the generic engine's convs that carry a bias
// and no BatchNorm (LeNet-style nets, 1x1 squeeze-excitation convs, segmentation heads).
MLC_EXPORT int mlc_conv_fwd_ex(const bf16* x, const bf16* w, bf16* y, const float* bias, int act, int N, int H,
                               int W, int C, int Co, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo,
                               hipStream_t st) {
  if (C % 8 || Co % 8 || KH > 15 || KW > 16) return -1;
  const int M = N * Ho * Wo, K = KH * KW * C;
  const int tile = pick_tile(M, Co);
  EpiBF16<IdentityRows, true> epi{y, Co, nullptr, nullptr, IdentityRows{}, nullptr};
  epi.bias = bias;
  epi.act = act;
#define MKB(R) (MatKC<R>{w, K, Co, K})
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
#define MKA(R) (MatKC<R>{x, C, M, K})
    MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
#define MKA(R) (ConvFwdA<R>{x, g, M, K})
  MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
#undef MKB
}

// Conv weight gradient plus the bias gradient: dw[Co][KH*KW*C] (+)= as mlc_conv_wgrad and
// dbias[Co] += the column sums of dy, summed from dy's staged tiles (MatMCSum) in the same
// GEMM.  Split-K partial tiles go to fp32 slabs of ws (+ one reduction pass) when it is big
// enough, else fp32 atomics.
MLC_EXPORT int mlc_conv_wgrad_bias(const bf16* dy, const bf16* x, float* dw, float* dbias, int N, int H, int W,
                                   int C, int Co, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo,
                                   int accumulate, float* ws, long ws_floats, hipStream_t st) {
  if (C % 8 || Co % 8 || !dbias) return -1;
  const int P = N * Ho * Wo, KK = KH * KW * C;
  const int tile = pick_tile(Co, KK);
  const bool plain = KH == 1 && KW == 1 && stride == 1 && pad == 0;
  const size_t slab = (size_t)Co * KK;
  int splits = g_mlc_det ? 1 : auto_splits(Co, KK, P, tile, plain ? g_split_target_mat : g_split_target);
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
#define MKA(R) (MatMCSum<R>{dy, Co, P, Co, dbias})
  if (ws && splits > 1 && (long)(splits * slab) <= ws_floats) {
    const int ktiles = (P + BK - 1) / BK;
    const int per = (ktiles + splits - 1) / splits;
    splits = (ktiles + per - 1) / per;
    EpiF32Slab epi{ws, KK, slab};
    hipError_t e;
#define MKB(R) (MatMC<R>{x, C, P, C})
    if (plain) e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
#define MKB(R) (ConvWgradB<R>{x, g, P, KK})
    else e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB); }();
#undef MKB
    if (e != hipSuccess) return e;
    const long n4 = (long)slab / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, dw, n4, splits, n4, accumulate);
    return hipGetLastError();
  }
  if (!accumulate) mlc_zero_f32(dw, (long)slab, st);
  EpiF32Atomic epi{dw, KK};
  if (plain) {
#define MKB(R) (MatMC<R>{x, C, P, C})
    MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
  }
#define MKB(R) (ConvWgradB<R>{x, g, P, KK})
  MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
#undef MKA
}

// Generic bf16 GEMM with fp32 output: C[M][N] (+)= op(A) op(B) (+ bias)
//   ta=0: A is [M][K] (lda);  ta=1: A is [K][M]
//   tb=0: B is [K][N] (ldb);  tb=1: B is [N][K]
// out_mode 0: store (+bias, accumulate flag), 1: atomic add (split-K allowed; the
// caller zeroes C unless accumulating)
#define GA_KC(R) (MatKC<R>{A, lda, M, K})
#define GA_MC(R) (MatMC<R>{A, lda, K, M})
#define GB_KC(R) (MatKC<R>{B, ldb, N, K})
#define GB_MC(R) (MatMC<R>{B, ldb, K, N})

MLC_EXPORT int mlc_gemm_f32out(const bf16* A, const bf16* B, float* C, const float* bias,
                               int M, int N, int K, int lda, int ldb, int ldc, int ta, int tb,
                               int out_mode, int accumulate, int splits, hipStream_t st) {
  if (K % 8 || lda % 8 || ldb % 8 || (ta && M % 8) || (!tb && N % 8)) return -1;
  const int tile = pick_tile(M, N);
  if (out_mode == 1) {
    if (splits <= 0) splits = auto_splits(M, N, K, tile, g_split_target_dense);
    if (g_mlc_det) splits = 1;
    EpiF32Atomic epi{C, ldc};
    if (!ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_KC, GB_KC);
    if (!ta && !tb) MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_KC, GB_MC);
    if (ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_MC, GB_KC);
    MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_MC, GB_MC);
  }
  EpiF32 epi{C, ldc, bias, accumulate};
  if (!ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_KC);
  if (!ta && !tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_MC);
  if (ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_KC);
  MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_MC);
}

// Dense-layer weight + bias gradient in one GEMM: dW[M][N] += dY^T X (fp32 atomics,
// split-K) and dbias[M] += column sums of dY, taken from dY's staged tiles.  dY [K][M]
// (lda), X [K][N] (ldb), M % 8 == N % 8 == 0.
// With a workspace (ws_floats >= splits*M*N, ldc == N) the split-K partial tiles go to fp32
// slabs and one reduction pass adds their sum into dW; otherwise fp32 atomics into dW.
MLC_EXPORT int mlc_linear_wgrad_bias_native(const bf16* A, const bf16* B, float* C, float* dbias, int M, int N, int K,
                                     int lda, int ldb, int ldc, int splits, float* ws, long ws_floats,
                                     hipStream_t st) {
  if (K % 8 || lda % 8 || ldb % 8 || M % 8 || N % 8) return -1;
  const int tile = pick_tile(M, N);
  if (splits <= 0) splits = auto_splits(M, N, K, tile, g_split_target_dense);
  if (g_mlc_det) splits = 1;   // one dW atomic and one bias column-sum add per element
  const size_t slab = (size_t)M * N;
#define GA_MCS(R) (MatMCSum<R>{A, lda, K, M, dbias})
  if (ws && ldc == N && splits > 1 && (long)(splits * slab) <= ws_floats) {
    const int ktiles = (K + BK - 1) / BK;
    const int per = (ktiles + splits - 1) / splits;
    splits = (ktiles + per - 1) / per;
    const int BMv = tile_bm(tile), BNv = tile_bn(tile);
    if (unsigned* cnt = split_counters(st, (long)((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv), splits, BMv, BNv)) {
      EpiSlabFused epi{ws, N, slab, cnt, 0, C, 1, {}};
      MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_MCS, GB_MC);
    }
    EpiF32Slab epi{ws, N, slab};
    const hipError_t e = [&]() -> hipError_t { MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_MCS, GB_MC); }();
    if (e != hipSuccess) return e;
    const long n4 = (long)slab / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, C, n4, splits, n4, 1);
    return hipGetLastError();
  }
  EpiF32Atomic epi{C, ldc};
  MLC_TILE_DISPATCH(tile, M, N, K, splits, st, epi, GA_MCS, GB_MC);
#undef GA_MCS
}

// bf16-output GEMM with a dense-layer epilogue: C = act(op(A) op(B) + bias) (pre-
// activation to preact when given), or C = (op(A) op(B)) * act'(dact) (+ addend).

// non-returning tile dispatch (for callers that continue after the GEMM)
template <class EPI, class FA, class FB>
static hipError_t launch_tiles(int tile, int M, int N, int K, int splits, hipStream_t st, const EPI& epi, FA fa,
                               FB fb) {
  if (tile == 1) return launch<256, 64>(fa.template make<256>(), fb.template make<64>(), epi, M, N, K, splits, st);
  if (tile == 2) return launch<64, 256>(fa.template make<64>(), fb.template make<256>(), epi, M, N, K, splits, st);
  if (tile == 3) return launch<256, 128>(fa.template make<256>(), fb.template make<128>(), epi, M, N, K, splits, st);
  if (tile == 4) return launch<128, 256>(fa.template make<128>(), fb.template make<256>(), epi, M, N, K, splits, st);
  return launch<128, 128>(fa.template make<128>(), fb.template make<128>(), epi, M, N, K, splits, st);
}
struct MkMatKC { const bf16* p; int ld, rows, K; template <int R> MatKC<R> make() const { return MatKC<R>{p, ld, rows, K}; } };
struct MkMatMC { const bf16* p; int ld, K, cols; template <int R> MatMC<R> make() const { return MatMC<R>{p, ld, K, cols}; } };
#define GA_KC_F (MkMatKC{A, lda, M, K})
#define GA_MC_F (MkMatMC{A, lda, K, M})
#define GB_KC_F (MkMatKC{B, ldb, N, K})
#define GB_MC_F (MkMatMC{B, ldb, K, N})

namespace {
// Split-K finish for the dense GEMM: ws holds `splits` fp32 slabs [splits][M][N] of
// partial sums (written with plain stores by EpiF32Slab); C = epilogue(sum of slabs).
__global__ void __launch_bounds__(256)
dense_finalize_kernel(const float* __restrict__ ws, int splits, DenseFinish fin, int M, int N) {
  const int G = N / 8;
  const int n8 = M * G;                    // < 2^31 for every dense layer here
  const size_t slab = (size_t)M * N;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n8; i += gridDim.x * 256) {
    const int m = i / G, c = (i - m * G) * 8;
    fin.run(ws, slab, splits, (size_t)m * N + c, m, c);
  }
}
}  // namespace

// bf16-output GEMM with a dense-layer epilogue: C = act(op(A) op(B) + bias) (pre-
// activation to preact when given), or C = (op(A) op(B)) * act'(dact) (+ addend).
// ws (optional, ws_floats fp32, any contents): when the output has too few tiles to fill
// the chip, the K reduction is split across workgroups into per-split fp32 slabs of ws
// (plain stores: ~4x cheaper than fp32 atomics into one buffer) and the epilogue runs in a
// finishing pass that sums the slabs.
MLC_EXPORT int mlc_gemm_bf16_ex_native(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int lda, int ldb,
                                int ldc, int ta, int tb, const float* bias, int act, bf16* preact,
                                const bf16* addend, const bf16* dact, float* ws, long ws_floats,
                                hipStream_t st) {
  if (K % 8 || N % 8 || ldc % 8 || lda % 8 || ldb % 8 || (ta && M % 8)) return -1;
  const int ktiles = (K + BK - 1) / BK;
  const long slab = (long)M * N;
  if (!ta && tb) {  // both operands K-contiguous: the three-wide tiles apply
    int dsplit = 1;
    const int dt = pick_dense_tile(M, N, K, dsplit);
    if (dt >= 5 && dt <= 7) {
      if (dsplit > 1 && ws && slab * dsplit <= ws_floats && ktiles >= 2 * dsplit) {
        const int per = (ktiles + dsplit - 1) / dsplit;
        dsplit = (ktiles + per - 1) / per;
        EpiF32Slab epi{ws, N, (size_t)slab};
        hipError_t e = dt == 5 ? launch<128, 96>(GA_KC(128), GB_KC(96), epi, M, N, K, dsplit, st)
                     : dt == 6 ? launch<128, 192>(GA_KC(128), GB_KC(192), epi, M, N, K, dsplit, st)
                               : launch<128, 288>(GA_KC(128), GB_KC(288), epi, M, N, K, dsplit, st);
        if (e != hipSuccess) return e;
        const DenseFinish fin{C, ldc, bias, act, preact, addend, dact};
        long blocks = ((long)M * (N / 8) + 255) / 256;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL(dense_finalize_kernel, dim3(blocks), dim3(256), 0, st, ws, dsplit, fin, M, N);
        return hipGetLastError();
      }
      EpiBF16<IdentityRows, true> epi{C, ldc, nullptr, nullptr, IdentityRows{}, addend};
      epi.bias = bias; epi.act = act; epi.preact = preact; epi.dact = dact;
      if (dt == 5) return launch<128, 96>(GA_KC(128), GB_KC(96), epi, M, N, K, 1, st);
      if (dt == 6) return launch<128, 192>(GA_KC(128), GB_KC(192), epi, M, N, K, 1, st);
      return launch<128, 288>(GA_KC(128), GB_KC(288), epi, M, N, K, 1, st);
    }
  }
  const int tile = pick_tile(M, N);
  const int BMv = tile_bm(tile), BNv = tile_bn(tile);
  const int tiles = ((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv);
  int splits = 1;
  // a narrow output (N <= 1024, e.g. BERT's 768-wide projections) on 128x64 tiles fills
  // the chip without split-K: no fp32 slabs, no finalize pass (MLC_DENSE_NARROW=1; measured
  // neutral on the BERT-base step against split-K 2 + finalize, so off by default)
  if (g_dense_narrow < 0) {
    const char* e = getenv("MLC_DENSE_NARROW");
    g_dense_narrow = e ? atoi(e) : 0;
  }
  if (g_dense_narrow && tile == 0 && N <= 1024 && tiles < 256 && ((M + 127) / 128) * ((N + 63) / 64) >= 256) {
    EpiBF16<IdentityRows, true> epi{C, ldc, nullptr, nullptr, IdentityRows{}, addend};
    epi.bias = bias; epi.act = act; epi.preact = preact; epi.dact = dact;
    if (!ta && tb) return launch<128, 64>(GA_KC(128), GB_KC(64), epi, M, N, K, 1, st);
    if (!ta && !tb) return launch<128, 64>(GA_KC(128), GB_MC(64), epi, M, N, K, 1, st);
  }
  if (ws)
    while (tiles * splits < g_dense_bf16_split_target && ktiles / (splits * 2) >= 4 && slab * splits * 2 <= ws_floats)
      splits *= 2;
  if (splits > 1) {
    {  // the launch rounds splits so that no split is empty: finish exactly those slabs
      const int per = (ktiles + splits - 1) / splits;
      splits = (ktiles + per - 1) / per;
    }
    const DenseFinish fin{C, ldc, bias, act, preact, addend, dact};
    if (unsigned* cnt = split_counters(st, tiles, splits, BMv, BNv)) {
      EpiSlabFused epi{ws, N, (size_t)slab, cnt, 1, nullptr, 0, fin};
      if (!ta && tb) return launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_KC_F);
      if (!ta && !tb) return launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_MC_F);
      if (ta && tb) return launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_KC_F);
      return launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_MC_F);
    }
    EpiF32Slab epi{ws, N, (size_t)slab};
    hipError_t e;
    if (!ta && tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_KC_F);
    else if (!ta && !tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_MC_F);
    else if (ta && tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_KC_F);
    else e = launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_MC_F);
    if (e != hipSuccess) return e;
    long blocks = ((long)M * (N / 8) + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(dense_finalize_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, fin, M, N);
    return hipGetLastError();
  }
  EpiBF16<IdentityRows, true> epi{C, ldc, nullptr, nullptr, IdentityRows{}, addend};
  epi.bias = bias; epi.act = act; epi.preact = preact; epi.dact = dact;
  if (!ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_KC);
  if (!ta && !tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_MC);
  if (ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_KC);
  MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_MC);
}

// bf16-output GEMM (same layout flags)
MLC_EXPORT int mlc_gemm_bf16out(const bf16* A, const bf16* B, bf16* C, int M, int N, int K,
                                int lda, int ldb, int ldc, int ta, int tb, hipStream_t st) {
  if (K % 8 || N % 8 || ldc % 8 || lda % 8 || ldb % 8 || (ta && M % 8)) return -1;
  const int tile = pick_tile(M, N);
  EpiBF16<> epi{C, ldc, nullptr, nullptr, IdentityRows{}};
  if (!ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_KC);
  if (!ta && !tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_KC, GB_MC);
  if (ta && tb) MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_KC);
  MLC_TILE_DISPATCH(tile, M, N, K, 1, st, epi, GA_MC, GB_MC);
}
