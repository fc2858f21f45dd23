// 256-row bf16 GEMM engine for gfx950: 8 waves, LDS-DMA staging, phase-interleaved.
//
//   C[M][N] = sum_k A[m][k] B[n][k]      A: 256-row block tile, B: BN = 256 or 128 columns
//
// Structure (cdna_hip_programming.md §5 "The 256^2 8-phase template", re-derived here):
// * 512 threads = 8 waves; BN = 256: waves 2 (M) x 4 (N), each owns 128x64 of C;
//   BN = 128: waves 4 x 2, each owns 64x64.  A wave's output is split into four
//   quadrants, one per (A half, B half) pair: a phase multiplies one A half (128 rows)
//   by one B half (BN/2 columns);
// * the four half-tiles (A0 A1 B0 B1) of a K-step are copied global -> LDS by
//   buffer_load ... lds (no VGPR round trip; a load past the operand, or a padding tap of
//   an implicit-GEMM conv, reads zero), two buffers, so K-step t+1 streams in while t
//   is multiplied;
// * four phases per K-step: {fragment reads of the half that becomes live; LDS-DMA issue
//   of one half of K-step t+1; counted s_waitcnt vmcnt for the half the NEXT phase reads;
//   s_barrier; v_mfma_f32_16x16x32_bf16 cluster}.  vmcnt is never 0 inside the loop: two to
//   three half-tiles stay in flight across every barrier;
// * LDS images (the DMA destination is lane-linear, so every swizzle is applied to the
//   per-lane SOURCE address and undone on the read):
//     K-contiguous operand ("KC", [rows][K]): R rows x 128 B, chunk c of row r in slot
//     c ^ ((r>>1)&7); fragments by ds_read_b128, conflict-free;
//     MN-contiguous operand ("MC", [K][cols]): 64 k-rows x 2R B, 16-B slot s of k-row r in
//     slot s ^ mcswz(r); fragments by two ds_read_b64_tr_b16, conflict-free;
// * the MFMA computes C^T tiles (B fragment as the A operand), so each lane ends with 4
//   consecutive columns of one output row: 8-byte stores straight from registers.
#include "common.h"
#include "convgeom.h"

namespace g256 {

using igemm::ConvGeom;
using igemm::FastDiv;
using igemm::NSTAT;
using igemm::tap_pat;
using igemm::NO_TAP;

constexpr int BM = 256, BK = 64, NTHR = 512;
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ Rsrc rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ void bar() { asm volatile("s_barrier" ::: "memory"); }
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void dma16(Rsrc rs, char* dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
}

// --------------------------------------------------------------------- LDS images
__device__ __forceinline__ int kcswz(int r) { return (r >> 1) & 7; }
template <int R> __device__ __forceinline__ int mcswz(int r) {
  if constexpr (R == 128) return ((r & 3) | (((r >> 3) & 1) << 2)) << 1;   // 256-B k-rows
  else return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;               // 128-B k-rows
}
// every operand half image is R rows/cols x 64 k = R * 128 B, copied by R/64 DMA
// wave-instructions (1 KiB each) per wave
template <int R> struct Img {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int NC = R / 64;
  // KC: copy c of wave w -> image rows (w*NC + c)*8 + lane/8, slot lane%8
  __device__ static int kc_row(int w, int c, int lane) { return (w * NC + c) * 8 + (lane >> 3); }
  __device__ static int kc_chunk(int w, int c, int lane) { return (lane & 7) ^ kcswz(kc_row(w, c, lane)); }
  // MC: copy c of wave w -> k-rows (w*NC + c)*(512/R) + lane/(R/8), slot lane%(R/8)
  __device__ static int mc_krow(int w, int c, int lane) { return (w * NC + c) * (512 / R) + lane / (R / 8); }
  __device__ static int mc_col(int w, int c, int lane) {   // first mn column of the 16-B chunk copied
    return ((lane % (R / 8)) ^ mcswz<R>(mc_krow(w, c, lane))) * 8;
  }
};

// fragments: 16 rows (rb..rb+15) x 32 k (k-step kk) of a half image, operand layout of
// v_mfma_f32_16x16x32_bf16 (lane l: row l&15, k = 8(l>>4) + e)
__device__ __forceinline__ bf16x8 frag_kc(const char* img, int rb, int kk, int lane) {
  const int r = rb + (lane & 15), c = kk * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * 128 + ((c ^ kcswz(r)) << 4));
}
template <int R>
__device__ __forceinline__ bf16x8 frag_mc(const char* img, int rb, int kk, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = rb + 4 * p;
  const int k0 = kk * 32 + 8 * g + q;
  auto addr = [&](int kr) {
    return img + kr * (2 * R) + ((((col >> 3) ^ mcswz<R>(kr))) << 4) + ((col & 7) << 1);
  };
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(addr(k0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(addr(k0 + 4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
template <class L, int R>
__device__ __forceinline__ bf16x8 frag(const char* img, int rb, int kk, int lane) {
  if constexpr (L::KC) return frag_kc(img, rb, kk, lane);
  else return frag_mc<R>(img, rb, kk, lane);
}

// --------------------------------------------------------------------- operands
// Interface: init(st, r0, tid) for the block's first row/col r0; copy(st, r0, h, kt, dead,
// dst, tid) issues the DMA of half h (rows r0 + h*R ..) of K-tile kt into `dst`; `dead`
// (OOB or 0, wave-uniform) turns a copy past the last K-tile into a zero read.

// K-contiguous matrix [rows][ld].  HR (<= R): rows of a half that are used - a 192-wide
// block tile stages its 96-row B halves in 128-row images whose last 32 rows read zero
// (OOB: no memory traffic) and are never multiplied.
template <int R, bool KTAIL, int HR = R>
struct MatKC {
  static constexpr bool KC = true;
  static constexpr int NC = R / 64;
  const bf16* p; int ld, rows, K;
  struct St { unsigned off[2][NC]; unsigned kc[NC]; };
  __device__ void init(St& st, int r0, int tid) const {
    const int w = tid >> 6, l = tid & 63;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int r = Img<R>::kc_row(w, c, l), ch = Img<R>::kc_chunk(w, c, l);
      st.kc[c] = (unsigned)ch * 8u;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        st.off[h][c] = r < HR && r0 + h * HR + r < rows ? (unsigned)(r * ld + ch * 8) * 2u : OOB;
    }
  }
  __device__ void copy(const St& st, int r0, int h, int kt, unsigned dead, char* dst, int tid) const {
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k0 = kt * BK;
    const Rsrc rs = rsrc(p + (size_t)(r0 + h * HR) * ld + k0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      unsigned v = st.off[h][c] | dead;
      if constexpr (KTAIL) v = (int)st.kc[c] < K - k0 ? v : OOB;
      dma16(rs, dst + (w * NC + c) * 1024, v);
    }
  }
};

// MN-contiguous matrix [K][ld] (the operand's rows are its columns); HR as in MatKC
template <int R, bool KTAIL, int HR = R>
struct MatMC {
  static constexpr bool KC = false;
  static constexpr int NC = R / 64;
  const bf16* p; int ld, K, cols;
  struct St { unsigned off[2][NC]; int kr[NC]; };
  __device__ void init(St& st, int r0, int tid) const {
    const int w = tid >> 6, l = tid & 63;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int kr = Img<R>::mc_krow(w, c, l), col = Img<R>::mc_col(w, c, l);
      st.kr[c] = kr;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        st.off[h][c] = col < HR && r0 + h * HR + col < cols ? (unsigned)(kr * ld + col) * 2u : OOB;
    }
  }
  __device__ void copy(const St& st, int r0, int h, int kt, unsigned dead, char* dst, int tid) const {
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k0 = kt * BK;
    const Rsrc rs = rsrc(p + (size_t)k0 * ld + r0 + h * HR);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      unsigned v = st.off[h][c] | dead;
      if constexpr (KTAIL) v = st.kr[c] < K - k0 ? v : OOB;
      dma16(rs, dst + (w * NC + c) * 1024, v);
    }
  }
};

// implicit-GEMM conv forward A operand: rows = output pixels (n, ho, wo), k = (r, s, ci)
// with ci fastest (NHWC x, [Co][KH][KW][C] weights).  Per copy: the row's offset from the
// half's first row and its filter-tap mask (bit r: row r of the filter lands inside the
// input, bit 16+s: column s does); a chunk of tap (r, s) is read iff (mask & P) == P.
template <int R, bool KTAIL>
struct ConvFwdA {
  static constexpr bool KC = true;
  static constexpr int NC = R / 64;
  const bf16* x; ConvGeom g; int M, K;
  struct St { unsigned off[2][NC], msk[2][NC]; long long b0[2]; unsigned kc[NC]; };
  __device__ long long rowoff(int m, int& hb, int& wb) const {
    unsigned t, wo, n, ho;
    g.fWo.divmod((unsigned)m, t, wo);
    g.fHo.divmod(t, n, ho);
    hb = (int)ho * g.stride - g.pad;
    wb = (int)wo * g.stride - g.padw;
    return (((long long)n * g.H + hb) * g.W + wb) * g.C;
  }
  __device__ void init(St& st, int r0, int tid) const {
    const int w = tid >> 6, l = tid & 63;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int hb, wb;
      const int mh = min(r0 + h * R, M - 1);
      st.b0[h] = rowoff(mh, hb, wb);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int m = r0 + h * R + Img<R>::kc_row(w, c, l);
        const bool ok = m < M;
        const long long o = rowoff(ok ? m : mh, hb, wb);
        st.off[h][c] = (unsigned)(o - st.b0[h]) * 2u;
        unsigned mk = 0;
        for (int r = 0; r < g.KH; ++r) mk |= ((unsigned)(hb + r * g.dil) < (unsigned)g.H) ? (1u << r) : 0u;
        for (int s = 0; s < g.KW; ++s) mk |= ((unsigned)(wb + s * g.dil) < (unsigned)g.W) ? (1u << (16 + s)) : 0u;
        st.msk[h][c] = ok ? mk : 0u;
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) st.kc[c] = (unsigned)Img<R>::kc_chunk(w, c, l) * 8u;
  }
  __device__ void copy(const St& st, int r0, int h, int kt, unsigned dead, char* dst, int tid) const {
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k0 = kt * BK;
    const Rsrc rsr = rsrc(x + st.b0[h]);
    if (g.C % BK == 0) {   // the whole K-tile is one filter tap: uniform decomposition
      unsigned rs_, cc, rr, ss;
      g.fC.divmod((unsigned)k0, rs_, cc);
      g.fKW.divmod(rs_, rr, ss);
      const unsigned P = tap_pat((int)rr, (int)ss);
      const unsigned toff = (unsigned)(((int)rr * g.dil * g.W + (int)ss * g.dil) * g.C + (int)cc) * 2u;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const unsigned v = (st.msk[h][c] & P) == P ? (st.off[h][c] + toff + st.kc[c] * 2u) | dead : OOB;
        dma16(rsr, dst + (w * NC + c) * 1024, v);
      }
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int k = k0 + (int)st.kc[c];
        unsigned rs_, cc, rr, ss;
        g.fC.divmod((unsigned)k, rs_, cc);
        g.fKW.divmod(rs_, rr, ss);
        const unsigned P = k < K ? tap_pat((int)rr, (int)ss) : NO_TAP;
        const unsigned toff = (unsigned)(((int)rr * g.dil * g.W + (int)ss * g.dil) * g.C + (int)cc) * 2u;
        const unsigned v = (st.msk[h][c] & P) == P ? (st.off[h][c] + toff) | dead : OOB;
        dma16(rsr, dst + (w * NC + c) * 1024, v);
      }
    }
  }
};

// --------------------------------------------------------------------- epilogues
// acc quad -> C[m][n .. n+3] (n % 4 == 0); `last` hooks run once per block.

// bf16 (dense: + bias, GELU, pre-activation copy, + addend) or fp32 (store / accumulate)
template <int FP32OUT>
struct EpiOut {
  bf16* c; float* cf; int ldc;
  const float* bias;       // [N] fp32, added before the activation
  int act;                 // 1 = exact-erf GELU
  bf16* preact;            // optional: pre-activation (bias added) store, ldc layout
  const bf16* addend;      // optional: + addend (residual), ldc layout
  int accumulate;          // fp32 out: C += result
  static constexpr bool STATS = false;
  __device__ __forceinline__ void quad(int m, int n, f32x4 v) const {
    float a[4] = {v[0], v[1], v[2], v[3]};
    const size_t o = (size_t)m * ldc + n;
    if (bias) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += b[q];
    }
    if constexpr (FP32OUT) {
      f32x4* dst = reinterpret_cast<f32x4*>(cf + o);
      f32x4 r = {a[0], a[1], a[2], a[3]};
      if (accumulate) r += *dst;
      *dst = r;
      return;
    }
    if (preact) *reinterpret_cast<uint2*>(preact + o) = make_uint2(pack2_bf16(a[0], a[1]), pack2_bf16(a[2], a[3]));
    if (act == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = 0.5f * a[q] * (1.f + erff(a[q] * 0.70710678118654752f));
    }
    if (addend) {
      const uint2 u = *reinterpret_cast<const uint2*>(addend + o);
      a[0] += __uint_as_float(u.x << 16); a[1] += __uint_as_float(u.x & 0xffff0000u);
      a[2] += __uint_as_float(u.y << 16); a[3] += __uint_as_float(u.y & 0xffff0000u);
    }
    *reinterpret_cast<uint2*>(c + o) = make_uint2(pack2_bf16(a[0], a[1]), pack2_bf16(a[2], a[3]));
  }
};

// dense-layer epilogue with igemm.hip's DenseFinish semantics, four columns at a time:
//   a = acc + bias;  act & 3: 0 none / 1 exact-erf GELU (u -> preact) / 2 GELU with the
//   derivative gelu'(u) -> preact / 3 ReLU (pre-activation -> preact);  a *= act'(dact)
//   (act & 4: dact holds the derivative; act 3: ReLU mask);  a += addend;  bf16 store
__device__ __forceinline__ float erf_e(float x, float e) {   // erf(x) from e = exp(-x*x), A&S 7.1.26
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * fabsf(x));
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  return copysignf(1.f - p * e, x);
}
struct EpiDense {
  bf16* c; int ldc; const float* bias; int act; bf16* preact; const bf16* addend; const bf16* dact;
  static constexpr bool STATS = false;
  __device__ __forceinline__ static uint2 pk(const float (&a)[4]) {
    return make_uint2(pack2_bf16(a[0], a[1]), pack2_bf16(a[2], a[3]));
  }
  __device__ __forceinline__ static void unpk(uint2 u, float (&z)[4]) {
    z[0] = __uint_as_float(u.x << 16); z[1] = __uint_as_float(u.x & 0xffff0000u);
    z[2] = __uint_as_float(u.y << 16); z[3] = __uint_as_float(u.y & 0xffff0000u);
  }
  __device__ __forceinline__ void quad(int m, int n, f32x4 v) const {
    float a[4] = {v[0], v[1], v[2], v[3]};
    const size_t o = (size_t)m * ldc + n;
    if (bias) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += b[q];
    }
    const int mode = act & 3;
    if (mode == 2) {
      float d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float u = a[q], ex = __expf(-0.5f * u * u);
        const float cdf = 0.5f * (1.f + erf_e(u * 0.70710678118654752f, ex));
        d[q] = cdf + u * 0.3989422804014327f * ex;
        a[q] = u * cdf;
      }
      if (preact) *reinterpret_cast<uint2*>(preact + o) = pk(d);
    } else {
      if (preact) *reinterpret_cast<uint2*>(preact + o) = pk(a);
      if (mode == 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          a[q] = 0.5f * a[q] * (1.f + erf_e(a[q] * 0.70710678118654752f, __expf(-0.5f * a[q] * a[q])));
      } else if (mode == 3) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = fmaxf(a[q], 0.f);
      }
    }
    if (dact) {
      float z[4];
      unpk(*reinterpret_cast<const uint2*>(dact + o), z);
      if (act & 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] *= z[q];
      } else if (mode == 3) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = z[q] > 0.f ? a[q] : 0.f;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float ex = __expf(-0.5f * z[q] * z[q]);
          a[q] *= 0.5f * (1.f + erf_e(z[q] * 0.70710678118654752f, ex)) + z[q] * 0.3989422804014327f * ex;
        }
      }
    }
    if (addend) {
      float b[4];
      unpk(*reinterpret_cast<const uint2*>(addend + o), b);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += b[q];
    }
    *reinterpret_cast<uint2*>(c + o) = pk(a);
  }
};

// conv forward: bf16 y store + per-channel BatchNorm partial sums of y and y^2 (of the
// bf16-rounded values) into NSTAT copies [NSTAT][N]
struct EpiConvStats {
  bf16* y; int ldc; float* sum; float* sumsq;
  static constexpr bool STATS = true;
  __device__ __forceinline__ f32x4 quad(int m, int n, f32x4 v) const {
    const uint2 u = make_uint2(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]));
    *reinterpret_cast<uint2*>(y + (size_t)m * ldc + n) = u;
    return (f32x4){__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
  }
};

// --------------------------------------------------------------------- kernel
template <int BN> struct Cfg {
  static constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  static constexpr int RB = BN / 2;                      // B half rows (columns of C)
  static constexpr int RBI = (RB + 63) / 64 * 64;        // rows of a B half's LDS image
  static constexpr int MT = 128 / WM / 16, NT = RB / WN / 16;   // 16x16 tiles per wave per half
  static constexpr int CA = 2, CB = RBI / 64;            // DMA copies per wave per half
  static constexpr int STAGE = 2 * Img<128>::BYTES + 2 * Img<RBI>::BYTES;
  static_assert(NT * WN * 16 == RB && MT * WM * 16 == 128, "tile / wave decomposition");
};

template <int BN, class LA, class LB, class EPI>
__global__ void __launch_bounds__(NTHR, 2)
gemm_kernel(const LA la, const LB lb, const EPI epi, int M, int N, int K) {
  using C = Cfg<BN>;
  constexpr int RA = 128, RB = C::RB, RBI = C::RBI, MT = C::MT, NT = C::NT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * C::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / C::WN, wc = wave % C::WN;

  // tile order: bijective XCD remap, then groups of 4 M-tiles sweeping N (L2 reuse)
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int id = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  constexpr int GM = 4;
  const int group = id / (GM * tiles_n), first_m = group * GM;
  const int gsize = min(tiles_m - first_m, GM);
  const int in_g = id % (GM * tiles_n);
  const int m0 = (first_m + in_g % gsize) * BM, n0 = (in_g / gsize) * BN;

  typename LA::St sa;
  typename LB::St sb;
  la.init(sa, m0, tid);
  lb.init(sb, n0, tid);
  const int nt = (K + BK - 1) / BK;

  f32x4 acc[2][2][MT][NT];   // [A half][B half][m-tile][n-tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto imgA = [&](int buf, int h) { return smem + buf * C::STAGE + h * Img<RA>::BYTES; };
  auto imgB = [&](int buf, int h) { return smem + buf * C::STAGE + 2 * Img<RA>::BYTES + h * Img<RBI>::BYTES; };

  // prologue: K-tile 0 into buffer 0, halves in the order the phases first read them
  la.copy(sa, m0, 0, 0, 0u, imgA(0, 0), tid);
  lb.copy(sb, n0, 0, 0, 0u, imgB(0, 0), tid);
  lb.copy(sb, n0, 1, 0, 0u, imgB(0, 1), tid);
  la.copy(sa, m0, 1, 0, 0u, imgA(0, 1), tid);
  vmwait<C::CA + C::CB>();   // A0, B0 landed (this wave)
  bar();                     // ... for every wave

  bf16x8 af[MT][2], bf0[NT][2], bf1[NT][2];
  auto mma = [&](int ha, int hb, bf16x8 (&bfr)[NT][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[ha][hb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[ha][hb][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto rdA = [&](const char* img) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = frag<LA, RA>(img, wr * (MT * 16) + 16 * i, kk, lane);
  };
  auto rdB = [&](const char* img, bf16x8 (&bfr)[NT][2]) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bfr[j][kk] = frag<LB, RBI>(img, wc * (NT * 16) + 16 * j, kk, lane);
  };

  for (int t = 0; t < nt; ++t) {
    const int b = t & 1, nb = b ^ 1;
    const unsigned dead = t + 1 < nt ? 0u : OOB;
    // P1: A0 x B0
    rdA(imgA(b, 0));
    rdB(imgB(b, 0), bf0);
    la.copy(sa, m0, 0, t + 1, dead, imgA(nb, 0), tid);
    lb.copy(sb, n0, 0, t + 1, dead, imgB(nb, 0), tid);
    vmwait<2 * C::CA + C::CB>();   // B1(t)
    bar();
    mma(0, 0, bf0);
    // P2: A0 x B1
    rdB(imgB(b, 1), bf1);
    lb.copy(sb, n0, 1, t + 1, dead, imgB(nb, 1), tid);
    vmwait<C::CA + 2 * C::CB>();   // A1(t)
    bar();
    mma(0, 1, bf1);
    // P3: A1 x B1
    rdA(imgA(b, 1));
    la.copy(sa, m0, 1, t + 1, dead, imgA(nb, 1), tid);
    bar();
    mma(1, 1, bf1);
    // P4: A1 x B0
    vmwait<C::CA + C::CB>();       // A0(t+1), B0(t+1)
    bar();
    mma(1, 0, bf0);
  }
  vmwait<0>();   // the (zero-filled) copies issued by the last K-tile

  // epilogue: acc[ha][hb][i][j], lane l = C[m][n .. n+3] with
  //   m = m0 + 128 ha + wr*16MT + 16 i + (l & 15),  n = n0 + RB hb + wc*16NT + 16 j + 4 (l >> 4)
  if constexpr (EPI::STATS) {
    float s1[2][NT][4], s2[2][NT][4];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) { s1[hb][j][q] = 0.f; s2[hb][j][q] = 0.f; }
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = m0 + 128 * ha + wr * (16 * MT) + 16 * i + (lane & 15);
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int n = n0 + RB * hb + wc * (16 * NT) + 16 * j + 4 * (lane >> 4);
            if (m < M && n < N) {
              const f32x4 r = epi.quad(m, n, acc[ha][hb][i][j]);
#pragma unroll
              for (int q = 0; q < 4; ++q) { s1[hb][j][q] += r[q]; s2[hb][j][q] += r[q] * r[q]; }
            }
          }
      }
    // reduce over the 16 lanes (rows) that share a column quad, one atomic per column
    const int slot = ((m0 >> 6) + wr) & (NSTAT - 1);
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float a = s1[hb][j][q], b = s2[hb][j][q];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
          const int n = n0 + RB * hb + wc * (16 * NT) + 16 * j + 4 * (lane >> 4) + q;
          if ((lane & 15) == 0 && n < N) {
            atomicAdd(epi.sum + (size_t)slot * N + n, a);
            atomicAdd(epi.sumsq + (size_t)slot * N + n, b);
          }
        }
  } else {
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = m0 + 128 * ha + wr * (16 * MT) + 16 * i + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int n = n0 + RB * hb + wc * (16 * NT) + 16 * j + 4 * (lane >> 4);
            if (n < N) epi.quad(m, n, acc[ha][hb][i][j]);
          }
      }
  }
}

template <int BN, class LA, class LB, class EPI>
static hipError_t launch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<BN, LA, LB, EPI>), dim3(tiles), dim3(NTHR), 0, st, la, lb, epi, M, N, K);
  return hipGetLastError();
}

// the block-tile width of a dense GEMM: the candidate whose tile count fills the 256 CUs
// best (one 512-thread block per CU; a partial last round costs a whole round)
static inline int pick_bn_dense(int M, int N) {
  const long tm = (M + 255) / 256;
  int best = 128;
  double best_eff = -1.0;
  for (int bn : {256, 192, 128}) {
    if (bn > 128 && N <= 128) continue;
    const long t = tm * ((N + bn - 1) / bn);
    const long rounds = (t + 255) / 256;
    const double eff = (double)M * N / ((double)rounds * 256 * 256 * bn);   // useful / issued tile work
    if (eff > best_eff + 1e-9) { best_eff = eff; best = bn; }
  }
  return best;
}

// BN = 128 when the 256-wide tile would leave half its columns empty or too few blocks
static inline int pick_bn(int M, int N) {
  if (N <= 128) return 128;
  const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
  return t256 >= 256 ? 256 : 128;
}

}  // namespace g256

using namespace g256;
using namespace igemm_host;

// C = A[M][K] . B[N][K]^T (+bias, act, addend) -> bf16 C (ldc) or fp32 Cf.
// Requires K % 8 == 0, N % 4 == 0, lda % 8 == 0, ldb % 8 == 0.  bn: 0 = auto, 128, 256.
MLC_EXPORT int mlc_gemm256_nt(const bf16* A, const bf16* B, bf16* C, float* Cf, int M, int N, int K, int lda,
                              int ldb, int ldc, const float* bias, int act, bf16* preact, const bf16* addend,
                              int accumulate, int bn, hipStream_t st) {
  if (K % 8 || N % 4 || lda % 8 || ldb % 8 || ldc % 4 || M <= 0 || N <= 0 || K <= 0) return -1;
  if ((C == nullptr) == (Cf == nullptr)) return -1;
  if (bn == 0) bn = pick_bn(M, N);
  const bool tail = K % BK != 0;
#define G_LAUNCH(BNV, TAIL, FP)                                                                   \
  return (int)launch<BNV>(MatKC<128, TAIL>{A, lda, M, K}, MatKC<BNV / 2, TAIL>{B, ldb, N, K},   \
                          EpiOut<FP>{C, Cf, ldc, bias, act, preact, addend, accumulate}, M, N, K, st)
  if (bn == 256) {
    if (Cf) { if (tail) G_LAUNCH(256, true, 1); G_LAUNCH(256, false, 1); }
    if (tail) G_LAUNCH(256, true, 0);
    G_LAUNCH(256, false, 0);
  }
  if (Cf) { if (tail) G_LAUNCH(128, true, 1); G_LAUNCH(128, false, 1); }
  if (tail) G_LAUNCH(128, true, 0);
  G_LAUNCH(128, false, 0);
#undef G_LAUNCH
}

// C = A[K][M]^T . B[K][N] with both operands MN-contiguous (the "TN" layout of a weight
// gradient dW = dY^T X) -> fp32 Cf (store or accumulate).  M % 8 == N % 8 == 0.
MLC_EXPORT int mlc_gemm256_tn(const bf16* A, const bf16* B, float* Cf, int M, int N, int K, int lda, int ldb,
                              int ldc, int accumulate, int bn, hipStream_t st) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 4 || M <= 0 || N <= 0 || K <= 0) return -1;
  if (bn == 0) bn = pick_bn(M, N);
  const bool tail = K % BK != 0;
#define G_LAUNCH(BNV, TAIL)                                                                       \
  return (int)launch<BNV>(MatMC<128, TAIL>{A, lda, K, M}, MatMC<BNV / 2, TAIL>{B, ldb, K, N},   \
                          EpiOut<1>{nullptr, Cf, ldc, nullptr, 0, nullptr, nullptr, accumulate}, M, N, K, st)
  if (bn == 256) { if (tail) G_LAUNCH(256, true); G_LAUNCH(256, false); }
  if (tail) G_LAUNCH(128, true);
  G_LAUNCH(128, false);
#undef G_LAUNCH
}

// y[N,Ho,Wo,Co] = conv(x[N,H,W,C], w[Co,KH,KW,C]) (+ BN partial sums of y / y^2 into
// sum/sumsq [NSTAT][Co], zeroed by the caller, when given).  C % 8 == Co % 8 == 0.
MLC_EXPORT int mlc_conv256_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq, int N, int H, int W,
                               int C, int Co, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int bn,
                               hipStream_t st) {
  if (C % 8 || Co % 8 || KH > 15 || KW > 16) return -1;
  const int M = N * Ho * Wo, K = KH * KW * C;
  if (bn == 0) bn = pick_bn(M, Co);
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  const bool tail = K % BK != 0;
  const bool stats = sum != nullptr;
#define G_CONV(BNV, TAIL)                                                                                      \
  do {                                                                                                         \
    if (stats)                                                                                                 \
      return (int)launch<BNV>(ConvFwdA<128, TAIL>{x, g, M, K}, MatKC<BNV / 2, TAIL>{w, K, Co, K},           \
                              EpiConvStats{y, Co, sum, sumsq}, M, Co, K, st);                                  \
    return (int)launch<BNV>(ConvFwdA<128, TAIL>{x, g, M, K}, MatKC<BNV / 2, TAIL>{w, K, Co, K},             \
                            EpiOut<0>{y, nullptr, Co, nullptr, 0, nullptr, nullptr, 0}, M, Co, K, st);        \
  } while (0)
  if (bn == 256) { if (tail) G_CONV(256, true); G_CONV(256, false); }
  if (tail) G_CONV(128, true);
  G_CONV(128, false);
#undef G_CONV
}

// Dense-layer GEMM on the 256-row engine: C[M][N] = A[M][K] . op(B) with the igemm.hip
// mlc_gemm_bf16_ex_native epilogue (bias, act, preact, addend, dact).  tb = 1: B is [N][K]
// (K-contiguous, the forward of x W^T); tb = 0: B is [K][N] (the input gradient dY W).
// bn: 0 = auto (pick_bn_dense), 128, 192 or 256.  K % 8 == N % 8 == 0, A not transposed.
MLC_EXPORT int mlc_g256_dense(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int lda, int ldb, int ldc,
                              int tb, const float* bias, int act, bf16* preact, const bf16* addend, const bf16* dact,
                              int bn, hipStream_t st) {
  if (K % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8 || M <= 0 || N <= 0 || K <= 0) return -1;
  if (bn == 0) bn = pick_bn_dense(M, N);
  const bool tail = K % BK != 0;
  const EpiDense epi{C, ldc, bias, act, preact, addend, dact};
#define G_D(BNV, TAIL, HRV)                                                                              \
  return tb ? (int)launch<BNV>(MatKC<128, TAIL>{A, lda, M, K}, MatKC<Cfg<BNV>::RBI, TAIL, HRV>{B, ldb, N, K}, \
                               epi, M, N, K, st)                                                      \
            : (int)launch<BNV>(MatKC<128, TAIL>{A, lda, M, K}, MatMC<Cfg<BNV>::RBI, TAIL, HRV>{B, ldb, K, N}, \
                               epi, M, N, K, st)
  if (bn == 256) { if (tail) G_D(256, true, 128); G_D(256, false, 128); }
  if (bn == 192) { if (tail) G_D(192, true, 96); G_D(192, false, 96); }
  if (tail) G_D(128, true, 64);
  G_D(128, false, 64);
#undef G_D
}
