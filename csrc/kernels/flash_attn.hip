// General-shape fused multi-head attention for gfx950 (flash-style, online softmax).
//
// transformer.hip's attn:: kernels hold a whole S x S score tile in registers and so only
// take head dim 64 with S in {64, 128} (BERT-base fine-tuning).  These kernels stream the
// keys (forward, dQ) or queries (dK/dV) through LDS in 64-row tiles, so S is any length
// (the last tile's rows past S are masked: -inf key bias / +inf log-sum-exp) and the head
// dim D is 64 or 128; the per-step work is O(S) registers and LDS.
// Reference behaviour: the attention inside the BERT encoder the reference fine-tunes
// through Catalyst; numerics match ops/transformer.py attn_fwd/attn_bwd.
//
// Layout: qkv [B*S][3*H*D] bf16 (q | k | v column blocks, head h at h*D), out / dout
// [B*S][H*D], key_bias [B][S] fp32 (0 / -inf padding mask, any finite bias works),
// lse / dot [B*H*S] fp32.  Dropout on the attention probabilities uses the softmax
// kernel's element index ((b*H + h)*S + q)*S + key (dropout.h), so every attention path
// drops the same elements.
//
// Work split (one 256-thread block = 4 waves x 32 rows, blocks XCD-remapped so the blocks
// sharing one (b, h) K/V slice sit on one XCD's L2):
// * forward: a wave owns 32 queries; scores are computed transposed, S^T = K Q^T
//   (v_mfma_f32_32x32x16_bf16, A = K rows from LDS, B = Q rows held in registers), so a
//   lane holds ONE query's scores for 32 keys of the 64-key tile and the running max /
//   sum are in-register plus one lane^32 exchange; the unnormalised probabilities feed
//   O^T += V^T P^T straight from the accumulators (B operand) with V read transposed
//   (ds_read_b64_tr_b16).  The accumulator key order is the natural order with bits 2
//   and 3 swapped, so every LDS tile stores logical row r at image row swap23(r).
// * backward, two kernels (no atomics): dq_kernel (a wave owns 32 queries, streams
//   K / V tiles) recomputes P from the saved log-sum-exp, forms dS and accumulates
//   dQ^T = K^T dS^T; it also writes dot = rowsum(dO * O), which equals sum_k P dP
//   with or without dropout.  dkv_kernel (a wave owns 32 keys, streams Q / dO tiles
//   plus their lse / dot) computes S = Q K^T directly (lane = key), and accumulates
//   dV^T = dO^T Pd and dK^T = Q^T dS.
// LDS images: [64 rows][D] bf16, 16-byte chunks XOR-swizzled so that both the row reads
// (ds_read_b128, the MFMA A/B fragment of one row) and the transposed reads are
// conflict-free (checked with the bank model of MI355X_MICROARCH.md §LDS: D=128 is the
// guide's dual-use image (b), D=64 a swizzle over row bits 1, 3, 4 found the same way).
#include "common.h"
#include "dropout.h"
#include <stdlib.h>

namespace {

constexpr int NT = 256;
constexpr int KT = 64;   // rows per streamed tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ int swap23(int k) { return (k & ~12) | ((k >> 1) & 4) | ((k << 1) & 8); }
// row (within a 32-row MFMA tile) of accumulator register r of lane half hh
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

template <int D>
__device__ __forceinline__ int off(int r, int c) {
  if constexpr (D == 64)
    return r * 128 + 16 * (c ^ ((((r >> 1) & 1) << 2) ^ ((r >> 3) & 1) ^ (((r >> 4) & 1) << 1)));
  else
    return r * 256 + 16 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}
// operand fragment of logical row `row` (k = d = 16s + 8*(lane>>5) + 0..7)
template <int D>
__device__ __forceinline__ bf16x8 rowf(const char* img, int row, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + off<D>(swap23(row), 2 * s + (lane >> 5)));
}
// transposed operand fragment: column d = base + (lane&31), k = image rows k0 + 8*(lane>>5) + 0..7
template <int D>
__device__ __forceinline__ bf16x8 trf(const char* img, int base, int k0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int kr = k0 + 8 * (g >> 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (LDS_PTR(s16x4))(img + off<D>(kr + q, col >> 3) + (col & 7) * 2));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (LDS_PTR(s16x4))(img + off<D>(kr + 4 + q, col >> 3) + (col & 7) * 2));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
// K-contiguous fragment of row `row` straight from global (ld elements per row)
__device__ __forceinline__ bf16x8 gfrag(const bf16* base, int ld, int row, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + (size_t)row * ld + 16 * s + 8 * (lane >> 5));
}
// accumulator registers 8s..8s+7 as a bf16 B fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int t = 0; t < 8; ++t) r[t] = (bf16)a[8 * s + t];
  return r;
}
__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
}
// store transposed accumulators acc[j][r] = X[lane's row][d = 32j + acc_row(r, hh)] as
// 8-byte pieces
template <int NJ>
__device__ __forceinline__ void store_rows(bf16* dst, const f32x16 (&acc)[NJ], int lane) {
  const int hh = lane >> 5;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 u;
      u.x = pack2_bf16(acc[j][4 * g], acc[j][4 * g + 1]);
      u.y = pack2_bf16(acc[j][4 * g + 2], acc[j][4 * g + 3]);
      *reinterpret_cast<uint2*>(dst + 32 * j + 8 * g + 4 * hh) = u;
    }
}

// a 64-row x D tile copied global -> registers -> swizzled LDS image (row r at swap23(r))
template <int D>
struct Tile {
  static constexpr int CH = D / 8, N = KT * CH / NT;
  uint4 v[N];
  __device__ __forceinline__ void load(const bf16* src, int ld, int tid, int valid = KT) {
    // rows past `valid` (the tail tile of an S that is not a multiple of 64) re-read the
    // last valid row: in bounds, finite, and masked out by the caller (-inf key bias /
    // +inf log-sum-exp), so they contribute exactly zero
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int c = tid + NT * j, r = min(c / CH, valid - 1), ch = c % CH;
      v[j] = *reinterpret_cast<const uint4*>(src + (size_t)r * ld + ch * 8);
    }
  }
  __device__ __forceinline__ void store(char* img, int tid) const {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int c = tid + NT * j, r = c / CH, ch = c % CH;
      *reinterpret_cast<uint4*>(img + off<D>(swap23(r), ch)) = v[j];
    }
  }
};

struct Geo {
  int b, hd, bh, blk;
};
__device__ __forceinline__ Geo geo(int H, int nblk) {
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  Geo g;
  g.bh = lin / nblk;
  g.blk = lin - g.bh * nblk;
  g.b = g.bh / H;
  g.hd = g.bh - g.b * H;
  return g;
}

// ------------------------------------------------------------------ forward
template <int D, bool DROP>
__global__ void __launch_bounds__(NT)
fwd_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, bf16* __restrict__ out,
           float* __restrict__ lse, int S, int H, int nqb, float sl2, uint32_t thr, float inv_keep,
           const uint32_t* __restrict__ seedp, uint32_t salt) {
  constexpr int NS = D / 16, NJ = D / 32, IMG = KT * D * 2, BUF = 2 * IMG + KT * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];   // [buffer][K | V | key bias * log2e]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const Geo G = geo(H, nqb);
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)G.b * S * ld + G.hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const int q = G.blk * 128 + 32 * w + l32;
  const int qc = min(q, S - 1);
  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = gfrag(Qg, ld, qc, s, lane);
  f32x16 o[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) zero(o[j]);
  float m = -INFINITY, l = 0.f;
  const float* kb = key_bias ? key_bias + (size_t)G.b * S : nullptr;
  const uint32_t seed = seedp ? *seedp : 0u;
  const uint32_t rowidx = ((uint32_t)G.bh * S + qc) * S;
  Tile<D> tk, tv;
  float kbv = 0.f;
  auto fetch = [&](int t) {
    const int valid = min(KT, S - t * KT);
    tk.load(Kg + (size_t)t * KT * ld, ld, tid, valid);
    tv.load(Vg + (size_t)t * KT * ld, ld, tid, valid);
    if (tid < KT) kbv = tid >= valid ? -INFINITY : kb ? kb[t * KT + tid] * LOG2E : 0.f;
  };
  auto put = [&](int t) {
    char* bp = smem + (t & 1) * BUF;
    tk.store(bp, tid);
    tv.store(bp + IMG, tid);
    if (tid < KT) reinterpret_cast<float*>(bp + 2 * IMG)[tid] = kbv;
  };
  fetch(0);
  put(0);
  __syncthreads();
  const int nt = (S + KT - 1) / KT;   // a partial last tile is masked
  for (int t = 0; t < nt; ++t) {
    const char* Ki = smem + (t & 1) * BUF;
    const char* Vi = Ki + IMG;
    const float* Kb = reinterpret_cast<const float*>(Ki + 2 * IMG);
    if (t + 1 < nt) fetch(t + 1);
    f32x16 a[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      zero(a[i]);
#pragma unroll
      for (int s = 0; s < NS; ++s) a[i] = mfma(rowf<D>(Ki, 32 * i + l32, s, lane), qf[s], a[i]);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(Kb + 32 * i + 8 * g + 4 * hh);   // keys of regs 4g..4g+3
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = a[i][4 * g + e] * sl2 + k4[e];
          a[i][4 * g + e] = x;
          tmax = fmaxf(tmax, x);
        }
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    if (__any(mn > m)) {   // rescale only when some query's running max moved (wave-uniform)
      const float corr = mn > m ? __builtin_amdgcn_exp2f(m - mn) : 1.f;   // m = -inf: 0
      l *= corr;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[j][r] *= corr;
      m = mn;
    }
    const float mref = m == -INFINITY ? 0.f : m;   // fully masked so far: p = 0, o stays 0
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(a[i][r] - mref);
        l += e;
        a[i][r] = e;
      }
    if constexpr (DROP) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          a[i][r] = keep(seed, salt, rowidx + t * KT + 32 * i + acc_row(r, hh), thr) ? a[i][r] * inv_keep : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = acc_frag(a[i], s);
#pragma unroll
        for (int j = 0; j < NJ; ++j) o[j] = mfma(trf<D>(Vi, 32 * j, 32 * i + 16 * s, lane), pb, o[j]);
      }
    if (t + 1 < nt) put(t + 1);
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[j][r] *= inv;
  if (q < S) {
    if (hh == 0) lse[(size_t)G.bh * S + q] = l > 0.f ? (m + __log2f(l)) * LN2 : INFINITY;
    store_rows<NJ>(out + ((size_t)G.b * S + q) * E + G.hd * D, o, lane);
  }
}

// ------------------------------------------------------------------ backward: dQ (+ dot)
template <int D, bool DROP>
__global__ void __launch_bounds__(NT)
dq_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, const bf16* __restrict__ out,
          const bf16* __restrict__ dout, const float* __restrict__ lse, float* __restrict__ dot,
          bf16* __restrict__ dqkv, int S, int H, int nqb, float scale, float sl2, uint32_t thr, float inv_keep,
          const uint32_t* __restrict__ seedp, uint32_t salt) {
  constexpr int NS = D / 16, NJ = D / 32, IMG = KT * D * 2, BUF = 2 * IMG + KT * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];   // [buffer][K | V | key bias * log2e]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const Geo G = geo(H, nqb);
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)G.b * S * ld + G.hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const bf16* Og = out + (size_t)G.b * S * E + G.hd * D;
  const bf16* dOg = dout + (size_t)G.b * S * E + G.hd * D;
  const int q = G.blk * 128 + 32 * w + l32;
  const int qc = min(q, S - 1);
  bf16x8 qf[NS], of[NS];
  float dt = 0.f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = gfrag(Qg, ld, qc, s, lane);
    of[s] = gfrag(dOg, E, qc, s, lane);
    const bf16x8 ov = gfrag(Og, E, qc, s, lane);
#pragma unroll
    for (int e = 0; e < 8; ++e) dt += (float)of[s][e] * (float)ov[e];
  }
  dt += __shfl_xor(dt, 32, 64);
  if (q < S && hh == 0) dot[(size_t)G.bh * S + q] = dt;
  const float l2 = lse[(size_t)G.bh * S + qc] * LOG2E;
  const float* kb = key_bias ? key_bias + (size_t)G.b * S : nullptr;
  const uint32_t seed = seedp ? *seedp : 0u;
  const uint32_t rowidx = ((uint32_t)G.bh * S + qc) * S;
  f32x16 dq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) zero(dq[j]);
  Tile<D> tk, tv;
  float kbv = 0.f;
  auto fetch = [&](int t) {
    const int valid = min(KT, S - t * KT);
    tk.load(Kg + (size_t)t * KT * ld, ld, tid, valid);
    tv.load(Vg + (size_t)t * KT * ld, ld, tid, valid);
    if (tid < KT) kbv = tid >= valid ? -INFINITY : kb ? kb[t * KT + tid] * LOG2E : 0.f;
  };
  auto put = [&](int t) {
    char* bp = smem + (t & 1) * BUF;
    tk.store(bp, tid);
    tv.store(bp + IMG, tid);
    if (tid < KT) reinterpret_cast<float*>(bp + 2 * IMG)[tid] = kbv;
  };
  fetch(0);
  put(0);
  __syncthreads();
  const int nt = (S + KT - 1) / KT;   // a partial last tile is masked
  for (int t = 0; t < nt; ++t) {
    const char* Ki = smem + (t & 1) * BUF;
    const char* Vi = Ki + IMG;
    const float* Kb = reinterpret_cast<const float*>(Ki + 2 * IMG);
    if (t + 1 < nt) fetch(t + 1);
    f32x16 sp[2], dp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      zero(sp[i]);
      zero(dp[i]);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sp[i] = mfma(rowf<D>(Ki, 32 * i + l32, s, lane), qf[s], sp[i]);
        dp[i] = mfma(rowf<D>(Vi, 32 * i + l32, s, lane), of[s], dp[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(Kb + 32 * i + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float p = __builtin_amdgcn_exp2f(sp[i][r] * sl2 + k4[e] - l2);
          float d = dp[i][r];
          if constexpr (DROP) d = keep(seed, salt, rowidx + t * KT + 32 * i + 8 * g + 4 * hh + e, thr) ? d * inv_keep : 0.f;
          sp[i][r] = scale * p * (d - dt);
        }
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sb = acc_frag(sp[i], s);
#pragma unroll
        for (int j = 0; j < NJ; ++j) dq[j] = mfma(trf<D>(Ki, 32 * j, 32 * i + 16 * s, lane), sb, dq[j]);
      }
    if (t + 1 < nt) put(t + 1);
    __syncthreads();
  }
  if (q < S) store_rows<NJ>(dqkv + ((size_t)G.b * S + q) * ld + G.hd * D, dq, lane);
}

// ------------------------------------------------------------------ backward: dK, dV
template <int D, bool DROP>
__global__ void __launch_bounds__(NT)
dkv_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, const bf16* __restrict__ dout,
           const float* __restrict__ lse, const float* __restrict__ dot, bf16* __restrict__ dqkv, int S, int H,
           int nkb, float scale, float sl2, uint32_t thr, float inv_keep, const uint32_t* __restrict__ seedp,
           uint32_t salt) {
  constexpr int NS = D / 16, NJ = D / 32, IMG = KT * D * 2, BUF = 2 * IMG + 2 * KT * 4;
  // [buffer][Q image | dO image | lse*log2e [64] | dot [64]]
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const Geo G = geo(H, nkb);
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)G.b * S * ld + G.hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const bf16* dOg = dout + (size_t)G.b * S * E + G.hd * D;
  const float* Lg = lse + (size_t)G.bh * S;
  const float* Dg = dot + (size_t)G.bh * S;
  const int key = G.blk * 128 + 32 * w + l32;
  const int kc = min(key, S - 1);
  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = gfrag(Kg, ld, kc, s, lane);
    vf[s] = gfrag(Vg, ld, kc, s, lane);
  }
  const float kbl = key_bias ? key_bias[(size_t)G.b * S + kc] * LOG2E : 0.f;
  const uint32_t seed = seedp ? *seedp : 0u;
  f32x16 dk[NJ], dv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    zero(dk[j]);
    zero(dv[j]);
  }
  Tile<D> tq, to;
  float ld_v = 0.f;   // this thread's lse / dot element of the next tile (threads 0..127)
  auto fetch = [&](int t) {
    const int valid = min(KT, S - t * KT);
    tq.load(Qg + (size_t)t * KT * ld, ld, tid, valid);
    to.load(dOg + (size_t)t * KT * E, E, tid, valid);
    // queries past S: lse = +inf makes their probabilities exactly 0
    if (tid < KT) ld_v = tid < valid ? Lg[t * KT + tid] * LOG2E : INFINITY;
    else if (tid < 2 * KT) ld_v = tid - KT < valid ? Dg[t * KT + tid - KT] : 0.f;
  };
  auto put = [&](int t) {
    char* bp = smem + (t & 1) * BUF;
    tq.store(bp, tid);
    to.store(bp + IMG, tid);
    if (tid < 2 * KT) reinterpret_cast<float*>(bp + 2 * IMG)[tid] = ld_v;
  };
  fetch(0);
  put(0);
  __syncthreads();
  const int nt = (S + KT - 1) / KT;   // a partial last tile is masked
  for (int t = 0; t < nt; ++t) {
    const char* bp = smem + (t & 1) * BUF;
    const char* Qi = bp;
    const char* Oi = bp + IMG;
    const float* Ls = reinterpret_cast<const float*>(bp + 2 * IMG);
    const float* Ds = Ls + KT;
    if (t + 1 < nt) fetch(t + 1);
    f32x16 sc[2], dp[2];   // C[q][key]: lane = key, register r = query 32i + acc_row(r, hh)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      zero(sc[i]);
      zero(dp[i]);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sc[i] = mfma(rowf<D>(Qi, 32 * i + l32, s, lane), kf[s], sc[i]);
        dp[i] = mfma(rowf<D>(Oi, 32 * i + l32, s, lane), vf[s], dp[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q0 = 32 * i + 8 * g + 4 * hh;   // registers 4g..4g+3 are queries q0..q0+3
        const f32x4 L4 = *reinterpret_cast<const f32x4*>(Ls + q0);
        const f32x4 D4 = *reinterpret_cast<const f32x4*>(Ds + q0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float p = __builtin_amdgcn_exp2f(sc[i][r] * sl2 + kbl - L4[e]);
          float d = dp[i][r], pd = p;
          if constexpr (DROP) {
            const bool kp = keep(seed, salt, ((uint32_t)G.bh * S + t * KT + q0 + e) * S + kc, thr);
            d = kp ? d * inv_keep : 0.f;
            pd = kp ? p * inv_keep : 0.f;
          }
          dp[i][r] = scale * p * (d - D4[e]);   // dS
          sc[i][r] = pd;                        // Pd
        }
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = acc_frag(sc[i], s);
        const bf16x8 sb = acc_frag(dp[i], s);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          dv[j] = mfma(trf<D>(Oi, 32 * j, 32 * i + 16 * s, lane), pb, dv[j]);
          dk[j] = mfma(trf<D>(Qi, 32 * j, 32 * i + 16 * s, lane), sb, dk[j]);
        }
      }
    if (t + 1 < nt) put(t + 1);
    __syncthreads();
  }
  if (key < S) {
    bf16* dst = dqkv + ((size_t)G.b * S + key) * ld + G.hd * D;
    store_rows<NJ>(dst + E, dk, lane);
    store_rows<NJ>(dst + 2 * E, dv, lane);
  }
}

// ------------------------------------------------------------------ backward, S = 128: fused
// One block per (b, h) holds the whole 128-query x 128-key problem, so P is recomputed once
// (not once per dq / dkv kernel) and there is one launch instead of two:
// * phase 0: every wave forms dot = rowsum(dO * O) for its 32 queries; Q, dO (as the
//   dkv_kernel's swap23 images) and K (natural row order, for the dQ GEMM's transposed
//   reads) are staged in LDS;
// * phase A (dkv_kernel orientation, lane = key): wave w owns keys 32w..32w+31, computes
//   S = Q K^T and dP = dO V^T over both 64-query tiles, P from the saved log-sum-exp, dS,
//   accumulates dV^T = dO^T Pd and dK^T = Q^T dS in registers, and writes dS (bf16) into a
//   [query][key] LDS image;
// * phase B (lane = query): wave w owns queries 32w..32w+31 and forms dQ^T = K^T dS^T from
//   the K and dS images.
// LDS: 3 x 16 KB operand images + the 32 KB dS image + lse / dot = 81 KB (one block per CU).
// (A 65 KB variant with K staged over Q after phase A, two blocks per CU at 231 VGPRs,
// measured 36.5 vs 28.3 us on BERT-base: the co-resident blocks share the matrix pipe and
// the extra barrier/staging did not pay.)
template <int D, bool DROP>
__global__ void __launch_bounds__(NT)
bwd128_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, const bf16* __restrict__ out,
              const bf16* __restrict__ dout, const float* __restrict__ lse, bf16* __restrict__ dqkv, int H,
              float scale, float sl2, uint32_t thr, float inv_keep, const uint32_t* __restrict__ seedp,
              uint32_t salt) {
  constexpr int S = 128, NS = D / 16, NJ = D / 32, IMG = KT * D * 2;
  constexpr int DS_BYTES = S * S * 2;
  __shared__ __attribute__((aligned(16))) char smem[6 * IMG + DS_BYTES + 2 * S * 4];
  char* Qi = smem;               // two 64-row images each, rows at swap23 (as Tile::store)
  char* Oi = smem + 2 * IMG;
  char* Ki = smem + 4 * IMG;     // 128 rows in natural order
  char* dSi = smem + 6 * IMG;    // [query at swap23][key] bf16, 256-B rows
  float* Ls = reinterpret_cast<float*>(dSi + DS_BYTES);
  float* Dt = Ls + S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const Geo G = geo(H, 1);
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)G.b * S * ld + G.hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const bf16* Og = out + (size_t)G.b * S * E + G.hd * D;
  const bf16* dOg = dout + (size_t)G.b * S * E + G.hd * D;
  const uint32_t seed = seedp ? *seedp : 0u;
  // ---- phase 0
  {
    Tile<D> q0, q1, o0, o1, k0, k1;
    q0.load(Qg, ld, tid);
    q1.load(Qg + (size_t)KT * ld, ld, tid);
    o0.load(dOg, E, tid);
    o1.load(dOg + (size_t)KT * E, E, tid);
    k0.load(Kg, ld, tid);
    k1.load(Kg + (size_t)KT * ld, ld, tid);
    const int qr = 32 * w + l32;
    float dt = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 of = gfrag(dOg, E, qr, s, lane), ov = gfrag(Og, E, qr, s, lane);
#pragma unroll
      for (int e = 0; e < 8; ++e) dt += (float)of[e] * (float)ov[e];
    }
    dt += __shfl_xor(dt, 32, 64);
    if (hh == 0) {
      Dt[qr] = dt;
      Ls[qr] = lse[(size_t)G.bh * S + qr] * LOG2E;
    }
    q0.store(Qi, tid);
    q1.store(Qi + IMG, tid);
    o0.store(Oi, tid);
    o1.store(Oi + IMG, tid);
    constexpr int CH = D / 8;
#pragma unroll
    for (int j = 0; j < Tile<D>::N; ++j) {   // K rows in natural order
      const int c = tid + NT * j, r = c / CH, ch = c % CH;
      *reinterpret_cast<uint4*>(Ki + off<D>(r, ch)) = k0.v[j];
      *reinterpret_cast<uint4*>(Ki + off<D>(r + KT, ch)) = k1.v[j];
    }
  }
  // this wave's keys: K / V fragments (B operands) and the key bias
  const int key = 32 * w + l32;
  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = gfrag(Kg, ld, key, s, lane);
    vf[s] = gfrag(Vg, ld, key, s, lane);
  }
  const float kbl = key_bias ? key_bias[(size_t)G.b * S + key] * LOG2E : 0.f;
  __syncthreads();
  // ---- phase A
  f32x16 dk[NJ], dv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    zero(dk[j]);
    zero(dv[j]);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const char* Qt = Qi + t * IMG;
    const char* Ot = Oi + t * IMG;
    f32x16 sc[2], dp[2];   // C[q][key]: lane = key, register r = query 64t + 32i + acc_row(r, hh)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      zero(sc[i]);
      zero(dp[i]);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sc[i] = mfma(rowf<D>(Qt, 32 * i + l32, s, lane), kf[s], sc[i]);
        dp[i] = mfma(rowf<D>(Ot, 32 * i + l32, s, lane), vf[s], dp[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q0 = KT * t + 32 * i + 8 * g + 4 * hh;   // registers 4g..4g+3: queries q0..q0+3
        const f32x4 L4 = *reinterpret_cast<const f32x4*>(Ls + q0);
        const f32x4 D4 = *reinterpret_cast<const f32x4*>(Dt + q0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float p = __builtin_amdgcn_exp2f(sc[i][r] * sl2 + kbl - L4[e]);
          float d = dp[i][r], pd = p;
          if constexpr (DROP) {
            const bool kp = keep(seed, salt, ((uint32_t)G.bh * S + q0 + e) * S + key, thr);
            d = kp ? d * inv_keep : 0.f;
            pd = kp ? p * inv_keep : 0.f;
          }
          const float ds = scale * p * (d - D4[e]);
          dp[i][r] = ds;
          sc[i][r] = pd;
          *reinterpret_cast<bf16*>(dSi + off<128>(swap23(q0 + e), key >> 3) + (key & 7) * 2) = (bf16)ds;
        }
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = acc_frag(sc[i], s);
        const bf16x8 sb = acc_frag(dp[i], s);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          dv[j] = mfma(trf<D>(Ot, 32 * j, 32 * i + 16 * s, lane), pb, dv[j]);
          dk[j] = mfma(trf<D>(Qt, 32 * j, 32 * i + 16 * s, lane), sb, dk[j]);
        }
      }
  }
  {
    bf16* dst = dqkv + ((size_t)G.b * S + key) * ld + G.hd * D;
    store_rows<NJ>(dst + E, dk, lane);
    store_rows<NJ>(dst + 2 * E, dv, lane);
  }
  __syncthreads();   // every wave's dS is in the image
  // ---- phase B: dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q], lane = query 32w + l32
  f32x16 dq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) zero(dq[j]);
  const int qr = 32 * w + l32;
#pragma unroll
  for (int s = 0; s < S / 16; ++s) {
    const bf16x8 sb = rowf<128>(dSi, qr, s, lane);
#pragma unroll
    for (int j = 0; j < NJ; ++j) dq[j] = mfma(trf<D>(Ki, 32 * j, 16 * s, lane), sb, dq[j]);
  }
  store_rows<NJ>(dqkv + ((size_t)G.b * S + qr) * ld + G.hd * D, dq, lane);
}

// ------------------------------------------------------------------ forward, S = 128
// The whole key range at once: K and V (128 rows each, two consecutive swap23 images = one
// 128-row image) land in LDS behind ONE barrier, the 4 key tiles of S^T = K Q^T are formed,
// and the softmax runs over the complete row (no running max / rescale), then O^T = V^T P^T.
// Same numerics and dropout indexing as fwd_kernel.
template <int D, bool DROP>
__global__ void __launch_bounds__(NT)
fwd128_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, bf16* __restrict__ out,
              float* __restrict__ lse, int H, float sl2, uint32_t thr, float inv_keep,
              const uint32_t* __restrict__ seedp, uint32_t salt) {
  constexpr int S = 128, NS = D / 16, NJ = D / 32, IMG = KT * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG + S * 4];   // K (2 images) | V (2) | bias
  char* Ki = smem;
  char* Vi = smem + 2 * IMG;
  float* Kb = reinterpret_cast<float*>(smem + 4 * IMG);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const Geo G = geo(H, 1);
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)G.b * S * ld + G.hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const int q = 32 * w + l32;
  {
    Tile<D> k0, k1, v0, v1;
    k0.load(Kg, ld, tid);
    k1.load(Kg + (size_t)KT * ld, ld, tid);
    v0.load(Vg, ld, tid);
    v1.load(Vg + (size_t)KT * ld, ld, tid);
    if (tid < S) Kb[tid] = key_bias ? key_bias[(size_t)G.b * S + tid] * LOG2E : 0.f;
    k0.store(Ki, tid);
    k1.store(Ki + IMG, tid);
    v0.store(Vi, tid);
    v1.store(Vi + IMG, tid);
  }
  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = gfrag(Qg, ld, q, s, lane);
  const uint32_t seed = seedp ? *seedp : 0u;
  const uint32_t rowidx = ((uint32_t)G.bh * S + q) * S;
  __syncthreads();
  f32x16 a[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    zero(a[i]);
#pragma unroll
    for (int s = 0; s < NS; ++s) a[i] = mfma(rowf<D>(Ki, 32 * i + l32, s, lane), qf[s], a[i]);
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 k4 = *reinterpret_cast<const f32x4*>(Kb + 32 * i + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = a[i][4 * g + e] * sl2 + k4[e];
        a[i][4 * g + e] = x;
        m = fmaxf(m, x);
      }
    }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float mref = m == -INFINITY ? 0.f : m;
  float l = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __builtin_amdgcn_exp2f(a[i][r] - mref);
      l += e;
      a[i][r] = e;
    }
  if constexpr (DROP) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        a[i][r] = keep(seed, salt, rowidx + 32 * i + acc_row(r, hh), thr) ? a[i][r] * inv_keep : 0.f;
  }
  f32x16 o[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) zero(o[j]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pb = acc_frag(a[i], s);
#pragma unroll
      for (int j = 0; j < NJ; ++j) o[j] = mfma(trf<D>(Vi, 32 * j, 32 * i + 16 * s, lane), pb, o[j]);
    }
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[j][r] *= inv;
  if (hh == 0) lse[(size_t)G.bh * S + q] = l > 0.f ? (m + __log2f(l)) * LN2 : INFINITY;
  store_rows<NJ>(out + ((size_t)G.b * S + q) * E + G.hd * D, o, lane);
}

// MLC_ATTN_BWD128=0 routes S = 128, D = 64 back to the streaming kernels (fwd_kernel and the
// dq / dkv pair)
int g_bwd128 = -1;

bool flash_shape_ok(int B, int S, int H, int D) {
  return B > 0 && H > 0 && S >= 1 && (D == 64 || D == 128);
}

}  // namespace

// out [B*S][H*D] = softmax(scale * Q K^T + key_bias) V per head, lse [B*H*S] (natural log;
// +inf for a fully masked row).  Any S >= 1 (a partial last 64-key tile is masked), D in {64, 128}.
MLC_EXPORT int mlc_flash_fwd(const bf16* qkv, const float* key_bias, bf16* out, float* lse, int B, int S, int H,
                             int D, float scale, float p, const uint32_t* seed, uint32_t salt, hipStream_t st) {
  if (!flash_shape_ok(B, S, H, D)) return -1;
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (g_bwd128 < 0) {
    const char* e = getenv("MLC_ATTN_BWD128");
    g_bwd128 = e ? atoi(e) : 1;
  }
  if (S == 128 && D == 64 && g_bwd128) {   // whole-key-range forward (MLC_ATTN_BWD128 covers both)
    const dim3 grid(B * H);
    if (t)
      hipLaunchKernelGGL((fwd128_kernel<64, true>), grid, dim3(NT), 0, st, qkv, key_bias, out, lse, H, scale * LOG2E,
                         t, k, seed, salt);
    else
      hipLaunchKernelGGL((fwd128_kernel<64, false>), grid, dim3(NT), 0, st, qkv, key_bias, out, lse, H, scale * LOG2E,
                         t, k, seed, salt);
    return hipGetLastError();
  }
  const int nqb = (S + 127) / 128;
  const dim3 grid(B * H * nqb);
#define FWD(DD, DR) hipLaunchKernelGGL((fwd_kernel<DD, DR>), grid, dim3(NT), 0, st, qkv, key_bias, out, lse, S, H, nqb, \
                                       scale * LOG2E, t, k, seed, salt)
  if (D == 64) { if (t) FWD(64, true); else FWD(64, false); }
  else { if (t) FWD(128, true); else FWD(128, false); }
#undef FWD
  return hipGetLastError();
}

// dqkv [B*S][3*H*D] fully overwritten (dQ | dK | dV); out = the forward's output; dot
// [B*H*S] fp32 scratch.
MLC_EXPORT int mlc_flash_bwd(const bf16* qkv, const float* key_bias, const bf16* out, const bf16* dout,
                             const float* lse, float* dot, bf16* dqkv, int B, int S, int H, int D, float scale,
                             float p, const uint32_t* seed, uint32_t salt, hipStream_t st) {
  if (g_bwd128 < 0) {
    const char* e = getenv("MLC_ATTN_BWD128");
    g_bwd128 = e ? atoi(e) : 1;
  }
  if (!flash_shape_ok(B, S, H, D)) return -1;
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (S == 128 && D == 64 && g_bwd128) {   // whole-problem fused backward (MLC_ATTN_BWD128)
    const dim3 grid(B * H);
    if (t)
      hipLaunchKernelGGL((bwd128_kernel<64, true>), grid, dim3(NT), 0, st, qkv, key_bias, out, dout, lse, dqkv, H,
                         scale, scale * LOG2E, t, k, seed, salt);
    else
      hipLaunchKernelGGL((bwd128_kernel<64, false>), grid, dim3(NT), 0, st, qkv, key_bias, out, dout, lse, dqkv, H,
                         scale, scale * LOG2E, t, k, seed, salt);
    return hipGetLastError();
  }
  const int nb = (S + 127) / 128;
  const dim3 grid(B * H * nb);
#define BWD(DD, DR)                                                                                              \
  do {                                                                                                           \
    hipLaunchKernelGGL((dq_kernel<DD, DR>), grid, dim3(NT), 0, st, qkv, key_bias, out, dout, lse, dot, dqkv, S, H, \
                       nb, scale, scale * LOG2E, t, k, seed, salt);                                              \
    hipLaunchKernelGGL((dkv_kernel<DD, DR>), grid, dim3(NT), 0, st, qkv, key_bias, dout, lse, dot, dqkv, S, H, nb, \
                       scale, scale * LOG2E, t, k, seed, salt);                                                  \
  } while (0)
  if (D == 64) { if (t) BWD(64, true); else BWD(64, false); }
  else { if (t) BWD(128, true); else BWD(128, false); }
#undef BWD
  return hipGetLastError();
}

// A/B knob of the S = 128 fused backward: value 0 / 1 sets it, < 0 only reads; returns the
// previous setting (resolving MLC_ATTN_BWD128 first)
MLC_EXPORT int mlc_flash_bwd128(int value) {
  if (g_bwd128 < 0) {
    const char* e = getenv("MLC_ATTN_BWD128");
    g_bwd128 = e ? atoi(e) : 1;
  }
  const int old = g_bwd128;
  if (value >= 0) g_bwd128 = value ? 1 : 0;
  return old;
}

