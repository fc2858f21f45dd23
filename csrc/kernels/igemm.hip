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
// Block: 256 threads = 4 waves (2x2), tile 128x128x64, each wave 64x64 = 2x2 MFMA
// 32x32 tiles.  Register-staged double-buffered LDS (64 KiB), one barrier per K-tile,
// XOR-swizzled LDS images (conflict-free b128 row reads and tr_b16 column reads),
// bijective XCD remap + grouped tile order for L2 reuse.
//
// Strided dgrad: output rows are ordered by stride-parity class (all pixels with
// hi%S==ph, wi%S==pw together) so a 128-row block belongs to ONE class, and every
// K-tile (one filter tap when Co%64==0) whose tap cannot reach that class is skipped:
// no MFMA work is spent on the structurally-zero taps of a stride-2 transpose conv.
//
// Epilogues: bf16 store through an LDS-staged 16 B/lane write (+ fused per-channel BN
// sum / sum-of-squares, spread over NSTAT copies to avoid same-address atomic
// contention), fp32 atomic add (split-K weight gradients), fp32 store (+bias).
#include "common.h"

namespace igemm {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE_BYTES = BM * BK * 2;           // 16 KiB per operand per stage
constexpr int LDS_BYTES = 4 * TILE_BYTES;         // A,B x 2 stages
constexpr int NSTAT = 32;                          // BN-stat partial copies

// ---------------------------------------------------------------- LDS images
// KC image: [128 rows][64 k] bf16, 128 B rows, 16 B chunk c of row r stored at
// chunk c ^ ((r>>1)&7): the 16-lane groups of ds_read_b128 hit 16 distinct slots.
__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// MC image: [64 k][128 mn] bf16, 256 B rows, chunk c of row k stored at c ^ ((k&3)<<2):
// each 32-lane half of a tr_b16 read covers 16 distinct slots.
__device__ __forceinline__ int mc_off(int k, int c) { return k * 256 + ((c ^ ((k & 3) << 2)) << 4); }

template <bool KC>
__device__ __forceinline__ void store_stage(char* lds, int tid, const uint4 (&v)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int off;
    if (KC) off = kc_off((tid >> 3) + 32 * i, tid & 7);
    else off = mc_off((tid >> 4) + 16 * i, tid & 15);
    *reinterpret_cast<uint4*>(lds + off) = v[i];
  }
}

// fragment of a 32-row (KC) / 32-col (MC) sub-tile for k-step s (16 deep)
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int base, int s, int lane) {
  if (KC) {
    const int r = base + (lane & 31), c = 2 * s + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(lds + kc_off(r, c));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m0 = base + 16 * (g & 1), k0 = 16 * s + 8 * (g >> 1);
    const int col = m0 + 4 * p;
    const int a0 = mc_off(k0 + q, col >> 3) + (col & 7) * 2;
    const int a1 = mc_off(k0 + 4 + q, col >> 3) + (col & 7) * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

__device__ __forceinline__ uint4 ld16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }

// Default K-tile iteration: every tile in [b, e).
struct AllTiles {
  __device__ int next(int kt, int) const { return kt; }
};

// ---------------------------------------------------------------- loaders
// A KC loader fills rows = m (or n) of the tile, 8 k per chunk: thread t owns rows
// (t>>3)+32i, chunk t&7.  An MC loader fills k-rows (t>>4)+16i, chunk (8 mn) t&15.

// plain row-major [rows][ld] matrix read K-contiguous
struct MatKC : AllTiles {
  static constexpr bool KC = true;
  const bf16* p; int ld, rows, K;
  int r_[4];
  __device__ void init(int m0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r_[i] = m0 + (tid >> 3) + 32 * i;
  }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
    const int k = k0 + (tid & 7) * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = (r_[i] < rows && k < K) ? ld16(p + (size_t)r_[i] * ld + k) : zero4();
  }
};

// plain row-major [K][ld] matrix whose rows are the reduction axis (MN-contiguous)
struct MatMC : AllTiles {
  static constexpr bool KC = false;
  const bf16* p; int ld, K, cols;
  int c_;
  __device__ void init(int n0, int tid) { c_ = n0 + (tid & 15) * 8; }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + (tid >> 4) + 16 * i;
      v[i] = (k < K && c_ < cols) ? ld16(p + (size_t)k * ld + c_) : zero4();
    }
  }
};

struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int Ho, Wo, Co;      // output
  int KH, KW, stride, pad, dil;
};

// decompose a reduction index k = ((r*KW)+s)*CC + c ; if CC % BK == 0 a whole K-tile
// shares one tap, so only the (wave-uniform) tile base needs the divisions.
__device__ __forceinline__ void tap_of(int k, int k0, int CC, int KW, int& r, int& s, int& c) {
  if (CC % BK == 0) {
    const int rs = k0 / CC;
    c = (k0 - rs * CC) + (k - k0);
    s = rs % KW; r = rs / KW;
  } else {
    c = k % CC; const int rs = k / CC; s = rs % KW; r = rs / KW;
  }
}

// conv fwd A operand: rows = output pixels, k = (r, s, ci) with ci fastest (C % 8 == 0)
struct ConvFwdA : AllTiles {
  static constexpr bool KC = true;
  const bf16* x; ConvGeom g; int M, K;
  int hb_[4], wb_[4]; int nb_[4];   // per-row base input coords, nb_ = -1 if row >= M
  __device__ void init(int m0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      if (m < M) {
        const int wo = m % g.Wo, t = m / g.Wo, ho = t % g.Ho, n = t / g.Ho;
        hb_[i] = ho * g.stride - g.pad; wb_[i] = wo * g.stride - g.pad; nb_[i] = n;
      } else { nb_[i] = -1; hb_[i] = 0; wb_[i] = 0; }
    }
  }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
    const int k = k0 + (tid & 7) * 8;
    int r, s, ci;
    tap_of(k, k0, g.C, g.KW, r, s, ci);
    const bool kv = k < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hi = hb_[i] + r * g.dil, wi = wb_[i] + s * g.dil;
      const bool ok = kv && nb_[i] >= 0 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      v[i] = ok ? ld16(x + (((size_t)nb_[i] * g.H + hi) * g.W + wi) * g.C + ci) : zero4();
    }
  }
};

// Row order of a dgrad output: for stride 1 the natural (n, hi, wi) order; for stride
// S > 1 parity-class-major: class c = ph*S + pw holds pixels hi = i*S+ph, wi = j*S+pw.
struct DgradRows {
  int N, H, W, S;
  __device__ __forceinline__ void decode(int m, int& n, int& hi, int& wi, int& cls) const {
    if (S == 1) {
      wi = m % W; const int t = m / W; hi = t % H; n = t / H; cls = 0;
      return;
    }
    int base = 0;
    for (int ph = 0; ph < S; ++ph) {
      const int Hc = (H - ph + S - 1) / S;
      for (int pw = 0; pw < S; ++pw) {
        const int Wc = (W - pw + S - 1) / S;
        const int sz = N * Hc * Wc;
        if (m < base + sz) {
          const int l = m - base;
          const int j = l % Wc, t = l / Wc, i = t % Hc;
          n = t / Hc; hi = i * S + ph; wi = j * S + pw; cls = ph * S + pw;
          return;
        }
        base += sz;
      }
    }
    n = N; hi = 0; wi = 0; cls = -1;
  }
};

// conv dgrad A operand: rows = input pixels q=(n,hi,wi) in DgradRows order,
// k = (r, s, co), co fastest
struct ConvDgradA {
  static constexpr bool KC = true;
  const bf16* dy; ConvGeom g; int M, K; DgradRows rows;
  int h_[4], w_[4], n_[4];
  int cls_;   // parity class shared by every row of the block, or -1 (mixed)
  __device__ void init(int m0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      if (m < M) {
        int n, hi, wi, c;
        rows.decode(m, n, hi, wi, c);
        h_[i] = hi + g.pad; w_[i] = wi + g.pad; n_[i] = n;
      } else { n_[i] = -1; h_[i] = 0; w_[i] = 0; }
    }
    cls_ = -1;
    if (g.stride > 1 && g.Co % BK == 0) {
      int n, hi, wi, c0, c1;
      rows.decode(m0, n, hi, wi, c0);
      rows.decode(min(m0 + BM, M) - 1, n, hi, wi, c1);
      if (c0 == c1) cls_ = c0;
    }
  }
  // first K-tile >= kt (and < e) whose filter tap can reach this block's class
  __device__ int next(int kt, int e) const {
    if (cls_ < 0) return kt;
    const int S = g.stride, ph = cls_ / S, pw = cls_ % S;
    for (; kt < e; ++kt) {
      const int rs = (kt * BK) / g.Co, s = rs % g.KW, r = rs / g.KW;
      const int a = ph + g.pad - r * g.dil, b = pw + g.pad - s * g.dil;
      if (((a % S) + S) % S == 0 && ((b % S) + S) % S == 0) break;
    }
    return kt;
  }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
    const int k = k0 + (tid & 7) * 8;
    int r, s, co;
    tap_of(k, k0, g.Co, g.KW, r, s, co);
    const bool kv = k < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int th = h_[i] - r * g.dil, tw = w_[i] - s * g.dil;
      bool ok = kv && n_[i] >= 0 && th >= 0 && tw >= 0;
      int ho = th, wo = tw;
      if (g.stride != 1) {
        ok = ok && (th % g.stride == 0) && (tw % g.stride == 0);
        ho = th / g.stride; wo = tw / g.stride;
      }
      ok = ok && ho < g.Ho && wo < g.Wo;
      v[i] = ok ? ld16(dy + (((size_t)n_[i] * g.Ho + ho) * g.Wo + wo) * g.Co + co) : zero4();
    }
  }
};

// conv dgrad B operand: k = (r, s, co) rows, cols = ci; W stored [co][r][s][ci]
struct ConvDgradB : AllTiles {
  static constexpr bool KC = false;
  const bf16* w; ConvGeom g; int K;
  int c_;
  __device__ void init(int n0, int tid) { c_ = n0 + (tid & 15) * 8; }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + (tid >> 4) + 16 * i;
      int r, s, co;
      tap_of(k, k0, g.Co, g.KW, r, s, co);
      v[i] = (k < K && c_ < g.C) ? ld16(w + (((size_t)co * g.KH + r) * g.KW + s) * g.C + c_) : zero4();
    }
  }
};

// conv wgrad B operand: k = output pixel p rows, cols = kk = (r, s, ci)
struct ConvWgradB : AllTiles {
  static constexpr bool KC = false;
  const bf16* x; ConvGeom g; int P, KK;
  int r_, s_, ci_; bool cv_;
  __device__ void init(int n0, int tid) {
    const int kk = n0 + (tid & 15) * 8;
    cv_ = kk < KK;
    ci_ = kk % g.C; const int rs = kk / g.C; s_ = rs % g.KW; r_ = rs / g.KW;
  }
  __device__ void load(int k0, int tid, uint4 (&v)[4]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = k0 + (tid >> 4) + 16 * i;
      const int wo = p % g.Wo, t = p / g.Wo, ho = t % g.Ho, n = t / g.Ho;
      const int hi = ho * g.stride - g.pad + r_ * g.dil, wi = wo * g.stride - g.pad + s_ * g.dil;
      const bool ok = cv_ && p < P && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      v[i] = ok ? ld16(x + (((size_t)n * g.H + hi) * g.W + wi) * g.C + ci_) : zero4();
    }
  }
};

// ---------------------------------------------------------------- epilogues
// acc[i][j][reg] holds C[m][n] with m = wm*64 + 32i + (reg&3) + 8(reg>>2) + 4(lane>>5),
// n = wn*64 + 32j + (lane&31)  (gfx950 32x32 C/D map)

struct IdentityRows {
  __device__ __forceinline__ size_t operator()(int m) const { return (size_t)m; }
};
struct DgradOutRows {  // DgradRows order -> NHWC pixel index
  DgradRows r;
  __device__ __forceinline__ size_t operator()(int m) const {
    int n, hi, wi, c;
    r.decode(m, n, hi, wi, c);
    return ((size_t)n * r.H + hi) * r.W + wi;
  }
};

template <class RowMap = IdentityRows>
struct EpiBF16 {  // bf16 [M][ld] store, optional per-column sum / sum of squares
  bf16* out; int ld; float* sum; float* sumsq; RowMap rowmap;
  __device__ void apply(f32x16 (&acc)[2][2], char* lds, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int tid) const {
    if (sum) {
      // copy slot spreads the per-channel atomics of different blocks over NSTAT rows
      const int slot = ((m0 / BM) * 2 + wm) & (NSTAT - 1);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) { const float v = acc[i][j][r]; s1 += v; s2 += v * v; }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        const int n = n0 + wn * 64 + 32 * j + lane;
        if (lane < 32 && n < N) {
          atomicAdd(sum + (size_t)slot * N + n, s1);
          atomicAdd(sumsq + (size_t)slot * N + n, s2);
        }
      }
    }
    // stage the 128x128 tile through LDS as bf16 rows of 272 B, then 16 B/lane stores
    constexpr int RS = 272;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int n = wn * 64 + 32 * j + (lane & 31);
          *reinterpret_cast<bf16*>(lds + m * RS + n * 2) = (bf16)acc[i][j][r];
        }
    __syncthreads();
    const int c = tid & 15;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = (tid >> 4) + 16 * it;
      const int m = m0 + row, n = n0 + c * 8;
      if (m < M && n < N)
        *reinterpret_cast<uint4*>(out + rowmap(m) * ld + n) = *reinterpret_cast<const uint4*>(lds + row * RS + c * 16);
    }
  }
};

struct EpiF32Atomic {  // fp32 [M][ld] += (split-K partial sums)
  float* out; int ld;
  __device__ void apply(f32x16 (&acc)[2][2], char*, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int) const {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + 32 * j + (lane & 31);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) atomicAdd(out + (size_t)m * ld + n, acc[i][j][r]);
        }
      }
  }
};

struct EpiF32 {  // fp32 [M][ld] = acc (+ bias[n]) (+= if accumulate)
  float* out; int ld; const float* bias; int accumulate;
  __device__ void apply(f32x16 (&acc)[2][2], char*, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int) const {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + 32 * j + (lane & 31);
        if (n >= N) continue;
        const float b = bias ? bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < M) {
            float* o = out + (size_t)m * ld + n;
            *o = (accumulate ? *o : 0.f) + acc[i][j][r] + b;
          }
        }
      }
  }
};

// ---------------------------------------------------------------- main loop
template <class LA, class LB, class EPI>
__global__ void __launch_bounds__(NTHR, 2)
gemm_kernel(LA la, LB lb, EPI epi, int M, int N, int K, int ktiles_per_split) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

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
  const int kt_begin = blockIdx.z * ktiles_per_split;
  const int kt_end = min(ktiles, kt_begin + ktiles_per_split);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  la.init(m0, tid);
  lb.init(n0, tid);
  int kt = la.next(kt_begin, kt_end);
  if (kt < kt_end) {
    uint4 ra[4], rb[4];
    la.load(kt * BK, tid, ra);
    lb.load(kt * BK, tid, rb);
    store_stage<LA::KC>(smem, tid, ra);
    store_stage<LB::KC>(smem + TILE_BYTES, tid, rb);
    __syncthreads();

    int cur = 0;
    while (kt < kt_end) {
      char* As = smem + cur * 2 * TILE_BYTES;
      char* Bs = As + TILE_BYTES;
      const int nxt = la.next(kt + 1, kt_end);
      const bool more = nxt < kt_end;
      if (more) {  // issue next tile's global loads before the MFMAs (T14)
        la.load(nxt * BK, tid, ra);
        lb.load(nxt * BK, tid, rb);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 a0 = read_frag<LA::KC>(As, wm * 64, s, lane);
        bf16x8 a1 = read_frag<LA::KC>(As, wm * 64 + 32, s, lane);
        bf16x8 b0 = read_frag<LB::KC>(Bs, wn * 64, s, lane);
        bf16x8 b1 = read_frag<LB::KC>(Bs, wn * 64 + 32, s, lane);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
      }
      if (more) {
        char* An = smem + (cur ^ 1) * 2 * TILE_BYTES;
        store_stage<LA::KC>(An, tid, ra);
        store_stage<LB::KC>(An + TILE_BYTES, tid, rb);
      }
      __syncthreads();
      cur ^= 1;
      kt = nxt;
    }
  }
  epi.apply(acc, smem, m0, n0, M, N, wm, wn, lane, tid);
}

template <class LA, class LB, class EPI>
static hipError_t launch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K,
                         int splits, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = (ktiles + splits - 1) / splits;
  splits = (ktiles + per - 1) / per;
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((gemm_kernel<LA, LB, EPI>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
  return hipGetLastError();
}

// pick a split-K factor so a small-output / long-K GEMM still fills 256 CUs
static int auto_splits(int M, int N, int K) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < 768 && ktiles / (s * 2) >= 8) s *= 2;
  return s;
}

}  // namespace igemm

using namespace igemm;

static ConvGeom mkgeom(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                       int dil, int Ho, int Wo) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Co = Co; g.KH = KH; g.KW = KW;
  g.stride = stride; g.pad = pad; g.dil = dil; g.Ho = Ho; g.Wo = Wo;
  return g;
}

MLC_EXPORT int mlc_bn_stat_copies() { return NSTAT; }

// y[N,Ho,Wo,Co] = conv(x[N,H,W,C], w[Co,KH,KW,C]).  If sum/sumsq are given they must
// hold NSTAT*Co fp32 (zeroed by the caller); per-channel partial sums of y and y^2 are
// accumulated into them (reduce over the NSTAT copies to get the BN statistics).
// Requires C % 8 == 0 and Co % 8 == 0.
MLC_EXPORT int mlc_conv_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq,
                            int N, int H, int W, int C, int Co, int KH, int KW, int stride,
                            int pad, int dil, int Ho, int Wo, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int M = N * Ho * Wo, K = KH * KW * C;
  EpiBF16<> epi{y, Co, sum, sumsq, IdentityRows{}};
  MatKC lb{{}, w, K, Co, K};
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    MatKC la{{}, x, C, M, K};
    return launch(la, lb, epi, M, Co, K, 1, st);
  }
  ConvFwdA la{{}, x, mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo), M, K};
  return launch(la, lb, epi, M, Co, K, 1, st);
}

// dx[N,H,W,C] = conv_transpose(dy[N,Ho,Wo,Co], w)
MLC_EXPORT int mlc_conv_dgrad(const bf16* dy, const bf16* w, bf16* dx, int N, int H, int W,
                              int C, int Co, int KH, int KW, int stride, int pad, int dil,
                              int Ho, int Wo, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int M = N * H * W, K = KH * KW * Co;
  ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  ConvDgradB lb{{}, w, g, K};
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}};
    MatKC la{{}, dy, Co, M, K};
    return launch(la, lb, epi, M, C, K, 1, st);
  }
  DgradRows rows{N, H, W, stride};
  ConvDgradA la{dy, g, M, K, rows};
  if (stride == 1) {
    EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}};
    return launch(la, lb, epi, M, C, K, 1, st);
  }
  EpiBF16<DgradOutRows> epi{dx, C, nullptr, nullptr, DgradOutRows{rows}};
  return launch(la, lb, epi, M, C, K, 1, st);
}

// dw[Co, KH*KW*C] (fp32) = sum_p dy[p][co] * im2col(x)[p][kk]; zeroes dw first unless
// accumulate != 0.  splits <= 0 picks a split-K factor automatically.
MLC_EXPORT int mlc_conv_wgrad(const bf16* dy, const bf16* x, float* dw, int N, int H, int W,
                              int C, int Co, int KH, int KW, int stride, int pad, int dil,
                              int Ho, int Wo, int splits, int accumulate, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int P = N * Ho * Wo, KK = KH * KW * C;
  if (!accumulate) (void)hipMemsetAsync(dw, 0, (size_t)Co * KK * sizeof(float), st);
  if (splits <= 0) splits = auto_splits(Co, KK, P);
  EpiF32Atomic epi{dw, KK};
  MatMC la{{}, dy, Co, P, Co};
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    MatMC lb{{}, x, C, P, C};
    return launch(la, lb, epi, Co, KK, P, splits, st);
  }
  ConvWgradB lb{{}, x, mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo), P, KK};
  return launch(la, lb, epi, Co, KK, P, splits, st);
}

// Generic bf16 GEMM with fp32 output: C[M][N] (+)= op(A) op(B) (+ bias)
//   ta=0: A is [M][K] (lda);  ta=1: A is [K][M]
//   tb=0: B is [K][N] (ldb);  tb=1: B is [N][K]
// out_mode 0: store (+bias, accumulate flag), 1: atomic add (split-K allowed; the
// caller zeroes C unless accumulating)
MLC_EXPORT int mlc_gemm_f32out(const bf16* A, const bf16* B, float* C, const float* bias,
                               int M, int N, int K, int lda, int ldb, int ldc, int ta, int tb,
                               int out_mode, int accumulate, int splits, hipStream_t st) {
  if (K % 8 || lda % 8 || ldb % 8 || (ta && M % 8) || (!tb && N % 8)) return -1;
  if (out_mode == 1) {
    if (splits <= 0) splits = auto_splits(M, N, K);
    EpiF32Atomic epi{C, ldc};
    if (!ta && tb) return launch(MatKC{{}, A, lda, M, K}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, splits, st);
    if (!ta && !tb) return launch(MatKC{{}, A, lda, M, K}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, splits, st);
    if (ta && tb) return launch(MatMC{{}, A, lda, K, M}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, splits, st);
    return launch(MatMC{{}, A, lda, K, M}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, splits, st);
  }
  EpiF32 epi{C, ldc, bias, accumulate};
  if (!ta && tb) return launch(MatKC{{}, A, lda, M, K}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, 1, st);
  if (!ta && !tb) return launch(MatKC{{}, A, lda, M, K}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, 1, st);
  if (ta && tb) return launch(MatMC{{}, A, lda, K, M}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, 1, st);
  return launch(MatMC{{}, A, lda, K, M}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, 1, st);
}

// bf16-output GEMM (same layout flags)
MLC_EXPORT int mlc_gemm_bf16out(const bf16* A, const bf16* B, bf16* C, int M, int N, int K,
                                int lda, int ldb, int ldc, int ta, int tb, hipStream_t st) {
  if (K % 8 || N % 8 || ldc % 8 || lda % 8 || ldb % 8 || (ta && M % 8)) return -1;
  EpiBF16<> epi{C, ldc, nullptr, nullptr, IdentityRows{}};
  if (!ta && tb) return launch(MatKC{{}, A, lda, M, K}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, 1, st);
  if (!ta && !tb) return launch(MatKC{{}, A, lda, M, K}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, 1, st);
  if (ta && tb) return launch(MatMC{{}, A, lda, K, M}, MatKC{{}, B, ldb, N, K}, epi, M, N, K, 1, st);
  return launch(MatMC{{}, A, lda, K, M}, MatMC{{}, B, ldb, K, N}, epi, M, N, K, 1, st);
}
