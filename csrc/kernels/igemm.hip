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

namespace igemm {

constexpr int BK = 64, NTHR = 256;
constexpr int NSTAT = 32;                          // BN-stat partial copies

// ------------------------------------------------------------------ fast division
struct FastDiv {
  unsigned d, mul, sh;
  __host__ __device__ FastDiv() : d(1), mul(0), sh(0) {}
  __host__ explicit FastDiv(unsigned dd) : d(dd) {
    sh = 0;
    while ((1u << sh) < d) ++sh;
    mul = (unsigned)((((unsigned long long)1 << 32) * ((1ull << sh) - d)) / d + 1);
  }
  __device__ __forceinline__ unsigned div(unsigned n) const { return (__umulhi(n, mul) + n) >> sh; }
  __device__ __forceinline__ void divmod(unsigned n, unsigned& q, unsigned& r) const {
    q = div(n); r = n - q * d;
  }
};

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

// tile of R rows (KC) / R cols (MC): NCH = R/32 chunks of 16 B per thread
template <bool KC, int R>
__device__ __forceinline__ void store_stage(char* lds, int tid, const uint4 (&v)[R / 32]) {
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    int off;
    if (KC) off = kc_off((tid >> 3) + 32 * i, tid & 7);
    else off = mc_off<R>(tid / (R / 8) + (NTHR / (R / 8)) * i, tid % (R / 8));
    *reinterpret_cast<uint4*>(lds + off) = v[i];
  }
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

__device__ __forceinline__ uint4 ld16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }

// Default K-tile iteration: every tile in [b, e).
struct AllTiles {
  template <class S>
  __device__ int next(const S&, int kt, int) const { return kt; }
};

// ---------------------------------------------------------------- geometry
struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int Ho, Wo, Co;      // output
  int KH, KW, stride, pad, dil;
  FastDiv fWo, fHo, fW, fH, fC, fCo, fKW;
};

// decompose k = ((r*KW)+s)*CC + c; if CC % BK == 0 a whole K-tile shares one tap, so
// only the (wave-uniform) tile base is decomposed.
__device__ __forceinline__ void tap_of(int k, int k0, const FastDiv& fCC, const FastDiv& fKW,
                                       int& r, int& s, int& c) {
  unsigned rs, cc, rr, ss;
  if (fCC.d % BK == 0) {
    fCC.divmod((unsigned)k0, rs, cc);
    c = (int)cc + (k - k0);
  } else {
    fCC.divmod((unsigned)k, rs, cc);
    c = (int)cc;
  }
  fKW.divmod(rs, rr, ss);
  r = (int)rr; s = (int)ss;
}

// ---------------------------------------------------------------- loaders
// KC loader of R rows: thread t owns rows (t>>3)+32i, chunk t&7 (8 k per chunk).
// MC loader of R cols: thread t owns chunk t%(R/8) (8 mn), k-rows t/(R/8) + (256/(R/8))i.

template <int R>
struct MatKC : AllTiles {
  static constexpr bool KC = true;
  const bf16* p; int ld, rows, K;
  struct St { int r[R / 32]; };
  __device__ void init(St& st, int m0, int tid) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) st.r[i] = m0 + (tid >> 3) + 32 * i;
  }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
    const int k = k0 + (tid & 7) * 8;
#pragma unroll
    for (int i = 0; i < R / 32; ++i)
      v[i] = (st.r[i] < rows && k < K) ? ld16(p + (size_t)st.r[i] * ld + k) : zero4();
  }
};

template <int R>
struct MatMC : AllTiles {
  static constexpr bool KC = false;
  const bf16* p; int ld, K, cols;
  struct St { int c; };
  __device__ void init(St& st, int n0, int tid) const { st.c = n0 + (tid % (R / 8)) * 8; }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int k = k0 + tid / (R / 8) + (NTHR / (R / 8)) * i;
      v[i] = (k < K && st.c < cols) ? ld16(p + (size_t)k * ld + st.c) : zero4();
    }
  }
};

// conv fwd A operand: rows = output pixels, k = (r, s, ci) with ci fastest (C % 8 == 0)
template <int R>
struct ConvFwdA : AllTiles {
  static constexpr bool KC = true;
  const bf16* x; ConvGeom g; int M, K;
  struct St { int hb[R / 32], wb[R / 32], nb[R / 32]; };  // per-row base input coords, nb=-1 if row >= M
  __device__ void init(St& st, int m0, int tid) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      // branch-free: a conditional store into st.* is sunk into a dynamic-index store
      // by the compiler, which moves the whole array to scratch
      const int m = m0 + (tid >> 3) + 32 * i;
      const bool ok = m < M;
      unsigned t, wo, n, ho;
      g.fWo.divmod((unsigned)(ok ? m : 0), t, wo);
      g.fHo.divmod(t, n, ho);
      st.hb[i] = (int)ho * g.stride - g.pad;
      st.wb[i] = (int)wo * g.stride - g.pad;
      st.nb[i] = ok ? (int)n : -1;
    }
  }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
    const int k = k0 + (tid & 7) * 8;
    int r, s, ci;
    tap_of(k, k0, g.fC, g.fKW, r, s, ci);
    const bool kv = k < K;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int hi = st.hb[i] + r * g.dil, wi = st.wb[i] + s * g.dil;
      const bool ok = kv && st.nb[i] >= 0 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      v[i] = ok ? ld16(x + (((size_t)st.nb[i] * g.H + hi) * g.W + wi) * g.C + ci) : zero4();
    }
  }
};

// Row order of a dgrad output: for stride 1 the natural (n, hi, wi) order; for stride 2
// parity-class-major: class c = ph*2 + pw holds pixels hi = 2i+ph, wi = 2j+pw.
struct DgradRows {
  int N, H, W, S;
  int nclass;            // parity classes with at least one contributing filter tap
  int base[4];           // start row of each listed class (INT_MAX when unused)
  int cid[4];            // class id (ph*2+pw) of each listed class
  FastDiv fWc[4], fHc[4];
  FastDiv fW, fH;
  __device__ __forceinline__ void decode(int m, int& n, int& hi, int& wi, int& cls) const {
    unsigned t, q, rr;
    if (S == 1) {
      fW.divmod((unsigned)m, t, rr); wi = (int)rr;
      fH.divmod(t, q, rr); hi = (int)rr; n = (int)q; cls = 0;
      return;
    }
    const int k = (m >= base[1]) + (m >= base[2]) + (m >= base[3]);
    // explicit selects: a runtime index into these arrays would force them to scratch
    const int b = k == 0 ? base[0] : k == 1 ? base[1] : k == 2 ? base[2] : base[3];
    const int c = k == 0 ? cid[0] : k == 1 ? cid[1] : k == 2 ? cid[2] : cid[3];
    const FastDiv fw = k == 0 ? fWc[0] : k == 1 ? fWc[1] : k == 2 ? fWc[2] : fWc[3];
    const FastDiv fh = k == 0 ? fHc[0] : k == 1 ? fHc[1] : k == 2 ? fHc[2] : fHc[3];
    const unsigned l = (unsigned)(m - b);
    fw.divmod(l, t, rr);
    const int j = (int)rr;
    fh.divmod(t, q, rr);
    n = (int)q; hi = 2 * (int)rr + (c >> 1); wi = 2 * j + (c & 1); cls = c;
  }
};

// conv dgrad A operand: rows = input pixels (DgradRows order), k = (r, s, co), co fastest
template <int R>
struct ConvDgradA {
  static constexpr bool KC = true;
  const bf16* dy; ConvGeom g; int M, K; DgradRows rows;
  // per-row coords; cls: parity class shared by every row of the block, or -1
  struct St { int h[R / 32], w[R / 32], n[R / 32]; int cls; };
  __device__ void init(St& st, int m0, int tid) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      const bool ok = m < M;
      int n, hi, wi, c;
      rows.decode(ok ? m : 0, n, hi, wi, c);
      st.h[i] = hi + g.pad;
      st.w[i] = wi + g.pad;
      st.n[i] = ok ? n : -1;
    }
    st.cls = -1;
    if (g.stride == 2 && g.Co % BK == 0) {
      int n, hi, wi, c0, c1;
      rows.decode(m0, n, hi, wi, c0);
      rows.decode(min(m0 + R, M) - 1, n, hi, wi, c1);
      if (c0 == c1) st.cls = c0;
    }
  }
  // first K-tile >= kt (and < e) whose filter tap can reach this block's class
  __device__ int next(const St& st, int kt, int e) const {
    if (st.cls < 0) return kt;
    const int ph = st.cls >> 1, pw = st.cls & 1;
    for (; kt < e; ++kt) {
      unsigned rs, rem, r, s;
      g.fCo.divmod((unsigned)(kt * BK), rs, rem);
      g.fKW.divmod(rs, r, s);
      if ((((ph + g.pad - (int)r * g.dil) & 1) == 0) && (((pw + g.pad - (int)s * g.dil) & 1) == 0)) break;
    }
    return kt;
  }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
    const int k = k0 + (tid & 7) * 8;
    int r, s, co;
    tap_of(k, k0, g.fCo, g.fKW, r, s, co);
    const bool kv = k < K;
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int th = st.h[i] - r * g.dil, tw = st.w[i] - s * g.dil;
      bool ok = kv && st.n[i] >= 0 && th >= 0 && tw >= 0;
      int ho = th, wo = tw;
      if (g.stride == 2) {
        ok = ok && ((th & 1) == 0) && ((tw & 1) == 0);
        ho = th >> 1; wo = tw >> 1;
      } else if (g.stride != 1) {
        ok = ok && (th % g.stride == 0) && (tw % g.stride == 0);
        ho = th / g.stride; wo = tw / g.stride;
      }
      ok = ok && ho < g.Ho && wo < g.Wo;
      v[i] = ok ? ld16(dy + (((size_t)st.n[i] * g.Ho + ho) * g.Wo + wo) * g.Co + co) : zero4();
    }
  }
};

// conv dgrad B operand: k = (r, s, co) rows, cols = ci; W stored [co][r][s][ci]
template <int R>
struct ConvDgradB : AllTiles {
  static constexpr bool KC = false;
  const bf16* w; ConvGeom g; int K;
  struct St { int c; };
  __device__ void init(St& st, int n0, int tid) const { st.c = n0 + (tid % (R / 8)) * 8; }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int k = k0 + tid / (R / 8) + (NTHR / (R / 8)) * i;
      int r, s, co;
      tap_of(k, k0, g.fCo, g.fKW, r, s, co);
      v[i] = (k < K && st.c < g.C) ? ld16(w + (((size_t)co * g.KH + r) * g.KW + s) * g.C + st.c) : zero4();
    }
  }
};

// conv wgrad B operand: k = output pixel p rows, cols = kk = (r, s, ci)
template <int R>
struct ConvWgradB : AllTiles {
  static constexpr bool KC = false;
  const bf16* x; ConvGeom g; int P, KK;
  struct St { int r, s, ci; bool cv; };
  __device__ void init(St& st, int n0, int tid) const {
    const int kk = n0 + (tid % (R / 8)) * 8;
    st.cv = kk < KK;
    unsigned rs, ci, r, s;
    g.fC.divmod((unsigned)kk, rs, ci);
    g.fKW.divmod(rs, r, s);
    st.ci = (int)ci; st.r = (int)r; st.s = (int)s;
  }
  __device__ void load(const St& st, int k0, int tid, uint4 (&v)[R / 32]) const {
#pragma unroll
    for (int i = 0; i < R / 32; ++i) {
      const int p = k0 + tid / (R / 8) + (NTHR / (R / 8)) * i;
      unsigned t, wo, n, ho;
      g.fWo.divmod((unsigned)p, t, wo);
      g.fHo.divmod(t, n, ho);
      const int hi = (int)ho * g.stride - g.pad + st.r * g.dil, wi = (int)wo * g.stride - g.pad + st.s * g.dil;
      const bool ok = st.cv && p < P && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      v[i] = ok ? ld16(x + (((size_t)n * g.H + hi) * g.W + wi) * g.C + st.ci) : zero4();
    }
  }
};

// ---------------------------------------------------------------- epilogues
// acc[i][j][reg] of wave (wm, wn) holds C[m][n] with
//   m = wm*64 + 32i + (reg&3) + 8(reg>>2) + 4(lane>>5),  n = wn*64 + 32j + (lane&31)

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

// BatchNorm-backward reduction fused into the epilogue of the dgrad that produces the
// final gradient dU of a BN's output (the branch-point sum is already in via addend):
//   dU <- dU * [mask > 0]   (ReLU of the BN being differentiated; mask = its output z)
//   sums_k[slot][0][c] += sum dU,  sums_k[slot][1][c] += sum dU*(y_k - mean_k)
// for up to two BNs sharing the same dU (a block's last BN and its downsample BN).  The
// masked dU is what gets stored, so the elementwise BN-backward pass needs neither z
// nor a separate residual-gradient copy.
struct BnBwdEpi {
  const bf16* mask = nullptr;
  const bf16* y0 = nullptr; const float* mean0 = nullptr; float* sums0 = nullptr;
  const bf16* y1 = nullptr; const float* mean1 = nullptr; float* sums1 = nullptr;
};

template <class RowMap = IdentityRows, bool kDense = false>
struct EpiBF16 {  // bf16 [M][ld] store (+ addend), optional per-column sum / sum of squares
  bf16* out; int ld; float* sum; float* sumsq; RowMap rowmap; const bf16* addend = nullptr;
  BnBwdEpi bn = {};
  // dense-layer extras: out = act(acc + bias) (pre-activation stored to preact), or
  // out = acc * act'(dact) for the backward of an activation (act 1 = exact-erf GELU)
  const float* bias = nullptr; int act = 0; bf16* preact = nullptr; const bf16* dact = nullptr;
  template <int BM, int BN>
  __device__ void apply(f32x16 (&acc)[2][2], char* lds, int m0, int n0, int M, int N,
                        int wm, int wn, int lane, int tid) const {
    if (sum) {
      // copy slot spreads the per-channel atomics of different blocks over NSTAT rows
      const int slot = ((m0 / 64) + wm) & (NSTAT - 1);
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
    // stage the BMxBN tile through LDS as bf16 rows of (BN+8)*2 B, then 16 B/lane stores
    constexpr int RS = (BN + 8) * 2;
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
    constexpr int CPR = BN / 8;              // 16 B chunks per row
    constexpr int RPI = NTHR / CPR;          // rows per iteration
    const int c = tid % CPR;
    const int nc = n0 + c * 8;
    const bool red = !kDense && bn.y0 != nullptr;
    float mu0[8], mu1[8], s1[8], s2[8], t2[8];
    if (red) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mu0[e] = nc < N ? bn.mean0[nc + e] : 0.f;
        mu1[e] = (bn.y1 && nc < N) ? bn.mean1[nc + e] : 0.f;
        s1[e] = 0.f; s2[e] = 0.f; t2[e] = 0.f;
      }
    }
    const bool dense = kDense && (bias || act || dact);
    if (!addend && !red && !dense) {  // plain store (forward convs / GEMMs)
#pragma unroll
      for (int it = 0; it < BM / RPI; ++it) {
        const int row = tid / CPR + RPI * it;
        const int m = m0 + row;
        if (m < M && nc < N)
          *reinterpret_cast<uint4*>(out + rowmap(m) * ld + nc) =
              *reinterpret_cast<const uint4*>(lds + row * RS + c * 16);
      }
      return;
    }
    // rows are processed U at a time: every global load of a chunk (addend, mask, y) is
    // issued before the chunk's stores, so the loads overlap instead of serialising
    // behind stores the compiler must assume alias them (out may alias addend)
    constexpr int ITERS = BM / RPI;
    constexpr int U = ITERS < 4 ? ITERS : 4;
    const bool has_add = addend != nullptr, has_mask = red && bn.mask, has_y1 = red && bn.y1;
#pragma unroll
    for (int it0 = 0; it0 < ITERS; it0 += U) {
      constexpr int UB = kDense ? 1 : U;   // BN-reduction operands (conv dgrad only)
      constexpr int UD = kDense ? U : 1;   // activation-derivative operand (dense only)
      uint4 vv[U], aa[U], zz[UB], p0[UB], p1[UB], du[UD];
      size_t off[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = tid / CPR + RPI * (it0 + u);
        const int m = m0 + row;
        ok[u] = m < M && nc < N;
        off[u] = ok[u] ? rowmap(m) * ld + nc : 0;
        vv[u] = *reinterpret_cast<const uint4*>(lds + row * RS + c * 16);
        const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
        aa[u] = (ok[u] && has_add) ? *reinterpret_cast<const uint4*>(addend + off[u]) : zero;
        if constexpr (!kDense) {
          zz[u] = (ok[u] && has_mask) ? *reinterpret_cast<const uint4*>(bn.mask + off[u]) : zero;
          p0[u] = (ok[u] && red) ? *reinterpret_cast<const uint4*>(bn.y0 + off[u]) : zero;
          p1[u] = (ok[u] && has_y1) ? *reinterpret_cast<const uint4*>(bn.y1 + off[u]) : zero;
        }
        if constexpr (kDense) du[u] = (ok[u] && dact) ? *reinterpret_cast<const uint4*>(dact + off[u]) : zero;
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
            for (int e = 0; e < 8; ++e) a[e] += bias[nc + e];
          }
          if (preact) *reinterpret_cast<uint4*>(preact + off[u]) = pack8(a);
          if (act == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = 0.5f * a[e] * (1.f + erff(a[e] * 0.70710678118654752f));
          }
          if (dact) {
            float z[8];
            unpack8(du[u], z);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float cdf = 0.5f * (1.f + erff(z[e] * 0.70710678118654752f));
              const float pdf = 0.3989422804014327f * __expf(-0.5f * z[e] * z[e]);
              a[e] *= cdf + z[e] * pdf;
            }
          }
          }
          if (has_add) {  // fused residual-gradient sum (dx of a branch point)
            float b[8];
            unpack8(aa[u], b);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += b[e];
          }
          if constexpr (!kDense) if (has_mask) {
            float z[8];
            unpack8(zz[u], z);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
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
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        rb[tid * 24 + e] = s1[e];
        rb[tid * 24 + 8 + e] = s2[e];
        rb[tid * 24 + 16 + e] = t2[e];
      }
      __syncthreads();
      if (tid < BN) {
        const int col = tid, cc = col >> 3, e = col & 7, n = n0 + col;
        float a = 0.f, b = 0.f, d = 0.f;
        for (int r = 0; r < RPI; ++r) {
          const float* q = rb + (cc + CPR * r) * 24;
          a += q[e]; b += q[8 + e]; d += q[16 + e];
        }
        if (n < N) {
          const int slot = (m0 / BM) & (NSTAT - 1);
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

struct EpiF32Atomic {  // fp32 [M][ld] += (split-K partial sums)
  float* out; int ld;
  template <int BM, int BN>
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
  template <int BM, int BN>
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
template <int BM, int BN, class LA, class LB, class EPI, int PF>
__global__ void __launch_bounds__(NTHR, 2)
gemm_kernel(const LA la, const LB lb, const EPI epi, int M, int N, int K, int ktiles_per_split) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
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
  const int kt_begin = blockIdx.z * ktiles_per_split;
  const int kt_end = min(ktiles, kt_begin + ktiles_per_split);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  typename LA::St sa;
  typename LB::St sb;
  la.init(sa, m0, tid);
  lb.init(sb, n0, tid);
  auto mfma_tile = [&](const char* As, const char* Bs) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a0 = read_frag<LA::KC, BM>(As, wm * 64, s, lane);
      bf16x8 a1 = read_frag<LA::KC, BM>(As, wm * 64 + 32, s, lane);
      bf16x8 b0 = read_frag<LB::KC, BN>(Bs, wn * 64, s, lane);
      bf16x8 b1 = read_frag<LB::KC, BN>(Bs, wn * 64 + 32, s, lane);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
  };
  if constexpr (PF == 1) {
  int kt = la.next(sa, kt_begin, kt_end);
  if (kt < kt_end) {
    uint4 ra[BM / 32], rb[BN / 32];
    la.load(sa, kt * BK, tid, ra);
    lb.load(sb, kt * BK, tid, rb);
    store_stage<LA::KC, BM>(smem, tid, ra);
    store_stage<LB::KC, BN>(smem + A_BYTES, tid, rb);
    __syncthreads();

    int cur = 0;
    while (kt < kt_end) {
      char* As = smem + cur * STAGE;
      char* Bs = As + A_BYTES;
      const int nxt = la.next(sa, kt + 1, kt_end);
      const bool more = nxt < kt_end;
      if (more) {  // issue next tile's global loads before the MFMAs (T14)
        la.load(sa, nxt * BK, tid, ra);
        lb.load(sb, nxt * BK, tid, rb);
      }
      mfma_tile(As, Bs);
      if (more) {
        char* An = smem + (cur ^ 1) * STAGE;
        store_stage<LA::KC, BM>(An, tid, ra);
        store_stage<LB::KC, BN>(An + A_BYTES, tid, rb);
      }
      __syncthreads();
      cur ^= 1;
      kt = nxt;
    }
  }
  } else {
    // PF == 2: two register sets, global loads issued two K-tiles ahead.  The loop
    // body is unrolled twice so each set's role is static (no runtime-indexed arrays).
    int kt = la.next(sa, kt_begin, kt_end);
    if (kt < kt_end) {
      uint4 a0[BM / 32], b0[BN / 32], a1[BM / 32], b1[BN / 32];
      la.load(sa, kt * BK, tid, a0);
      lb.load(sb, kt * BK, tid, b0);
      store_stage<LA::KC, BM>(smem, tid, a0);
      store_stage<LB::KC, BN>(smem + A_BYTES, tid, b0);
      int k1 = la.next(sa, kt + 1, kt_end);
      if (k1 < kt_end) {
        la.load(sa, k1 * BK, tid, a1);
        lb.load(sb, k1 * BK, tid, b1);
      }
      __syncthreads();
      int cur = 0;
      while (true) {
        // phase A: compute kt; set 1 holds k1 (in flight); set 0 is free
        int k2 = k1 < kt_end ? la.next(sa, k1 + 1, kt_end) : kt_end;
        if (k2 < kt_end) {
          la.load(sa, k2 * BK, tid, a0);
          lb.load(sb, k2 * BK, tid, b0);
        }
        mfma_tile(smem + cur * STAGE, smem + cur * STAGE + A_BYTES);
        if (k1 < kt_end) {
          store_stage<LA::KC, BM>(smem + (cur ^ 1) * STAGE, tid, a1);
          store_stage<LB::KC, BN>(smem + (cur ^ 1) * STAGE + A_BYTES, tid, b1);
        }
        __syncthreads();
        cur ^= 1;
        kt = k1;
        if (kt >= kt_end) break;
        // phase B: compute kt; set 0 holds k2; set 1 is free
        k1 = k2 < kt_end ? la.next(sa, k2 + 1, kt_end) : kt_end;
        if (k1 < kt_end) {
          la.load(sa, k1 * BK, tid, a1);
          lb.load(sb, k1 * BK, tid, b1);
        }
        mfma_tile(smem + cur * STAGE, smem + cur * STAGE + A_BYTES);
        if (k2 < kt_end) {
          store_stage<LA::KC, BM>(smem + (cur ^ 1) * STAGE, tid, a0);
          store_stage<LB::KC, BN>(smem + (cur ^ 1) * STAGE + A_BYTES, tid, b0);
        }
        __syncthreads();
        cur ^= 1;
        kt = k2;
        if (kt >= kt_end) break;
      }
    }
  }
  epi.template apply<BM, BN>(acc, smem, m0, n0, M, N, wm, wn, lane, tid);
}

// K-tile prefetch depth of the main loop (1 = next tile, 2 = two tiles ahead); set by
// mlc_gemm_config for A/B measurements, default chosen from the microbenchmarks
static int g_prefetch = 1;

template <int BM, int BN, class LA, class LB, class EPI>
static hipError_t launch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K,
                         int splits, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles;
  const int per = (ktiles + splits - 1) / splits;
  splits = (ktiles + per - 1) / per;
  dim3 grid(tiles, 1, splits);
  if (g_prefetch >= 2 && per >= 3)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 2>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, EPI, 1>), grid, dim3(NTHR), 0, st, la, lb, epi, M, N, K, per);
  return hipGetLastError();
}

// tile shape: 0 = 128x128, 1 = 256x64 (narrow N), 2 = 64x256 (narrow M)
static int pick_tile(int M, int N) {
  if (N <= 64 && M > 64) return 1;
  if (M <= 64 && N > 64) return 2;
  return 0;
}

// pick a split-K factor so a small-output / long-K GEMM still fills 256 CUs
static int auto_splits(int M, int N, int K, int tile) {
  const int BMv = tile == 1 ? 256 : tile == 2 ? 64 : 128;
  const int BNv = tile == 1 ? 64 : tile == 2 ? 256 : 128;
  const int tiles = ((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv);
  const int ktiles = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < 768 && ktiles / (s * 2) >= 4) s *= 2;
  return s;
}

}  // namespace igemm

using namespace igemm;

static ConvGeom mkgeom(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                       int dil, int Ho, int Wo) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Co = Co; g.KH = KH; g.KW = KW;
  g.stride = stride; g.pad = pad; g.dil = dil; g.Ho = Ho; g.Wo = Wo;
  g.fWo = FastDiv(Wo); g.fHo = FastDiv(Ho); g.fW = FastDiv(W); g.fH = FastDiv(H);
  g.fC = FastDiv(C); g.fCo = FastDiv(Co); g.fKW = FastDiv(KW);
  return g;
}

// Row plan of a dgrad output.  Stride 2: one row range per parity class that at least
// one filter tap reaches (a 1x1/s2 conv reaches only class (0,0)); rows of the other
// classes are structurally zero and are filled by a memset/copy instead of GEMM blocks.
static DgradRows mkrows(int N, int H, int W, int S, int KH, int KW, int pad, int dil, int* rows_out) {
  DgradRows r;
  r.N = N; r.H = H; r.W = W; r.S = S;
  r.fW = FastDiv(W); r.fH = FastDiv(H);
  r.nclass = 0;
  for (int k = 0; k < 4; ++k) { r.base[k] = 0x7fffffff; r.cid[k] = 0; }
  if (S != 2) { *rows_out = N * H * W; r.nclass = 1; r.base[0] = 0; return r; }
  int b = 0;
  for (int c = 0; c < 4; ++c) {
    const int ph = c >> 1, pw = c & 1;
    const int Hc = (H - ph + 1) / 2, Wc = (W - pw + 1) / 2;
    bool rv = false, sv = false;
    for (int t = 0; t < KH; ++t) rv |= (((ph + pad - t * dil) % 2) + 2) % 2 == 0;
    for (int t = 0; t < KW; ++t) sv |= (((pw + pad - t * dil) % 2) + 2) % 2 == 0;
    if (!rv || !sv || Hc <= 0 || Wc <= 0) continue;
    const int k = r.nclass++;
    r.base[k] = b; r.cid[k] = c;
    r.fHc[k] = FastDiv(Hc);
    r.fWc[k] = FastDiv(Wc);
    b += N * Hc * Wc;
  }
  *rows_out = b;
  return r;
}

// dispatch one GEMM over the three tile shapes; MK(R) builds the loaders for R rows
#define MLC_TILE_DISPATCH(TILE, M, N, K, SPLITS, ST, EPI, MKA, MKB)                              \
  do {                                                                                         \
    if ((TILE) == 1) return launch<256, 64>(MKA(256), MKB(64), EPI, M, N, K, SPLITS, ST);      \
    if ((TILE) == 2) return launch<64, 256>(MKA(64), MKB(256), EPI, M, N, K, SPLITS, ST);      \
    return launch<128, 128>(MKA(128), MKB(128), EPI, M, N, K, SPLITS, ST);                     \
  } while (0)

MLC_EXPORT int mlc_bn_stat_copies() { return NSTAT; }

MLC_EXPORT int mlc_gemm_config(int prefetch) {
  const int old = igemm::g_prefetch;
  if (prefetch == 1 || prefetch == 2) igemm::g_prefetch = prefetch;
  return old;
}

// y[N,Ho,Wo,Co] = conv(x[N,H,W,C], w[Co,KH,KW,C]).  If sum/sumsq are given they must
// hold NSTAT*Co fp32 (zeroed by the caller); per-channel partial sums of y and y^2 are
// accumulated into them (reduce over the NSTAT copies to get the BN statistics).
// Requires C % 8 == 0 and Co % 8 == 0.
MLC_EXPORT int mlc_conv_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq,
                            int N, int H, int W, int C, int Co, int KH, int KW, int stride,
                            int pad, int dil, int Ho, int Wo, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int M = N * Ho * Wo, K = KH * KW * C;
  const int tile = pick_tile(M, Co);
  EpiBF16<> epi{y, Co, sum, sumsq, IdentityRows{}};
#define MKB(R) (MatKC<R>{{}, w, K, Co, K})
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
#define MKA(R) (MatKC<R>{{}, x, C, M, K})
    MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
#define MKA(R) (ConvFwdA<R>{{}, x, g, M, K})
  MLC_TILE_DISPATCH(tile, M, Co, K, 1, st, epi, MKA, MKB);
#undef MKA
#undef MKB
}

// dx[N,H,W,C] = conv_transpose(dy[N,Ho,Wo,Co], w) (+ addend, same layout as dx; may
// alias dx) -- the addend fuses the gradient sum at a residual branch point.
// bn_y0 != null additionally fuses the backward reduction of the BatchNorm(s) whose
// output gradient dx is (see BnBwdEpi): dx is stored masked by bn_mask > 0 and the
// partial sums go to bn_sums{0,1}[NSTAT][2][C] (zeroed by the caller).  Only valid when
// every dx row is produced by the GEMM (not for stride-2 convs with unreachable taps).
MLC_EXPORT int mlc_conv_dgrad(const bf16* dy, const bf16* w, bf16* dx, const bf16* addend, int N,
                              int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                              int dil, int Ho, int Wo, const bf16* bn_mask, const bf16* bn_y0,
                              const float* bn_mean0, float* bn_sums0, const bf16* bn_y1,
                              const float* bn_mean1, float* bn_sums1, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int K = KH * KW * Co;
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
  BnBwdEpi bn{bn_mask, bn_y0, bn_mean0, bn_sums0, bn_y1, bn_mean1, bn_sums1};
  if (bn_y0 && (!bn_mean0 || !bn_sums0 || (bn_y1 && (!bn_mean1 || !bn_sums1)))) return -1;
#define MKB(R) (ConvDgradB<R>{{}, w, g, K})
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    const int M = N * H * W;
    const int tile = pick_tile(M, C);
    EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}, addend, bn};
#define MKA(R) (MatKC<R>{{}, dy, Co, M, K})
    MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
#undef MKA
  }
  int M = 0;
  const DgradRows rows = mkrows(N, H, W, stride == 2 ? 2 : 1, KH, KW, pad, dil, &M);
  const int tile = pick_tile(M, C);
#define MKA(R) (ConvDgradA<R>{dy, g, M, K, rows})
  if (stride != 2) {
    EpiBF16<> epi{dx, C, nullptr, nullptr, IdentityRows{}, addend, bn};
    MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
  }
  if (M < N * H * W) {  // classes no tap reaches: dx = addend there (or 0)
    if (bn_y0) return -1;
    const size_t bytes = (size_t)N * H * W * C * sizeof(bf16);
    if (addend) { if (addend != dx) (void)hipMemcpyAsync(dx, addend, bytes, hipMemcpyDeviceToDevice, st); }
    else (void)hipMemsetAsync(dx, 0, bytes, st);
  }
  if (M == 0) return hipGetLastError();
  EpiBF16<DgradOutRows> epi{dx, C, nullptr, nullptr, DgradOutRows{rows}, addend, bn};
  MLC_TILE_DISPATCH(tile, M, C, K, 1, st, epi, MKA, MKB);
#undef MKA
#undef MKB
}

// dw[Co, KH*KW*C] (fp32) = sum_p dy[p][co] * im2col(x)[p][kk]; zeroes dw first unless
// accumulate != 0.  splits <= 0 picks a split-K factor automatically.
MLC_EXPORT int mlc_conv_wgrad(const bf16* dy, const bf16* x, float* dw, int N, int H, int W,
                              int C, int Co, int KH, int KW, int stride, int pad, int dil,
                              int Ho, int Wo, int splits, int accumulate, hipStream_t st) {
  if (C % 8 || Co % 8) return -1;
  const int P = N * Ho * Wo, KK = KH * KW * C;
  const int tile = pick_tile(Co, KK);
  if (!accumulate) (void)hipMemsetAsync(dw, 0, (size_t)Co * KK * sizeof(float), st);
  if (splits <= 0) splits = auto_splits(Co, KK, P, tile);
  EpiF32Atomic epi{dw, KK};
#define MKA(R) (MatMC<R>{{}, dy, Co, P, Co})
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
#define MKB(R) (MatMC<R>{{}, x, C, P, C})
    MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
  }
  const ConvGeom g = mkgeom(N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo);
#define MKB(R) (ConvWgradB<R>{{}, x, g, P, KK})
  MLC_TILE_DISPATCH(tile, Co, KK, P, splits, st, epi, MKA, MKB);
#undef MKB
#undef MKA
}

// Generic bf16 GEMM with fp32 output: C[M][N] (+)= op(A) op(B) (+ bias)
//   ta=0: A is [M][K] (lda);  ta=1: A is [K][M]
//   tb=0: B is [K][N] (ldb);  tb=1: B is [N][K]
// out_mode 0: store (+bias, accumulate flag), 1: atomic add (split-K allowed; the
// caller zeroes C unless accumulating)
#define GA_KC(R) (MatKC<R>{{}, A, lda, M, K})
#define GA_MC(R) (MatMC<R>{{}, A, lda, K, M})
#define GB_KC(R) (MatKC<R>{{}, B, ldb, N, K})
#define GB_MC(R) (MatMC<R>{{}, B, ldb, K, N})

MLC_EXPORT int mlc_gemm_f32out(const bf16* A, const bf16* B, float* C, const float* bias,
                               int M, int N, int K, int lda, int ldb, int ldc, int ta, int tb,
                               int out_mode, int accumulate, int splits, hipStream_t st) {
  if (K % 8 || lda % 8 || ldb % 8 || (ta && M % 8) || (!tb && N % 8)) return -1;
  const int tile = pick_tile(M, N);
  if (out_mode == 1) {
    if (splits <= 0) splits = auto_splits(M, N, K, tile);
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

// bf16-output GEMM with a dense-layer epilogue: C = act(op(A) op(B) + bias) (pre-
// activation to preact when given), or C = (op(A) op(B)) * act'(dact) (+ addend).

// non-returning tile dispatch (for callers that continue after the GEMM)
template <class EPI, class FA, class FB>
static hipError_t launch_tiles(int tile, int M, int N, int K, int splits, hipStream_t st, const EPI& epi, FA fa,
                               FB fb) {
  if (tile == 1) return launch<256, 64>(fa.template make<256>(), fb.template make<64>(), epi, M, N, K, splits, st);
  if (tile == 2) return launch<64, 256>(fa.template make<64>(), fb.template make<256>(), epi, M, N, K, splits, st);
  return launch<128, 128>(fa.template make<128>(), fb.template make<128>(), epi, M, N, K, splits, st);
}
struct MkMatKC { const bf16* p; int ld, rows, K; template <int R> MatKC<R> make() const { return MatKC<R>{{}, p, ld, rows, K}; } };
struct MkMatMC { const bf16* p; int ld, K, cols; template <int R> MatMC<R> make() const { return MatMC<R>{{}, p, ld, K, cols}; } };
#define GA_KC_F (MkMatKC{A, lda, M, K})
#define GA_MC_F (MkMatMC{A, lda, K, M})
#define GB_KC_F (MkMatKC{B, ldb, N, K})
#define GB_MC_F (MkMatMC{B, ldb, K, N})

namespace {
// Split-K finish for the dense GEMM: ws [M][N] fp32 holds the split-K sums (zero on
// entry; re-zeroed here so the next call can reuse it), C = epilogue(ws) in bf16.
__global__ void __launch_bounds__(256)
dense_finalize_kernel(float* __restrict__ ws, bf16* __restrict__ C, int ldc, const float* __restrict__ bias,
                      int act, bf16* __restrict__ preact, const bf16* __restrict__ addend,
                      const bf16* __restrict__ dact, int M, int N) {
  const long n8 = (long)M * (N / 8);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const int m = (int)(i / (N / 8)), c = (int)(i % (N / 8)) * 8;
    float4* w4 = reinterpret_cast<float4*>(ws + (size_t)m * N + c);
    const float4 p = w4[0], q = w4[1];
    w4[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    w4[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    float a[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
    const size_t o = (size_t)m * ldc + c;
    if (bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += bias[c + e];
    }
    if (preact) *reinterpret_cast<uint4*>(preact + o) = pack8(a);
    if (act == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = 0.5f * a[e] * (1.f + erff(a[e] * 0.70710678118654752f));
    }
    if (dact) {
      float z[8];
      unpack8(*reinterpret_cast<const uint4*>(dact + o), z);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float cdf = 0.5f * (1.f + erff(z[e] * 0.70710678118654752f));
        a[e] *= cdf + z[e] * 0.3989422804014327f * __expf(-0.5f * z[e] * z[e]);
      }
    }
    if (addend) {
      float b[8];
      unpack8(*reinterpret_cast<const uint4*>(addend + o), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    *reinterpret_cast<uint4*>(C + o) = pack8(a);
  }
}
}  // namespace

// bf16-output GEMM with a dense-layer epilogue: C = act(op(A) op(B) + bias) (pre-
// activation to preact when given), or C = (op(A) op(B)) * act'(dact) (+ addend).
// ws (optional, M*N fp32, zero on entry and on exit): when the output has too few tiles
// to fill the chip, the K reduction is split across workgroups into ws with fp32 atomics
// and the epilogue runs in a finishing pass.
MLC_EXPORT int mlc_gemm_bf16_ex(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int lda, int ldb,
                                int ldc, int ta, int tb, const float* bias, int act, bf16* preact,
                                const bf16* addend, const bf16* dact, float* ws, hipStream_t st) {
  if (K % 8 || N % 8 || ldc % 8 || lda % 8 || ldb % 8 || (ta && M % 8)) return -1;
  const int tile = pick_tile(M, N);
  const int BMv = tile == 1 ? 256 : tile == 2 ? 64 : 128, BNv = tile == 1 ? 64 : tile == 2 ? 256 : 128;
  const int tiles = ((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv);
  const int ktiles = (K + BK - 1) / BK;
  int splits = 1;
  if (ws) while (tiles * splits < 384 && ktiles / (splits * 2) >= 4) splits *= 2;
  if (splits > 1) {
    EpiF32Atomic epi{ws, N};
    hipError_t e;
    if (!ta && tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_KC_F);
    else if (!ta && !tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_KC_F, GB_MC_F);
    else if (ta && tb) e = launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_KC_F);
    else e = launch_tiles(tile, M, N, K, splits, st, epi, GA_MC_F, GB_MC_F);
    if (e != hipSuccess) return e;
    long blocks = ((long)M * (N / 8) + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(dense_finalize_kernel, dim3(blocks), dim3(256), 0, st, ws, C, ldc, bias, act, preact,
                       addend, dact, M, N);
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
