// Transformer-encoder kernels (BERT family) for gfx950.
//
// * LayerNorm forward, fused with  s = x + dropout(r)  (the residual add of a post-LN
//   block) and an optional dropout on the output (embedding LN).  One 64-lane wave per
//   row, the row held in registers (H <= 64*4*MAXC), two-pass mean/variance, 8-byte
//   (4 x bf16) vector accesses.
// * LayerNorm backward: ds (+ the dropout-masked dr for the residual branch) and
//   dgamma/dbeta partial sums (per-block LDS reduction, one atomic per column per block
//   into one of NSTAT copies) + a finalize that writes them into the grad arena.
// * Attention softmax: P = softmax(scale*S + key_bias) with attention dropout; backward
//   dS = scale * P * (dP - sum(P*dP)).
// * Column sums for bias gradients (2D grid, partials into NSTAT copies, finalize).
//
// Dropout masks are a counter-based hash of (seed, site salt, element index): nothing is
// stored, backward regenerates the mask, and the seed lives in device memory so a
// captured HIP graph advances it on every replay.
#include "common.h"
#include "dropout.h"
#include <type_traits>

namespace {

constexpr int NT = 256;
constexpr int NSTAT = 32;

// 8-byte loads through an ext-vector type (see ldg16 in common.h); callers issue them from
// a clamped, always-valid column so no load sits under a per-lane branch
__device__ __forceinline__ void load4(const bf16* p, float* f) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 u = *reinterpret_cast<const u32x2*>(p);
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void load4f(const float* p, float* f) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const f32x4v v = *reinterpret_cast<const f32x4v*>(p);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
__device__ __forceinline__ void store4(bf16* p, const float* f) {
  uint2 u;
  u.x = pack2_bf16(f[0], f[1]);
  u.y = pack2_bf16(f[2], f[3]);
  *reinterpret_cast<uint2*>(p) = u;
}

// ------------------------------------------------------------------ LayerNorm fwd
template <int MAXC>
__global__ void __launch_bounds__(NT)
ln_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r, bf16* __restrict__ s_out,
              bf16* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
              const float* __restrict__ gamma, const float* __restrict__ beta, int T, int H, float eps,
              uint32_t thr_in, float inv_keep_in, uint32_t thr_out, float inv_keep_out,
              const uint32_t* __restrict__ seedp, uint32_t salt_in, uint32_t salt_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * (NT / 64) + wave;
  if (row >= T) return;
  const int nch = H >> 2;
  const uint32_t seed = seedp ? *seedp : 0u;
  const size_t base = (size_t)row * H;
  float v[MAXC][4];
  // gamma / beta are issued with the row loads: fetched after the two reductions they
  // were a second dependent memory round trip at the end of every (short-lived) wave
  float ga[MAXC][4], be[MAXC][4];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    load4f(gamma + 4 * (c < nch ? c : 0), ga[k]);
    load4f(beta + 4 * (c < nch ? c : 0), be[k]);
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    const size_t o = base + 4 * (c < nch ? c : 0);
    float xv[4], rr[4];
    load4(x + o, xv);
    if (r) load4(r + o, rr);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[k][e] = 0.f;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = xv[e];
      if (r) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float q = rr[e];
          if (thr_in) q = keep(seed, salt_in, (uint32_t)(base + 4 * c + e), thr_in) ? q * inv_keep_in : 0.f;
          v[k][e] += q;
        }
        if (s_out) store4(s_out + base + 4 * c, v[k]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) sum += v[k][e];
    }
  }
  const float mean = wave_sum(sum) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[k][e] - mean; sq += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / (float)H + eps);
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 4 * c + e;
        o[e] = (v[k][e] - mean) * rstd * ga[k][e] + be[k][e];
        if (thr_out)
          o[e] = keep(seed, salt_out, (uint32_t)(base + col), thr_out) ? o[e] * inv_keep_out : 0.f;
      }
      store4(y + base + 4 * c, o);
    }
  }
}

// ------------------------------------------------------------------ LayerNorm bwd
// dy -> (optional output-dropout backward) -> LN backward -> ds; dr = dropout_in'(ds).
// Rows are grid-strided over waves; dgamma/dbeta accumulate per lane in registers.
template <int MAXC>
__global__ void __launch_bounds__(NT)
ln_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ s, const float* __restrict__ mean_in,
              const float* __restrict__ rstd_in, const float* __restrict__ gamma, bf16* __restrict__ ds,
              bf16* __restrict__ dr, float* __restrict__ sums, int T, int H, uint32_t thr_in, float inv_keep_in,
              uint32_t thr_out, float inv_keep_out, const uint32_t* __restrict__ seedp, uint32_t salt_in,
              uint32_t salt_out, int ncopy) {
  __shared__ float red[NT / 64][2][64 * 4 * MAXC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = H >> 2;
  const uint32_t seed = seedp ? *seedp : 0u;
  float dg[MAXC][4], db[MAXC][4];
#pragma unroll
  for (int k = 0; k < MAXC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) { dg[k][e] = 0.f; db[k][e] = 0.f; }
  float gam[MAXC][4];   // this lane's gamma columns, loaded once
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    load4f(gamma + 4 * (c < nch ? c : 0), gam[k]);
  }
  const int waves_total = gridDim.x * (NT / 64);
  for (int row = blockIdx.x * (NT / 64) + wave; row < T; row += waves_total) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float g[MAXC][4], xh[MAXC][4];
    float a = 0.f, b = 0.f;
    float dv[MAXC][4], svv[MAXC][4];
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {   // every row load in flight before any math
      const int c = lane + 64 * k;
      const size_t o = base + 4 * (c < nch ? c : 0);
      load4(dy + o, dv[k]);
      load4(s + o, svv[k]);
    }
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int c = lane + 64 * k;
#pragma unroll
      for (int e = 0; e < 4; ++e) { g[k][e] = 0.f; xh[k][e] = 0.f; }
      if (c < nch) {
        float* d = dv[k];
        const float* sv = svv[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * c + e;
          if (thr_out) d[e] = keep(seed, salt_out, (uint32_t)(base + col), thr_out) ? d[e] * inv_keep_out : 0.f;
          xh[k][e] = (sv[e] - mean) * rstd;
          db[k][e] += d[e];
          dg[k][e] += d[e] * xh[k][e];
          g[k][e] = d[e] * gam[k][e];
          a += g[k][e];
          b += g[k][e] * xh[k][e];
        }
      }
    }
    a = wave_sum(a) / (float)H;
    b = wave_sum(b) / (float)H;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (g[k][e] - a - xh[k][e] * b);
        store4(ds + base + 4 * c, o);
        if (dr) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (thr_in) o[e] = keep(seed, salt_in, (uint32_t)(base + 4 * c + e), thr_in) ? o[e] * inv_keep_in : 0.f;
          store4(dr + base + 4 * c, o);
        }
      }
    }
  }
  // block reduction of dgamma / dbeta, then one atomic per column into copy slot
#pragma unroll
  for (int k = 0; k < MAXC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = 4 * (lane + 64 * k) + e;
      red[wave][0][col] = dg[k][e];
      red[wave][1][col] = db[k][e];
    }
  __syncthreads();
  float* dst = sums + (size_t)(blockIdx.x % ncopy) * 2 * H;
  for (int col = threadIdx.x; col < H; col += NT) {
    float x0 = 0.f, x1 = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) { x0 += red[w][0][col]; x1 += red[w][1][col]; }
    atomicAdd(dst + col, x0);
    atomicAdd(dst + H + col, x1);
  }
}

// dgamma/dbeta from the NSTAT copies, accumulated into the grad arena slots
__global__ void __launch_bounds__(NT)
ln_bwd_finalize_kernel(const float* __restrict__ sums, float* __restrict__ dgamma, float* __restrict__ dbeta, int H,
                       int ncopy) {
  // 8 lanes per column, each summing every 8th copy, then a fixed-order shuffle reduction
  // (deterministic): one lane per column looping over all copies ran 3 blocks of serial
  // loads, 11 us per call on BERT-base (24 calls per step)
  constexpr int FL = 8;
  const int c = blockIdx.x * (NT / FL) + (int)(threadIdx.x / FL), q = threadIdx.x % FL;
  float g = 0.f, b = 0.f;
  if (c < H) {
#pragma unroll 4
    for (int k = q; k < ncopy; k += FL) { g += sums[(size_t)k * 2 * H + c]; b += sums[(size_t)k * 2 * H + H + c]; }
  }
#pragma unroll
  for (int o = 1; o < FL; o <<= 1) { g += __shfl_xor(g, o, 64); b += __shfl_xor(b, o, 64); }
  if (c >= H || q != 0) return;
  dgamma[c] += g;
  dbeta[c] += b;
}

// all LayerNorms of a model in one launch: blockIdx.y picks the LayerNorm (its NSTAT sums
// scratch, grad slots and width), the rest is ln_bwd_finalize_kernel.  The native BERT runs
// it once at the end of backward instead of 25 finalize launches on the critical path.
struct LnFin {
  const float* sums;
  float* dgamma;
  float* dbeta;
  long H;
};
__global__ void __launch_bounds__(NT)
ln_finalize_many_kernel(const LnFin* __restrict__ d, int ncopy) {
  constexpr int FL = 8;
  const LnFin f = d[blockIdx.y];
  const int H = (int)f.H;
  const int c = blockIdx.x * (NT / FL) + (int)(threadIdx.x / FL), q = threadIdx.x % FL;
  float g = 0.f, b = 0.f;
  if (c < H) {
#pragma unroll 4
    for (int k = q; k < ncopy; k += FL) { g += f.sums[(size_t)k * 2 * H + c]; b += f.sums[(size_t)k * 2 * H + H + c]; }
  }
#pragma unroll
  for (int o = 1; o < FL; o <<= 1) { g += __shfl_xor(g, o, 64); b += __shfl_xor(b, o, 64); }
  if (c >= H || q != 0) return;
  f.dgamma[c] += g;
  f.dbeta[c] += b;
}

// ------------------------------------------------------------------ embedding backward
// dE = ds [B*S][H] bf16 scattered into the three embedding gradients, two launches:
// * embed_bwd_kernel, block (s, y) = position s, batch rows y*BB .. y*BB+BB-1, threads along
//   the columns (4 each) so every atomic wave-instruction covers 256 contiguous bytes of one
//   row (64 lanes in 64 rows run ~17x slower, MI355X_MICROARCH.md float atomics):
//   word[ids[t]] += ds[t] (fp32 atomics, as index_add) and pt[s][k] += the block's sum over
//   its tokens of type k (gridDim.y adders per address);
// * embed_bwd_finish_kernel: pos[s] += sum_k pt[s][k], tok[k] += sum_s pt[s][k], and pt is
//   zeroed again for the next step.  (Summing tok_type straight from every block put ~500
//   adders on each address of one 3 KB row: the whole pass took 98 us.)
constexpr int EMB_MAXT = 4;
__global__ void __launch_bounds__(NT)
embed_bwd_kernel(const bf16* __restrict__ ds, const long* __restrict__ ids, const long* __restrict__ tt,
                 float* __restrict__ word, float* __restrict__ pt, int B, int S, int H, int ntypes, int BB) {
  const int s = blockIdx.x;
  const int b0 = blockIdx.y * BB, b1 = min(B, b0 + BB);
  // lane-consecutive columns: each atomic wave-instruction is 64 consecutive floats
  for (int c = threadIdx.x; c < H; c += NT) {
    float ta[EMB_MAXT] = {0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b < b1; ++b) {
      const long t = (long)b * S + s;
      const float d = (float)ds[t * H + c];
      atomicAdd(word + ids[t] * H + c, d);
      const int ty = tt ? (int)tt[t] : 0;
#pragma unroll
      for (int k = 0; k < EMB_MAXT; ++k) ta[k] += ty == k ? d : 0.f;
    }
    for (int k = 0; k < ntypes; ++k) atomicAdd(pt + ((long)s * ntypes + k) * H + c, ta[k]);
  }
}

constexpr int EMB_SB = 8;   // positions per finish thread
__global__ void __launch_bounds__(NT)
embed_bwd_finish_kernel(float* __restrict__ pt, float* __restrict__ pos, float* __restrict__ tok, int S, int H,
                        int ntypes) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= H) return;
  const int s0 = blockIdx.y * EMB_SB, s1 = min(S, s0 + EMB_SB);
  float tk[EMB_MAXT] = {0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; ++s) {
    float ps = 0.f;
    for (int k = 0; k < ntypes; ++k) {
      float* q = pt + ((long)s * ntypes + k) * H + c;
      const float v = *q;
      *q = 0.f;
      ps += v;
      tk[k] += v;
    }
    pos[(long)s * H + c] += ps;
  }
  if (tok)
    for (int k = 0; k < ntypes; ++k) atomicAdd(tok + (long)k * H + c, tk[k]);
}

// ------------------------------------------------------------------ softmax
// rows of length L (keys); row r belongs to batch (r / rows_per_batch) for the key bias
template <int MAXC>
__global__ void __launch_bounds__(NT)
softmax_fwd_kernel(const bf16* __restrict__ S, const float* __restrict__ key_bias, bf16* __restrict__ P,
                   bf16* __restrict__ Pd, long R, int L, int rows_per_batch, float scale, uint32_t thr,
                   float inv_keep, const uint32_t* __restrict__ seedp, uint32_t salt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * (NT / 64) + wave;
  if (row >= R) return;
  const int nch = L >> 2;
  const size_t base = (size_t)row * L;
  const float* kb = key_bias ? key_bias + (size_t)(row / rows_per_batch) * L : nullptr;
  float v[MAXC][4];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[k][e] = -INFINITY;
    if (c < nch) {
      load4(S + base + 4 * c, v[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[k][e] = v[k][e] * scale + (kb ? kb[4 * c + e] : 0.f);
        mx = fmaxf(mx, v[k][e]);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[k][e] = (v[k][e] == -INFINITY) ? 0.f : __expf(v[k][e] - mx);
      sum += v[k][e];
    }
  const float tot = wave_sum(sum);
  const float inv = tot > 0.f ? 1.f / tot : 0.f;   // fully masked row -> zeros
  const uint32_t seed = seedp ? *seedp : 0u;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      float p[4], q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        p[e] = v[k][e] * inv;
        q[e] = (thr && !keep(seed, salt, (uint32_t)(base + 4 * c + e), thr)) ? 0.f : p[e] * inv_keep;
      }
      store4(P + base + 4 * c, p);
      if (Pd) store4(Pd + base + 4 * c, q);
    }
  }
}

template <int MAXC>
__global__ void __launch_bounds__(NT)
softmax_bwd_kernel(const bf16* __restrict__ P, const bf16* __restrict__ dPd, bf16* __restrict__ dS, long R, int L,
                   float scale, uint32_t thr, float inv_keep, const uint32_t* __restrict__ seedp, uint32_t salt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * (NT / 64) + wave;
  if (row >= R) return;
  const int nch = L >> 2;
  const size_t base = (size_t)row * L;
  const uint32_t seed = seedp ? *seedp : 0u;
  float p[MAXC][4], d[MAXC][4];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) { p[k][e] = 0.f; d[k][e] = 0.f; }
    if (c < nch) {
      load4(P + base + 4 * c, p[k]);
      load4(dPd + base + 4 * c, d[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (thr) d[k][e] = keep(seed, salt, (uint32_t)(base + 4 * c + e), thr) ? d[k][e] * inv_keep : 0.f;
        dot += p[k][e] * d[k][e];
      }
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = scale * p[k][e] * (d[k][e] - dot);
      store4(dS + base + 4 * c, o);
    }
  }
}

// ------------------------------------------------------------------ bias grads
// partial column sums: block (x, y) sums rows [y*RB, (y+1)*RB) of 8*NT columns and adds
// them into copy (y % NSTAT) of scratch[NSTAT][C] (8 adds per address at most per
// NSTAT blocks); colsum_finalize folds the copies into out (+=)
__global__ void __launch_bounds__(NT)
colsum_partial_kernel(const bf16* __restrict__ g, float* __restrict__ scratch, int R, int C, int RB, int ncopy) {
  const int c8 = blockIdx.x * NT + threadIdx.x;
  if (c8 * 8 >= C) return;
  const int r0 = blockIdx.y * RB, r1 = min(R, r0 + RB);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = r0; r < r1; ++r) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(g + (size_t)r * C + c8 * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += f[e];
  }
  float* dst = scratch + (size_t)(blockIdx.y % ncopy) * C + c8 * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) atomicAdd(dst + e, acc[e]);
}

__global__ void __launch_bounds__(NT)
colsum_finalize_kernel(float* __restrict__ scratch, float* __restrict__ out, int C, int ncopy) {
  constexpr int FL = 8;   // 8 lanes per column + fixed-order shuffle (as ln_bwd_finalize_kernel)
  const int c = blockIdx.x * (NT / FL) + (int)(threadIdx.x / FL), q = threadIdx.x % FL;
  float s = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int k = q; k < ncopy; k += FL) { s += scratch[(size_t)k * C + c]; scratch[(size_t)k * C + c] = 0.f; }
  }
#pragma unroll
  for (int o = 1; o < FL; o <<= 1) s += __shfl_xor(s, o, 64);
  if (c < C && q == 0) out[c] += s;
}

// ------------------------------------------------------------------ dropout (standalone)
__global__ void __launch_bounds__(NT)
dropout_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long n4, uint32_t thr, float inv_keep,
               const uint32_t* __restrict__ seedp, uint32_t salt) {
  const uint32_t seed = *seedp;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    float f[4];
    load4(x + 4 * i, f);
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = keep(seed, salt, (uint32_t)(4 * i + e), thr) ? f[e] * inv_keep : 0.f;
    store4(y + 4 * i, f);
  }
}

template <class K>
int pick_maxc(int cols, K&& launch) {
  const int per_lane = (cols / 4 + 63) / 64;
  if (per_lane <= 1) return launch(std::integral_constant<int, 1>{});
  if (per_lane <= 2) return launch(std::integral_constant<int, 2>{});
  if (per_lane <= 4) return launch(std::integral_constant<int, 4>{});
  if (per_lane <= 8) return launch(std::integral_constant<int, 8>{});
  return -1;
}

// ------------------------------------------------------------------ fused attention
// One workgroup per (batch, head), S/32 waves; wave w owns query rows 32w..32w+31.  Q, K, V
// are read in place from the QKV projection output [B*S][3*E] (head h = columns h*64..),
// the context is written straight into [B*S][E] and the backward writes dQ/dK/dV straight
// into dQKV [B*S][3*E]: no head split / merge copies, no S x S tensor in HBM (the backward
// recomputes P from the saved per-row log-sum-exp).
//
// Scores are computed transposed, S^T = K Q^T (v_mfma_f32_32x32x16_bf16: A = K rows,
// B = Q rows, both K-contiguous fragments loaded from global), so each lane holds ONE
// query's scores for half of the keys: the softmax row reductions are in-register plus a
// single lane^32 exchange.  The probabilities then feed the next MFMA as its B operand
// directly from the accumulator registers: in the 32x32 C layout lane half hh holds keys
// 16s + {0..3, 8..11} + 4hh of a 16-key step, i.e. the natural key order with bits 2 and 3
// swapped, so the A operand (V^T / K^T, read with ds_read_b64_tr_b16 from LDS) is staged
// with its key rows permuted the same way (swap23).  Dropout masks reuse the counter hash
// of the softmax kernel at the same element index ((b*H + h)*S + q)*S + key.
namespace attn {
constexpr int D = 64;  // head dim

// [rows][64] / [rows][128] bf16 LDS images, 16-B chunks XOR-swizzled for tr16 column reads
template <int W>
__device__ __forceinline__ int img_off(int r, int c) {
  if (W == 64) return r * 128 + ((c ^ (((r >> 1) & 1) << 2)) << 4);
  return r * 256 + ((c ^ ((r & 3) << 2)) << 4);
}
__device__ __forceinline__ int swap23(int k) { return (k & ~12) | ((k >> 1) & 4) | ((k << 1) & 8); }

// MFMA operand fragment (row/col base+(lane&31), k = k0 + 8*(lane>>5) + 0..7) read
// transposed from a [k][W] image
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int base, int k0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int kr = k0 + 8 * (g >> 1);
  const int a0 = img_off<W>(kr + q, col >> 3) + (col & 7) * 2;
  const int a1 = img_off<W>(kr + 4 + q, col >> 3) + (col & 7) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(lds + a1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
// K-contiguous fragment of row `row` straight from global (ld elements per row)
__device__ __forceinline__ bf16x8 g_frag(const bf16* base, int ld, int row, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + (size_t)row * ld + 16 * s + 8 * (lane >> 5));
}
// accumulator registers 8s..8s+7 as a bf16 B fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int t = 0; t < 8; ++t) r[t] = (bf16)a[8 * s + t];
  return r;
}
// copy a [rows][64] head slice (row stride ld) into an LDS image; rows permuted by swap23
template <int ROWS, bool PERM>
__device__ __forceinline__ void stage64(char* img, const bf16* src, int ld, int tid, int nthr) {
  for (int c = tid; c < ROWS * 8; c += nthr) {
    const int r = c >> 3, ch = c & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)r * ld + ch * 8);
    *reinterpret_cast<uint4*>(img + img_off<64>(PERM ? swap23(r) : r, ch)) = v;
  }
}
// store a transposed C tile pair: acc[j][r] = X[row][d = 32j + (r&3) + 8(r>>2) + 4hh] for
// this lane's row, as 8-byte pieces
__device__ __forceinline__ void store_rows(bf16* dst, const f32x16 (&acc)[2], int lane) {
  const int hh = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float f[4] = {acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]};
      store4(dst + 32 * j + 8 * g + 4 * hh, f);
    }
}
__device__ __forceinline__ int key_of(int i, int r, int hh) { return 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh; }

template <int S>
__global__ void __launch_bounds__(2 * S)
fwd_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, bf16* __restrict__ out,
           float* __restrict__ lse, int H, float scale, uint32_t thr, float inv_keep,
           const uint32_t* __restrict__ seedp, uint32_t salt) {
  constexpr int NKT = S / 32, NTH = 2 * S;
  __shared__ __attribute__((aligned(16))) char smem[S * 128];   // V image, key rows swap23
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int bh = blockIdx.x, b = bh / H, hd = bh - b * H;
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)b * S * ld + hd * D;
  const bf16* Kg = Qg + E;
  stage64<S, true>(smem, Qg + 2 * E, ld, tid, NTH);
  const int q = 32 * w + l32;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = g_frag(Qg, ld, q, s, lane);
  f32x16 acc[NKT];
#pragma unroll
  for (int i = 0; i < NKT; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g_frag(Kg, ld, 32 * i + l32, s, lane), qf[s], acc[i], 0, 0, 0);
  }
  // softmax over this lane's query (keys split between lane and lane^32)
  const float* kb = key_bias ? key_bias + (size_t)b * S : nullptr;
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float x = acc[i][r] * scale + (kb ? kb[key_of(i, r, hh)] : 0.f);
      acc[i][r] = x;
      mx = fmaxf(mx, x);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = acc[i][r] == -INFINITY ? 0.f : __expf(acc[i][r] - mx);
      acc[i][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  if (hh == 0) lse[(size_t)bh * S + q] = sum > 0.f ? mx + __logf(sum) : INFINITY;
  const uint32_t seed = seedp ? *seedp : 0u;
  const uint32_t rowidx = ((uint32_t)bh * S + q) * S;
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = acc[i][r] * inv;
      acc[i][r] = (thr && !keep(seed, salt, rowidx + key_of(i, r, hh), thr)) ? 0.f : p * inv_keep;
    }
  __syncthreads();
  // O^T = V^T Pd^T
  f32x16 o[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pb = acc_frag(acc[i], s);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        o[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<64>(smem, 32 * j, 32 * i + 16 * s, lane), pb, o[j], 0,
                                                       0, 0);
    }
  store_rows(out + ((size_t)b * S + q) * E + hd * D, o, lane);
}

template <int S>
__global__ void __launch_bounds__(2 * S)
bwd_kernel(const bf16* __restrict__ qkv, const float* __restrict__ key_bias, const bf16* __restrict__ dout,
           const float* __restrict__ lse, bf16* __restrict__ dqkv, int H, float scale, uint32_t thr, float inv_keep,
           const uint32_t* __restrict__ seedp, uint32_t salt) {
  constexpr int NKT = S / 32, NTH = 2 * S, IMG = S * 128;
  // K (key rows swap23), Q, dO images [*][64]; Pd, dS images [q][key]
  __shared__ __attribute__((aligned(16))) char smem[3 * IMG + 2 * S * S * 2];
  char* Ki = smem;
  char* Qi = smem + IMG;
  char* Oi = smem + 2 * IMG;
  char* Pi = smem + 3 * IMG;
  char* Si = Pi + S * S * 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int bh = blockIdx.x, b = bh / H, hd = bh - b * H;
  const int E = H * D, ld = 3 * E;
  const bf16* Qg = qkv + (size_t)b * S * ld + hd * D;
  const bf16* Kg = Qg + E;
  const bf16* Vg = Qg + 2 * E;
  const bf16* dOg = dout + (size_t)b * S * E + hd * D;
  bf16* dQg = dqkv + (size_t)b * S * ld + hd * D;
  stage64<S, true>(Ki, Kg, ld, tid, NTH);
  stage64<S, false>(Qi, Qg, ld, tid, NTH);
  stage64<S, false>(Oi, dOg, E, tid, NTH);
  const int q = 32 * w + l32;
  // recompute S^T and dPd^T = V dO^T
  f32x16 sp[NKT], dp[NKT];
  {
    bf16x8 qf[4], of[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = g_frag(Qg, ld, q, s, lane);
      of[s] = g_frag(dOg, E, q, s, lane);
    }
#pragma unroll
    for (int i = 0; i < NKT; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { sp[i][r] = 0.f; dp[i][r] = 0.f; }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sp[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g_frag(Kg, ld, 32 * i + l32, s, lane), qf[s], sp[i], 0, 0, 0);
        dp[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g_frag(Vg, ld, 32 * i + l32, s, lane), of[s], dp[i], 0, 0, 0);
      }
    }
  }
  const float* kb = key_bias ? key_bias + (size_t)b * S : nullptr;
  const float l = lse[(size_t)bh * S + q];
  const uint32_t seed = seedp ? *seedp : 0u;
  const uint32_t rowidx = ((uint32_t)bh * S + q) * S;
  float dot = 0.f;
  uint64_t kept = 0;   // dropout keep bit of register (i, r) at bit 16i + r
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = key_of(i, r, hh);
      const float x = sp[i][r] * scale + (kb ? kb[key] : 0.f);
      const float p = x == -INFINITY ? 0.f : __expf(x - l);
      const bool kp = !thr || keep(seed, salt, rowidx + key, thr);
      kept |= (uint64_t)kp << (16 * i + r);
      const float d = kp ? dp[i][r] * inv_keep : 0.f;    // dP
      sp[i][r] = p;
      dp[i][r] = d;
      dot += p * d;
    }
  dot += __shfl_xor(dot, 32, 64);
  // Pd and dS into registers (sp, dp) and into the [q][key] images for dK / dV
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool kp = (kept >> (16 * i + r)) & 1;
      const float p = sp[i][r];
      dp[i][r] = scale * p * (dp[i][r] - dot);
      sp[i][r] = kp ? p * inv_keep : 0.f;
    }
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int key0 = 32 * i + 8 * g + 4 * hh;
      const int off = img_off<S>(q, key0 >> 3) + (key0 & 7) * 2;
      float f[4] = {sp[i][4 * g], sp[i][4 * g + 1], sp[i][4 * g + 2], sp[i][4 * g + 3]};
      float e[4] = {dp[i][4 * g], dp[i][4 * g + 1], dp[i][4 * g + 2], dp[i][4 * g + 3]};
      store4(reinterpret_cast<bf16*>(Pi + off), f);
      store4(reinterpret_cast<bf16*>(Si + off), e);
    }
  __syncthreads();
  // dQ^T = K^T dS^T  (dS^T straight from registers)
  {
    f32x16 dq[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < NKT; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sb = acc_frag(dp[i], s);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          dq[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<64>(Ki, 32 * j, 32 * i + 16 * s, lane), sb, dq[j], 0,
                                                          0, 0);
      }
    store_rows(dQg + (size_t)q * ld, dq, lane);
  }
  // dV^T = dO^T Pd and dK^T = Q^T dS for this wave's 32 keys, summed over all queries
  f32x16 dv[2], dk[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dv[j][r] = 0.f; dk[j][r] = 0.f; }
#pragma unroll
  for (int s = 0; s < S / 16; ++s) {
    const bf16x8 pb = tr_frag<S>(Pi, 32 * w, 16 * s, lane);
    const bf16x8 sb = tr_frag<S>(Si, 32 * w, 16 * s, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      dv[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<64>(Oi, 32 * j, 16 * s, lane), pb, dv[j], 0, 0, 0);
      dk[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<64>(Qi, 32 * j, 16 * s, lane), sb, dk[j], 0, 0, 0);
    }
  }
  const int key = 32 * w + l32;
  store_rows(dQg + (size_t)key * ld + E, dk, lane);
  store_rows(dQg + (size_t)key * ld + 2 * E, dv, lane);
}
}  // namespace attn

}  // namespace

// Fused multi-head attention (head dim 64, S in {64, 128}).  qkv [B*S][3*H*64] bf16;
// key_bias [B][S] fp32 (0 / -inf) or null; out [B*S][H*64]; lse [B*H*S] fp32 (saved for
// the backward).  Attention-probability dropout p with the softmax kernel's mask indexing.
MLC_EXPORT int mlc_attn_fwd(const bf16* qkv, const float* key_bias, bf16* out, float* lse, int B, int S, int H,
                            float scale, float p, const uint32_t* seed, uint32_t salt, hipStream_t st) {
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (S == 128)
    hipLaunchKernelGGL(attn::fwd_kernel<128>, dim3(B * H), dim3(256), 0, st, qkv, key_bias, out, lse, H, scale, t, k,
                       seed, salt);
  else if (S == 64)
    hipLaunchKernelGGL(attn::fwd_kernel<64>, dim3(B * H), dim3(128), 0, st, qkv, key_bias, out, lse, H, scale, t, k,
                       seed, salt);
  else
    return -1;
  return hipGetLastError();
}

// dqkv [B*S][3*H*64] is fully overwritten (dQ | dK | dV)
MLC_EXPORT int mlc_attn_bwd(const bf16* qkv, const float* key_bias, const bf16* dout, const float* lse, bf16* dqkv,
                            int B, int S, int H, float scale, float p, const uint32_t* seed, uint32_t salt,
                            hipStream_t st) {
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (S == 128)
    hipLaunchKernelGGL(attn::bwd_kernel<128>, dim3(B * H), dim3(256), 0, st, qkv, key_bias, dout, lse, dqkv, H, scale,
                       t, k, seed, salt);
  else if (S == 64)
    hipLaunchKernelGGL(attn::bwd_kernel<64>, dim3(B * H), dim3(128), 0, st, qkv, key_bias, dout, lse, dqkv, H, scale,
                       t, k, seed, salt);
  else
    return -1;
  return hipGetLastError();
}

// y = dropout_out(LN(x + dropout_in(r)) * gamma + beta); s_out = x + dropout_in(r) when r
// is given (needed by the backward); mean/rstd [T].  H % 4 == 0, H <= 2048.
MLC_EXPORT int mlc_ln_fwd(const bf16* x, const bf16* r, bf16* s_out, bf16* y, float* mean, float* rstd,
                          const float* gamma, const float* beta, int T, int H, float eps, float p_in,
                          float p_out, const uint32_t* seed, uint32_t salt_in, uint32_t salt_out,
                          hipStream_t st) {
  if (H % 4) return -1;
  const uint32_t ti = p_in > 0.f ? drop_threshold(p_in) : 0u, to = p_out > 0.f ? drop_threshold(p_out) : 0u;
  const float ki = p_in > 0.f ? 1.f / (1.f - p_in) : 1.f, ko = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
  const int blocks = (T + NT / 64 - 1) / (NT / 64);
  return pick_maxc(H, [&](auto mc) {
    hipLaunchKernelGGL((ln_fwd_kernel<decltype(mc)::value>), dim3(blocks), dim3(NT), 0, st, x, r, s_out, y, mean,
                       rstd, gamma, beta, T, H, eps, ti, ki, to, ko, seed, salt_in, salt_out);
    return (int)hipGetLastError();
  });
}

// sums: NSTAT*2*H fp32 scratch (zeroed by the caller); dgamma/dbeta accumulate (+=)
MLC_EXPORT int mlc_ln_bwd(const bf16* dy, const bf16* s, const float* mean, const float* rstd, const float* gamma,
                          bf16* ds, bf16* dr, float* sums, float* dgamma, float* dbeta, int T, int H, float p_in,
                          float p_out, const uint32_t* seed, uint32_t salt_in, uint32_t salt_out, hipStream_t st) {
  if (H % 4) return -1;
  const uint32_t ti = p_in > 0.f ? drop_threshold(p_in) : 0u, to = p_out > 0.f ? drop_threshold(p_out) : 0u;
  const float ki = p_in > 0.f ? 1.f / (1.f - p_in) : 1.f, ko = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
  // each block ends with 2*H dgamma/dbeta atomics: 512 blocks (2 per CU, 2 rows per wave
  // at T = 4096) halves that traffic; measured on BERT-base 32x128: 7.93 ms/step at 1024
  // blocks, 7.83 at 512, 7.86 at 256
  int blocks = (T + NT / 64 - 1) / (NT / 64);
  if (blocks > 512) blocks = 512;
  if (g_mlc_det && blocks > g_mlc_ncopy) return -2;
  int rc = pick_maxc(H, [&](auto mc) {
    hipLaunchKernelGGL((ln_bwd_kernel<decltype(mc)::value>), dim3(blocks), dim3(NT), 0, st, dy, s, mean, rstd, gamma,
                       ds, dr, sums, T, H, ti, ki, to, ko, seed, salt_in, salt_out, g_mlc_ncopy);
    return (int)hipGetLastError();
  });
  if (rc || !dgamma) return rc;   // no dgamma: the caller finalizes later (mlc_ln_finalize_many)
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((H + NT / 8 - 1) / (NT / 8)), dim3(NT), 0, st, sums, dgamma, dbeta, H,
                     g_mlc_ncopy);
  return hipGetLastError();
}

// word/pos/tok += the embedding gradient ds (see embed_bwd_kernel); ids/tt int64 [B*S]
// (token types < ntypes <= 4; tt and tok null: one type, no token-type table); pt: fp32
// scratch [S][ntypes][H], zero on entry and left zeroed.  H % 4 == 0.
MLC_EXPORT int mlc_embed_bwd(const bf16* ds, const long* ids, const long* tt, float* word, float* pos, float* tok,
                             float* pt, int B, int S, int H, int ntypes, hipStream_t st) {
  if (H % 4 || S < 1 || ntypes < 1 || ntypes > EMB_MAXT || (tok != nullptr) != (tt != nullptr)) return -1;
  int ny = (512 + S - 1) / S;                  // ~512 blocks: split the batch rows
  if (ny > B) ny = B;
  if (ny < 1) ny = 1;
  const int BB = (B + ny - 1) / ny;
  const dim3 grid(S, (B + BB - 1) / BB);
  hipLaunchKernelGGL(embed_bwd_kernel, grid, dim3(NT), 0, st, ds, ids, tt, word, pt, B, S, H, ntypes, BB);
  hipLaunchKernelGGL(embed_bwd_finish_kernel, dim3((H + NT - 1) / NT, (S + EMB_SB - 1) / EMB_SB), dim3(NT), 0, st, pt,
                     pos, tok, S, H, ntypes);
  return hipGetLastError();
}

// desc: n LnFin entries in device memory (sums scratch of NSTAT copies, dgamma, dbeta, H);
// every dgamma/dbeta += the sum of its copies.  maxH bounds the widths.
MLC_EXPORT int mlc_ln_finalize_many(const void* desc, int n, int maxH, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ln_finalize_many_kernel, dim3((maxH + NT / 8 - 1) / (NT / 8), n), dim3(NT), 0, st,
                     reinterpret_cast<const LnFin*>(desc), g_mlc_ncopy);
  return hipGetLastError();
}

MLC_EXPORT int mlc_softmax_fwd(const bf16* S, const float* key_bias, bf16* P, bf16* Pd, long R, int L,
                               int rows_per_batch, float scale, float p, const uint32_t* seed, uint32_t salt,
                               hipStream_t st) {
  if (L % 4) return -1;
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const long blocks = (R + NT / 64 - 1) / (NT / 64);
  return pick_maxc(L, [&](auto mc) {
    hipLaunchKernelGGL((softmax_fwd_kernel<decltype(mc)::value>), dim3(blocks), dim3(NT), 0, st, S, key_bias, P,
                       Pd, R, L, rows_per_batch, scale, t, k, seed, salt);
    return (int)hipGetLastError();
  });
}

MLC_EXPORT int mlc_softmax_bwd(const bf16* P, const bf16* dPd, bf16* dS, long R, int L, float scale, float p,
                               const uint32_t* seed, uint32_t salt, hipStream_t st) {
  if (L % 4) return -1;
  const uint32_t t = p > 0.f ? drop_threshold(p) : 0u;
  const float k = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const long blocks = (R + NT / 64 - 1) / (NT / 64);
  return pick_maxc(L, [&](auto mc) {
    hipLaunchKernelGGL((softmax_bwd_kernel<decltype(mc)::value>), dim3(blocks), dim3(NT), 0, st, P, dPd, dS, R, L,
                       scale, t, k, seed, salt);
    return (int)hipGetLastError();
  });
}

// out[C] += column sums of g[R][C] (C % 8 == 0).  scratch: NSTAT*C fp32, zero on entry
// (left zeroed on exit, so one buffer can serve every call of a step).
MLC_EXPORT int mlc_colsum_acc(const bf16* g, float* out, float* scratch, int R, int C, hipStream_t st) {
  if (C % 8) return -1;
  const int xb = (C / 8 + NT - 1) / NT;
  int RB = (R * xb + 511) / 512;       // ~512 blocks
  if (RB < 16) RB = 16;
  dim3 grid(xb, (R + RB - 1) / RB);
  if (g_mlc_det && (int)grid.y > g_mlc_ncopy) return -2;
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(NT), 0, st, g, scratch, R, C, RB, g_mlc_ncopy);
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3((C + NT / 8 - 1) / (NT / 8)), dim3(NT), 0, st, scratch, out, C,
                     g_mlc_ncopy);
  return hipGetLastError();
}

MLC_EXPORT int mlc_dropout(const bf16* x, bf16* y, long n, float p, const uint32_t* seed, uint32_t salt,
                           hipStream_t st) {
  if (n % 4) return -1;
  long blocks = (n / 4 + NT - 1) / NT;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks), dim3(NT), 0, st, x, y, n / 4, drop_threshold(p),
                     1.f / (1.f - p), seed, salt);
  return hipGetLastError();
}
