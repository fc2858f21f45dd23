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
#include <type_traits>

namespace {

constexpr int NT = 256;
constexpr int NSTAT = 32;

__device__ __forceinline__ uint32_t hash_u32(uint32_t seed, uint32_t salt, uint32_t i) {
  uint32_t x = i * 0x9E3779B9u ^ (seed * 0x85EBCA6Bu + salt * 0xC2B2AE35u);
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// keep with probability 1-p: compare the top 24 bits against the threshold
__device__ __forceinline__ bool keep(uint32_t seed, uint32_t salt, uint32_t i, uint32_t thr) {
  return (hash_u32(seed, salt, i) >> 8) >= thr;
}
__host__ __device__ __forceinline__ uint32_t drop_threshold(float p) {
  return (uint32_t)(p * 16777216.0f);
}

__device__ __forceinline__ void load4(const bf16* p, float* f) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void store4(bf16* p, const float* f) {
  uint2 u;
  u.x = f2bf_bits(f[0]) | (f2bf_bits(f[1]) << 16);
  u.y = f2bf_bits(f[2]) | (f2bf_bits(f[3]) << 16);
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
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[k][e] = 0.f;
    if (c < nch) {
      load4(x + base + 4 * c, v[k]);
      if (r) {
        float rr[4];
        load4(r + base + 4 * c, rr);
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
        o[e] = (v[k][e] - mean) * rstd * gamma[col] + beta[col];
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
              uint32_t salt_out) {
  __shared__ float red[NT / 64][2][64 * 4 * MAXC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = H >> 2;
  const uint32_t seed = seedp ? *seedp : 0u;
  float dg[MAXC][4], db[MAXC][4];
#pragma unroll
  for (int k = 0; k < MAXC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) { dg[k][e] = 0.f; db[k][e] = 0.f; }
  const int waves_total = gridDim.x * (NT / 64);
  for (int row = blockIdx.x * (NT / 64) + wave; row < T; row += waves_total) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float g[MAXC][4], xh[MAXC][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int c = lane + 64 * k;
#pragma unroll
      for (int e = 0; e < 4; ++e) { g[k][e] = 0.f; xh[k][e] = 0.f; }
      if (c < nch) {
        float d[4], sv[4];
        load4(dy + base + 4 * c, d);
        load4(s + base + 4 * c, sv);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * c + e;
          if (thr_out) d[e] = keep(seed, salt_out, (uint32_t)(base + col), thr_out) ? d[e] * inv_keep_out : 0.f;
          xh[k][e] = (sv[e] - mean) * rstd;
          db[k][e] += d[e];
          dg[k][e] += d[e] * xh[k][e];
          g[k][e] = d[e] * gamma[col];
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
  float* dst = sums + (size_t)(blockIdx.x % NSTAT) * 2 * H;
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
ln_bwd_finalize_kernel(const float* __restrict__ sums, float* __restrict__ dgamma, float* __restrict__ dbeta, int H) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= H) return;
  float g = 0.f, b = 0.f;
  for (int k = 0; k < NSTAT; ++k) { g += sums[(size_t)k * 2 * H + c]; b += sums[(size_t)k * 2 * H + H + c]; }
  dgamma[c] += g;
  dbeta[c] += b;
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
colsum_partial_kernel(const bf16* __restrict__ g, float* __restrict__ scratch, int R, int C, int RB) {
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
  float* dst = scratch + (size_t)(blockIdx.y % NSTAT) * C + c8 * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) atomicAdd(dst + e, acc[e]);
}

__global__ void __launch_bounds__(NT)
colsum_finalize_kernel(float* __restrict__ scratch, float* __restrict__ out, int C) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < NSTAT; ++k) { s += scratch[(size_t)k * C + c]; scratch[(size_t)k * C + c] = 0.f; }
  out[c] += s;
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

}  // namespace

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
  int blocks = (T + NT / 64 - 1) / (NT / 64);
  if (blocks > 1024) blocks = 1024;
  int rc = pick_maxc(H, [&](auto mc) {
    hipLaunchKernelGGL((ln_bwd_kernel<decltype(mc)::value>), dim3(blocks), dim3(NT), 0, st, dy, s, mean, rstd, gamma,
                       ds, dr, sums, T, H, ti, ki, to, ko, seed, salt_in, salt_out);
    return (int)hipGetLastError();
  });
  if (rc) return rc;
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((H + NT - 1) / NT), dim3(NT), 0, st, sums, dgamma, dbeta, H);
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
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(NT), 0, st, g, scratch, R, C, RB);
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, st, scratch, out, C);
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
