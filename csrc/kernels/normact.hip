// BatchNorm with any activation, for the generic native engine (batchnorm.hip keeps the
// ReLU-only passes the ResNet engine is tuned on).  NHWC bf16, 16 B per lane, threads own
// a fixed 8-channel group (grid = multiple of C/8 threads).
//
//   stats      per-channel sum / sum-of-squares of x into 32 partial copies (a BatchNorm
//              whose input no conv epilogue reduced: after a pool, a concat, a torch op)
//   apply      z = act(y*scale + shift [+ res*rscale + rshift])
//   bwd        dU = dz * act'(a) (a = the pre-activation, recomputed from y [and res], or the
//              derivative read off z), S1 = sum dU, S2 = sum dU*(y - mean) per channel, then
//              dy = k1*dU + k2 + k3*(y - mean) and dres = dU (mlc_bn_bwd_finalize gives k*)
//
// Activation codes (ACT_*): 0 identity, 1 ReLU, 2 ReLU6, 3 SiLU, 4 sigmoid, 5 tanh,
// 6 hardswish, 7 leaky ReLU (slope `alpha`), 8 GELU (erf), 9 ELU (alpha), 10 hardsigmoid.
#include "common.h"

namespace normact {

constexpr int NT = 256;
constexpr int NCOPY = 32;

__device__ __forceinline__ float sigm(float a) { return 1.f / (1.f + __expf(-a)); }

__device__ __forceinline__ float act_f(float a, int act, float alpha) {
  switch (act) {
    case 1: return fmaxf(a, 0.f);
    case 2: return fminf(fmaxf(a, 0.f), 6.f);
    case 3: return a * sigm(a);
    case 4: return sigm(a);
    case 5: return tanhf(a);
    case 6: return a * fminf(fmaxf(a + 3.f, 0.f), 6.f) * (1.f / 6.f);
    case 7: return a > 0.f ? a : alpha * a;
    case 8: return 0.5f * a * (1.f + erff(a * 0.70710678118654752f));
    case 9: return a > 0.f ? a : alpha * (__expf(a) - 1.f);
    case 10: return fminf(fmaxf(a + 3.f, 0.f), 6.f) * (1.f / 6.f);
    default: return a;
  }
}

// d act / d a at pre-activation a (z = act(a) as stored, used where it is the cheaper input;
// the masks of the piecewise-linear codes are taken from a, which matches torch: ReLU'(0) = 0,
// ReLU6'(6) = 0, hardswish at +-3 as torch's hardswish_backward)
__device__ __forceinline__ float act_df(float a, float z, int act, float alpha) {
  switch (act) {
    case 1: return a > 0.f ? 1.f : 0.f;
    case 2: return (a > 0.f && a < 6.f) ? 1.f : 0.f;
    case 3: { const float s = sigm(a); return s * (1.f + a * (1.f - s)); }
    case 4: return z * (1.f - z);
    case 5: return 1.f - z * z;
    case 6: return a < -3.f ? 0.f : (a <= 3.f ? (2.f * a + 3.f) * (1.f / 6.f) : 1.f);
    case 7: return a > 0.f ? 1.f : alpha;
    case 8: {
      const float cdf = 0.5f * (1.f + erff(a * 0.70710678118654752f));
      return cdf + a * 0.3989422804014327f * __expf(-0.5f * a * a);
    }
    case 9: return a > 0.f ? 1.f : alpha * __expf(a);
    case 10: return (a > -3.f && a < 3.f) ? (1.f / 6.f) : 0.f;
    default: return 1.f;
  }
}

// per-thread constants of its channel group
struct Ch {
  float sc[8], sh[8], rs[8], rh[8];
};
// per-sample factor of the BN output (stochastic depth: the drop-path mask / keep of a block,
// folded into its last BN's passes), s[n] for rows n*hw .. (n+1)*hw - 1; identity only (act 0)
struct RowScale {
  const float* s;
  long hw;
};

__device__ __forceinline__ void load_ch(Ch& c, const float* scale, const float* shift, const float* rscale,
                                        const float* rshift, int c0) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    c.sc[j] = scale[c0 + j];
    c.sh[j] = shift[c0 + j];
    c.rs[j] = rscale ? rscale[c0 + j] : 1.f;
    c.rh[j] = rscale ? rshift[c0 + j] : 0.f;
  }
}

// element offset of 8-channel chunk i (row i / G, group i % G) in rows of stride ld elements
// (ld == 8G: dense rows; otherwise a channel slice of wider rows - a DenseNet concat buffer's
// channels - and rows * G < 2^32, checked on the host)
__device__ __forceinline__ long chunk_off(long i, int G, long ld) {
  if (ld == 8L * G) return i * 8;
  const unsigned q = (unsigned)i / (unsigned)G;
  return (long)q * ld + (long)((unsigned)i - q * (unsigned)G) * 8;
}

// x rows of stride x_ld (chunk_off); copies of row stride ld
__global__ void __launch_bounds__(NT)
stats_kernel(const bf16* __restrict__ x, float* __restrict__ sum, float* __restrict__ sumsq, long rows, int C,
             int ncopy, int ld, long x_ld) {
  __shared__ float rb[NT][17];
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const long total = rows * G;
  long i = gtid;
  for (; i + stride < total; i += 2 * stride) {
    float f[8], g[8];
    const uint4 a = ldg16(x + chunk_off(i, G, x_ld)), b = ldg16(x + chunk_off(i + stride, G, x_ld));
    unpack8(a, f);
    unpack8(b, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] += f[e] + g[e]; s2[e] += f[e] * f[e] + g[e] * g[e]; }
  }
  if (i < total) {
    float f[8];
    unpack8(ldg16(x + chunk_off(i, G, x_ld)), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] += f[e]; s2[e] += f[e] * f[e]; }
  }
  const int t = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) { rb[t][e] = s1[e]; rb[t][8 + e] = s2[e]; }
  __syncthreads();
  const int lanes = NT < G ? NT : G;
  const int base_cg = (int)(((long)blockIdx.x * NT) % G);
  if (t < lanes) {
    float a[8], b[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { a[e] = 0.f; b[e] = 0.f; }
    for (int u = t; u < NT; u += G)
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += rb[u][e]; b[e] += rb[u][8 + e]; }
    const int cg = (base_cg + t) % G;
    const long slot = blockIdx.x % ncopy;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(sum + slot * ld + cg * 8 + e, a[e]);
      atomicAdd(sumsq + slot * ld + cg * 8 + e, b[e]);
    }
  }
}

// z chunk i = act(y*scale + shift [* row scale] [+ res*rscale + rshift]); y and res loads
// issued together (one round trip per chunk)
template <int ACT>
__device__ __forceinline__ void apply_chunk(const bf16* __restrict__ y, long yo, const bf16* __restrict__ res,
                                            bf16* __restrict__ z, long i, int G, const Ch& c, int act, float alpha,
                                            const RowScale& rsc) {
  const uint4 yv = ldg16(y + yo);
  const uint4 rv = res ? ldg16(res + i * 8) : make_uint4(0u, 0u, 0u, 0u);
  float f[8];
  unpack8(yv, f);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = f[j] * c.sc[j] + c.sh[j];
  if (rsc.s) {
    const float m = rsc.s[(i / G) / rsc.hw];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= m;
  }
  if (res) {
    float r[8];
    unpack8(rv, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += r[j] * c.rs[j] + c.rh[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = act_f(f[j], act, alpha);
  *reinterpret_cast<uint4*>(z + i * 8) = pack8(f);
}

// The elementwise passes are instantiated per activation code (ACT = 0..10: the activation
// folds to straight-line code, so the loop keeps its loads in flight; a run-time code made
// the switch of act_f / act_df a per-element branch, which cost EfficientNet's SiLU passes
// 2-3x their memory time) and once for a code read at run time (ACT = -1).
template <int ACT>
__global__ void __launch_bounds__(NT)
apply_kernel(const bf16* __restrict__ y, const bf16* __restrict__ res, bf16* __restrict__ z,
             const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ rscale,
             const float* __restrict__ rshift, long rows, int C, int act_, float alpha, RowScale rsc) {
  const int act = ACT >= 0 ? ACT : act_;
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int c0 = (int)(gtid % G) * 8;
  Ch c;
  load_ch(c, scale, shift, rscale, rshift, c0);
  const long total = rows * G;
  for (long i = gtid; i < total; i += stride)
    apply_chunk<ACT>(y, i * 8, res, z, i, G, c, act, alpha, rsc);
}

// the fused finalize of batchnorm.hip (bn_fwd_fused_kernel) for the generic engine: each block
// reduces the conv epilogue's partial statistic copies for its slice of <= 32 channel groups
// into LDS (scale, shift), row-part-0 blocks publish mean / invstd / scale / shift and the
// running statistics, then the apply loop over the slice's rows
constexpr int FG = 32;

template <int ACT>
__global__ void __launch_bounds__(NT)
apply_fused_kernel(const bf16* __restrict__ y, const bf16* __restrict__ res, bf16* __restrict__ z,
                   const float* __restrict__ sum, const float* __restrict__ sumsq, int ncopy,
                   const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ mean_out,
                   float* __restrict__ invstd_out, float* __restrict__ scale_out, float* __restrict__ shift_out,
                   float* __restrict__ run_mean, float* __restrict__ run_var, const float* __restrict__ rscale,
                   const float* __restrict__ rshift, long rows, int C, float eps, float momentum, int act_,
                   float alpha, RowScale rsc, const float* __restrict__ prev_tot, int prev_c,
                   float* __restrict__ tot_out, long y_ld) {
  const int act = ACT >= 0 ? ACT : act_;
  __shared__ float red[2][NT], lsc[FG * 8], lsh[FG * 8];
  const int G = C >> 3;
  const int gb = slice_groups(G, FG), nslices = G / gb;
  const int slice = blockIdx.x % nslices, part = blockIdx.x / nslices, nparts = gridDim.x / nslices;
  const int t = threadIdx.x, nch = gb * 8, c0 = slice * nch;
  {
    const int P = NT / nch, p = t / nch, cl = t % nch;
    float a = 0.f, b = 0.f;
    if (p < P) {
#pragma unroll 16
      for (int k = p; k < ncopy; k += P) { a += sum[(long)k * C + c0 + cl]; b += sumsq[(long)k * C + c0 + cl]; }
    }
    red[0][t] = a;
    red[1][t] = b;
    __syncthreads();
    if (t < nch) {
      for (int q = 1; q < P; ++q) { a += red[0][q * nch + t]; b += red[1][q * nch + t]; }
      const int ch = c0 + t;
      // channels [0, prev_c): totals published by the previous BN of a DenseNet concat chain
      // (this BN's own copies hold only the new segment's sums there: zeros)
      if (prev_tot && ch < prev_c) { a += prev_tot[ch]; b += prev_tot[prev_c + ch]; }
      if (tot_out && part == 0) { tot_out[ch] = a; tot_out[C + ch] = b; }
      const float inv_count = 1.f / (float)rows;
      const float mean = a * inv_count;
      const float var = fmaxf(b * inv_count - mean * mean, 0.f);
      const float inv = rsqrtf(var + eps);
      const float g = gamma[ch] * inv, h = beta[ch] - mean * g;
      lsc[t] = g;
      lsh[t] = h;
      if (part == 0) {
        mean_out[ch] = mean;
        invstd_out[ch] = inv;
        scale_out[ch] = g;
        shift_out[ch] = h;
        if (run_mean) {
          const float unbiased = rows > 1 ? var * (float)rows / (float)(rows - 1) : var;
          run_mean[ch] = (1.f - momentum) * run_mean[ch] + momentum * mean;
          run_var[ch] = (1.f - momentum) * run_var[ch] + momentum * unbiased;
        }
      }
    }
    __syncthreads();
  }
  const int rpi = NT / gb;
  if (t >= rpi * gb) return;
  const int gl = t % gb, cg = slice * gb + gl;
  Ch c;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    c.sc[j] = lsc[gl * 8 + j];
    c.sh[j] = lsh[gl * 8 + j];
    c.rs[j] = rscale ? rscale[cg * 8 + j] : 1.f;
    c.rh[j] = rscale ? rshift[cg * 8 + j] : 0.f;
  }
  for (long r = (long)part * rpi + t / gb; r < rows; r += (long)nparts * rpi)
    apply_chunk<ACT>(y, r * y_ld + cg * 8, res, z, r * G + cg, G, c, act, alpha, rsc);
}

// dU of one chunk: dz * act'(a), a recomputed from y (and res) with the forward's affine
template <int ACT>
__device__ __forceinline__ void dU8(float (&d)[8], const uint4& zv, const uint4& yv, const uint4& rv, bool has_res,
                                    const Ch& c, int act_, float alpha) {
  const int act = ACT >= 0 ? ACT : act_;
  if (act == 0) return;
  float yy[8], zz[8], a[8];
  unpack8(yv, yy);
  unpack8(zv, zz);
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = yy[j] * c.sc[j] + c.sh[j];
  if (has_res) {
    float r[8];
    unpack8(rv, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += r[j] * c.rs[j] + c.rh[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] *= act_df(a[j], zz[j], act, alpha);
}

template <int ACT>
__global__ void __launch_bounds__(NT)
bwd_reduce_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ z, const bf16* __restrict__ y,
                  const bf16* __restrict__ res, const float* __restrict__ mean, const float* __restrict__ scale,
                  const float* __restrict__ shift, const float* __restrict__ rscale, const float* __restrict__ rshift,
                  float* __restrict__ sums, long rows, int C, int act, float alpha, int direct, RowScale rsc,
                  int ncopy, long y_ld) {
  __shared__ float rb[NT][17];
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int c0 = (int)(gtid % G) * 8;
  Ch c;
  load_ch(c, scale, shift, rscale, rshift, c0);
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; s1[j] = 0.f; s2[j] = 0.f; }
  const long total = rows * G;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  for (long i0 = gtid; i0 < total; i0 += 2 * stride) {
    const bool two = i0 + stride < total;
    const long i1 = two ? i0 + stride : i0;
    uint4 dv[2], yv[2], zv[2], rv[2];
    dv[0] = ldg16(dz + i0 * 8); dv[1] = ldg16(dz + i1 * 8);
    yv[0] = ldg16(y + chunk_off(i0, G, y_ld)); yv[1] = ldg16(y + chunk_off(i1, G, y_ld));
    zv[0] = z ? ldg16(z + i0 * 8) : z4; zv[1] = z ? ldg16(z + i1 * 8) : z4;
    rv[0] = res ? ldg16(res + i0 * 8) : z4; rv[1] = res ? ldg16(res + i1 * 8) : z4;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !two) break;
      float d[8], yy[8];
      unpack8(dv[k], d);
      unpack8(yv[k], yy);
      dU8<ACT>(d, zv[k], yv[k], rv[k], res != nullptr, c, act, alpha);
      if (rsc.s) {
        const float m = rsc.s[((k ? i1 : i0) / G) / rsc.hw];
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] *= m;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (yy[j] - mu[j]); }
    }
  }
  const int t = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) { rb[t][e] = s1[e]; rb[t][8 + e] = s2[e]; }
  __syncthreads();
  const int lanes = NT < G ? NT : G;
  const int base_cg = (int)(((long)blockIdx.x * NT) % G);
  if (t < lanes) {
    float a[8], b[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { a[e] = 0.f; b[e] = 0.f; }
    for (int u = t; u < NT; u += G)
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += rb[u][e]; b[e] += rb[u][8 + e]; }
    const int cg = (base_cg + t) % G;
    if (direct) {   // one row of partial sums per block (every channel group covered): no atomics
      float* dst = sums + (long)blockIdx.x * 2 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dst[cg * 8 + e] = a[e];
        dst[C + cg * 8 + e] = b[e];
      }
    } else {
      float* dst = sums + (long)(blockIdx.x % ncopy) * 2 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(dst + cg * 8 + e, a[e]);
        atomicAdd(dst + C + cg * 8 + e, b[e]);
      }
    }
  }
}

// dy = k1*dU + k2 + k3*(y - mean) (coef from mlc_bn_bwd_finalize), dres = dU
template <int ACT>
__global__ void __launch_bounds__(NT)
bwd_apply_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ z, const bf16* __restrict__ y,
                 const bf16* __restrict__ res, const float* __restrict__ mean, const float* __restrict__ coef,
                 const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ rscale,
                 const float* __restrict__ rshift, bf16* __restrict__ dy, bf16* __restrict__ dres, long rows, int C,
                 int act, float alpha, RowScale rsc, const bf16* __restrict__ add, long add_ld, long y_ld,
                 bf16* __restrict__ dy2, int gsplit) {
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int c0 = (int)(gtid % G) * 8;
  Ch c;
  load_ch(c, scale, shift, rscale, rshift, c0);
  float mu[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j];
    k1[j] = coef[c0 + j];
    k2[j] = coef[C + c0 + j];
    k3[j] = coef[2 * C + c0 + j];
  }
  const long total = rows * G;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  for (long i = gtid; i < total; i += stride) {
    const uint4 dv = ldg16(dz + i * 8), yv = ldg16(y + chunk_off(i, G, y_ld));
    const uint4 zv = z ? ldg16(z + i * 8) : z4, rv = res ? ldg16(res + i * 8) : z4;
    // another consumer's gradient of y, rows of stride add_ld (a DenseNet concat's slice)
    const uint4 av = add ? ldg16(add + chunk_off(i, G, add_ld)) : z4;
    float d[8], yy[8], o[8];
    unpack8(dv, d);
    unpack8(yv, yy);
    dU8<ACT>(d, zv, yv, rv, res != nullptr, c, act, alpha);
    if (dres) *reinterpret_cast<uint4*>(dres + i * 8) = pack8(d);
    if (rsc.s) {
      const float m = rsc.s[(i / G) / rsc.hw];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] *= m;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = k1[j] * d[j] + k2[j] + k3[j] * (yy[j] - mu[j]);
    if (add) {
      float q[8];
      unpack8(av, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += q[j];
    }
    bf16* dst = dy + i * 8;
    if (dy2) {      // channel groups [0, gsplit) to dy (rows of 8*gsplit), the rest to dy2
      const unsigned q = (unsigned)i / (unsigned)G, g = (unsigned)i - q * (unsigned)G;
      dst = (int)g < gsplit ? dy + ((long)q * gsplit + g) * 8 : dy2 + ((long)q * (G - gsplit) + (g - gsplit)) * 8;
    }
    *reinterpret_cast<uint4*>(dst) = pack8(o);
  }
}

// S1 / S2 of channel c summed over the nrow partial rows [nrow][2][C], then the backward
// coefficients (dy = k1*dU + k2 + k3*(y - mean)) and dgamma / dbeta (batchnorm.hip's math)
__global__ void __launch_bounds__(NT)
bwd_finalize_rows_kernel(const float* __restrict__ part, int nrow, const float* __restrict__ invstd,
                         const float* __restrict__ gamma, float* __restrict__ coef, float* __restrict__ dgamma,
                         float* __restrict__ dbeta, long rows, int C) {
  // one wave per channel, its 64 lanes over the rows (a handful of independent loads each,
  // the finalize must not run on a few CUs: C/4 blocks)
  const int c = blockIdx.x * (NT / 64) + (threadIdx.x >> 6), q = threadIdx.x & 63;
  float S1 = 0.f, S2 = 0.f;
  if (c < C) {
    for (int k = q; k < nrow; k += 64) {
      S1 += part[(size_t)k * 2 * C + c];
      S2 += part[(size_t)k * 2 * C + C + c];
    }
  }
  S1 = wave_sum(S1);
  S2 = wave_sum(S2);
  if (c >= C || q != 0) return;
  const float invM = 1.f / (float)rows;
  const float is = invstd[c];
  const float k1 = gamma[c] * is;
  coef[c] = k1;
  coef[C + c] = -k1 * S1 * invM;
  coef[2 * C + c] = -k1 * is * is * S2 * invM;
  if (dgamma) { dgamma[c] = S2 * is; dbeta[c] = S1; }
}

// y = act(x) and dx = dy * act'(x) for a torch-free activation between native ops
template <int ACT>
__global__ void __launch_bounds__(NT)
act_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long n8, int act_, float alpha) {
  const int act = ACT >= 0 ? ACT : act_;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float f[8];
    unpack8(ldg16(x + i * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = act_f(f[j], act, alpha);
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(f);
  }
}

template <int ACT>
__global__ void __launch_bounds__(NT)
act_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, const bf16* __restrict__ y,
               bf16* __restrict__ dx, long n8, int act_, float alpha) {
  const int act = ACT >= 0 ? ACT : act_;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float d[8], a[8], z[8];
    unpack8(ldg16(dy + i * 8), d);
    unpack8(ldg16(x + i * 8), a);
    unpack8(ldg16(y + i * 8), z);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= act_df(a[j], z[j], act, alpha);
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(d);
  }
}

// channel gate (squeeze-excitation): out[n, p, c] = act(y[n, p, c] * g[n, c] [+ res[n, p, c]])
// over NHWC y [N, HW, C] and g [N, C] (bf16); act: 0 none, 1 ReLU (SE-ResNeXt's block tail)
__global__ void __launch_bounds__(NT)
chscale_fwd_kernel(const bf16* __restrict__ y, const bf16* __restrict__ g, const bf16* __restrict__ res,
                   bf16* __restrict__ out, long total, long plane, int G, int relu) {
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long n = i / plane;
    const int cg = (int)(i % G);
    float f[8], s[8], r[8];
    unpack8(ldg16(y + i * 8), f);
    unpack8(ldg16(g + (n * G + cg) * 8), s);
    if (res) unpack8(ldg16(res + i * 8), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] *= s[e];
      if (res) f[e] += r[e];
      if (relu) f[e] = fmaxf(f[e], 0.f);
    }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(f);
  }
}

// its backward in one pass: dy = dout * g, dg[n, c] += sum_p dout * y (fp32, zeroed by the
// caller).  Block (x, n, t) covers CS_ROWS pixel rows of image n and a tile of CT <= 64
// channel groups (16-byte chunks); thread t keeps ONE channel group (t % CT) and walks rows
// t / CT, + R, ... (R = 256 / CT rows per sweep), so its sums stay in registers; the R row
// partials are combined through LDS in a fixed order and leave the block as one float atomic
// per channel.
constexpr int CS_ROWS = 128;
__global__ void __launch_bounds__(NT)
chscale_bwd_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y, const bf16* __restrict__ g,
                   const bf16* __restrict__ z, const bf16* __restrict__ add, bf16* __restrict__ dy,
                   bf16* __restrict__ dres, float* __restrict__ dg, int HW, int G) {
  __shared__ float part[NT * 8];
  const int n = blockIdx.y;
  const int CT = G < 64 ? G : 64, R = NT / CT;
  const int ct0 = blockIdx.z * CT;
  const int t = threadIdx.x, cgl = t % CT, rs = t / CT;
  const int cg = ct0 + cgl;
  const bool act = rs < R && cg < G;
  const int r0 = blockIdx.x * CS_ROWS, r1 = min(HW, r0 + CS_ROWS);
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  if (act) {
    float s[8];
    unpack8(ldg16(g + ((long)n * G + cg) * 8), s);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    constexpr int U = 2;
    for (int rb = r0 + rs; rb < r1; rb += R * U) {
      uint4 dv[U], yv[U], zv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = min(rb + u * R, r1 - 1);      // clamped: always a valid row
        const long i = ((long)n * HW + r) * G + cg;
        dv[u] = ldg16(dout + i * 8);
        yv[u] = ldg16(y + i * 8);
        zv[u] = z ? ldg16(z + i * 8) : zero;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u * R;
        if (r >= r1) break;
        const long i = ((long)n * HW + r) * G + cg;
        float d[8], f[8];
        unpack8(dv[u], d);
        unpack8(yv[u], f);
        if (z) {
          float m[8];
          unpack8(zv[u], m);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
        }
        if (dres) *reinterpret_cast<uint4*>(dres + i * 8) = pack8(d);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a[e] += d[e] * f[e];
          d[e] *= s[e];
        }
        if (add) {                      // the other consumers' gradient of y (GradAcc)
          float q[8];
          unpack8(ldg16(add + i * 8), q);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] += q[e];
        }
        *reinterpret_cast<uint4*>(dy + i * 8) = pack8(d);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[t * 8 + e] = a[e];
  __syncthreads();
  // channel c of the tile: the R row partials of its group, in row order
  for (int c = t; c < CT * 8; c += NT) {
    const int gl = c >> 3, e = c & 7;
    if (ct0 + gl >= G) continue;
    float acc = 0.f;
    for (int q = 0; q < R; ++q) acc += part[(q * CT + gl) * 8 + e];
    atomicAdd(dg + ((long)n * G + ct0 + gl) * 8 + e, acc);
  }
}

inline int grid_for(long rows, int C, int cap = 1024) {
  const int G = C >> 3;
  long blocks = (rows * G + NT * 4 - 1) / (NT * 4);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  long m;
  if (G > NT) {
    m = G % NT == 0 ? G / NT : G;
  } else {
    int a = G, b = NT;
    while (b) { const int r = a % b; a = b; b = r; }
    m = G / a;
  }
  return (int)(((blocks + m - 1) / m) * m);
}

// launch an ACT-templated pass with the specialisation of the run-time code `act`
#define NA_CASE(K, A, grid, st, ...) \
  case A: hipLaunchKernelGGL(K<A>, dim3(grid), dim3(NT), 0, st, __VA_ARGS__); break;
#define NA_LAUNCH(K, grid, st, act, ...)                                                              \
  do {                                                                                              \
    switch (act) {                                                                                  \
      NA_CASE(K, 0, grid, st, __VA_ARGS__) NA_CASE(K, 1, grid, st, __VA_ARGS__)                     \
      NA_CASE(K, 2, grid, st, __VA_ARGS__) NA_CASE(K, 3, grid, st, __VA_ARGS__)                     \
      NA_CASE(K, 4, grid, st, __VA_ARGS__) NA_CASE(K, 5, grid, st, __VA_ARGS__)                     \
      NA_CASE(K, 6, grid, st, __VA_ARGS__) NA_CASE(K, 7, grid, st, __VA_ARGS__)                     \
      NA_CASE(K, 8, grid, st, __VA_ARGS__) NA_CASE(K, 9, grid, st, __VA_ARGS__)                     \
      NA_CASE(K, 10, grid, st, __VA_ARGS__)                                                         \
      default: hipLaunchKernelGGL(K<-1>, dim3(grid), dim3(NT), 0, st, __VA_ARGS__);                 \
    }                                                                                               \
  } while (0)

// block cap of the reducing passes: every block ends in C*2 float atomics onto one of 32
// partial copies, so the per-address atomic chains grow with the block count (A/B knob
// MLC_NORMACT_CAP; the streaming loop is unrolled by two to keep enough loads in flight)
inline int reduce_cap() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_NORMACT_CAP");
    v = e ? atoi(e) : 512;
    if (v < 32) v = 32;
  }
  return v;
}

// block cap of the one-call backward's reduction (mlc_bnact_bwd): its blocks store partial rows
// (no atomics), so the row finalize grows with blocks x C while a wider grid keeps more loads in
// flight.  Default (0): 1024 blocks for tensors of >= 2^26 elements (EfficientNet's early
// expanded activations), else 512 - on the generic zoo 1024 everywhere is +2.6 % on
// EfficientNet-b0 and -1.7 % on SE-ResNeXt-50, and 1024 up to 256 channels still loses on
// SE-ResNeXt (profiles/round6/normact_bwd_cap_ab*.jsonl); A/B knob MLC_NORMACT_BWD_CAP
inline int bwd_cap(long rows, int C) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_NORMACT_BWD_CAP");
    v = e ? atoi(e) : 0;
  }
  if (v <= 0) return rows * C >= (1L << 26) ? 1024 : 512;
  return v < 32 ? 32 : v;
}

// block cap of the streaming (apply) passes (A/B knob MLC_NORMACT_APPLY_CAP)
inline int apply_cap() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_NORMACT_APPLY_CAP");
    v = e ? atoi(e) : 768;
    if (v < 32) v = 32;
  }
  return v;
}

// y's row stride (0: dense); -1 when it cannot be addressed (chunk_off's 32-bit row index)
inline long y_stride(long y_ld, long rows, int C) {
  if (y_ld == 0) return C;
  if (y_ld < C || y_ld % 8 || (y_ld != C && rows * (C / 8) >= (1L << 32))) return -1;
  return y_ld;
}

inline int blocks_for(long work) {
  long b = (work + NT - 1) / NT;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace normact

using namespace normact;

// sum/sumsq: 32*C fp32 each, zeroed by the caller; C % 8 == 0
// Atomic partial-sum copies of the reductions below: NCOPY, or in deterministic mode one copy per
// block (g_mlc_ncopy of them; every copy then has exactly one adder per element, and the
// finalize kernels sum the copies in a fixed order).
inline int det_blocks_ok(int blocks) { return !g_mlc_det || blocks <= g_mlc_ncopy; }
inline int atomic_copies() { return g_mlc_det ? g_mlc_ncopy : NCOPY; }

MLC_EXPORT int mlc_bn_stats(const bf16* x, float* sum, float* sumsq, long rows, int C, hipStream_t st) {
  if (C % 8) return -1;
  const int blocks = grid_for(rows, C, reduce_cap());
  if (!det_blocks_ok(blocks)) return -2;
  hipLaunchKernelGGL(stats_kernel, dim3(blocks), dim3(NT), 0, st, x, sum, sumsq, rows, C, atomic_copies(), C,
                     (long)C);
  return hipGetLastError();
}

// the same into copies of row stride ld >= C (a channel slice of a wider BatchNorm's statistics:
// a DenseNet concat's new segment, its older channels' sums copied from the previous BN), x
// read as rows of stride x_ld (0: dense; > C: the new segment in place in the block's concat
// buffer)
MLC_EXPORT int mlc_bn_stats_ld(const bf16* x, float* sum, float* sumsq, long rows, int C, int ld, long x_ld,
                               hipStream_t st) {
  x_ld = y_stride(x_ld, rows, C);
  if (C % 8 || ld < C || x_ld < 0) return -1;
  const int blocks = grid_for(rows, C, reduce_cap());
  if (!det_blocks_ok(blocks)) return -2;
  hipLaunchKernelGGL(stats_kernel, dim3(blocks), dim3(NT), 0, st, x, sum, sumsq, rows, C, atomic_copies(), ld, x_ld);
  return hipGetLastError();
}

MLC_EXPORT int mlc_bnact_apply(const bf16* y, const bf16* res, bf16* z, const float* scale, const float* shift,
                               const float* rscale, const float* rshift, long rows, int C, int act, float alpha,
                               const float* row_scale, long hw, hipStream_t st) {
  if (C % 8 || (rscale && !rshift) || (row_scale && (act != 0 || hw < 1))) return -1;
  const RowScale rsc{row_scale, hw};
  NA_LAUNCH(apply_kernel, grid_for(rows, C, apply_cap()), st, act, y, res, z, scale, shift, rscale, rshift, rows, C, act,
            alpha, rsc);
  return hipGetLastError();
}

// finalize (from the conv epilogue's ncopy partial statistic copies) + apply in one launch;
// -1 when the shape does not fit (the caller then runs mlc_bn_finalize + mlc_bnact_apply)
MLC_EXPORT int mlc_bnact_fused(const bf16* y, const bf16* res, bf16* z, const float* sum, const float* sumsq,
                               int ncopy, const float* gamma, const float* beta, float* mean, float* invstd,
                               float* scale, float* shift, float* run_mean, float* run_var, const float* rscale,
                               const float* rshift, long rows, int C, float eps, float momentum, int act, float alpha,
                               const float* row_scale, long hw, const float* prev_tot, int prev_c, float* tot_out,
                               long y_ld, hipStream_t st) {
  const int G = C >> 3;
  y_ld = y_stride(y_ld, rows, C);
  if (C % 8 || (rscale && !rshift) || (row_scale && (act != 0 || hw < 1)) || rows < 1 || ncopy < 1 || ncopy > 64 ||
      G < 1 || prev_c < 0 || prev_c > C || y_ld < 0)
    return -1;
  const int gb = slice_groups(G, FG), nslices = G / gb, rpi = NT / gb;
  long parts = (rows + (long)rpi * 4 - 1) / ((long)rpi * 4);
  long cap = apply_cap() / nslices;
  if (cap < 1) cap = 1;
  if (parts > cap) parts = cap;
  if (parts < 1) parts = 1;
  const RowScale rsc{row_scale, hw};
  NA_LAUNCH(apply_fused_kernel, parts * nslices, st, act, y, res, z, sum, sumsq, ncopy, gamma, beta, mean, invstd,
            scale, shift, run_mean, run_var, rscale, rshift, rows, C, eps, momentum, act, alpha, rsc, prev_tot, prev_c,
            tot_out, y_ld);
  return hipGetLastError();
}

// sums: 32*2*C fp32, zeroed by the caller
MLC_EXPORT int mlc_bnact_bwd_reduce(const bf16* dz, const bf16* z, const bf16* y, const bf16* res, const float* mean,
                                    const float* scale, const float* shift, const float* rscale, const float* rshift,
                                    float* sums, long rows, int C, int act, float alpha, const float* row_scale, long hw,
                                    long y_ld, hipStream_t st) {
  y_ld = y_stride(y_ld, rows, C);
  if (C % 8 || (row_scale && (act != 0 || hw < 1)) || y_ld < 0) return -1;
  const RowScale rsc{row_scale, hw};
  const int blocks = grid_for(rows, C, reduce_cap());
  if (!det_blocks_ok(blocks)) return -2;
  NA_LAUNCH(bwd_reduce_kernel, blocks, st, act, dz, z, y, res, mean, scale, shift, rscale,
            rshift, sums, rows, C, act, alpha, 0, rsc, atomic_copies(), y_ld);
  return hipGetLastError();
}

// The whole BN(+act) backward in one call, with the reduction written as one row of partial
// sums per block (plain stores; `part` holds part_floats >= blocks*2*C floats, C <= 2048)
// instead of float atomics onto 32 copies: reduce -> finalize over the rows -> apply.
// rscale / rshift (optional): the residual is another BatchNorm's input, applied in the
// forward as res*rscale + rshift (a folded shortcut BN); the activation derivative is taken
// at that pre-activation.  dy2 (optional): dy split by channel - channels [0, c_split) to dy
// (rows of c_split), the rest to dy2 (rows of C - c_split): the two operands' gradients of a
// DenseNet concatenation, each dense.
MLC_EXPORT int mlc_bnact_bwd(const bf16* dz, const bf16* z, const bf16* y, const bf16* res, const float* mean,
                             const float* scale, const float* shift, const float* rscale, const float* rshift,
                             const float* invstd, const float* gamma,
                             float* part, long part_floats, float* coef, float* dgamma, float* dbeta, bf16* dy,
                             bf16* dres, long rows, int C, int act, float alpha, const float* row_scale, long hw,
                             const bf16* add, long add_ld, long y_ld, bf16* dy2, int c_split, hipStream_t st) {
  if (row_scale && (act != 0 || hw < 1)) return -1;
  if (dy2 && (c_split <= 0 || c_split >= C || c_split % 8 || rows * (C / 8) >= (1L << 32))) return -1;
  if (add && (add_ld < C || add_ld % 8 || (add_ld != C && rows * (C / 8) >= (1L << 32)))) return -1;
  y_ld = y_stride(y_ld, rows, C);
  if (y_ld < 0) return -1;
  const RowScale rsc{row_scale, hw};
  const int G = C >> 3;
  if (C % 8 || G > NT || part_floats < 2L * C || (rscale && !rshift)) return -1;
  long cap = part_floats / (2L * C);
  if (cap > bwd_cap(rows, C)) cap = bwd_cap(rows, C);
  int blocks = grid_for(rows, C, (int)cap);
  while (blocks > cap && blocks > 1) blocks = grid_for(rows, C, blocks / 2);   // rounding to C/8 multiples
  if ((long)blocks * 2 * C > part_floats) return -1;
  NA_LAUNCH(bwd_reduce_kernel, blocks, st, act, dz, z, y, res, mean, scale, shift, rscale, rshift, part, rows, C, act,
            alpha, 1, rsc, 1, y_ld);
  hipLaunchKernelGGL(bwd_finalize_rows_kernel, dim3((C + NT / 64 - 1) / (NT / 64)), dim3(NT), 0, st, part, blocks,
                     invstd, gamma, coef, dgamma, dbeta, rows, C);
  NA_LAUNCH(bwd_apply_kernel, grid_for(rows, C, apply_cap()), st, act, dz, z, y, res, mean, coef, scale, shift, rscale, rshift,
            dy, dres, rows, C, act, alpha, rsc, add, add_ld, y_ld, dy2, c_split / 8);
  return hipGetLastError();
}

MLC_EXPORT int mlc_bnact_bwd_apply(const bf16* dz, const bf16* z, const bf16* y, const bf16* res, const float* mean,
                                   const float* coef, const float* scale, const float* shift, const float* rscale,
                                   const float* rshift, bf16* dy, bf16* dres, long rows, int C, int act, float alpha,
                                   const float* row_scale, long hw, const bf16* add, long add_ld, long y_ld,
                                   bf16* dy2, int c_split, hipStream_t st) {
  if (dy2 && (c_split <= 0 || c_split >= C || c_split % 8 || rows * (C / 8) >= (1L << 32))) return -1;
  y_ld = y_stride(y_ld, rows, C);
  if (C % 8 || (row_scale && (act != 0 || hw < 1)) || y_ld < 0 ||
      (add && (add_ld < C || add_ld % 8 || (add_ld != C && rows * (C / 8) >= (1L << 32)))))
    return -1;
  const RowScale rsc{row_scale, hw};
  NA_LAUNCH(bwd_apply_kernel, grid_for(rows, C, apply_cap()), st, act, dz, z, y, res, mean, coef, scale, shift, rscale, rshift,
            dy, dres, rows, C, act, alpha, rsc, add, add_ld, y_ld, dy2, c_split / 8);
  return hipGetLastError();
}

MLC_EXPORT int mlc_act_fwd(const bf16* x, bf16* y, long n, int act, float alpha, hipStream_t st) {
  if (n % 8) return -1;
  NA_LAUNCH(act_fwd_kernel, blocks_for(n / 8), st, act, x, y, n / 8, act, alpha);
  return hipGetLastError();
}

MLC_EXPORT int mlc_chscale_fwd(const bf16* y, const bf16* g, const bf16* res, bf16* out, int N, long HW, int C,
                               int relu, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * HW * (C / 8);
  hipLaunchKernelGGL(chscale_fwd_kernel, dim3(blocks_for(total)), dim3(NT), 0, st, y, g, res, out, total,
                     HW * (C / 8), C / 8, relu);
  return hipGetLastError();
}

// dg: N*C fp32, zeroed by the caller; z / dres optional (ReLU mask, residual gradient);
// add optional (summed into dy)
MLC_EXPORT int mlc_chscale_bwd(const bf16* dout, const bf16* y, const bf16* g, const bf16* z, const bf16* add,
                               bf16* dy, bf16* dres, float* dg, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || N > 65535) return -1;
  const int G = C / 8, CT = G < 64 ? G : 64;
  hipLaunchKernelGGL(chscale_bwd_kernel, dim3((HW + CS_ROWS - 1) / CS_ROWS, N, (G + CT - 1) / CT), dim3(NT), 0, st,
                     dout, y, g, z, add, dy, dres, dg, HW, G);
  return hipGetLastError();
}

MLC_EXPORT int mlc_act_bwd(const bf16* dy, const bf16* x, const bf16* y, bf16* dx, long n, int act, float alpha,
                           hipStream_t st) {
  if (n % 8) return -1;
  NA_LAUNCH(act_bwd_kernel, blocks_for(n / 8), st, act, dy, x, y, dx, n / 8, act, alpha);
  return hipGetLastError();
}
