// Training BatchNorm for NHWC bf16 activations, fused with residual-add and ReLU.
//
// Forward statistics are NOT computed here: the producing conv accumulates per-channel
// sum / sum-of-squares in its epilogue (igemm.hip EpiBF16), a C-thread finalize turns
// them into (scale, shift), and BN forward is a single read-y / write-z pass:
// z = act(y*scale + shift [+ residual]).
// Backward is two passes: a per-channel reduction of dU and dU*(y-mean) (dU = dz masked
// by z>0 when the ReLU is fused), then an elementwise pass producing dy (and the
// residual-branch gradient dU).
//
// Channel-group ownership: launches use a thread count that is a multiple of C/8, so
// each thread owns one fixed 8-channel group for its whole grid-stride loop and keeps
// the per-channel constants in registers.  All accesses are 16 B per lane.
#include "common.h"

namespace {

constexpr int NT = 256;

// per-channel finalize: reduce the conv epilogue's NSTAT partial copies, publish batch
// mean / invstd, the fused affine (scale, shift) and update the running statistics.
// 8 lanes per channel (32 channels per block) each sum every 8th copy, then a shuffle
// reduction: the copies are all in flight at once instead of one dependent load chain.
constexpr int FL = 8;
__global__ void __launch_bounds__(NT)
bn_finalize_kernel(const float* __restrict__ sum, const float* __restrict__ sumsq, int ncopy,
                   const float* __restrict__ gamma, const float* __restrict__ beta,
                   float* __restrict__ save_mean, float* __restrict__ save_invstd,
                   float* __restrict__ scale, float* __restrict__ shift,
                   float* __restrict__ run_mean, float* __restrict__ run_var,
                   long rows, int C, float eps, float momentum) {
  const int c = blockIdx.x * (NT / FL) + (threadIdx.x / FL), q = threadIdx.x % FL;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int k = q; k < ncopy; k += FL) { s1 += sum[(long)k * C + c]; s2 += sumsq[(long)k * C + c]; }
  }
#pragma unroll
  for (int o = 1; o < FL; o <<= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
  if (c >= C || q != 0) return;
  const float inv_count = 1.f / (float)rows;
  const float mean = s1 * inv_count;
  const float var = fmaxf(s2 * inv_count - mean * mean, 0.f);
  const float inv = rsqrtf(var + eps);
  save_mean[c] = mean;
  save_invstd[c] = inv;
  const float g = gamma[c] * inv;
  scale[c] = g;
  shift[c] = beta[c] - mean * g;
  if (run_mean) {
    const float unbiased = rows > 1 ? var * (float)rows / (float)(rows - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
  }
}

// z = act(y*scale + shift [+ res*rscale + rshift]) -- the residual's own affine lets a
// block's downsample-branch BatchNorm be applied here instead of in a pass of its own
// U chunks per thread per iteration: all U loads are issued (from clamped, always-valid
// indices) before any compute or store, so a thread keeps U x 16 B (x2 with a residual) in
// flight instead of one dependent load-store pair
template <int U>
__global__ void __launch_bounds__(NT)
bn_fwd_apply_kernel(const bf16* __restrict__ y, const bf16* __restrict__ res, bf16* __restrict__ z,
                    const float* __restrict__ scale_, const float* __restrict__ shift_,
                    const float* __restrict__ rscale_, const float* __restrict__ rshift_,
                    long rows, int C, int relu) {
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int cg = (int)(gtid % G);
  const int c0 = cg * 8;
  float scale[8], shift[8], rscale[8], rshift[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    scale[j] = scale_[c0 + j]; shift[j] = shift_[c0 + j];
    rscale[j] = rscale_ ? rscale_[c0 + j] : 1.f; rshift[j] = rscale_ ? rshift_[c0 + j] : 0.f;
  }
  const long total = rows * G;
  const long last = total - G + cg;        // the last chunk of this thread's channel group
  for (long i0 = gtid; i0 < total; i0 += stride * U) {
    uint4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = min(i0 + u * stride, last);
      yv[u] = *reinterpret_cast<const uint4*>(y + i * 8);
      if (res) rv[u] = *reinterpret_cast<const uint4*>(res + i * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      float f[8];
      unpack8(yv[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * scale[j] + shift[j];
      if (res) {
        float r[8];
        unpack8(rv[u], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += r[j] * rscale[j] + rshift[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      if (i < total) *reinterpret_cast<uint4*>(z + i * 8) = pack8(f);
    }
  }
}

// Partial reductions for BN backward: copy k = block % NSTAT of sums[NSTAT][2][C]
// receives  sum dU  and  sum dU*(y-mean)  of the block's rows (copies keep the
// same-address atomic contention low: every address sees ~blocks/NSTAT adds).
constexpr int NSTAT = 32;

__global__ void __launch_bounds__(NT)
bn_bwd_reduce_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ z, const bf16* __restrict__ y,
                     const float* __restrict__ mean, float* __restrict__ sums, long rows, int C, int ncopy) {
  __shared__ float red[2][NT][9];
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int cg = (int)(gtid % G);
  const int c0 = cg * 8;
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; s1[j] = 0.f; s2[j] = 0.f; }
  const long total = rows * G;
  // 4 chunks per lane in flight through ext-vector loads (with HIP's uint4 struct loads
  // hipcc waited vmcnt(0) after every load of this accumulating loop)
  constexpr int U = 4;
  for (long i0 = gtid; i0 < total; i0 += stride * U) {
    uint4 dv[U], yv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      const long off = (i < total ? i : i0) * 8;
      dv[u] = ldg16(dz + off);
      yv[u] = ldg16(y + off);
      zv[u] = z ? ldg16(z + off) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u * stride >= total) break;
      float d[8], yy[8];
      unpack8(dv[u], d);
      unpack8(yv[u], yy);
      if (z) {
        float zz[8];
        unpack8(zv[u], zz);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = zz[j] > 0.f ? d[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (yy[j] - mu[j]); }
    }
  }
  // combine threads of this block owning the same channel group (tid = tid' mod G)
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][t][j] = s1[j]; red[1][t][j] = s2[j]; }
  __syncthreads();
  const int lanes = NT < G ? NT : G;  // distinct groups present in this block
  const int base_cg = (int)(((long)blockIdx.x * NT) % G);
  float* dst = sums + (size_t)(blockIdx.x % ncopy) * 2 * C;
  if (t < lanes) {
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
    for (int u = t; u < NT; u += G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] += red[0][u][j]; b[j] += red[1][u][j]; }
    }
    const int cgt = (base_cg + t) % G;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(dst + cgt * 8 + j, a[j]);
      atomicAdd(dst + C + cgt * 8 + j, b[j]);
    }
  }
}

// per-channel: reduce the NSTAT copies, publish dgamma/dbeta and the three
// coefficients of  dy = k1*dU + k2 + k3*(y-mean)  (coef[0:C]=k1, [C:2C]=k2, [2C:3C]=k3);
// 8 lanes per channel as in bn_finalize_kernel
__global__ void __launch_bounds__(NT)
bn_bwd_finalize_kernel(const float* __restrict__ sums, const float* __restrict__ invstd,
                       const float* __restrict__ gamma, float* __restrict__ coef,
                       float* __restrict__ dgamma, float* __restrict__ dbeta, long rows, int C, int ncopy) {
  const int c = blockIdx.x * (NT / FL) + (threadIdx.x / FL), q = threadIdx.x % FL;
  float S1 = 0.f, S2 = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int k = q; k < ncopy; k += FL) {
      S1 += sums[(size_t)k * 2 * C + c];
      S2 += sums[(size_t)k * 2 * C + C + c];
    }
  }
#pragma unroll
  for (int o = 1; o < FL; o <<= 1) { S1 += __shfl_xor(S1, o, 64); S2 += __shfl_xor(S2, o, 64); }
  if (c >= C || q != 0) return;
  const float invM = 1.f / (float)rows;
  const float is = invstd[c];
  const float k1 = gamma[c] * is;
  coef[c] = k1;
  coef[C + c] = -k1 * S1 * invM;
  coef[2 * C + c] = -k1 * is * is * S2 * invM;
  if (dgamma) { dgamma[c] = S2 * is; dbeta[c] = S1; }
}

// dy = k1*dU + k2 + k3*(y-mean);  dres = dU (optional)
template <int U>
__global__ void __launch_bounds__(NT)
bn_bwd_apply_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ z, const bf16* __restrict__ y,
                    const float* __restrict__ mean, const float* __restrict__ coef,
                    bf16* __restrict__ dy, bf16* __restrict__ dres, long rows, int C) {
  const int G = C >> 3;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const long stride = (long)gridDim.x * NT;
  const int cg = (int)(gtid % G);
  const int c0 = cg * 8;
  float mu[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j];
    k1[j] = coef[c0 + j];
    k2[j] = coef[C + c0 + j];
    k3[j] = coef[2 * C + c0 + j];
  }
  const long total = rows * G;
  const long last = total - G + cg;
  for (long i0 = gtid; i0 < total; i0 += stride * U) {
    uint4 dv[U], yv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = min(i0 + u * stride, last);
      dv[u] = *reinterpret_cast<const uint4*>(dz + i * 8);
      yv[u] = *reinterpret_cast<const uint4*>(y + i * 8);
      if (z) zv[u] = *reinterpret_cast<const uint4*>(z + i * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      float d[8], yy[8], o[8];
      unpack8(dv[u], d);
      unpack8(yv[u], yy);
      if (z) {
        float zz[8];
        unpack8(zv[u], zz);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = zz[j] > 0.f ? d[j] : 0.f;
      }
      if (i < total) {
        if (dres) *reinterpret_cast<uint4*>(dres + i * 8) = pack8(d);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = k1[j] * d[j] + k2[j] + k3[j] * (yy[j] - mu[j]);
        *reinterpret_cast<uint4*>(dy + i * 8) = pack8(o);
      }
    }
  }
}

// ---- finalize folded into the apply pass (one launch per BN instead of two) -------------
// The per-channel finalize kernels sat on the critical path between a GEMM and its apply
// pass, 53 + 53 of them per ResNet-50 step (~5 us each with the dependency gap).  Here each
// block first reduces the NSTAT partial copies for the channels it touches into LDS: a block
// owns a slice of FG <= 32 channel groups (<= 256 channels, 64 KB of partial sums read from
// L2) and strides over the rows; blocks of row-part 0 also publish the per-channel outputs
// (batch mean / invstd, scale / shift, running statistics - or dgamma / dbeta), so those
// are written once.  Not used in deterministic mode (one copy per contributing block).
constexpr int FG = 32;

__device__ __forceinline__ void fused_geom(int G, int& gb, int& nslices) {
  gb = slice_groups(G, FG);
  nslices = G / gb;
}

// red[0][c], red[1][c] (c < nch) = sum over the ncopy copies of a[k*stride + c0 + c] and
// b[k*stride + c0 + c]: the block's threads split the copies (P = NT / nch phases, each
// thread's loads all issued before they are summed), then one LDS pass folds the phases
__device__ __forceinline__ void fused_reduce(const float* __restrict__ a, const float* __restrict__ b, long stride,
                                             int ncopy, int c0, int nch, int t, float (&red)[2][NT]) {
  const int P = NT / nch, p = t / nch, cl = t % nch;
  float x = 0.f, y = 0.f;
  if (p < P) {
#pragma unroll 16
    for (int k = p; k < ncopy; k += P) { x += a[k * stride + c0 + cl]; y += b[k * stride + c0 + cl]; }
  }
  red[0][t] = x;
  red[1][t] = y;
  __syncthreads();
  if (t < nch) {
    for (int q = 1; q < P; ++q) { x += red[0][q * nch + t]; y += red[1][q * nch + t]; }
  }
  __syncthreads();
  if (t < nch) { red[0][t] = x; red[1][t] = y; }
  __syncthreads();
}

template <int U>
__global__ void __launch_bounds__(NT)
bn_fwd_fused_kernel(const bf16* __restrict__ y, const bf16* __restrict__ res, bf16* __restrict__ z,
                    const float* __restrict__ sum, const float* __restrict__ sumsq, int ncopy,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    float* __restrict__ save_mean, float* __restrict__ save_invstd,
                    float* __restrict__ scale_out, float* __restrict__ shift_out,
                    float* __restrict__ run_mean, float* __restrict__ run_var,
                    const float* __restrict__ rscale_, const float* __restrict__ rshift_,
                    long rows, int C, float eps, float momentum, int relu) {
  __shared__ float lsc[FG * 8], lsh[FG * 8], red[2][NT];
  const int G = C >> 3;
  int gb, nslices;
  fused_geom(G, gb, nslices);
  const int slice = blockIdx.x % nslices, part = blockIdx.x / nslices, nparts = gridDim.x / nslices;
  const int t = threadIdx.x, nch = gb * 8, c0 = slice * nch;
  fused_reduce(sum, sumsq, (long)C, ncopy, c0, nch, t, red);
  if (t < nch) {
    const int c = c0 + t;
    const float s1 = red[0][t], s2 = red[1][t];
    const float inv_count = 1.f / (float)rows;
    const float mean = s1 * inv_count;
    const float var = fmaxf(s2 * inv_count - mean * mean, 0.f);
    const float inv = rsqrtf(var + eps);
    const float g = gamma[c] * inv, h = beta[c] - mean * g;
    lsc[t] = g;
    lsh[t] = h;
    if (part == 0) {
      save_mean[c] = mean;
      save_invstd[c] = inv;
      scale_out[c] = g;
      shift_out[c] = h;
      if (run_mean) {
        const float unbiased = rows > 1 ? var * (float)rows / (float)(rows - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
      }
    }
  }
  __syncthreads();
  const int rpi = NT / gb;                          // rows per block iteration
  if (t >= rpi * gb) return;
  const int g = t % gb, cg = slice * gb + g;
  float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = lsc[g * 8 + j];
    sh[j] = lsh[g * 8 + j];
    rsc[j] = rscale_ ? rscale_[cg * 8 + j] : 1.f;
    rsh[j] = rscale_ ? rshift_[cg * 8 + j] : 0.f;
  }
  // U rows per thread per iteration, every load issued before any use (one round trip per
  // U chunks; the y and residual loads of a chunk together)
  const long step = (long)nparts * rpi;
  for (long r0 = (long)part * rpi + t / gb; r0 < rows; r0 += step * U) {
    uint4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = min(r0 + u * step, rows - 1);      // clamped: always a valid row
      yv[u] = ldg16(y + (r * G + cg) * 8);
      rv[u] = res ? ldg16(res + (r * G + cg) * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + u * step;
      if (r >= rows) break;
      float f[8];
      unpack8(yv[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * sc[j] + sh[j];
      if (res) {
        float q[8];
        unpack8(rv[u], q);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += q[j] * rsc[j] + rsh[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      *reinterpret_cast<uint4*>(z + (r * G + cg) * 8) = pack8(f);
    }
  }
}

// dy = k1*dU + k2 + k3*(y-mean) with (k1, k2, k3) from the reduction copies (sums [ncopy][2][C])
// folded in; dres = dU (optional); z != null applies the ReLU mask z > 0 to dz
template <int U>
__global__ void __launch_bounds__(NT)
bn_bwd_fused_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ z, const bf16* __restrict__ y,
                    const float* __restrict__ mean, const float* __restrict__ sums, int ncopy,
                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                    float* __restrict__ dgamma, float* __restrict__ dbeta, bf16* __restrict__ dy,
                    bf16* __restrict__ dres, long rows, int C) {
  __shared__ float lk[3][FG * 8], lmu[FG * 8], red[2][NT];
  const int G = C >> 3;
  int gb, nslices;
  fused_geom(G, gb, nslices);
  const int slice = blockIdx.x % nslices, part = blockIdx.x / nslices, nparts = gridDim.x / nslices;
  const int t = threadIdx.x, nch = gb * 8, c0 = slice * nch;
  fused_reduce(sums, sums + C, 2L * C, ncopy, c0, nch, t, red);
  if (t < nch) {
    const int c = c0 + t;
    const float S1 = red[0][t], S2 = red[1][t];
    const float invM = 1.f / (float)rows;
    const float is = invstd[c];
    const float k1 = gamma[c] * is;
    lk[0][t] = k1;
    lk[1][t] = -k1 * S1 * invM;
    lk[2][t] = -k1 * is * is * S2 * invM;
    lmu[t] = mean[c];
    if (part == 0 && dgamma) { dgamma[c] = S2 * is; dbeta[c] = S1; }
  }
  __syncthreads();
  const int rpi = NT / gb;
  if (t >= rpi * gb) return;
  const int g = t % gb, cg = slice * gb + g;
  float k1[8], k2[8], k3[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = lk[0][g * 8 + j];
    k2[j] = lk[1][g * 8 + j];
    k3[j] = lk[2][g * 8 + j];
    mu[j] = lmu[g * 8 + j];
  }
  const long step = (long)nparts * rpi;
  for (long r0 = (long)part * rpi + t / gb; r0 < rows; r0 += step * U) {
    uint4 dv[U], yv[U], zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = min(r0 + u * step, rows - 1);      // clamped: always a valid row
      const long i = r * G + cg;
      dv[u] = ldg16(dz + i * 8);
      yv[u] = ldg16(y + i * 8);
      zv[u] = z ? ldg16(z + i * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + u * step;
      if (r >= rows) break;
      const long i = r * G + cg;
      float d[8], yy[8], o[8];
      unpack8(dv[u], d);
      unpack8(yv[u], yy);
      if (z) {
        float zz[8];
        unpack8(zv[u], zz);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = zz[j] > 0.f ? d[j] : 0.f;
      }
      if (dres) *reinterpret_cast<uint4*>(dres + i * 8) = pack8(d);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k1[j] * d[j] + k2[j] + k3[j] * (yy[j] - mu[j]);
      *reinterpret_cast<uint4*>(dy + i * 8) = pack8(o);
    }
  }
}

// A/B knobs of the elementwise passes: chunks per thread per iteration (1, 2, 4) and the
// block cap of grid_for
int g_unroll = 1;
// measured: 512-768 beat 1024 by ~0.4 % on ResNet-50, 2048+ lose 2 %; 512 vs 768 +0.3 % in
// 3 interleaved rounds (profiles/round6/bn_knobs_ab.jsonl), 1536 -1.5 %, unroll 2 / 4 -0.3 %
int g_max_blocks = 512;
int g_fused = 1;

// block-count granularity that keeps blocks * NT a multiple of G
long grid_mult(int G) {
  if (G > NT) return G / NT;
  int a = G, b = NT;
  while (b) { const int r = a % b; a = b; b = r; }
  return G / a;
}

int grid_for(long rows, int C) {
  const int G = C >> 3;
  long total = rows * G;
  // threads must be a multiple of G: blocks*256 % G == 0 always holds for G | 256;
  // for G > 256 (C > 2048) make the block count a multiple of G/256.
  long blocks = (total + NT * 4 - 1) / (NT * 4);   // ~4 chunks per thread
  if (blocks > g_max_blocks) blocks = g_max_blocks;
  if (blocks < 1) blocks = 1;
  // the grid's thread count must be a multiple of G: G | 256 always holds; otherwise
  // (e.g. C = 48, DeepLab's low-level projection: G = 6) round the block count up to a
  // multiple of G / gcd(G, 256); for G > 256 (C > 2048) to a multiple of G/256
  const long m = grid_mult(G);
  blocks = ((blocks + m - 1) / m) * m;
  return (int)blocks;
}

// grid of the fused passes: ~g_max_blocks blocks, a multiple of the channel slices
int fused_grid(long rows, int C) {
  const int G = C >> 3;
  const int gb = slice_groups(G, FG), nslices = G / gb;
  const int rpi = NT / gb;
  long parts = (rows + (long)rpi * 4 - 1) / ((long)rpi * 4);   // ~4 rows per thread at least
  long cap = g_max_blocks / nslices;
  if (cap < 1) cap = 1;
  if (parts > cap) parts = cap;
  if (parts < 1) parts = 1;
  return (int)(parts * nslices);
}

bool fused_ok(int C, int ncopy) {
  const int G = C >> 3;
  if (g_fused != 1 || C % 8 || ncopy < 1 || ncopy > 64) return false;   // deterministic copies: the finalize kernel
  return G >= 1;
}

bool shape_ok(int C) {
  const int G = C >> 3;
  if (C % 8) return false;
  return G <= NT || G % NT == 0;
}

}  // namespace

int g_mlc_ncopy = NSTAT;
int g_mlc_det = 0;

// deterministic mode on/off; ncopy = partial-sum copies of every reduction (>= NSTAT;
// deterministic mode needs at least one per contributing block, the launchers check)
MLC_EXPORT int mlc_set_deterministic(int det, int ncopy) {
  g_mlc_det = det ? 1 : 0;
  g_mlc_ncopy = ncopy >= NSTAT ? ncopy : NSTAT;
  return 0;
}
MLC_EXPORT int mlc_get_stat_copies() { return g_mlc_ncopy; }
MLC_EXPORT int mlc_get_deterministic() { return g_mlc_det; }

MLC_EXPORT int mlc_bn_finalize(const float* sum, const float* sumsq, int ncopy, const float* gamma,
                               const float* beta, float* save_mean, float* save_invstd, float* scale,
                               float* shift, float* run_mean, float* run_var, long rows, int C,
                               float eps, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + NT / FL - 1) / (NT / FL)), dim3(NT), 0, st, sum, sumsq, ncopy,
                     gamma, beta, save_mean, save_invstd, scale, shift, run_mean, run_var, rows, C, eps,
                     momentum);
  return hipGetLastError();
}

MLC_EXPORT int mlc_bn_fwd_apply2(const bf16* y, const bf16* res, bf16* z, const float* scale,
                                 const float* shift, const float* rscale, const float* rshift, long rows,
                                 int C, int relu, hipStream_t st) {
  if (!shape_ok(C) || (rscale && !rshift)) return -1;
  const dim3 grid(grid_for(rows, C));
  if (g_unroll >= 4)
    hipLaunchKernelGGL(bn_fwd_apply_kernel<4>, grid, dim3(NT), 0, st, y, res, z, scale, shift, rscale, rshift,
                       rows, C, relu);
  else if (g_unroll == 2)
    hipLaunchKernelGGL(bn_fwd_apply_kernel<2>, grid, dim3(NT), 0, st, y, res, z, scale, shift, rscale, rshift,
                       rows, C, relu);
  else
    hipLaunchKernelGGL(bn_fwd_apply_kernel<1>, grid, dim3(NT), 0, st, y, res, z, scale, shift, rscale, rshift,
                       rows, C, relu);
  return hipGetLastError();
}

MLC_EXPORT int mlc_bn_fwd_apply(const bf16* y, const bf16* res, bf16* z, const float* scale,
                                const float* shift, long rows, int C, int relu, hipStream_t st) {
  return mlc_bn_fwd_apply2(y, res, z, scale, shift, nullptr, nullptr, rows, C, relu, st);
}

// sums must hold ncopy*2*C floats (mlc_get_stat_copies), zeroed by the caller
MLC_EXPORT int mlc_bn_bwd_reduce(const bf16* dz, const bf16* z, const bf16* y, const float* mean,
                                 float* sums, long rows, int C, hipStream_t st) {
  if (!shape_ok(C)) return -1;
  // every block ends with 2*C atomics: wide tensors get fewer, longer-running blocks
  // (1024 blocks at C = 2048 issued 4M atomics and took 122 us on a 51 MB tensor)
  int blocks = grid_for(rows, C);
  const int G = C >> 3;
  if (G >= 64) {
    int cap = 65536 / G;
    if (cap < 256) cap = 256;
    const long m = grid_mult(G);
    cap = (int)(((cap + m - 1) / m) * m);
    if (blocks > cap) blocks = cap;
  }
  if (g_mlc_det && blocks > g_mlc_ncopy) return -2;   // a copy per block or not deterministic
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(blocks), dim3(NT), 0, st, dz, z, y,
                     mean, sums, rows, C, g_mlc_ncopy);
  return hipGetLastError();
}

// coef must hold 3*C floats
MLC_EXPORT int mlc_bn_bwd_finalize(const float* sums, const float* invstd, const float* gamma,
                                   float* coef, float* dgamma, float* dbeta, long rows, int C,
                                   hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + NT / FL - 1) / (NT / FL)), dim3(NT), 0, st, sums, invstd,
                     gamma, coef, dgamma, dbeta, rows, C, g_mlc_ncopy);
  return hipGetLastError();
}

// finalize + apply in one launch (bn_fwd_fused_kernel); returns -1 when the shape / copy
// count does not fit (the caller then runs mlc_bn_finalize + mlc_bn_fwd_apply2)
MLC_EXPORT int mlc_bn_fwd_fused(const bf16* y, const bf16* res, bf16* z, const float* sum, const float* sumsq,
                                int ncopy, const float* gamma, const float* beta, float* save_mean,
                                float* save_invstd, float* scale, float* shift, float* run_mean, float* run_var,
                                const float* rscale, const float* rshift, long rows, int C, float eps,
                                float momentum, int relu, hipStream_t st) {
  if (!fused_ok(C, ncopy) || (rscale && !rshift) || rows < 1) return -1;
#define MLC_BNF(U) hipLaunchKernelGGL(bn_fwd_fused_kernel<U>, dim3(fused_grid(rows, C)), dim3(NT), 0, st, y, res, z, \
                                      sum, sumsq, ncopy, gamma, beta, save_mean, save_invstd, scale, shift, run_mean, \
                                      run_var, rscale, rshift, rows, C, eps, momentum, relu)
  if (g_unroll >= 4) MLC_BNF(4); else if (g_unroll == 2) MLC_BNF(2); else MLC_BNF(1);
#undef MLC_BNF
  return hipGetLastError();
}

// backward finalize + apply in one launch (bn_bwd_fused_kernel); -1: not applicable
MLC_EXPORT int mlc_bn_bwd_fused(const bf16* dz, const bf16* z, const bf16* y, const float* mean, const float* sums,
                                int ncopy, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                                bf16* dy, bf16* dres, long rows, int C, hipStream_t st) {
  if (!fused_ok(C, ncopy) || rows < 1) return -1;
#define MLC_BNB(U) hipLaunchKernelGGL(bn_bwd_fused_kernel<U>, dim3(fused_grid(rows, C)), dim3(NT), 0, st, dz, z, y, \
                                      mean, sums, ncopy, invstd, gamma, dgamma, dbeta, dy, dres, rows, C)
  if (g_unroll >= 4) MLC_BNB(4); else if (g_unroll == 2) MLC_BNB(2); else MLC_BNB(1);
#undef MLC_BNB
  return hipGetLastError();
}

MLC_EXPORT int mlc_bn_bwd_apply(const bf16* dz, const bf16* z, const bf16* y, const float* mean,
                                const float* coef, bf16* dy, bf16* dres, long rows, int C,
                                hipStream_t st) {
  if (!shape_ok(C)) return -1;
  const dim3 grid(grid_for(rows, C));
  if (g_unroll >= 4)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<4>, grid, dim3(NT), 0, st, dz, z, y, mean, coef, dy, dres, rows, C);
  else if (g_unroll == 2)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, grid, dim3(NT), 0, st, dz, z, y, mean, coef, dy, dres, rows, C);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, grid, dim3(NT), 0, st, dz, z, y, mean, coef, dy, dres, rows, C);
  return hipGetLastError();
}

// A/B knobs: key 0 = chunks per thread of the apply passes, 1 = block cap, 2 = finalize
// folded into the apply passes (1 on, 2 off; mlc_bn_{fwd,bwd}_fused return -1 when off);
// value < 0 only reads.  Returns the previous value.
MLC_EXPORT int mlc_bn_get_set(int key, int value) {
  int* k = key == 0 ? &g_unroll : key == 1 ? &g_max_blocks : key == 2 ? &g_fused : nullptr;
  if (!k) return -1;
  const int old = *k;
  if (value > 0) *k = value;
  return old;
}
