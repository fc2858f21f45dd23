// Segmentation-model kernels (U-Net decoder and head) for gfx950, NHWC bf16.
//
// * upcat: x2 nearest upsample of the decoder input fused with the channel concat of the
//   encoder skip: out[n,y,x,:C1] = lo[n,y/2,x/2,:], out[n,y,x,C1:] = skip[n,y,x,:].  One
//   16-byte chunk per thread, both sources and the destination read/written once.
//   Backward: dlo = 2x2 sum-pool of dout[..., :C1] (fp32 accumulate), dskip = dout[..., C1:].
// * seg head + BCE-with-logits + soft-Dice loss, K <= 4 classes (one
//   sigmoid per class, the Severstal-style multi-label masks): the 1x1 output conv
//   (Cin -> K, + bias) is K per-pixel dot products, so it is fused with the loss.  Forward: logit, sigmoid, and the four global sums the loss needs (BCE sum,
//   sum s*t, sum s, sum t) reduced per block then one atomic each.  Backward (the Dice
//   gradient needs the global sums, hence a second pass): dlogit, dx = dlogit * w, and
//   dw / db block-reduced into the grad arena.
//   loss = bce_w * mean(BCE) + dice_w * (1 - (2*I + eps) / (U + eps)),  I = sum s*t,
//   U = sum s + sum t  (contrib/criterion.BCEDiceLoss).
// * bilinear x2 upsampling (align_corners=True) of the FPN heads: forward 4 taps per
//   output chunk, backward as a gather over the outputs that read an input pixel.
// * GroupNorm + ReLU of the FPN heads: per-(sample, channel) sums, then one elementwise pass
//   (forward and backward each: a reduction pass + an apply pass).
#include "common.h"

namespace {

constexpr int NT = 256;

__global__ void __launch_bounds__(NT)
upcat_fwd_kernel(const bf16* __restrict__ lo, const bf16* __restrict__ skip, bf16* __restrict__ out, int N, int h,
                 int w, int C1, int C2) {
  const int H = 2 * h, W = 2 * w, C = C1 + C2, cpr = C / 8;
  const long total = (long)N * H * W * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long p = i / cpr;                  // output pixel (n, y, x)
    const int x = (int)(p % W);
    const long t = p / W;
    const int y = (int)(t % H);
    const long n = t / H;
    uint4 v;
    if (c8 * 8 < C1) {
      v = *reinterpret_cast<const uint4*>(lo + ((n * h + (y >> 1)) * w + (x >> 1)) * C1 + c8 * 8);
    } else {
      v = *reinterpret_cast<const uint4*>(skip + p * C2 + (c8 * 8 - C1));
    }
    *reinterpret_cast<uint4*>(out + p * C + c8 * 8) = v;
  }
}

__global__ void __launch_bounds__(NT)
upcat_bwd_lo_kernel(const bf16* __restrict__ dout, bf16* __restrict__ dlo, int N, int h, int w, int C1, int C) {
  const int W = 2 * w, cpr = C1 / 8;
  const long total = (long)N * h * w * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long q = i / cpr;                  // low-res pixel (n, yy, xx)
    const int xx = (int)(q % w);
    const long t = q / w;
    const int yy = (int)(t % h);
    const long n = t / h;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const long p = (n * 2 * h + 2 * yy + a) * W + 2 * xx + b;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(dout + p * C + c8 * 8), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
      }
    *reinterpret_cast<uint4*>(dlo + q * C1 + c8 * 8) = pack8(acc);
  }
}

__global__ void __launch_bounds__(NT)
upcat_bwd_skip_kernel(const bf16* __restrict__ dout, bf16* __restrict__ dskip, long P, int C1, int C2) {
  const int C = C1 + C2, cpr = C2 / 8;
  const long total = P * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long p = i / cpr;
    *reinterpret_cast<uint4*>(dskip + p * C2 + c8 * 8) =
        *reinterpret_cast<const uint4*>(dout + p * C + C1 + c8 * 8);
  }
}

// block-wide sum of NV floats per thread; result valid in thread 0
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wave * NV + k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float s = 0.f;
      for (int q = 0; q < NT / 64; ++q) s += red[q * NV + k];
      v[k] = s;
    }
  }
}

// K (<= 8) per-pixel logits z_k = b_k + x[p] . w_k, weights [K][C] staged in LDS
template <int K>
__device__ __forceinline__ void pixel_logits(const bf16* xp, const float* w, const float* b, int C, float (&z)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) z[k] = b[k];
  for (int c = 0; c < C; c += 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xp + c), f);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) z[k] += f[e] * w[k * C + c + e];
  }
}

// sums[0..3] += (BCE sum, sum s*t, sum s, sum t) over pixels and classes; target [P][K]
template <int K>
__global__ void __launch_bounds__(NT)
seg_head_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                    const float* __restrict__ target, float* __restrict__ logits, float* __restrict__ sums, long P,
                    int C) {
  __shared__ float red[NT / 64 * 4];
  __shared__ float ws[K * 256];
  __shared__ float bs[K];
  for (int c = threadIdx.x; c < K * C; c += NT) ws[c] = w[c];
  if (threadIdx.x < K) bs[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (long p = (long)blockIdx.x * NT + threadIdx.x; p < P; p += (long)gridDim.x * NT) {
    float z[K];
    pixel_logits<K>(x + p * C, ws, bs, C, z);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float t = target[p * K + k];
      const float sg = 1.f / (1.f + __expf(-z[k]));
      if (logits) logits[p * K + k] = z[k];
      acc[0] += fmaxf(z[k], 0.f) - z[k] * t + log1pf(__expf(-fabsf(z[k])));
      acc[1] += sg * t;
      acc[2] += sg;
      acc[3] += t;
    }
  }
  block_sum<4>(acc, red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(sums + k, acc[k]);
  }
}

// dx[p] = sum_k dz_pk w_k;  dw[k][c] += sum_p dz_pk x[p,c];  db[k] += sum_p dz_pk
template <int K>
__global__ void __launch_bounds__(NT)
seg_head_bwd_kernel(const bf16* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                    const float* __restrict__ target, const float* __restrict__ sums, bf16* __restrict__ dx,
                    float* __restrict__ dw, float* __restrict__ db, long P, int C, float bce_w, float dice_w,
                    float eps) {
  __shared__ float red[NT / 64 * K];
  __shared__ float ws[K * 256];
  __shared__ float bs[K];
  __shared__ float dws[NT / 64][K * 256];
  for (int c = threadIdx.x; c < K * C; c += NT) ws[c] = w[c];
  if (threadIdx.x < K) bs[threadIdx.x] = bias[threadIdx.x];
  for (int c = threadIdx.x; c < NT / 64 * K * 256; c += NT) (&dws[0][0])[c] = 0.f;
  __syncthreads();
  const float I = sums[1], U = sums[2] + sums[3];
  const float inv_n = 1.f / ((float)P * K);
  const float den = U + eps, num = 2.f * I + eps;
  // d(1 - dice)/ds = -(2 t den - num) / den^2
  const float ka = -2.f / den, kb = num / (den * den);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dbias[K];
#pragma unroll
  for (int k = 0; k < K; ++k) dbias[k] = 0.f;
  // per-wave partials of dw in LDS (K*C <= 1024), summed over waves at the end
  for (long p0 = (long)blockIdx.x * NT; p0 < P; p0 += (long)gridDim.x * NT) {
    const long p = p0 + threadIdx.x;
    const bool ok = p < P;                    // every lane runs the wave reductions
    float dz[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dz[k] = 0.f;
    if (ok) {
      float z[K];
      pixel_logits<K>(x + p * C, ws, bs, C, z);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float t = target[p * K + k];
        const float sg = 1.f / (1.f + __expf(-z[k]));
        dz[k] = bce_w * (sg - t) * inv_n + dice_w * (ka * t + kb) * sg * (1.f - sg);
      }
    }
    for (int c = 0; c < C; c += 8) {
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, g[8];
      if (ok) unpack8(*reinterpret_cast<const uint4*>(x + p * C + c), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        g[e] = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) g[e] += dz[k] * ws[k * C + c + e];
      }
      if (ok) *reinterpret_cast<uint4*>(dx + p * C + c) = pack8(g);
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float r = wave_sum(f[e] * dz[k]);
          if (lane == 0) dws[wave][k * C + c + e] += r;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) dbias[k] += dz[k];
  }
  block_sum<K>(dbias, red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) atomicAdd(db + k, dbias[k]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < K * C; c += NT) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) s += dws[q][c];
    atomicAdd(dw + c, s);
  }
}

// Bilinear upsampling with align_corners=True (FPN's segmentation heads,
// `mlcomp/contrib/segmentation/fpn/decoder.py`), NHWC bf16, C % 8 == 0.  Source coordinate
// of output o: f = o * (In-1)/(Out-1) in fp32 as PyTorch computes it, i0 = floor(f),
// i1 = min(i0+1, In-1), weight f - i0 on i1.
struct Lerp { int i0, i1; float l; };
__device__ __forceinline__ Lerp lerp_at(int o, float scale, int in) {
  const float f = scale * (float)o;
  int i0 = (int)f;
  i0 = i0 < in - 1 ? i0 : in - 1;
  return Lerp{i0, i0 + (i0 < in - 1 ? 1 : 0), f - (float)i0};
}
__device__ __forceinline__ float lerp_w(const Lerp& a, int i) {
  return (a.i0 == i ? 1.f - a.l : 0.f) + (a.i1 == i ? a.l : 0.f);
}

__global__ void __launch_bounds__(NT)
bilinear_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C, int Ho, int Wo,
                    float sy, float sx) {
  const int cpr = C / 8;
  const long total = (long)N * Ho * Wo * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long p = i / cpr;
    const int ox = (int)(p % Wo);
    const long t = p / Wo;
    const int oy = (int)(t % Ho);
    const long n = t / Ho;
    const Lerp ly = lerp_at(oy, sy, H), lx = lerp_at(ox, sx, W);
    const bf16* b = x + n * H * W * (long)C + c8 * 8;
    float v00[8], v01[8], v10[8], v11[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ly.i0 * W + lx.i0) * C), v00);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ly.i0 * W + lx.i1) * C), v01);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ly.i1 * W + lx.i0) * C), v10);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ly.i1 * W + lx.i1) * C), v11);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      o[e] = (1.f - ly.l) * ((1.f - lx.l) * v00[e] + lx.l * v01[e]) + ly.l * ((1.f - lx.l) * v10[e] + lx.l * v11[e]);
    *reinterpret_cast<uint4*>(y + p * C + c8 * 8) = pack8(o);
  }
}

// first output whose floor(o * scale) reaches i (one below it to absorb fp32 rounding;
// outputs outside the exact range get weight 0 from lerp_w)
__device__ __forceinline__ int first_out(int i, int in, int out) {
  if (in <= 1 || i <= 0) return 0;
  const long num = (long)i * (out - 1);
  const int o = (int)((num + (in - 1) - 1) / (in - 1)) - 1;
  return o > 0 ? o : 0;
}

// gather form of the backward: input pixel (iy, ix) sums the outputs whose interpolation
// reads it (source index i0 or i1 equal to it) - no atomics, every dx written once
__global__ void __launch_bounds__(NT)
bilinear_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N, int H, int W, int C, int Ho, int Wo,
                    float sy, float sx) {
  const int cpr = C / 8;
  const long total = (long)N * H * W * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long p = i / cpr;
    const int ix = (int)(p % W);
    const long t = p / W;
    const int iy = (int)(t % H);
    const long n = t / H;
    const int oy0 = first_out(iy - 1, H, Ho), oy1 = iy + 1 >= H ? Ho : first_out(iy + 1, H, Ho) + 2;
    const int ox0 = first_out(ix - 1, W, Wo), ox1 = ix + 1 >= W ? Wo : first_out(ix + 1, W, Wo) + 2;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16* b = dy + n * Ho * Wo * (long)C + c8 * 8;
    for (int oy = oy0; oy < (oy1 < Ho ? oy1 : Ho); ++oy) {
      const float wy = lerp_w(lerp_at(oy, sy, H), iy);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox < (ox1 < Wo ? ox1 : Wo); ++ox) {
        const float w = wy * lerp_w(lerp_at(ox, sx, W), ix);
        if (w == 0.f) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(b + ((long)oy * Wo + ox) * C), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += w * f[e];
      }
    }
    *reinterpret_cast<uint4*>(dx + p * C + c8 * 8) = pack8(acc);
  }
}

// GroupNorm + ReLU over NHWC bf16 (FPN's segmentation heads, GroupNorm(32, 128)), C % 8 == 0
// and C/8 dividing 256.  Statistics are per (sample, channel) partial sums reduced per
// block and added with one atomic per channel; the per-group mean / rstd (and in the
// backward the per-group means of gamma*dy and gamma*dy*xhat) are combined from them on the
// fly by the elementwise passes, so each tensor is read once per pass.
constexpr int GN_ROWS = 256;   // pixel rows per block of the reduction passes

// MODE 0: st[n][c] += (sum x, sum x^2);  MODE 1: st[n][c] += (sum dym*xhat, sum dym) with
// dym = dz * [xhat*gamma + beta > 0] (ReLU mask recomputed), xhat from fst (forward stats)
template <int MODE>
__global__ void __launch_bounds__(NT)
gn_reduce_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dz, const float* __restrict__ fst,
                 const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ st, int HW,
                 int C, int G, float eps) {
  __shared__ float red[NT][17];
  const int cpr = C / 8, rg = NT / cpr, t = threadIdx.x;
  const int n = blockIdx.y, c8 = t % cpr, r0 = blockIdx.x * GN_ROWS + t / cpr;
  const int Cg = C / G;
  const float cnt = (float)HW * (float)Cg;
  float s1[8], s2[8], mu[8], rs[8], ga[8], be[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  if (MODE == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8 * 8 + e, g0 = (c / Cg) * Cg;
      float a = 0.f, b = 0.f;
      for (int k = 0; k < Cg; ++k) { a += fst[((long)n * C + g0 + k) * 2]; b += fst[((long)n * C + g0 + k) * 2 + 1]; }
      mu[e] = a / cnt;
      rs[e] = rsqrtf(fmaxf(b / cnt - mu[e] * mu[e], 0.f) + eps);
      ga[e] = gamma[c];
      be[e] = beta[c];
    }
  }
  const long base = (long)n * HW;
  const int rend = min(HW, (int)(blockIdx.x + 1) * GN_ROWS);
  for (int r = r0; r < rend; r += rg) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + (base + r) * C + c8 * 8), f);
    if (MODE == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] += f[e]; s2[e] += f[e] * f[e]; }
    } else {
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(dz + (base + r) * C + c8 * 8), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (f[e] - mu[e]) * rs[e];
        const float dm = xh * ga[e] + be[e] > 0.f ? d[e] : 0.f;
        s1[e] += dm * xh;
        s2[e] += dm;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[t][e] = s1[e]; red[t][8 + e] = s2[e]; }
  __syncthreads();
  // one thread per channel; C may exceed the block (up to 8 * NT channels), so loop
  for (int c = t; c < C; c += NT) {
    const int cc8 = c / 8, e = c % 8;
    float a = 0.f, b = 0.f;
    for (int j = 0; j < rg; ++j) { a += red[j * cpr + cc8][e]; b += red[j * cpr + cc8][8 + e]; }
    atomicAdd(st + ((long)n * C + c) * 2, a);
    atomicAdd(st + ((long)n * C + c) * 2 + 1, b);
  }
}

// MODE 0: z = relu(xhat*gamma + beta);  MODE 1: dx from dz and the backward sums bst
template <int MODE>
__global__ void __launch_bounds__(NT)
gn_apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dz, const float* __restrict__ fst,
                const float* __restrict__ bst, const float* __restrict__ gamma, const float* __restrict__ beta,
                bf16* __restrict__ out, int N, int HW, int C, int G, float eps) {
  const int cpr = C / 8, Cg = C / G;
  const float cnt = (float)HW * (float)Cg;
  const long total = (long)N * HW * cpr;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cpr);
    const long p = i / cpr;
    const int n = (int)(p / HW);
    float f[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(x + p * C + c8 * 8), f);
    float d[8];
    if (MODE == 1) unpack8(*reinterpret_cast<const uint4*>(dz + p * C + c8 * 8), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8 * 8 + e, g0 = (c / Cg) * Cg;
      float a = 0.f, b = 0.f, A = 0.f, B = 0.f;
      for (int k = 0; k < Cg; ++k) {
        const long q = ((long)n * C + g0 + k) * 2;
        a += fst[q];
        b += fst[q + 1];
        if (MODE == 1) { A += gamma[g0 + k] * bst[q]; B += gamma[g0 + k] * bst[q + 1]; }
      }
      const float mu = a / cnt, rs = rsqrtf(fmaxf(b / cnt - mu * mu, 0.f) + eps);
      const float xh = (f[e] - mu) * rs, y = xh * gamma[c] + beta[c];
      if (MODE == 0) {
        o[e] = fmaxf(y, 0.f);
      } else {
        const float dm = y > 0.f ? d[e] : 0.f;
        o[e] = rs * (gamma[c] * dm - B / cnt - xh * (A / cnt));
      }
    }
    *reinterpret_cast<uint4*>(out + p * C + c8 * 8) = pack8(o);
  }
}

inline int grid_for(long work) {
  long b = (work + NT - 1) / NT;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

}  // namespace

// out [N,2h,2w,C1+C2] = concat(upsample2x(lo [N,h,w,C1]), skip [N,2h,2w,C2]); C2 may be 0
MLC_EXPORT int mlc_upcat_fwd(const bf16* lo, const bf16* skip, bf16* out, int N, int h, int w, int C1, int C2,
                             hipStream_t st) {
  if (C1 % 8 || C2 % 8 || (C2 && !skip)) return -1;
  const long work = (long)N * 4 * h * w * ((C1 + C2) / 8);
  hipLaunchKernelGGL(upcat_fwd_kernel, dim3(grid_for(work)), dim3(NT), 0, st, lo, skip, out, N, h, w, C1, C2);
  return hipGetLastError();
}

MLC_EXPORT int mlc_upcat_bwd(const bf16* dout, bf16* dlo, bf16* dskip, int N, int h, int w, int C1, int C2,
                             hipStream_t st) {
  if (C1 % 8 || C2 % 8) return -1;
  hipLaunchKernelGGL(upcat_bwd_lo_kernel, dim3(grid_for((long)N * h * w * (C1 / 8))), dim3(NT), 0, st, dout, dlo, N,
                     h, w, C1, C1 + C2);
  if (C2 && dskip) {
    const long P = (long)N * 4 * h * w;
    hipLaunchKernelGGL(upcat_bwd_skip_kernel, dim3(grid_for(P * (C2 / 8))), dim3(NT), 0, st, dout, dskip, P, C1, C2);
  }
  return hipGetLastError();
}

// y [N,Ho,Wo,C] = bilinear upsampling (align_corners=True) of x [N,H,W,C]; C % 8 == 0
MLC_EXPORT int mlc_bilinear_up_fwd(const bf16* x, bf16* y, int N, int H, int W, int C, int Ho, int Wo,
                                   hipStream_t st) {
  if (C % 8 || H < 1 || W < 1 || Ho < 1 || Wo < 1) return -1;
  const float sy = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f, sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  hipLaunchKernelGGL(bilinear_fwd_kernel, dim3(grid_for((long)N * Ho * Wo * (C / 8))), dim3(NT), 0, st, x, y, N, H, W,
                     C, Ho, Wo, sy, sx);
  return hipGetLastError();
}

// dx [N,H,W,C] from dy [N,Ho,Wo,C] (gather, fp32 accumulate); C % 8 == 0
MLC_EXPORT int mlc_bilinear_up_bwd(const bf16* dy, bf16* dx, int N, int H, int W, int C, int Ho, int Wo,
                                   hipStream_t st) {
  if (C % 8 || H < 1 || W < 1 || Ho < 1 || Wo < 1) return -1;
  const float sy = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f, sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  hipLaunchKernelGGL(bilinear_bwd_kernel, dim3(grid_for((long)N * H * W * (C / 8))), dim3(NT), 0, st, dy, dx, N, H, W,
                     C, Ho, Wo, sy, sx);
  return hipGetLastError();
}

// GroupNorm + ReLU forward: z [N,HW,C] from x; fst [N][C][2] fp32 (zeroed by the caller)
// receives the per-channel sums the backward reuses.  C % 8 == 0, 256 % (C/8) == 0, G | C.
MLC_EXPORT int mlc_gn_relu_fwd(const bf16* x, const float* gamma, const float* beta, bf16* z, float* fst, int N,
                               int HW, int C, int G, float eps, hipStream_t st) {
  if (C % 8 || NT % (C / 8) || C % G || C > NT * 8) return -1;
  const dim3 rgrid((HW + GN_ROWS - 1) / GN_ROWS, N);
  hipLaunchKernelGGL(gn_reduce_kernel<0>, rgrid, dim3(NT), 0, st, x, nullptr, nullptr, nullptr, nullptr, fst, HW,
                     C, G, eps);
  hipLaunchKernelGGL(gn_apply_kernel<0>, dim3(grid_for((long)N * HW * (C / 8))), dim3(NT), 0, st, x, nullptr, fst,
                     nullptr, gamma, beta, z, N, HW, C, G, eps);
  return hipGetLastError();
}

// backward: dx from dz (ReLU mask recomputed), bst [N][C][2] fp32 scratch (zeroed by the
// caller) = per-channel (sum dym*xhat, sum dym): dgamma / dbeta are its sums over n
MLC_EXPORT int mlc_gn_relu_bwd(const bf16* x, const bf16* dz, const float* gamma, const float* beta,
                               const float* fst, float* bst, bf16* dx, int N, int HW, int C, int G, float eps,
                               hipStream_t st) {
  if (C % 8 || NT % (C / 8) || C % G || C > NT * 8) return -1;
  const dim3 rgrid((HW + GN_ROWS - 1) / GN_ROWS, N);
  hipLaunchKernelGGL(gn_reduce_kernel<1>, rgrid, dim3(NT), 0, st, x, dz, fst, gamma, beta, bst, HW, C, G, eps);
  hipLaunchKernelGGL(gn_apply_kernel<1>, dim3(grid_for((long)N * HW * (C / 8))), dim3(NT), 0, st, x, dz, fst, bst,
                     gamma, beta, dx, N, HW, C, G, eps);
  return hipGetLastError();
}

// x [P][C] bf16 (C % 8 == 0, C <= 256), w [K][C], bias [K], target [P][K] fp32 in {0,1}
// (soft ok); logits [P][K] fp32 (optional); sums [4] fp32 zeroed by the caller.  K <= 4.
#define SEG_K_DISPATCH(KERNEL, ...)                                                                       \
  switch (K) {                                                                                          \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                                          \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                                          \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                                          \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                                          \
    default: return -1;                                                                                 \
  }
MLC_EXPORT int mlc_seg_head_fwd(const bf16* x, const float* w, const float* bias, const float* target, float* logits,
                                float* sums, long P, int C, int K, hipStream_t st) {
  if (C % 8 || C > 256 || K < 1 || K > 4) return -1;
  const int grid = grid_for(P) < 2048 ? grid_for(P) : 2048;
  SEG_K_DISPATCH(seg_head_fwd_kernel, dim3(grid), dim3(NT), 0, st, x, w, bias, target, logits, sums, P, C);
  return hipGetLastError();
}

// dx [P][C] bf16 written; dw [K][C] / db [K] accumulated (+=)
MLC_EXPORT int mlc_seg_head_bwd(const bf16* x, const float* w, const float* bias, const float* target,
                                const float* sums, bf16* dx, float* dw, float* db, long P, int C, int K, float bce_w,
                                float dice_w, float eps, hipStream_t st) {
  if (C % 8 || C > 256 || K < 1 || K > 4) return -1;
  const int grid = grid_for(P) < 2048 ? grid_for(P) : 2048;
  SEG_K_DISPATCH(seg_head_bwd_kernel, dim3(grid), dim3(NT), 0, st, x, w, bias, target, sums, dx, dw, db, P, C, bce_w,
                 dice_w, eps);
  return hipGetLastError();
}
