// ResNet stem tail fused: BatchNorm-apply + ReLU + 3x3/2 max-pool (forward) and
// max-pool backward + ReLU mask + BatchNorm backward (two passes).
//
// The stem's post-BN activation z = relu(y*scale + shift) [N,112,112,64] is consumed only
// by the max-pool, so it is never written: the forward reads the conv output y once and
// writes the pooled tensor (4x smaller) and the window argmax.  The backward recomputes the
// pooled-gradient scatter dU (a gather of at most 2x2 windows per input pixel) in both
// passes instead of storing it: pass 1 reduces sum dU and sum dU*(y-mean) per channel,
// pass 2 writes dy = k1*dU + k2 + k3*(y-mean).  Compared with separate BN-apply, max-pool,
// max-pool-backward, BN-reduce and BN-apply passes this moves ~2.3 GB less per ResNet-50
// step at batch 256.
//
// The argmax byte is 255 when the window maximum of y*scale+shift is <= 0: the ReLU
// zeroed the pooled value, so no gradient flows (same as ReLU-then-pool in the reference
// graph, torchvision resnet: conv1 -> bn1 -> relu -> maxpool).
//
// Layout: NHWC bf16, C/8 channel groups of 16 B per lane.  A block owns ROWS consecutive
// rows of one image plane; thread t keeps channel group t % G for the whole block
// (G | 256), so per-channel constants stay in registers and no index division is needed.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int NSTAT = 32;   // == batchnorm.hip NSTAT (partial-sum copies)
constexpr unsigned char NOGRAD = 255;

__device__ __forceinline__ uint4 ld16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }

// pooled[n,ho,wo,c] = max(0, max_{3x3 window} y*scale+shift), idx = argmax tap or 255
__global__ void __launch_bounds__(NT)
stem_pool_fwd_kernel(const bf16* __restrict__ y, const float* __restrict__ scale,
                     const float* __restrict__ shift, bf16* __restrict__ out,
                     uint8_t* __restrict__ idx, bf16* __restrict__ ymax, int H, int W, int C, int Ho, int Wo,
                     int rows_total, int ROWS, int gshift) {
  const int G = C >> 3;
  const int cg = threadIdx.x & (G - 1);
  const int c0 = cg * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j]; }
  const int per_row = Wo << gshift;
  // rows x (pixels, groups) flattened so every lane has work (ROWS*per_row % 256 == 0 on
  // the ResNet shapes); it % G stays equal to threadIdx.x % G because G | 256
  for (int it = threadIdx.x; it < ROWS * per_row; it += NT) {
    const int rr = it / per_row;
    const int row = blockIdx.x * ROWS + rr;         // n*Ho + ho
    if (row >= rows_total) break;
    const int wo = (it - rr * per_row) >> gshift;
    const int n = row / Ho, ho = row - n * Ho;
    {
      const int h0 = 2 * ho - 1;
      const int w0 = 2 * wo - 1;
      float best[8], bv[8];
      int arg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; bv[j] = 0.f; }
      // branch-free: the 9 taps load from clamped (always valid) addresses, all in flight
      // at once; taps outside the image are masked out of the max
      uint4 v[3][3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int h = min(max(h0 + kh, 0), H - 1);
        const bf16* rowp = y + ((size_t)n * H + h) * W * C + c0;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) v[kh][kw] = ld16(rowp + (size_t)min(max(w0 + kw, 0), W - 1) * C);
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const bool hok = (unsigned)(h0 + kh) < (unsigned)H;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const bool ok = hok && (unsigned)(w0 + kw) < (unsigned)W;
          float f[8];
          unpack8(v[kh][kw], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = ok ? f[j] * sc[j] + sh[j] : -INFINITY;
            if (a > best[j]) { best[j] = a; arg[j] = kh * 3 + kw; bv[j] = f[j]; }
          }
        }
      }
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t a = best[j] > 0.f ? (uint32_t)arg[j] : (uint32_t)NOGRAD;
        best[j] = fmaxf(best[j], 0.f);
        if (j < 4) lo |= a << (8 * j); else hi |= a << (8 * (j - 4));
      }
      const size_t o = ((size_t)row * Wo + wo) * C + c0;
      *reinterpret_cast<uint4*>(out + o) = pack8(best);
      *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
      // the pre-BN value at the argmax: the backward's reduction runs over the pooled tensor
      // (exact: y is bf16, so is this copy)
      if (ymax) *reinterpret_cast<uint4*>(ymax + o) = pack8(bv);
    }
  }
}

// dU at input pixel (n,h,w), channels c0..c0+7: the pooled gradients of the (at most
// 2x2) windows that cover it and chose it.  For 3x3/2 pad 1: an even h is tap 1 of window
// h/2; an odd h is tap 2 of window (h-1)/2 and tap 0 of window (h+1)/2.
__device__ __forceinline__ void gather_du(const bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                                          int n, int h, int w, int c0, int C, int Ho, int Wo,
                                          float (&d)[8]) {
  // candidate windows: rows (ha, kha) and (hb, khb), cols likewise; the second candidate
  // exists only for odd coordinates inside the pooled extent.  All four (row, col) loads
  // are issued unconditionally from clamped addresses (no branches around loads, so they
  // are all in flight together) and invalid ones are masked by an impossible tap.
  const bool hodd = h & 1, wodd = w & 1;
  const int ha = h >> 1, kha = hodd ? 2 : 1;
  const int hb = min((h >> 1) + 1, Ho - 1), khb = 0;
  const bool hbok = hodd && (h >> 1) + 1 < Ho;
  const int wa = w >> 1, kwa = wodd ? 2 : 1;
  const int wb = min((w >> 1) + 1, Wo - 1), kwb = 0;
  const bool wbok = wodd && (w >> 1) + 1 < Wo;
  const size_t ra = ((size_t)n * Ho + ha) * Wo, rb = ((size_t)n * Ho + hb) * Wo;
  const size_t o[4] = {(ra + wa) * C + c0, (ra + wb) * C + c0, (rb + wa) * C + c0, (rb + wb) * C + c0};
  const uint32_t pos[4] = {(uint32_t)(kha * 3 + kwa), wbok ? (uint32_t)(kha * 3 + kwb) : 99u,
                           hbok ? (uint32_t)(khb * 3 + kwa) : 99u,
                           (hbok && wbok) ? (uint32_t)(khb * 3 + kwb) : 99u};
  // loads through ext-vector types: with HIP's uint2/uint4 structs hipcc serialised
  // these loads (vmcnt(0) after each) in the reduce variant of the kernel below
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x2 av[4];
  u32x4 gw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    av[q] = *reinterpret_cast<const u32x2*>(idx + o[q]);
    gw[q] = *reinterpret_cast<const u32x4*>(dp + o[q]);
  }
  uint2 ai[4];
  uint4 gv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ai[q] = make_uint2(av[q].x, av[q].y);
    gv[q] = make_uint4(gw[q].x, gw[q].y, gw[q].z, gw[q].w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float g[8];
    unpack8(gv[q], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t word = j < 4 ? ai[q].x : ai[q].y;
      d[j] += (((word >> (8 * (j & 3))) & 0xffu) == pos[q]) ? g[j] : 0.f;
    }
  }
}

// APPLY = false: sums[blockIdx % NSTAT][0/1][c] += sum dU, sum dU*(y-mean)
// APPLY = true : dy = k1*dU + k2 + k3*(y-mean) with coef = [k1 | k2 | k3]
template <bool APPLY>
__global__ void __launch_bounds__(NT)
stem_pool_bwd_kernel(const bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                     const bf16* __restrict__ y, const float* __restrict__ mean,
                     const float* __restrict__ coef, float* __restrict__ sums, bf16* __restrict__ dy,
                     int H, int W, int C, int Ho, int Wo, int rows_total, int ROWS,
                     int gshift, int ncopy) {
  const int G = C >> 3;
  const int cg = threadIdx.x & (G - 1);
  const int c0 = cg * 8;
  float mu[8], k1[8], k2[8], k3[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j];
    s1[j] = 0.f; s2[j] = 0.f;
    if (APPLY) { k1[j] = coef[c0 + j]; k2[j] = coef[C + c0 + j]; k3[j] = coef[2 * C + c0 + j]; }
  }
  const int per_row = W << gshift;
  for (int it = threadIdx.x; it < ROWS * per_row; it += NT) {
    const int rr = it / per_row;
    const int row = blockIdx.x * ROWS + rr;         // n*H + h
    if (row >= rows_total) break;
    const int w = (it - rr * per_row) >> gshift;
    const int n = row / H, h = row - n * H;
    {
      float d[8], yy[8];
      const size_t o = ((size_t)row * W + w) * C + c0;
      unpack8(ld16(y + o), yy);
      gather_du(dp, idx, n, h, w, c0, C, Ho, Wo, d);
      if (APPLY) {
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = k1[j] * d[j] + k2[j] + k3[j] * (yy[j] - mu[j]);
        *reinterpret_cast<uint4*>(dy + o) = pack8(r);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += d[j]; s2[j] += d[j] * (yy[j] - mu[j]); }
      }
    }
  }
  if (APPLY) return;
  // threads t, t+G, t+2G, ... own the same channel group: shuffle within the wave, then
  // one LDS slot per (wave, group)
  __shared__ float red[NT / 64][64][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int o = G; o < 64; o <<= 1) {
      s1[j] += __shfl_xor(s1[j], o, 64);
      s2[j] += __shfl_xor(s2[j], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[wave][lane][j] = s1[j]; red[wave][lane][8 + j] = s2[j]; }
  }
  __syncthreads();
  // G <= 64 here (checked by the launcher): threads < G*16 each finish one (group, value)
  if (threadIdx.x < G * 16) {
    const int g = threadIdx.x >> 4, v = threadIdx.x & 15;
    float acc = 0.f;
#pragma unroll
    for (int wv = 0; wv < NT / 64; ++wv) acc += red[wv][g][v];
    float* dst = sums + (size_t)(blockIdx.x % ncopy) * 2 * C;
    atomicAdd(dst + (v < 8 ? 0 : C) + g * 8 + (v & 7), acc);
  }
}

// ---------------------------------------------------------------- space-to-depth stem input
// The 7x7/2 pad-3 stem conv over 3 channels is run as a 4x4/1 conv over the 2x2
// space-to-depth image: out[n,ho,wo] = sum_{r,s<4} X2[n,ho+r,wo+s,:] . W2[:,r,s,:] with
//   X2[n,i,j,(dy*2+dx)*3+ci] = x[n, 2i+dy-pad, 2j+dx-pad, ci]   (zero outside the image)
// and W2 the 7x7 filter zero-extended to 8x8 and regrouped the same way (models/
// native_resnet.py).  Channels 12..15 are zero so every pixel is two 16-byte chunks: the
// implicit-GEMM loaders see C = 16 and K = 4*4*16 = 256 (4 K-tiles) instead of the 7x7x8 =
// 392 (7 K-tiles, 62% padding) of the direct form.
__global__ void __launch_bounds__(NT)
stem_s2d_kernel(const bf16* __restrict__ x, bf16* __restrict__ out, int N, int H, int W, int Cs,
                int Hb, int Wb, int pad) {
  const bool vec = (Cs % 8) == 0;
  const long total = (long)N * Hb * Wb;
  for (long p = (long)blockIdx.x * NT + threadIdx.x; p < total; p += (long)gridDim.x * NT) {
    const int j = (int)(p % Wb);
    const long t = p / Wb;
    const int i = (int)(t % Hb);
    const int n = (int)(t / Hb);
    float v[16];
#pragma unroll
    for (int q = 12; q < 16; ++q) v[q] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int h = 2 * i + dy - pad, w = 2 * j + dx - pad;
        const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        const bf16* src = x + (((size_t)n * H + (ok ? h : 0)) * W + (ok ? w : 0)) * Cs;
        float f[8];
        if (vec) {   // 16-byte pixel rows (channels padded to 8): one vector load
          typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 u = *reinterpret_cast<const u32x4*>(src);
          unpack8(make_uint4(u.x, u.y, u.z, u.w), f);
        } else {
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) f[ci] = (float)src[ci];
        }
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) v[(dy * 2 + dx) * 3 + ci] = ok ? f[ci] : 0.f;
      }
    }
    uint4* dst = reinterpret_cast<uint4*>(out + p * 16);
    dst[0] = pack8(v);
    dst[1] = pack8(v + 8);
  }
}


constexpr int ROWS_PER_BLOCK = 4;

// The backward's reduction from the pooled side: sum dU = sum over pooled outputs of dp
// (ReLU-active windows), sum dU*(y-mean) = sum of dp*(ymax-mean) (an input pixel chosen by
// several windows gets each window's gradient: the same sums as over the scattered dU).  Reads
// dp, idx and ymax (4x smaller than y) instead of y plus a 2x2 window gather per input pixel.
__global__ void __launch_bounds__(NT)
stem_pool_reduce_pooled_kernel(const bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                               const bf16* __restrict__ ymax, const float* __restrict__ mean,
                               float* __restrict__ sums, int C, long total_groups, int ncopy) {
  const int G = C >> 3;
  const int cg = threadIdx.x & (G - 1);    // constant per thread: G | 256, stride NT*gridDim
  const int c0 = cg * 8;
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; s1[j] = 0.f; s2[j] = 0.f; }
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total_groups; i += (long)gridDim.x * NT) {
    const size_t o = (size_t)i * 8;
    float g[8], v[8];
    unpack8(ld16(dp + o), g);
    unpack8(ld16(ymax + o), v);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 a = *reinterpret_cast<const u32x2*>(idx + o);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t word = j < 4 ? a.x : a.y;
      const bool on = ((word >> (8 * (j & 3))) & 0xffu) != NOGRAD;
      const float d = on ? g[j] : 0.f;
      s1[j] += d;
      s2[j] += d * (v[j] - mu[j]);
    }
  }
  __shared__ float red[NT / 64][64][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int o = G; o < 64; o <<= 1) {
      s1[j] += __shfl_xor(s1[j], o, 64);
      s2[j] += __shfl_xor(s2[j], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[wave][lane][j] = s1[j]; red[wave][lane][8 + j] = s2[j]; }
  }
  __syncthreads();
  if (threadIdx.x < G * 16) {
    const int g = threadIdx.x >> 4, v = threadIdx.x & 15;
    float acc = 0.f;
#pragma unroll
    for (int wv = 0; wv < NT / 64; ++wv) acc += red[wv][g][v];
    float* dst = sums + (size_t)(blockIdx.x % ncopy) * 2 * C;
    atomicAdd(dst + (v < 8 ? 0 : C) + g * 8 + (v & 7), acc);
  }
}

bool shape_ok(int C) {   // G = C/8 a power of two <= 64 (one wave covers every group)
  const int G = C >> 3;
  return C % 8 == 0 && G >= 1 && G <= 64 && (G & (G - 1)) == 0;
}

}  // namespace

MLC_EXPORT int mlc_stem_pool_fwd(const bf16* y, const float* scale, const float* shift, bf16* out,
                                 uint8_t* idx, bf16* ymax, int N, int H, int W, int C, hipStream_t st) {
  if (!shape_ok(C)) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;   // 3x3, stride 2, pad 1
  const int rows = N * Ho;
  const int blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  hipLaunchKernelGGL(stem_pool_fwd_kernel, dim3(blocks), dim3(NT), 0, st, y, scale, shift, out, idx, ymax,
                     H, W, C, Ho, Wo, rows, ROWS_PER_BLOCK, __builtin_ctz(C >> 3));
  return hipGetLastError();
}

// sums: NSTAT*2*C fp32, zeroed by the caller (the per-step workspace memset)
MLC_EXPORT int mlc_stem_pool_bwd_reduce(const bf16* dp, const uint8_t* idx, const bf16* y,
                                        const float* mean, float* sums, int N, int H, int W, int C,
                                        hipStream_t st) {
  if (!shape_ok(C)) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int rows = N * H;
  const int blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  if (g_mlc_det && blocks > g_mlc_ncopy) return -2;
  hipLaunchKernelGGL(stem_pool_bwd_kernel<false>, dim3(blocks), dim3(NT), 0, st, dp, idx, y, mean,
                     nullptr, sums, nullptr, H, W, C, Ho, Wo, rows, ROWS_PER_BLOCK, __builtin_ctz(C >> 3),
                     g_mlc_ncopy);
  return hipGetLastError();
}

// the same sums from the pooled side (ymax from mlc_stem_pool_fwd)
MLC_EXPORT int mlc_stem_pool_bwd_reduce_pooled(const bf16* dp, const uint8_t* idx, const bf16* ymax,
                                               const float* mean, float* sums, int N, int H, int W, int C,
                                               hipStream_t st) {
  if (!shape_ok(C)) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long groups = (long)N * Ho * Wo * (C / 8);
  long blocks = (groups + NT - 1) / NT;
  if (blocks > 1024) blocks = 1024;
  if (g_mlc_det && blocks > g_mlc_ncopy) return -2;
  hipLaunchKernelGGL(stem_pool_reduce_pooled_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, dp, idx, ymax, mean,
                     sums, C, groups, g_mlc_ncopy);
  return hipGetLastError();
}

MLC_EXPORT int mlc_stem_pool_bwd_apply(const bf16* dp, const uint8_t* idx, const bf16* y,
                                       const float* mean, const float* coef, bf16* dy, int N, int H,
                                       int W, int C, hipStream_t st) {
  if (!shape_ok(C)) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int rows = N * H;
  const int blocks = (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  hipLaunchKernelGGL(stem_pool_bwd_kernel<true>, dim3(blocks), dim3(NT), 0, st, dp, idx, y, mean, coef,
                     nullptr, dy, H, W, C, Ho, Wo, rows, ROWS_PER_BLOCK, __builtin_ctz(C >> 3), g_mlc_ncopy);
  return hipGetLastError();
}

MLC_EXPORT int mlc_stem_s2d(const bf16* x, bf16* out, int N, int H, int W, int Cs, int pad,
                            hipStream_t st) {
  if (Cs < 3 || ((H + 2 * pad) & 1) || ((W + 2 * pad) & 1)) return -1;
  const int Hb = (H + 2 * pad) / 2, Wb = (W + 2 * pad) / 2;
  const long total = (long)N * Hb * Wb;
  long blocks = (total + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(stem_s2d_kernel, dim3((int)blocks), dim3(NT), 0, st, x, out, N, H, W, Cs, Hb, Wb, pad);
  return hipGetLastError();
}
