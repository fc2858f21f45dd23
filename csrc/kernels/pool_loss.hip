// NHWC pooling, softmax cross-entropy, and small layout/cast kernels.
#include "common.h"

namespace {
constexpr int NT = 256;
}

// ------------------------------------------------------------------ max pool
// y[n,ho,wo,c] = max over window; idx (uint8) = argmax window position (kh*KW+kw).
// One thread per (output pixel, 8-channel group); 16 B loads.
__global__ void __launch_bounds__(NT)
maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, uint8_t* __restrict__ idx,
                   int N, int H, int W, int C, int Ho, int Wo, int K, int S, int P) {
  const int G = C >> 3;
  const long total = (long)N * Ho * Wo * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cg = (int)(i % G);
    long t = i / G;
    const int wo = (int)(t % Wo); t /= Wo;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    float best[8]; int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
    for (int kh = 0; kh < K; ++kh) {
      const int hi = ho * S - P + kh;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int wi = wo * S - P + kw;
        if ((unsigned)wi >= (unsigned)W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * H + hi) * W + wi) * C + cg * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j]) { best[j] = f[j]; arg[j] = kh * K + kw; }
      }
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + i * 8) = a;
  }
}

// dx[n,hi,wi,c] = sum over output windows containing (hi,wi) whose argmax is it
__global__ void __launch_bounds__(NT)
maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx, bf16* __restrict__ dx,
                   int N, int H, int W, int C, int Ho, int Wo, int K, int S, int P) {
  const int G = C >> 3;
  const long total = (long)N * H * W * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cg = (int)(i % G);
    long t = i / G;
    const int wi = (int)(t % W); t /= W;
    const int hi = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // output rows whose window covers hi: ho*S - P <= hi <= ho*S - P + K - 1
    const int ho_lo = max(0, (hi + P - K + S) / S), ho_hi = min(Ho - 1, (hi + P) / S);
    const int wo_lo = max(0, (wi + P - K + S) / S), wo_hi = min(Wo - 1, (wi + P) / S);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = hi - (ho * S - P);
      if (kh < 0 || kh >= K) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = wi - (wo * S - P);
        if (kw < 0 || kw >= K) continue;
        const long o = (((long)n * Ho + ho) * Wo + wo) * C + cg * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), g);
        const int pos = kh * K + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t w = j < 4 ? a.x : a.y;
          if ((int)((w >> (8 * (j & 3))) & 0xff) == pos) acc[j] += g[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// ------------------------------------------------------------------ global avg pool
// y[n,c] = mean_hw x[n,hw,c]   (one block per (n, 2048-channel slab), threads over c8 x hw)
__global__ void __launch_bounds__(NT)
avgpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int HW, int C) {
  const int n = blockIdx.x;
  const int G = C >> 3;
  __shared__ float part[NT][8];
  // threads: cg = t % G, hw-lane = t / G
  const int t = threadIdx.x;
  const int lanes = G >= NT ? 1 : NT / G;
  for (int cgb = 0; cgb < G; cgb += NT) {
    const int cg = cgb + (G >= NT ? t : t % G);
    const int hl = G >= NT ? 0 : t / G;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (cg < G)
      for (int hw = hl; hw < HW; hw += lanes) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + ((long)n * HW + hw) * C + cg * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[t][j] = acc[j];
    __syncthreads();
    if (hl == 0 && cg < G) {
      for (int u = 1; u < lanes; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += part[t + u * G][j];
      const float inv = 1.f / (float)HW;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
      *reinterpret_cast<uint4*>(y + (long)n * C + cg * 8) = pack8(acc);
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(NT)
avgpool_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ add, bf16* __restrict__ dx, int N, int HW,
                   int C) {
  const int G = C >> 3;
  const long total = (long)N * HW * G;
  const float inv = 1.f / (float)HW;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int cg = (int)(i % G);
    const long n = i / G / HW;
    const uint4 av = add ? ldg16(add + i * 8) : make_uint4(0u, 0u, 0u, 0u);
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + n * C + cg * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= inv;
    if (add) {                          // the other consumers' gradient of x (GradAcc)
      float q[8];
      unpack8(av, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += q[j];
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(f);
  }
}

// ------------------------------------------------------------------ softmax CE
// One block per row.  logits fp32 [B][V]; loss_sum += sum_rows (lse - x[y]) (atomic),
// dlogits (bf16) = (softmax - onehot) * scale; correct += (argmax == y).
// Optional label smoothing eps: target = (1-eps)*onehot + eps/V.
__global__ void __launch_bounds__(NT)
softmax_ce_kernel(const float* __restrict__ logits, const long* __restrict__ labels,
                  bf16* __restrict__ dlogits, float* __restrict__ loss_sum, float* __restrict__ correct,
                  int V, int ld, float scale, float smoothing) {
  const int row = blockIdx.x;
  const float* x = logits + (long)row * ld;
  __shared__ float sm[NT / 64], si[NT / 64];
  __shared__ int sarg[NT / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  float mx = -INFINITY; int am = 0;
  for (int i = t; i < V; i += NT) if (x[i] > mx) { mx = x[i]; am = i; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64); const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  if (lane == 0) { sm[w] = mx; sarg[w] = am; }
  __syncthreads();
  mx = sm[0]; am = sarg[0];
  for (int k = 1; k < NT / 64; ++k) if (sm[k] > mx || (sm[k] == mx && sarg[k] < am)) { mx = sm[k]; am = sarg[k]; }
  float s = 0.f, sx = 0.f;
  for (int i = t; i < V; i += NT) { s += __expf(x[i] - mx); sx += x[i]; }
  s = wave_sum(s); sx = wave_sum(sx);
  __syncthreads();
  if (lane == 0) { sm[w] = s; si[w] = sx; }
  __syncthreads();
  s = 0.f; sx = 0.f;
  for (int k = 0; k < NT / 64; ++k) { s += sm[k]; sx += si[k]; }
  const float lse = mx + __logf(s);
  const long y = labels[row];
  if (t == 0) {
    const float nll = lse - x[y];
    const float smooth = lse - sx / (float)V;
    atomicAdd(loss_sum, (1.f - smoothing) * nll + smoothing * smooth);
    if (correct) atomicAdd(correct, am == y ? 1.f : 0.f);
  }
  if (dlogits) {
    const float inv_s = 1.f / s;
    for (int i = t; i < ld; i += NT) {
      float g = 0.f;  // padded columns [V, ld) get zero gradient
      if (i < V) {
        const float p = __expf(x[i] - mx) * inv_s;
        const float tgt = (i == y ? (1.f - smoothing) : 0.f) + smoothing / (float)V;
        g = (p - tgt) * scale;
      }
      dlogits[(long)row * ld + i] = (bf16)g;
    }
  }
}

// column sums of a bf16 [R][C] matrix into fp32 out[C] (bias gradients)
__global__ void __launch_bounds__(NT)
colsum_kernel(const bf16* __restrict__ g, float* __restrict__ out, int R, int C) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += (float)g[(long)r * C + c];
  out[c] = s;
}

// ------------------------------------------------------------------ layout / cast
// NCHW fp32 (or bf16 flag) -> NHWC bf16 with channel padding to Cp (zeros)
__global__ void __launch_bounds__(NT)
nchw_to_nhwc_kernel(const float* __restrict__ x, bf16* __restrict__ y, int N, int C, int HW, int Cp) {
  const long total = (long)N * HW * Cp;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c = (int)(i % Cp);
    const long t = i / Cp;
    const int hw = (int)(t % HW);
    const long n = t / HW;
    y[i] = c < C ? (bf16)x[(n * C + c) * HW + hw] : (bf16)0.f;
  }
}

// fp32 -> bf16 cast (n % 8 == 0 fast path)
__global__ void __launch_bounds__(NT)
cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n8) {
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

// ------------------------------------------------------------------ windowed average pool
// y[n,ho,wo,c] = sum over the KxK/S window (pad P) / div, div = K*K (count_include_pad) or the
// number of in-image taps; one thread per (output pixel, 8-channel group), fp32 sums.  The
// backward gathers, per input pixel, the (at most ceil(K/S)^2) windows that cover it.  Inception's
// 3x3/1 branch pools (the stock NHWC avg_pool2d backward ran ~260 us per call at batch 80).
__device__ __forceinline__ int ap_div(int ho, int wo, int H, int W, int K, int S, int P, int cip) {
  if (cip) return K * K;
  const int h0 = ho * S - P, w0 = wo * S - P;
  const int nh = min(h0 + K, H) - max(h0, 0), nw = min(w0 + K, W) - max(w0, 0);
  return nh * nw;
}

__global__ void __launch_bounds__(NT)
avgpool2d_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C, int Ho,
                     int Wo, int K, int S, int P, int cip) {
  const int G = C / 8;
  const long total = (long)N * Ho * Wo * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int g = (int)(i % G);
    long t = i / G;
    const int wo = (int)(t % Wo);
    t /= Wo;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < K; ++kh) {
      const int h = ho * S - P + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int w = wo * S - P + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        float f[8];
        unpack8(ldg16(x + (((long)n * H + h) * W + w) * C + g * 8), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
      }
    }
    const float inv = 1.f / (float)ap_div(ho, wo, H, W, K, S, P, cip);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(acc);
  }
}

__global__ void __launch_bounds__(NT)
avgpool2d_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ add, bf16* __restrict__ dx, int N, int H,
                     int W, int C, int Ho, int Wo, int K, int S, int P, int cip) {
  const int G = C / 8;
  const long total = (long)N * H * W * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int g = (int)(i % G);
    long t = i / G;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    // windows ho with ho*S - P <= h <= ho*S - P + K - 1
    const int ho_lo = max(0, (h + P - K + S) / S), ho_hi = min(Ho - 1, (h + P) / S);
    const int wo_lo = max(0, (w + P - K + S) / S), wo_hi = min(Wo - 1, (w + P) / S);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (add) unpack8(ldg16(add + i * 8), acc);      // another consumer's gradient of x
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      if (h + P - ho * S >= K || h + P - ho * S < 0) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        if (w + P - wo * S >= K || w + P - wo * S < 0) continue;
        float f[8];
        unpack8(ldg16(dy + (((long)n * Ho + ho) * Wo + wo) * C + g * 8), f);
        const float inv = 1.f / (float)ap_div(ho, wo, H, W, K, S, P, cip);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e] * inv;
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// adaptive_avg_pool2d(x, (Ho, Wo)) with PyTorch's bins: output row o averages input rows
// [floor(o*H/Ho), ceil((o+1)*H/Ho)) (bins overlap when Ho does not divide H); fp32 sums,
// one bf16 rounding (PSPNet's 1/2/3/6 pyramid).  Backward: a gather over the bins that
// contain the input element (no atomics).
__device__ __forceinline__ int abin_lo(int o, int in, int out) { return (int)(((long)o * in) / out); }
__device__ __forceinline__ int abin_hi(int o, int in, int out) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// one block per output bin (n, oh, ow): threads split the bin's pixels (lanes) and the 8-channel
// groups, fp32 partial sums combined in LDS (the layout of avgpool_fwd_kernel) - a thread per
// output chunk summing a whole bin serially left a 1x1 / 2x2 pyramid level with a few thousand
// threads on a few CUs
__global__ void __launch_bounds__(NT)
adaptive_avg_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C, int Ho,
                        int Wo) {
  __shared__ float part[NT][8];
  const int bin = blockIdx.x;
  const int ow = bin % Wo, oh = (bin / Wo) % Ho, n = bin / (Wo * Ho);
  const int h0 = abin_lo(oh, H, Ho), h1 = abin_hi(oh, H, Ho);
  const int w0 = abin_lo(ow, W, Wo), w1 = abin_hi(ow, W, Wo);
  const int bw = w1 - w0, area = (h1 - h0) * bw;
  const float inv = 1.f / (float)area;
  const int G = C >> 3, t = threadIdx.x;
  const int lanes = G >= NT ? 1 : NT / G;
  for (int cgb = 0; cgb < G; cgb += NT) {
    const int cg = cgb + (G >= NT ? t : t % G);
    const int pl = G >= NT ? 0 : t / G;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (cg < G && pl < lanes)
      for (int p = pl; p < area; p += lanes) {
        const int h = h0 + p / bw, w = w0 + p % bw;
        float f[8];
        unpack8(ldg16(x + (((long)n * H + h) * W + w) * C + cg * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[t][j] = acc[j];
    __syncthreads();
    if (pl == 0 && cg < G) {
      for (int u = 1; u < lanes; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += part[t + u * G][j];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
      *reinterpret_cast<uint4*>(y + ((long)bin * C) + cg * 8) = pack8(acc);
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(NT)
adaptive_avg_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                        int Wo) {
  const int G = C / 8;
  const long total = (long)N * H * W * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int g = (int)(i % G);
    long t = i / G;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    // bins o with lo(o) <= h < hi(o): o in [floor(h*Ho/H), ceil((h+1)*Ho/H) - 1], each checked
    const int ho_a = max(0, (int)(((long)h * Ho) / H) - 1), ho_b = min(Ho - 1, (int)(((long)(h + 1) * Ho) / H) + 1);
    const int wo_a = max(0, (int)(((long)w * Wo) / W) - 1), wo_b = min(Wo - 1, (int)(((long)(w + 1) * Wo) / W) + 1);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ho = ho_a; ho <= ho_b; ++ho) {
      const int h0 = abin_lo(ho, H, Ho), h1 = abin_hi(ho, H, Ho);
      if (h < h0 || h >= h1) continue;
      for (int wo = wo_a; wo <= wo_b; ++wo) {
        const int w0 = abin_lo(wo, W, Wo), w1 = abin_hi(wo, W, Wo);
        if (w < w0 || w >= w1) continue;
        float f[8];
        unpack8(ldg16(dy + (((long)n * Ho + ho) * Wo + wo) * C + g * 8), f);
        const float inv = 1.f / (float)((h1 - h0) * (w1 - w0));
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e] * inv;
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

static int blocks_for(long work) {
  long b = (work + NT - 1) / NT;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

MLC_EXPORT int mlc_maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C,
                               int Ho, int Wo, int K, int S, int P, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(blocks_for((long)N * Ho * Wo * (C / 8))), dim3(NT), 0,
                     st, x, y, idx, N, H, W, C, Ho, Wo, K, S, P);
  return hipGetLastError();
}

MLC_EXPORT int mlc_maxpool_bwd(const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W,
                               int C, int Ho, int Wo, int K, int S, int P, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(blocks_for((long)N * H * W * (C / 8))), dim3(NT), 0,
                     st, dy, idx, dx, N, H, W, C, Ho, Wo, K, S, P);
  return hipGetLastError();
}

MLC_EXPORT int mlc_avgpool_fwd(const bf16* x, bf16* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(N), dim3(NT), 0, st, x, y, HW, C);
  return hipGetLastError();
}

MLC_EXPORT int mlc_avgpool_bwd(const bf16* dy, const bf16* add, bf16* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(blocks_for((long)N * HW * (C / 8))), dim3(NT), 0, st,
                     dy, add, dx, N, HW, C);
  return hipGetLastError();
}

// logits/dlogits rows have stride ld >= V (columns [V, ld) are padding)
MLC_EXPORT int mlc_softmax_ce(const float* logits, const long* labels, bf16* dlogits, float* loss_sum,
                              float* correct, int B, int V, int ld, float scale, float smoothing,
                              hipStream_t st) {
  hipLaunchKernelGGL(softmax_ce_kernel, dim3(B), dim3(NT), 0, st, logits, labels, dlogits, loss_sum,
                     correct, V, ld, scale, smoothing);
  return hipGetLastError();
}

MLC_EXPORT int mlc_colsum(const bf16* g, float* out, int R, int C, hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, st, g, out, R, C);
  return hipGetLastError();
}

MLC_EXPORT int mlc_nchw_to_nhwc(const float* x, bf16* y, int N, int C, int HW, int Cp, hipStream_t st) {
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(blocks_for((long)N * HW * Cp)), dim3(NT), 0, st, x, y,
                     N, C, HW, Cp);
  return hipGetLastError();
}

MLC_EXPORT int mlc_cast_f32_bf16(const float* x, bf16* y, long n, hipStream_t st) {
  if (n % 8) return -1;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(blocks_for(n / 8)), dim3(NT), 0, st, x, y, n / 8);
  return hipGetLastError();
}

MLC_EXPORT int mlc_avgpool2d_fwd(const bf16* x, bf16* y, int N, int H, int W, int C, int Ho, int Wo, int K, int S,
                                 int P, int cip, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool2d_fwd_kernel, dim3(blocks_for((long)N * Ho * Wo * (C / 8))), dim3(NT), 0, st, x, y, N, H,
                     W, C, Ho, Wo, K, S, P, cip);
  return hipGetLastError();
}

// dx = avg-pool backward of dy (+ add, the other consumers' gradient of x, when non-null)
MLC_EXPORT int mlc_avgpool2d_bwd(const bf16* dy, const bf16* add, bf16* dx, int N, int H, int W, int C, int Ho,
                                 int Wo, int K, int S, int P, int cip, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool2d_bwd_kernel, dim3(blocks_for((long)N * H * W * (C / 8))), dim3(NT), 0, st, dy, add, dx, N, H,
                     W, C, Ho, Wo, K, S, P, cip);
  return hipGetLastError();
}

// x [N][H][W][C] -> y [N][Ho][Wo][C] (adaptive average pool, PyTorch's bins); C % 8 == 0
MLC_EXPORT int mlc_adaptive_avg_fwd(const bf16* x, bf16* y, int N, int H, int W, int C, int Ho, int Wo,
                                    hipStream_t st) {
  if (C % 8 || Ho < 1 || Wo < 1 || H < 1 || W < 1) return -1;
  hipLaunchKernelGGL(adaptive_avg_fwd_kernel, dim3((unsigned)(N * Ho * Wo)), dim3(NT), 0, st, x, y, N, H, W, C, Ho,
                     Wo);
  return hipGetLastError();
}

MLC_EXPORT int mlc_adaptive_avg_bwd(const bf16* dy, bf16* dx, int N, int H, int W, int C, int Ho, int Wo,
                                    hipStream_t st) {
  if (C % 8 || Ho < 1 || Wo < 1 || H < 1 || W < 1) return -1;
  hipLaunchKernelGGL(adaptive_avg_bwd_kernel, dim3(blocks_for((long)N * H * W * (C / 8))), dim3(NT), 0, st, dy, dx,
                     N, H, W, C, Ho, Wo);
  return hipGetLastError();
}
