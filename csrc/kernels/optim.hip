// Fused optimizers over flat parameter arenas (one launch for the whole model).
//
// The native engine keeps every parameter of a model in ONE contiguous fp32 master
// buffer (decayed parameters first, then the no-decay ones: BN affine, biases), grads in
// a parallel fp32 buffer that the RCCL bucketer all-reduces in place, and a bf16 mirror
// of the decayed (matmul) weights that the MFMA kernels read.  An update is therefore a
// single bandwidth-bound pass: read p, g, state; write p, state, bf16(p).
// Learning rate and the grad scale live in device memory so the step can be captured in
// a HIP graph and replayed with a new LR without re-capture.
#include "common.h"
#include <stdlib.h>

namespace {
constexpr int NT = 256;

__device__ __forceinline__ void store_bf16x4(bf16* dst, const float* f) {
  uint2 u;
  u.x = pack2_bf16(f[0], f[1]);
  u.y = pack2_bf16(f[2], f[3]);
  *reinterpret_cast<uint2*>(dst) = u;
}
}  // namespace

typedef float v4f __attribute__((ext_vector_type(4)));
// U float4 chunks per thread in flight: every load of an iteration (issued through
// ext-vector types from clamped, always-valid indices) precedes its compute and stores, so
// the loads of U chunks overlap instead of each waiting for the previous chunk's stores
constexpr int OPT_U = 2;

// hyper[0] = lr, hyper[1] = grad scale (e.g. 1/world_size / loss scale)
__global__ void __launch_bounds__(NT)
sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
           bf16* __restrict__ pbf, const float* __restrict__ hyper, long n4, long ndecay4,
           long nbf4, float momentum, float dampening, float wd, int nesterov, int first) {
  const float lr = hyper[0], gs = hyper[1];
  const long stride = (long)gridDim.x * NT;
  v4f* P = reinterpret_cast<v4f*>(p);
  const v4f* Gr = reinterpret_cast<const v4f*>(g);
  v4f* Mo = reinterpret_cast<v4f*>(m);
  const bool mom = momentum != 0.f;
  for (long i0 = (long)blockIdx.x * NT + threadIdx.x; i0 < n4; i0 += stride * OPT_U) {
    v4f pv[OPT_U], gv[OPT_U], mv[OPT_U];
#pragma unroll
    for (int u = 0; u < OPT_U; ++u) {
      const long i = min(i0 + u * stride, n4 - 1);
      pv[u] = P[i];
      gv[u] = Gr[i];
      mv[u] = mom && !first ? Mo[i] : (v4f){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < OPT_U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) break;
      const float w = i < ndecay4 ? wd : 0.f;
      float pp[4], mm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[j] = pv[u][j];
        float d = gv[u][j] * gs + w * pp[j];
        if (mom) {
          mm[j] = first ? d : momentum * mv[u][j] + (1.f - dampening) * d;
          d = nesterov ? d + momentum * mm[j] : mm[j];
        }
        pp[j] -= lr * d;
      }
      P[i] = (v4f){pp[0], pp[1], pp[2], pp[3]};
      if (mom) Mo[i] = (v4f){mm[0], mm[1], mm[2], mm[3]};
      if (pbf && i < nbf4) store_bf16x4(pbf + i * 4, pp);
    }
  }
}

// Adam / AdamW, in torch.optim.Adam(W)'s form: m = b1 m + (1-b1) d, v = b2 v + (1-b2) d^2,
// p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)  (AdamW: p *= 1 - lr*wd first).
// hyper: [lr, grad_scale, bias_correction1, bias_correction2]
__global__ void __launch_bounds__(NT)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, bf16* __restrict__ pbf, const float* __restrict__ hyper, long n4,
            long ndecay4, long nbf4, float b1, float b2, float eps, float wd, int decoupled) {
  const float lr = hyper[0], gs = hyper[1];
  const float step_size = lr / hyper[2], bc2s = sqrtf(hyper[3]);
  const long stride = (long)gridDim.x * NT;
  v4f* P = reinterpret_cast<v4f*>(p);
  const v4f* Gr = reinterpret_cast<const v4f*>(g);
  v4f* Mo = reinterpret_cast<v4f*>(m);
  v4f* Vo = reinterpret_cast<v4f*>(v);
  for (long i0 = (long)blockIdx.x * NT + threadIdx.x; i0 < n4; i0 += stride * OPT_U) {
    v4f pv[OPT_U], gv[OPT_U], mv[OPT_U], vv[OPT_U];
#pragma unroll
    for (int u = 0; u < OPT_U; ++u) {
      const long i = min(i0 + u * stride, n4 - 1);
      pv[u] = P[i];
      gv[u] = Gr[i];
      mv[u] = Mo[i];
      vv[u] = Vo[i];
    }
#pragma unroll
    for (int u = 0; u < OPT_U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) break;
      const float wdi = i < ndecay4 ? wd : 0.f;
      float pp[4], mm[4], ww[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[j] = pv[u][j];
        float d = gv[u][j] * gs;
        if (!decoupled) d += wdi * pp[j];
        mm[j] = b1 * mv[u][j] + (1.f - b1) * d;
        ww[j] = b2 * vv[u][j] + (1.f - b2) * d * d;
        if (decoupled) pp[j] -= lr * wdi * pp[j];
        pp[j] -= step_size * mm[j] / (sqrtf(ww[j]) / bc2s + eps);
      }
      P[i] = (v4f){pp[0], pp[1], pp[2], pp[3]};
      Mo[i] = (v4f){mm[0], mm[1], mm[2], mm[3]};
      Vo[i] = (v4f){ww[0], ww[1], ww[2], ww[3]};
      if (pbf && i < nbf4) store_bf16x4(pbf + i * 4, pp);
    }
  }
}

// Adam with 8-float chunks per lane (two adjacent float4 of every array, one 16-byte bf16
// store), optionally with nontemporal loads/stores (the 3.3 GB BERT-base update stream has
// no reuse); A/B variants of adam_kernel selected by mlc_opt_config (key 0).
template <bool NTMP>
__device__ __forceinline__ v4f ld4(const v4f* p) {
  if constexpr (NTMP) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NTMP>
__device__ __forceinline__ void st4(v4f* p, v4f v) {
  if constexpr (NTMP) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NTMP>
__global__ void __launch_bounds__(NT)
adam8_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
             bf16* __restrict__ pbf, const float* __restrict__ hyper, long n8, long ndecay4, long nbf4, float b1,
             float b2, float eps, float wd, int decoupled) {
  const float lr = hyper[0], gs = hyper[1];
  const float step_size = lr / hyper[2], bc2s = sqrtf(hyper[3]);
  v4f* P = reinterpret_cast<v4f*>(p);
  const v4f* Gr = reinterpret_cast<const v4f*>(g);
  v4f* Mo = reinterpret_cast<v4f*>(m);
  v4f* Vo = reinterpret_cast<v4f*>(v);
  for (long c = (long)blockIdx.x * NT + threadIdx.x; c < n8; c += (long)gridDim.x * NT) {
    v4f pv[2], gv[2], mv[2], vv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pv[h] = ld4<NTMP>(P + 2 * c + h);
      gv[h] = ld4<NTMP>(Gr + 2 * c + h);
      mv[h] = ld4<NTMP>(Mo + 2 * c + h);
      vv[h] = ld4<NTMP>(Vo + 2 * c + h);
    }
    float pp[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float wdi = 2 * c + h < ndecay4 ? wd : 0.f;
      float mm[4], ww[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float q = pv[h][j];
        float d = gv[h][j] * gs;
        if (!decoupled) d += wdi * q;
        mm[j] = b1 * mv[h][j] + (1.f - b1) * d;
        ww[j] = b2 * vv[h][j] + (1.f - b2) * d * d;
        if (decoupled) q -= lr * wdi * q;
        q -= step_size * mm[j] / (sqrtf(ww[j]) / bc2s + eps);
        pp[4 * h + j] = q;
      }
      st4<NTMP>(P + 2 * c + h, (v4f){pp[4 * h], pp[4 * h + 1], pp[4 * h + 2], pp[4 * h + 3]});
      st4<NTMP>(Mo + 2 * c + h, (v4f){mm[0], mm[1], mm[2], mm[3]});
      st4<NTMP>(Vo + 2 * c + h, (v4f){ww[0], ww[1], ww[2], ww[3]});
    }
    if (pbf) {
      if (2 * c + 1 < nbf4) *reinterpret_cast<uint4*>(pbf + 8 * c) = pack8(pp);
      else if (2 * c < nbf4) store_bf16x4(pbf + 8 * c, pp);
    }
  }
}

// A/B knob (MLC_ADAM_VARIANT): 0 = adam_kernel (float4 x 2 in flight), 1 = adam8_kernel
// (default: BERT-base-sized update 710 -> 635 us, 5.2 TB/s counted at 30 B/param),
// 2 = adam8 with nontemporal accesses (1141 us: measured much slower, kept for A/B)
int g_adam_variant = -1;

// out[0] += sum(x^2) over a flat fp32 buffer (for grad-norm clipping)
__global__ void __launch_bounds__(NT)
sqnorm_kernel(const float* __restrict__ x, long n, float* __restrict__ out, float scale) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const float v = x[i] * scale;
    s += v * v;
  }
  s = wave_sum(s);
  __shared__ float red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < NT / 64; ++k) t += red[k];
    atomicAdd(out, t);
  }
}

static int blocks_for(long work) {
  long b = (work + NT * OPT_U - 1) / (NT * OPT_U);
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

// n, ndecay, nbf must be multiples of 4 (the arena pads every segment to 4 floats)
MLC_EXPORT int mlc_sgd(float* p, const float* g, float* m, bf16* pbf, const float* hyper, long n,
                       long ndecay, long nbf, float momentum, float dampening, float wd, int nesterov,
                       int first, hipStream_t st) {
  if (n % 4 || ndecay % 4 || nbf % 4) return -1;
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks_for(n / 4)), dim3(NT), 0, st, p, g, m, pbf, hyper, n / 4,
                     ndecay / 4, nbf / 4, momentum, dampening, wd, nesterov, first);
  return hipGetLastError();
}

MLC_EXPORT int mlc_adam(float* p, const float* g, float* m, float* v, bf16* pbf, const float* hyper,
                        long n, long ndecay, long nbf, float b1, float b2, float eps, float wd,
                        int decoupled, hipStream_t st) {
  if (n % 4 || ndecay % 4 || nbf % 4) return -1;
  if (g_adam_variant < 0) {
    const char* e = getenv("MLC_ADAM_VARIANT");
    g_adam_variant = e ? atoi(e) : 1;
  }
  if (g_adam_variant > 0 && n >= 8) {
    const long n8 = n / 8;
    long b = (n8 + NT - 1) / NT;
    if (b > 16384) b = 16384;
    if (g_adam_variant == 2)
      hipLaunchKernelGGL(adam8_kernel<true>, dim3(b), dim3(NT), 0, st, p, g, m, v, pbf, hyper, n8, ndecay / 4,
                         nbf / 4, b1, b2, eps, wd, decoupled);
    else
      hipLaunchKernelGGL(adam8_kernel<false>, dim3(b), dim3(NT), 0, st, p, g, m, v, pbf, hyper, n8, ndecay / 4,
                         nbf / 4, b1, b2, eps, wd, decoupled);
    if (n % 8) {   // the last float4 (segments are padded to 4 floats)
      const long o = n8 * 8;
      const long nbr = nbf > o ? nbf - o : 0, ndr = ndecay > o ? ndecay - o : 0;
      hipLaunchKernelGGL(adam_kernel, dim3(1), dim3(NT), 0, st, p + o, g + o, m + o, v + o, nbr ? pbf + o : nullptr,
                         hyper, 1L, ndr / 4, nbr / 4, b1, b2, eps, wd, decoupled);
    }
    return hipGetLastError();
  }
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n / 4)), dim3(NT), 0, st, p, g, m, v, pbf, hyper,
                     n / 4, ndecay / 4, nbf / 4, b1, b2, eps, wd, decoupled);
  return hipGetLastError();
}

// zero up to four fp32 buffers in one launch (a training step's scratch workspace and its
// gradient arenas: one dispatch instead of one memset each)
struct Zero4 {
  float* p[4];
  long n[4];
};

__global__ void __launch_bounds__(256) zero4_kernel(Zero4 z) {
  const long stride = (long)gridDim.x * 256;
  for (int b = 0; b < 4; ++b) {
    float* p = z.p[b];
    if (!p) continue;
    const long n = z.n[b];
    const long n4 = ((uintptr_t)p % 16 == 0) ? n / 4 : 0;    // 16-byte stores where aligned
    float4* q = reinterpret_cast<float4*>(p);
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long i = n4 * 4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) p[i] = 0.f;
  }
}

MLC_EXPORT int mlc_zero4(float* p0, long n0, float* p1, long n1, float* p2, long n2, float* p3, long n3,
                         hipStream_t st) {
  Zero4 z{{p0, p1, p2, p3}, {p0 ? n0 : 0, p1 ? n1 : 0, p2 ? n2 : 0, p3 ? n3 : 0}};
  long most = 0;
  for (int b = 0; b < 4; ++b) most = z.n[b] > most ? z.n[b] : most;
  long blocks = (most / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(zero4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, z);
  return hipGetLastError();
}

MLC_EXPORT int mlc_sqnorm(const float* x, long n, float* out, float scale, hipStream_t st) {
  long b = (n + NT * 8 - 1) / (NT * 8);
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(sqnorm_kernel, dim3(b), dim3(NT), 0, st, x, n, out, scale);
  return hipGetLastError();
}

// optimizer A/B knobs: key 0 = Adam kernel variant (see g_adam_variant); value < 0 only
// reads.  Returns the previous value.
MLC_EXPORT int mlc_opt_config(int key, int value) {
  if (key != 0) return -1;
  if (g_adam_variant < 0) {
    const char* e = getenv("MLC_ADAM_VARIANT");
    g_adam_variant = e ? atoi(e) : 1;
  }
  const int old = g_adam_variant;
  if (value >= 0) g_adam_variant = value;
  return old;
}

