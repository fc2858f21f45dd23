// Shared helpers for the mlcomp_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T) __attribute__((address_space(3))) T*

#define MLC_EXPORT extern "C" __attribute__((visibility("default")))

// Per-channel / per-column reductions (BN statistics in the conv epilogue, BN and LN
// backward sums, bias column sums) add each block's partial into copy (block % ncopy) of
// a [ncopy][...] scratch and a finalize kernel folds the copies in a fixed order.  The
// default ncopy = 32 spreads the same-address float atomics.  Deterministic mode
// (mlc_set_deterministic, MLC_DETERMINISTIC=1) raises ncopy so that every contributing
// block owns its copy - one add onto zero, exact and order-free - and runs split-K
// GEMMs unsplit (one atomic contribution per output element) or through fp32 slabs.
// Host-side state, defined in batchnorm.hip; launchers pass ncopy to their kernels.
extern int g_mlc_ncopy;
extern int g_mlc_det;
// ordered per-channel statistics pass (normact.hip), shared by the conv launchers
extern "C" int mlc_bn_stats(const bf16* x, float* sum, float* sumsq, long rows, int C, hipStream_t st);

static __device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
static __device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// unpack 8 bf16 held in a uint4 into floats
// channel-group slice of the folded-finalize BN passes (batchnorm.hip / normact.hip *_fused
// kernels): the largest divisor of G (8-channel groups) not above cap, so every C % 8 == 0
// splits into equal slices (DenseNet's 36 / 44 / 52 groups, EfficientNet's 40 / 60 / 84)
static __host__ __device__ __forceinline__ int slice_groups(int G, int cap) {
  int d = G < cap ? G : cap;
  while (d > 1 && G % d) --d;
  return d;
}

static __device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// float -> bf16 with the hardware converter (v_cvt_pk_bf16_f32: round-to-nearest-even,
// NaN stays NaN); one instruction per PAIR of values, so pack two at a time
static __device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  const bf16x2 r = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(uint32_t, r);
}
static __device__ __forceinline__ uint32_t f2bf_bits(float f) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (bf16)f);
}

static __device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2_bf16(f[0], f[1]);
  r.y = pack2_bf16(f[2], f[3]);
  r.z = pack2_bf16(f[4], f[5]);
  r.w = pack2_bf16(f[6], f[7]);
  return r;
}

// 16-byte global load through an ext-vector type.  Loading HIP's uint4 struct directly
// lets hipcc split a conditional load into four branch-wrapped dword loads (seen in the
// conv epilogues) or serialise a batch of loads with vmcnt(0) after each; the vector type
// keeps one dwordx4 per chunk and lets the loads of a batch fly together.
static __device__ __forceinline__ uint4 ldg16(const void* p) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// 8 consecutive floats (two 16-byte loads)
static __device__ __forceinline__ void ldg8f(const float* p, float* f) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const f32x4v a = *reinterpret_cast<const f32x4v*>(p), b = *reinterpret_cast<const f32x4v*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md T1):
// blocks dealt round-robin to the 8 XCDs end up owning contiguous tile ranges.
static __device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = orig & 7, loc = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Zero n floats on stream st with a kernel.  Used instead of hipMemsetAsync for the
// accumulation targets of atomics: a memset captured into a HIP graph becomes a memset
// node that the runtime may run on a copy engine, outside the kernels' L2 ordering.
static __global__ void __launch_bounds__(256) mlc_zero_f32_kernel(float* __restrict__ p, long n) {
  // scalar stores: targets are arena slices with any 4-byte offset
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = 0.f;
}
static inline void mlc_zero_f32(float* p, long n, hipStream_t st) {
  if (n <= 0) return;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(mlc_zero_f32_kernel, dim3(blocks), dim3(256), 0, st, p, n);
}
