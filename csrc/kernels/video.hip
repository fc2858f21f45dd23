// Temporal unfold / fold of the 3-D convolutions (mlcomp_amd/ops/glayers.py Conv3dAs2d).
//
// A Conv3d with a (kt, kh, kw) kernel runs as a 2-D conv over the N*To output frames whose
// input channels are the kt temporal taps of each channel (channel c*kt + j of output frame
// (n, to) holds input frame ti = to*st + j*dil - pad of channel c, zero outside [0, T)); the
// filter is the Conv3d weight viewed as [Co, C*kt, kh, kw].  These two kernels build that
// frame tensor from the NTHWC (channels_last_3d) activation and fold its gradient back, in
// place of the torch pad / index_select / index_add glue of round 5:
//
//   unfold: one thread per (output frame row, 8-channel group): kt 16-byte loads (one per
//           tap, zero-filled outside the clip), the 8 x kt values interleaved in registers,
//           kt 16-byte stores of the contiguous 8*kt-element output chunk;
//   fold:   one thread per (input row, 8-channel group), a GATHER over the kt taps that read
//           it (no atomics, deterministic): for each tap j with (ti + pad - j*dil) a multiple
//           of st inside [0, To*st), the tap's chunk (kt 16-byte loads, shared through L2 with
//           the neighbouring frames' threads) is loaded and its 8 values summed in fp32;
//           an optional addend (another branch's gradient of the same activation: a residual
//           block's identity path or its shortcut conv) starts the sum, so autograd does not
//           add the two branch gradients in a pass of its own.
//
// Both are streaming passes (bandwidth bound); C % 8 == 0, kt <= 8.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int KTMAX = 8;

__device__ __forceinline__ uint4 ld16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }

template <int KT>
__global__ void __launch_bounds__(NT)
temporal_unfold_kernel(const bf16* __restrict__ x, bf16* __restrict__ out, int N, int T, int HW, int C, int st,
                       int pad, int dil, int To) {
  const int G = C >> 3;
  const long total = (long)N * To * HW * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int g = (int)(i % G);
    const long row = i / G;                       // (n, to, p)
    const int p = (int)(row % HW);
    const long f = row / HW;
    const int to = (int)(f % To), n = (int)(f / To);
    uint4 u[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int ti = to * st + j * dil - pad;
      u[j] = (unsigned)ti < (unsigned)T ? ld16(x + (((long)n * T + ti) * HW + p) * C + g * 8)
                                        : make_uint4(0u, 0u, 0u, 0u);
    }
    // interleave: output element c*KT + j = tap j of channel c (all indices compile-time)
    bf16 w[8 * KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const bf16* b = reinterpret_cast<const bf16*>(&u[j]);
#pragma unroll
      for (int c = 0; c < 8; ++c) w[c * KT + j] = b[c];
    }
    uint4* dst = reinterpret_cast<uint4*>(out + row * (long)C * KT + (long)g * 8 * KT);
#pragma unroll
    for (int q = 0; q < KT; ++q) dst[q] = reinterpret_cast<const uint4*>(w)[q];
  }
}

template <int KT>
__global__ void __launch_bounds__(NT)
temporal_fold_kernel(const bf16* __restrict__ dcol, const bf16* __restrict__ add, bf16* __restrict__ dx, int N,
                     int T, int HW, int C, int st, int pad, int dil, int To) {
  const int G = C >> 3;
  const long total = (long)N * T * HW * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int g = (int)(i % G);
    const long row = i / G;                       // (n, ti, p)
    const int p = (int)(row % HW);
    const long f = row / HW;
    const int ti = (int)(f % T), n = (int)(f / T);
    float acc[8];
    if (add) {
      const uint4 a = ld16(add + row * C + g * 8);
      const bf16* b = reinterpret_cast<const bf16*>(&a);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = (float)b[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int num = ti + pad - j * dil;
      if (num < 0 || num % st) continue;
      const int to = num / st;
      if (to >= To) continue;
      // the tap's 8*KT-element chunk (KT 16-byte loads), element c*KT + j for the 8 channels
      const uint4* src = reinterpret_cast<const uint4*>(dcol + ((((long)n * To + to) * HW + p) * C + (long)g * 8) * KT);
      uint4 u[KT];
#pragma unroll
      for (int q = 0; q < KT; ++q) u[q] = src[q];
      const bf16* b = reinterpret_cast<const bf16*>(u);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (float)b[e * KT + j];
    }
    bf16 o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)acc[e];
    *reinterpret_cast<uint4*>(dx + row * C + g * 8) = *reinterpret_cast<const uint4*>(o);
  }
}

inline int grid_of(long work) {
  long b = (work + NT - 1) / NT;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

// x [N][T][HW][C] bf16 -> out [N][To][HW][C*kt] bf16 (see above)
MLC_EXPORT int mlc_temporal_unfold(const bf16* x, bf16* out, int N, int T, int HW, int C, int kt, int st, int pad,
                                   int dil, int To, hipStream_t stream) {
  if (C % 8 || kt < 1 || kt > KTMAX || st < 1 || dil < 1 || To < 1) return -1;
  const dim3 grid(grid_of((long)N * To * HW * (C / 8)));
#define MLC_UNFOLD(K) hipLaunchKernelGGL(temporal_unfold_kernel<K>, grid, dim3(NT), 0, stream, x, out, N, T, HW, C, \
                                         st, pad, dil, To)
  switch (kt) {
    case 1: MLC_UNFOLD(1); break;
    case 2: MLC_UNFOLD(2); break;
    case 3: MLC_UNFOLD(3); break;
    case 4: MLC_UNFOLD(4); break;
    case 5: MLC_UNFOLD(5); break;
    case 6: MLC_UNFOLD(6); break;
    case 7: MLC_UNFOLD(7); break;
    default: MLC_UNFOLD(8); break;
  }
#undef MLC_UNFOLD
  return hipGetLastError();
}

// dcol [N][To][HW][C*kt] -> dx [N][T][HW][C] (overwritten; + add [N][T][HW][C] when non-null):
// the gradient of the unfold
MLC_EXPORT int mlc_temporal_fold(const bf16* dcol, const bf16* add, bf16* dx, int N, int T, int HW, int C, int kt, int st, int pad,
                                 int dil, int To, hipStream_t stream) {
  if (C % 8 || kt < 1 || kt > KTMAX || st < 1 || dil < 1 || To < 1) return -1;
  const dim3 grid(grid_of((long)N * T * HW * (C / 8)));
#define MLC_FOLD(K) hipLaunchKernelGGL(temporal_fold_kernel<K>, grid, dim3(NT), 0, stream, dcol, add, dx, N, T, HW, C, st, \
                                       pad, dil, To)
  switch (kt) {
    case 1: MLC_FOLD(1); break;
    case 2: MLC_FOLD(2); break;
    case 3: MLC_FOLD(3); break;
    case 4: MLC_FOLD(4); break;
    case 5: MLC_FOLD(5); break;
    case 6: MLC_FOLD(6); break;
    case 7: MLC_FOLD(7); break;
    default: MLC_FOLD(8); break;
  }
#undef MLC_FOLD
  return hipGetLastError();
}
