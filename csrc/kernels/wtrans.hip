// Transposed + flipped bf16 weight copies for the input-gradient GEMMs (gfx950).
//
// A stride-1 conv's input gradient is itself a stride-1 conv of dY with the filter
// flipped in space and its channel axes swapped:
//   dX[n,h,w,ci] = sum_{r,s,co} dY[n, h+pad'-r*d, ...] * Wt[ci][r][s][co],
//   Wt[ci][r][s][co] = W[co][KH-1-r][KW-1-s][ci],  pad' = d*(K-1) - pad.
// With Wt in memory the dgrad runs on the forward conv's loaders (both operands
// K-contiguous, read with ds_read_b128) instead of reading W as an MN-contiguous tile
// through ds_read_b64_tr_b16 - half the LDS read instructions per MFMA.  Wt changes only
// when the optimizer updates W, so the whole model's copies are refreshed by ONE launch
// per step between forward and backward (NativeContext.refresh_wt).
//
// One block = one filter tap x 64 (co) x 64 (ci) tile, staged through LDS: 16-byte
// coalesced reads along ci, 16-byte coalesced writes along co.
#include "common.h"

namespace {

struct WtDesc {  // int64 fields, filled by the host (ops/functional.WtTable)
  long long src, dst, co, taps, ci, first_block;
};

__global__ void __launch_bounds__(256)
wt_transpose_kernel(const WtDesc* __restrict__ d, int n) {
  // the descriptor owning this block: largest i with first_block <= blockIdx.x
  const long long b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].first_block <= b) lo = mid; else hi = mid - 1;
  }
  const WtDesc e = d[lo];
  const int Co = (int)e.co, T = (int)e.taps, Ci = (int)e.ci;
  const int tco = (Co + 63) >> 6, tci = (Ci + 63) >> 6;
  int rem = (int)(b - e.first_block);
  const int t = rem / (tco * tci);
  rem -= t * tco * tci;
  const int co0 = (rem / tci) * 64, ci0 = (rem % tci) * 64;
  const bf16* src = reinterpret_cast<const bf16*>(e.src);
  bf16* dst = reinterpret_cast<bf16*>(e.dst);

  // [64 co][64 ci] tile, row padded by 8 elements so the column reads spread over banks
  __shared__ unsigned short tile[64][72];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (tid >> 3) + 32 * i, c = (tid & 7) * 8;
    const int co = co0 + r, ci = ci0 + c;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (co < Co && ci < Ci) v = ldg16(src + ((size_t)co * T + t) * Ci + ci);
    *reinterpret_cast<uint4*>(&tile[r][c]) = v;
  }
  __syncthreads();
  const int tf = T - 1 - t;  // flipped tap (r, s) -> (KH-1-r, KW-1-s) is T-1-t
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (tid >> 3) + 32 * i, c = (tid & 7) * 8;  // r: ci row of Wt, c: co chunk
    const int ci = ci0 + r, co = co0 + c;
    if (ci >= Ci || co >= Co) continue;
    unsigned short u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = tile[c + k][r];
    uint4 o;
    o.x = u[0] | ((unsigned)u[1] << 16);
    o.y = u[2] | ((unsigned)u[3] << 16);
    o.z = u[4] | ((unsigned)u[5] << 16);
    o.w = u[6] | ((unsigned)u[7] << 16);
    *reinterpret_cast<uint4*>(dst + ((size_t)ci * T + tf) * Co + co) = o;
  }
}

}  // namespace

// descs: device array of n WtDesc (int64 x 6); blocks: total block count (sum over
// descriptors of taps * ceil(Co/64) * ceil(Ci/64)).  Co and Ci must be multiples of 8.
MLC_EXPORT int mlc_wt_transpose(const void* descs, int n, long blocks, hipStream_t st) {
  if (n <= 0 || blocks <= 0) return 0;
  hipLaunchKernelGGL(wt_transpose_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     reinterpret_cast<const WtDesc*>(descs), n);
  return (int)hipGetLastError();
}
