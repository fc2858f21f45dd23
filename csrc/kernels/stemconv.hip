// ResNet stem convolution (the 7x7/2 conv over 3 channels, run as a 4x4/1 conv over the
// 2x2 space-to-depth image, stem.hip / ops.functional.stem_s2d) as a persistent
// register-resident-filter kernel.
//
// The GEMM is M = N*112*112 pixels x N = 64 channels x K = 4*4*16 = 256.  Through the
// generic implicit-GEMM engine (igemm.hip, 256x64 tiles, K = 4 tiles of 64) every block
// pays a full pipeline prologue + drain + epilogue for 4 K-tiles and re-stages the same
// 32 KB filter in LDS: ~500 us at batch 512 (~2 TB/s against ~1.04 GB of compulsory
// traffic, scripts/bench_stem.py).  Here:
//   * each wave holds the whole filter as MFMA A-fragments in VGPRs (2 channel blocks x 16
//     K-steps x 8 bf16 = 128 VGPRs), loaded once; the output is C^T (rows = channels,
//     cols = pixels), so a tile is 32 consecutive pixels x 64 channels = 4 KB of
//     consecutive y;
//   * the tile goes out through a per-wave LDS stage as four contiguous 1 KB wave stores
//     (direct 8 B stores from the MFMA layout, 128 B apart per lane, ran the kernel
//     write-bound: 480 us vs 160 us with the stores removed);
//   * the BN statistics (sum, sum of squares per channel, from the fp32 accumulators) stay
//     in per-lane registers over all of the wave's tiles (a lane's channels never change)
//     and are reduced across lanes once, at the end: 64 atomics per wave, not per tile.
// Two image-operand paths (MLC_STEM_IMPL):
//   1 (band, default): a block owns bands of R output rows of one image; the R+3 input
//     rows of a band are one contiguous range of the s2d image, copied to LDS with
//     LDS-DMA (buffer_load ... lds) while the previous band computes (double-buffered);
//     the B-fragments are ds_read_b128 from it.  Each input byte leaves HBM / L2 about
//     (R+3)/R times instead of 16 times.
//   0 (direct): lane (p, h) reads its B-fragment (16 B: channels 8h..8h+7 of s2d pixel
//     (oh+r, ow+s)) straight from global memory per K-step (r, s), NB-1 tiles prefetched.
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int SC_NT = 256;
constexpr int SC_BAND_BYTES = 48 * 1024;   // one band image buffer (x2 for double-buffering)

__device__ __forceinline__ bf16x8 ldfrag(const bf16* p) { return __builtin_bit_cast(bf16x8, ldg16(p)); }

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// filter fragments: A[co][k], co = 32b + p, k = 16s + 8h
__device__ __forceinline__ void load_filter(bf16x8 (&wf)[2][16], const bf16* w, int p, int h) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 16; ++s) wf[b][s] = ldfrag(w + (32 * b + p) * 256 + 16 * s + 8 * h);
}

// acc[r] of channel block b: channel 32b + (r&3) + 8(r>>2) + 4h of pixel p.  Stage the tile as
// [pixel][channel] rows (16 B chunk c of row p at c ^ (p & 7)) and write its valid pixels
// (q < nvalid) with 16 B per lane, 1 KB contiguous per wave store.  The stage accesses are
// inline asm (with their own lgkmcnt waits): the compiler cannot tell them apart from the
// band kernel's LDS-DMA target and would otherwise wait vmcnt(0) - draining the DMA and
// every store in flight - before each tile's first stage write.
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_tile(char* stage, const f32x16& c0, const f32x16& c1, bf16* yt, int nvalid,
                                           int lane, int p, int h) {
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)stage;
  u32x2v v[8];
  unsigned a[8];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x16& c = b ? c1 : c0;
      v[4 * b + g] = u32x2v{pack2_bf16(c[4 * g], c[4 * g + 1]), pack2_bf16(c[4 * g + 2], c[4 * g + 3])};
      a[4 * b + g] = sbase + p * 128 + (((4 * b + g) ^ (p & 7)) << 4) + 8 * h;
    }
  // the previous tile's stage reads completed inside their own asm block
  asm volatile(
      "ds_write_b64 %0, %8\n\tds_write_b64 %1, %9\n\tds_write_b64 %2, %10\n\tds_write_b64 %3, %11\n\t"
      "ds_write_b64 %4, %12\n\tds_write_b64 %5, %13\n\tds_write_b64 %6, %14\n\tds_write_b64 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)" ::"v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),
      "v"(a[7]), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7])
      : "memory");
  const int cc = lane & 7;
  unsigned ra[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = 8 * i + (lane >> 3);
    ra[i] = sbase + q * 128 + ((cc ^ (q & 7)) << 4);
  }
  u32x4v r0, r1, r2, r3;
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(ra[0]), "v"(ra[1]), "v"(ra[2]), "v"(ra[3])
      : "memory");
  const u32x4v rv[4] = {r0, r1, r2, r3};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = 8 * i + (lane >> 3);
    if (q < nvalid) *reinterpret_cast<u32x4v*>(yt + q * 64 + cc * 8) = rv[i];
  }
}

__device__ __forceinline__ void add_stats(float (&a1)[2][16], float (&a2)[2][16], const f32x16& c0,
                                          const f32x16& c1) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    a1[0][r] += c0[r]; a2[0][r] += c0[r] * c0[r];
    a1[1][r] += c1[r]; a2[1][r] += c1[r] * c1[r];
  }
}

// reduce over the 32 pixels (lanes) of each half; lanes 0 / 32 add their half's 32
// channels into copy `slot`
__device__ __forceinline__ void flush_stats(float (&a1)[2][16], float (&a2)[2][16], float* s1, float* s2, int slot,
                                            int p, int h) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float u = a1[b][r], v = a2[b][r];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) { u += __shfl_xor(u, o, 64); v += __shfl_xor(v, o, 64); }
      if (p == 0) {
        const int co = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
        atomicAdd(s1 + slot * 64 + co, u);
        atomicAdd(s2 + slot * 64 + co, v);
      }
    }
}

template <bool STATS, int NB>
__global__ void __launch_bounds__(SC_NT, 1)
stem_conv_direct_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, bf16* __restrict__ y,
                        float* __restrict__ s1, float* __restrict__ s2, int M, int HWo, int Wo, int Hb, int Wb,
                        int ntiles, int ncopy) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, p = lane & 31;
  __shared__ __attribute__((aligned(16))) char lds[4][32 * 128];
  char* stage = lds[wave];
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = (int)((long)ntiles * blk / gridDim.x), t1 = (int)((long)ntiles * (blk + 1) / gridDim.x);
  int t = t0 + wave;
  if (t >= t1) return;
  bf16x8 wf[2][16];
  load_filter(wf, w, p, h);
  float a1[2][16] = {}, a2[2][16] = {};

  auto load = [&](bf16x8 (&f)[16], int tt) {
    int pix = tt * 32 + p;
    if (pix >= M) pix = M - 1;
    const int n = pix / HWo, rem = pix - n * HWo;
    const int oh = rem / Wo, ow = rem - oh * Wo;
    const bf16* b0 = x + (((long)n * Hb + oh) * Wb + ow) * 16 + 8 * h;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int s = 0; s < 4; ++s) f[4 * r + s] = ldfrag(b0 + (r * Wb + s) * 16);
  };
  auto compute = [&](const bf16x8 (&f)[16], int tt) {
    f32x16 c0 = {}, c1 = {};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[0][s], f[s], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[1][s], f[s], c1, 0, 0, 0);
    }
    const long tile0 = (long)tt * 32;
    const int nvalid = (int)min(32L, (long)M - tile0);
    if (y) store_tile(stage, c0, c1, y + tile0 * 64, nvalid, lane, p, h);
    if (STATS && p < nvalid) add_stats(a1, a2, c0, c1);
  };

  // NB fragment buffers in a ring, NB-1 tiles prefetched, always issued (clamped to the
  // last tile): a fixed load count per tile, so the wait before each tile's MFMAs is a
  // counted vmcnt, not a drain
  bf16x8 f[NB][16];
#pragma unroll
  for (int i = 0; i < NB - 1; ++i) load(f[i], min(t + 4 * i, t1 - 1));
  bool more = true;
  while (more) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (more) {
        load(f[(j + NB - 1) % NB], min(t + 4 * (NB - 1), t1 - 1));
        compute(f[j], t);
        t += 4;
        more = t < t1;
      }
    }
  }
  if (STATS) flush_stats(a1, a2, s1, s2, blk % ncopy, p, h);
}

// band b: image b / bpi, output rows R*(b % bpi) .. +R (fewer in the last band of an image)
template <bool STATS>
__global__ void __launch_bounds__(SC_NT, 1)
stem_conv_band_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, bf16* __restrict__ y,
                      float* __restrict__ s1, float* __restrict__ s2, int Ho, int Wo, int Hb, int Wb, int R, int bpi,
                      int nbands, int ncopy) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, p = lane & 31;
  // two distinct LDS objects (not one [2][...] array indexed at run time): the compiler can
  // then prove the ds_reads of one band do not alias the LDS-DMA filling the other, instead
  // of waiting for the DMA before every read
  __shared__ __attribute__((aligned(16))) char img0[SC_BAND_BYTES];
  __shared__ __attribute__((aligned(16))) char img1[SC_BAND_BYTES];
  __shared__ __attribute__((aligned(16))) char stg[4][32 * 128];
  char* stage = stg[wave];
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int b0 = (int)((long)nbands * blk / gridDim.x), b1 = (int)((long)nbands * (blk + 1) / gridDim.x);
  if (b0 >= b1) return;
  const unsigned row_bytes = (unsigned)Wb * 32u;

  // LDS-DMA of band bb into `img`: rows oh0 .. oh0+rr+2 are one contiguous range;
  // lane-linear 16 B chunks, 4 KB per block round, zero past the range (OOB voffset)
  auto fetch = [&](int bb, char* img) {
    const int n = bb / bpi, oh0 = (bb - n * bpi) * R;
    const int rr = min(R, Ho - oh0);
    const unsigned bytes = (unsigned)(rr + 3) * row_bytes;
    const Rsrc rs = make_rsrc(reinterpret_cast<const char*>(x) + ((long)n * Hb + oh0) * row_bytes, bytes);
    char* dst = img + __builtin_amdgcn_readfirstlane(wave) * 1024;
    for (unsigned off = 0; off < bytes; off += SC_NT * 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + off), 16,
                                               off + tid * 16, 0, 0, 0);
  };

  bf16x8 wf[2][16];
  load_filter(wf, w, p, h);
  float a1[2][16] = {}, a2[2][16] = {};
  int stores = 0;   // wave stores issued since the last DMA (vmcnt retires in issue order)

  auto band = [&](int bb, const char* img, char* nimg) {
    // this thread's DMA of band bb landed; the tile stores issued after it may stay in
    // flight (a full band: 7 tiles x 4 stores per wave)
    if (stores >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
    else if (stores >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (stores >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ... everyone's, and the previous band read by all (a bare barrier: __syncthreads'
    // release fence would also drain the stores)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stores = 0;
    if (bb + 1 < b1) fetch(bb + 1, nimg);
    const int n = bb / bpi, oh0 = (bb - n * bpi) * R;
    const int P = min(R, Ho - oh0) * Wo;                  // output pixels of the band
    bf16* yb = y ? y + ((long)n * Ho + oh0) * Wo * 64 : nullptr;
    const char* im = img + 16 * h;
    auto lds_load = [&](bf16x8 (&f)[16], int j) {
      const int q = min(j * 32 + p, P - 1);
      const int row = q / Wo, col = q - row * Wo;
      const char* src = im + (row * Wb + col) * 32;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) f[4 * r + s] = *reinterpret_cast<const bf16x8*>(src + (r * Wb + s) * 32);
    };
    auto compute = [&](const bf16x8 (&f)[16], int j) {
      f32x16 c0 = {}, c1 = {};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[0][s], f[s], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[1][s], f[s], c1, 0, 0, 0);
      }
      const int nvalid = min(32, P - j * 32);
      if (yb) {
        store_tile(stage, c0, c1, yb + (long)j * 32 * 64, nvalid, lane, p, h);
        stores += 4;
      }
      if (STATS && p < nvalid) add_stats(a1, a2, c0, c1);
    };
    // the next tile's fragments are read while this tile's MFMAs run
    bf16x8 fa[16], fb[16];
    int j = wave;
    if (j * 32 >= P) return;
    lds_load(fa, j);
    for (;;) {
      if ((j + 4) * 32 < P) lds_load(fb, j + 4);
      compute(fa, j);
      j += 4;
      if (j * 32 >= P) break;
      if ((j + 4) * 32 < P) lds_load(fa, j + 4);
      compute(fb, j);
      j += 4;
      if (j * 32 >= P) break;
    }
  };

  fetch(b0, img0);
  for (int bb = b0; bb < b1; bb += 2) {
    band(bb, img0, img1);
    if (bb + 1 < b1) band(bb + 1, img1, img0);
  }
  if (STATS) flush_stats(a1, a2, s1, s2, blk % ncopy, p, h);
}

int g_sc_cus = 0;

}  // namespace

// y[N,Ho,Wo,64] = 4x4/1 conv of the s2d image x[N,Hb,Wb,16] (Hb = Ho+3, Wb = Wo+3) with
// w[64,4,4,16]; s1/s2 (NSTAT*64 fp32, zeroed by the caller) receive per-channel partial
// sums of y and y^2 as in mlc_conv_fwd, or are null.  Returns -2 in deterministic mode
// (float atomics from several waves per copy): the caller uses mlc_conv_fwd then.
MLC_EXPORT int mlc_stem_conv_fwd(const bf16* x, const bf16* w, bf16* y, float* s1, float* s2, int N, int Hb,
                                 int Wb, hipStream_t st) {
  if (s1 && g_mlc_det) return -2;
  const int Ho = Hb - 3, Wo = Wb - 3;
  if (Ho <= 0 || Wo <= 0) return -1;
  if ((long)N * Ho * Wo + 31 > 0x7fffffffL || (long)N * Hb * Wb * 32 > 0x7fffffffL) return -1;
  if (!g_sc_cus) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    g_sc_cus = cus;
  }
  if (getenv("MLC_STEM_NOSTORE")) y = nullptr;   // probe: statistics only
  static const int impl = getenv("MLC_STEM_IMPL") ? atoi(getenv("MLC_STEM_IMPL")) : 1;
  // band rows: the R+3 input rows of a band fill at most one LDS image buffer
  const int R = min(8, SC_BAND_BYTES / (Wb * 32) - 3);
  if (impl == 1 && R >= 1) {
    const int bpi = (Ho + R - 1) / R, nbands = N * bpi;
    const int blocks = min(g_sc_cus, nbands);
    if (s1)
      stem_conv_band_kernel<true><<<blocks, SC_NT, 0, st>>>(x, w, y, s1, s2, Ho, Wo, Hb, Wb, R, bpi, nbands,
                                                            g_mlc_ncopy);
    else
      stem_conv_band_kernel<false><<<blocks, SC_NT, 0, st>>>(x, w, y, s1, s2, Ho, Wo, Hb, Wb, R, bpi, nbands,
                                                             g_mlc_ncopy);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const int M = N * Ho * Wo;
  const int ntiles = (M + 31) / 32;
  const int blocks = min(g_sc_cus, (ntiles + 3) / 4);
  // MLC_STEM_NB: fragment ring depth of the direct path (2 or 3)
  static const int nb = getenv("MLC_STEM_NB") ? atoi(getenv("MLC_STEM_NB")) : 2;
#define SC_LAUNCH(S, B) stem_conv_direct_kernel<S, B><<<blocks, SC_NT, 0, st>>>(x, w, y, s1, s2, M, Ho * Wo, Wo, Hb, \
                                                                              Wb, ntiles, g_mlc_ncopy)
  if (s1) {
    if (nb == 3) SC_LAUNCH(true, 3); else SC_LAUNCH(true, 2);
  } else {
    if (nb == 3) SC_LAUNCH(false, 3); else SC_LAUNCH(false, 2);
  }
#undef SC_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
