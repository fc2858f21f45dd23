// Grouped and depthwise convolutions, NHWC bf16, for the generic native engine
// (ResNeXt / SE-ResNeXt grouped 3x3s, EfficientNet / MobileNet depthwise kxk).
//
// Grouped (groups > 1, Cg = channels per group, in == out, Cg | 16 or 16 | Cg) on the
// v_mfma_f32_16x16x32_bf16 matrix cores.  The GEMM is block-diagonal: an output block of
// 16 channels reads KB = max(16, Cg) input channels per filter tap (for Cg < 16 the 16
// channels of the 16/Cg groups the block spans, with the off-group weights zero).  That
// wastes 16/Cg of the MFMA work for Cg < 16 but keeps every operand a 16-byte NHWC chunk;
// these layers are bound by HBM / L1 traffic, not by the matrix cores.
//   forward     y[p][oc]   = sum_{t,kb} x[p@t][cbase+kb] * WB[ob][j][t*KB+kb]
//   dgrad       dx[q][ic]  = the same kernel over dy, with the stride-fractional tap map
//               (a tap reaches q iff (q + pad - r*dil) % S == 0) and WB built from the
//               transposed weight
//   wgrad       dw[oc][t][ci] = sum_p dy[p][oc] * x[p@t][ci]: K = pixels, both operands
//               staged through LDS [px][16] and read with ds_read_b64_tr_b16
// WB is the 16-column-block expansion of the [Co][KH][KW][Cg] filter (one tiny kernel per
// use), laid out [ob][j][Kpad] so a lane's B fragment is one 16-byte load.
//
// Depthwise (groups == C, one filter per channel) on the VALU: 18 FLOP per output, pure
// bandwidth.  Threads own a fixed 8-channel group (16 B accesses, grid = multiple of C/8
// threads, as the BatchNorm passes) and walk pixels; the weight gradient reduces per
// thread, then per block (LDS), then over 32 partial copies.
#include <numeric>
#include "common.h"
#include <stdlib.h>

namespace gconv {

constexpr int NT = 256;
constexpr int NCOPY = 32;   // partial-sum copies of the cross-block reductions

struct GGeom {
  int N, Hi, Wi, Ci;        // operand image (x; dy for the transposed map)
  int Ho, Wo, Co;           // output image (y; dx for the transposed map)
  int KH, KW, S, P, D;
  int Cg, KB, T, Kp;        // K-side channels per group, K channels per tap (mult. of 16), taps,
                            // padded K (mult. of 32)
  int Cog;                  // output channels per group
  long M;                   // output pixels
};

// first K-side channel (8-aligned) of the 16-channel output block starting at oc0: the block
// spans the groups oc0/Cog .. (oc0+15)/Cog, whose K-side channels start at (oc0/Cog)*Cg
__device__ __host__ __forceinline__ int blk_cbase(int oc0, int Cog, int Cg) { return (oc0 / Cog) * Cg & ~7; }

__device__ __forceinline__ bf16x8 ldfrag(const bf16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

// ------------------------------------------------------------------ weight expansion
// WB[ob][j][k] (k < Kp): the B operand of the 16-column output block ob.  tr = 0: the
// forward filter w[Co][T][Cg]; tr = 1: the dgrad filter (output channel = the conv's
// input channel, K over the conv's output channels of the group).
// Cout: output channels (rows of wb: Cout rounded up to 16), Cin: K-side channels; Cg / Cog:
// K-side / output channels per group
__global__ void __launch_bounds__(NT)
expand_kernel(const bf16* __restrict__ w, bf16* __restrict__ wb, int Cout, int Cin, int T, int Cg, int Cog,
              int KB, int Kp, int tr) {
  const long total = (long)((Cout + 15) / 16 * 16) * Kp;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int k = (int)(i % Kp);
    const int oc = (int)(i / Kp);           // = ob*16 + j
    float v = 0.f;
    if (k < T * KB && oc < Cout) {
      const int t = k / KB, kb = k % KB;
      const int g = oc / Cog;
      const int ci = blk_cbase(oc & ~15, Cog, Cg) + kb;   // the K-side channel
      if (ci < Cin && ci / Cg == g) {
        // forward: w[oc][t][ci - g*Cg]; transposed: the conv's output channel is ci and its
        // filter rows hold Cog (= the conv's input width per group) values
        v = tr ? (float)w[((long)ci * T + t) * Cog + (oc - g * Cog)] : (float)w[((long)oc * T + t) * Cg + (ci - g * Cg)];
      }
    }
    wb[i] = (bf16)v;
  }
}

// ------------------------------------------------------------------ grouped fwd / dgrad
// Block: 4 waves x 2 sub-tiles of 16 output pixels = 128 pixels, one 16-channel output
// block (blockIdx.y).  Optional per-channel sum / sum-of-squares into NCOPY copies.
template <bool TR>
__global__ void __launch_bounds__(NT)
gconv_kernel(const bf16* __restrict__ in, const bf16* __restrict__ wb, bf16* __restrict__ out,
             float* __restrict__ sum, float* __restrict__ sumsq, GGeom g) {
  __shared__ __attribute__((aligned(16))) bf16 stage[4][32 * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ob = blockIdx.y;
  const int oc0 = ob * 16;
  const int cbase = blk_cbase(oc0, g.Cog, g.Cg);     // first K-side channel of the block
  const long m0 = (long)blockIdx.x * 128 + wave * 32;
  const int hl = lane >> 4;                          // k-chunk (8 channels) of the lane
  // the two sub-tiles' rows of this lane
  int n[2], ph[2], pw[2];
  bool ok[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const long m = m0 + 16 * s + (lane & 15);
    ok[s] = m < g.M;
    const long mm = ok[s] ? m : 0;
    pw[s] = (int)(mm % g.Wo);
    const long t = mm / g.Wo;
    ph[s] = (int)(t % g.Ho);
    n[s] = (int)(t / g.Ho);
  }
  f32x4 acc[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16* wrow = wb + (long)(oc0 + (lane & 15)) * g.Kp + 8 * hl;
  const bf16x8 zero = {};
  for (int k0 = 0; k0 < g.Kp; k0 += 32) {
    const int k = k0 + 8 * hl;
    const bf16x8 b = ldfrag(wrow + k0);
    const int t = k / g.KB, kb = k - t * g.KB;
    const bool kv = t < g.T;
    const int r = kv ? t / g.KW : 0, c = kv ? t - r * g.KW : 0;
    bf16x8 a[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int hi, wi;
      bool v = kv && ok[s];
      if (!TR) {
        hi = ph[s] * g.S - g.P + r * g.D;
        wi = pw[s] * g.S - g.P + c * g.D;
      } else {
        const int nh = ph[s] + g.P - r * g.D, nw = pw[s] + g.P - c * g.D;
        v = v && nh >= 0 && nw >= 0 && nh % g.S == 0 && nw % g.S == 0;
        hi = nh / g.S;
        wi = nw / g.S;
      }
      v = v && (unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi && cbase + kb < g.Ci;
      a[s] = v ? ldfrag(in + (((long)n[s] * g.Hi + hi) * g.Wi + wi) * g.Ci + cbase + kb) : zero;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b, acc[s], 0, 0, 0);
  }
  // C/D map: lane -> column j = lane & 15, rows 4*(lane>>4) + i
  const int j = lane & 15;
  if (sum) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long m = m0 + 16 * s + 4 * hl + i;
        const float v = m < g.M ? acc[s][i] : 0.f;
        s1 += v;
        s2 += v * v;
      }
    s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
    s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16 && oc0 + j < g.Co) {
      const int slot = (int)((blockIdx.x * 4 + wave) % NCOPY);
      atomicAdd(sum + (long)slot * g.Co + oc0 + j, s1);
      atomicAdd(sumsq + (long)slot * g.Co + oc0 + j, s2);
    }
  }
  // stage the 32 x 16 bf16 tile, then 16-byte row-chunk stores (2 lanes per row)
  bf16* st = stage[wave];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) st[(16 * s + 4 * hl + i) * 16 + j] = (bf16)acc[s][i];
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  {
    const long m = m0 + (lane >> 1);
    if (m < g.M && oc0 + 8 * (lane & 1) < g.Co)      // Co % 8 == 0: whole 8-channel chunks
      *reinterpret_cast<uint4*>(out + m * g.Co + oc0 + 8 * (lane & 1)) =
          *reinterpret_cast<const uint4*>(st + (lane >> 1) * 16 + 8 * (lane & 1));
  }
}

// ------------------------------------------------------------------ grouped fwd / dgrad, row-band tiles
// gconv_kernel gives each block ONE 16-channel output block, so every A-operand load is a
// 16-byte half of a 32-byte per-pixel chunk, scattered C*2 bytes apart: ~1 TB/s
// (profiles/round5/generic/gconv_resnext_b128.jsonl).  Here a block owns R full output rows
// of one image and a 64-channel slab (4 output blocks, one per wave, whole groups: in == out
// channels per group, Cg | 64 or Cg == 64): the slab's input rows (with the conv padding) are
// staged once into LDS as 128-byte pixel rows with coalesced 16-byte loads, every A fragment
// is a ds_read_b128 from there (16-byte chunk c of pixel i at c ^ ((i >> 1) & 7), pixel
// parity picking the 128-byte half of the bank row: conflict-free at stride 1), and the
// output slab goes back through the same LDS as 128-byte pixel rows.  FLIP: the stride-1
// input gradient as a forward conv of dy with the transposed filter (tr = 1 expansion), taps
// mirrored and pad (KH-1)*D - P.
constexpr int TB_CS = 64;           // channel slab
constexpr int TB_MAXPX = 256;       // output pixels per block (16 MFMA rows)
constexpr int TB_LDS = 48 * 1024;

struct TGeom {
  int Hi, Wi, C;                    // operand image [N][Hi][Wi][C]
  int Ho, Wo;                       // output image [N][Ho][Wo][C]
  int KH, KW, S, P, D, T, Kp;
  int Cog, Cg;                      // output / K-side channels per group
  int R, rows_in, Wp, bands;        // output rows per block, staged input rows / cols, blocks per image
  int wc0;                          // operand column of staged column 0 (-P, or the strided origin)
};

__host__ __device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__device__ __forceinline__ int tb_off(int pix, int c) { return pix * 128 + ((c ^ ((pix >> 1) & 7)) << 4); }

// LDS-DMA staging (buffer_load ... lds, no VGPR round trip, every load of the stage in flight
// at once): `npix` staged pixels of 128-byte slab rows into `img` in the tb_off layout.  A
// wave instruction fills 8 consecutive pixel rows (1 KB, lane-linear), so the swizzle moves to
// the source side: lane l fetches logical chunk (l & 7) ^ ((P >> 1) & 7) of pixel P.  voff(P, c)
// is that chunk's byte offset from the resource base, or TB_OOB for zeros (padding).
typedef __amdgpu_buffer_rsrc_t TRsrc;
constexpr unsigned TB_OOB = 0x80000000u;
__device__ __forceinline__ TRsrc tb_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}
template <class F>
__device__ __forceinline__ void tb_dma(char* img, int npix, TRsrc rs, F voff) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  char* dst0 = img + __builtin_amdgcn_readfirstlane(wave) * 1024;
  for (int r = 0; r * 32 < npix; ++r) {
    const int P = r * 32 + wave * 8 + (lane >> 3), c = (lane & 7) ^ ((P >> 1) & 7);
    const unsigned vo = P < npix ? voff(P, c) : TB_OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst0 + r * 4096), 16, vo,
                                             0, 0, 0);
  }
}

// MODE 0: forward; 1: stride-1 input gradient (FLIP); 2: strided input gradient - output
// pixel (oh, ow) takes tap (r, c) from dy pixel ((oh + P - rD) / S, (ow + P - cD) / S) when
// both divide (the transposed conv; the operand rows staged are those the band reaches)
template <int KB, int MODE>
__global__ void __launch_bounds__(NT)
gconv_band_kernel(const bf16* __restrict__ in, const bf16* __restrict__ wb, bf16* __restrict__ out,
                  float* __restrict__ sum, float* __restrict__ sumsq, TGeom g) {
  __shared__ __attribute__((aligned(16))) char lds[TB_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x / g.bands, oh0 = (blockIdx.x - n * g.bands) * g.R;
  const int cs0 = blockIdx.y * TB_CS;
  const int rows = min(g.R, g.Ho - oh0), npx = rows * g.Wo;
  const int hi0 = MODE == 2 ? floordiv(oh0 + g.P - (g.KH - 1) * g.D, g.S) : oh0 * g.S - g.P;
  // ---- stage the slab's input rows hi0 .. hi0+rows_in-1, columns wc0 .. wc0+Wp-1 (zeros outside)
  {
    const TRsrc rs = tb_rsrc(in + (long)n * g.Hi * g.Wi * g.C + cs0);
    tb_dma(lds, g.rows_in * g.Wp, rs, [&](int pix, int c) -> unsigned {
      const int ir = pix / g.Wp, ic = pix - ir * g.Wp;
      const int hi = hi0 + ir, wi = ic + g.wc0;
      return (unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi
                 ? (unsigned)((hi * g.Wi + wi) * g.C + 8 * c) * 2u : TB_OOB;
    });
  }
  // ---- B fragments of this wave's 16-channel output block (all K-steps, registers)
  constexpr int MAXKS = (9 * KB + 31) / 32;   // up to 3x3 taps
  const int ob = wave, oc0 = cs0 + 16 * ob;
  const int nks = g.Kp / 32;
  const int cb = blk_cbase(oc0, g.Cog, g.Cg) - cs0;   // first K-side channel in the slab
  const int hl = lane >> 4, j = lane & 15;
  bf16x8 bfr[MAXKS];
  const bf16* wrow = wb + (long)(oc0 + j) * g.Kp + 8 * hl;
#pragma unroll
  for (int ks = 0; ks < MAXKS; ++ks) bfr[ks] = ks < nks ? ldfrag(wrow + 32 * ks) : bf16x8{};
  // per K-step: this lane's tap offset (in staged pixels) and LDS chunk; -1 = padding k
  // (MODE 2: toff = r*D, tcol = c*D of the unmirrored tap)
  int toff[MAXKS], tch[MAXKS], tcol[MAXKS];
#pragma unroll
  for (int ks = 0; ks < MAXKS; ++ks) {
    const int k = 32 * ks + 8 * hl, t = k / KB, kb = k - t * KB;
    tcol[ks] = 0;
    if (ks < nks && t < g.T) {
      int r = t / g.KW, c = t - r * g.KW;
      if (MODE == 1) { r = g.KH - 1 - r; c = g.KW - 1 - c; }
      if (MODE == 2) {
        toff[ks] = r * g.D;
        tcol[ks] = c * g.D;
      } else {
        toff[ks] = r * g.D * g.Wp + c * g.D;
      }
      tch[ks] = (cb + kb) >> 3;
    } else {
      toff[ks] = -1;
      tch[ks] = 0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's DMA (and B loads) landed
  __syncthreads();
  // ---- MFMA rows of 16 output pixels (flattened over the band's rows)
  const int nrow = (npx + 15) / 16;
  f32x4 acc[TB_MAXPX / 16];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int m = 0; m < TB_MAXPX / 16; ++m) {
    acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (m < nrow) {   // block-uniform
      const int q = min(16 * m + j, npx - 1);
      const int oh = q / g.Wo, ow = q - oh * g.Wo;
      const int base = oh * g.S * g.Wp + ow * g.S;
      const int ro = oh0 + oh + g.P - hi0 * g.S, co = ow + g.P - g.wc0 * g.S;   // MODE 2 (oh: row in band)
#pragma unroll
      for (int ks = 0; ks < MAXKS; ++ks) {
        if (ks < nks) {
          bf16x8 a = {};
          if (MODE == 2) {
            const int nh = ro - toff[ks], nw = co - tcol[ks];
            const int qh = g.S == 2 ? nh >> 1 : nh / g.S, qw = g.S == 2 ? nw >> 1 : nw / g.S;
            if (toff[ks] >= 0 && qh * g.S == nh && qw * g.S == nw)
              a = *reinterpret_cast<const bf16x8*>(lds + tb_off(qh * g.Wp + qw, tch[ks]));
          } else if (toff[ks] >= 0) {
            a = *reinterpret_cast<const bf16x8*>(lds + tb_off(base + toff[ks], tch[ks]));
          }
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[ks], acc[m], 0, 0, 0);
        }
      }
      if (sum) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = 16 * m + 4 * hl + i < npx ? acc[m][i] : 0.f;
          s1 += v;
          s2 += v * v;
        }
      }
    }
  }
  if (sum) {
    s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
    s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
      const int slot = (int)((blockIdx.x * 4 + wave) % NCOPY);
      atomicAdd(sum + (long)slot * g.C + oc0 + j, s1);
      atomicAdd(sumsq + (long)slot * g.C + oc0 + j, s2);
    }
  }
  // ---- output slab through LDS: [px][64 ch] rows, then 16-byte stores, 128 B per pixel
  __syncthreads();   // every wave is done reading the staged input
#pragma unroll
  for (int m = 0; m < TB_MAXPX / 16; ++m) {
    if (m < nrow) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 16 * m + 4 * hl + i;
        const int ch = 16 * ob + j;
        *reinterpret_cast<bf16*>(lds + tb_off(q, ch >> 3) + (ch & 7) * 2) = (bf16)acc[m][i];
      }
    }
  }
  __syncthreads();
  bf16* ob_base = out + ((long)n * g.Ho + oh0) * g.Wo * g.C + cs0;
  for (int i = tid; i < npx * 8; i += NT) {
    const int q = i >> 3, c = i & 7;
    *reinterpret_cast<uint4*>(ob_base + (long)q * g.C + 8 * c) = *reinterpret_cast<const uint4*>(lds + tb_off(q, c));
  }
}

// band geometry when the row-band kernel applies (else false): in == out channels per group,
// 64-channel slabs of whole groups, taps <= 3x3, the staged input rows within TB_LDS
inline bool band_geom(TGeom& t, int Hi, int Wi, int C, int Co, int Ho, int Wo, int KH, int KW, int S, int P, int D,
                      int Cg, int Cog, int KB, int Kp) {
  static const int on = getenv("MLC_GCONV_BAND") ? atoi(getenv("MLC_GCONV_BAND")) : 1;
  if (!on) return false;   // MLC_GCONV_BAND=0: the per-16-channel kernel only
  if (C != Co || Cg != Cog || C % TB_CS || !(KB == 16 || KB == 32 || KB == 64) || KH * KW > 9) return false;
  if (!(Cg <= 16 ? 16 % Cg == 0 : TB_CS % Cg == 0)) return false;
  const int Wp = (Wo - 1) * S + (KW - 1) * D + 1;
  int R = min(Ho, TB_MAXPX / Wo);
  while (R >= 1 && ((R - 1) * S + (KH - 1) * D + 1) * Wp * 128 > TB_LDS) --R;
  if (R < 1 || R * Wo * 128 > TB_LDS) return false;
  t.Hi = Hi; t.Wi = Wi; t.C = C; t.Ho = Ho; t.Wo = Wo; t.KH = KH; t.KW = KW; t.S = S; t.P = P; t.D = D;
  t.T = KH * KW; t.Kp = Kp; t.Cog = Cog; t.Cg = Cg;
  t.R = R; t.rows_in = (R - 1) * S + (KH - 1) * D + 1; t.Wp = Wp; t.bands = (Ho + R - 1) / R;
  t.wc0 = -P;
  return true;
}

// the strided input gradient (MODE 2): operand dy [Hi=Hdy][Wi=Wdy], output dx [Ho][Wo]; the
// staged dy rows of a band of R dx rows are at most (R-1+(KH-1)D)/S + 2, columns wc0 ..
inline bool band_geom_tr(TGeom& t, int Hi, int Wi, int C, int Co, int Ho, int Wo, int KH, int KW, int S, int P,
                         int D, int Cg, int Cog, int KB, int Kp) {
  if (!band_geom(t, Hi, Wi, C, Co, Ho, Wo, KH, KW, 1, 0, 1, Cg, Cog, KB, Kp)) return false;  // shape gates
  const int wc0 = floordiv(P - (KW - 1) * D, S);
  const int Wp = floordiv(Wo - 1 + P, S) - wc0 + 1;
  auto rows_in = [&](int R) { return (R - 1 + (KH - 1) * D) / S + 2; };
  int R = min(Ho, TB_MAXPX / Wo);
  while (R >= 1 && rows_in(R) * Wp * 128 > TB_LDS) --R;
  if (R < 1) return false;
  t.S = S; t.P = P; t.D = D; t.R = R; t.rows_in = rows_in(R); t.Wp = Wp; t.bands = (Ho + R - 1) / R; t.wc0 = wc0;
  return true;
}

template <int MODE>
inline void launch_band(const TGeom& t, int N, int KB, const bf16* in, const bf16* wb, bf16* out, float* sum,
                        float* sumsq, hipStream_t st) {
  const dim3 grid((unsigned)(N * t.bands), t.C / TB_CS);
  if (KB == 16) hipLaunchKernelGGL((gconv_band_kernel<16, MODE>), grid, dim3(NT), 0, st, in, wb, out, sum, sumsq, t);
  else if (KB == 32) hipLaunchKernelGGL((gconv_band_kernel<32, MODE>), grid, dim3(NT), 0, st, in, wb, out, sum, sumsq, t);
  else hipLaunchKernelGGL((gconv_band_kernel<64, MODE>), grid, dim3(NT), 0, st, in, wb, out, sum, sumsq, t);
}

// ------------------------------------------------------------------ grouped wgrad, row bands
// dw[oc][t][ci] (+)= sum_p dy[p][oc] x[p@t][ci] with the forward's row-band staging: a block
// walks a run of (image, band) pairs of one 64-channel slab, stages the band's x rows and its
// dy pixels [px][64] in LDS with coalesced 16-byte loads, and each wave (one 16-channel output
// block) runs K = 32 pixels per MFMA with both operands read transposed (ds_read_b64_tr_b16,
// as gconv_wgrad_kernel's tr_frag, from the swizzled 128-byte pixel rows); the T x KB/16
// accumulator tiles stay in registers over the whole run, then one atomic per in-group weight.
typedef short s16x4b __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 band_tr_frag(const char* lds, int pa, int pb, int ch) {
  // lane rows pa (8g+q) and pb (8g+4+q), channels ch..ch+3 (ch % 4 == 0)
  const int within = (ch & 7) * 2;
  const s16x4b lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4b))(lds + tb_off(pa, ch >> 3) + within));
  const s16x4b hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4b))(lds + tb_off(pb, ch >> 3) + within));
  typedef short s16x8b __attribute__((ext_vector_type(8)));
  const s16x8b r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int KB>
__global__ void __launch_bounds__(NT)
gconv_band_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ dw, TGeom g,
                        int nb_total, int per_block) {
  __shared__ __attribute__((aligned(16))) char ldx[TB_LDS];
  __shared__ __attribute__((aligned(16))) char ldy[TB_MAXPX * 128];
  constexpr int NSUB = KB / 16, MAXT = 9;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cs0 = blockIdx.y * TB_CS, ob = wave, oc0 = cs0 + 16 * ob;
  const int cb = blk_cbase(oc0, g.Cog, g.Cg) - cs0;
  const int gq = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  // tap offsets (staged pixels) for this kernel's taps
  int toff[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int r = t / g.KW, c = t - r * g.KW;
    toff[t] = t < g.T ? r * g.D * g.Wp + c * g.D : 0;
  }
  f32x4 acc[MAXT][NSUB];
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) acc[t][sb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int b0 = blockIdx.x * per_block, b1 = min(nb_total, b0 + per_block);
  for (int bb = b0; bb < b1; ++bb) {
    const int n = bb / g.bands, oh0 = (bb - n * g.bands) * g.R;
    const int rows = min(g.R, g.Ho - oh0), npx = rows * g.Wo, npx32 = (npx + 31) & ~31;
    const int hi0 = oh0 * g.S - g.P;
    __syncthreads();   // the previous band's LDS reads are done
    tb_dma(ldx, g.rows_in * g.Wp, tb_rsrc(x + (long)n * g.Hi * g.Wi * g.C + cs0), [&](int pix, int c) -> unsigned {
      const int ir = pix / g.Wp, ic = pix - ir * g.Wp;
      const int hi = hi0 + ir, wi = ic + g.wc0;
      return (unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi
                 ? (unsigned)((hi * g.Wi + wi) * g.C + 8 * c) * 2u : TB_OOB;
    });
    tb_dma(ldy, npx32, tb_rsrc(dy + ((long)n * g.Ho + oh0) * g.Wo * g.C + cs0), [&](int q, int c) -> unsigned {
      return q < npx ? (unsigned)(q * g.C + 8 * c) * 2u : TB_OOB;
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int px0 = 0; px0 < npx32; px0 += 32) {
      const int ra = px0 + 8 * gq + qq, rb = ra + 4;
      const bf16x8 fa = band_tr_frag(ldy, ra, rb, 16 * ob + 4 * pp);
      // the x pixels of rows ra / rb at tap (0, 0) (dy is zero past npx: clamp)
      const int qa = min(ra, npx - 1), qb = min(rb, npx - 1);
      const int oha = qa / g.Wo, ohb = qb / g.Wo;
      const int basea = oha * g.S * g.Wp + (qa - oha * g.Wo) * g.S;
      const int baseb = ohb * g.S * g.Wp + (qb - ohb * g.Wo) * g.S;
#pragma unroll
      for (int t = 0; t < MAXT; ++t) {
        if (t < g.T) {
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb) {
            const bf16x8 fb = band_tr_frag(ldx, basea + toff[t], baseb + toff[t], cb + 16 * sb + 4 * pp);
            acc[t][sb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[t][sb], 0, 0, 0);
          }
        }
      }
    }
  }
  // D[m = oc][n = ci]: lane column n = lane & 15, rows 4*(lane>>4) + i; off-group products dropped
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    if (t < g.T) {
#pragma unroll
      for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int oc = oc0 + 4 * gq + i, ci = cs0 + cb + 16 * sb + i16;
          const int grp = oc / g.Cog;
          if (ci / g.Cg == grp && ci < g.C) atomicAdd(dw + ((long)oc * g.T + t) * g.Cg + (ci - grp * g.Cg), acc[t][sb][i]);
        }
    }
  }
}

// ------------------------------------------------------------------ grouped wgrad
// dw[oc][t][cl] (+)= sum_p dy[p][oc] x[p@t][ci].  Block: 4 waves, one 16-channel output
// block (blockIdx.y), up to NCB column blocks (tap, 16-channel input block) (blockIdx.z
// selects which), a pixel chunk (blockIdx.x).  Each wave stages 32 pixels of dy [32][16]
// and of every column block's x gather [32][16] in its own LDS region and feeds the
// MFMA with ds_read_b64_tr_b16 transposed reads (K = pixels).
typedef short s16x4t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 tr_frag(const bf16* tile, int lane) {
  // 16x16x32 operand whose K index is the tile row (32 rows x 16 cols, 32-byte rows):
  // lane l gets column (l & 15), rows 8*(l>>4) + 0..7
  const int q = (lane & 15) >> 2, p = lane & 3, g = lane >> 4;
  const bf16* a0 = tile + (8 * g + q) * 16 + 4 * p;
  const bf16* a1 = tile + (8 * g + 4 + q) * 16 + 4 * p;
  const s16x4t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4t))(a0));
  const s16x4t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4t))(a1));
  typedef short s16x8t __attribute__((ext_vector_type(8)));
  const s16x8t r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

constexpr int WG_NCB = 9;   // column blocks per block (3x3 taps of one 16-channel block)

__global__ void __launch_bounds__(NT)
gconv_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ dw, GGeom g,
                   int ncb_total, long chunk) {
  // per wave: dy tile + WG_NCB x tiles, 32 x 16 bf16 each
  __shared__ __attribute__((aligned(16))) bf16 lds[4][(1 + WG_NCB) * 32 * 16];
  __shared__ float red[4][WG_NCB][16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ob = blockIdx.y, oc0 = ob * 16;
  const int cbase = blk_cbase(oc0, g.Cog, g.Cg);
  const int nsub = g.KB / 16;                       // 16-channel input blocks per tap
  const int cb0 = blockIdx.z * WG_NCB;
  const int ncb = min(WG_NCB, ncb_total - cb0);
  bf16* tA = lds[wave];
  f32x4 acc[WG_NCB];
#pragma unroll
  for (int c = 0; c < WG_NCB; ++c) acc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // this lane's staging role: pixel row (lane >> 1), 8-channel half (lane & 1)
  const int prow = lane >> 1, half = lane & 1;
  // per column block of this block: tap (r, s) and input-channel offset
  int tr_[WG_NCB], ts_[WG_NCB], tc_[WG_NCB];
#pragma unroll
  for (int c = 0; c < WG_NCB; ++c) {
    const int cb = cb0 + (c < ncb ? c : 0);
    const int t = cb / nsub, sb = cb - t * nsub;
    tr_[c] = t / g.KW;
    ts_[c] = t - tr_[c] * g.KW;
    tc_[c] = cbase + 16 * sb + 8 * half;
  }
  const long pbeg = (long)blockIdx.x * chunk, pend = min(g.M, pbeg + chunk);
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  for (long p0 = pbeg + 32 * wave; p0 < pend; p0 += 128) {
    const long p = p0 + prow;
    const bool pv = p < pend;
    int n = 0, ho = 0, wo = 0;
    if (pv) {
      wo = (int)(p % g.Wo);
      const long t = p / g.Wo;
      ho = (int)(t % g.Ho);
      n = (int)(t / g.Ho);
    }
    uint4 va = pv && oc0 + 8 * half < g.Co ? ldg16(dy + p * g.Co + oc0 + 8 * half) : z4;
    uint4 vb[WG_NCB];
#pragma unroll
    for (int c = 0; c < WG_NCB; ++c) {
      const int hi = ho * g.S - g.P + tr_[c] * g.D, wi = wo * g.S - g.P + ts_[c] * g.D;
      const bool v = pv && c < ncb && (unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi &&
                     tc_[c] < g.Ci;
      vb[c] = v ? ldg16(x + (((long)n * g.Hi + hi) * g.Wi + wi) * g.Ci + tc_[c]) : z4;
    }
    __builtin_amdgcn_wave_barrier();   // the previous iteration's reads are done (same wave)
    *reinterpret_cast<uint4*>(tA + prow * 16 + 8 * half) = va;
#pragma unroll
    for (int c = 0; c < WG_NCB; ++c)
      *reinterpret_cast<uint4*>(tA + (1 + c) * 512 + prow * 16 + 8 * half) = vb[c];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const bf16x8 fa = tr_frag(tA, lane);
#pragma unroll
    for (int c = 0; c < WG_NCB; ++c) {
      if (c < ncb) {   // wave-uniform
        const bf16x8 fb = tr_frag(tA + (1 + c) * 512, lane);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[c], 0, 0, 0);
      }
    }
  }
  // C map: column (input channel within the block) = lane & 15, row (oc) = 4*(lane>>4)+i.
  // Reduce the 4 waves through LDS, then one atomic per kept element.
  const int col = lane & 15;
#pragma unroll
  for (int c = 0; c < WG_NCB; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][c][4 * (lane >> 4) + i][col] = acc[c][i];
  __syncthreads();
  for (int e = threadIdx.x; e < ncb * 256; e += NT) {
    const int c = e >> 8, row = (e >> 4) & 15, cl = e & 15;
    const float v = red[0][c][row][cl] + red[1][c][row][cl] + red[2][c][row][cl] + red[3][c][row][cl];
    const int cb = cb0 + c, t = cb / nsub, sb = cb - t * nsub;
    const int oc = oc0 + row, ci = cbase + 16 * sb + cl;
    if (oc >= g.Co || ci >= g.Ci || ci / g.Cg != oc / g.Cog) continue;   // off the block diagonal
    atomicAdd(dw + ((long)oc * g.T + t) * g.Cg + (ci - (oc / g.Cog) * g.Cg), v);
  }
}

// ------------------------------------------------------------------ depthwise
// weights [T][C] (tap-major, bf16), C % 8 == 0; y[n,ho,wo,c] = sum_t x[..@t][c] * w[t][c]
constexpr int DW_OW = 4;   // outputs per thread along W

__device__ __forceinline__ void red_stats(float (&s1)[8], float (&s2)[8], float* sum, float* sumsq, int C, int G) {
  __shared__ float rb[NT][17];
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
    const long slot = blockIdx.x % NCOPY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(sum + slot * C + cg * 8 + e, a[e]);
      atomicAdd(sumsq + slot * C + cg * 8 + e, b[e]);
    }
  }
}

__global__ void __launch_bounds__(NT)
dw_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, bf16* __restrict__ y, float* __restrict__ sum,
              float* __restrict__ sumsq, int N, int H, int W, int C, int Ho, int Wo, int KH, int KW, int S, int P,
              int D) {
  const int G = C >> 3;
  const int Wq = (Wo + DW_OW - 1) / DW_OW;
  const long total = (long)N * Ho * Wq * G;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const int cg = (int)(gtid % G);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  for (long i = gtid; i < total; i += (long)gridDim.x * NT) {
    long t = i / G;
    const int wq = (int)(t % Wq); t /= Wq;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const int wo0 = wq * DW_OW;
    float acc[DW_OW][8];
#pragma unroll
    for (int o = 0; o < DW_OW; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
    for (int r = 0; r < KH; ++r) {
      const int hi = ho * S - P + r * D;
      if ((unsigned)hi >= (unsigned)H) continue;
      const bf16* xr = x + ((long)n * H + hi) * W * C + cg * 8;
      for (int s = 0; s < KW; ++s) {
        float wv[8];
        unpack8(ldg16(w + (long)(r * KW + s) * C + cg * 8), wv);
#pragma unroll
        for (int o = 0; o < DW_OW; ++o) {
          const int wi = (wo0 + o) * S - P + s * D;
          if (wo0 + o < Wo && (unsigned)wi < (unsigned)W) {
            float xv[8];
            unpack8(ldg16(xr + (long)wi * C), xv);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[o][e] += xv[e] * wv[e];
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < DW_OW; ++o) {
      if (wo0 + o >= Wo) break;
      *reinterpret_cast<uint4*>(y + (((long)n * Ho + ho) * Wo + wo0 + o) * C + cg * 8) = pack8(acc[o]);
      if (sum) {   // statistics of the fp32 accumulators, as the implicit-GEMM epilogues
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += acc[o][e]; s2[e] += acc[o][e] * acc[o][e]; }
      }
    }
  }
  if (sum) red_stats(s1, s2, sum, sumsq, C, G);
}

// dx[n,h,w,c] = sum over taps reaching (h, w) of dy[n,ho,wo,c] * w[t][c]
__global__ void __launch_bounds__(NT)
dw_dgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w, bf16* __restrict__ dx, int N, int H, int W,
                int C, int Ho, int Wo, int KH, int KW, int S, int P, int D) {
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
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int r = 0; r < KH; ++r) {
      const int nh = hi + P - r * D;
      if (nh < 0 || nh % S) continue;
      const int ho = nh / S;
      if (ho >= Ho) continue;
      for (int s = 0; s < KW; ++s) {
        const int nw = wi + P - s * D;
        if (nw < 0 || nw % S) continue;
        const int wo = nw / S;
        if (wo >= Wo) continue;
        float gv[8], wv[8];
        unpack8(ldg16(dy + (((long)n * Ho + ho) * Wo + wo) * C + cg * 8), gv);
        unpack8(ldg16(w + (long)(r * KW + s) * C + cg * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += gv[e] * wv[e];
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// partial dw over this thread's output pixels for taps [t0, t0 + TC), reduced per block
// and added into copy (block % NCOPY) of ws[NCOPY][T][C]
constexpr int DW_TC = 9;

__global__ void __launch_bounds__(NT)
dw_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int N, int H, int W,
                int C, int Ho, int Wo, int KH, int KW, int S, int P, int D, int t0) {
  __shared__ float rb[NT][DW_TC * 8 + 1];
  const int G = C >> 3;
  const int T = KH * KW;
  const int tc = min(DW_TC, T - t0);
  const long total = (long)N * Ho * Wo * G;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const int cg = (int)(gtid % G);
  float acc[DW_TC][8];
#pragma unroll
  for (int k = 0; k < DW_TC; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  int tr[DW_TC], ts[DW_TC];
#pragma unroll
  for (int k = 0; k < DW_TC; ++k) {
    const int tt = t0 + (k < tc ? k : 0);
    tr[k] = tt / KW;
    ts[k] = tt - tr[k] * KW;
  }
  for (long i = gtid; i < total; i += (long)gridDim.x * NT) {
    long t = i / G;
    const int wo = (int)(t % Wo); t /= Wo;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    float gv[8];
    unpack8(ldg16(dy + i * 8), gv);
#pragma unroll
    for (int k = 0; k < DW_TC; ++k) {
      if (k >= tc) break;
      const int hi = ho * S - P + tr[k] * D, wi = wo * S - P + ts[k] * D;
      if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) continue;
      float xv[8];
      unpack8(ldg16(x + (((long)n * H + hi) * W + wi) * C + cg * 8), xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] += gv[e] * xv[e];
    }
  }
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < DW_TC; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[tid][k * 8 + e] = acc[k][e];
  __syncthreads();
  const int lanes = NT < G ? NT : G;
  const int base_cg = (int)(((long)blockIdx.x * NT) % G);
  float* dst = ws + (long)(blockIdx.x % NCOPY) * T * C;
  for (int q = tid; q < lanes * tc * 8; q += NT) {
    const int l = q % lanes, ke = q / lanes;
    const int k = ke >> 3, e = ke & 7;
    float a = 0.f;
    for (int u = l; u < NT; u += G) a += rb[u][k * 8 + e];
    const int c = ((base_cg + l) % G) * 8 + e;
    atomicAdd(dst + (long)(t0 + k) * C + c, a);
  }
}

// ---- strip kernels (KW in {3, 5, 7}, stride 1 / 2, dilation 1): a thread owns one 8-channel
// group and a strip of DW_SW consecutive output columns of one output row.  The x row
// segment a strip needs for one filter row is loaded ONCE ((DW_SW-1)*S + KW vectors instead
// of DW_SW*KW), every load is straight-line (out-of-range taps load a clamped address and are
// zeroed), so a thread has ~20 16-byte loads in flight instead of one.
constexpr int DW_SW = 8;

// n / d for 0 <= n < 2^31 as a multiply-high, an add and a shift, with the divisor's magic
// number computed on the host: the strip kernels split their item index into (image, row,
// strip, channel group) once per item, and three 64-bit divisions there cost more
// instructions than the item's FMAs
struct FastDiv {
  unsigned d, m, s;
  FastDiv() = default;
  explicit FastDiv(unsigned dv) : d(dv), m(0), s(0) {
    while ((1u << s) < d) ++s;   // ceil(log2 d)
    m = (unsigned)((((unsigned long long)1 << 32) * (((unsigned long long)1 << s) - d)) / d + 1);
  }
  __device__ __forceinline__ unsigned div(unsigned n) const { return (__umulhi(n, m) + n) >> s; }
};
// item i = ((n * R + row) * Q + q) * G + cg
struct Idx3 {
  FastDiv g, q, r;
};
struct Item {
  int n, row, q, cg;
};
__device__ __forceinline__ Item split_item(long i, const Idx3& ix) {
  const unsigned u = (unsigned)i, t0 = ix.g.div(u), t1 = ix.q.div(t0), t2 = ix.r.div(t1);
  return Item{(int)t2, (int)(t1 - t2 * ix.r.d), (int)(t0 - t1 * ix.q.d), (int)(u - t0 * ix.g.d)};
}

__device__ __forceinline__ uint4 ld_or_zero(const bf16* base, long off, bool ok) {
  const uint4 v = ldg16(base + (ok ? off : 0));
  return ok ? v : make_uint4(0u, 0u, 0u, 0u);
}

// forward: acc[o] = sum_{r,s} x[ho*S-P+r][(wo0+o)*S-P+s] * w[r][s]
template <int KW, int S>
__global__ void __launch_bounds__(NT)
dw_fwd_strip_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, bf16* __restrict__ y,
                    float* __restrict__ sum, float* __restrict__ sumsq, int N, int H, int W, int C, int Ho, int Wo,
                    int KH, int P, Idx3 ix) {
  constexpr int XS = (DW_SW - 1) * S + KW;
  const int G = C >> 3;
  const int Wq = (Wo + DW_SW - 1) / DW_SW;
  const long total = (long)N * Ho * Wq * G;
  const long gtid = (long)blockIdx.x * NT + threadIdx.x;
  const int cg = (int)(gtid % G);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  for (long i = gtid; i < total; i += (long)gridDim.x * NT) {
    const Item it = split_item(i, ix);
    const int wq = it.q, ho = it.row, n = it.n;
    const int wo0 = wq * DW_SW;
    const int wi0 = wo0 * S - P;
    float acc[DW_SW][8];
#pragma unroll
    for (int o = 0; o < DW_SW; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
    for (int r = 0; r < KH; ++r) {
      const int hi = ho * S - P + r;
      if ((unsigned)hi >= (unsigned)H) continue;
      const bf16* xr = x + ((long)n * H + hi) * W * C + cg * 8;
      uint4 xv[XS], wv[KW];
#pragma unroll
      for (int j = 0; j < XS; ++j) {
        const int wi = wi0 + j;
        xv[j] = ld_or_zero(xr, (long)wi * C, (unsigned)wi < (unsigned)W);
      }
#pragma unroll
      for (int q = 0; q < KW; ++q) wv[q] = ldg16(w + (long)(r * KW + q) * C + cg * 8);
#pragma unroll
      for (int q = 0; q < KW; ++q) {
        float wf[8];
        unpack8(wv[q], wf);
#pragma unroll
        for (int o = 0; o < DW_SW; ++o) {
          float xf[8];
          unpack8(xv[o * S + q], xf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[o][e] += xf[e] * wf[e];
        }
      }
    }
#pragma unroll
    for (int o = 0; o < DW_SW; ++o) {
      if (wo0 + o < Wo) {
        *reinterpret_cast<uint4*>(y + (((long)n * Ho + ho) * Wo + wo0 + o) * C + cg * 8) = pack8(acc[o]);
        if (sum) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += acc[o][e]; s2[e] += acc[o][e] * acc[o][e]; }
        }
      }
    }
  }
  if (sum) red_stats(s1, s2, sum, sumsq, C, G);
}

// weight gradient of filter row r: acc[q] = sum over pixels dy[p] * x[p@(r,q)], reduced per
// block (LDS) and added into copy (spatial block % NCOPY) of ws[NCOPY][KH*KW][C].
// The KH filter rows re-read the same dy rows and overlapping x rows. With xcd != 0 the grid
// is 1-D and the KH row-blocks of one spatial block sit on one XCD (dispatch round-robins
// blocks over the 8 XCDs) in consecutive dispatch slots, so they run together and share those
// reads through that XCD's L2. Otherwise blockIdx.y is the filter row, and the KH slices of the
// grid sweep the whole tensor one after another.
template <int KW, int S>
__global__ void __launch_bounds__(NT)
dw_wgrad_strip_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int N,
                      int H, int W, int C, int Ho, int Wo, int KH, int P, int xcd, Idx3 ix) {
  constexpr int XS = (DW_SW - 1) * S + KW;
  __shared__ float rb[NT][KW * 8 + 1];
  const int G = C >> 3;
  int r = blockIdx.y, sb = blockIdx.x, nb = gridDim.x;
  if (xcd) {
    const int k = blockIdx.x >> 3;
    r = k % KH;
    sb = (k / KH) * 8 + (blockIdx.x & 7);
    nb = gridDim.x / KH;
  }
  const int Wq = (Wo + DW_SW - 1) / DW_SW;
  const long total = (long)N * Ho * Wq * G;
  const long gtid = (long)sb * NT + threadIdx.x;
  const int cg = (int)(gtid % G);
  float acc[KW][8];
#pragma unroll
  for (int q = 0; q < KW; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[q][e] = 0.f;
  for (long i = gtid; i < total; i += (long)nb * NT) {
    const Item it = split_item(i, ix);
    const int wq = it.q, ho = it.row, n = it.n;
    const int hi = ho * S - P + r;
    if ((unsigned)hi >= (unsigned)H) continue;
    const int wo0 = wq * DW_SW;
    const int wi0 = wo0 * S - P;
    const bf16* dyr = dy + ((long)n * Ho + ho) * Wo * C + cg * 8;
    const bf16* xr = x + ((long)n * H + hi) * W * C + cg * 8;
    uint4 gv[DW_SW], xv[XS];
#pragma unroll
    for (int o = 0; o < DW_SW; ++o) gv[o] = ld_or_zero(dyr, (long)(wo0 + o) * C, wo0 + o < Wo);
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int wi = wi0 + j;
      xv[j] = ld_or_zero(xr, (long)wi * C, (unsigned)wi < (unsigned)W);
    }
#pragma unroll
    for (int o = 0; o < DW_SW; ++o) {
      float gf[8];
      unpack8(gv[o], gf);
#pragma unroll
      for (int q = 0; q < KW; ++q) {
        float xf[8];
        unpack8(xv[o * S + q], xf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[q][e] += gf[e] * xf[e];
      }
    }
  }
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < KW; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[tid][q * 8 + e] = acc[q][e];
  __syncthreads();
  const int lanes = NT < G ? NT : G;
  const int base_cg = (int)(((long)sb * NT) % G);
  float* dst = ws + (long)(sb % NCOPY) * KH * KW * C;
  for (int qq = tid; qq < lanes * KW * 8; qq += NT) {
    const int l = qq % lanes, ke = qq / lanes;
    const int q = ke >> 3, e = ke & 7;
    float a = 0.f;
    for (int u = l; u < NT; u += G) a += rb[u][q * 8 + e];
    const int c = ((base_cg + l) % G) * 8 + e;
    atomicAdd(dst + (long)(r * KW + q) * C + c, a);
  }
}

// input gradient: dx[hi][wi0+o] = sum_{r,s} dy[(hi+P-r)/S][(wi0+o+P-s)/S] * w[r][s] over the
// taps whose offsets divide by S.  wi0 is a multiple of 8, so with P = 2*ph + PP the dy
// column a (o, s) pair reads is a compile-time offset from the strip's first column.
constexpr int fdiv2(int a) { return a >= 0 ? a / 2 : -((-a + 1) / 2); }

template <int KW, int S, int PP>
__global__ void __launch_bounds__(NT)
dw_dgrad_strip_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w, bf16* __restrict__ dx, int N, int H,
                      int W, int C, int Ho, int Wo, int KH, int P, Idx3 ix) {
  constexpr int FB = S == 1 ? -(KW - 1) : fdiv2(PP - (KW - 1));
  constexpr int NW = S == 1 ? DW_SW + KW - 1 : (DW_SW - 1 + PP) / 2 - FB + 1;
  const int G = C >> 3;
  const int Wq = (W + DW_SW - 1) / DW_SW;
  const long total = (long)N * H * Wq * G;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const Item it = split_item(i, ix);
    const int cg = it.cg, wq = it.q, hi = it.row, n = it.n;
    const int wi0 = wq * DW_SW;
    const int col0 = S == 1 ? wi0 + P + FB : wi0 / 2 + (P - PP) / 2 + FB;
    float acc[DW_SW][8];
#pragma unroll
    for (int o = 0; o < DW_SW; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
    for (int r = 0; r < KH; ++r) {
      const int nh = hi + P - r;
      if (nh < 0 || (S == 2 && (nh & 1))) continue;
      const int ho = S == 1 ? nh : nh >> 1;
      if (ho >= Ho) continue;
      const bf16* dr = dy + ((long)n * Ho + ho) * Wo * C + cg * 8;
      uint4 gv[NW], wv[KW];
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const int wo = col0 + j;
        gv[j] = ld_or_zero(dr, (long)wo * C, (unsigned)wo < (unsigned)Wo);
      }
#pragma unroll
      for (int q = 0; q < KW; ++q) wv[q] = ldg16(w + (long)(r * KW + q) * C + cg * 8);
#pragma unroll
      for (int q = 0; q < KW; ++q) {
        float wf[8];
        unpack8(wv[q], wf);
#pragma unroll
        for (int o = 0; o < DW_SW; ++o) {
          if (S == 2 && ((o + PP - q) & 1)) continue;             // compile-time
          const int j = S == 1 ? o - q - FB : (o + PP - q) / 2 - FB;
          float gf[8];
          unpack8(gv[j], gf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[o][e] += gf[e] * wf[e];
        }
      }
    }
#pragma unroll
    for (int o = 0; o < DW_SW; ++o)
      if (wi0 + o < W) *reinterpret_cast<uint4*>(dx + (((long)n * H + hi) * W + wi0 + o) * C + cg * 8) = pack8(acc[o]);
  }
}

// dw[t][c] (+)= sum over the NCOPY copies
__global__ void __launch_bounds__(NT)
copies_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, long n, int accumulate) {
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    float a = accumulate ? out[i] : 0.f;
    for (int k = 0; k < NCOPY; ++k) a += ws[(long)k * n + i];
    out[i] = a;
  }
}

// threads of a grid-stride pass over (row, 8-channel group) keep one group when the thread
// count is a multiple of G = C/8 (as batchnorm.hip's grid_for)
// block counts of the channel-group passes are multiples of this (a thread keeps one group)
inline long group_mult(int G) {
  if (G > NT) return G % NT == 0 ? G / NT : G;
  int a = G, b = NT;
  while (b) { const int r = a % b; a = b; b = r; }
  return G / a;
}
inline int grid_groups(long work, int G, int cap, int per_thread = 4) {
  long blocks = (work + (long)NT * per_thread - 1) / ((long)NT * per_thread);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  const long m = group_mult(G);
  blocks = ((blocks + m - 1) / m) * m;
  return (int)blocks;
}
// deterministic mode: the largest block cap whose rounded grid stays within NCOPY blocks
// (one ws copy per block), 0 when no such grid exists
inline int det_group_cap(int G) {
  const long m = group_mult(G);
  return m <= NCOPY ? (int)((NCOPY / m) * m) : 0;
}

inline int blocks_for(long work) {
  long b = (work + NT - 1) / NT;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

inline int dw_wg_items() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_DW_WG_ITEMS");
    v = e ? atoi(e) : 32;
    if (v < 1) v = 1;
  }
  return v;
}

inline int dw_fwd_items() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_DW_FWD_ITEMS");
    v = e ? atoi(e) : 4;
    if (v < 1) v = 1;
  }
  return v;
}

// block cap of the depthwise input-gradient strips (A/B knob MLC_DW_DGRAD_CAP)
inline int dw_dgrad_cap() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_DW_DGRAD_CAP");
    v = e ? atoi(e) : 8192;
    if (v < 64) v = 64;
  }
  return v;
}

// MLC_DW_XCD=0: the depthwise weight gradient's filter rows as grid.y slices (A/B)
inline bool dw_xcd() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_DW_XCD");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

inline Idx3 idx3(int G, int Q, int R) { return Idx3{FastDiv((unsigned)G), FastDiv((unsigned)Q), FastDiv((unsigned)R)}; }
inline bool items_fit(int N, int R, int Q, int G) { return (long)N * R * Q * G < (1L << 31); }

// MLC_DW_STRIPS=0 selects the per-pixel depthwise kernels (A/B)
inline bool dw_strips() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLC_DW_STRIPS");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

// K-side channels per tap that every 16-channel output block needs (its groups' K-side
// channel span, 8-aligned), rounded up to 16
inline int block_kb(int Cout, int Cog, int Cg) {
  int kb = 16;
  for (int oc0 = 0; oc0 < Cout; oc0 += 16) {
    const int last = (oc0 + 15 < Cout ? oc0 + 15 : Cout - 1) / Cog;
    const int hi = ((last + 1) * Cg + 7) & ~7;
    const int w = hi - blk_cbase(oc0, Cog, Cg);
    if (w > kb) kb = w;
  }
  return (kb + 15) / 16 * 16;
}

// any group widths (C/groups may differ from Co/groups), channel counts multiple of 8; the
// K-side span of a 16-channel output block is bounded so the block-diagonal waste stays small
inline bool grouped_ok(int C, int Co, int groups) {
  if (groups < 2 || C % groups || Co % groups || C % 8 || Co % 8) return false;
  return block_kb(Co, Co / groups, C / groups) <= 256 && block_kb(C, C / groups, Co / groups) <= 256;
}

inline GGeom mkg(int N, int Hi, int Wi, int Ci, int Ho, int Wo, int Co, int KH, int KW, int S, int P, int D,
                 int Cg, int Cog) {
  GGeom g;
  g.N = N; g.Hi = Hi; g.Wi = Wi; g.Ci = Ci; g.Ho = Ho; g.Wo = Wo; g.Co = Co;
  g.KH = KH; g.KW = KW; g.S = S; g.P = P; g.D = D;
  g.Cg = Cg; g.Cog = Cog; g.KB = block_kb(Co, Cog, Cg); g.T = KH * KW; g.Kp = (g.T * g.KB + 31) / 32 * 32;
  g.M = (long)N * Ho * Wo;
  return g;
}

}  // namespace gconv

using namespace gconv;

// elements of the expanded filter (bf16) that mlc_gconv_fwd (tr 0) / _dgrad (tr 1) need in
// `wb`, for a conv with C input and Co output channels
MLC_EXPORT long mlc_gconv_wb_elems(int C, int Co, int KH, int KW, int groups, int tr) {
  if (groups < 1 || C % groups || Co % groups) return -1;
  const int Cout = tr ? C : Co, Cog = Cout / groups, Cg = (tr ? Co : C) / groups;
  const int KB = block_kb(Cout, Cog, Cg);
  return (long)((Cout + 15) / 16 * 16) * ((KH * KW * KB + 31) / 32 * 32);
}

// y[N,Ho,Wo,Co] = grouped conv of x[N,H,W,C] with w[Co][KH][KW][C/groups]; wb: scratch of
// mlc_gconv_wb_elems bf16; sum/sumsq (optional, zeroed, 32*Co fp32 each): BN statistics
MLC_EXPORT int mlc_gconv_fwd(const bf16* x, const bf16* w, bf16* wb, bf16* y, float* sum, float* sumsq, int N, int H,
                             int W, int C, int Co, int KH, int KW, int S, int P, int D, int Ho, int Wo, int groups,
                             hipStream_t st) {
  if (!grouped_ok(C, Co, groups) || ((sum == nullptr) != (sumsq == nullptr))) return -1;
  if (g_mlc_det && sum) {
    // deterministic mode: the epilogue's statistics are float atomics from many blocks per
    // copy; take them in the ordered statistics pass over y instead
    const int rc = mlc_gconv_fwd(x, w, wb, y, nullptr, nullptr, N, H, W, C, Co, KH, KW, S, P, D, Ho, Wo, groups, st);
    return rc ? rc : mlc_bn_stats(y, sum, sumsq, (long)N * Ho * Wo, Co, st);
  }
  const GGeom g = mkg(N, H, W, C, Ho, Wo, Co, KH, KW, S, P, D, C / groups, Co / groups);
  hipLaunchKernelGGL(expand_kernel, dim3(blocks_for((long)(Co + 15) / 16 * 16 * g.Kp)), dim3(NT), 0, st, w, wb, Co,
                     C, g.T, g.Cg, g.Cog, g.KB, g.Kp, 0);
  TGeom t;
  if (band_geom(t, H, W, C, Co, Ho, Wo, KH, KW, S, P, D, g.Cg, g.Cog, g.KB, g.Kp)) {
    launch_band<0>(t, N, g.KB, x, wb, y, sum, sumsq, st);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((g.M + 127) / 128), (Co + 15) / 16);
  hipLaunchKernelGGL(gconv_kernel<false>, grid, dim3(NT), 0, st, x, wb, y, sum, sumsq, g);
  return hipGetLastError();
}

// dx[N,H,W,C] from dy[N,Ho,Wo,Co] (same w, groups): the stride-fractional tap map
MLC_EXPORT int mlc_gconv_dgrad(const bf16* dy, const bf16* w, bf16* wb, bf16* dx, int N, int H, int W, int C, int Co,
                               int KH, int KW, int S, int P, int D, int Ho, int Wo, int groups, hipStream_t st) {
  if (!grouped_ok(C, Co, groups)) return -1;
  // the roles swap: operand image dy (Co channels), output dx (C channels)
  const GGeom g = mkg(N, Ho, Wo, Co, H, W, C, KH, KW, S, P, D, Co / groups, C / groups);
  hipLaunchKernelGGL(expand_kernel, dim3(blocks_for((long)(C + 15) / 16 * 16 * g.Kp)), dim3(NT), 0, st, w, wb, C,
                     Co, g.T, g.Cg, g.Cog, g.KB, g.Kp, 1);
  TGeom t;
  // stride 1: a forward conv of dy over the transposed filter, taps mirrored
  if (S == 1 && D * (KH - 1) >= P && D * (KW - 1) - P == D * (KH - 1) - P &&
      band_geom(t, Ho, Wo, Co, C, H, W, KH, KW, 1, D * (KH - 1) - P, D, g.Cg, g.Cog, g.KB, g.Kp)) {
    launch_band<1>(t, N, g.KB, dy, wb, dx, nullptr, nullptr, st);
    return hipGetLastError();
  }
  if (S > 1 && band_geom_tr(t, Ho, Wo, Co, C, H, W, KH, KW, S, P, D, g.Cg, g.Cog, g.KB, g.Kp)) {
    launch_band<2>(t, N, g.KB, dy, wb, dx, nullptr, nullptr, st);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((g.M + 127) / 128), (C + 15) / 16);
  hipLaunchKernelGGL(gconv_kernel<true>, grid, dim3(NT), 0, st, dy, wb, dx, nullptr, nullptr, g);
  return hipGetLastError();
}

// dw[Co][KH][KW][C/groups] fp32 (+)= grouped weight gradient
MLC_EXPORT int mlc_gconv_wgrad(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C, int Co, int KH,
                               int KW, int S, int P, int D, int Ho, int Wo, int groups, int accumulate, hipStream_t st) {
  if (!grouped_ok(C, Co, groups)) return -1;
  const GGeom g = mkg(N, H, W, C, Ho, Wo, Co, KH, KW, S, P, D, C / groups, Co / groups);
  if (!accumulate) mlc_zero_f32(dw, (long)Co * g.T * g.Cg, st);
  TGeom t;
  static const int band_wg = getenv("MLC_GCONV_BAND_WGRAD") ? atoi(getenv("MLC_GCONV_BAND_WGRAD")) : 1;
  // deterministic mode: no band kernel (several blocks add into one weight element) and a
  // single pixel chunk below, so every element gets exactly one add
  if (band_wg && !g_mlc_det && band_geom(t, H, W, C, Co, Ho, Wo, KH, KW, S, P, D, g.Cg, g.Cog, g.KB, g.Kp)) {
    // runs of bands per block: ~640 blocks over the chip (2 per CU fit the 80 KB of LDS)
    const int slabs = C / TB_CS, nb_total = N * t.bands;
    int per = (int)(((long)nb_total * slabs + 639) / 640);
    if (per < 1) per = 1;
    const dim3 grid((unsigned)((nb_total + per - 1) / per), slabs);
    if (g.KB == 16) hipLaunchKernelGGL(gconv_band_wgrad_kernel<16>, grid, dim3(NT), 0, st, dy, x, dw, t, nb_total, per);
    else if (g.KB == 32) hipLaunchKernelGGL(gconv_band_wgrad_kernel<32>, grid, dim3(NT), 0, st, dy, x, dw, t, nb_total, per);
    else hipLaunchKernelGGL(gconv_band_wgrad_kernel<64>, grid, dim3(NT), 0, st, dy, x, dw, t, nb_total, per);
    return hipGetLastError();
  }
  const int ncb = g.T * (g.KB / 16);
  const int zb = (ncb + WG_NCB - 1) / WG_NCB;
  const int base = ((Co + 15) / 16) * zb;
  // enough pixel chunks to give the chip ~2048 blocks, at least 128 pixels each
  long chunks = (2048 + base - 1) / base;
  const long maxc = (g.M + 127) / 128;
  if (chunks > maxc) chunks = maxc;
  if (g_mlc_det) chunks = 1;
  if (chunks < 1) chunks = 1;
  long chunk = (g.M + chunks - 1) / chunks;
  chunk = (chunk + 127) / 128 * 128;
  chunks = (g.M + chunk - 1) / chunk;
  const dim3 grid((unsigned)chunks, (Co + 15) / 16, zb);
  hipLaunchKernelGGL(gconv_wgrad_kernel, grid, dim3(NT), 0, st, dy, x, dw, g, ncb, chunk);
  return hipGetLastError();
}

// depthwise: w [KH][KW][C] bf16 (tap-major); C % 8 == 0
MLC_EXPORT int mlc_dwconv_fwd(const bf16* x, const bf16* w, bf16* y, float* sum, float* sumsq, int N, int H, int W,
                              int C, int KH, int KW, int S, int P, int D, int Ho, int Wo, hipStream_t st) {
  if (C % 8 || ((sum == nullptr) != (sumsq == nullptr))) return -1;
  if (g_mlc_det && sum) {   // ordered statistics pass instead of the epilogue's atomics
    const int rc = mlc_dwconv_fwd(x, w, y, nullptr, nullptr, N, H, W, C, KH, KW, S, P, D, Ho, Wo, st);
    return rc ? rc : mlc_bn_stats(y, sum, sumsq, (long)N * Ho * Wo, C, st);
  }
  const int G = C / 8;
  const int Wqo = (Wo + DW_SW - 1) / DW_SW;
  if (D == 1 && (S == 1 || S == 2) && (KW == 3 || KW == 5 || KW == 7) && dw_strips() && items_fit(N, Ho, Wqo, G)) {
    const long work = (long)N * Ho * Wqo * G;
    // the BN statistics end every block in 2*C float atomics: fewer, longer blocks (MLC_DW_FWD_ITEMS)
    const dim3 grid(grid_groups(work, G, 2048, sum ? dw_fwd_items() : 4));
    const Idx3 ix = idx3(G, Wqo, Ho);
#define DWF(K, SS) hipLaunchKernelGGL((dw_fwd_strip_kernel<K, SS>), grid, dim3(NT), 0, st, x, w, y, sum, sumsq, N, H, \
                                      W, C, Ho, Wo, KH, P, ix)
    if (S == 1) { if (KW == 3) DWF(3, 1); else if (KW == 5) DWF(5, 1); else DWF(7, 1); }
    else { if (KW == 3) DWF(3, 2); else if (KW == 5) DWF(5, 2); else DWF(7, 2); }
#undef DWF
    return hipGetLastError();
  }
  const long work = (long)N * Ho * ((Wo + DW_OW - 1) / DW_OW) * G;
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(grid_groups(work, G, 2048)), dim3(NT), 0, st, x, w, y, sum, sumsq, N, H, W,
                     C, Ho, Wo, KH, KW, S, P, D);
  return hipGetLastError();
}

MLC_EXPORT int mlc_dwconv_dgrad(const bf16* dy, const bf16* w, bf16* dx, int N, int H, int W, int C, int KH, int KW,
                                int S, int P, int D, int Ho, int Wo, hipStream_t st) {
  if (C % 8) return -1;
  const int Wqi = (W + DW_SW - 1) / DW_SW;
  if (D == 1 && (S == 1 || S == 2) && (KW == 3 || KW == 5 || KW == 7) && dw_strips() && items_fit(N, H, Wqi, C / 8)) {
    const long work = (long)N * H * Wqi * (C / 8);
    const int nb = blocks_for(work);
    const dim3 grid(nb < dw_dgrad_cap() ? nb : dw_dgrad_cap());
    const Idx3 ix = idx3(C / 8, Wqi, H);
#define DWD(K, SS, PP) hipLaunchKernelGGL((dw_dgrad_strip_kernel<K, SS, PP>), grid, dim3(NT), 0, st, dy, w, dx, N, H, \
                                          W, C, Ho, Wo, KH, P, ix)
    if (S == 1) { if (KW == 3) DWD(3, 1, 0); else if (KW == 5) DWD(5, 1, 0); else DWD(7, 1, 0); }
    else if (P & 1) { if (KW == 3) DWD(3, 2, 1); else if (KW == 5) DWD(5, 2, 1); else DWD(7, 2, 1); }
    else { if (KW == 3) DWD(3, 2, 0); else if (KW == 5) DWD(5, 2, 0); else DWD(7, 2, 0); }
#undef DWD
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dw_dgrad_kernel, dim3(blocks_for((long)N * H * W * (C / 8))), dim3(NT), 0, st, dy, w, dx, N, H,
                     W, C, Ho, Wo, KH, KW, S, P, D);
  return hipGetLastError();
}

// dw [KH][KW][C] fp32 (+)=; ws: scratch of 32*KH*KW*C fp32 (zeroed here)
MLC_EXPORT int mlc_dwconv_wgrad(const bf16* dy, const bf16* x, float* dw, float* ws, int N, int H, int W, int C,
                                int KH, int KW, int S, int P, int D, int Ho, int Wo, int accumulate, hipStream_t st) {
  if (C % 8) return -1;
  const int G = C / 8, T = KH * KW;
  mlc_zero_f32(ws, (long)NCOPY * T * C, st);
  // deterministic mode: at most NCOPY blocks, so every copy of ws has one adder per element
  // (copies_reduce_kernel sums the copies in a fixed order)
  const int cap_strip = g_mlc_det ? det_group_cap(G) : 512, cap_tap = g_mlc_det ? det_group_cap(G) : 1024;
  if (cap_strip == 0) return -2;
  const int Wqo = (Wo + DW_SW - 1) / DW_SW;
  if (D == 1 && (S == 1 || S == 2) && (KW == 3 || KW == 5 || KW == 7) && dw_strips() && items_fit(N, Ho, Wqo, G)) {
    const long work = (long)N * Ho * Wqo * G;
    const Idx3 ix = idx3(G, Wqo, Ho);
    // items per thread: every block ends in KW*C float atomics (device-scope, past the XCD's
    // L2), so small-spatial layers (7x7, 14x14) want few, long-running blocks (MLC_DW_WG_ITEMS)
    int nb = grid_groups(work, G, cap_strip, dw_wg_items());
    // XCD-grouped row-blocks (not in deterministic mode, whose grid is capped at NCOPY blocks):
    // the spatial block count rounded up to a multiple of 8 that keeps the channel-group
    // alignment of group_mult
    const long m = group_mult(G), l8 = m * 8 / std::gcd(m, 8L);
    const int xcd = !g_mlc_det && dw_xcd();
    if (xcd) nb = (int)(((nb + l8 - 1) / l8) * l8);
    const dim3 grid = xcd ? dim3(nb * KH) : dim3(nb, KH);
#define DWW(K, SS) hipLaunchKernelGGL((dw_wgrad_strip_kernel<K, SS>), grid, dim3(NT), 0, st, dy, x, ws, N, H, W, C, \
                                      Ho, Wo, KH, P, xcd, ix)
    if (S == 1) { if (KW == 3) DWW(3, 1); else if (KW == 5) DWW(5, 1); else DWW(7, 1); }
    else { if (KW == 3) DWW(3, 2); else if (KW == 5) DWW(5, 2); else DWW(7, 2); }
#undef DWW
    hipLaunchKernelGGL(copies_reduce_kernel, dim3(blocks_for((long)T * C)), dim3(NT), 0, st, ws, dw, (long)T * C,
                       accumulate);
    return hipGetLastError();
  }
  const long work = (long)N * Ho * Wo * G;
  const int blocks = grid_groups(work, G, cap_tap);
  for (int t0 = 0; t0 < T; t0 += DW_TC)
    hipLaunchKernelGGL(dw_wgrad_kernel, dim3(blocks), dim3(NT), 0, st, dy, x, ws, N, H, W, C, Ho, Wo, KH, KW, S, P, D,
                       t0);
  hipLaunchKernelGGL(copies_reduce_kernel, dim3(blocks_for((long)T * C)), dim3(NT), 0, st, ws, dw, (long)T * C,
                     accumulate);
  return hipGetLastError();
}
