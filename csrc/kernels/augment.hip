// Device half of the native input pipeline (host half: csrc/runtime/records.cpp).
//
// src: a batch of raw uint8 HWC records [B][H][W][C] (C <= 4, copied to the device as
// is); par: per sample {y0, x0, h, w, flip} - the source box of a RandomResizedCrop /
// centre crop and a horizontal flip.  One pass crops, resizes the box to oh x ow
// (bilinear, half-pixel centres, clamped at the box edge: torchvision's Resize of the
// cropped region, antialias off), flips, normalises (x - mean) / std and writes:
//   layout 0: the native ResNet stem's 2x2 space-to-depth image of the pad-3 image,
//             bf16 [B][(oh+6)/2][(ow+6)/2][16], channel (dy*2+dx)*3 + ci, 12..15 zero
//             (ops.functional.stem_s2d layout);
//   layout 1: NHWC bf16 with channels padded to 8;
//   layout 2: NCHW fp32 (the torch engine).
#include "common.h"

namespace {

constexpr int NT = 256;

struct Box {
  float y0, x0, sy, sx;   // source box origin and scale (box / output)
  int h, w, flip;
};

__device__ __forceinline__ Box box(const int* par, int b, int oh, int ow) {
  const int* p = par + 5 * b;
  Box r;
  r.y0 = (float)p[0]; r.x0 = (float)p[1]; r.h = p[2]; r.w = p[3]; r.flip = p[4];
  r.sy = (float)r.h / (float)oh;
  r.sx = (float)r.w / (float)ow;
  return r;
}

// bilinear sample of the box at output pixel (oy, ox): out[c] for c < C
template <int C>
__device__ __forceinline__ void sample(const uint8_t* img, int W, const Box& bx, int oy, int ox, int ow,
                                       float* out) {
  if (bx.flip) ox = ow - 1 - ox;
  float fy = ((float)oy + 0.5f) * bx.sy - 0.5f, fx = ((float)ox + 0.5f) * bx.sx - 0.5f;
  fy = fminf(fmaxf(fy, 0.f), (float)(bx.h - 1));
  fx = fminf(fmaxf(fx, 0.f), (float)(bx.w - 1));
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = min(y0 + 1, bx.h - 1), x1 = min(x0 + 1, bx.w - 1);
  const float wy = fy - (float)y0, wx = fx - (float)x0;
  const int by = (int)bx.y0, bxo = (int)bx.x0;
  const uint8_t* p00 = img + ((size_t)(by + y0) * W + bxo + x0) * C;
  const uint8_t* p01 = img + ((size_t)(by + y0) * W + bxo + x1) * C;
  const uint8_t* p10 = img + ((size_t)(by + y1) * W + bxo + x0) * C;
  const uint8_t* p11 = img + ((size_t)(by + y1) * W + bxo + x1) * C;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float top = (float)p00[c] + wx * ((float)p01[c] - (float)p00[c]);
    const float bot = (float)p10[c] + wx * ((float)p11[c] - (float)p10[c]);
    out[c] = top + wy * (bot - top);
  }
}

template <int C>
__global__ void __launch_bounds__(NT)
augment_s2d_kernel(const uint8_t* __restrict__ src, const int* __restrict__ par, const float* __restrict__ ms,
                   bf16* __restrict__ out, int B, int H, int W, int oh, int ow, int Hb, int Wb) {
  const long total = (long)B * Hb * Wb;
  for (long q = (long)blockIdx.x * NT + threadIdx.x; q < total; q += (long)gridDim.x * NT) {
    const int j = (int)(q % Wb);
    const long t = q / Wb;
    const int i = (int)(t % Hb);
    const int b = (int)(t / Hb);
    const Box bx = box(par, b, oh, ow);
    const uint8_t* img = src + (size_t)b * H * W * C;
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int oy = 2 * i + dy - 3, ox = 2 * j + dx - 3;   // stem padding 3
        if ((unsigned)oy < (unsigned)oh && (unsigned)ox < (unsigned)ow) {
          float f[C];
          sample<C>(img, W, bx, oy, ox, ow, f);
#pragma unroll
          for (int c = 0; c < 3 && c < C; ++c) v[(dy * 2 + dx) * 3 + c] = (f[c] - ms[c]) * ms[4 + c];
        }
      }
    uint4* dst = reinterpret_cast<uint4*>(out + q * 16);
    dst[0] = pack8(v);
    dst[1] = pack8(v + 8);
  }
}

template <int C>
__global__ void __launch_bounds__(NT)
augment_pix_kernel(const uint8_t* __restrict__ src, const int* __restrict__ par, const float* __restrict__ ms,
                   void* __restrict__ out, int B, int H, int W, int oh, int ow, int layout) {
  const long total = (long)B * oh * ow;
  for (long q = (long)blockIdx.x * NT + threadIdx.x; q < total; q += (long)gridDim.x * NT) {
    const int ox = (int)(q % ow);
    const long t = q / ow;
    const int oy = (int)(t % oh);
    const int b = (int)(t / oh);
    const Box bx = box(par, b, oh, ow);
    float f[C];
    sample<C>(src + (size_t)b * H * W * C, W, bx, oy, ox, ow, f);
    if (layout == 1) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = (f[c] - ms[c]) * ms[4 + c];
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(out) + q * 8) = pack8(v);
    } else {
      float* o = reinterpret_cast<float*>(out);
#pragma unroll
      for (int c = 0; c < C; ++c) o[(((size_t)b * C + c) * oh + oy) * ow + ox] = (f[c] - ms[c]) * ms[4 + c];
    }
  }
}

}  // namespace

// mean_istd: 8 floats {mean[0..3], 1/std[0..3]} (uint8 scale) on the device
MLC_EXPORT int mlc_augment(const uint8_t* src, const int* par, const float* mean_istd, void* out, int B, int H,
                           int W, int C, int oh, int ow, int layout, hipStream_t st) {
  if (C < 1 || C > 4 || B <= 0 || oh <= 0 || ow <= 0 || layout < 0 || layout > 2) return -1;
  if (layout == 0 && (C != 3 || (oh & 1) || (ow & 1))) return -1;
  if (layout == 1 && C > 8) return -1;
  const int Hb = (oh + 6) / 2, Wb = (ow + 6) / 2;
  const long total = layout == 0 ? (long)B * Hb * Wb : (long)B * oh * ow;
  long blocks = (total + NT - 1) / NT;
  if (blocks > 16384) blocks = 16384;
  if (layout == 0) {
    hipLaunchKernelGGL(augment_s2d_kernel<3>, dim3((int)blocks), dim3(NT), 0, st, src, par, mean_istd,
                       reinterpret_cast<bf16*>(out), B, H, W, oh, ow, Hb, Wb);
    return hipGetLastError();
  }
#define AUG_PIX(CC) hipLaunchKernelGGL(augment_pix_kernel<CC>, dim3((int)blocks), dim3(NT), 0, st, src, par, \
                                       mean_istd, out, B, H, W, oh, ow, layout)
  if (C == 1) AUG_PIX(1);
  else if (C == 2) AUG_PIX(2);
  else if (C == 3) AUG_PIX(3);
  else AUG_PIX(4);
#undef AUG_PIX
  return hipGetLastError();
}
