// Convolution geometry shared by the implicit-GEMM engines (igemm.hip: 128x128 tiles,
// gemm256.hip: 256-row LDS-DMA tiles): multiply-shift division, NHWC conv geometry, the
// per-row filter-tap masks and the stride-parity classes of a transposed (dgrad) conv.
// The K axis of every conv GEMM is walked in 64-deep steps (one filter tap per step when
// the channel count is a multiple of 64).
#pragma once
#include "common.h"

namespace igemm {

constexpr int NSTAT = 32;   // BN-statistic partial copies (spread same-address atomics)

// ------------------------------------------------------------------ fast division
struct FastDiv {
  unsigned d, mul, sh;
  __host__ __device__ FastDiv() : d(1), mul(0), sh(0) {}
  __host__ explicit FastDiv(unsigned dd) : d(dd) {
    sh = 0;
    while ((1u << sh) < d) ++sh;
    mul = (unsigned)((((unsigned long long)1 << 32) * ((1ull << sh) - d)) / d + 1);
  }
  __device__ __forceinline__ unsigned div(unsigned n) const { return (__umulhi(n, mul) + n) >> sh; }
  __device__ __forceinline__ void divmod(unsigned n, unsigned& q, unsigned& r) const {
    q = div(n); r = n - q * d;
  }
};

// ---------------------------------------------------------------- geometry
struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int Ho, Wo, Co;      // output
  int KH, KW, stride, pad, dil;
  int padw;            // W-axis padding (pad is the H-axis one; equal unless packed, see unpack_pad)
  FastDiv fWo, fHo, fW, fH, fC, fCo, fKW;
};

// Per-row tap mask: bit r (r < 15) = filter row r lands inside the input, bit 16+s =
// filter column s does; a K chunk of tap (r, s) is loaded iff (mask & P) == P with
// P = 1<<r | 1<<(16+s).  P = 1<<15 (never set) marks a chunk past K.
__device__ __forceinline__ unsigned tap_pat(int r, int s) { return (1u << r) | (1u << (16 + s)); }
constexpr unsigned NO_TAP = 1u << 15;

// Transposed-conv (dgrad) geometry of ONE stride-parity class: output rows are the input
// pixels (n, hi = i*S+ph, wi = j*S+pw), i < Hc, j < Wc.  Only filter taps r = r0 +
// rstep*a (a < nr), s = s0 + sstep*b (b < ns) reach the class; for them the dy pixel is
// (i + dh0 - a*dhs, j + dw0 - b*dws).  The K loop runs over (a, b, 64-channel block of
// Co): K = nr*ns*ncb*64, channels past Co read as zero.
struct DgradClass {
  int S, ph, pw, Hc, Wc;
  FastDiv fWc, fHc;
  int r0, s0, rstep, sstep, nr, ns, ncb;
  FastDiv fns, fncb;
  int dh0, dhs, dw0, dws;
  long long tmin;      // smallest tap offset (elements), folded into the base
  __device__ __forceinline__ void decode(int m, int& n, int& i, int& j) const {
    unsigned t, q, rr;
    fWc.divmod((unsigned)m, t, rr); j = (int)rr;
    fHc.divmod(t, q, rr); i = (int)rr; n = (int)q;
  }
  // K-tile -> (a, b, first channel)
  __device__ __forceinline__ void tap(int kt, int& a, int& b, int& co0) const {
    unsigned t, cb, aa, bb;
    fncb.divmod((unsigned)kt, t, cb);
    fns.divmod(t, aa, bb);
    a = (int)aa; b = (int)bb; co0 = (int)cb * 64;
  }
};

}  // namespace igemm

namespace igemm_host {
using igemm::ConvGeom;
using igemm::DgradClass;
using igemm::FastDiv;

// The conv exports take one int `pad`: a plain value pads both axes; (1 << 30) | (pad_w << 15)
// | pad_h packs per-axis paddings (a 1x7 / 7x1 conv with padding (0, 3) / (3, 0)).
constexpr int PAD_PACKED = 1 << 30;
static inline void unpack_pad(int pad, int& ph, int& pw) {
  if (pad & PAD_PACKED) { ph = pad & 0x7fff; pw = (pad >> 15) & 0x7fff; }
  else { ph = pad; pw = pad; }
}
static inline int pack_pad(int ph, int pw) { return ph == pw ? ph : (PAD_PACKED | (pw << 15) | ph); }

static inline ConvGeom mkgeom(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad,
                       int dil, int Ho, int Wo) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Co = Co; g.KH = KH; g.KW = KW;
  int ph, pw;
  unpack_pad(pad, ph, pw);
  g.stride = stride; g.pad = ph; g.padw = pw; g.dil = dil; g.Ho = Ho; g.Wo = Wo;
  g.fWo = FastDiv(Wo); g.fHo = FastDiv(Ho); g.fW = FastDiv(W); g.fH = FastDiv(H);
  g.fC = FastDiv(C); g.fCo = FastDiv(Co); g.fKW = FastDiv(KW);
  return g;
}

static inline int gcd_i(int a, int b) { while (b) { const int t = a % b; a = b; b = t; } return a; }

// The stride-parity class (ph, pw) of a dgrad output: the filter taps that reach it form
// arithmetic progressions r = r0 + rstep*a, s = s0 + sstep*b.  A class no tap reaches has
// nr*ns == 0 and is still launched (K = 0) so its rows get the epilogue (0 + addend, BN).
static inline DgradClass mkclass(int S, int ph, int pw, int H, int W, int Ho, int Wo, int Co, int KH, int KW,
                          int pad, int dil) {
  DgradClass c;
  c.S = S; c.ph = ph; c.pw = pw;
  c.Hc = (H - ph + S - 1) / S; c.Wc = (W - pw + S - 1) / S;
  c.fWc = FastDiv(c.Wc > 0 ? c.Wc : 1); c.fHc = FastDiv(c.Hc > 0 ? c.Hc : 1);
  int pad_h, pad_w;
  unpack_pad(pad, pad_h, pad_w);
  auto axis = [&](int p, int KK, int pd, int& r0, int& step, int& n, int& d0, int& ds) {
    r0 = -1; n = 0;
    for (int r = 0; r < KK; ++r)
      if ((((p + pd - r * dil) % S) + S) % S == 0) { if (r0 < 0) r0 = r; ++n; }
    step = S / gcd_i(S, dil);
    if (n == 0) { r0 = 0; d0 = 0; ds = 0; return; }
    d0 = (p + pd - r0 * dil) / S;
    ds = step * dil / S;
  };
  axis(ph, KH, pad_h, c.r0, c.rstep, c.nr, c.dh0, c.dhs);
  axis(pw, KW, pad_w, c.s0, c.sstep, c.ns, c.dw0, c.dws);
  c.ncb = (Co + 63) / 64;
  c.fns = FastDiv(c.ns > 0 ? c.ns : 1); c.fncb = FastDiv(c.ncb);
  c.tmin = (c.nr > 0 && c.ns > 0)
               ? ((long long)(c.dh0 - (c.nr - 1) * c.dhs) * Wo + (c.dw0 - (c.ns - 1) * c.dws)) * Co : 0;
  (void)Ho;
  return c;
}

}  // namespace igemm_host
