// dcn_offset_conv.hip — the offset conv (deform_conv.py:16-21, :58) and its backward.
//
// The offset conv has only J = 2*N*G = 18 output channels, so as an MFMA GEMM 14 of
// every 32 tile rows are padding and every MFMA needs its own per-lane gather (the
// 32x32x2 f32 MFMA versions of these kernels were load-issue bound at 3-4x their MFMA
// floor). These kernels are VALU implicit GEMMs built around wave-uniform operands: the
// J offset-channel values that every lane of a wave needs at the same time (weights in
// the forward / input-gradient passes, ∂offsets in the weight-gradient pass) are read
// with scalar loads from small transposed copies, so each coalesced vector load feeds
// J (or 4*J) FMAs:
//   K3  fwd   lanes = output pixels (NCHW x)    acc[J]      weights  wT[c][tap][J]   scalar
//   K7a ∂W    lanes = channels (xT, float4)     acc[J][4]   ∂offT[p][J]              scalar
//   K7b ∂x    lanes = input pixels (NCHW ∂x)    acc[32 ch]  weights  wT2[j][tap][C]  scalar
#include <algorithm>

#include "dcn_device.h"

namespace dcn {

constexpr int kJB = 18;  // offset channels per pass (one pass for the reference's 3x3)
constexpr int kCB = 32;  // channels per K7b pass

// Padded sizes: the uniform operand runs are zero-padded so every scalar load is
// unconditional (the compiler then merges them into s_load_dwordx8/x16).
__host__ __device__ static inline int pad_j(int J) { return (J + kJB - 1) / kJB * kJB; }
__host__ __device__ static inline int pad_c(int C) { return (C + kCB - 1) / kCB * kCB; }

// wT[(c*KK + tap)*Jp + j] = w_off[j][c][tap] (0 for j >= J)
__global__ __launch_bounds__(256) void woff_to_ctj(const float* __restrict__ w,
                                                   float* __restrict__ wt, int J, int Jp, int C,
                                                   int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Jp * C * KK) return;
  const int r = i / Jp, j = i - r * Jp;  // r = c*KK + tap
  const int c = r / KK, tap = r - c * KK;
  wt[i] = j < J ? w[((size_t)j * C + c) * KK + tap] : 0.f;
}
// wT2[(j*KK + tap)*Cp + c] = w_off[j][c][tap] (0 for c >= C)
__global__ __launch_bounds__(256) void woff_to_jtc(const float* __restrict__ w,
                                                   float* __restrict__ wt, int J, int C, int Cp,
                                                   int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= J * KK * Cp) return;
  const int r = i / Cp, c = i - r * Cp;  // r = j*KK + tap
  const int j = r / KK, tap = r - j * KK;
  wt[i] = c < C ? w[((size_t)j * C + c) * KK + tap] : 0.f;
}
// goffT[(b*HW + p)*Jp + j] = goff[b][j][p] (0 for j >= J)
__global__ __launch_bounds__(256) void goff_to_pj(const float* __restrict__ goff,
                                                  float* __restrict__ goffT, int J, int Jp,
                                                  int HW, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over (b, j, p), p fastest: coalesced reads
  if (i >= total) return;
  const int p = (int)(i % HW);
  const long bj = i / HW;
  const int j = (int)(bj % Jp), b = (int)(bj / Jp);
  goffT[((size_t)b * HW + p) * Jp + j] = j < J ? goff[((size_t)b * J + j) * HW + p] : 0.f;
}

// ---------------------------------------------------------------------------
// K3: off[b][j][p] = b_off[j] + Σ_{c,tap} w_off[j][c][tap] · x[b][c][tap-shifted p]
// One thread per output pixel, kJB accumulators; grid.y = passes over j.
// ---------------------------------------------------------------------------
// grid.z = kSplit channel slices; slice z writes part[z][b][j][m] (summed by
// offset_conv_combine in a fixed order: the offsets are bitwise reproducible).
constexpr int kSplit = 8;

template <int KK>
__global__ __launch_bounds__(256) void offset_conv_fwd_valu(Geo g, const float* __restrict__ x,
                                                           const float* __restrict__ wt,
                                                           float* __restrict__ part) {
  const long Mtot = (long)g.B * g.HW;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const bool pok = p < Mtot;
  const int b = pok ? (int)(p / g.HW) : 0;
  const int m = pok ? (int)(p - (long)b * g.HW) : 0;
  const int ho = m / g.Wo, wo = m - (m / g.Wo) * g.Wo;
  int offs[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    const int i = t / g.kw, kx = t - i * g.kw;
    const int y = ho * g.sh - g.ph + i * g.dh, xx = wo * g.sw - g.pw + kx * g.dw;
    offs[t] = (pok && y >= 0 && y < g.H && xx >= 0 && xx < g.W) ? y * g.W + xx : -1;
  }
  const int j0 = blockIdx.y * kJB;
  const int jn = min(kJB, g.J - j0);
  const int Jp = pad_j(g.J);
  float acc[kJB];
#pragma unroll
  for (int jj = 0; jj < kJB; ++jj) acc[jj] = 0.f;
  const float* xb = x + (size_t)b * g.C * g.HWi;
  const int cper = (g.C + kSplit - 1) / kSplit;
  const int cbeg = blockIdx.z * cper, cend = min(g.C, cbeg + cper);
#pragma unroll 2
  for (int c = cbeg; c < cend; ++c) {
    const float* xc = xb + (size_t)c * g.HWi;
    float v[KK];
#pragma unroll
    for (int t = 0; t < KK; ++t) v[t] = offs[t] >= 0 ? xc[offs[t]] : 0.f;
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      const float* w = wt + ((size_t)c * KK + t) * Jp + j0;  // wave-uniform, zero-padded
#pragma unroll
      for (int jj = 0; jj < kJB; ++jj) acc[jj] = fmaf(v[t], w[jj], acc[jj]);
    }
  }
  if (!pok) return;
  float* pz = part + (size_t)blockIdx.z * g.B * g.J * g.HW;
#pragma unroll
  for (int jj = 0; jj < kJB; ++jj)
    if (jj < jn) pz[((size_t)b * g.J + j0 + jj) * g.HW + m] = acc[jj];
}

// K3 fast path (column stride 1, column dilation 1): one thread = kPX consecutive output
// pixels of a row, so each scalar-loaded weight feeds kPX FMAs and a channel's
// KH x (kPX+KW-1) input patch is loaded once for kPX*KH*KW pixel-taps.
template <int KH, int KW, int kPX>
__global__ __launch_bounds__(256) void offset_conv_fwd_row(Geo g, const float* __restrict__ x,
                                                          const float* __restrict__ wt,
                                                          float* __restrict__ part, int gpr) {
  constexpr int SPAN = kPX + KW - 1;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;  // (b, ho, group)
  const long T = (long)g.B * g.Ho * gpr;
  const bool tok = t < T;
  const long tt = tok ? t : 0;
  const int grp = (int)(tt % gpr);
  const long bh = tt / gpr;
  const int ho = (int)(bh % g.Ho), b = (int)(bh / g.Ho);
  const int wo0 = grp * kPX;
  const int x0 = wo0 - g.pw;  // input column of tap kx=0 for pixel wo0 (sw = dw = 1)
  int rowoff[KH];
  bool rowok[KH];
#pragma unroll
  for (int i = 0; i < KH; ++i) {
    const int y = ho * g.sh - g.ph + i * g.dh;
    rowok[i] = tok && y >= 0 && y < g.H;
    rowoff[i] = rowok[i] ? y * g.W : 0;
  }
  bool colok[SPAN];
#pragma unroll
  for (int k = 0; k < SPAN; ++k) colok[k] = x0 + k >= 0 && x0 + k < g.W;
  const int j0 = blockIdx.y * kJB;
  const int jn = min(kJB, g.J - j0);
  const int Jp = pad_j(g.J);
  float acc[kPX][kJB];
#pragma unroll
  for (int q = 0; q < kPX; ++q)
#pragma unroll
    for (int jj = 0; jj < kJB; ++jj) acc[q][jj] = 0.f;
  const float* xb = x + (size_t)b * g.C * g.HWi;
  const int cper = (g.C + kSplit - 1) / kSplit;
  const int cbeg = blockIdx.z * cper, cend = min(g.C, cbeg + cper);
  for (int c = cbeg; c < cend; ++c) {
    const float* xc = xb + (size_t)c * g.HWi + x0;
    float v[KH][SPAN];
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
      for (int k = 0; k < SPAN; ++k) v[i][k] = (rowok[i] && colok[k]) ? xc[rowoff[i] + k] : 0.f;
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
      for (int kx = 0; kx < KW; ++kx) {
        const float* w = wt + ((size_t)c * (KH * KW) + i * KW + kx) * Jp + j0;  // wave-uniform
#pragma unroll
        for (int jj = 0; jj < kJB; ++jj) {
          const float wv = w[jj];
#pragma unroll
          for (int q = 0; q < kPX; ++q) acc[q][jj] = fmaf(v[i][q + kx], wv, acc[q][jj]);
        }
      }
  }
  if (!tok) return;
  float* pz = part + (size_t)blockIdx.z * g.B * g.J * g.HW + ((size_t)b * g.J + j0) * g.HW +
              (size_t)ho * g.Wo + wo0;
#pragma unroll
  for (int jj = 0; jj < kJB; ++jj)
    if (jj < jn)
#pragma unroll
      for (int q = 0; q < kPX; ++q)
        if (wo0 + q < g.Wo) pz[(size_t)jj * g.HW + q] = acc[q][jj];
}

__global__ __launch_bounds__(256) void offset_conv_combine(const float* __restrict__ part,
                                                          const float* __restrict__ b_off,
                                                          float* __restrict__ off, int J, int HW,
                                                          long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = b_off[(i / HW) % J];
#pragma unroll
  for (int z = 0; z < kSplit; ++z) v += part[(size_t)z * n + i];
  off[i] = v;
}

constexpr int kWgradRpw = 4;  // output rows per wave in offset_wgrad_valu

struct WgradGrid {
  unsigned nbx, ny, nz;
  int cper;  // channels per wave (64 lanes x VEC)
};
static int wgrad_rpw() { return exp_flag(7) ? exp_flag(7) : kWgradRpw; }
static WgradGrid wgrad_grid(const Geo& g, int rpw) {
  const long waves = ((long)g.B * g.Ho + rpw - 1) / rpw;
  WgradGrid w;
  w.cper = g.C % 4 == 0 ? 256 : 64;
  w.nbx = (unsigned)((waves + 3) / 4);
  w.ny = (unsigned)(g.kh * g.kw * ((g.J + kJB - 1) / kJB));
  w.nz = (unsigned)((g.C + w.cper - 1) / w.cper);
  return w;
}
static size_t goffT_rows_floats(const Geo& g) {
  return ((size_t)g.B * g.HW * pad_j(g.J) + 63) / 64 * 64;
}

// ---------------------------------------------------------------------------
// K7a: ∂w_off[j][c][tap] += Σ_p ∂off[b][j][p] · x[b][c][tap-shifted p]
// One wave = (tap, j pass, 64*VEC-channel chunk, pixel range); lane = VEC channels
// (xT rows, 1 KiB per wave load at VEC=4); ∂offT[p][j0..] is wave-uniform (scalar).
// ---------------------------------------------------------------------------
template <int VEC>
__global__ __launch_bounds__(256) void offset_wgrad_valu(Geo g, const float* __restrict__ xT,
                                                         const float* __restrict__ goffT,
                                                         float* __restrict__ part, int rpw,
                                                         int nbx, int ny, int nz) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
  // 1-D grid, (tap, j pass) fastest: the KK tap blocks of one pixel range are neighbours
  // in the XCD-aware order, so xT rows fetched for one tap are L2 hits for the others
  const unsigned lid = xcd_block().x;
  const int by = (int)(lid % ny), bx = (int)((lid / ny) % nbx), bz = (int)(lid / ny / nbx);
  const int KK = g.kh * g.kw;
  const int Jp = pad_j(g.J);
  const int tap = by % KK, j0 = (by / KK) * kJB;
  const int c = (bz * 64 + lane) * VEC;
  const bool cok = c < g.C;
  // this wave's output rows (flattened (b, ho)); a tap's valid pixels in a row are one
  // contiguous wo range, so the inner loop is branch-free pointer strides (the per-pixel
  // (b, ho, wo) walk cost more scalar instructions than the FMAs)
  const int rows = g.B * g.Ho;
  const int rstart = min(rows, (bx * 4 + wave) * rpw), rend = min(rows, rstart + rpw);
  const int ti = tap / g.kw, tx = tap - ti * g.kw;
  const int dyo = ti * g.dh - g.ph, dxo = tx * g.dw - g.pw;
  const int wlo = dxo >= 0 ? 0 : (-dxo + g.sw - 1) / g.sw;
  const int whi = g.W - 1 - dxo < 0 ? 0 : min(g.Wo, (g.W - 1 - dxo) / g.sw + 1);
  const int cc = cok ? c : 0;
  const long sstep = (long)g.sw * g.C;
  float acc[kJB][VEC];
#pragma unroll
  for (int jj = 0; jj < kJB; ++jj)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[jj][e] = 0.f;
  constexpr int U = 4;  // pixels whose xT rows / ∂offT rows are in flight together
  for (int row = rstart; row < rend; ++row) {
    const int b = row / g.Ho, ho = row - b * g.Ho;
    const int y = ho * g.sh + dyo;
    if (y < 0 || y >= g.H || wlo >= whi) continue;  // wave-uniform
    const float* src = xT + (((size_t)b * g.H + y) * g.W + (wlo * g.sw + dxo)) * g.C + cc;
    const float* gp = goffT + ((size_t)b * g.HW + (size_t)ho * g.Wo + wlo) * Jp + j0;
    const int n = whi - wlo;
    for (int i = 0; i < n; i += U) {
      float v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float* sp = src + min(i + u, n - 1) * sstep;
        if constexpr (VEC == 4) {
          const float4 t = *reinterpret_cast<const float4*>(sp);
          v[u][0] = cok ? t.x : 0.f;
          v[u][1] = cok ? t.y : 0.f;
          v[u][2] = cok ? t.z : 0.f;
          v[u][3] = cok ? t.w : 0.f;
        } else {
          v[u][0] = cok ? *sp : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i + u >= n) break;
        const float* gq = gp + (size_t)(i + u) * Jp;  // wave-uniform, zero-padded
#pragma unroll
        for (int jj = 0; jj < kJB; ++jj) {
          const float gv = gq[jj];
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[jj][e] = fmaf(gv, v[u][e], acc[jj][e]);
        }
      }
    }
  }
  // The block's 4 waves cover consecutive pixel ranges of the same (tap, j pass, chunk):
  // fold waves 1..3 into wave 0 through LDS (fixed order), then write one partial per
  // block; wgrad_reduce sums the partials in block order. No float atomics, so ∂w_off is
  // bitwise reproducible (device-scope atomics from 8 XCDs also serialised badly here).
  constexpr int R = 6;  // accumulator rows per LDS round
  __shared__ float red[3][R][VEC][64];
#pragma unroll
  for (int r0 = 0; r0 < kJB; r0 += R) {
    if (wave > 0)
#pragma unroll
      for (int jr = 0; jr < R; ++jr)
#pragma unroll
        for (int e = 0; e < VEC; ++e) red[wave - 1][jr][e][lane] = acc[r0 + jr][e];
    __syncthreads();
    if (wave == 0)
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int jr = 0; jr < R; ++jr)
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[r0 + jr][e] += red[w][jr][e][lane];
    __syncthreads();
  }
  if (wave != 0) return;
  constexpr int E = kJB * VEC * 64;
  float* pb = part + ((size_t)(by * nz + bz) * nbx + bx) * E;
#pragma unroll
  for (int jj = 0; jj < kJB; ++jj)
#pragma unroll
    for (int e = 0; e < VEC; ++e) pb[(jj * VEC + e) * 64 + lane] = acc[jj][e];
}

// ∂w_off = Σ over pixel blocks of offset_wgrad_valu's partials, in block order. One
// 1024-thread block per 64 partial elements: wave w sums blocks ≡ w (mod 16), then the
// 16 wave sums are folded in wave order (deterministic).
template <int VEC>
__global__ __launch_bounds__(1024) void wgrad_reduce(Geo g, const float* __restrict__ part,
                                                     float* __restrict__ gw, int nbx, int nz) {
  constexpr int E = kJB * VEC * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int idx = blockIdx.x * 64 + lane;  // element within E
  const int yz = blockIdx.y;
  const float* pp = part + (size_t)yz * nbx * E + idx;
  float s = 0.f;
#pragma unroll 4
  for (int bx = w; bx < nbx; bx += 16) s += pp[(size_t)bx * E];
  __shared__ float red[16][64];
  red[w][lane] = s;
  __syncthreads();
  if (w != 0) return;
  s = red[0][lane];
#pragma unroll
  for (int k = 1; k < 16; ++k) s += red[k][lane];
  const int KK = g.kh * g.kw;
  const int y = yz / nz, z = yz - y * nz;
  const int tap = y % KK, j0 = (y / KK) * kJB;
  const int jj = idx / (VEC * 64), e = (idx / 64) % VEC;
  const int c = (z * 64 + lane) * VEC + e;
  if (j0 + jj < g.J && c < g.C) gw[((size_t)(j0 + jj) * g.C + c) * KK + tap] = s;
}

// ---------------------------------------------------------------------------
// K7b: ∂x[b][c][y][x] (+)= Σ_{j,tap} w_off[j][c][tap] · ∂off[b][j][(y+pad-tap·dil)/s]
// One thread per input pixel and kCB channels (grid.y); weights wave-uniform.
// ---------------------------------------------------------------------------
template <int KK>
__global__ __launch_bounds__(256) void offset_dgrad_valu(Geo g, const float* __restrict__ wt2,
                                                         const float* __restrict__ goff,
                                                         float* __restrict__ gx,
                                                         const float* __restrict__ gxT_in) {
  const long Mi = (long)g.B * g.HWi;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const bool pok = p < Mi;
  const int b = pok ? (int)(p / g.HWi) : 0;
  const int yx = pok ? (int)(p - (long)b * g.HWi) : 0;
  const int y = yx / g.W, xx = yx - (yx / g.W) * g.W;
  int goffs[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    const int i = t / g.kw, kx = t - i * g.kw;
    const int tt = y + g.ph - i * g.dh, u = xx + g.pw - kx * g.dw;
    goffs[t] = -1;
    if (pok && tt >= 0 && u >= 0 && tt % g.sh == 0 && u % g.sw == 0) {
      const int ho = tt / g.sh, wo = u / g.sw;
      if (ho < g.Ho && wo < g.Wo) goffs[t] = ho * g.Wo + wo;
    }
  }
  const int c0 = blockIdx.y * kCB;
  const int cn = min(kCB, g.C - c0);
  const int Cp = pad_c(g.C);
  float acc[kCB];
  if (gxT_in) {  // start from the sampling-route ∂x (channels-last): one 128-B run per pixel
    const float* src = gxT_in + ((size_t)b * g.HWi + yx) * g.C + c0;
    if (pok && cn == kCB && (g.C & 3) == 0) {  // 16-B aligned: 8 dwordx4 loads
#pragma unroll
      for (int q = 0; q < kCB / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(src + 4 * q);
        acc[4 * q] = v.x, acc[4 * q + 1] = v.y, acc[4 * q + 2] = v.z, acc[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int cc = 0; cc < kCB; ++cc) acc[cc] = (pok && cc < cn) ? src[cc] : 0.f;
    }
  } else {
#pragma unroll
    for (int cc = 0; cc < kCB; ++cc) acc[cc] = 0.f;
  }
  const float* gb = goff + (size_t)b * g.J * g.HW;
  for (int j = 0; j < g.J; ++j) {
    const float* gj = gb + (size_t)j * g.HW;
    float v[KK];
#pragma unroll
    for (int t = 0; t < KK; ++t) v[t] = goffs[t] >= 0 ? gj[goffs[t]] : 0.f;
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      const float* w = wt2 + ((size_t)j * KK + t) * Cp + c0;  // wave-uniform, zero-padded
#pragma unroll
      for (int cc = 0; cc < kCB; ++cc) acc[cc] = fmaf(v[t], w[cc], acc[cc]);
    }
  }
  if (!pok) return;
#pragma unroll
  for (int cc = 0; cc < kCB; ++cc)
    if (cc < cn) {
      float* d = gx + ((size_t)b * g.C + c0 + cc) * g.HWi + yx;
      *d = gxT_in ? acc[cc] : *d + acc[cc];
    }
}

// ---------------------------------------------------------------------------
// Generic fallbacks (kernel sizes without an instantiation): plain per-thread loops.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void offset_conv_fwd_generic(Geo g, const float* __restrict__ x,
                                                              const float* __restrict__ w_off,
                                                              const float* __restrict__ b_off,
                                                              float* __restrict__ off) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)g.B * g.J * g.HW) return;
  const int m = (int)(idx % g.HW);
  const int j = (int)((idx / g.HW) % g.J), b = (int)(idx / ((long)g.HW * g.J));
  const int ho = m / g.Wo, wo = m - ho * g.Wo;
  float acc = 0.f;
  for (int c = 0; c < g.C; ++c)
    for (int i = 0; i < g.kh; ++i)
      for (int k = 0; k < g.kw; ++k) {
        const int y = ho * g.sh - g.ph + i * g.dh, xx = wo * g.sw - g.pw + k * g.dw;
        if (y < 0 || y >= g.H || xx < 0 || xx >= g.W) continue;
        acc = fmaf(w_off[(((size_t)j * g.C + c) * g.kh + i) * g.kw + k],
                   x[((size_t)b * g.C + c) * g.HWi + y * g.W + xx], acc);
      }
  off[idx] = acc + b_off[j];
}

// one thread per (b, j, m): scatter into ∂x and ∂w_off with atomics
__global__ __launch_bounds__(256) void offset_bwd_generic(Geo g, const float* __restrict__ x,
                                                         const float* __restrict__ w_off,
                                                         const float* __restrict__ goff,
                                                         float* __restrict__ gx,
                                                         float* __restrict__ gw) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)g.B * g.J * g.HW) return;
  const int m = (int)(idx % g.HW);
  const int j = (int)((idx / g.HW) % g.J), b = (int)(idx / ((long)g.HW * g.J));
  const int ho = m / g.Wo, wo = m - ho * g.Wo;
  const float gv = goff[idx];
  for (int c = 0; c < g.C; ++c)
    for (int i = 0; i < g.kh; ++i)
      for (int k = 0; k < g.kw; ++k) {
        const int y = ho * g.sh - g.ph + i * g.dh, xx = wo * g.sw - g.pw + k * g.dw;
        if (y < 0 || y >= g.H || xx < 0 || xx >= g.W) continue;
        const size_t wi = (((size_t)j * g.C + c) * g.kh + i) * g.kw + k;
        const size_t xi = ((size_t)b * g.C + c) * g.HWi + y * g.W + xx;
        atomicAdd(gw + wi, gv * x[xi]);
        atomicAdd(gx + xi, gv * w_off[wi]);
      }
}

#define DCN_KK_DISPATCH(KKV, ...) \
  switch (KKV) {                   \
    case 1: { constexpr int KKc = 1; __VA_ARGS__; } break; \
    case 4: { constexpr int KKc = 4; __VA_ARGS__; } break; \
    case 6: { constexpr int KKc = 6; __VA_ARGS__; } break; \
    case 9: { constexpr int KKc = 9; __VA_ARGS__; } break; \
    default: generic = true; break; \
  }

size_t offset_conv_wt_floats(const Geo& g) {
  const size_t KK = (size_t)g.kh * g.kw;
  return std::max((size_t)pad_j(g.J) * g.C * KK, (size_t)g.J * KK * pad_c(g.C));
}
size_t offset_conv_fpart_floats(const Geo& g) { return (size_t)kSplit * g.B * g.J * g.HW; }

// goffT rows, then offset_wgrad_valu's per-block partials.
size_t offset_conv_goffT_floats(const Geo& g) {
  const WgradGrid w = wgrad_grid(g, 1);  // sized for the smallest row count per wave
  return goffT_rows_floats(g) + (size_t)w.nbx * w.ny * w.nz * kJB * w.cper;
}

hipError_t launch_offset_conv_fwd(const Geo& g, const float* x, const float* w_off,
                                  const float* b_off, float* off, float* wt, float* part,
                                  hipStream_t s) {
  const int KK = g.kh * g.kw;
  bool generic = false;
  const long Mtot = (long)g.B * g.HW;
  const int n = pad_j(g.J) * g.C * KK;
  hipLaunchKernelGGL(woff_to_ctj, dim3((n + 255) / 256), dim3(256), 0, s, w_off, wt, g.J,
                     pad_j(g.J), g.C, KK);
  if (g.sw == 1 && g.dw == 1 && g.kh == 3 && g.kw == 3 && !exp_flag(4)) {
    auto go = [&](auto kern, int npx) {
      const int gpr = (g.Wo + npx - 1) / npx;
      const long T = (long)g.B * g.Ho * gpr;
      dim3 grid((unsigned)((T + 255) / 256), (g.J + kJB - 1) / kJB, kSplit);
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g, x, wt, part, gpr);
    };
    // r01 A/B at config 3 (8 channel slices): 2 px/thread 0.248 ms, 4 px 0.297, 8 px 0.46
    // (occupancy beats weight reuse); the 1-px generic kernel 0.52
    go(offset_conv_fwd_row<3, 3, 2>, 2);
  } else {
    dim3 grid((unsigned)((Mtot + 255) / 256), (g.J + kJB - 1) / kJB, kSplit);
    DCN_KK_DISPATCH(KK, hipLaunchKernelGGL(offset_conv_fwd_valu<KKc>, grid, dim3(256), 0, s, g,
                                           x, wt, part));
  }
  if (!generic) {
    const long n = (long)g.B * g.J * g.HW;
    hipLaunchKernelGGL(offset_conv_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       part, b_off, off, g.J, g.HW, n);
  } else {
    const long total = (long)g.B * g.J * g.HW;
    hipLaunchKernelGGL(offset_conv_fwd_generic, dim3((unsigned)((total + 255) / 256)), dim3(256),
                       0, s, g, x, w_off, b_off, off);
  }
  return hipGetLastError();
}

// xT: channels-last x; goffT, wt2: scratch ([B][HW][J], [J][KK][C]). grad_x is accumulated,
// or (gxT_in) overwritten with transpose(gxT_in) + the offset-conv route.
hipError_t launch_offset_conv_bwd(const Geo& g, const float* x, const float* xT,
                                  const float* w_off, const float* goff, float* goffT, float* wt2,
                                  float* gx, float* gw_off, float* gb_off, const float* gxT_in,
                                  hipStream_t s) {
  const int KK = g.kh * g.kw;
  launch_channel_sum(goff, g.B, g.J, g.HW, gb_off, s);
  bool generic = false;
  DCN_KK_DISPATCH(KK, (void)KKc);
  if (generic) {
    hipError_t e = hipMemsetAsync(gw_off, 0, (size_t)g.J * g.C * KK * sizeof(float), s);
    if (e != hipSuccess) return e;
    if (gxT_in) {  // the generic kernel accumulates into NCHW ∂x
      e = launch_nhwc_to_nchw(gxT_in, gx, g.B, g.C, g.HWi, s);
      if (e != hipSuccess) return e;
    }
    const long total = (long)g.B * g.J * g.HW;
    hipLaunchKernelGGL(offset_bwd_generic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       g, x, w_off, goff, gx, gw_off);
    return hipGetLastError();
  }
  {
    const long total = (long)g.B * pad_j(g.J) * g.HW;
    hipLaunchKernelGGL(goff_to_pj, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, goff,
                       goffT, g.J, pad_j(g.J), g.HW, total);
  }
  {
    const int rpw = wgrad_rpw();
    const WgradGrid w = wgrad_grid(g, rpw);
    float* part = goffT + goffT_rows_floats(g);
    dim3 grid(w.nbx * w.ny * w.nz), rgrid(kJB * w.cper / 64, w.ny * w.nz);
    const int nbx = (int)w.nbx, ny = (int)w.ny, nz = (int)w.nz;
    if (w.cper == 256) {
      hipLaunchKernelGGL(offset_wgrad_valu<4>, grid, dim3(256), 0, s, g, xT, goffT, part, rpw,
                         nbx, ny, nz);
      hipLaunchKernelGGL(wgrad_reduce<4>, rgrid, dim3(1024), 0, s, g, part, gw_off, w.nbx, w.nz);
    } else {
      hipLaunchKernelGGL(offset_wgrad_valu<1>, grid, dim3(256), 0, s, g, xT, goffT, part, rpw,
                         nbx, ny, nz);
      hipLaunchKernelGGL(wgrad_reduce<1>, rgrid, dim3(1024), 0, s, g, part, gw_off, w.nbx, w.nz);
    }
  }
  {
    const int n = g.J * KK * pad_c(g.C);
    hipLaunchKernelGGL(woff_to_jtc, dim3((n + 255) / 256), dim3(256), 0, s, w_off, wt2, g.J, g.C,
                       pad_c(g.C), KK);
    const long Mi = (long)g.B * g.HWi;
    {
      dim3 grid((unsigned)((Mi + 255) / 256), (g.C + kCB - 1) / kCB);
      DCN_KK_DISPATCH(KK, hipLaunchKernelGGL(offset_dgrad_valu<KKc>, grid, dim3(256), 0, s, g,
                                             wt2, goff, gx, gxT_in));
    }
  }
  return hipGetLastError();
}

}  // namespace dcn
