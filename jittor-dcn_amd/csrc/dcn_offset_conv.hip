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
#include "dcn_swizzle.h"

// r05 (config 4): two-row workgroups on the 3-tap weight ring, offset forward 0.0362-0.0369
// -> 0.0338-0.0342 ms (one wave per SIMD at 296 registers, but no L2 wait per tap)
#ifndef OFFC_KF2
#define OFFC_KF2 14
#endif
#ifndef OFFC_ROWS
#define OFFC_ROWS 2
#endif
// r05 (config 4): the ∂W_off kernel on pre-split records gathered as bf16 pairs measured
// 0.092-0.0926 ms for the offset backward against 0.0913-0.0916 on fp32 split in the loop
// (its 32 two-byte LDS reads per step cost more than the split), so it splits in the loop
// r05 (config 4): the ∂x kernel on the side stream beside ∂W_off + its fold (they share
// only their inputs): offset backward 0.0914-0.092 -> 0.0896-0.0901 ms
#ifndef OFFB_CONC
#define OFFB_CONC 1
#endif
// r05 (config 4): the ∂x kernel on pre-split records, offset backward 0.0944-0.0951 ->
// 0.092-0.0926 ms (k loop 11.3 -> 7.9 us per workgroup, r05 phase stamps)
// ∂x kernel: Wc fragments kPf - 1 k-steps ahead (r05, config 4: 3 -> 5, offset backward
// 0.0913-0.0921 -> 0.0895-0.0905 ms; 135 registers)
// fp32 ∂x kernel (offset_dgrad_mfma): weight fragments kPf steps ahead (r05, config 3: 3 and 4
// measured no faster than 2)
#ifndef OFFDM_PF
#define OFFDM_PF 2
#endif
#ifndef OFFD_PF
#define OFFD_PF 5
#endif
// r05 (config 4): two channel groups per ∂W_off workgroup, offset backward 0.0921-0.0933 ->
// 0.0899-0.0908 ms (the shared ∂offset staging is half the instructions per channel)
#ifndef STAGE_NOSC
#define STAGE_NOSC 1
#endif
#ifndef OFFW_CPB
#define OFFW_CPB 2
#endif
#ifndef OFFW_CGB
#define OFFW_CGB 2
#endif
#ifndef OFFW_SB
#define OFFW_SB 1
#endif
#ifndef OFFW_PF
#define OFFW_PF 3
#endif
#ifndef OFFW_SG
#define OFFW_SG 8
#endif

namespace dcn {

constexpr int kJB = 18;  // offset channels per pass (one pass for the reference's 3x3)
constexpr int kCB = 32;  // channels per K7b pass
constexpr int kOcgMaxW = 128;  // ocg_col2im: input row width held in LDS

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
// wT2[(j*KK + tap)*Cp + c] = w_off[j][c][tap] for rows < J*KK (0 for c >= C and for the
// padding rows up to `rows`)
__global__ __launch_bounds__(256) void woff_to_jtc(const float* __restrict__ w,
                                                   float* __restrict__ wt, int J, int C, int Cp,
                                                   int KK, int rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * Cp) return;
  const int r = i / Cp, c = i - r * Cp;  // r = j*KK + tap
  const int j = r / KK, tap = r - j * KK;
  wt[i] = (c < C && r < J * KK) ? w[((size_t)j * C + c) * KK + tap] : 0.f;
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
static int wgrad_rpw() { return kWgradRpw; }
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
// K7 on MFMA (stride 1). Both backward products contract against the same shifted
// ∂offset operand G[p][tj] = ∂off[b][j][y+ph-i·dh][x+pw-k·dw] (0 outside the output),
// indexed by INPUT pixel p = (y, x) and tj = j·KK + tap (tap = i·kw + k):
//   ∂w_off[j][c][tap] = Σ_p xT[p][c] · G[p][tj]          M = c, N = tj, K = pixels
//   ∂x[c][p]          = Σ_tj w_off[j][c][tap] · G[p][tj]  M = c, N = pixels, K = tj
// With the channels on the MFMA rows, the J·KK = 162 (j, tap) columns pad only to 176
// (92 % useful) instead of J = 18 -> 32. G is never materialised: a block stages the
// ∂offset rows its pixels reach into LDS as S[sr][sc][j] (zero where the output has no
// pixel), and G[p][tj] = S[base(p) + toff(tj)] with base(p) = ((y-y0)·SW + x)·J and
// toff(tj) = ((kh-1-i)·dh·SW + (kw-1-k)·dw)·J + j. 16x16x4 f32 MFMA = exact f32 products
// accumulated in k order (deterministic, no atomics).
// ---------------------------------------------------------------------------
struct MfmaStage {
  int SW;      // staged columns: W + (kw-1)·dw
  int rowsB;   // input rows per ∂W chunk
  int cpi;     // ∂W chunks per image
  int spi;     // ∂x pixel strips (64 px) per image
  int SRx;     // staged rows bound for a ∂x strip
  size_t lds_w, lds_x;  // dynamic LDS bytes
};
constexpr int kMfmaLds = 64 * 1024;
constexpr int kDgPx = 64;  // ∂x pixels per block (4 waves = 4 x 64 channels)
constexpr int kDgTP = 68;  // bf16 ∂x epilogue: LDS pitch (floats) of a 64-channel pixel row
constexpr int kWgMfmaRows = 7;  // config 3: 56 rows = 8 chunks, 2048 blocks = 2 full rounds

static int tj_pad4(const Geo& g) { return (g.J * g.kh * g.kw + 3) / 4 * 4; }

// geometry the MFMA kernels take (stride 1, C % 4 == 0, C <= 256, J*KK <= 176, LDS fits)
static bool mfma_stage(const Geo& g, MfmaStage* m) {
  if (g.sh != 1 || g.sw != 1 || g.C % 4 != 0 || g.C > 256 || g.J * g.kh * g.kw > 176)
    return false;
  m->SW = g.W + (g.kw - 1) * g.dw;
  const size_t row_bytes = (size_t)m->SW * g.J * sizeof(float);
  const int halo = (g.kh - 1) * g.dh;
  int rows = std::min(kWgMfmaRows, g.H);
  while (rows > 0 && (size_t)(rows + halo) * row_bytes > kMfmaLds) --rows;
  if (rows == 0) return false;
  m->cpi = (g.H + rows - 1) / rows;
  m->rowsB = (g.H + m->cpi - 1) / m->cpi;  // balanced chunks
  m->lds_w = (size_t)(m->rowsB + halo) * row_bytes;
  m->spi = (g.HWi + kDgPx - 1) / kDgPx;
  m->SRx = (kDgPx - 1) / g.W + 2 + halo;
  m->lds_x = (size_t)tj_pad4(g) * sizeof(int) + (size_t)m->SRx * row_bytes;
  return m->lds_x <= kMfmaLds;
}
// fp32 ∂W_off on offset_wgrad_mfma_m1 (3x3, J = 18; W % 4 == 0, C % 64 == 0), and how many row
// chunks one of its workgroups sums (2: half the partials written and folded; one per
// workgroup measured 0.449 against 0.435 ms). Every other geometry:
// offset_wgrad_mfma, one partial per chunk.
static bool wgrad_m1(const Geo& g) {
  const int TJ = g.J * g.kh * g.kw;
  return g.dt != DCN_BF16 && g.W % 4 == 0 && g.C % 64 == 0 && TJ > 160 && TJ <= 162;
}
static int wgrad_cpb(const Geo& g, const MfmaStage& m) {
  return (wgrad_m1(g) && m.cpi % 2 == 0) ? 2 : 1;
}
static size_t wgrad_mfma_part_floats(const Geo& g, const MfmaStage& m) {
  return (size_t)g.B * m.cpi * g.C * g.J * g.kh * g.kw;
}

// S[(sr*SW + sc)*J + j] = ∂off[b][j][y0 + sr - (kh-1)·dh + ph][sc - (kw-1)·dw + pw]
// kU loads per thread are in flight together (clamped in-bounds addresses, masked after),
// so staging costs a few memory latencies per block, not one per element.
__device__ __forceinline__ void stage_goff(const Geo& g, const float* __restrict__ goff, int b,
                                           int y0, int SR, int SW, float* S) {
  constexpr int kU = 8;
  const int plane = SR * SW, n = plane * g.J;
  // n <= 16384 (64 KiB of LDS) and plane <= 8192: umulhi by ceil(2^32/d) is the exact
  // quotient there (checked for every d <= 8192, idx < 65536), instead of ~40-instruction
  // integer divides per element
  const unsigned mp = 0xffffffffu / (unsigned)plane + 1u, ms = 0xffffffffu / (unsigned)SW + 1u;
  // buffer loads: a position outside the image reads 0 through the range check (no select
  // after the load, which ties each load's wait to its own condition register)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(goff + (size_t)b * g.J * g.HW),
                                                    0, (int)((size_t)g.J * g.HW * 4), 0x00020000);
  for (int i0 = threadIdx.x; i0 < n; i0 += blockDim.x * kU) {
    float v[kU];
    int dst[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // sc fastest: coalesced reads
      const int idx = min(i0 + u * (int)blockDim.x, n - 1);
      const int j = (int)__umulhi((unsigned)idx, mp), rem = idx - j * plane;
      const int sr = (int)__umulhi((unsigned)rem, ms), sc = rem - sr * SW;
      const int ho = y0 + sr - (g.kh - 1) * g.dh + g.ph, wo = sc - (g.kw - 1) * g.dw + g.pw;
#if STAGE_NOSC
      const bool ok = ((unsigned)ho < (unsigned)g.Ho) & ((unsigned)wo < (unsigned)g.Wo);
#else
      const bool ok = ho >= 0 && ho < g.Ho && wo >= 0 && wo < g.Wo;
#endif
      const unsigned o = ok ? (unsigned)((j * g.HW + ho * g.Wo + wo) * 4) : 0x80000000u;
      v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
      dst[u] = rem * g.J + j;
    }
    // unconditional: a slot past n holds element n-1 (clamped idx) and rewrites it with its
    // own value, so no exec-masked store blocks (each makes the waitcnt pass drain, vmcnt(0));
    // the barrier keeps all kU loads issued before the first store
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kU; ++u) S[dst[u]] = v[u];
  }
}

__device__ __forceinline__ int g_toff(const Geo& g, int tj, int SW) {
  const int KK = g.kh * g.kw;
  if (tj >= g.J * KK) return 0;  // padding column: any finite staged value
  const int j = tj / KK, t = tj - j * KK;
  const int i = t / g.kw, k = t - i * g.kw;
  return ((g.kh - 1 - i) * g.dh * SW + (g.kw - 1 - k) * g.dw) * g.J + j;
}

// ∂W_off partials: block = (chunk of rowsB input rows of one image, 64 channels); wave w
// owns N-tiles w, w+4, w+8 (all 4 channel tiles), so no cross-wave reduction. Lane
// (n = l&15, q = l>>4) loads channels c0+4n..+3 of pixel x0+q as one float4: element e
// is row n of M-tile e (tile e = channels c0+4r+e). part[chunk][c][tj].
// 4 channels of xT through a buffer resource: fp32 (16 B) or bf16 (8 B, widened; DCN_BF16
// passes its channels-last bf16 copy, whose products are then exact f32 MFMA products too)
template <typename XT>
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, int soff) {
  if constexpr (sizeof(XT) == 4) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                       __uint_as_float(v[3]));
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, soff, 0);
    return make_float4(__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u),
                       __uint_as_float(v[1] << 16), __uint_as_float(v[1] & 0xffff0000u));
  }
}

template <int NTW, bool W4, typename XT = float>
__global__ __launch_bounds__(256) void offset_wgrad_mfma(Geo g, const XT* __restrict__ xT,
                                                        const float* __restrict__ goff,
                                                        float* __restrict__ part, int rowsB,
                                                        int cpi, int chunk0) {
  extern __shared__ float S[];
  const int chunk = chunk0 + blockIdx.x;
  const int b = chunk / cpi, y0 = (chunk - b * cpi) * rowsB;
  const int nrows = min(rowsB, g.H - y0);
  const int SW = g.W + (g.kw - 1) * g.dw;
  stage_goff(g, goff, b, y0, nrows + (g.kh - 1) * g.dh, SW, S);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = lane & 15, q = lane >> 4;
  const int TJ = g.J * g.kh * g.kw;
  int toff[NTW];
  // wave-uniform: N-tiles wholly past TJ (config 3: tile 11 = tj 176..191 of 162) are
  // skipped, not multiplied (their sums were never stored)
  bool tv[NTW];
#pragma unroll
  for (int u = 0; u < NTW; ++u) {
    toff[u] = g_toff(g, 16 * (w + 4 * u) + n, SW);
    tv[u] = 16 * (w + 4 * u) < TJ;
  }
  const int cb = blockIdx.y * 64;
  const bool cok = cb + 4 * n < g.C;
  f32x4 acc[4][NTW];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int u = 0; u < NTW; ++u) acc[e][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // The chunk's K-steps (4 pixels of one row each) run through a kPf-deep register ring of
  // xT loads; buffer loads (clamped in-bounds offsets, masked after) keep the prefetch from
  // being folded back into a load-then-wait per step. The step count is padded to a
  // multiple of kPf with zero-operand steps, so the unrolled body has no early exit.
  constexpr int kPf = 4;
  const int nq = (g.W + 3) / 4, nsteps = nrows * nq;
  constexpr int XB = (int)sizeof(XT);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<XT*>(xT + ((size_t)b * g.H + y0) * g.W * g.C), 0,
      (int)((size_t)max(nrows, 1) * g.W * g.C * XB), 0x00020000);
  const int cl = cok ? cb + 4 * n : 0;
  float4 ring[kPf];
  if (W4) {
    // W % 4 == 0: step ks covers pixels 4ks..4ks+3 of the chunk, so the xT offset is
    // linear in ks and a row change is wave-uniform: all per-step addressing is one
    // scalar add (no per-lane divides, clamps or multiplies in the loop)
    const unsigned lane_x = (unsigned)((q * g.C + cl) * XB);
    const int step_x = 4 * XB * g.C, last = (nsteps - 1) * step_x;
    int lo = 0;  // scalar byte offset of the step being loaded
#pragma unroll
    for (int d = 0; d < kPf; ++d, lo += step_x) ring[d] = buf_ld4<XT>(rsrc, lane_x, min(lo, last));
    int bv0[NTW];  // lane part of the B addresses
#pragma unroll
    for (int u = 0; u < NTW; ++u) bv0[u] = q * g.J + toff[u];
    int sb = 0, sx = 0;  // S offset (floats) of the step being multiplied, its step in row
    const int row_skip = (SW - g.W) * g.J;
    for (int ks0 = 0; ks0 < nsteps; ks0 += kPf) {
#pragma unroll
      for (int d = 0; d < kPf; ++d) {
        const unsigned keep = ks0 + d < nsteps ? 0xffffffffu : 0u;  // wave-uniform
        const float ax = __uint_as_float(__float_as_uint(ring[d].x) & keep);
        const float ay = __uint_as_float(__float_as_uint(ring[d].y) & keep);
        const float az = __uint_as_float(__float_as_uint(ring[d].z) & keep);
        const float aw = __uint_as_float(__float_as_uint(ring[d].w) & keep);
        // the padding steps past nsteps read LDS beyond the staged rows: mask B as well as
        // A (0 x a stale NaN/Inf bit pattern would poison the accumulator)
        float bv[NTW];
#pragma unroll
        for (int u = 0; u < NTW; ++u)
          bv[u] = tv[u] ? __uint_as_float(__float_as_uint(S[sb + bv0[u]]) & keep) : 0.f;
        sb += 4 * g.J;
        if (++sx == nq) sx = 0, sb += row_skip;
#pragma unroll
        for (int u = 0; u < NTW; ++u)
          if (tv[u]) mfma16x4_acc(acc[0][u], acc[1][u], acc[2][u], acc[3][u], ax, ay, az, aw, bv[u]);
        ring[d] = buf_ld4<XT>(rsrc, lane_x, min(lo, last));
        lo += step_x;
      }
    }
  } else {
    // (row, column) of the step being loaded, kPf steps ahead of the one being multiplied
    int ly = 0, lx = q;
    auto load_next = [&]() {
      const unsigned off =
          (unsigned)(((min(ly, nrows - 1) * g.W + min(lx, g.W - 1)) * g.C + cl) * XB);
      lx += 4;
      if (lx >= nq * 4) lx = q, ++ly;
      return buf_ld4<XT>(rsrc, off, 0);
    };
#pragma unroll
    for (int d = 0; d < kPf; ++d) ring[d] = load_next();
    int cy = 0, cx = q;  // the step being multiplied
    for (int ks0 = 0; ks0 < nsteps; ks0 += kPf) {
#pragma unroll
      for (int d = 0; d < kPf; ++d) {
        // bitwise mask: exact zeros (also for the padding steps past nsteps), no branch
        const unsigned keep = (cok && cx < g.W && cy < nrows) ? 0xffffffffu : 0u;
        const float ax = __uint_as_float(__float_as_uint(ring[d].x) & keep);
        const float ay = __uint_as_float(__float_as_uint(ring[d].y) & keep);
        const float az = __uint_as_float(__float_as_uint(ring[d].z) & keep);
        const float aw = __uint_as_float(__float_as_uint(ring[d].w) & keep);
        const float* sp = S + (min(cy, nrows - 1) * SW + min(cx, g.W - 1)) * g.J;
        cx += 4;
        if (cx >= nq * 4) cx = q, ++cy;
        float bv[NTW];
#pragma unroll
        for (int u = 0; u < NTW; ++u) bv[u] = tv[u] ? sp[toff[u]] : 0.f;
#pragma unroll
        for (int u = 0; u < NTW; ++u)
          if (tv[u]) mfma16x4_acc(acc[0][u], acc[1][u], acc[2][u], acc[3][u], ax, ay, az, aw, bv[u]);
        ring[d] = load_next();  // after the slot's last use: no register copy
      }
    }
  }
  float* pp = part + (size_t)chunk * g.C * TJ;
#pragma unroll
  for (int u = 0; u < NTW; ++u) {
    const int tj = 16 * (w + 4 * u) + n;
    if (tj >= TJ) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = cb + 4 * (4 * q + r) + e;
        if (c < g.C) pp[(size_t)c * TJ + tj] = acc[e][u][r];
      }
  }
}

// ∂W_off partials with one M-tile (16 channels) per wave over every N-tile: TJ = 160 + NV tap
// columns (3x3, J = 18: NV = 2) as 10 N-tiles of 16 on the f32 MFMA plus the last NV <= 2
// columns on the VALU, so the 4 waves carry equal MFMA work and none multiplies padding
// (offset_wgrad_mfma<3>: 4 M-tiles per wave over 3 of 12 N-tiles = 192 tap columns, 30 of
// them padding, wave 3 lighter). Lane (n = l&15, q = l>>4): A = xT[pixel 4ks+q][channel
// cw+n] (fp32, W % 4 == 0, C % 64 == 0); tile T: B = ∂offset at tap column 16T+n of pixel
// 4ks+q. part[chunk][c][tj] as offset_wgrad_mfma; the same xT register ring and the same
// zero-operand padding steps.
// A workgroup sums cpb consecutive row chunks of one image (cpi % cpb == 0) into one partial:
// part[grp][c][tj], grp = chunk / cpb.
__global__ __launch_bounds__(256) void offset_wgrad_mfma_m1(Geo g, const float* __restrict__ xT,
                                                           const float* __restrict__ goff,
                                                           float* __restrict__ part, int rowsB,
                                                           int cpi, int grp0, int cpb) {
  extern __shared__ float S[];
  const int grp = grp0 + blockIdx.x;
  const int SW = g.W + (g.kw - 1) * g.dw;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, q = lane >> 4;
  const int TJ = g.J * g.kh * g.kw, NV = TJ - 160;
  int bv0[10], vv0[2];
#pragma unroll
  for (int t = 0; t < 10; ++t) bv0[t] = q * g.J + g_toff(g, 16 * t + n, SW);
#pragma unroll
  for (int r = 0; r < 2; ++r) vv0[r] = q * g.J + g_toff(g, 160 + r, SW);  // 0 past TJ
  const int cw = blockIdx.y * 64 + 16 * w;
  f32x4 acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float va[2] = {0.f, 0.f};
  for (int cc = 0; cc < cpb; ++cc) {
    const int chunk = grp * cpb + cc;
    const int b = chunk / cpi, y0 = (chunk - b * cpi) * rowsB;
    const int nrows = min(rowsB, g.H - y0);
    if (cc) __syncthreads();  // the previous chunk's LDS reads are done
    stage_goff(g, goff, b, y0, nrows + (g.kh - 1) * g.dh, SW, S);
    __syncthreads();
    constexpr int kPf = 4;
    const int nq = g.W / 4, nsteps = nrows * nq;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(xT + ((size_t)b * g.H + y0) * g.W * g.C), 0,
        (int)((size_t)max(nrows, 1) * g.W * g.C * 4), 0x00020000);
    const unsigned lane_x = (unsigned)((q * g.C + cw + n) * 4);
    const int step_x = 16 * g.C, last = (nsteps - 1) * step_x;
    auto ld = [&](int so) {
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, lane_x, so, 0));
    };
    float ring[kPf];
    int lo = 0;
#pragma unroll
    for (int d = 0; d < kPf; ++d, lo += step_x) ring[d] = ld(min(lo, last));
    int sb = 0, sx = 0;
    const int row_skip = (SW - g.W) * g.J;
    for (int ks0 = 0; ks0 < nsteps; ks0 += kPf) {
#pragma unroll
      for (int d = 0; d < kPf; ++d) {
        const unsigned keep = ks0 + d < nsteps ? 0xffffffffu : 0u;  // wave-uniform
        const float a = __uint_as_float(__float_as_uint(ring[d]) & keep);
        float bv[10], vb[2];
#pragma unroll
        for (int t = 0; t < 10; ++t) bv[t] = __uint_as_float(__float_as_uint(S[sb + bv0[t]]) & keep);
#pragma unroll
        for (int r = 0; r < 2; ++r) vb[r] = __uint_as_float(__float_as_uint(S[sb + vv0[r]]) & keep);
        sb += 4 * g.J;
        if (++sx == nq) sx = 0, sb += row_skip;
        mfma16x4_a5(acc[0], acc[1], acc[2], acc[3], acc[4], a, bv[0], bv[1], bv[2], bv[3], bv[4]);
        mfma16x4_a5(acc[5], acc[6], acc[7], acc[8], acc[9], a, bv[5], bv[6], bv[7], bv[8], bv[9]);
        va[0] = fmaf(a, vb[0], va[0]);
        va[1] = fmaf(a, vb[1], va[1]);
        ring[d] = ld(min(lo, last));
        lo += step_x;
        // keep the load here, kPf steps ahead of its use: left alone, the scheduler hoists
        // the later steps' MFMAs above it, so the ring's loads issue at the end of the
        // unrolled body, just before the next iteration's first use (a barrier that holds
        // only the vector-memory instructions, mask 0x78F, still lets that happen)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }  // chunks
  float* pp = part + (size_t)grp * g.C * TJ;
  // D: row (channel cw + 4q + r), column (tap column 16t + n)
#pragma unroll
  for (int t = 0; t < 10; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) pp[(size_t)(cw + 4 * q + r) * TJ + 16 * t + n] = acc[t][r];
  // the VALU columns: lane (n, q) holds channel cw+n over pixels ≡ q (mod 4); fixed xor tree
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float v = va[r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (r < NV && q == 0) pp[(size_t)(cw + n) * TJ + 160 + r] = v;
  }
}

// The same ∂W_off partials on v_mfma_f32_32x32x2f32 (C % 128 == 0 besides m1's conditions): a
// wave owns 32 channels (M = 32) over the 160 MFMA tap columns as 5 N-tiles of 32, K = 2
// pixels per step, the last NV <= 2 columns on the VALU. Per step a wave reads 5 + 2 LDS
// words per lane for 5 MFMAs (m1: 10 + 2 for 10 16x16x4 MFMAs of the same flops), and a
// workgroup (4 waves, 128 channels) stages each ∂offset chunk for twice m1's channels. Lane
// (i = l&31, k = l>>5): A = xT[pixel 2ks+k][channel cw+i]; tile T: B = ∂offset at tap column
// 32T+i of pixel 2ks+k; D[row][col] in register r of lane col + 32·hi, row = drow(r, hi).
__global__ __launch_bounds__(256) void offset_wgrad_mfma_m2(Geo g, const float* __restrict__ xT,
                                                           const float* __restrict__ goff,
                                                           float* __restrict__ part, int rowsB,
                                                           int cpi, int grp0, int cpb) {
  extern __shared__ float S[];
  const int grp = grp0 + blockIdx.x;
  const int SW = g.W + (g.kw - 1) * g.dw;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 31, k = lane >> 5;
  const int TJ = g.J * g.kh * g.kw, NV = TJ - 160;
  int bv0[5], vv0[2];
#pragma unroll
  for (int t = 0; t < 5; ++t) bv0[t] = k * g.J + g_toff(g, 32 * t + i, SW);
#pragma unroll
  for (int r = 0; r < 2; ++r) vv0[r] = k * g.J + g_toff(g, 160 + r, SW);  // 0 past TJ
  const int cw = blockIdx.y * 128 + 32 * w;
  f32x16 acc[5];
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float va[2] = {0.f, 0.f};
  for (int cc = 0; cc < cpb; ++cc) {
    const int chunk = grp * cpb + cc;
    const int b = chunk / cpi, y0 = (chunk - b * cpi) * rowsB;
    const int nrows = min(rowsB, g.H - y0);
    if (cc) __syncthreads();  // the previous chunk's LDS reads are done
    stage_goff(g, goff, b, y0, nrows + (g.kh - 1) * g.dh, SW, S);
    __syncthreads();
    constexpr int kPf = 4;
    const int nq = g.W / 2, nsteps = nrows * nq;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(xT + ((size_t)b * g.H + y0) * g.W * g.C), 0,
        (int)((size_t)max(nrows, 1) * g.W * g.C * 4), 0x00020000);
    const unsigned lane_x = (unsigned)((k * g.C + cw + i) * 4);
    const int step_x = 8 * g.C, last = (nsteps - 1) * step_x;
    auto ld = [&](int so) {
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, lane_x, so, 0));
    };
    float ring[kPf];
    int lo = 0;
#pragma unroll
    for (int d = 0; d < kPf; ++d, lo += step_x) ring[d] = ld(min(lo, last));
    int sb = 0, sx = 0;
    const int row_skip = (SW - g.W) * g.J;
    for (int ks0 = 0; ks0 < nsteps; ks0 += kPf) {
#pragma unroll
      for (int d = 0; d < kPf; ++d) {
        const unsigned keep = ks0 + d < nsteps ? 0xffffffffu : 0u;  // wave-uniform
        const float a = __uint_as_float(__float_as_uint(ring[d]) & keep);
        float bv[5], vb[2];
#pragma unroll
        for (int t = 0; t < 5; ++t) bv[t] = __uint_as_float(__float_as_uint(S[sb + bv0[t]]) & keep);
#pragma unroll
        for (int r = 0; r < 2; ++r) vb[r] = __uint_as_float(__float_as_uint(S[sb + vv0[r]]) & keep);
        sb += 2 * g.J;
        if (++sx == nq) sx = 0, sb += row_skip;
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] = mfma32(a, bv[t], acc[t]);
        va[0] = fmaf(a, vb[0], va[0]);
        va[1] = fmaf(a, vb[1], va[1]);
        ring[d] = ld(min(lo, last));
        lo += step_x;
        __builtin_amdgcn_sched_barrier(0);  // the load stays kPf steps ahead (see m1)
      }
    }
  }  // chunks
  float* pp = part + (size_t)grp * g.C * TJ;
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) pp[(size_t)(cw + drow(r, k)) * TJ + 32 * t + i] = acc[t][r];
  // the VALU columns: lane (i, k) holds channel cw+i over pixels ≡ k (mod 2)
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float v = va[r];
    v += __shfl_xor(v, 32);
    if (r < NV && k == 0) pp[(size_t)(cw + i) * TJ + 160 + r] = v;
  }
}

// ∂w_off[j][c][tap] = Σ_chunk part[chunk][c][j·KK + tap], chunks in order: 64 elements per
// 1024-thread block, wave w sums chunks ≡ w (mod 16), the 16 wave sums fold in order.
// a lane's 4 consecutive elements as one float4 (1 KiB per wave load, 256 elements per block;
// E = C·J·kh·kw is a multiple of 4 since mfma_stage requires C % 4 == 0); per element the same
// additions in the same order as r05's one-element-per-lane form
__global__ __launch_bounds__(1024) void wgrad_mfma_reduce(Geo g, const float* __restrict__ part,
                                                         int nchunk, float* __restrict__ gw) {
  const int KK = g.kh * g.kw, TJ = g.J * KK;
  const long E = (long)g.C * TJ;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i0 = (long)blockIdx.x * 256 + 4 * lane;
  const long ic = i0 < E ? i0 : 0;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int ch = w; ch < nchunk; ch += 16) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)ch * E + ic);
    s[0] += v.x;
    s[1] += v.y;
    s[2] += v.z;
    s[3] += v.w;
  }
  __shared__ float red[16][256];
#pragma unroll
  for (int e = 0; e < 4; ++e) red[w][4 * lane + e] = s[e];
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long i = i0 + e;
    if (i >= E) break;
    float t0 = red[0][4 * lane + e];
#pragma unroll
    for (int k = 1; k < 16; ++k) t0 += red[k][4 * lane + e];
    const int c = (int)(i / TJ), tj = (int)(i - (long)c * TJ);
    const int j = tj / KK, t = tj - j * KK;
    gw[((size_t)j * g.C + c) * KK + t] = t0;
  }
}

// ∂x (+)= convᵀ: block = one 64-pixel strip of an image, wave w = channels 64w..64w+63
// (4 M-tiles) x the strip's 4 pixel N-tiles; K = tj in steps of 4. A = w_off from wt2
// (L2-resident, buffer loads two K-steps ahead), B = the staged ∂offset rows.
// D lane map: pixel p0+16u+(l&15), channels c+16m+4(l>>4)+r: the ∂x row store is 16 lanes
// x 4 B contiguous per channel, and the ∂xT add is one float4 per lane.
// (256, 4): 4 blocks per CU so one block's MFMA phase overlaps another's ∂x epilogue
// (r01: 225 -> 217 us at config 3)
__global__ __launch_bounds__(256, 4) void offset_dgrad_mfma(Geo g, const float* __restrict__ wt2,
                                                        int Cp, const float* __restrict__ goff,
                                                        float* __restrict__ gx,
                                                        const float* __restrict__ gxT_in,
                                                        int spi, int blk0) {
  extern __shared__ float smem[];
  const int TJp = (g.J * g.kh * g.kw + 3) / 4 * 4;
  int* T = reinterpret_cast<int*>(smem);
  float* S = smem + TJp;
  const int bid = blk0 + blockIdx.x;
  const int b = bid / spi, p0 = (bid - b * spi) * kDgPx;
  const int np = min(kDgPx, g.HWi - p0);
  const int y0 = p0 / g.W, y1 = (p0 + np - 1) / g.W;
  const int SW = g.W + (g.kw - 1) * g.dw;
  stage_goff(g, goff, b, y0, y1 - y0 + 1 + (g.kh - 1) * g.dh, SW, S);
  for (int t = threadIdx.x; t < TJp; t += blockDim.x) T[t] = g_toff(g, t, SW);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, q = lane >> 4;
  const int cw = 64 * w;
  if (cw >= g.C) return;
  int base[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = p0 + min(16 * u + n, np - 1);
    const int y = p / g.W, x = p - y * g.W;
    base[u] = ((y - y0) * SW + x) * g.J;
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[m][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int KS = TJp / 4;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wt2), 0,
                                                      TJp * Cp * (int)sizeof(float), 0x00020000);
  const unsigned lo = (unsigned)((q * Cp + cw + n) * 4);
  // A[c = n (+16m)][k = tj = 4ks + q]; slot d of the ring holds K-step ks0 + d
  auto lda = [&](int ks, float (&a)[4]) {
    const int so = min(ks, KS - 1) * 4 * Cp * 4;
#pragma unroll
    for (int m = 0; m < 4; ++m)
      a[m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, lo + 64 * m, so, 0));
  };
  constexpr int kPf = OFFDM_PF;
  float ra[kPf][4];
#pragma unroll
  for (int d = 0; d < kPf; ++d) lda(d, ra[d]);
  for (int ks0 = 0; ks0 < KS; ks0 += kPf) {
#pragma unroll
    for (int d = 0; d < kPf; ++d) {
      const int ks = ks0 + d;
      // a padding step past KS multiplies zero weights (wt2 rows >= J*KK are zero, and
      // the clamped load re-reads the last row: masked here)
      const unsigned keep = ks < KS ? 0xffffffffu : 0u;
      const int to = T[min(ks, KS - 1) * 4 + q];
      float bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u] = S[base[u] + to];
      float a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = __uint_as_float(__float_as_uint(ra[d][m]) & keep);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        mfma16x4_acc(acc[0][u], acc[1][u], acc[2][u], acc[3][u], a[0], a[1], a[2], a[3], bv[u]);
      lda(ks + kPf, ra[d]);
      // the loads stay kPf steps ahead (offset_wgrad_mfma_m1 says why)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int pl = 16 * u + n;
    if (pl >= np) continue;
    const size_t p = (size_t)p0 + pl;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int c = cw + 16 * m + 4 * q;
      if (c >= g.C) continue;  // C % 4 == 0: c..c+3 all in or all out
      const f32x4 v = acc[m][u];
      float* d = gx + ((size_t)b * g.C + c) * g.HWi + p;
      if (gxT_in) {
        const float4 t = *reinterpret_cast<const float4*>(gxT_in + ((size_t)b * g.HWi + p) * g.C + c);
        d[0] = t.x + v[0];
        d[g.HWi] = t.y + v[1];
        d[2 * (size_t)g.HWi] = t.z + v[2];
        d[3 * (size_t)g.HWi] = t.w + v[3];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r * (size_t)g.HWi] += v[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K3 on the bf16 matrix cores (DCN_BF16). The inputs are bf16, so every product w·x is
// exact in fp32 and the MFMA sums are fp32: the arithmetic of the fp32 kernels on the
// same values, in another summation order.
//   off[b][j][p] = b_off[j] + Σ_{tap, c} w_off[j][c][tap] · xT[b][shift_tap(p)][c]
// One block = 32 output pixels of one image x all J <= 32 offset channels: one 32x32 f32
// tile of v_mfma_f32_32x32x16_bf16 (pixels on the rows, offset channels on the columns).
// Its 4 waves split the input channels; A = the channels-last bf16 x (lane: 8 channels of
// one pixel, one 16-B load), B = the weights as wb[tap][j][c] (lane: 8 channels of one j),
// so no LDS staging and no transpose. The 4 channel partials fold through LDS in wave
// order, then + bias, then the bf16 rounding the sampling uses (off32 = that value).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// The B fragments in MFMA lane order, so a wave's B load is one contiguous 1 KiB:
// wb[((tap*NKS + ks)*64 + lane)*8 + e] = w_off[j = lane&31][c = 16ks + 8(lane>>5) + e][tap]
// (bf16), 0 for j >= J or c >= C; NKS = Cp/16 k-steps per tap
__global__ __launch_bounds__(256) void woff_to_tjc_bf16(const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ wb, int J, int C,
                                                       int Cp, int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < KK * 32 * Cp) swz_tjc(w, wb, J, C, Cp, KK, i);
}

__device__ __forceinline__ bf16x8_t ld_bf16x8(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
// the same from an address that is only 8-byte aligned (two 8-byte loads)
__device__ __forceinline__ bf16x8_t ld_bf16x8_a8(const bf16_t* p) {
  const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 4);
  return __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

template <int SPT>  // 16-channel k-steps per tap and wave, loads issued together
__global__ __launch_bounds__(256) void offset_conv_fwd_mfma_bf16(
    Geo g, const bf16_t* __restrict__ xT, const bf16_t* __restrict__ wb, int Cp,
    const float* __restrict__ b_off, float* __restrict__ off32, bf16_t* __restrict__ off,
    int tiles) {
  __shared__ f32x16 red[3][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Block3 blk = xcd_block();
  const int tile = blk.x, b = blk.z;
  const int r = lane & 31, hh = lane >> 5;
  const int p = tile * 32 + r;
  const bool pok = p < g.HW;
  const int ho = pok ? p / g.Wo : 0, wo = pok ? p - (p / g.Wo) * g.Wo : 0;
  const int c0 = w * SPT * 16 + 8 * hh;  // this lane's first channel in each tap
  const bf16_t* xb = xT + (size_t)b * g.HWi * g.C;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const int KK = g.kh * g.kw;
  // software pipeline over the taps: tap t+1's operands are loaded before tap t's MFMAs
  // (one memory latency per kernel instead of one per tap)
  bf16x8_t a[2][SPT], bv[2][SPT];
  auto load = [&](int t, bf16x8_t(&ra)[SPT], bf16x8_t(&rb)[SPT]) {
    const int tt = min(t, KK - 1);  // past the last tap: a harmless re-load
    const int i = tt / g.kw, k = tt - i * g.kw;
    const int y = ho * g.sh - g.ph + i * g.dh, x = wo * g.sw - g.pw + k * g.dw;
    const bool ok = pok && y >= 0 && y < g.H && x >= 0 && x < g.W;
    const bf16_t* xp = xb + (size_t)(ok ? y * g.W + x : 0) * g.C;
    const bf16_t* wp = wb + ((size_t)(tt * (Cp / 16) + w * SPT) * 64 + lane) * 8;
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int c = c0 + 16 * u;
      const bool cin = c < g.C;  // the launcher takes C % 16 == 0: whole 8-channel runs
      ra[u] = ld_bf16x8(xp + (cin ? c : 0));
      if (!(ok && cin)) ra[u] = bf16x8_t{};
      rb[u] = ld_bf16x8(wp + 512 * u);  // zero-padded to Cp (multiple of 64)
    }
  };
  load(0, a[0], bv[0]);
  for (int t = 0; t < KK; t += 2) {
    load(t + 1, a[1], bv[1]);
#pragma unroll
    for (int u = 0; u < SPT; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][u], bv[0][u], acc, 0, 0, 0);
    if (t + 1 >= KK) break;
    load(t + 2, a[0], bv[0]);
#pragma unroll
    for (int u = 0; u < SPT; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][u], bv[1][u], acc, 0, 0, 0);
  }
  if (w > 0) red[w - 1][lane] = acc;
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const f32x16 o = red[q][lane];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += o[i];
  }
  // + bias, bf16 rounding; the tile goes through LDS as [j][pixel] so that the stores are
  // runs of 32 consecutive pixels per offset channel (lane = pixel), not 4-byte scatters
  // (lane = channel: every store instruction touched 64 lines)
  __shared__ float T[32][33];
  const float bj = r < g.J ? b_off[r] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) T[r][(i & 3) + 8 * (i >> 2) + 4 * hh] = bf2f(f2bf(acc[i] + bj));
  // wave 0 alone reads back what its own lanes wrote: LDS ops of one wave run in order, so
  // only the compiler must not move the reads above the writes
  __builtin_amdgcn_wave_barrier();
  const int pp = tile * 32 + r;
  if (pp < g.HW) {
    for (int j = hh; j < g.J; j += 2) {
      const float v = T[j][r];
      const size_t o = ((size_t)b * g.J + j) * g.HW + pp;
      off32[o] = v;
      off[o] = f2bf(v);  // exact: v is a bf16 value
    }
  }
}

// The same product with the x window in LDS: block = up to 32 output pixels of ONE output
// row (Wo >= 16), so the window is kh input rows x SWc columns. Each wave stages its own
// channel slice ([row][col][16·SPT channels + 8 pad] bf16: 16-B lane reads conflict-free)
// with coalesced 128-B-per-pixel loads (zeros outside the image via buffer-resource range
// checks), then reads its A fragments from LDS: each x byte leaves L2 once per block, not
// once per tap and pixel, and the global loads touch whole lines (the register-direct
// kernel's 16-B-per-pixel gathers touched 32 lines per load instruction).
// FOLD (f3): the window is staged from the NCHW bf16 x instead of xT, and the
// block writes its own input row (window row ph: stride 1, Ho == H) to xT — the channels-last
// copy K1 / the fused forward / K5 read — so x is read in one pass and the separate transpose
// launch disappears, as offset_conv_fwd_mfma_xt does for fp32 (offset_fwd_bf16_fold_ok).
// ROWS (FOLD only, r05): output rows per block; the window holds kh + ROWS - 1 input rows,
// so x leaves L2 (kh + ROWS - 1) / ROWS times instead of kh times, and each weight fragment
// loaded serves ROWS rows (config 4 measured the staging as the bandwidth-bound phase).
template <int SPT, bool FOLD = false, int ROWS = 1>
__global__ __launch_bounds__(256) void offset_conv_fwd_mfma_bf16_row(
    Geo g, const bf16_t* __restrict__ xT, const bf16_t* __restrict__ wb, int Cp,
    const float* __restrict__ b_off, float* __restrict__ off32, bf16_t* __restrict__ off,
    int tpr, int SWc, const bf16_t* __restrict__ x_nchw = nullptr, bf16_t* __restrict__ xT_out = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_row[];
  constexpr int P = 16 * SPT + 8;  // LDS pixel pitch (bf16)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Block3 blk = xcd_block();
  static_assert(ROWS == 1 || FOLD, "row blocks stage through the fold path");
  const int hb = blk.x / tpr, wo0 = (blk.x - hb * tpr) * 32, b = blk.z;
  const int ho = hb * ROWS;  // first output row
  const int r = lane & 31, hh = lane >> 5;
  const int KH = g.kh, KK = g.kh * g.kw;
  const int KHR = KH + ROWS - 1;  // staged window rows
  bf16_t* L = reinterpret_cast<bf16_t*>(smem_row) + (size_t)w * KHR * SWc * P;
  const int cw = w * SPT * 16;  // this wave's first channel
  // B = weight fragments (L2-resident) in a 3-tap register ring; r05: the first two taps
  // are requested before the window staging, so their latency hides behind it, and the
  // loop keeps two taps in flight (one ahead waited an L2 latency per tap)
  bf16x8_t bv[3][SPT];
  auto ldb = [&](int t, bf16x8_t(&rb)[SPT]) {
    const int tt = min(t, KK - 1);
    const bf16_t* wp = wb + ((size_t)(tt * (Cp / 16) + w * SPT) * 64 + lane) * 8;
#pragma unroll
    for (int u = 0; u < SPT; ++u) rb[u] = ld_bf16x8(wp + 512 * u);
  };
  // (two-row workgroups: the first two taps are requested after the staging, as the
  // registers are the occupancy limit)
  if constexpr (ROWS == 1) {
    ldb(0, bv[0]);
    ldb(1, bv[1]);
  }
  if constexpr (FOLD) {
    // zero the slice (image borders and the channel padding past C stay zero), then the
    // in-image part from NCHW rows: item = (channel pair, window row, 4-pixel chunk), two
    // 8-B loads (channels c, c+1) -> four 32-bit LDS stores of (c, c+1) per pixel
    const int nz = KHR * SWc * P / 8;
    for (int i = lane; i < nz; i += 64) reinterpret_cast<uint4*>(L)[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    const int NQ = g.W / 4, x0 = -g.pw;  // wo0 == 0 (tpr == 1)
    const int nit = 8 * SPT * KHR * NQ;
    // r05: a lane's items all in flight at once (kF per batch: one batch for kh = 3,
    // W <= 32, C = 256), through a buffer resource, so rows outside the image and channels
    // past C read zeros and every LDS store is unconditional (r04's serial loop waited
    // one memory latency per item, ~10 per block at config 4). A slot past nit repeats item
    // nit-1 (same value, same place).
    const auto rxn = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(x_nchw + (size_t)b * g.C * g.HWi), 0,
        (int)((size_t)g.C * g.HWi * 2), 0x00020000);
    // quotients by NQ and KH as umulhi by ceil(2^32/d), exact here (it < 2^16); d = 1 wraps
    // that multiplier to 0 and is taken apart
    const unsigned mq = 0xffffffffu / (unsigned)NQ + 1u, mk = 0xffffffffu / (unsigned)KHR + 1u;
    constexpr int kF = ROWS == 1 ? 12 : OFFC_KF2;
    for (int it0 = lane; it0 < nit; it0 += 64 * kF) {
      uint2 u0[kF], u1[kF];
      int dst[kF];
#pragma unroll
      for (int u = 0; u < kF; ++u) {
        const int it = min(it0 + 64 * u, nit - 1);
        const int rest = NQ == 1 ? it : (int)__umulhi((unsigned)it, mq), q = it - rest * NQ;
        const int cp = KHR == 1 ? rest : (int)__umulhi((unsigned)rest, mk), i = rest - cp * KHR;
        const int y = ho - g.ph + i, c = cw + 2 * cp;
        const bool ok = y >= 0 && y < g.H && c < g.C;
        const unsigned o = ok ? (unsigned)(((c * g.H + y) * g.W + 4 * q) * 2) : 0x80000000u;
        const auto a = __builtin_amdgcn_raw_buffer_load_b64(rxn, o, 0, 0);
        const auto a1 = __builtin_amdgcn_raw_buffer_load_b64(rxn, o + (unsigned)(g.HWi * 2), 0, 0);
        u0[u] = make_uint2(a[0], a[1]);
        u1[u] = make_uint2(a1[0], a1[1]);
        dst[u] = (i * SWc + 4 * q - x0) * P + 2 * cp;
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < kF; ++u) {
        unsigned* d = reinterpret_cast<unsigned*>(L + dst[u]);
        constexpr int PW = P / 2;  // pixel pitch in 32-bit words
        d[0] = (u0[u].x & 0xffffu) | (u1[u].x << 16);
        d[PW] = (u0[u].x >> 16) | (u1[u].x & 0xffff0000u);
        d[2 * PW] = (u0[u].y & 0xffffu) | (u1[u].y << 16);
        d[3 * PW] = (u0[u].y >> 16) | (u1[u].y & 0xffff0000u);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // input rows ho.. (window rows ph..) -> xT[b][ho][px][cw ..]: 16-B runs of 8 channels
    const int nch = min(16 * SPT, g.C - cw);
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) {
      if (ho + rr >= g.H) break;  // block-uniform
      const int ir = g.ph + rr;
      for (int it = lane; it < g.W * (16 * SPT / 8); it += 64) {
        const int ch8 = it % (16 * SPT / 8), px = it / (16 * SPT / 8);
        if (8 * ch8 >= nch) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(L + (ir * SWc + px - x0) * P + 8 * ch8);
        *reinterpret_cast<uint4*>(xT_out + (((size_t)b * g.H + ho + rr) * g.W + px) * g.C + cw +
                                  8 * ch8) = v;
      }
    }
  } else {
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(xT + (size_t)b * g.HWi * g.C), 0, (int)((size_t)g.HWi * g.C * 2),
        0x00020000);
    constexpr int CPP = 2 * SPT;  // 16-B chunks per pixel in the slice
    const int total = KH * SWc * CPP;
    const int x0 = wo0 * g.sw - g.pw;
    constexpr int kU = 4;
    for (int c0 = lane; c0 < total; c0 += 64 * kU) {
      uint4 v[kU];
      int dst[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int ci = c0 + 64 * u;
        const int pix = ci / CPP, part = ci - pix * CPP;
        const int i = pix / SWc, col = pix - i * SWc;
        const int y = ho * g.sh - g.ph + i * g.dh, x = x0 + col;
        const int c = cw + 8 * part;
        const bool ok = ci < total && y >= 0 && y < g.H && x >= 0 && x < g.W && c < g.C;
        const unsigned o = ok ? (unsigned)(((y * g.W + x) * g.C + c) * 2) : 0x80000000u;
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0);
        v[u] = make_uint4(q[0], q[1], q[2], q[3]);
        dst[u] = ci < total ? pix * P + 8 * part : -1;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (dst[u] >= 0) *reinterpret_cast<uint4*>(L + dst[u]) = v[u];
    }
  }
  if constexpr (ROWS > 1) {
    ldb(0, bv[0]);
    ldb(1, bv[1]);
  }
  // the wave reads only its own slice: LDS ops of one wave run in order, so only the
  // compiler must keep the reads below the writes
  __builtin_amdgcn_wave_barrier();
  f32x16 acc[ROWS];
#pragma unroll
  for (int rr = 0; rr < ROWS; ++rr)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[rr][i] = 0.f;
  // lanes past the row's last pixel (Wo < 32) read the last pixel's window (discarded)
  const int rc = min(r, (SWc - 1 - (g.kw - 1) * g.dw) / g.sw);
  auto mma = [&](int t, const bf16x8_t(&rb)[SPT]) {
    const int i = t / g.kw, k = t - i * g.kw;
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) {
      const bf16_t* ap = L + ((i + rr) * SWc + rc * g.sw + k * g.dw) * P + 8 * hh;
      bf16x8_t a[SPT];
#pragma unroll
      for (int u = 0; u < SPT; ++u) a[u] = ld_bf16x8(ap + 16 * u);
#pragma unroll
      for (int u = 0; u < SPT; ++u)
        acc[rr] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], rb[u], acc[rr], 0, 0, 0);
    }
  };
  for (int t = 0; t < KK; t += 3) {
    ldb(t + 2, bv[2]);
    mma(t, bv[0]);
    if (t + 1 >= KK) break;
    ldb(t + 3, bv[0]);
    mma(t + 1, bv[1]);
    if (t + 2 >= KK) break;
    ldb(t + 4, bv[1]);
    mma(t + 2, bv[2]);
  }
  // fold the 4 channel partials in wave order through the (now free) window LDS
  __syncthreads();
  f32x16* red = reinterpret_cast<f32x16*>(smem_row);
  f32x16 sum;
  if constexpr (ROWS == 1) {
    if (w > 0) red[(w - 1) * 64 + lane] = acc[0];
    __syncthreads();
    if (w != 0) return;
    sum = acc[0];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const f32x16 o = red[q * 64 + lane];
#pragma unroll
      for (int i = 0; i < 16; ++i) sum[i] += o[i];
    }
  } else {
    // every wave's partial of row rr at red[rr][w]; wave rr folds its row in wave order
    // (((w0 + w1) + w2) + w3: the ROWS = 1 order, same bits)
#pragma unroll
    for (int rr = 0; rr < ROWS; ++rr) red[(rr * 4 + w) * 64 + lane] = acc[rr];
    __syncthreads();
    if (w >= ROWS || ho + w >= g.Ho) return;
    sum = red[(w * 4) * 64 + lane];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const f32x16 o = red[(w * 4 + q) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 16; ++i) sum[i] += o[i];
    }
  }
  const int rw = ROWS == 1 ? 0 : w;  // the output row this wave writes (ho + rw)
  float(*T)[33] = reinterpret_cast<float(*)[33]>(smem_row + 4 * ROWS * 64 * sizeof(f32x16) +
                                                  (size_t)rw * 32 * 33 * sizeof(float));
  const float bj = r < g.J ? b_off[r] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) T[r][(i & 3) + 8 * (i >> 2) + 4 * hh] = bf2f(f2bf(sum[i] + bj));
  __builtin_amdgcn_wave_barrier();
  if (wo0 + r < g.Wo) {
    const int pp = (ho + rw) * g.Wo + wo0 + r;
    for (int j = hh; j < g.J; j += 2) {
      const float v = T[j][r];
      const size_t o = ((size_t)b * g.J + j) * g.HW + pp;
      off32[o] = v;
      off[o] = f2bf(v);  // exact: v is a bf16 value
    }
  }
}

// LDS bytes of offset_conv_fwd_mfma_bf16_row (0: the row kernel does not apply)
static size_t fwd_bf16_row_lds(const Geo& g, int* SWc, int rows = 1) {
  if (g.Wo < 16) return 0;
  const int spt = (g.C + 63) / 64;
  *SWc = (std::min(32, g.Wo) - 1) * g.sw + (g.kw - 1) * g.dw + 1;
  const size_t win = (size_t)4 * (g.kh + rows - 1) * *SWc * (16 * spt + 8) * 2;
  // the partial fold: 4 waves' 64-B fragments per row, then one 32x33 fp32 tile per row
  const size_t need = std::max(win, (size_t)rows * (4 * 64 * 64 + 32 * 33 * 4));
  return need <= (rows == 1 ? 64 : 128) * 1024 ? need : 0;
}

bool offset_fwd_mfma_bf16_ok(const Geo& g) {
  return g.dt == DCN_BF16 && g.G == 1 && g.J <= 32 && g.C % 16 == 0;
}
size_t offset_fwd_bf16_wb_elems(const Geo& g) {
  const int Cp = (g.C + 63) / 64 * 64;
  return (size_t)g.kh * g.kw * 32 * Cp;
}

// xT: channels-last bf16 x; wb: scratch of offset_fwd_bf16_wb_elems(g) bf16 values.
bool offset_fwd_bf16_fold_ok(const Geo& g) {
  int SWc = 0;
  return offset_fwd_mfma_bf16_ok(g) && fwd_bf16_row_lds(g, &SWc) && g.sh == 1 && g.sw == 1 &&
         g.dh == 1 && g.dw == 1 && g.Ho == g.H && g.Wo == g.W && g.W <= 32 && g.W % 4 == 0 &&
         g.ph >= 0 && g.ph < g.kh && g.pw >= 0 && g.pw < g.kw && g.C % 8 == 0;
}

PrepJob prep_tjc(const Geo& g, const bf16_t* w_off, bf16_t* wb) {
  const int KK = g.kh * g.kw, Cp = (g.C + 63) / 64 * 64;
  return PrepJob{PREP_TJC, (long)KK * 32 * Cp, w_off, wb, 0, g.J, g.C, Cp, KK, 0};
}

hipError_t launch_offset_conv_fwd_bf16(const Geo& g, const bf16_t* xT, const bf16_t* w_off,
                                       const float* b_off, float* off32, bf16_t* off, bf16_t* wb,
                                       hipStream_t s, const bf16_t* x_nchw, bool wb_ready) {
  if (!offset_fwd_mfma_bf16_ok(g)) return hipErrorInvalidValue;
  if (x_nchw && !offset_fwd_bf16_fold_ok(g)) return hipErrorInvalidValue;
  const int KK = g.kh * g.kw, Cp = (g.C + 63) / 64 * 64;
  const int n = KK * 32 * Cp;
  if (!wb_ready)
    hipLaunchKernelGGL(woff_to_tjc_bf16, dim3((n + 255) / 256), dim3(256), 0, s, w_off, wb, g.J,
                       g.C, Cp, KK);
  const int tiles = (g.HW + 31) / 32, spt = Cp / 64;  // 16-channel steps per tap and wave
  int SWc = 0;
  const size_t lds = fwd_bf16_row_lds(g, &SWc);
  if (lds) {
    const int tpr = (g.Wo + 31) / 32;
    dim3 grid(tpr * g.Ho, 1, g.B);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, xT, wb, Cp, b_off, off32, off, tpr, SWc,
                         x_nchw, const_cast<bf16_t*>(xT));
    };
    if (x_nchw) {  // f3: x read once, xT written by the same blocks
      int SW2 = 0;
      const size_t lds2 = OFFC_ROWS > 1 ? fwd_bf16_row_lds(g, &SW2, OFFC_ROWS) : 0;
      if (lds2) {  // OFFC_ROWS output rows per block (tpr == 1 on the fold path)
        const dim3 grid2((g.Ho + OFFC_ROWS - 1) / OFFC_ROWS, 1, g.B);
        auto go2 = [&](auto kern) -> hipError_t {
          if (lds2 > 64 * 1024) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)lds2);
            if (e != hipSuccess) return e;
          }
          hipLaunchKernelGGL(kern, grid2, dim3(256), lds2, s, g, xT, wb, Cp, b_off, off32, off,
                             tpr, SW2, x_nchw, const_cast<bf16_t*>(xT));
          return hipGetLastError();
        };
        constexpr int R = OFFC_ROWS > 1 ? OFFC_ROWS : 2;
        if (spt == 1) return go2(offset_conv_fwd_mfma_bf16_row<1, true, R>);
        if (spt == 2) return go2(offset_conv_fwd_mfma_bf16_row<2, true, R>);
        if (spt == 3) return go2(offset_conv_fwd_mfma_bf16_row<3, true, R>);
        return go2(offset_conv_fwd_mfma_bf16_row<4, true, R>);
      }
      if (spt == 1) go(offset_conv_fwd_mfma_bf16_row<1, true>);
      else if (spt == 2) go(offset_conv_fwd_mfma_bf16_row<2, true>);
      else if (spt == 3) go(offset_conv_fwd_mfma_bf16_row<3, true>);
      else go(offset_conv_fwd_mfma_bf16_row<4, true>);
      return hipGetLastError();
    }
    if (spt == 1) go(offset_conv_fwd_mfma_bf16_row<1>);
    else if (spt == 2) go(offset_conv_fwd_mfma_bf16_row<2>);
    else if (spt == 3) go(offset_conv_fwd_mfma_bf16_row<3>);
    else go(offset_conv_fwd_mfma_bf16_row<4>);
    return hipGetLastError();
  }
  dim3 grid(tiles, 1, g.B);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, g, xT, wb, Cp, b_off, off32, off, tiles);
  };
  if (spt == 1) go(offset_conv_fwd_mfma_bf16<1>);
  else if (spt == 2) go(offset_conv_fwd_mfma_bf16<2>);
  else if (spt == 3) go(offset_conv_fwd_mfma_bf16<3>);
  else go(offset_conv_fwd_mfma_bf16<4>);  // C <= 256 on the bf16 path
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K7 on the bf16 matrix cores (DCN_BF16, stride 1). x and w_off are bf16 values; the fp32
// ∂offset is split exactly-enough into hi = bf16(g) and lo = bf16(g - hi) (|g - hi - lo|
// <= 2^-16 |g|), each product is exact in fp32 and the sums are fp32, so the results
// match the fp32 kernels' to about fp32 rounding before their final bf16 rounding.
// K index k = tap·J8 + j (offset channels padded to J8 = a multiple of 8), so a lane's 8
// consecutive k are 8 consecutive offset channels of one tap: one 32-B run of the staged
// ∂offset rows S[(sr·SW + sc)·PJ + j] (stage_goff8: the f32 kernels' staging with a PJ
// stride and zero padding channels).
//   ∂x_b[c][q]      = Σ_k Wc[c][k] · G[q][k]     M = c, N = q (pixels), K = (tap, j)
//   ∂w_off[j][c][t] = Σ_q x[c][q]  · G[q][k]     M = c, N = k,          K = q
// with G[q][t·J8 + j] = ∂off[j][q - shift_t] = S[base(q) + toff8(t) + j].
// ---------------------------------------------------------------------------
__host__ __device__ static inline int j8(int J) { return (J + 7) / 8 * 8; }
// LDS pixel pitch of the staged ∂offset rows: J8 + 4 floats (an odd number of 16-B bank
// groups), so lanes 8 pixels apart (∂x: 16-B reads) or 8 pixels apart across the two lane
// halves (∂W_off) fall on different banks; J8 itself put them on the same bank
__host__ __device__ static inline int pj8(int J) { return j8(J) + 4; }
__host__ __device__ static inline int kt16(const Geo& g) {
  return (g.kh * g.kw * j8(g.J) + 15) / 16 * 16;
}

// Wc[c][k = t·J8 + j] = w_off[j][c][t] (bf16, 0 for padding), stored in MFMA A-fragment
// order so that a wave's A load is one contiguous 1 KiB: element e of lane l of k-step ks
// of 32-channel M-tile mt is Wc[32mt + (l&31)][16ks + 8(l>>5) + e], at
// wc[((mt·NKS + ks)·64 + l)·8 + e], NKS = KT16/16.
__global__ __launch_bounds__(256) void woff_to_ck_bf16(const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ wc, int J, int J8,
                                                      int C, int KK, int KT16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < C * KT16) swz_ck(w, wc, J, J8, C, KK, KT16, i);
}

template <int kU = 8>
__device__ __forceinline__ void stage_goff8(const Geo& g, const float* __restrict__ goff, int b,
                                            int y0, int SR, int SW, int J8, int PJ, float* S) {
  const int plane = SR * SW, n = plane * J8;
  const unsigned mp = 0xffffffffu / (unsigned)plane + 1u, ms = 0xffffffffu / (unsigned)SW + 1u;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(goff + (size_t)b * g.J * g.HW),
                                                    0, (int)((size_t)g.J * g.HW * 4), 0x00020000);
  for (int i0 = threadIdx.x; i0 < n; i0 += blockDim.x * kU) {
    float v[kU];
    int dst[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // sc fastest: coalesced reads (stage_goff's buffer loads)
      const int idx = min(i0 + u * (int)blockDim.x, n - 1);
      const int j = (int)__umulhi((unsigned)idx, mp), rem = idx - j * plane;
      const int sr = (int)__umulhi((unsigned)rem, ms), sc = rem - sr * SW;
      const int ho = y0 + sr - (g.kh - 1) * g.dh + g.ph, wo = sc - (g.kw - 1) * g.dw + g.pw;
#if STAGE_NOSC
      // bitwise, not short-circuit: && made hipcc wrap every element's load in its own
      // exec-masked branch (~29 instructions per element, r05)
      const bool ok = (j < g.J) & ((unsigned)ho < (unsigned)g.Ho) & ((unsigned)wo < (unsigned)g.Wo);
#else
      const bool ok = j < g.J && ho >= 0 && ho < g.Ho && wo >= 0 && wo < g.Wo;
#endif
      const unsigned o = ok ? (unsigned)((j * g.HW + ho * g.Wo + wo) * 4) : 0x80000000u;
      v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
      dst[u] = rem * PJ + j;
    }
    // unconditional: a slot past n holds element n-1 (clamped idx) and rewrites it with its
    // own value, so no exec-masked store blocks (each makes the waitcnt pass drain, vmcnt(0));
    // the barrier keeps all kU loads issued before the first store
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kU; ++u) S[dst[u]] = v[u];
  }
}

// stage_goff8 with each value written pre-split: Sb[(sr·SW + sc)·PB + j] = hi = bf16(v) and
// Sb[... + J8 + j] = lo = bf16(v - hi) (PB = 2·PJ bf16: the fp32 layout's bytes, so the same
// pixel stride and 16-B alignment), split8's bits exactly; r05: the ∂x kernel read fp32 and
// split in its k loop, once per wave and tap reuse (≈ 70 of its 125 VALU per step: the loop
// was VALU-bound at twice its MFMA time)
template <int kU = 8>
__device__ __forceinline__ void stage_goff8_split(const Geo& g, const float* __restrict__ goff,
                                                  int b, int y0, int SR, int SW, int J8, int PB,
                                                  bf16_t* Sb) {
  const int plane = SR * SW, n = plane * J8;
  const unsigned mp = 0xffffffffu / (unsigned)plane + 1u, ms = 0xffffffffu / (unsigned)SW + 1u;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(goff + (size_t)b * g.J * g.HW),
                                                    0, (int)((size_t)g.J * g.HW * 4), 0x00020000);
  for (int i0 = threadIdx.x; i0 < n; i0 += blockDim.x * kU) {
    float v[kU];
    int dst[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int idx = min(i0 + u * (int)blockDim.x, n - 1);
      const int j = (int)__umulhi((unsigned)idx, mp), rem = idx - j * plane;
      const int sr = (int)__umulhi((unsigned)rem, ms), sc = rem - sr * SW;
      const int ho = y0 + sr - (g.kh - 1) * g.dh + g.ph, wo = sc - (g.kw - 1) * g.dw + g.pw;
#if STAGE_NOSC
      // bitwise, not short-circuit: && made hipcc wrap every element's load in its own
      // exec-masked branch (~29 instructions per element, r05)
      const bool ok = (j < g.J) & ((unsigned)ho < (unsigned)g.Ho) & ((unsigned)wo < (unsigned)g.Wo);
#else
      const bool ok = j < g.J && ho >= 0 && ho < g.Ho && wo >= 0 && wo < g.Wo;
#endif
      const unsigned o = ok ? (unsigned)((j * g.HW + ho * g.Wo + wo) * 4) : 0x80000000u;
      v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
      dst[u] = rem * PB + j;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const __bf16 h = (__bf16)v[u];
      Sb[dst[u]] = __builtin_bit_cast(bf16_t, h);
      Sb[dst[u] + J8] = __builtin_bit_cast(bf16_t, (__bf16)(v[u] - (float)h));
    }
  }
}

__device__ __forceinline__ int toff8(const Geo& g, int t, int SW, int PJ) {
  const int i = t / g.kw, k = t - i * g.kw;
  return ((g.kh - 1 - i) * g.dh * SW + (g.kw - 1 - k) * g.dw) * PJ;
}

// 8 fp32 -> (hi, lo) bf16 fragments
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8_t& hi, bf16x8_t& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    hi[e] = h;
    lo[e] = (__bf16)(v[e] - (float)h);
  }
}

// ∂x: block = 64 input pixels of one image (2 N-tiles) x all channels; wave w = channels
// 64w..64w+63 (2 M-tiles); D[c][q] + the sampling route's channels-last ∂x, written as
// bf16 NCHW (the API's grad_x). r04: the epilogue reads and writes through buffer resources
// (32-bit offsets), which cut 160 VGPRs + 64 AGPRs to 121 registers: 4 workgroups per CU
// instead of 2, so config 4's 832 workgroups run in one round.
__global__ __launch_bounds__(256, 3) void offset_dgrad_bf16(Geo g, const bf16_t* __restrict__ wc,
                                                        int KT16, const float* __restrict__ goff,
                                                        const float* __restrict__ gxT_in,
                                                        bf16_t* __restrict__ gx, int spi) {
  extern __shared__ float S[];
  const int J8 = j8(g.J), KK = g.kh * g.kw, KT = KK * J8;
  const int bid = blockIdx.x;
  const int b = bid / spi, p0 = (bid - b * spi) * kDgPx;
  const int np = min(kDgPx, g.HWi - p0);
  const int y0 = p0 / g.W, y1 = (p0 + np - 1) / g.W;
  const int SW = g.W + (g.kw - 1) * g.dw;
  const int PJ = pj8(g.J);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int cw = 64 * w;
  // A = Wc fragments (L2-resident), kPf k-steps ahead in a register ring; the first ones
  // are issued before the ∂offset staging so that their latency hides behind it
  const int NKS = KT16 / 16;
  const int wt = cw < g.C ? w : 0;  // idle waves (C < 256) load wave 0's (in range)
  const bf16_t* wr0 = wc + ((size_t)(2 * wt) * NKS * 64 + lane) * 8;  // M-tiles 2w, 2w+1
  const bf16_t* wr1 = wr0 + (size_t)NKS * 512;
  constexpr int kPf = OFFD_PF;
  bf16x8_t ra0[kPf], ra1[kPf];
  auto lda = [&](int ks, int d) {
    const int kc = min(ks, NKS - 1);
    ra0[d] = ld_bf16x8(wr0 + 512 * kc);
    ra1[d] = ld_bf16x8(wr1 + 512 * kc);
  };
#pragma unroll
  for (int d = 0; d < kPf - 1; ++d) lda(d, d);
  // pre-split hi/lo records (PB = 2·PJ bf16 per pixel) and, past the staged rows, the k-step
  // table: tab[2·ks + hh] = the bf16 offset of step ks's 8 k of half hh (toff8 + j0), or -1
  // for the K padding (zero operands)
  const int PB = 2 * PJ;
  bf16_t* Sb = reinterpret_cast<bf16_t*>(S);
  int* tab = reinterpret_cast<int*>(S + (size_t)((kDgPx - 1) / g.W + 2 + (g.kh - 1) * g.dh) * SW * PJ);
  stage_goff8_split(g, goff, b, y0, y1 - y0 + 1 + (g.kh - 1) * g.dh, SW, J8, PB, Sb);
  if (threadIdx.x < 2 * NKS) {
    const int k = 8 * (int)threadIdx.x;
    const int t = k / J8, j0 = k - t * J8;
    tab[threadIdx.x] = k < KT ? toff8(g, t, SW, PB) + j0 : -1;
  }
  __syncthreads();
  const bool live = cw < g.C;  // (C < 256: idle waves still meet the epilogue barrier)
  int base[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = p0 + min(32 * u + r, np - 1);
    const int y = p / g.W, x = p - y * g.W;
    base[u] = ((y - y0) * SW + x) * PB;
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][u][i] = 0.f;
  for (int ks0 = 0; ks0 < (live ? NKS : 0); ks0 += kPf) {
#pragma unroll
    for (int d = 0; d < kPf; ++d) {
      const int ks = ks0 + d;
      lda(ks + kPf - 1, (d + kPf - 1) % kPf);
      __builtin_amdgcn_sched_barrier(0);
      if (ks < NKS) {  // wave-uniform
        const int e = tab[2 * ks + hh];
        bf16x8_t bh[2], bl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16_t* sp = Sb + base[u] + max(e, 0);
          bh[u] = *reinterpret_cast<const bf16x8_t*>(sp);
          bl[u] = *reinterpret_cast<const bf16x8_t*>(sp + J8);
        }
        if (16 * ks + 16 > KT) {  // wave-uniform: only the last step can hold K padding
          const unsigned keep = e >= 0 ? 0xffffffffu : 0u;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            uint4 h = __builtin_bit_cast(uint4, bh[u]), l = __builtin_bit_cast(uint4, bl[u]);
            h.x &= keep, h.y &= keep, h.z &= keep, h.w &= keep;
            l.x &= keep, l.y &= keep, l.z &= keep, l.w &= keep;
            bh[u] = __builtin_bit_cast(bf16x8_t, h);
            bl[u] = __builtin_bit_cast(bf16x8_t, l);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra0[d], bh[u], acc[0][u], 0, 0, 0);
          acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra1[d], bh[u], acc[1][u], 0, 0, 0);
          acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra0[d], bl[u], acc[0][u], 0, 0, 0);
          acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra1[d], bl[u], acc[1][u], 0, 0, 0);
        }
      }
    }
  }
  // ∂x = the sampling route (channels-last gxT_in) + D, as bf16 NCHW. gxT_in is read as
  // whole 256-B pixel rows (this wave's 64 channels) into LDS and read back per D lane
  // (pixel r, channel of register i); the bf16 stores are 64-B pixel runs per channel.
  __syncthreads();  // every wave is done with S: its space holds the transposes
  if (!live) return;
  float* T = S + w * 32 * kDgTP;
  const auto rgx = __builtin_amdgcn_make_buffer_rsrc(gx + (size_t)b * g.C * g.HWi, 0,
                                                     (int)((size_t)g.C * g.HWi * 2), 0x00020000);
  const auto rgt = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(gxT_in + (size_t)b * g.HWi * g.C), 0, (int)((size_t)g.HWi * g.C * 4),
      0x00020000);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      float4 tv[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int pl = min(32 * u + 4 * (4 * h2 + it) + (lane >> 4), np - 1);
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(
            rgt, (unsigned)(((p0 + pl) * g.C + cw + 4 * (lane & 15)) * 4), 0, 0);
        tv[it] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                             __uint_as_float(q[3]));
      }
#pragma unroll
      for (int it = 0; it < 4; ++it)
        *reinterpret_cast<float4*>(T + (4 * (4 * h2 + it) + (lane >> 4)) * kDgTP + 4 * (lane & 15)) = tv[it];
    }
    __builtin_amdgcn_wave_barrier();
    {
      // 32-bit offsets into this image's planes through a buffer resource (64-bit addresses per
      // store held 2 VGPRs each and capped the kernel at 2 waves per SIMD); a pixel past np
      // stores out of range (dropped)
      const int pl = 32 * u + r;
      const unsigned pb = pl < np ? (unsigned)(p0 + pl) * 2u : 0x80000000u;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int cl = 32 * m + (i & 3) + 8 * (i >> 2) + 4 * hh;
          const unsigned o = pl < np ? (unsigned)(cw + cl) * (unsigned)g.HWi * 2u + pb : pb;
          __builtin_amdgcn_raw_buffer_store_b16(
              (unsigned short)f2bf(T[r * kDgTP + cl] + acc[m][u][i]), rgx, o, 0, 0);
        }
    }
    __builtin_amdgcn_wave_barrier();  // the next half overwrites T
  }
}

// ∂w_off partials: block = (chunk of rowsB input rows of one image, 64 channels); wave w
// owns N-tiles w and w+4 of the KT16/32 (t, j) tiles x both 32-channel M-tiles.
// part[chunk][c][j·KK + t] (the f32 kernel's format: wgrad_mfma_reduce folds it).
// CGB (r05): 64-channel groups per workgroup (4 waves each) sharing one staging of the
// ∂offset rows (the staging was instruction-bound, a third of the workgroup's time)
template <int CGB = 1>
__global__ __launch_bounds__(256 * CGB) void offset_wgrad_bf16(Geo g, const bf16_t* __restrict__ x,
                                                        const float* __restrict__ goff,
                                                        float* __restrict__ part, int rowsB,
                                                        int cpi, int cpb) {
  extern __shared__ float S[];
  const int J8 = j8(g.J), KK = g.kh * g.kw, KT = KK * J8;
  const int SW = g.W + (g.kw - 1) * g.dw;
  const int PJ = pj8(g.J);
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) & 3, cgl = threadIdx.x >> 8;
  const int r = lane & 31, hh = lane >> 5;
  const int cgi = blockIdx.y * CGB + cgl;  // this wave's 64-channel group
  const int cb = cgi * 64;
  const int nchunk = g.B * cpi;
  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][u][i] = 0.f;
  // this lane's N column in each owned tile: k = 32·tile + r = t·J8 + j. A wave's second
  // tile may not exist (w + 4 >= NTt): its MFMAs then multiply zeros, which costs that wave
  // nothing the other waves do not spend anyway and keeps the loop free of branches.
  int kofs[2];
  unsigned kmask[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int kk = 32 * (w + 4 * u) + r;
    const bool kok = kk < KT;
    const int t = kk / J8, j = kk - t * J8;
    kofs[u] = kok ? toff8(g, t, SW, PJ) + j : 0;
    kmask[u] = kok ? 0xffffffffu : 0u;
  }
  // the block sums cpb consecutive chunks (of any images) into one partial: fewer partial
  // bytes to write and fold
  for (int ci = 0; ci < cpb; ++ci) {
  const int chunk = blockIdx.x * cpb + ci;
  if (chunk >= nchunk) break;  // workgroup-uniform
  const int b = chunk / cpi, y0 = (chunk - b * cpi) * rowsB;
  const int nrows = min(rowsB, g.H - y0);
  const int npx = nrows * g.W;  // a multiple of 4 (W % 4 == 0)
  // A = this block's 64 channel planes of x through a buffer resource, kPf steps ahead in a
  // register ring. A step past the chunk loads nothing (offset out of range: zeros); the
  // ragged last step's upper 4 pixels read x beyond the chunk (or zeros past the planes),
  // which meet zero B rows.
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x + ((size_t)b * g.C + cb) * g.HWi), 0, (int)(64 * (size_t)g.HWi * 2),
      0x00020000);
  const unsigned xl0 = (unsigned)((r * g.HWi + y0 * g.W + 8 * hh) * 2);
  const unsigned xl1 = xl0 + (unsigned)(32 * g.HWi * 2);
  const int nsteps = (npx + 15) / 16;
  constexpr int kPf = OFFW_PF;
  bf16x8_t ra0[kPf], ra1[kPf];
  auto lda = [&](int i, int d) {
    const bool in = i < nsteps && 16 * i + 8 * hh < npx;
    const unsigned o = (unsigned)(32 * i);
    ra0[d] = __builtin_bit_cast(bf16x8_t,
                                __builtin_amdgcn_raw_buffer_load_b128(rx, in ? xl0 + o : 0x80000000u, 0, 0));
    ra1[d] = __builtin_bit_cast(bf16x8_t,
                                __builtin_amdgcn_raw_buffer_load_b128(rx, in ? xl1 + o : 0x80000000u, 0, 0));
  };
#pragma unroll
  for (int d = 0; d < kPf - 1; ++d) lda(d, d);
  if (ci > 0) __syncthreads();  // the previous chunk's staged rows are no longer read
  stage_goff8<OFFW_SG>(g, goff, b, y0, nrows + (g.kh - 1) * g.dh, SW, J8, PJ, S);
  __syncthreads();
  // (row, column) in the chunk of this lane's first pixel q = 16i + 8hh: q and W are
  // multiples of 4, so pixels q..q+3 share a row, as do q+4..q+7
  int yq = (8 * hh) / g.W, xq = 8 * hh - yq * g.W;
  for (int i0 = 0; i0 < nsteps; i0 += kPf) {
#pragma unroll
    for (int d = 0; d < kPf; ++d) {
      const int i = i0 + d;
      lda(i + kPf - 1, (d + kPf - 1) % kPf);
#if OFFW_SB
      __builtin_amdgcn_sched_barrier(0);
#endif
      if (i < nsteps) {  // wave-uniform
        const int q = 16 * i + 8 * hh;
        // pixels past the chunk read a staged row in range (S[0..]) and are masked to zero
        const bool ok0 = q < npx, ok1 = q + 4 < npx;
        const int s0 = ok0 ? (yq * SW + xq) * PJ : 0;
        const int s1 = !ok1 ? 0 : xq + 4 < g.W ? s0 + 4 * PJ : (yq + 1) * SW * PJ;
        const unsigned m0 = ok0 ? 0xffffffffu : 0u, m1 = ok1 ? 0xffffffffu : 0u;
        bf16x8_t bh[2], bl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = __uint_as_float(__float_as_uint(S[s0 + e * PJ + kofs[u]]) & (m0 & kmask[u]));
            v[4 + e] =
                __uint_as_float(__float_as_uint(S[s1 + e * PJ + kofs[u]]) & (m1 & kmask[u]));
          }
          split8(v, bh[u], bl[u]);
        }
        xq += 16;
        while (xq >= g.W) xq -= g.W, ++yq;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra0[d], bh[u], acc[0][u], 0, 0, 0);
          acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra1[d], bh[u], acc[1][u], 0, 0, 0);
          acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra0[d], bl[u], acc[0][u], 0, 0, 0);
          acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra1[d], bl[u], acc[1][u], 0, 0, 0);
        }
      }
    }
  }
  }  // chunks
  // partials in MFMA fragment order (each lane's 16 accumulators are 64 contiguous bytes,
  // a wave's tile one 4 KiB run): part[(((chunk·CG + cg)·NT + tile)·2 + m)·64 + lane][16]
  // with NT = ceil(KT/32) tiles; wgrad_frag_reduce folds the chunks and scatters to ∂w_off
  const int NT = (KT + 31) / 32, CG = g.C / 64;
  // (columns j >= J inside a tap are written as zeros; only k >= KT is skipped)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tile = w + 4 * u;
    if (tile >= NT) continue;  // wave-uniform
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float* pp = part + (((((size_t)blockIdx.x * CG + cgi) * NT + tile) * 2 + m) * 64 + lane) * 16;
      if (!kmask[u]) continue;  // a padding K column: the fold never reads it
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(pp + 4 * q) =
            make_float4(acc[m][u][4 * q], acc[m][u][4 * q + 1], acc[m][u][4 * q + 2],
                        acc[m][u][4 * q + 3]);
    }
  }
}

// ∂w_off[j][c][t] = Σ_chunk (fragment-ordered partials of offset_wgrad_bf16), chunks in
// order: 256 fragment elements per 1024-thread block (a lane's 4 consecutive elements as one
// float4: 1 KiB per wave load), wave w sums chunks ≡ w (mod 16), the 16 wave sums fold in
// order (deterministic; per element the same additions in the same order as r05's
// one-element-per-lane form, which read 256 B per wave load and took 23 µs at config 4);
// each element then lands at its (j, c, t).
__global__ __launch_bounds__(1024) void wgrad_frag_reduce(Geo g, const float* __restrict__ part,
                                                         int nchunk, float* __restrict__ gw) {
  const int J8 = j8(g.J), KK = g.kh * g.kw, NT = (KK * J8 + 31) / 32;
  const long E = (long)(g.C / 64) * NT * 2 * 1024;  // a multiple of 2048
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long i0 = (long)blockIdx.x * 256 + 4 * lane;
  const long ic = i0 < E ? i0 : 0;
  // the 4 elements share their K column (the same 16-element register group): padding K
  // columns (k >= KK·J8) were never written, so they are not read either
  const int kcol = 32 * (int)(((ic >> 10) >> 1) % NT) + (int)((ic >> 4) & 31);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (kcol < KK * J8) {
#pragma unroll 8
    for (int ch = w; ch < nchunk; ch += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)ch * E + ic);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  __shared__ float4 red[16][64];
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || i0 >= E) return;
  s = red[0][lane];
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    const float4 v = red[k][lane];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long i = i0 + e;
    const int reg = (int)(i & 15), fl = (int)((i >> 4) & 63);
    const long tm = i >> 10;  // ((cg·NT + tile)·2 + m)
    const int m = (int)(tm & 1), tile = (int)((tm >> 1) % NT), cg = (int)((tm >> 1) / NT);
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (fl >> 5);
    const int c = 64 * cg + 32 * m + row, k = 32 * tile + (fl & 31);
    const int t = k / J8, j = k - t * J8;
    if (t < KK && j < g.J) gw[((size_t)j * g.C + c) * KK + t] = sv[e];
  }
}
static size_t wgrad_frag_part_floats(const Geo& g, const MfmaStage& ms) {
  const int NT = (g.kh * g.kw * j8(g.J) + 31) / 32;
  return (size_t)g.B * ms.cpi * (g.C / 64) * NT * 2 * 1024;
}

// Which bf16 offset backwards the MFMA kernels take (else the fp32 ones on fp32 copies)
static void bwd_bf16_lds(const Geo& g, const MfmaStage& ms, size_t* lds_w, size_t* lds_x) {
  const size_t row = (size_t)ms.SW * pj8(g.J) * sizeof(float);
  *lds_w = (size_t)(ms.rowsB + (g.kh - 1) * g.dh) * row;
  // (+ offset_dgrad_bf16's k-step table past the staged rows: 2 ints per step, <= 16 steps)
  *lds_x = std::max((size_t)ms.SRx * row + 32 * sizeof(int), (size_t)4 * 32 * kDgTP * sizeof(float));
}
bool offset_bwd_bf16_ok(const Geo& g) {
  MfmaStage ms;
  // (H·W % 8 and W % 4: a chunk's pixel runs start 8-byte aligned in every channel plane)
  // offset_dgrad_bf16 addresses one image's x (bf16) and channels-last ∂x (fp32) planes
  // through buffer resources with 32-bit byte offsets (a tall plane wrapped them)
  if (!(g.dt == DCN_BF16 && mfma_stage(g, &ms) && g.C % 64 == 0 && g.HWi % 8 == 0 &&
        g.W % 4 == 0 && g.kh * g.kw * j8(g.J) <= 256 && !get_force_generic() &&
        (size_t)g.HWi * g.C * 4 < ((size_t)1 << 31)))
    return false;
  size_t lw, lx;
  bwd_bf16_lds(g, ms, &lw, &lx);
  return lw <= (size_t)kMfmaLds && lx <= (size_t)kMfmaLds;
}
size_t offset_bwd_bf16_wc_elems(const Geo& g) { return (size_t)g.C * kt16(g); }

// DCN_BF16 offset-conv backward: x bf16 NCHW, w_off bf16, goff fp32; writes gw_off /
// gb_off (fp32) and gx (bf16 NCHW) = transpose(gxT_in) + the offset-conv route.
// part: the goffT scratch (offset_conv_goffT_floats); wc: offset_bwd_bf16_wc_elems.
PrepJob prep_ck(const Geo& g, const bf16_t* w_off, bf16_t* wc) {
  return PrepJob{PREP_CK, (long)g.C * kt16(g), w_off, wc, 0, g.J, j8(g.J), g.C, g.kh * g.kw,
                 kt16(g)};
}

hipError_t launch_offset_conv_bwd_bf16(const Geo& g, const bf16_t* x, const bf16_t* w_off,
                                       const float* goff, const float* gxT_in, bf16_t* wc,
                                       float* part, bf16_t* gx, float* gw_off, float* gb_off,
                                       hipStream_t s, hipStream_t aux, hipEvent_t fork,
                                       hipEvent_t join, bool wc_ready, float* bsum_part) {
  MfmaStage ms;
  if (!offset_bwd_bf16_ok(g) || !mfma_stage(g, &ms)) return hipErrorInvalidValue;
  const int KK = g.kh * g.kw, J8 = j8(g.J), KT16 = kt16(g);
  // side stream (when given): the Wc swizzle for ∂x and the ∂b_off channel sums, beside ∂W_off
  hipStream_t s2 = aux ? aux : s;
  hipError_t e = hipSuccess;
  if (aux) {
    e = hipEventRecord(fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    if (e != hipSuccess) return e;
  }
  const int n = g.C * KT16;
  if (!wc_ready)
    hipLaunchKernelGGL(woff_to_ck_bf16, dim3((n + 255) / 256), dim3(256), 0, s2, w_off, wc, g.J,
                       J8, g.C, KK, KT16);
  // ∂b_off: one block per channel (r02, config 4: the two-level (channel, image) sum that the
  // fp32 path runs on its side stream measured 0.122 against 0.112 ms for this scope here)
  // bsum_part (B·J floats): ∂b_off as the two-level (channel, image) sum on the main stream
  // after ∂W_off's fold instead (A/B knob of the caller)
  if (gb_off && !bsum_part) launch_channel_sum(goff, g.B, g.J, g.HW, gb_off, s2);
  size_t lds_w, lds_x;
  bwd_bf16_lds(g, ms, &lds_w, &lds_x);
  // chunks per workgroup (config 4: 1 -> 48 + 11 us, 2 -> 42 + 7, 4 -> 53 + 6 for ∂W_off + fold)
  const int cpb = OFFW_CPB;
  const int nblk = (g.B * ms.cpi + cpb - 1) / cpb;
  if (OFFW_CGB == 2 && (g.C / 64) % 2 == 0)
    hipLaunchKernelGGL(offset_wgrad_bf16<2>, dim3(nblk, g.C / 128), dim3(512), lds_w, s, g, x, goff,
                       part, ms.rowsB, ms.cpi, cpb);
  else
  hipLaunchKernelGGL(offset_wgrad_bf16<1>, dim3(nblk, g.C / 64), dim3(256), lds_w, s, g, x, goff,
                     part, ms.rowsB, ms.cpi, cpb);
  const long E = (long)(g.C / 64) * ((KK * J8 + 31) / 32) * 2 * 1024;
  hipLaunchKernelGGL(wgrad_frag_reduce, dim3((unsigned)((E + 255) / 256)), dim3(1024), 0, s, g,
                     part, nblk, gw_off);
  if (gb_off && bsum_part) launch_channel_sum_2l(goff, g.B, g.J, g.HW, bsum_part, gb_off, s);
#if OFFB_CONC
  // (A/B) ∂x on the side stream, concurrent with ∂W_off + its fold on the main one
  if (aux)
    hipLaunchKernelGGL(offset_dgrad_bf16, dim3(g.B * ms.spi), dim3(256), lds_x, aux, g, wc, KT16,
                       goff, gxT_in, gx, ms.spi);
#endif
  if (aux) {
    e = hipEventRecord(join, aux);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
    if (e != hipSuccess) return e;
  }
#if OFFB_CONC
  if (!aux)
#endif
  hipLaunchKernelGGL(offset_dgrad_bf16, dim3(g.B * ms.spi), dim3(256), lds_x, s, g, wc, KT16, goff,
                     gxT_in, gx, ms.spi);
  return hipGetLastError();
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

// ---------------------------------------------------------------------------
// K3 on the f32 matrix cores, fused with the x -> xT transpose (fp32, 3x3, stride 1, pad 1,
// Ho == H, Wo == W <= 62, W % 4 == 0, C % 16 == 0, J <= 18).
//   off[b][j][ho][p] = b_off[j] + Σ_{c, tap} w_off[j][c][tap] · x[b][c][ho-1+ty][p-1+tx]
// One workgroup = ROWS output rows of one image; wave w computes 16 pixels (p = 4m + (w&3),
// m = 0..15) of row w>>2 over ALL channels, walking them in 16-channel chunks that the
// workgroup stages together, double-buffered: the ROWS+2 input rows of the chunk (loaded
// from NCHW x with coalesced 16-B row loads, written channels-last into LDS at a pitch of
// 20 floats per pixel, so one 16-B LDS read gives a lane 4 consecutive channels) and the
// chunk's weights in MFMA fragment order. The next chunk's loads are in flight while the
// current chunk computes; one LDS-only barrier per chunk.
// v_mfma_f32_16x16x4_f32: A row m = pixel 4m + (w&3), A column k = lane group g (channel
// 4g + s at step s), B = weights, D = 16 pixels x offset channels 0-15. Offset channels
// 16-17 run on the VALU from the same A values (lane-group partials summed at the end in a
// fixed order). The window rows 1..ROWS are the input rows ho0.. (Ho == H): the workgroup
// writes them to xT, so no separate transpose pass reads x again. Every sum has a fixed
// order: deterministic.
// ---------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kXtCP = 20, kXtRWmax = 64, kXtWts = 9 * 64 * 4 + 9 * 4 * 8;  // floats

// per 16-channel chunk cg, kXtWts floats: B[t][lane][s] = w_off[j = lane&15][c][t] with
// c = 16cg + 4(lane>>4) + s, then V[t][g][2s + jj] = w_off[16 + jj][16cg + 4g + s][t]
// (0 for j >= J)
__global__ __launch_bounds__(256) void woff_to_f32frag(const float* __restrict__ w,
                                                       float* __restrict__ wf, int J, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C / 16 * kXtWts) return;
  const int cg = i / kXtWts, k = i - cg * kXtWts;
  int j, c, t;
  if (k < 9 * 256) {
    const int s = k & 3, lane = (k >> 2) & 63;
    t = k >> 8;
    j = lane & 15;
    c = 16 * cg + 4 * (lane >> 4) + s;
  } else {
    const int v = k - 9 * 256, jj = v & 1, s = (v >> 1) & 3, gg = (v >> 3) & 3;
    t = v >> 5;
    j = 16 + jj;
    c = 16 * cg + 4 * gg + s;
  }
  wf[i] = j < J ? w[((size_t)j * C + c) * 9 + t] : 0.f;
}

template <int ROWS>  // output rows per workgroup; 4 * ROWS waves
__global__ __launch_bounds__(ROWS * 256) __attribute__((amdgpu_waves_per_eu(2))) void
offset_conv_fwd_mfma_xt(Geo g, const float* __restrict__ x, const float* __restrict__ wf,
                        const float* __restrict__ b_off, float* __restrict__ off,
                        float* __restrict__ xT) {
  constexpr int NT = ROWS * 256, NR = ROWS + 2, CP = kXtCP;
  constexpr int RW = kXtRWmax;              // window row pitch (pixels): compile-time offsets
  constexpr int WIN = NR * RW * CP;         // floats per window buffer
  constexpr int BUF = WIN + kXtWts;
  constexpr int kSx = (16 * NR * 16 + NT - 1) / NT, kSw = (kXtWts / 4 + NT - 1) / NT;
  // 2 buffers, then a trash slot per lane: staging slots with nothing to stage write there,
  // so the LDS stores need no exec-masked branch (a masked block makes the waitcnt pass
  // assume its waits may not have run and drain the chunks in flight, vmcnt(0), every step)
  constexpr int TRASH = 2 * BUF;
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF + 256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Block3 blk = xcd_block();
  const int ho0 = blk.x * ROWS, b = blk.z;
  const int H = g.H, W = g.W, C = g.C, NQ = W / 4;
  const int m = lane & 15, gq = lane >> 4;
  const int nch = C / 16;
  // zero padding columns 0 and W+1 of both buffers (never overwritten)
  for (int i = tid; i < 2 * NR * 2 * 16; i += NT) {
    const int cc = i & 15, z = (i >> 4) & 1, row = (i >> 5) % NR, bf = i / (32 * NR);
    lds[bf * BUF + (row * RW + (z ? W + 1 : 0)) * CP + cc] = 0.f;
  }
  float4 sx0[kSx], sw0[kSw], sx1[kSx], sw1[kSw];  // chunks k+1 and k+2 in flight
  // per-lane staging addresses, the same for every chunk. Lane = (channel fastest, then 4
  // pixels): the global loads read 64-B runs of 16 channel rows, and the channels-last LDS
  // writes of one instruction fall in 64 different banks
  int gx[kSx], lx[kSx];
#pragma unroll
  for (int u = 0; u < kSx; ++u) {
    const int idx = tid + NT * u, cc = idx & 15, rest = idx >> 4;
    const int q = rest % NQ, row = rest / NQ;
    const int y = ho0 - 1 + row;
    const bool in = row < NR;
    gx[u] = in && y >= 0 && y < H ? (cc * H + y) * W + 4 * q : -1;
    lx[u] = in ? (row * RW + 1 + 4 * q) * CP + cc : TRASH - BUF + lane;  // (relative to L)
  }
  // branch-free loads (buffer range checks give the zeros), so no conditional load makes the
  // compiler drain the prefetch early
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + (size_t)b * C * H * W),
                                                    0, (int)((size_t)C * H * W * 4), 0x00020000);
  const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wf), 0,
                                                    (int)((size_t)(C / 16) * kXtWts * 4), 0x00020000);
  const auto rxt = __builtin_amdgcn_make_buffer_rsrc(xT + (size_t)b * C * H * W, 0,
                                                     (int)((size_t)C * H * W * 4), 0x00020000);
  auto load_chunk = [&](int k, float4(&sx)[kSx], float4(&sw)[kSw]) __attribute__((always_inline)) {
    k = min(k, nch - 1);  // past the end: a harmless re-load (no conditional loads)
#pragma unroll
    for (int u = 0; u < kSx; ++u) {
      const unsigned o = gx[u] >= 0 ? (unsigned)(k * 16 * H * W + gx[u]) * 4u : 0x80000000u;
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0);
      sx[u] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                          __uint_as_float(q[3]));
    }
#pragma unroll
    for (int u = 0; u < kSw; ++u) {
      const int idx = tid + NT * u;
      const unsigned o = idx < kXtWts / 4 ? (unsigned)(k * kXtWts + 4 * idx) * 4u : 0x80000000u;
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(rw, o, 0, 0);
      sw[u] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                          __uint_as_float(q[3]));
    }
  };
  auto store_chunk = [&](int bf, const float4(&sx)[kSx], const float4(&sw)[kSw])
                         __attribute__((always_inline)) {
    float* L = lds + bf * BUF;
    const int tr = (1 - bf) * BUF;  // lx's trash slots are relative to buffer 1
#pragma unroll
    for (int u = 0; u < kSx; ++u) {
      float* d = L + lx[u] + (lx[u] >= TRASH - BUF ? tr : 0);
      d[0] = sx[u].x;
      d[CP] = sx[u].y;
      d[2 * CP] = sx[u].z;
      d[3 * CP] = sx[u].w;
    }
#pragma unroll
    for (int u = 0; u < kSw; ++u) {
      const int idx = tid + NT * u;
      float* d = idx < kXtWts / 4 ? L + WIN + 4 * idx : lds + TRASH + 4 * (lane & 31);
      *reinterpret_cast<float4*>(d) = sw[u];
    }
  };
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  float e0 = 0.f, e1 = 0.f;
  // Wave w's pixel tile: pixels 16w .. 16w+15 of the ROWS x W block, row-major, so tiles
  // span rows and only the last one can hold padding (r02 gave each row 4 tiles of 16
  // pixels: 64 MFMA rows per 56-pixel row at config 3). A waves past the block's last
  // tile only stage. A row m = pixel 16w + m (clamped; the clamped rows are discarded).
  const int npx = ROWS * W;
  const bool has_tile = 16 * w < npx;
  const int pa = min(16 * w + m, npx - 1), ra = pa / W, ca = pa - ra * W;
  auto step = [&](int k, float4(&sxn)[kSx], float4(&swn)[kSw]) __attribute__((always_inline)) {
    // LDS buffer k&1 holds chunk k; (sxn, swn) chunk k+1; the other set chunk k+2 (in flight)
    const int bf = k & 1;
    const bool live = k < nch;  // the pair's second step past an odd chunk count: staging only
    const float* L = lds + bf * BUF;
    {  // input rows ho0.. (window rows 1..ROWS), this chunk's 16 channels -> xT
      const int part = tid & 3;
      constexpr int kXs = (ROWS * RW + NT / 4 - 1) / (NT / 4);  // fixed trip count: the
#pragma unroll                                                // waitcnt pass keeps counting
      for (int u = 0; u < kXs; ++u) {
        // branch-free: slots past the block read LDS word 0 and store out of range (dropped)
        const int i = (tid >> 2) + u * (NT / 4);
        const int r = i / W, px = i - r * W, y = ho0 + r;
        const bool ok = live && i < ROWS * W && y < H;
        const float4 v = *reinterpret_cast<const float4*>(
            L + (ok ? ((1 + r) * RW + 1 + px) * CP + 4 * part : 0));
        const unsigned o = ok ? (unsigned)(((y * W + px) * C + k * 16 + 4 * part) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v.x, v.y, v.z, v.w}),
                                               rxt, o, 0, 0);
      }
    }
    const float* LB = L + WIN;
    if (has_tile && live) {
#pragma unroll 1
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
        const int t = ty * 3 + tx;
        const float4 bw = *reinterpret_cast<const float4*>(LB + (t * 64 + lane) * 4);
        const float4 v0 = *reinterpret_cast<const float4*>(LB + 9 * 256 + (t * 4 + gq) * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(LB + 9 * 256 + (t * 4 + gq) * 8 + 4);
        const float4 a =
            *reinterpret_cast<const float4*>(L + ((ra + ty) * RW + ca + tx) * CP + 4 * gq);
        acc = mfma16(a.x, bw.x, acc);
        acc = mfma16(a.y, bw.y, acc);
        acc = mfma16(a.z, bw.z, acc);
        acc = mfma16(a.w, bw.w, acc);
        e0 = fmaf(a.x, v0.x, e0);
        e1 = fmaf(a.x, v0.y, e1);
        e0 = fmaf(a.y, v0.z, e0);
        e1 = fmaf(a.y, v0.w, e1);
        e0 = fmaf(a.z, v1.x, e0);
        e1 = fmaf(a.z, v1.y, e1);
        e0 = fmaf(a.w, v1.z, e0);
        e1 = fmaf(a.w, v1.w, e1);
      }
    }
    // unconditional: past the last chunk it stages a re-loaded chunk nobody reads
    store_chunk(bf ^ 1, sxn, swn);
    load_chunk(k + 3, sxn, swn);
    lds_barrier();
  };
  load_chunk(0, sx0, sw0);
  load_chunk(1, sx1, sw1);
  store_chunk(0, sx0, sw0);
  load_chunk(2, sx0, sw0);
  lds_barrier();
  // both steps of a pair always run: a conditional second step is a path on which the
  // waitcnt pass sees the other register set's loads missing, and it then waits for them
  // (vmcnt 4..1 instead of 9..6) in every first step
  for (int k = 0; k < nch; k += 2) {
    step(k, sx1, sw1);
    step(k + 1, sx0, sw0);
  }
  // through LDS as [row][j][64 pixels], then runs of consecutive pixels per offset channel
  float* T = lds;  // the buffers are free: the last barrier followed the last reads
  const int j = lane & 15;
  if (has_tile) {
    // lane groups' VALU partials (channels 4g..4g+3 of every chunk) in a fixed order
    float s0 = e0, s1 = e1;
    s0 += __shfl_xor(s0, 16);
    s1 += __shfl_xor(s1, 16);
    s0 += __shfl_xor(s0, 32);
    s1 += __shfl_xor(s1, 32);
    if (j < g.J) {
      const float bj = b_off[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // D row 4gq + i = pixel 16w + 4gq + i
        const int p = 16 * w + 4 * gq + i, ro = p / W;
        if (p < npx) T[(ro * 18 + j) * 64 + p - ro * W] = acc[i] + bj;
      }
    }
    if (lane < 16 && 16 * w + m < npx) {
      const int p = 16 * w + m, ro = p / W, co = p - ro * W;
      if (g.J > 16) T[(ro * 18 + 16) * 64 + co] = s0 + b_off[16];
      if (g.J > 17) T[(ro * 18 + 17) * 64 + co] = s1 + b_off[17];
    }
  }
  __syncthreads();
  for (int i = tid; i < ROWS * g.J * W; i += NT) {
    const int r = i / (g.J * W), rem = i - r * g.J * W, jo = rem / W, p = rem - jo * W;
    const int ho = ho0 + r;
    if (ho < H) off[((size_t)(b * g.J + jo) * H + ho) * W + p] = T[(r * 18 + jo) * 64 + p];
  }
}

bool offset_fwd_mfma_xt_ok(const Geo& g) {
  return g.dt == DCN_F32 && g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1 && g.dh == 1 &&
         g.dw == 1 && g.ph == 1 && g.pw == 1 && g.Ho == g.H && g.Wo == g.W &&
         g.W + 2 <= kXtRWmax && g.W % 4 == 0 && g.C % 16 == 0 && g.J >= 1 && g.J <= 18 &&
         (size_t)g.C * g.H * g.W * 4 < (1u << 31);  // one image of x / xT per buffer range
}

// off and xT (channels-last x) from x in one pass; wf: offset_conv_wt_floats(g) scratch
hipError_t launch_offset_conv_fwd_xt(const Geo& g, const float* x, const float* w_off,
                                     const float* b_off, float* off, float* xT, float* wf,
                                     hipStream_t s) {
  if (!offset_fwd_mfma_xt_ok(g)) return hipErrorInvalidValue;
  const int n = g.C / 16 * kXtWts;
  hipLaunchKernelGGL(woff_to_f32frag, dim3((n + 255) / 256), dim3(256), 0, s, w_off, wf, g.J, g.C);
  if (g.B > 0) {
    auto go = [&](auto kern, int rows, int nt) {
      hipLaunchKernelGGL(kern, dim3((g.H + rows - 1) / rows, 1, g.B), dim3(nt), 0, s, g, x, wf,
                         b_off, off, xT);
    };
    go(offset_conv_fwd_mfma_xt<2>, 2, 512);
  }
  return hipGetLastError();
}

size_t offset_conv_wt_floats(const Geo& g) {
  const size_t KK = (size_t)g.kh * g.kw;
  return std::max({(size_t)pad_j(g.J) * g.C * KK, (size_t)tj_pad4(g) * pad_c(g.C),
                   (size_t)(g.C + 15) / 16 * kXtWts});  // offset_conv_fwd_mfma_xt's weights
}
size_t offset_conv_fpart_floats(const Geo& g) { return (size_t)kSplit * g.B * g.J * g.HW; }

// goffT rows, then offset_wgrad_valu's per-block partials.
// (or, on the MFMA path, offset_wgrad_mfma's per-chunk partials)
size_t offset_conv_goffT_floats(const Geo& g) {
  const WgradGrid w = wgrad_grid(g, 1);  // sized for the smallest row count per wave
  size_t n = goffT_rows_floats(g) + (size_t)w.nbx * w.ny * w.nz * kJB * w.cper;
  MfmaStage ms;
  if (mfma_stage(g, &ms)) n = std::max(n, wgrad_mfma_part_floats(g, ms));
  if (offset_bwd_bf16_ok(g)) n = std::max(n, wgrad_frag_part_floats(g, ms));
  return n;
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
  if (g.sw == 1 && g.dw == 1 && g.kh == 3 && g.kw == 3) {
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

bool offset_bwd_chunkable(const Geo& g) {
  MfmaStage ms;
  const int KK = g.kh * g.kw;
  return (KK == 1 || KK == 4 || KK == 6 || KK == 9) && mfma_stage(g, &ms) &&
         !get_force_generic();
}

hipError_t launch_offset_bwd_prep(const Geo& g, const float* w_off, float* wt2, hipStream_t s) {
  const int rows = tj_pad4(g), Cp = pad_c(g.C);
  hipLaunchKernelGGL(woff_to_jtc, dim3((rows * Cp + 255) / 256), dim3(256), 0, s, w_off, wt2, g.J,
                     g.C, Cp, g.kh * g.kw, rows);
  return hipGetLastError();
}

// images [b0, b0+nb): their ∂W_off chunk partials (goffT region) and their ∂x.
// xT: fp32 channels-last x, or (xT_bf16) the bf16 one.
hipError_t launch_offset_bwd_chunk(const Geo& g, const void* xT, bool xT_bf16, const float* goff,
                                   float* goffT, const float* wt2, float* gx,
                                   const float* gxT_in, int b0, int nb, hipStream_t s,
                                   hipStream_t s_dx) {
  MfmaStage ms;
  if (!mfma_stage(g, &ms)) return hipErrorInvalidValue;
  if (nb <= 0) return hipSuccess;
  if (!s_dx) s_dx = s;
  const int TJ = g.J * g.kh * g.kw, NT = (TJ + 15) / 16;
  dim3 grid(nb * ms.cpi, (g.C + 63) / 64);
  auto wg = [&](auto kern, auto* xp) {
    hipLaunchKernelGGL(kern, grid, dim3(256), ms.lds_w, s, g, xp, goff, goffT, ms.rowsB, ms.cpi,
                       b0 * ms.cpi);
  };
  // W % 4 == 0 and C % 64 == 0: linear K-step addressing (see the kernel)
  const bool w4 = g.W % 4 == 0 && g.C % 64 == 0;
  if (xT_bf16) {
    const bf16_t* xb = static_cast<const bf16_t*>(xT);
    if (NT <= 4) w4 ? wg(offset_wgrad_mfma<1, true, bf16_t>, xb) : wg(offset_wgrad_mfma<1, false, bf16_t>, xb);
    else if (NT <= 8) w4 ? wg(offset_wgrad_mfma<2, true, bf16_t>, xb) : wg(offset_wgrad_mfma<2, false, bf16_t>, xb);
    else w4 ? wg(offset_wgrad_mfma<3, true, bf16_t>, xb) : wg(offset_wgrad_mfma<3, false, bf16_t>, xb);
  } else if (wgrad_m1(g)) {
    const int cpb = wgrad_cpb(g, ms);
    if (g.C % 128 == 0)
      hipLaunchKernelGGL(offset_wgrad_mfma_m2, dim3(nb * ms.cpi / cpb, g.C / 128), dim3(256),
                         ms.lds_w, s, g, static_cast<const float*>(xT), goff, goffT, ms.rowsB,
                         ms.cpi, b0 * ms.cpi / cpb, cpb);
    else
      hipLaunchKernelGGL(offset_wgrad_mfma_m1, dim3(nb * ms.cpi / cpb, g.C / 64), dim3(256),
                         ms.lds_w, s, g, static_cast<const float*>(xT), goff, goffT, ms.rowsB,
                         ms.cpi, b0 * ms.cpi / cpb, cpb);
  } else {
    const float* xf = static_cast<const float*>(xT);
    if (NT <= 4) w4 ? wg(offset_wgrad_mfma<1, true>, xf) : wg(offset_wgrad_mfma<1, false>, xf);
    else if (NT <= 8) w4 ? wg(offset_wgrad_mfma<2, true>, xf) : wg(offset_wgrad_mfma<2, false>, xf);
    else w4 ? wg(offset_wgrad_mfma<3, true>, xf) : wg(offset_wgrad_mfma<3, false>, xf);
  }
  hipLaunchKernelGGL(offset_dgrad_mfma, dim3(nb * ms.spi), dim3(256), ms.lds_x, s_dx, g, wt2,
                     pad_c(g.C), goff, gx, gxT_in, ms.spi, b0 * ms.spi);
  return hipGetLastError();
}

hipError_t launch_offset_bwd_finish(const Geo& g, const float* goff, const float* goffT,
                                    float* gw_off, float* gb_off, hipStream_t s,
                                    float* bsum_part) {
  MfmaStage ms;
  if (!mfma_stage(g, &ms)) return hipErrorInvalidValue;
  const long E = (long)g.C * g.J * g.kh * g.kw;
  hipLaunchKernelGGL(wgrad_mfma_reduce, dim3((unsigned)((E + 255) / 256)), dim3(1024), 0, s, g,
                     goffT, g.B * ms.cpi / wgrad_cpb(g, ms), gw_off);
  if (gb_off && bsum_part) launch_channel_sum_2l(goff, g.B, g.J, g.HW, bsum_part, gb_off, s);
  else if (gb_off) launch_channel_sum(goff, g.B, g.J, g.HW, gb_off, s);
  return hipGetLastError();
}

// xT: channels-last x; goffT, wt2: scratch ([B][HW][J], [J][KK][C]). grad_x is accumulated,
// or (gxT_in) overwritten with transpose(gxT_in) + the offset-conv route.
hipError_t launch_offset_conv_bwd(const Geo& g, const float* x, const float* xT,
                                  const float* w_off, const float* goff, float* goffT, float* wt2,
                                  float* gx, float* gw_off, float* gb_off, const float* gxT_in,
                                  hipStream_t s, hipStream_t aux, hipEvent_t fork,
                                  hipEvent_t join, float* bsum_part) {
  const int KK = g.kh * g.kw;
  bool generic = false;
  DCN_KK_DISPATCH(KK, (void)KKc);
  if (!generic && offset_bwd_chunkable(g)) {
    hipError_t e = launch_offset_bwd_prep(g, w_off, wt2, s);
    // r06 (aux given): the ∂x kernel on the side stream beside ∂W_off and its reduction, as
    // the bf16 backward does since r05 (the two share only their inputs; each alone keeps the
    // f32 MFMA busy ≈0.6 of its time, profiles/r06a_mfma_busy_config3.json)
    if (e == hipSuccess && aux) {
      e = hipEventRecord(fork, s);
      if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    }
    if (e == hipSuccess)
      e = launch_offset_bwd_chunk(g, xT, false, goff, goffT, wt2, gx, gxT_in, 0, g.B, s, aux);
    // (∂b_off, when asked for, on the main stream after the ∂W_off fold and before the join:
    // the ∂x kernel on the side stream is the longer branch, r06)
    if (e == hipSuccess) e = launch_offset_bwd_finish(g, goff, goffT, gw_off, gb_off, s, bsum_part);
    if (e == hipSuccess && aux) {
      e = hipEventRecord(join, aux);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
    }
    return e;
  }
  if (gb_off && bsum_part) launch_channel_sum_2l(goff, g.B, g.J, g.HW, bsum_part, gb_off, s);
  else if (gb_off) launch_channel_sum(goff, g.B, g.J, g.HW, gb_off, s);
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
                       pad_c(g.C), KK, g.J * KK);
    const long Mi = (long)g.B * g.HWi;
    {
      dim3 grid((unsigned)((Mi + 255) / 256), (g.C + kCB - 1) / kCB);
      DCN_KK_DISPATCH(KK, hipLaunchKernelGGL(offset_dgrad_valu<KKc>, grid, dim3(256), 0, s, g,
                                             wt2, goff, gx, gxT_in));
    }
  }
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// r05: the offset conv as GEMMs for the geometries the K3 / K7 kernels above serve only with
// their VALU forms (stride or dilation != 1, e.g. BASELINE config 5: C = 512, J = 72, 14x14
// stride 2 dilation 2, where K3 ran at 0.06 and K7 at 0.09 of the f32 MFMA peak). The conv is
// an ordinary convolution (deform_conv.py:16-21), so with its own im2col
//   ocol[p][t·C + c] = x[b][c][ho·sh - ph + i·dh][wo·sw - pw + k·dw]   (p = b·HW + m, t = i·kw + k)
// in the layout of the deformable columns (k = t·C + c: the `col` workspace region serves),
//   fwd   offT[p][j] = Σ_k W'[j][k] ocol[p][k]           (W'[j][t·C + c] = w_off[j][c][t])
//   ∂W    ∂W'[j][k]  = Σ_p ∂offT[p][j] ocol[p][k]
//   ∂x    ∂ocol[p][k] = Σ_j ∂offT[p][j] W'[j][k], then the fixed-order gather of ∂ocol into ∂x
// on the vendor f32 MFMA GEMMs (dcn_gemm.cpp); every sum has a fixed order (deterministic).
// ---------------------------------------------------------------------------
bool offset_conv_gemm_ok(const Geo& g) {
  const long P = (long)g.B * g.HW, K = (long)g.C * g.kh * g.kw;
  return g.dt == DCN_F32 && g.C % 4 == 0 && g.W <= kOcgMaxW && g.kh * g.kw <= 9 &&
         P * K < (1l << 31) &&
         (long)g.B * g.HWi * g.C < (1l << 31);
}

// ocol from channels-last xT, one float4 (4 channels) per thread
__global__ __launch_bounds__(256) void ocg_im2col(Geo g, const float* __restrict__ xT,
                                                  float* __restrict__ ocol) {
  const int C4 = g.C >> 2, KK = g.kh * g.kw;
  const long n = (long)g.B * g.HW * KK * C4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c4 = (int)(i % C4);
    const long r = i / C4;
    const int t = (int)(r % KK);
    const long p = r / KK;
    const int m = (int)(p % g.HW), b = (int)(p / g.HW);
    const int ho = m / g.Wo, wo = m - ho * g.Wo, ti = t / g.kw, tk = t - ti * g.kw;
    const int y = ho * g.sh - g.ph + ti * g.dh, x = wo * g.sw - g.pw + tk * g.dw;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y >= 0 && y < g.H && x >= 0 && x < g.W)
      v = *reinterpret_cast<const float4*>(xT + (((size_t)b * g.H + y) * g.W + x) * g.C + 4 * c4);
    reinterpret_cast<float4*>(ocol)[i] = v;  // i = (p·KK + t)·C4 + c4
  }
}

// W'[j][t·C + c] = w_off[j][c][t]
__global__ __launch_bounds__(256) void ocg_wprime(const float* __restrict__ w, float* __restrict__ wp,
                                                  int J, int C, int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= J * C * KK) return;
  const int j = i / (C * KK), r = i - j * C * KK, t = r / C, c = r - t * C;
  wp[i] = w[((size_t)j * C + c) * KK + t];
}

// off[b][j][m] = offT[b·HW + m][j] + b_off[j] (the bias last, as offset_conv_combine)
__global__ __launch_bounds__(256) void ocg_offt_to_off(const float* __restrict__ offT,
                                                       const float* __restrict__ b_off,
                                                       float* __restrict__ off, int J, int HW,
                                                       long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over (b, j, m): coalesced stores
  if (i >= total) return;
  const int m = (int)(i % HW);
  const long bj = i / HW;
  const int j = (int)(bj % J), b = (int)(bj / J);
  off[i] = offT[((size_t)b * HW + m) * J + j] + b_off[j];
}

// ∂w_off[j][c][t] = ∂W'[j][t·C + c]
__global__ __launch_bounds__(256) void ocg_wgrad_out(const float* __restrict__ gwp,
                                                     float* __restrict__ gw, int J, int C, int KK) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over (j, c, t)
  if (i >= J * C * KK) return;
  const int j = i / (C * KK), r = i - j * C * KK, c = r / KK, t = r - c * KK;
  gw[i] = gwp[(size_t)j * C * KK + (size_t)t * C + c];
}

// ∂x[b][c][y][x] = (gxT_in ? gxT_in[b][y][x][c] : ∂x[b][c][y][x]) + Σ over the taps t that
// reach (y, x) from an output pixel, in tap order, of ∂ocol[b·HW + m][t·C + c]. One workgroup
// per (image, row y, 64-channel slice): lanes run over channels (coalesced ∂ocol rows), the
// row's sums go through LDS so the NCHW stores run along x. Which output row each kernel row
// ti reaches from y, and which output column each (x, kernel column tk) comes from, are
// tabulated once per workgroup (no integer division in the loop).
constexpr int kOcgT = 9;     // taps tabulated per input pixel (kh·kw <= 9)
constexpr int kOcgXC = 16;   // input pixels of a row per pass (LDS tile rows)
// workgroup = (image, row y, 256-channel slice); lane = 4 channels (16-B loads of the ∂ocol
// rows), the 4 waves split the row's pixels; passes of kOcgXC pixels through an LDS tile so
// the NCHW stores run along x
__global__ __launch_bounds__(256) void ocg_col2im(Geo g, const float* __restrict__ docol,
                                                  const float* __restrict__ gxT_in,
                                                  float* __restrict__ gx) {
  __shared__ float4 tile[kOcgXC][65];
  __shared__ int src[kOcgMaxW][kOcgT];  // ∂ocol element offset of (x, tap) in the image, or -1
  const int y = blockIdx.x, c0 = blockIdx.y * 256, b = blockIdx.z;
  const int cl = threadIdx.x & 63, xs = threadIdx.x >> 6;
  const int c = c0 + 4 * cl, KK = g.kh * g.kw;
  const int K = KK * g.C;
  for (int i = threadIdx.x; i < g.W * kOcgT; i += 256) {
    const int x = i / kOcgT, t = i - x * kOcgT;
    int o = -1;
    if (t < KK) {
      const int ti = t / g.kw, tk = t - ti * g.kw;
      const int yy = y + g.ph - ti * g.dh, xx = x + g.pw - tk * g.dw;
      if (yy >= 0 && xx >= 0 && yy % g.sh == 0 && xx % g.sw == 0 && yy / g.sh < g.Ho &&
          xx / g.sw < g.Wo)
        o = ((yy / g.sh) * g.Wo + xx / g.sw) * K + t * g.C;
    }
    src[x][t] = o;
  }
  __syncthreads();
  const float* db = docol + (size_t)b * g.HW * K + min(c, g.C - 4);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int x0 = 0; x0 < g.W; x0 += kOcgXC) {
    const int nx = min(kOcgXC, g.W - x0);
    for (int xl = xs; xl < nx; xl += 4) {
      const int x = x0 + xl;
      // every tap's load unconditional (a lane past C or a tap that does not reach (y, x)
      // reads a valid element and drops it): no branch, so no wait per load
      float4 v[kOcgT];
#pragma unroll
      for (int t = 0; t < kOcgT; ++t)
        v[t] = *reinterpret_cast<const float4*>(db + max(src[x][t], 0));
      float4 s = z4;
#pragma unroll
      for (int t = 0; t < kOcgT; ++t)  // tap order
        if (src[x][t] >= 0) s = make_float4(s.x + v[t].x, s.y + v[t].y, s.z + v[t].z, s.w + v[t].w);
      if (gxT_in && c < g.C) {  // the sampling route's channels-last ∂x, along the channels
        const float4 q =
            *reinterpret_cast<const float4*>(gxT_in + (((size_t)b * g.H + y) * g.W + x) * g.C + c);
        s = make_float4(q.x + s.x, q.y + s.y, q.z + s.z, q.w + s.w);
      }
      tile[xl][cl] = s;
    }
    __syncthreads();
    // NCHW stores: runs of nx pixels per channel
    for (int i = threadIdx.x; i < 256 * nx; i += 256) {
      const int cc = i / nx, xl = i - cc * nx;
      if (c0 + cc >= g.C) continue;
      const float4 t4 = tile[xl][cc >> 2];
      const float v = (cc & 3) == 0 ? t4.x : (cc & 3) == 1 ? t4.y : (cc & 3) == 2 ? t4.z : t4.w;
      const size_t o = (((size_t)b * g.C + c0 + cc) * g.H + y) * g.W + x0 + xl;
      gx[o] = gxT_in ? v : gx[o] + v;
    }
    __syncthreads();
  }
}

hipError_t launch_ocg_im2col(const Geo& g, const float* xT, float* ocol, hipStream_t s) {
  const long n = (long)g.B * g.HW * g.kh * g.kw * (g.C / 4);
  const unsigned nb = (unsigned)std::min<long>((n + 255) / 256, 256l * 64);
  hipLaunchKernelGGL(ocg_im2col, dim3(nb), dim3(256), 0, s, g, xT, ocol);
  return hipGetLastError();
}
hipError_t launch_ocg_wprime(const Geo& g, const float* w_off, float* wp, hipStream_t s) {
  const int n = g.J * g.C * g.kh * g.kw;
  hipLaunchKernelGGL(ocg_wprime, dim3((n + 255) / 256), dim3(256), 0, s, w_off, wp, g.J, g.C,
                     g.kh * g.kw);
  return hipGetLastError();
}
hipError_t launch_ocg_offt_to_off(const Geo& g, const float* offT, const float* b_off, float* off,
                                  hipStream_t s) {
  const long n = (long)g.B * g.J * g.HW;
  hipLaunchKernelGGL(ocg_offt_to_off, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, offT,
                     b_off, off, g.J, g.HW, n);
  return hipGetLastError();
}
hipError_t launch_ocg_goff_to_pj(const Geo& g, const float* goff, float* goffT, hipStream_t s) {
  const long n = (long)g.B * g.J * g.HW;
  hipLaunchKernelGGL(goff_to_pj, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, goff, goffT,
                     g.J, g.J, g.HW, n);
  return hipGetLastError();
}
hipError_t launch_ocg_wgrad_out(const Geo& g, const float* gwp, float* gw_off, hipStream_t s) {
  const int n = g.J * g.C * g.kh * g.kw;
  hipLaunchKernelGGL(ocg_wgrad_out, dim3((n + 255) / 256), dim3(256), 0, s, gwp, gw_off, g.J, g.C,
                     g.kh * g.kw);
  return hipGetLastError();
}
hipError_t launch_ocg_col2im(const Geo& g, const float* docol, const float* gxT_in, float* gx,
                             hipStream_t s) {
  hipLaunchKernelGGL(ocg_col2im, dim3(g.H, (g.C + 255) / 256, g.B), dim3(256), 0, s, g, docol,
                     gxT_in, gx);
  return hipGetLastError();
}

}  // namespace dcn

