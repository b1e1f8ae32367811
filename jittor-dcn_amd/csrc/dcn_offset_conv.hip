// dcn_offset_conv.hip — the offset conv (deform_conv.py:16-21, :58) and its backward
// as implicit GEMMs on the exact-fp32 MFMA v_mfma_f32_32x32x2_f32 (gfx950).
//
// Operand maps (gfx950, 32x32x2 f32): lane l supplies A[i=l&31][k=l>>5] and
// B[k=l>>5][j=l&31]; D[row][col] lives in lane col=l&31, register r: row = drow(r, l>>5).
// Only the lane&31 index of an operand can be made contiguous in memory, so each
// kernel puts a memory-contiguous dimension there and stages the other operand in LDS:
//   K3  fwd   D[j][pixel]   A = w_off  (LDS, [c][tap][j], odd pitch)   B = x NCHW (lanes = pixels)
//   K7a ∂W    D[j][c]       A = ∂offT  (channels-last rows, lanes = j)  B = xT (lanes = channels)
//   K7b ∂x    D[c][pixel]   A = w_off  (LDS, [j][tap][c], odd pitch)   B = ∂off NCHW (lanes = pixels)
// Taps are padded to an even count (slot s of lane half hi = tap 2s+hi) so a k pair never
// straddles channels; padded taps carry zero weights.
#include "dcn_device.h"

namespace dcn {

// LDS chunking of w_off: 32 channels (K3) / 32 offset channels (K7b) per stage for
// kernels up to 3x3 (S <= 5, 42 KiB), 8 for larger kernels.
template <int S>
struct Chunk {
  static constexpr int v = S <= 5 ? 32 : 8;
};

// off[b][j][p] = b_off[j] + Σ_{c,tap} w_off[j][c][tap] · x[b][c][tap-shifted p]
// Block = 4 waves x 2 tiles x 32 pixels; grid.y = tiles of 32 offset channels j.
template <int S>
__global__ __launch_bounds__(256) void offset_conv_fwd_mfma(Geo g, const float* __restrict__ x,
                                                           const float* __restrict__ w_off,
                                                           const float* __restrict__ b_off,
                                                           float* __restrict__ off) {
  constexpr int kCCh = Chunk<S>::v;
  __shared__ float wt[kCCh * 2 * S * 33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5;
  const int KK = g.kh * g.kw, KKp = 2 * S;
  const long Mtot = (long)g.B * g.HW;
  const int j0 = blockIdx.y * 32;
  long pt[2];
  bool pok[2];
  int b[2], m[2], offs[2][S];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    pt[t] = ((long)blockIdx.x * 8 + wave * 2 + t) * 32 + (lane & 31);
    pok[t] = pt[t] < Mtot;
    b[t] = pok[t] ? (int)(pt[t] / g.HW) : 0;
    m[t] = pok[t] ? (int)(pt[t] - (long)b[t] * g.HW) : 0;
    const int ho = m[t] / g.Wo, wo = m[t] - (m[t] / g.Wo) * g.Wo;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int tap = 2 * s + hi;
      offs[t][s] = -1;
      if (pok[t] && tap < KK) {
        const int i = tap / g.kw, kx = tap - i * g.kw;
        const int y = ho * g.sh - g.ph + i * g.dh, xx = wo * g.sw - g.pw + kx * g.dw;
        if (y >= 0 && y < g.H && xx >= 0 && xx < g.W) offs[t][s] = y * g.W + xx;
      }
    }
  }
  const float* xb0 = x + (size_t)b[0] * g.C * g.HWi;
  const float* xb1 = x + (size_t)b[1] * g.C * g.HWi;
  f32x16 acc0 = {0}, acc1 = {0};
  for (int c0 = 0; c0 < g.C; c0 += kCCh) {
    __syncthreads();
    // stage w_off[j0..j0+31][c0..c0+31][tap] -> wt[(c*KKp + tap)*33 + j]; reads run along (c, tap)
    const int nstage = 32 * kCCh * KKp;
    for (int e = tid; e < nstage; e += 256) {
      const int jl = e / (kCCh * KKp), rem = e - jl * (kCCh * KKp);
      const int cl = rem / KKp, tap = rem - cl * KKp;
      const int j = j0 + jl, c = c0 + cl;
      float v = 0.f;
      if (j < g.J && c < g.C && tap < KK) v = w_off[((size_t)j * g.C + c) * KK + tap];
      wt[(cl * KKp + tap) * 33 + jl] = v;
    }
    __syncthreads();
    const int cn = min(kCCh, g.C - c0);
    // software pipeline: the x values of channel cl+1 are in flight while cl's MFMAs run
    float v0[S], v1[S];
    auto fetch = [&](int cl, float* d0, float* d1) {
      const float* x0 = xb0 + (size_t)(c0 + cl) * g.HWi;
      const float* x1 = xb1 + (size_t)(c0 + cl) * g.HWi;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        d0[s] = offs[0][s] >= 0 ? x0[offs[0][s]] : 0.f;
        d1[s] = offs[1][s] >= 0 ? x1[offs[1][s]] : 0.f;
      }
    };
    fetch(0, v0, v1);
    for (int cl = 0; cl < cn; ++cl) {
      float n0[S], n1[S];
      if (cl + 1 < cn) fetch(cl + 1, n0, n1);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float a = wt[(cl * KKp + 2 * s + hi) * 33 + (lane & 31)];
        acc0 = mfma32(a, v0[s], acc0);
        acc1 = mfma32(a, v1[s], acc1);
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        v0[s] = n0[s];
        v1[s] = n1[s];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = j0 + drow(r, hi);
    if (j < g.J) {
      if (pok[0]) off[((size_t)b[0] * g.J + j) * g.HW + m[0]] = acc0[r] + b_off[j];
      if (pok[1]) off[((size_t)b[1] * g.J + j) * g.HW + m[1]] = acc1[r] + b_off[j];
    }
  }
}

// ∂w_off[j][c][tap] += Σ_p ∂off[b][j][p] · x[b][c][tap-shifted p]
// One wave = one (tap, 32-channel tile, 32-offset-channel tile, pixel range): D[j][c]
// with A from the channels-last ∂offT[b][p][j] rows and B from the channels-last
// xT[b][y][x][c] rows (both contiguous across lanes).
__global__ __launch_bounds__(256) void offset_wgrad_mfma(Geo g, const float* __restrict__ xT,
                                                         const float* __restrict__ goffT,
                                                         float* __restrict__ gw, int ppw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hi = lane >> 5, l31 = lane & 31;
  const long Mtot = (long)g.B * g.HW;
  const long pstart = ((long)blockIdx.x * 4 + wave) * ppw;
  if (pstart >= Mtot) return;
  const long pend = min(pstart + (long)ppw, Mtot);
  const int KK = g.kh * g.kw;
  const int tap = blockIdx.z % KK, j0 = (blockIdx.z / KK) * 32;
  const int ti = tap / g.kw, tx = tap - ti * g.kw;
  const int dyo = ti * g.dh - g.ph, dxo = tx * g.dw - g.pw;
  const int c = blockIdx.y * 32 + l31;
  const bool cok = c < g.C;
  const bool jok = j0 + l31 < g.J;
  long p = pstart + hi;
  int b = (int)(p / g.HW);
  int mm = (int)(p - (long)b * g.HW);
  int ho = mm / g.Wo, wo = mm - ho * g.Wo;
  f32x16 acc = {0};
  // 8 pixel pairs per batch: all 16 loads issued before the 8 MFMAs consume them
  constexpr int U = 8;
  for (long q0 = pstart; q0 < pend; q0 += 2 * U) {
    float a[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = 0.f;
      bv[u] = 0.f;
      if (q0 + 2 * u + hi < pend) {
        const size_t pix = (size_t)b * g.HW + (size_t)ho * g.Wo + wo;
        if (jok) a[u] = goffT[pix * g.J + j0 + l31];
        const int y = ho * g.sh + dyo, xx = wo * g.sw + dxo;
        if (cok && y >= 0 && y < g.H && xx >= 0 && xx < g.W)
          bv[u] = xT[(((size_t)b * g.H + y) * g.W + xx) * g.C + c];
      }
      wo += 2;
      if (wo >= g.Wo) {
        wo -= g.Wo;
        if (++ho >= g.Ho) {
          ho = 0;
          ++b;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = mfma32(a[u], bv[u], acc);
  }
  if (!cok) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = j0 + drow(r, hi);
    if (j < g.J) atomicAdd(gw + ((size_t)j * g.C + c) * KK + tap, acc[r]);
  }
}

// ∂x[b][c][y][x] += Σ_{j,tap} w_off[j][c][tap] · ∂off[b][j][(y+pad-tap·dil)/s]
// D[c (32)][input pixel (32)]; A = w_off slice staged in LDS [j][tap][c]; B = ∂off.
// Each wave: 2 tiles of 32 input pixels; each tile's outputs are owned (RMW, no atomics).
template <int S>
__global__ __launch_bounds__(256) void offset_dgrad_mfma(Geo g, const float* __restrict__ w_off,
                                                         const float* __restrict__ goff,
                                                         float* __restrict__ gx) {
  constexpr int JC = Chunk<S>::v;
  __shared__ float wl[JC * 2 * S * 33];  // [j][tap][c] (odd pitch)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5;
  const int KK = g.kh * g.kw, KKp = 2 * S;
  const int ct0 = blockIdx.y * 32;
  const long Mi = (long)g.B * g.HWi;
  long pt[2];
  bool pok[2];
  int bb[2], yx[2], goffs[2][S];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    pt[t] = ((long)blockIdx.x * 8 + wave * 2 + t) * 32 + (lane & 31);
    pok[t] = pt[t] < Mi;
    bb[t] = pok[t] ? (int)(pt[t] / g.HWi) : 0;
    yx[t] = pok[t] ? (int)(pt[t] - (long)bb[t] * g.HWi) : 0;
    const int y = yx[t] / g.W, xx = yx[t] - (yx[t] / g.W) * g.W;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int tap = 2 * s + hi;
      goffs[t][s] = -1;
      if (pok[t] && tap < KK) {
        const int i = tap / g.kw, kx = tap - i * g.kw;
        const int tt = y + g.ph - i * g.dh, u = xx + g.pw - kx * g.dw;
        if (tt >= 0 && u >= 0 && tt % g.sh == 0 && u % g.sw == 0) {
          const int ho = tt / g.sh, wo = u / g.sw;
          if (ho < g.Ho && wo < g.Wo) goffs[t][s] = ho * g.Wo + wo;
        }
      }
    }
  }
  const float* gb0 = goff + (size_t)bb[0] * g.J * g.HW;
  const float* gb1 = goff + (size_t)bb[1] * g.J * g.HW;
  f32x16 acc0 = {0}, acc1 = {0};
  for (int jc = 0; jc < g.J; jc += JC) {
    __syncthreads();
    for (int e = tid; e < JC * KKp * 32; e += 256) {
      const int jl = e / (KKp * 32), rem = e - jl * (KKp * 32);
      const int cl = rem / KKp, tap = rem - cl * KKp;  // reads run along (c, tap) of one j
      const int c = ct0 + cl, jj = jc + jl;
      float v = 0.f;
      if (jj < g.J && c < g.C && tap < KK) v = w_off[((size_t)jj * g.C + c) * KK + tap];
      wl[(jl * KKp + tap) * 33 + cl] = v;
    }
    __syncthreads();
    const int jn = min(JC, g.J - jc);
    float v0[S], v1[S];
    auto fetch = [&](int jl, float* d0, float* d1) {
      const float* g0 = gb0 + (size_t)(jc + jl) * g.HW;
      const float* g1 = gb1 + (size_t)(jc + jl) * g.HW;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        d0[s] = goffs[0][s] >= 0 ? g0[goffs[0][s]] : 0.f;
        d1[s] = goffs[1][s] >= 0 ? g1[goffs[1][s]] : 0.f;
      }
    };
    fetch(0, v0, v1);
    for (int jl = 0; jl < jn; ++jl) {
      float n0[S], n1[S];
      if (jl + 1 < jn) fetch(jl + 1, n0, n1);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float a = wl[(jl * KKp + 2 * s + hi) * 33 + (lane & 31)];
        acc0 = mfma32(a, v0[s], acc0);
        acc1 = mfma32(a, v1[s], acc1);
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        v0[s] = n0[s];
        v1[s] = n1[s];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = ct0 + drow(r, hi);
    if (c < g.C) {
      if (pok[0]) gx[((size_t)bb[0] * g.C + c) * g.HWi + yx[0]] += acc0[r];
      if (pok[1]) gx[((size_t)bb[1] * g.C + c) * g.HWi + yx[1]] += acc1[r];
    }
  }
}

#define DCN_S_DISPATCH(SV, ...) \
  switch (SV) {                  \
    case 1: { constexpr int S = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int S = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int S = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int S = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int S = 5; __VA_ARGS__; } break; \
    case 8: { constexpr int S = 8; __VA_ARGS__; } break; \
    case 13: { constexpr int S = 13; __VA_ARGS__; } break; \
    default: return hipErrorInvalidValue; \
  }

static int slots_for(const Geo& g) {
  int S = (g.kh * g.kw + 1) / 2;
  if (S > 5 && S <= 8) S = 8;
  else if (S > 8 && S <= 13) S = 13;
  return S;
}

hipError_t launch_offset_conv_fwd(const Geo& g, const float* x, const float* w_off,
                                  const float* b_off, float* off, hipStream_t s) {
  const long Mtot = (long)g.B * g.HW;
  const long tiles = (Mtot + 31) / 32;
  dim3 grid((unsigned)((tiles + 7) / 8), (g.J + 31) / 32);
  DCN_S_DISPATCH(slots_for(g), hipLaunchKernelGGL(offset_conv_fwd_mfma<S>, grid, dim3(256), 0,
                                                  s, g, x, w_off, b_off, off));
  return hipGetLastError();
}

// goffT: scratch [B][HW][J]; xT: channels-last x [B][H][W][C]. grad_x is accumulated.
hipError_t launch_offset_conv_bwd(const Geo& g, const float* xT, const float* w_off,
                                  const float* goff, float* goffT, float* gx, float* gw_off,
                                  float* gb_off, hipStream_t s) {
  const int KK = g.kh * g.kw;
  hipError_t e = hipMemsetAsync(gw_off, 0, (size_t)g.J * g.C * KK * sizeof(float), s);
  if (e != hipSuccess) return e;
  launch_channel_sum(goff, g.B, g.J, g.HW, gb_off, s);
  e = launch_nchw_to_nhwc(goff, goffT, g.B, g.J, g.HW, s);
  if (e != hipSuccess) return e;
  {
    const long Mtot = (long)g.B * g.HW;
    const int ppw = 2048;
    const long waves = (Mtot + ppw - 1) / ppw;
    dim3 grid((unsigned)((waves + 3) / 4), (g.C + 31) / 32, KK * ((g.J + 31) / 32));
    hipLaunchKernelGGL(offset_wgrad_mfma, grid, dim3(256), 0, s, g, xT, goffT, gw_off, ppw);
  }
  {
    const long Mi = (long)g.B * g.HWi;
    const long tiles = (Mi + 31) / 32;
    dim3 grid((unsigned)((tiles + 7) / 8), (g.C + 31) / 32);
    DCN_S_DISPATCH(slots_for(g), hipLaunchKernelGGL(offset_dgrad_mfma<S>, grid, dim3(256), 0, s,
                                                    g, w_off, goff, gx));
  }
  return hipGetLastError();
}

}  // namespace dcn
