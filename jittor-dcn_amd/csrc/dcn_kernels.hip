// dcn_kernels.hip — hand-written CDNA4 (gfx950) kernels of the DeformConv2d hot path.
//
// Semantics follow /root/reference/deform_conv.py:56-81 exactly:
//   * sample for output (h, w), tap n:  row ≈ w + Δx[n], col ≈ h + Δy[n]   (Q1, :39/:47)
//   * coordinates normalised by the OUTPUT size and unnormalised by the INPUT
//     size with align_corners=True (Q2, :37-38 + grid_sample)
//   * no per-tap base position (Q3, :64-66); offsets [Δx(0..N-1) | Δy(0..N-1)] (Q4, :62)
//   * columns ordered k = n*C + c (Q5, :72-74)
// The coordinate chain is evaluated in fp32 in the reference's own op order; this
// file is compiled with -ffp-contract=off so no FMA changes which side of an
// integer a coordinate lands on (Q6). Interpolation and reductions use explicit
// fmaf where a fused multiply-add is wanted.
#include <climits>

#include "dcn_internal.h"

namespace dcn {

static int g_force_generic = 0;
void set_force_generic(int on) { g_force_generic = on; }
int get_force_generic() { return g_force_generic; }

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// Sampling coordinates: deform_conv.py:64-68 (grid (w,h) + offset), :37-39
// (norm by (W_out-1),(H_out-1); grid = [norm_y, norm_x]) and grid_sample's
// align_corners=True unnormalisation ((g+1)/2)*(size-1). grid[...,0] = norm_y
// indexes the input COLUMN (width), grid[...,1] = norm_x the input ROW.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ref_coord(int h, int w, float dx, float dy,
                                          const Geo& g, float& iy, float& ix) {
  const float cx = (float)w + dx;                 // grid x + offset x
  float nx = cx / (float)(g.Wo - 1);              // coords[...,0] / (W_out - 1)
  nx = nx * 2.0f;
  nx = nx - 1.0f;
  iy = ((nx + 1.0f) / 2.0f) * (float)(g.H - 1);   // unnormalise over input H
  const float cy = (float)h + dy;
  float ny = cy / (float)(g.Ho - 1);
  ny = ny * 2.0f;
  ny = ny - 1.0f;
  ix = ((ny + 1.0f) / 2.0f) * (float)(g.W - 1);   // unnormalise over input W
}

// A sample contributes only if at least one of its four corners can be inside
// the image: floor(row) in [-1, H-1] and floor(col) in [-1, W-1]. Otherwise the
// value and every derivative are exactly 0 (zeros padding). NaN -> invalid.
struct Tap {
  int r0, c0;
  float fr, fc;
  bool ok;
};

__device__ __forceinline__ Tap make_tap(float iy, float ix, const Geo& g) {
  Tap t;
  const float r0f = floorf(iy), c0f = floorf(ix);
  t.ok = (r0f >= -1.0f) && (r0f <= (float)(g.H - 1)) && (c0f >= -1.0f) &&
         (c0f <= (float)(g.W - 1));
  t.r0 = t.ok ? (int)r0f : 0;
  t.c0 = t.ok ? (int)c0f : 0;
  t.fr = t.ok ? iy - r0f : 0.f;
  t.fc = t.ok ? ix - c0f : 0.f;
  return t;
}

// Canonical fp32 bilinear combination (shared by every kernel and by the C
// oracle so window/generic kernels agree bit for bit).
__device__ __forceinline__ float bilerp(float fr, float fc, float x00, float x01,
                                        float x10, float x11) {
  const float gr = 1.0f - fr, gc = 1.0f - fc;
  float v = (gr * gc) * x00;
  v = fmaf(gr * fc, x01, v);
  v = fmaf(fr * gc, x10, v);
  v = fmaf(fr * fc, x11, v);
  return v;
}

__device__ __forceinline__ float ldx(const float* __restrict__ xp, int r, int c,
                                     const Geo& g) {
  return (r >= 0 && r < g.H && c >= 0 && c < g.W) ? xp[r * g.W + c] : 0.f;
}

// ---------------------------------------------------------------------------
// Generic kernels (global-memory gathers): one thread per (b, group, tap, pixel).
// Used for tiny shapes, for pathological offsets and as an independent
// cross-check of the LDS-window kernels in the parity tests.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void im2col_generic(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      float* __restrict__ col, int b0, int nb) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)nb * g.G * g.N * g.HW;
  if (idx >= total) return;
  const int m = (int)(idx % g.HW);
  long t = idx / g.HW;
  const int n = (int)(t % g.N);
  t /= g.N;
  const int gi = (int)(t % g.G);
  const int bl = (int)(t / g.G);
  const int b = b0 + bl;
  const int h = m / g.Wo, w = m - h * g.Wo;
  const float* ob = off + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  float iy, ix;
  ref_coord(h, w, ob[(size_t)n * g.HW + m], ob[(size_t)(g.N + n) * g.HW + m], g, iy, ix);
  const Tap tp = make_tap(iy, ix, g);
  for (int cl = 0; cl < g.Cg; ++cl) {
    const int c = gi * g.Cg + cl;
    float v = 0.f;
    if (tp.ok) {
      const float* xp = x + ((size_t)b * g.C + c) * g.HWi;
      v = bilerp(tp.fr, tp.fc, ldx(xp, tp.r0, tp.c0, g), ldx(xp, tp.r0, tp.c0 + 1, g),
                 ldx(xp, tp.r0 + 1, tp.c0, g), ldx(xp, tp.r0 + 1, tp.c0 + 1, g));
    }
    col[((size_t)bl * g.K + (size_t)n * g.C + c) * g.HW + m] = v;
  }
}

__device__ __forceinline__ void scatter_global(float* __restrict__ gxp, int r, int c,
                                               float v, const Geo& g) {
  if (v != 0.f && r >= 0 && r < g.H && c >= 0 && c < g.W) atomicAdd(gxp + r * g.W + c, v);
}

__global__ __launch_bounds__(256) void col2im_generic(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      const float* __restrict__ gcol,
                                                      float* __restrict__ gx,
                                                      float* __restrict__ goff, int b0, int nb) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)nb * g.G * g.N * g.HW;
  if (idx >= total) return;
  const int m = (int)(idx % g.HW);
  long t = idx / g.HW;
  const int n = (int)(t % g.N);
  t /= g.N;
  const int gi = (int)(t % g.G);
  const int bl = (int)(t / g.G);
  const int b = b0 + bl;
  const int h = m / g.Wo, w = m - h * g.Wo;
  const float* ob = off + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  float iy, ix;
  ref_coord(h, w, ob[(size_t)n * g.HW + m], ob[(size_t)(g.N + n) * g.HW + m], g, iy, ix);
  const Tap tp = make_tap(iy, ix, g);
  float diy = 0.f, dix = 0.f;
  if (tp.ok) {
    const float gr = 1.0f - tp.fr, gc = 1.0f - tp.fc;
    for (int cl = 0; cl < g.Cg; ++cl) {
      const int c = gi * g.Cg + cl;
      const float gv = gcol[((size_t)bl * g.K + (size_t)n * g.C + c) * g.HW + m];
      const float* xp = x + ((size_t)b * g.C + c) * g.HWi;
      const float x00 = ldx(xp, tp.r0, tp.c0, g), x01 = ldx(xp, tp.r0, tp.c0 + 1, g);
      const float x10 = ldx(xp, tp.r0 + 1, tp.c0, g), x11 = ldx(xp, tp.r0 + 1, tp.c0 + 1, g);
      diy = fmaf(gv, fmaf(tp.fc, x11 - x01, gc * (x10 - x00)), diy);
      dix = fmaf(gv, fmaf(tp.fr, x11 - x10, gr * (x01 - x00)), dix);
      float* gxp = gx + ((size_t)b * g.C + c) * g.HWi;
      scatter_global(gxp, tp.r0, tp.c0, gv * (gr * gc), g);
      scatter_global(gxp, tp.r0, tp.c0 + 1, gv * (gr * tp.fc), g);
      scatter_global(gxp, tp.r0 + 1, tp.c0, gv * (tp.fr * gc), g);
      scatter_global(gxp, tp.r0 + 1, tp.c0 + 1, gv * (tp.fr * tp.fc), g);
    }
  }
  // ∂off = ∂row * (H-1)/(W_out-1) (Δx channel n), ∂col * (W-1)/(H_out-1) (Δy channel N+n)
  const float sy = (float)(g.H - 1) / (float)(g.Wo - 1);
  const float sx = (float)(g.W - 1) / (float)(g.Ho - 1);
  float* gob = goff + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  gob[(size_t)n * g.HW + m] = diy * sy;
  gob[(size_t)(g.N + n) * g.HW + m] = dix * sx;
}

// ---------------------------------------------------------------------------
// LDS-window kernels (the production K1 / K5).
//
// Block = 256 threads = 256 consecutive output pixels m of one image and one
// deform group; each thread keeps its NT taps' corner index + fractions in
// registers for the whole channel loop. The block reduces the min/max corner
// row/col of its valid samples and stages exactly that input window (plus the
// zero border) for CC channels at a time into LDS with coalesced row loads.
// Because output pixels run along w and w drives the input ROW (Q1), lanes of a
// wave read LDS rows r, r+1, ... — the row pitch WCp is forced odd so those land
// in distinct banks. col / ∂col are read and written coalesced along m.
// ---------------------------------------------------------------------------
constexpr int kTPB = 256;
constexpr int kRedFloats = 32;  // reduction scratch at the LDS base (16-B aligned after)

__device__ __forceinline__ void block_minmax(int& rmin, int& rmax, int& cmin, int& cmax,
                                             int* red) {
  for (int o = 32; o > 0; o >>= 1) {
    rmin = min(rmin, __shfl_xor(rmin, o));
    rmax = max(rmax, __shfl_xor(rmax, o));
    cmin = min(cmin, __shfl_xor(cmin, o));
    cmax = max(cmax, __shfl_xor(cmax, o));
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[wave * 4 + 0] = rmin;
    red[wave * 4 + 1] = rmax;
    red[wave * 4 + 2] = cmin;
    red[wave * 4 + 3] = cmax;
  }
  __syncthreads();
  rmin = red[0];
  rmax = red[1];
  cmin = red[2];
  cmax = red[3];
  for (int wv = 1; wv < kTPB / 64; ++wv) {
    rmin = min(rmin, red[wv * 4 + 0]);
    rmax = max(rmax, red[wv * 4 + 1]);
    cmin = min(cmin, red[wv * 4 + 2]);
    cmax = max(cmax, red[wv * 4 + 3]);
  }
  __syncthreads();
}

template <int NT>
struct TapSet {
  int r0[NT], c0[NT];
  float fr[NT], fc[NT];
  bool ok[NT];
};

// Compute this thread's taps and the block's window. Returns false if no sample
// of the block touches the image.
template <int NT>
__device__ __forceinline__ bool setup_window(const Geo& g, const float* __restrict__ off,
                                             int b, int gi, int m, bool mok, TapSet<NT>& ts,
                                             int* red, int& rlo, int& clo, int& WR, int& WC) {
  const int h = mok ? m / g.Wo : 0, w = mok ? m - (m / g.Wo) * g.Wo : 0;
  const float* ob = off + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  int rmin = INT_MAX, rmax = INT_MIN, cmin = INT_MAX, cmax = INT_MIN;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    Tap tp;
    tp.ok = false;
    tp.r0 = tp.c0 = 0;
    tp.fr = tp.fc = 0.f;
    if (mok) {
      float iy, ix;
      ref_coord(h, w, ob[(size_t)n * g.HW + m], ob[(size_t)(NT + n) * g.HW + m], g, iy, ix);
      tp = make_tap(iy, ix, g);
    }
    ts.r0[n] = tp.r0;
    ts.c0[n] = tp.c0;
    ts.fr[n] = tp.fr;
    ts.fc[n] = tp.fc;
    ts.ok[n] = tp.ok;
    if (tp.ok) {
      rmin = min(rmin, tp.r0);
      rmax = max(rmax, tp.r0);
      cmin = min(cmin, tp.c0);
      cmax = max(cmax, tp.c0);
    }
  }
  block_minmax(rmin, rmax, cmin, cmax, red);
  if (rmin > rmax) return false;
  rlo = rmin;
  clo = cmin;
  WR = rmax - rmin + 2;  // rows r0 .. r0+1
  WC = cmax - cmin + 2;
  return true;
}

template <int NT>
__global__ __launch_bounds__(kTPB) void im2col_window(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      float* __restrict__ col, int b0,
                                                      int lds_floats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* red = reinterpret_cast<int*>(smem);
  float* win = smem + kRedFloats;
  const int tid = threadIdx.x;
  const int m = blockIdx.x * kTPB + tid;
  const int gi = blockIdx.y, bl = blockIdx.z, b = b0 + bl;
  const bool mok = m < g.HW;
  TapSet<NT> ts;
  int rlo = 0, clo = 0, WR = 0, WC = 0;
  const bool any = setup_window<NT>(g, off, b, gi, m, mok, ts, red, rlo, clo, WR, WC);
  const size_t nstride = (size_t)g.C * g.HW;  // col distance between taps n and n+1
  float* colp = col + ((size_t)bl * g.K + (size_t)gi * g.Cg) * g.HW + m;
  if (!any) {
    if (mok)
      for (int cl = 0; cl < g.Cg; ++cl)
#pragma unroll
        for (int n = 0; n < NT; ++n) colp[(size_t)cl * g.HW + n * nstride] = 0.f;
    return;
  }
  const int WCp = WC | 1;
  const int plane = WR * WCp;
  const int CC = min(g.Cg, (lds_floats - kRedFloats) / plane);
  const float* xg = x + ((size_t)b * g.C + (size_t)gi * g.Cg) * g.HWi;
  if (CC <= 0 || WCp > kTPB) {
    // Window larger than LDS (pathological offsets): gather straight from L2.
    if (!mok) return;
    for (int cl = 0; cl < g.Cg; ++cl) {
      const float* xp = xg + (size_t)cl * g.HWi;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        float v = 0.f;
        if (ts.ok[n])
          v = bilerp(ts.fr[n], ts.fc[n], ldx(xp, ts.r0[n], ts.c0[n], g),
                     ldx(xp, ts.r0[n], ts.c0[n] + 1, g), ldx(xp, ts.r0[n] + 1, ts.c0[n], g),
                     ldx(xp, ts.r0[n] + 1, ts.c0[n] + 1, g));
        colp[(size_t)cl * g.HW + n * nstride] = v;
      }
    }
    return;
  }
  int li[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) li[n] = ts.ok[n] ? (ts.r0[n] - rlo) * WCp + (ts.c0[n] - clo) : 0;

  // staging map: thread -> (row-in-pass rr0, column cc)
  const int rpp = kTPB / WCp;
  const int cc = tid % WCp, rr0 = tid / WCp;
  for (int cs = 0; cs < g.Cg; cs += CC) {
    const int CCa = min(CC, g.Cg - cs);
    if (rr0 < rpp) {
      const int RR = CCa * WR;
      int cl = 0, r = rr0;
      while (r >= WR) { r -= WR; ++cl; }
      const int gc = clo + cc;
      const bool cin = cc < WC && gc >= 0 && gc < g.W;
      for (int rr = rr0; rr < RR; rr += rpp) {
        const int gr = rlo + r;
        float v = 0.f;
        if (cin && gr >= 0 && gr < g.H) v = xg[(size_t)(cs + cl) * g.HWi + gr * g.W + gc];
        win[rr * WCp + cc] = v;
        r += rpp;
        while (r >= WR) { r -= WR; ++cl; }
      }
    }
    __syncthreads();
    if (mok) {
      for (int cl = 0; cl < CCa; ++cl) {
        const float* L = win + cl * plane;
        float* dst = colp + (size_t)(cs + cl) * g.HW;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const float* p = L + li[n];
          const float v = ts.ok[n] ? bilerp(ts.fr[n], ts.fc[n], p[0], p[1], p[WCp], p[WCp + 1]) : 0.f;
          dst[n * nstride] = v;
        }
      }
    }
    __syncthreads();
  }
}

template <int NT>
__global__ __launch_bounds__(kTPB) void col2im_window(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      const float* __restrict__ gcol,
                                                      float* __restrict__ gx,
                                                      float* __restrict__ goff, int b0,
                                                      int lds_floats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* red = reinterpret_cast<int*>(smem);
  float* win = smem + kRedFloats;
  const int tid = threadIdx.x;
  const int m = blockIdx.x * kTPB + tid;
  const int gi = blockIdx.y, bl = blockIdx.z, b = b0 + bl;
  const bool mok = m < g.HW;
  TapSet<NT> ts;
  int rlo = 0, clo = 0, WR = 0, WC = 0;
  const bool any = setup_window<NT>(g, off, b, gi, m, mok, ts, red, rlo, clo, WR, WC);
  float diy[NT], dix[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) diy[n] = dix[n] = 0.f;
  const size_t nstride = (size_t)g.C * g.HW;
  const float* gcolp = gcol + ((size_t)bl * g.K + (size_t)gi * g.Cg) * g.HW + m;
  const float* xg = x + ((size_t)b * g.C + (size_t)gi * g.Cg) * g.HWi;
  float* gxg = gx + ((size_t)b * g.C + (size_t)gi * g.Cg) * g.HWi;
  if (any) {
    const int WCp = WC | 1;
    const int plane = WR * WCp;
    const int CC = min(g.Cg, (lds_floats - kRedFloats) / (2 * plane));
    if (CC <= 0 || WCp > kTPB) {
      if (mok) {
        for (int cl = 0; cl < g.Cg; ++cl) {
          const float* xp = xg + (size_t)cl * g.HWi;
          float* gxp = gxg + (size_t)cl * g.HWi;
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            if (!ts.ok[n]) continue;
            const float gv = gcolp[(size_t)cl * g.HW + n * nstride];
            const int r0 = ts.r0[n], c0 = ts.c0[n];
            const float fr = ts.fr[n], fc = ts.fc[n], gr = 1.0f - fr, gc = 1.0f - fc;
            const float x00 = ldx(xp, r0, c0, g), x01 = ldx(xp, r0, c0 + 1, g);
            const float x10 = ldx(xp, r0 + 1, c0, g), x11 = ldx(xp, r0 + 1, c0 + 1, g);
            diy[n] = fmaf(gv, fmaf(fc, x11 - x01, gc * (x10 - x00)), diy[n]);
            dix[n] = fmaf(gv, fmaf(fr, x11 - x10, gr * (x01 - x00)), dix[n]);
            scatter_global(gxp, r0, c0, gv * (gr * gc), g);
            scatter_global(gxp, r0, c0 + 1, gv * (gr * fc), g);
            scatter_global(gxp, r0 + 1, c0, gv * (fr * gc), g);
            scatter_global(gxp, r0 + 1, c0 + 1, gv * (fr * fc), g);
          }
        }
      }
    } else {
      float* dwin = win + CC * plane;  // ∂x window accumulators
      int li[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) li[n] = ts.ok[n] ? (ts.r0[n] - rlo) * WCp + (ts.c0[n] - clo) : 0;
      const int rpp = kTPB / WCp;
      const int cc = tid % WCp, rr0 = tid / WCp;
      const int gcc = clo + cc;
      const bool cin = cc < WC && gcc >= 0 && gcc < g.W;
      for (int cs = 0; cs < g.Cg; cs += CC) {
        const int CCa = min(CC, g.Cg - cs);
        const int RR = CCa * WR;
        if (rr0 < rpp) {
          int cl = 0, r = rr0;
          while (r >= WR) { r -= WR; ++cl; }
          for (int rr = rr0; rr < RR; rr += rpp) {
            const int gr = rlo + r;
            float v = 0.f;
            if (cin && gr >= 0 && gr < g.H) v = xg[(size_t)(cs + cl) * g.HWi + gr * g.W + gcc];
            win[rr * WCp + cc] = v;
            dwin[rr * WCp + cc] = 0.f;
            r += rpp;
            while (r >= WR) { r -= WR; ++cl; }
          }
        }
        __syncthreads();
        if (mok) {
          for (int cl = 0; cl < CCa; ++cl) {
            const float* L = win + cl * plane;
            float* D = dwin + cl * plane;
            const float* gp = gcolp + (size_t)(cs + cl) * g.HW;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              if (!ts.ok[n]) continue;
              const float gv = gp[n * nstride];
              const float* p = L + li[n];
              const float x00 = p[0], x01 = p[1], x10 = p[WCp], x11 = p[WCp + 1];
              const float fr = ts.fr[n], fc = ts.fc[n], gr = 1.0f - fr, gc = 1.0f - fc;
              diy[n] = fmaf(gv, fmaf(fc, x11 - x01, gc * (x10 - x00)), diy[n]);
              dix[n] = fmaf(gv, fmaf(fr, x11 - x10, gr * (x01 - x00)), dix[n]);
              if (gv != 0.f) {
                float* q = D + li[n];
                atomicAdd(q, gv * (gr * gc));
                atomicAdd(q + 1, gv * (gr * fc));
                atomicAdd(q + WCp, gv * (fr * gc));
                atomicAdd(q + WCp + 1, gv * (fr * fc));
              }
            }
          }
        }
        __syncthreads();
        // flush the ∂x window to global memory (windows of neighbouring tiles overlap)
        if (rr0 < rpp) {
          int cl = 0, r = rr0;
          while (r >= WR) { r -= WR; ++cl; }
          for (int rr = rr0; rr < RR; rr += rpp) {
            const int gr = rlo + r;
            const float v = dwin[rr * WCp + cc];
            if (cin && gr >= 0 && gr < g.H && v != 0.f)
              atomicAdd(gxg + (size_t)(cs + cl) * g.HWi + gr * g.W + gcc, v);
            r += rpp;
            while (r >= WR) { r -= WR; ++cl; }
          }
        }
        __syncthreads();
      }
    }
  }
  if (mok) {
    const float sy = (float)(g.H - 1) / (float)(g.Wo - 1);
    const float sx = (float)(g.W - 1) / (float)(g.Ho - 1);
    float* gob = goff + ((size_t)b * g.J + (size_t)gi * 2 * NT) * g.HW + m;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      gob[(size_t)n * g.HW] = diy[n] * sy;
      gob[(size_t)(NT + n) * g.HW] = dix[n] * sx;
    }
  }
}

// LDS budget per block: K1 keeps CC x-planes, K5 CC x-planes + CC ∂x-planes.
constexpr int kLdsFloatsK1 = 12288;  // 48 KiB -> 3 blocks / CU
constexpr int kLdsFloatsK5 = 16384;  // 64 KiB -> 2 blocks / CU

#define DCN_NT_DISPATCH(NTV, ...) \
  switch (NTV) {                   \
    case 1: { constexpr int NT = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int NT = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int NT = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int NT = 4; __VA_ARGS__; } break; \
    case 6: { constexpr int NT = 6; __VA_ARGS__; } break; \
    case 9: { constexpr int NT = 9; __VA_ARGS__; } break; \
    default: use_generic = true; break; \
  }

hipError_t launch_im2col(const Geo& g, const float* x, const float* off, float* col, int b0,
                         int nb, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  bool use_generic = g_force_generic != 0;
  if (!use_generic) {
    dim3 grid((g.HW + kTPB - 1) / kTPB, g.G, nb);
    const size_t lds = (size_t)kLdsFloatsK1 * sizeof(float);
    DCN_NT_DISPATCH(g.N, hipLaunchKernelGGL(im2col_window<NT>, grid, dim3(kTPB), lds, s, g, x,
                                            off, col, b0, kLdsFloatsK1));
  }
  if (use_generic) {
    const long total = (long)nb * g.G * g.N * g.HW;
    hipLaunchKernelGGL(im2col_generic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       g, x, off, col, b0, nb);
  }
  return hipGetLastError();
}

hipError_t launch_col2im_coord(const Geo& g, const float* x, const float* off,
                               const float* gcol, float* gx, float* goff, int b0, int nb,
                               hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  bool use_generic = g_force_generic != 0;
  if (!use_generic) {
    dim3 grid((g.HW + kTPB - 1) / kTPB, g.G, nb);
    const size_t lds = (size_t)kLdsFloatsK5 * sizeof(float);
    DCN_NT_DISPATCH(g.N, hipLaunchKernelGGL(col2im_window<NT>, grid, dim3(kTPB), lds, s, g, x,
                                            off, gcol, gx, goff, b0, kLdsFloatsK5));
  }
  if (use_generic) {
    const long total = (long)nb * g.G * g.N * g.HW;
    hipLaunchKernelGGL(col2im_generic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       g, x, off, gcol, gx, goff, b0, nb);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Offset conv (deform_conv.py:16-21, :58) as implicit GEMMs on the exact-fp32
// MFMA v_mfma_f32_32x32x2_f32. Operand maps (gfx950): lane l supplies
// A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31]; D[row][col] lives in lane col=l&31,
// register r: row = (r&3) + 8*(r>>2) + 4*(l>>5). Taps are padded to an even
// count (slot s of parity hi = tap 2s+hi) so a k-pair never straddles channels.
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int drow(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

// off[b][j][p] = b_off[j] + Σ_{c,tap} w_off[j][c][tap] · x[b][c][p·s - pad + tap·dil]
// D[j (32)][pixel (32)] per wave; A = w_off rows, B = gathered x (coalesced along pixels).
template <int S>
__global__ __launch_bounds__(256) void offset_conv_fwd_mfma(Geo g, const float* __restrict__ x,
                                                           const float* __restrict__ w_off,
                                                           const float* __restrict__ b_off,
                                                           float* __restrict__ off) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hi = lane >> 5;
  const long Mtot = (long)g.B * g.HW;
  const long p = ((long)blockIdx.x * 4 + wave) * 32 + (lane & 31);
  if (((long)blockIdx.x * 4 + wave) * 32 >= Mtot) return;  // whole wave past the end
  const bool pok = p < Mtot;
  int b = 0, m = 0, ho = 0, wo = 0;
  if (pok) {
    b = (int)(p / g.HW);
    m = (int)(p - (long)b * g.HW);
    ho = m / g.Wo;
    wo = m - ho * g.Wo;
  }
  const int KK = g.kh * g.kw;
  int offs[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int tap = 2 * s + hi;
    offs[s] = -1;
    if (pok && tap < KK) {
      const int i = tap / g.kw, kx = tap - i * g.kw;
      const int y = ho * g.sh - g.ph + i * g.dh, xx = wo * g.sw - g.pw + kx * g.dw;
      if (y >= 0 && y < g.H && xx >= 0 && xx < g.W) offs[s] = y * g.W + xx;
    }
  }
  const int j0 = blockIdx.y * 32;
  const int ja = j0 + (lane & 31);
  const bool jok = ja < g.J;
  const float* wrow = w_off + (size_t)(jok ? ja : 0) * g.C * KK;
  const float* xb = x + (size_t)b * g.C * g.HWi;
  f32x16 acc = {0};
  for (int c = 0; c < g.C; ++c) {
    const float* xc = xb + (size_t)c * g.HWi;
    const float* wc = wrow + (size_t)c * KK;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int tap = 2 * s + hi;
      const float a = (jok && tap < KK) ? wc[tap] : 0.f;
      const float bv = offs[s] >= 0 ? xc[offs[s]] : 0.f;
      acc = mfma32(a, bv, acc);
    }
  }
  if (!pok) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = j0 + drow(r, hi);
    if (j < g.J) off[((size_t)b * g.J + j) * g.HW + m] = acc[r] + b_off[j];
  }
}

// ∂w_off[j][c][tap] += Σ_p ∂off[b][j][p] · x[b][c][p·s - pad + tap·dil]
// D[j (32)][(c,tap) (32)]; A = ∂off (pixel pair on k), B = gathered x.
__global__ __launch_bounds__(256) void offset_wgrad_mfma(Geo g, const float* __restrict__ x,
                                                         const float* __restrict__ goff,
                                                         float* __restrict__ gw, int ppw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hi = lane >> 5;
  const long Mtot = (long)g.B * g.HW;
  const long pstart = ((long)blockIdx.x * 4 + wave) * ppw;
  if (pstart >= Mtot) return;
  const long pend = min(pstart + (long)ppw, Mtot);
  const int KK = g.kh * g.kw;
  const int CKK = g.C * KK;
  const int kb = blockIdx.y * 32 + (lane & 31);
  const bool kok = kb < CKK;
  const int c = kok ? kb / KK : 0;
  const int tap = kok ? kb - c * KK : 0;
  const int ti = tap / g.kw, tx = tap - ti * g.kw;
  const int dyo = ti * g.dh - g.ph, dxo = tx * g.dw - g.pw;
  const int ja = blockIdx.z * 32 + (lane & 31);
  const bool jok = ja < g.J;
  // this lane's pixel = q + hi
  long p = pstart + hi;
  int b = (int)(p / g.HW);
  int m = (int)(p - (long)b * g.HW);
  int ho = m / g.Wo, wo = m - ho * g.Wo;
  f32x16 acc = {0};
  for (long q = pstart; q < pend; q += 2) {
    float a = 0.f, bv = 0.f;
    if (q + hi < pend) {
      const int mm = ho * g.Wo + wo;
      if (jok) a = goff[((size_t)b * g.J + ja) * g.HW + mm];
      const int y = ho * g.sh + dyo, xx = wo * g.sw + dxo;
      if (kok && y >= 0 && y < g.H && xx >= 0 && xx < g.W)
        bv = x[((size_t)b * g.C + c) * g.HWi + y * g.W + xx];
    }
    acc = mfma32(a, bv, acc);
    wo += 2;
    if (wo >= g.Wo) {
      wo -= g.Wo;
      if (++ho >= g.Ho) {
        ho = 0;
        ++b;
      }
    }
  }
  if (!kok) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = blockIdx.z * 32 + drow(r, hi);
    if (j < g.J) atomicAdd(gw + (size_t)j * CKK + kb, acc[r]);
  }
}

// ∂x[b][c][y][x] += Σ_{j,tap} w_off[j][c][tap] · ∂off[b][j][(y+pad-tap·dil)/s]
// D[c (32)][input pixel (32)]; A = w_off, B = gathered ∂off. RMW (tiles own their outputs).
template <int S>
__global__ __launch_bounds__(256) void offset_dgrad_mfma(Geo g, const float* __restrict__ w_off,
                                                         const float* __restrict__ goff,
                                                         float* __restrict__ gx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hi = lane >> 5;
  const long Mi = (long)g.B * g.HWi;
  const long tile0 = ((long)blockIdx.x * 4 + wave) * 32;
  if (tile0 >= Mi) return;
  const long p = tile0 + (lane & 31);
  const bool pok = p < Mi;
  int b = 0, yx = 0, y = 0, xx = 0;
  if (pok) {
    b = (int)(p / g.HWi);
    yx = (int)(p - (long)b * g.HWi);
    y = yx / g.W;
    xx = yx - y * g.W;
  }
  const int KK = g.kh * g.kw;
  int goffs[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int tap = 2 * s + hi;
    goffs[s] = -1;
    if (pok && tap < KK) {
      const int i = tap / g.kw, kx = tap - i * g.kw;
      const int t = y + g.ph - i * g.dh, u = xx + g.pw - kx * g.dw;
      if (t >= 0 && u >= 0 && t % g.sh == 0 && u % g.sw == 0) {
        const int ho = t / g.sh, wo = u / g.sw;
        if (ho < g.Ho && wo < g.Wo) goffs[s] = ho * g.Wo + wo;
      }
    }
  }
  const int ca = blockIdx.y * 32 + (lane & 31);
  const bool cok = ca < g.C;
  f32x16 acc = {0};
  const float* gb = goff + (size_t)b * g.J * g.HW;
  for (int j = 0; j < g.J; ++j) {
    const float* gj = gb + (size_t)j * g.HW;
    const float* wj = w_off + ((size_t)j * g.C + (cok ? ca : 0)) * KK;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int tap = 2 * s + hi;
      const float a = (cok && tap < KK) ? wj[tap] : 0.f;
      const float bv = goffs[s] >= 0 ? gj[goffs[s]] : 0.f;
      acc = mfma32(a, bv, acc);
    }
  }
  if (!pok) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = blockIdx.y * 32 + drow(r, hi);
    if (c < g.C) {
      float* q = gx + ((size_t)b * g.C + c) * g.HWi + yx;
      *q += acc[r];
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
                                  const float* b_off, float* off, float* /*wt_scratch*/,
                                  hipStream_t s) {
  const long Mtot = (long)g.B * g.HW;
  const long tiles = (Mtot + 31) / 32;
  dim3 grid((unsigned)((tiles + 3) / 4), (g.J + 31) / 32);
  DCN_S_DISPATCH(slots_for(g), hipLaunchKernelGGL(offset_conv_fwd_mfma<S>, grid, dim3(256), 0,
                                                  s, g, x, w_off, b_off, off));
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void channel_sum(const float* __restrict__ in, int B, int Cn,
                                                   int HW, float* __restrict__ out) {
  // out[ch] = Σ_{b,m} in[b][ch][m]; one block per channel, deterministic order.
  __shared__ float red[256];
  const int ch = blockIdx.x;
  float s = 0.f;
  for (int b = 0; b < B; ++b) {
    const float* p = in + ((size_t)b * Cn + ch) * HW;
    for (int m = threadIdx.x; m < HW; m += 256) s += p[m];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[ch] = red[0];
}

hipError_t launch_offset_conv_bwd(const Geo& g, const float* x, const float* w_off,
                                  const float* goff, float* gx, float* gw_off, float* gb_off,
                                  hipStream_t s) {
  const int KK = g.kh * g.kw;
  hipError_t e = hipMemsetAsync(gw_off, 0, (size_t)g.J * g.C * KK * sizeof(float), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(channel_sum, dim3(g.J), dim3(256), 0, s, goff, g.B, g.J, g.HW, gb_off);
  {
    const long Mtot = (long)g.B * g.HW;
    const int ppw = 2048;
    const long waves = (Mtot + ppw - 1) / ppw;
    dim3 grid((unsigned)((waves + 3) / 4), (g.C * KK + 31) / 32, (g.J + 31) / 32);
    hipLaunchKernelGGL(offset_wgrad_mfma, grid, dim3(256), 0, s, g, x, goff, gw_off, ppw);
  }
  {
    const long Mi = (long)g.B * g.HWi;
    const long tiles = (Mi + 31) / 32;
    dim3 grid((unsigned)((tiles + 3) / 4), (g.C + 31) / 32);
    DCN_S_DISPATCH(slots_for(g), hipLaunchKernelGGL(offset_dgrad_mfma<S>, grid, dim3(256), 0, s,
                                                    g, w_off, goff, gx));
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Bias (deform_conv.py:79-80) and reductions.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bias_add_kernel(float* __restrict__ out,
                                                       const float* __restrict__ bias, int O,
                                                       int HW, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int o = (int)((i / HW) % O);
    out[i] += bias[o];
  }
}

__global__ __launch_bounds__(256) void bias_add_vec4(float4* __restrict__ out,
                                                     const float* __restrict__ bias, int O,
                                                     int HW4, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float bv = bias[(int)((i / HW4) % O)];
    float4 v = out[i];
    v.x += bv;
    v.y += bv;
    v.z += bv;
    v.w += bv;
    out[i] = v;
  }
}

hipError_t launch_bias_add(const Geo& g, float* out, const float* bias, int b0, int nb,
                           hipStream_t s) {
  float* o = out + (size_t)b0 * g.O * g.HW;
  const long n = (long)nb * g.O * g.HW;
  if (g.HW % 4 == 0) {
    const long n4 = n / 4;
    const unsigned grid = (unsigned)min((n4 + 255) / 256, 8192L);
    hipLaunchKernelGGL(bias_add_vec4, dim3(grid), dim3(256), 0, s, reinterpret_cast<float4*>(o),
                       bias, g.O, g.HW / 4, n4);
  } else {
    const unsigned grid = (unsigned)min((n + 255) / 256, 8192L);
    hipLaunchKernelGGL(bias_add_kernel, dim3(grid), dim3(256), 0, s, o, bias, g.O, g.HW, n);
  }
  return hipGetLastError();
}

hipError_t launch_bias_grad(const Geo& g, const float* gout, float* gb, hipStream_t s) {
  hipLaunchKernelGGL(channel_sum, dim3(g.O), dim3(256), 0, s, gout, g.B, g.O, g.HW, gb);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ parts,
                                                           int nparts, size_t n,
                                                           float* __restrict__ dst) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float s = 0.f;
    for (int p = 0; p < nparts; ++p) s += parts[(size_t)p * n + i];
    dst[i] = s;
  }
}

hipError_t launch_sum_partials(const float* parts, int nparts, size_t n, float* dst,
                               hipStream_t s) {
  const unsigned grid = (unsigned)min((n + 255) / 256, (size_t)4096);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(grid), dim3(256), 0, s, parts, nparts, n, dst);
  return hipGetLastError();
}

}  // namespace dcn
