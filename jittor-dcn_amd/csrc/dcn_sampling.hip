// dcn_sampling.hip — the deformable bilinear sampling kernels of the hot path (gfx950):
//   K1  im2col_cl     columns colT[b][m][n*C + c]            (deform_conv.py:30-54, :62-73)
//   K5a offgrad_cl    ∂offset from ∂colT                     (autodiff of :37-38, :47-52)
//   K5b bins + dx_gather_cl  ∂x by deterministic gather     (autodiff of :41-52)
// plus the NCHW <-> NHWC transposes they need.
//
// Layout: channels-last ("CL"). x is transposed once to xT[b][r][q][c]; columns are
// stored row-per-pixel colT[b][m][k], k = n*C + c (the reference's own column order,
// deform_conv.py:72-73). A wave therefore handles a whole sample (one tap of one
// output pixel) at a time with its lanes on consecutive channels: every corner read
// and every column write is a contiguous 16-byte-per-lane run (1 KiB per wave
// instruction at C = 256); the per-sample coordinates are computed once and
// broadcast across the sample's lanes.
//
// ∂x without atomics: LDS float atomics (ds_add_f32) measured ~0.3 lanes/clk/CU on
// MI355X and global float atomics cap at ~1.3 TB/s, both far too slow for the
// 4·B·HW·N·C scatter. Instead each sample is binned by its top-left corner
// (a stable sort per image by bin, sample index breaking ties: K5b below), and each input
// pixel gathers the ∂col rows of the
// four bins whose 2x2 footprint covers it — a fixed summation order, so ∂x is bitwise
// reproducible.
#include <climits>
#include <cstdlib>
#include <type_traits>

#include <rocprim/block/block_radix_sort.hpp>

#include "dcn_device.h"

namespace dcn {

static int g_force_generic = 0;


void set_force_generic(int on) { g_force_generic = on; }
// 1 = the chunked three-kernel bins even where one block sort per segment applies (the
// parity tests compare the two bit for bit; dcn_debug_bins_chunked)
#ifndef BINS_CHUNKED
#define BINS_CHUNKED 0  // (an A/B build sets 1: tools/ab.sh)
#endif
static int g_bins_chunked = BINS_CHUNKED;
void set_bins_chunked(int on) { g_bins_chunked = on; }
int get_force_generic() { return g_force_generic; }

// ---------------------------------------------------------------------------
// Channel-lane mapping: a sample's Cg channels are covered by LP lanes, each
// owning VEC consecutive channels; SP = 64/LP samples share a wave instruction.
// ---------------------------------------------------------------------------
struct LaneMap {
  int CQ;  // channel units (of VEC channels) per group
  int LP;  // lanes per sample (power of two, <= 64)
  int SP;  // samples per wave step
};

static LaneMap lane_map(int Cg, int vec) {
  LaneMap L;
  L.CQ = (Cg + vec - 1) / vec;
  L.LP = 1;
  while (L.LP < L.CQ && L.LP < 64) L.LP <<= 1;
  L.SP = 64 / L.LP;
  return L;
}

template <int VEC>
struct Vec;
template <>
struct Vec<4> {
  typedef float4 T;
  __device__ static T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <>
struct Vec<1> {
  typedef float T;
  __device__ static T zero() { return 0.f; }
};

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T ldv(const float* p, bool ok) {
  if (!ok) return Vec<VEC>::zero();
  return *reinterpret_cast<const typename Vec<VEC>::T*>(p);
}
template <int VEC>
__device__ __forceinline__ void stv(float* p, typename Vec<VEC>::T v) {
  *reinterpret_cast<typename Vec<VEC>::T*>(p) = v;
}

template <typename T>
__device__ __forceinline__ float4 ld4_if(const T* p, bool ok) {
  return ok ? ld4(p) : make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float4 bilerp4(float fr, float fc, float4 a, float4 b, float4 c,
                                          float4 d) {
  return make_float4(bilerp(fr, fc, a.x, b.x, c.x, d.x), bilerp(fr, fc, a.y, b.y, c.y, d.y),
                     bilerp(fr, fc, a.z, b.z, c.z, d.z), bilerp(fr, fc, a.w, b.w, c.w, d.w));
}
__device__ __forceinline__ float bilerp4(float fr, float fc, float a, float b, float c, float d) {
  return bilerp(fr, fc, a, b, c, d);
}

// Per-sample state computed by lane i for sample s0 + i and broadcast with shfl.
struct SampleBcast {
  int r0, c0, m, n;
  float fr, fc;
  bool ok;
};

__device__ __forceinline__ SampleBcast bcast(const SampleBcast& v, int src) {
  SampleBcast o;
  o.r0 = __shfl(v.r0, src);
  o.c0 = __shfl(v.c0, src);
  o.m = __shfl(v.m, src);
  o.n = __shfl(v.n, src);
  o.fr = __shfl(v.fr, src);
  o.fc = __shfl(v.fc, src);
  o.ok = __shfl((int)v.ok, src) != 0;
  return o;
}

__device__ __forceinline__ SampleBcast lane_sample(const Geo& g, const float* off, int b, int gi,
                                                   int s, int NS) {
  SampleBcast v;
  v.ok = false;
  v.r0 = v.c0 = v.m = v.n = 0;
  v.fr = v.fc = 0.f;
  if (s < NS) {
    v.m = s / g.N;
    v.n = s - v.m * g.N;
    const Tap t = sample_tap(g, off, b, gi, v.n, v.m);
    v.ok = t.ok;
    v.r0 = t.r0;
    v.c0 = t.c0;
    v.fr = t.fr;
    v.fc = t.fc;
  }
  return v;
}

template <int VEC>
struct Corners {
  typename Vec<VEC>::T a, b, c, d;  // (r0,c0) (r0,c0+1) (r0+1,c0) (r0+1,c0+1)
};

template <int VEC>
__device__ __forceinline__ void load_corners(const float* __restrict__ xb, const SampleBcast& sm,
                                             const Geo& g, int c, Corners<VEC>& q) {
  const bool r0ok = sm.ok && sm.r0 >= 0, r1ok = sm.ok && sm.r0 + 1 < g.H;
  const bool c0ok = sm.c0 >= 0, c1ok = sm.c0 + 1 < g.W;
  const float* p00 = xb + ((long)sm.r0 * g.W + sm.c0) * (long)g.C + c;
  const long rs = (long)g.W * g.C;
  q.a = ldv<VEC>(p00, r0ok && c0ok);
  q.b = ldv<VEC>(p00 + g.C, r0ok && c1ok);
  q.c = ldv<VEC>(p00 + rs, r1ok && c0ok);
  q.d = ldv<VEC>(p00 + rs + g.C, r1ok && c1ok);
}

// Samples per software-pipelined batch: all of a batch's row loads are issued before
// the first one is consumed, so each wave keeps 4*U (K1) / 5*U (K5a) 1-KiB rows in flight.
constexpr int kU = 4;

// ---------------------------------------------------------------------------
// K1: colT[bl][m][n*C + gi*Cg + c] = bilinear(xT[b][.][.][gi*Cg + c]).
// One wave = 64 consecutive samples s = m*N + n of one image and group.
// ---------------------------------------------------------------------------
template <int VEC>
__global__ __launch_bounds__(256) void im2col_cl(Geo g, LaneMap L, const float* __restrict__ xT,
                                                 const float* __restrict__ off,
                                                 float* __restrict__ colT, int b0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Block3 blk = xcd_block();
  const int gi = blk.y, bl = blk.z, b = b0 + bl;
  const int NS = g.HW * g.N;
  const int s0 = (blk.x * 4 + wave) * 64;
  if (s0 >= NS) return;
  const SampleBcast mine = lane_sample(g, off, b, gi, s0 + lane, NS);
  const int sub = lane / L.LP, u0 = lane - sub * L.LP;
  const float* xb = xT + (size_t)b * g.HWi * g.C + (size_t)gi * g.Cg;
  float* cb = colT + (size_t)bl * g.HW * g.K + (size_t)gi * g.Cg;
  for (int it = 0; it < 64; it += kU * L.SP) {
    SampleBcast sm[kU];
    bool live[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int src = it + u * L.SP + sub;
      sm[u] = bcast(mine, src & 63);
      live[u] = src < 64 && s0 + src < NS;
    }
    for (int cu = u0; cu < L.CQ; cu += L.LP) {
      const int c = cu * VEC;
      Corners<VEC> q[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) load_corners<VEC>(xb, sm[u], g, c, q[u]);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (!live[u]) continue;
        const typename Vec<VEC>::T v = sm[u].ok ? bilerp4(sm[u].fr, sm[u].fc, q[u].a, q[u].b,
                                                          q[u].c, q[u].d)
                                                : Vec<VEC>::zero();
        stv<VEC>(cb + (size_t)sm[u].m * g.K + (size_t)sm[u].n * g.C + c, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K1 (LDS-staged): one block = one kTH x kTW tile of output pixels of one image.
// The block's samples (pixel-major, N taps each) are resolved once into LDS records;
// then, per 64-channel slice, the xT window the tile's samples land in — the tile's
// zero-offset footprint plus a MAR-pixel margin, zero outside the image — is staged in
// LDS with coalesced 256-B row reads, and every sample's four corners come from LDS.
// A sample whose corners leave the window (|offset| beyond the margin) reads them from
// global memory instead; both paths compute the same canonical bilerp, so the columns
// are bit-identical to im2col_cl's. Used for deform_groups == 1, N <= kMaxTaps,
// C % 4 == 0 (the reference's own configuration space).
// ---------------------------------------------------------------------------
constexpr int kMaxTaps = 9;
constexpr int kSkip = INT_MIN, kZero = INT_MIN + 1;  // record r0 markers

template <int TH, int TW, int MAR>
struct Win {
  static constexpr int R = TW + 2 * MAR;  // window rows (input r follows output w, Q1)
  static constexpr int Q = TH + 2 * MAR;  // window cols (input q follows output h)
  static constexpr int PIX = R * Q;
};

// xT element type XT: float, or bf16 (DCN_BF16: the channels-last copy of the bf16 input,
// half the window bytes; staged into LDS as fp32, so the arithmetic is unchanged)
// LDS image of 4 channels of the xT window: float4 for fp32, the raw 8 bytes for bf16 (half
// the LDS per block, twice the blocks per CU: the bf16 K1 was LDS-occupancy bound)
template <typename XT>
struct WinT;
template <>
struct WinT<float> {
  typedef float4 T;
  __device__ static T raw(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ static T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ static float4 f(T v) { return v; }
};
template <>
struct WinT<bf16_t> {
  typedef uint2 T;
  __device__ static T raw(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
  __device__ static T zero() { return make_uint2(0u, 0u); }
  __device__ static float4 f(T u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
};

template <int TH, int TW, int MAR, int CS, bool NT, typename OT = float, typename XT = float>
__global__ __launch_bounds__(256) void im2col_lds(Geo g, const XT* __restrict__ xT,
                                                  const float* __restrict__ off,
                                                  OT* __restrict__ colT, int b0, int tw_n) {
  typedef Win<TH, TW, MAR> Wn;
  constexpr int kTP = TH * TW;
  constexpr int LPS = CS / 4, GS = 256 / LPS;  // lanes per sample, samples per block step
  typedef WinT<XT> WT;
  __shared__ typename WT::T win[Wn::PIX * LPS];
  __shared__ int4 rec[kTP * kMaxTaps];
  const int tid = threadIdx.x;
  const Block3 blk = xcd_block();
  const int bl = blk.z, b = b0 + bl;
  const int th_i = blk.x / tw_n, tw_i = blk.x - th_i * tw_n;
  const int h0 = th_i * TH, w0 = tw_i * TW;
  // window origin: the tile's zero-offset footprint (grid_sample scale (H-1)/(Wo-1))
  const int rlo = (int)floorf((float)w0 * (float)(g.H - 1) / (float)(g.Wo - 1)) - MAR;
  const int qlo = (int)floorf((float)h0 * (float)(g.W - 1) / (float)(g.Ho - 1)) - MAR;
  const int NSB = kTP * g.N;
  for (int sidx = tid; sidx < NSB; sidx += 256) {
    const int p = sidx / g.N, n = sidx - p * g.N;
    const int h = h0 + p / TW, w = w0 + p % TW;
    int4 r = make_int4(kSkip, 0, 0, 0);
    if (h < g.Ho && w < g.Wo) {
      const Tap t = sample_tap(g, off, b, 0, n, h * g.Wo + w);
      r = t.ok ? make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc))
               : make_int4(kZero, 0, 0, 0);
    }
    rec[sidx] = r;
  }
  const XT* xb = xT + (size_t)b * g.HWi * g.C;
  OT* cb = colT + (size_t)bl * g.HW * g.K;
  const int grp = tid / LPS, cl = tid % LPS;  // GS sample groups of LPS lanes
  for (int cs = 0; cs < g.C; cs += CS) {
    const int c = cs + cl * 4;
    const bool cok = c < g.C;
    __syncthreads();  // records ready / previous slice consumed
    {
      constexpr int TOT = Wn::PIX * LPS, IT = (TOT + 255) / 256;
      typename WT::T v[IT];
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int idx = tid + k * 256;
        const int pix = idx / LPS, l = idx % LPS;
        const int rr = pix / Wn::Q, qq = pix - rr * Wn::Q;
        const int r = rlo + rr, q = qlo + qq, cc = cs + l * 4;
        const bool ok = idx < TOT && r >= 0 && r < g.H && q >= 0 && q < g.W && cc < g.C;
        v[k] = ok ? WT::raw(xb + ((size_t)r * g.W + q) * g.C + cc) : WT::zero();
      }
#pragma unroll
      for (int k = 0; k < IT; ++k)
        if (tid + k * 256 < TOT) win[tid + k * 256] = v[k];
    }
    __syncthreads();
    for (int s = grp; s < NSB; s += GS) {
      const int4 r = rec[s];
      if (r.x == kSkip) continue;
      const int p = s / g.N, n = s - p * g.N;
      const int m = (h0 + p / TW) * g.Wo + w0 + p % TW;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r.x != kZero) {
        const float fr = __int_as_float(r.z), fc = __int_as_float(r.w);
        const int rr = r.x - rlo, qq = r.y - qlo;
        float4 a, bq, cq, d;
        if (rr >= 0 && rr + 1 < Wn::R && qq >= 0 && qq + 1 < Wn::Q) {
          const typename WT::T* w4 = win + (rr * Wn::Q + qq) * LPS + cl;
          a = WT::f(w4[0]);
          bq = WT::f(w4[LPS]);
          cq = WT::f(w4[Wn::Q * LPS]);
          d = WT::f(w4[(Wn::Q + 1) * LPS]);
        } else {  // outside the staged window: global corner reads
          const bool r0ok = r.x >= 0, r1ok = r.x + 1 < g.H, c0ok = r.y >= 0, c1ok = r.y + 1 < g.W;
          const XT* p00 = xb + ((long)r.x * g.W + r.y) * (long)g.C + c;
          const long rs = (long)g.W * g.C;
          a = ld4_if(p00, cok && r0ok && c0ok);
          bq = ld4_if(p00 + g.C, cok && r0ok && c1ok);
          cq = ld4_if(p00 + rs, cok && r1ok && c0ok);
          d = ld4_if(p00 + rs + g.C, cok && r1ok && c1ok);
        }
        o = bilerp4(fr, fc, a, bq, cq, d);
      }
      if (cok) st4<NT>(cb + (size_t)m * g.K + (size_t)n * g.C + c, o);
    }
  }
}

// K1 for bf16 x and columns with 8 channels per lane: a sample's 512-B column row (C = 256)
// is one half-wave's 16-B-per-lane store, so a wave instruction writes two samples (1 KiB)
// and gathers its corners with 16-B LDS reads. The 4-channel form moved 8 B per lane and ran
// at the fp32 kernel's samples/s (r02 config 4: 0.087 ms, 0.37 of HBM). Same window, records
// and arithmetic (canonical bilerp per channel, one rounding to bf16): the same column bits.
__device__ __forceinline__ void bf8_unpack(uint4 u, float4& lo, float4& hi) {
  lo = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  hi = make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                   __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u));
}
__device__ __forceinline__ uint4 ld8_if(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}

template <int TH, int TW, int MAR, int CS, bool NT = true>
__global__ __launch_bounds__(256) void im2col_lds_b8(Geo g, const bf16_t* __restrict__ xT,
                                                     const float* __restrict__ off,
                                                     bf16_t* __restrict__ colT, int b0, int tw_n) {
  typedef Win<TH, TW, MAR> Wn;
  constexpr int kTP = TH * TW;
  constexpr int LPW = CS / 4;                // window slots (4 channels, 8 B) per pixel
  constexpr int LPS = CS / 8, GS = 256 / LPS;  // lanes per sample, samples per block step
  __shared__ uint2 win[Wn::PIX * LPW];
  __shared__ int4 rec[kTP * kMaxTaps];
  const int tid = threadIdx.x;
  const Block3 blk = xcd_block();
  const int bl = blk.z, b = b0 + bl;
  const int th_i = blk.x / tw_n, tw_i = blk.x - th_i * tw_n;
  const int h0 = th_i * TH, w0 = tw_i * TW;
  const int rlo = (int)floorf((float)w0 * (float)(g.H - 1) / (float)(g.Wo - 1)) - MAR;
  const int qlo = (int)floorf((float)h0 * (float)(g.W - 1) / (float)(g.Ho - 1)) - MAR;
  const int NSB = kTP * g.N;
  for (int sidx = tid; sidx < NSB; sidx += 256) {
    const int p = sidx / g.N, n = sidx - p * g.N;
    const int h = h0 + p / TW, w = w0 + p % TW;
    int4 r = make_int4(kSkip, 0, 0, 0);
    if (h < g.Ho && w < g.Wo) {
      const Tap t = sample_tap(g, off, b, 0, n, h * g.Wo + w);
      r = t.ok ? make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc))
               : make_int4(kZero, 0, 0, 0);
    }
    rec[sidx] = r;
  }
  const bf16_t* xb = xT + (size_t)b * g.HWi * g.C;
  bf16_t* cb = colT + (size_t)bl * g.HW * g.K;
  const int grp = tid / LPS, cl = tid % LPS;
  for (int cs = 0; cs < g.C; cs += CS) {
    const int c = cs + cl * 8;
    const bool cok = c < g.C;  // C % 8 == 0: whole 8-channel runs
    __syncthreads();  // records ready / previous slice consumed
    {
      constexpr int TOT = Wn::PIX * LPW, IT = (TOT + 255) / 256;
      uint2 v[IT];
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int idx = tid + k * 256;
        const int pix = idx / LPW, l = idx % LPW;
        const int rr = pix / Wn::Q, qq = pix - rr * Wn::Q;
        const int r = rlo + rr, q = qlo + qq, cc = cs + l * 4;
        const bool ok = idx < TOT && r >= 0 && r < g.H && q >= 0 && q < g.W && cc < g.C;
        v[k] = ok ? *reinterpret_cast<const uint2*>(xb + ((size_t)r * g.W + q) * g.C + cc)
                  : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int k = 0; k < IT; ++k)
        if (tid + k * 256 < TOT) win[tid + k * 256] = v[k];
    }
    __syncthreads();
    for (int s = grp; s < NSB; s += GS) {
      const int4 r = rec[s];
      if (r.x == kSkip) continue;
      const int p = s / g.N, n = s - p * g.N;
      const int m = (h0 + p / TW) * g.Wo + w0 + p % TW;
      uint4 o = make_uint4(0u, 0u, 0u, 0u);
      if (r.x != kZero) {
        const float fr = __int_as_float(r.z), fc = __int_as_float(r.w);
        const int rr = r.x - rlo, qq = r.y - qlo;
        uint4 ua, ub, uc, ud;
        if (rr >= 0 && rr + 1 < Wn::R && qq >= 0 && qq + 1 < Wn::Q) {
          const uint4* w8 = reinterpret_cast<const uint4*>(win + (rr * Wn::Q + qq) * LPW) + cl;
          ua = w8[0];
          ub = w8[LPW / 2];
          uc = w8[Wn::Q * LPW / 2];
          ud = w8[(Wn::Q + 1) * LPW / 2];
        } else {  // outside the staged window: global corner reads
          const bool r0ok = r.x >= 0, r1ok = r.x + 1 < g.H, c0ok = r.y >= 0, c1ok = r.y + 1 < g.W;
          const bf16_t* p00 = xb + ((long)r.x * g.W + r.y) * (long)g.C + c;
          const long rs = (long)g.W * g.C;
          ua = ld8_if(p00, cok && r0ok && c0ok);
          ub = ld8_if(p00 + g.C, cok && r0ok && c1ok);
          uc = ld8_if(p00 + rs, cok && r1ok && c0ok);
          ud = ld8_if(p00 + rs + g.C, cok && r1ok && c1ok);
        }
        float4 a0, a1, b0v, b1v, c0v, c1v, d0, d1;
        bf8_unpack(ua, a0, a1);
        bf8_unpack(ub, b0v, b1v);
        bf8_unpack(uc, c0v, c1v);
        bf8_unpack(ud, d0, d1);
        const float4 lo = bilerp4(fr, fc, a0, b0v, c0v, d0), hi = bilerp4(fr, fc, a1, b1v, c1v, d1);
        o = make_uint4((unsigned)f2bf(lo.x) | ((unsigned)f2bf(lo.y) << 16),
                       (unsigned)f2bf(lo.z) | ((unsigned)f2bf(lo.w) << 16),
                       (unsigned)f2bf(hi.x) | ((unsigned)f2bf(hi.y) << 16),
                       (unsigned)f2bf(hi.z) | ((unsigned)f2bf(hi.w) << 16));
      }
      if (cok) {
        unsigned* dst = reinterpret_cast<unsigned*>(cb + (size_t)m * g.K + (size_t)n * g.C + c);
        if constexpr (NT) {
          __builtin_nontemporal_store(o.x, dst);
          __builtin_nontemporal_store(o.y, dst + 1);
          __builtin_nontemporal_store(o.z, dst + 2);
          __builtin_nontemporal_store(o.w, dst + 3);
        } else {
          *reinterpret_cast<uint4*>(dst) = o;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K5a: ∂off for every sample from its ∂colT row and the four xT corner rows.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void acc_dgrad(float fr, float fc, float gv, float a, float b, float c,
                                          float d, float& diy, float& dix) {
  diy = fmaf(gv, dbilerp_row(fc, a, b, c, d), diy);
  dix = fmaf(gv, dbilerp_col(fr, a, b, c, d), dix);
}
__device__ __forceinline__ void acc_dgrad(float fr, float fc, float4 gv, float4 a, float4 b,
                                          float4 c, float4 d, float& diy, float& dix) {
  acc_dgrad(fr, fc, gv.x, a.x, b.x, c.x, d.x, diy, dix);
  acc_dgrad(fr, fc, gv.y, a.y, b.y, c.y, d.y, diy, dix);
  acc_dgrad(fr, fc, gv.z, a.z, b.z, c.z, d.z, diy, dix);
  acc_dgrad(fr, fc, gv.w, a.w, b.w, c.w, d.w, diy, dix);
}

template <int VEC>
__global__ __launch_bounds__(256) void offgrad_cl(Geo g, LaneMap L, const float* __restrict__ xT,
                                                  const float* __restrict__ off,
                                                  const float* __restrict__ gcolT,
                                                  float* __restrict__ goff, int b0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Block3 blk = xcd_block();
  const int gi = blk.y, bl = blk.z, b = b0 + bl;
  const int NS = g.HW * g.N;
  const int s0 = (blk.x * 4 + wave) * 64;
  if (s0 >= NS) return;
  const SampleBcast mine = lane_sample(g, off, b, gi, s0 + lane, NS);
  const int sub = lane / L.LP, u0 = lane - sub * L.LP;
  const float* xb = xT + (size_t)b * g.HWi * g.C + (size_t)gi * g.Cg;
  const float* gb = gcolT + (size_t)bl * g.HW * g.K + (size_t)gi * g.Cg;
  float* gob = goff + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  const float sy = (float)(g.H - 1) / (float)(g.Wo - 1);
  const float sx = (float)(g.W - 1) / (float)(g.Ho - 1);
  for (int it = 0; it < 64; it += kU * L.SP) {
    SampleBcast sm[kU];
    bool live[kU];
    float diy[kU], dix[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int src = it + u * L.SP + sub;
      sm[u] = bcast(mine, src & 63);
      live[u] = src < 64 && s0 + src < NS;
      diy[u] = dix[u] = 0.f;
    }
    for (int cu = u0; cu < L.CQ; cu += L.LP) {
      const int c = cu * VEC;
      Corners<VEC> q[kU];
      typename Vec<VEC>::T gv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        gv[u] = ldv<VEC>(gb + (size_t)sm[u].m * g.K + (size_t)sm[u].n * g.C + c,
                         live[u] && sm[u].ok);
        load_corners<VEC>(xb, sm[u], g, c, q[u]);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (sm[u].ok)
          acc_dgrad(sm[u].fr, sm[u].fc, gv[u], q[u].a, q[u].b, q[u].c, q[u].d, diy[u], dix[u]);
    }
    // reduce over the LP lanes of each sample (fixed tree: deterministic)
#pragma unroll
    for (int u = 0; u < kU; ++u)
      for (int o = L.LP >> 1; o > 0; o >>= 1) {
        diy[u] += __shfl_xor(diy[u], o);
        dix[u] += __shfl_xor(dix[u], o);
      }
    if (u0 == 0) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (!live[u]) continue;
        gob[(size_t)sm[u].n * g.HW + sm[u].m] = diy[u] * sy;
        gob[(size_t)(g.N + sm[u].n) * g.HW + sm[u].m] = dix[u] * sx;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K5b: sample bins. Bin of a valid sample = its top-left corner (r0, c0) in
// [-1, H-1] x [-1, W-1] -> (r0+1)*(W+1) + (c0+1); NB = (H+1)*(W+1) bins per segment
// (image, group). Within a bin the samples are ordered by sample index s = m*N + n (that
// order fixes K5's summation order, so ∂x and ∂offset are bitwise reproducible).
//
// Three kernels, no atomics (r03; r02's count / scan / fill / rank took ~0.98 ms per
// config-3 step on the side stream, 0.60 of it in the rank loop):
//   bins_chunk_sort  a segment's samples in chunks of kBinChunk: each chunk's bins are
//                    computed from the offsets and sorted in LDS (rocprim block radix sort,
//                    stable, so equal bins keep ascending s); the chunk's sorted entries
//                    {bin, index, fr, fc} are written, and per bin present its run length
//                    H[seg][chunk][bin] and run start R[seg][chunk][bin];
//   bins_scan_table  one workgroup per segment: H becomes each (chunk, bin) run's first
//                    position in the segment's bin order (bin-major, chunk-minor), start[bin]
//                    each bin's first position; every access a coalesced 16-B one;
//   bins_emit        one thread per bin copies the bin's runs, chunk by chunk, to its output
//                    range: the packed records of the fused K5 (brec) or the sorted sample
//                    lists (slist), written in output order.
// ---------------------------------------------------------------------------
constexpr int kBinT = 256, kBinIPT = 16, kBinChunk = kBinT * kBinIPT;
constexpr int kBinLBits = 12;  // sample index within a chunk (< 4096) in a packed entry
static_assert(kBinChunk == 1 << kBinLBits, "packed entry layout");

// H / R row length: NB bins plus the sentinel NB (whose start is the end of the last bin),
// padded to a multiple of 4 for the 16-B accesses of bins_scan_table
__host__ __device__ __forceinline__ int bins_nbp(int NB) { return (NB + 1 + 3) / 4 * 4; }

__device__ __forceinline__ unsigned sample_bin(const Geo& g, const float* __restrict__ off, int b,
                                               int gi, int s, int NB, Tap* tp) {
  const Tap t = sample_tap(g, off, b, gi, s % g.N, s / g.N);
  if (tp) *tp = t;
  return t.ok ? (unsigned)((t.r0 + 1) * (g.W + 1) + (t.c0 + 1)) : (unsigned)NB;
}

__global__ __launch_bounds__(kBinT) void bins_chunk_sort(Geo g, const float* __restrict__ off,
                                                         int b0, int nch, int NB, unsigned kbits,
                                                         int* __restrict__ H, int* __restrict__ R,
                                                         uint4* __restrict__ sorted,
                                                         float4* __restrict__ rec) {
  using Sort = rocprim::block_radix_sort<unsigned, kBinT, kBinIPT, unsigned short>;
  __shared__ typename Sort::storage_type sst;
  __shared__ unsigned skey[kBinChunk];
  __shared__ float2 frfc[kBinChunk];
  const int tid = threadIdx.x, ch = blockIdx.x, bg = blockIdx.y;
  const int NS = g.HW * g.N, gi = bg % g.G, b = b0 + bg / g.G;
  unsigned key[kBinIPT];
  unsigned short val[kBinIPT];
#pragma unroll
  for (int u = 0; u < kBinIPT; ++u) {
    const int l = tid * kBinIPT + u, s = ch * kBinChunk + l;
    val[u] = (unsigned short)l;
    Tap t;
    t.ok = false;
    t.fr = t.fc = 0.f;
    key[u] = s < NS ? sample_bin(g, off, b, gi, s, NB, &t)
                    : (unsigned)NB + 1;  // past the end: after every bin and the invalid samples
    frfc[l] = make_float2(t.fr, t.fc);
    if (rec && s < NS)  // dx_gather_cl's per-sample records (the unfused K5 only)
      rec[(size_t)bg * NS + s] = make_float4(__int_as_float(t.ok ? (int)key[u] : -1), t.fr, t.fc, 0.f);
  }
  Sort().sort(key, val, sst, 0, kbits);  // blocked result: thread t holds ranks t*IPT + u
  uint4* out = sorted + ((size_t)bg * nch + ch) * kBinChunk;
#pragma unroll
  for (int u = 0; u < kBinIPT; ++u) skey[tid * kBinIPT + u] = key[u];
  __syncthreads();  // skey complete; frfc was complete before the sort's own barriers
#pragma unroll
  for (int u = 0; u < kBinIPT; ++u) {
    const float2 f = frfc[val[u]];
    out[tid * kBinIPT + u] =
        make_uint4((key[u] << kBinLBits) | val[u], __float_as_uint(f.x), __float_as_uint(f.y), 0u);
  }
  // run lengths and starts: the thread holding a run's first entry counts it (runs are short)
  const size_t row = ((size_t)bg * nch + ch) * bins_nbp(NB);
#pragma unroll
  for (int u = 0; u < kBinIPT; ++u) {
    const int i = tid * kBinIPT + u;
    const unsigned k = key[u];
    if (k < (unsigned)NB && (i == 0 || skey[i - 1] != k)) {
      int c = 1;
      while (i + c < kBinChunk && skey[i + c] == k) ++c;
      H[row + k] = c;
      R[row + k] = i;
    }
  }
}

// One workgroup per segment: the (chunk, bin) runs in bin-major order get their first
// positions in the segment's bin order. H is chunk-major ([chunk][bin], bins padded to a
// multiple of 4), so thread t owns bins 4t..4t+3 and every access is a coalesced 16-B one:
// pass 1 sums each bin over the chunks, a block scan over the bins gives start[bin], pass 2
// replaces H[c][bin] by start[bin] + the runs of the earlier chunks. Bins beyond 4096 are
// handled in rounds, carrying the running total.
// (r05: the block size is a template parameter; BINS_SCAN_T picks it: a smaller block fits
// beside the ∂W GEMM workgroups it runs next to on the side stream)
#ifndef BINS_SCAN_T
#define BINS_SCAN_T 1024
#endif
template <int T = 1024>
__global__ __launch_bounds__(T) void bins_scan_table(int NB, int nch, int* __restrict__ H,
                                                     int* __restrict__ start) {
  constexpr int NW = T / 64;
  __shared__ int wsum[NW + 1];  // exclusive wave prefixes, then the block total
  const int bg = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int NBp = bins_nbp(NB);
  int* Hs = H + (size_t)bg * nch * NBp;
  int* st = start + (size_t)bg * (NB + 1);
  int carry = 0;
  for (int b0 = 0; b0 < NBp; b0 += 4 * T) {
    const int bb = b0 + 4 * tid;
    const bool act = bb < NBp;
    int4 tot = make_int4(0, 0, 0, 0);
    if (act) {
#pragma unroll 8
      for (int c = 0; c < nch; ++c) {
        const int4 v = *reinterpret_cast<const int4*>(Hs + (size_t)c * NBp + bb);
        tot.x += v.x; tot.y += v.y; tot.z += v.z; tot.w += v.w;
      }
    }
    const int local = tot.x + tot.y + tot.z + tot.w;
    int v = local;  // inclusive scan over the block
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int i = 0; i < NW; ++i) {
        const int t = wsum[i];
        wsum[i] = acc;
        acc += t;
      }
      wsum[NW] = acc;
    }
    __syncthreads();
    const int e = carry + v - local + wsum[wv];
    carry += wsum[NW];
    int run[4] = {e, e + tot.x, e + tot.x + tot.y, e + tot.x + tot.y + tot.z};
    if (act) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (bb + i <= NB) st[bb + i] = run[i];
#pragma unroll 8
      for (int c = 0; c < nch; ++c) {
        int4* p = reinterpret_cast<int4*>(Hs + (size_t)c * NBp + bb);
        const int4 hv = *p;
        *p = make_int4(run[0], run[1], run[2], run[3]);
        run[0] += hv.x; run[1] += hv.y; run[2] += hv.z; run[3] += hv.w;
      }
    }
    __syncthreads();
  }
}

// One thread per bin: its runs (chunk by chunk, each already in ascending s) go to the bin's
// output range in order; a run's length is the next chunk's first position minus its own.
// brec (fused K5): {∂colT row offset m*K + n*C, fr, fc, ∂offset index n*HW + m}; else
// slist (dx_gather_cl): the sample index.
__global__ __launch_bounds__(256) void bins_emit(Geo g, int nch, int NB,
                                                 const int* __restrict__ H,
                                                 const int* __restrict__ R,
                                                 const int* __restrict__ start,
                                                 const uint4* __restrict__ sorted,
                                                 int4* __restrict__ brec,
                                                 int* __restrict__ slist) {
  const int bin = blockIdx.x * 256 + threadIdx.x, bg = blockIdx.y;
  if (bin >= NB) return;
  const int NS = g.HW * g.N, NBp = bins_nbp(NB);
  const int* Hs = H + (size_t)bg * nch * NBp + bin;
  const int* Rs = R + (size_t)bg * nch * NBp + bin;
  const uint4* so = sorted + (size_t)bg * nch * kBinChunk;
  const int* stb = start + (size_t)bg * (NB + 1);
  auto copy_run = [&](int c, int pos, int n, int r) {
    const uint4* src = so + (size_t)c * kBinChunk + r;
    for (int j = 0; j < n; ++j) {
      const uint4 e = src[j];
      const int s = c * kBinChunk + (int)(e.x & (kBinChunk - 1));
      const size_t o = (size_t)bg * NS + pos + j;
      if (brec) {
        const int m = s / g.N, tap = s - m * g.N;
        brec[o] = make_int4(m * g.K + tap * g.C, (int)e.y, (int)e.z, tap * g.HW + m);
      } else {
        slist[o] = s;
      }
    }
  };
  constexpr int kPre = 8;  // chunks whose run positions / starts are loaded up front
  if (nch <= kPre) {
    int hb[kPre + 1], rr[kPre];
#pragma unroll
    for (int c = 0; c < kPre; ++c) {
      hb[c] = c < nch ? Hs[(size_t)c * NBp] : 0;
      rr[c] = c < nch ? Rs[(size_t)c * NBp] : 0;
    }
    hb[kPre] = stb[bin + 1];
#pragma unroll
    for (int c = 0; c < kPre; ++c) {
      if (c >= nch) break;
      const int next = c + 1 < nch ? hb[c + 1] : hb[kPre];
      if (next > hb[c]) copy_run(c, hb[c], next - hb[c], rr[c]);
    }
    return;
  }
  int pos = Hs[0];
  for (int c = 0; c < nch; ++c) {
    const int next = c + 1 < nch ? Hs[(size_t)(c + 1) * NBp] : stb[bin + 1];
    if (next > pos) copy_run(c, pos, next - pos, Rs[(size_t)c * NBp]);
    pos = next;
  }
}

// One workgroup per segment when the segment's samples fit one block sort (NS <= 8192:
// config 4's 7,056 per image), for the fused K5 only: the same stable radix sort on the bin
// key (ascending sample index within a bin) over the whole segment at once, then each
// thread writes the packed records of its sorted positions and the bin starts its key
// boundaries open. One launch replaces chunk sort + scan table + emit (r04: 127 µs of
// side-stream kernels per config-4 step, running beside the ∂W / ∂col products and taking
// their CUs), no H / R / sorted scratch, and the records are the same bits in the same order.
constexpr int kBsT = 1024, kBsIPT = 8, kBsMax = kBsT * kBsIPT;
__global__ __launch_bounds__(kBsT) void bins_sort_seg(Geo g, const float* __restrict__ off, int b0,
                                                      int NB, unsigned kbits,
                                                      int* __restrict__ start,
                                                      int4* __restrict__ brec,
                                                      float* __restrict__ goff) {
  using Sort = rocprim::block_radix_sort<unsigned, kBsT, kBsIPT, unsigned short>;
  __shared__ typename Sort::storage_type sst;
  __shared__ unsigned lastk[kBsT];
  // the segment's offsets ([2N][HW] fp32 <= 64 KiB, since HW·N <= kBsMax), staged with
  // coalesced loads: every sample's (Δx, Δy) is then an LDS read (a sample's two planes are
  // HW apart, so read from global they were 4-B gathers, one line per lane)
  __shared__ __attribute__((aligned(16))) float offL[2 * kBsMax];
  const int tid = threadIdx.x, bg = blockIdx.x;
  const int NS = g.HW * g.N, gi = bg % g.G, b = b0 + bg / g.G;
  {
    const float* ob = off + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
    const int n = 2 * g.N * g.HW;
    if ((g.HW & 3) == 0 && ((reinterpret_cast<uintptr_t>(ob) & 15) == 0)) {
      for (int i = tid; i < n / 4; i += kBsT)
        reinterpret_cast<float4*>(offL)[i] = reinterpret_cast<const float4*>(ob)[i];
    } else {
      for (int i = tid; i < n; i += kBsT) offL[i] = ob[i];
    }
  }
  __syncthreads();
  // the segment's sample taps from the staged offsets (sample_tap's arithmetic: same bits)
  auto tap_of = [&](int n, int m) {
    const int h = m / g.Wo, w = m - h * g.Wo;
    float iy, ix;
    ref_coord(h, w, offL[n * g.HW + m], offL[(g.N + n) * g.HW + m], g, iy, ix);
    return make_tap(iy, ix, g);
  };
  unsigned key[kBsIPT];
  unsigned short val[kBsIPT];
#pragma unroll
  for (int u = 0; u < kBsIPT; ++u) {
    const int s = tid * kBsIPT + u;  // blocked: input order = sample order
    val[u] = (unsigned short)s;
    key[u] = (unsigned)NB + 1;
    if (s < NS) {  // sample_bin's key
      const Tap t = tap_of(s % g.N, s / g.N);
      key[u] = t.ok ? (unsigned)((t.r0 + 1) * (g.W + 1) + (t.c0 + 1)) : (unsigned)NB;
    }
  }
  Sort().sort(key, val, sst, 0, kbits);  // stable; thread t now holds ranks t*IPT + u
  lastk[tid] = key[kBsIPT - 1];
  __syncthreads();
  int* st = start + (size_t)bg * (NB + 1);
  int4* out = brec + (size_t)bg * NS;
  unsigned prev = tid > 0 ? lastk[tid - 1] : ~0u;  // ~0u: before bin 0
#pragma unroll
  for (int u = 0; u < kBsIPT; ++u) {
    const int pos = tid * kBsIPT + u;
    const unsigned k = key[u];
    // bins (prev, k] (clamped to the sentinel NB) start at this position
    if (k != prev) {
      const int lo = prev == ~0u ? 0 : (int)prev + 1, hi = min((int)k, NB);
      for (int bn = lo; bn <= hi; ++bn) st[bn] = pos;
    }
    if (k == (unsigned)NB) {  // in no bin (every corner outside): K5 never sees it, ∂offset 0
      const int s = val[u], m = s / g.N, tap = s - m * g.N;
      float* gob = goff + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
      gob[(size_t)tap * g.HW + m] = 0.f;
      gob[(size_t)(g.N + tap) * g.HW + m] = 0.f;
    }
    if (k < (unsigned)NB) {
      const int s = val[u], m = s / g.N, tap = s - m * g.N;
      const Tap t = tap_of(tap, m);
      out[pos] = make_int4(m * g.K + tap * g.C, __float_as_int(t.fr), __float_as_int(t.fc),
                           tap * g.HW + m);
    }
    prev = k;
  }
  // every key below the sentinel: the bins after the last one end at the segment's end
  if (tid == kBsT - 1 && key[kBsIPT - 1] < (unsigned)NB)
    for (int bn = (int)key[kBsIPT - 1] + 1; bn <= NB; ++bn) st[bn] = kBsMax;
}

// ---------------------------------------------------------------------------
// K5 fused (∂x + ∂offset from ONE pass over the binned ∂col rows).
// One block = a kTR x kTQ tile (template parameters) of INPUT pixels of one image and kTR+1 waves. Bin
// (br, bc) holds the samples whose top-left corner is (br-1, bc-1) (K5b); wave w walks
// bin row br = R0+w (bin columns Q0..Q0+kTQ-1, and W too in the last column of tiles;
// samples in sorted order), reading each ∂colT row once, and accumulates into the two pixel
// rows that bin row touches: r0 (tile row w-1, weight 1-fr) and r0+1 (tile row w, weight
// fr). The bin loop is unrolled, so accumulator indices are static (registers). Tile row t
// is then wave t's lower row + wave t+1's upper row, combined through LDS in that fixed
// order. Bin column Q0 also feeds pixel column Q0-1, the left tile's last one: that share
// is written as boundary partials as soon as the column is done (cpart[b][r][tile
// column][lower, upper][C]: wave w's two rows, so no registers stay held for them), which
// col2im_fold adds to the left tile's ∂xT afterwards. No bin column is read by two tiles
// (r02 read the shared column from both sides: (kTQ+1)/kTQ of the ∂col rows).
// ∂offset of a sample is computed once, by the block that reads its bin (bin row R0 is
// read by two tiles: the lower one, w >= 1, owns it), from the tile's (kTR+1) x (kTQ+1)
// xT window (rows R0..R0+kTR, columns Q0-1..Q0+kTQ-1) staged in LDS (corners outside the
// image: zero). ∂offset uses offgrad_cl's op order (per-lane channel sums, then wave_sum's
// fixed xor tree, taken for the 2U sums of a batch at once by wave_sum8). Used for deform_groups == 1, C % 4 == 0, C <= 256.
// ---------------------------------------------------------------------------

// Packed fp32 (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32: two lanes' elements per
// instruction): each element's operation is the scalar one, so the results are the same bits.
// K5 is bound by VALU issue (r03 PMC at config 3: 202 M VALU instructions, ≈112 per sample),
// so halving the elementwise ones is its lever.
__device__ __forceinline__ f32x2 lo2(float4 v) { return f32x2{v.x, v.y}; }
__device__ __forceinline__ f32x2 hi2(float4 v) { return f32x2{v.z, v.w}; }
__device__ __forceinline__ float4 cat4(f32x2 a, f32x2 b) { return make_float4(a.x, a.y, b.x, b.y); }
__device__ __forceinline__ float4 fma4(float w, float4 g, float4 a) {
  const f32x2 w2 = {w, w};
  return cat4(__builtin_elementwise_fma(w2, lo2(g), lo2(a)),
              __builtin_elementwise_fma(w2, hi2(g), hi2(a)));
}
// acc_dgrad on 4 channels with the per-element dbilerp_row / _col in packed form; the
// per-channel accumulation chains stay in order x, y, z, w (same bits as acc_dgrad)
__device__ __forceinline__ void acc_dgrad4p(float fr, float fc, float4 gv, float4 a, float4 b,
                                            float4 c, float4 d, float& diy, float& dix) {
  const f32x2 fr2 = {fr, fr}, fc2 = {fc, fc}, gr2 = {1.0f - fr, 1.0f - fr},
              gc2 = {1.0f - fc, 1.0f - fc};
  // dbilerp_row = fmaf(fc, d - b, (1-fc) * (c - a)); dbilerp_col = fmaf(fr, d - c, (1-fr) * (b - a))
  const f32x2 rl = __builtin_elementwise_fma(fc2, lo2(d) - lo2(b), gc2 * (lo2(c) - lo2(a)));
  const f32x2 rh = __builtin_elementwise_fma(fc2, hi2(d) - hi2(b), gc2 * (hi2(c) - hi2(a)));
  const f32x2 sl = __builtin_elementwise_fma(fr2, lo2(d) - lo2(c), gr2 * (lo2(b) - lo2(a)));
  const f32x2 sh = __builtin_elementwise_fma(fr2, hi2(d) - hi2(c), gr2 * (hi2(b) - hi2(a)));
  diy = fmaf(gv.x, rl.x, diy);
  dix = fmaf(gv.x, sl.x, dix);
  diy = fmaf(gv.y, rl.y, diy);
  dix = fmaf(gv.y, sl.y, dix);
  diy = fmaf(gv.z, rh.x, diy);
  dix = fmaf(gv.z, sh.x, dix);
  diy = fmaf(gv.w, rh.y, diy);
  dix = fmaf(gv.w, sh.y, dix);
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int U, int kTQ, typename GT = float, typename XT = float, int WPE = 6, int kTR = 4>
__global__ __launch_bounds__((kTR + 1) * 64) __attribute__((amdgpu_waves_per_eu(WPE))) void col2im_tile(Geo g, const XT* __restrict__ xT,
                                                           const int4* __restrict__ brec,
                                                           const int* __restrict__ start,
                                                           const GT* __restrict__ gcolT,
                                                           float* __restrict__ gxT,
                                                           float* __restrict__ goff,
                                                           float* __restrict__ cpart, int b0,
                                                           int tq_n) {
  constexpr int kC2iThreads = (kTR + 1) * 64, WR = kTR + 1, WQ = kTQ + 1;
  static_assert(U <= 4, "wave_sum8 takes at most 8 ∂offset sums per batch");
  // float4 slots: a zero row (window row -1: wave 0's ∂offset reads it only at image row
  // -1, so no select), the xT window; then the upper rows
  constexpr int ZR = WQ * 64, WIN = WR * WQ * 64, UPR = kTR * kTQ * 64;
  // the window holds xT's own element type (bf16: 8 B per lane and pixel, widened when a
  // bin's corners are read): r05, half the LDS of the fp32 image, so 4 instead of 3
  // workgroups of 8 waves fit a CU (the upper-row exchange after the loop, fp32, is the
  // larger use then)
  typedef typename std::conditional<sizeof(XT) == 2, uint2, float4>::type WinT;
  constexpr int kWinB = (ZR + WIN) * (int)sizeof(WinT), kUprB = UPR * 16;
  __shared__ __attribute__((aligned(16))) char lds_raw[kWinB > kUprB ? kWinB : kUprB];
  WinT* const lwin = reinterpret_cast<WinT*>(lds_raw);
  WinT* const lds = lwin + ZR;                                 // the window
  float4* const lds_ = reinterpret_cast<float4*>(lds_raw);    // the upper rows
  auto widen = [](const WinT& v) -> float4 {
    if constexpr (sizeof(XT) == 2)
      return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                         __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
    else
      return v;
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Block3 blk = xcd_block();
  const int bl = blk.z, b = b0 + bl;
  const int tr_i = blk.x / tq_n, tq_i = blk.x - tr_i * tq_n;
  const int R0 = tr_i * kTR, Q0 = tq_i * kTQ;
  const int c = lane * 4;
  const bool cok = c < g.C;
  const XT* xb = xT + (size_t)b * g.HWi * g.C;
  // xT rows R0..R0+kTR, cols Q0-1..Q0+kTQ-1 (zero outside the image) into registers; they go
  // to LDS after each wave has started its record / ∂col row stream, and the barrier
  // orders LDS only, so the stream's first rows are in flight across it (r01 staged the
  // window first: the stream began a full staging round trip later)
  constexpr int WIT = (WIN + kC2iThreads - 1) / kC2iThreads;
  WinT wv[WIT];
#pragma unroll
  for (int k = 0; k < WIT; ++k) {
    const int idx = tid + k * kC2iThreads;
    const int pix = idx >> 6, l = idx & 63;
    const int r = R0 + pix / WQ, q = Q0 - 1 + pix % WQ, cc = l * 4;
    wv[k] = (idx < WIN && r < g.H && q >= 0 && q < g.W && cc < g.C)
                ? *reinterpret_cast<const WinT*>(xb + ((size_t)r * g.W + q) * g.C + cc)
                : WinT{};
  }
  const int NB = (g.H + 1) * (g.W + 1);
  const int* st = start + (size_t)bl * (NB + 1);
  const int4* rb = brec + (size_t)bl * g.HW * g.N;
  const GT* gb = gcolT + (size_t)bl * g.HW * g.K;
  float* gob = goff + (size_t)b * g.J * g.HW;
  const float sy = (float)(g.H - 1) / (float)(g.Wo - 1);
  const float sx = (float)(g.W - 1) / (float)(g.Ho - 1);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 up[kTQ], dn[kTQ];  // pixel rows r0 (tile row w-1) and r0+1 (tile row w)
#pragma unroll
  for (int j = 0; j < kTQ; ++j) up[j] = dn[j] = z4;
  float4 lup = z4, ldn = z4;  // the same two rows at pixel column Q0-1 (boundary partial)
  const int br = R0 + w;  // bin row = r0 + 1
  const bool act = br <= g.H;
  const bool drow = w >= 1 || br == 0;  // owns the ∂offset of this bin row
  // the row's bins (br, Q0..Q0+kTQ-1; ..W in the last tile column) are consecutive, so
  // their records are one contiguous range: fetch it 64 records per vector load (lane l <-
  // record l) and take each with v_readlane — no scalar-load round trip per sample
  const int bin0 = min(br, g.H) * (g.W + 1) + Q0;
  const int nbin = tq_i == tq_n - 1 ? g.W - Q0 + 1 : kTQ;
  int bst[kTQ + 2];
#pragma unroll
  for (int k = 0; k <= kTQ + 1; ++k)  // wave-uniform: scalar registers, scalar loop bounds
    bst[k] = __builtin_amdgcn_readfirstlane(act ? st[bin0 + min(k, nbin)] : 0);
  const int rowlo = bst[0], rowhi = bst[nbin];
  // Software pipeline over the row's records (contiguous across its bins), 64 records (a
  // segment) at a time: lane l holds record seg+l (a buffer load that returns 0 past the
  // end, so no branch), and every load inside a segment is
  // unconditional (indices clamped into it). hipcc then counts vmcnt across the loop instead
  // of draining it at each conditional load (r02: one conditional page reload per batch made
  // every batch wait for all loads and ∂offset stores in flight). Batch k+1's records
  // (v_readlane) and ∂colT rows are issued before batch k is consumed. Batches never
  // straddle a bin, so each bin's compute keeps static accumulator indices while the
  // prefetch flows across bin boundaries. A sample's ∂offset stays in the lane of its
  // record until the segment ends: one scattered vector store per segment, none per sample.
  const auto rrec = __builtin_amdgcn_make_buffer_rsrc(const_cast<int4*>(rb), 0,
                                                      (int)(g.HW * g.N * 16), 0x00020000);
  int seg = rowlo, segend = rowlo;
  int rowhi_c = bst[1] > rowlo ? bst[1] : rowhi;  // end of the current phase's records
  int4 pg = make_int4(0, 0, 0, 0);
  auto load_seg = [&](int s0) {
    seg = s0;
    segend = min(s0 + 64, rowhi_c);
    const unsigned o = s0 + lane < segend ? (unsigned)(s0 + lane) * 16u : 0x80000000u;
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(rrec, o, 0, 0);
    pg = make_int4((int)q[0], (int)q[1], (int)q[2], (int)q[3]);
  };
  int4 nR[U];
  // rows in flight as loaded (bf16: 8 B per lane, converted when consumed); buffer loads, the
  // lanes past C out of range (they read 0: no select on the values)
  typedef typename std::conditional<sizeof(GT) == 2, uint2, float4>::type RowT;
  RowT nx[U];
  const auto rcol = __builtin_amdgcn_make_buffer_rsrc(const_cast<GT*>(gb), 0,
                                                      (int)((size_t)g.HW * g.K * sizeof(GT)),
                                                      0x00020000);
  const unsigned coff = cok ? (unsigned)(c * sizeof(GT)) : 0x80000000u;
  // two register sets for the batch stream, used in turn (a batch reads one while the next
  // batch's loads land in the other), so no batch copies its rows into place
  int4 mR[U];
  RowT mx[U];
  auto issue_into = [&](int ni, int4(&tR)[U], RowT(&tx)[U]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = min(ni + u, segend - 1) - seg;  // wave-uniform, in [0, 64)
      tR[u] = make_int4(__builtin_amdgcn_readlane(pg.x, l), __builtin_amdgcn_readlane(pg.y, l),
                        __builtin_amdgcn_readlane(pg.z, l), __builtin_amdgcn_readlane(pg.w, l));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned o = (unsigned)tR[u].x * (unsigned)sizeof(GT) + coff;
      if constexpr (sizeof(GT) == 2) {
        const auto q = __builtin_amdgcn_raw_buffer_load_b64(rcol, o, 0, 0);
        tx[u] = make_uint2(q[0], q[1]);
      } else {
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rcol, o, 0, 0);
        tx[u] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                            __uint_as_float(q[3]));
      }
    }
  };
  auto issue = [&](int ni) __attribute__((always_inline)) { issue_into(ni, nR, nx); };
  // two phases: bin column 0 (its left-boundary partials die with it), then columns 1..
  const int mid = bst[1];
  const bool any0 = act && mid > rowlo, any1 = act && rowhi > mid;
  if (any0) {
    load_seg(rowlo);
    issue(rowlo);
  } else if (any1) {
    load_seg(mid);
    issue(mid);
  }
#pragma unroll
  for (int k = 0; k < WIT; ++k)
    if (tid + k * kC2iThreads < WIN) lds[tid + k * kC2iThreads] = wv[k];
  for (int k = tid; k < ZR; k += kC2iThreads) lwin[k] = WinT{};
  lds_barrier();
  // the samples [rlo, rhi) of bin columns BJ0..BJ1-1, segment by segment (the first segment
  // already loaded and issued)
  auto phase = [&](auto BJ0, auto BJ1, int rlo, int rhi) __attribute__((always_inline)) {
    constexpr int kB0 = decltype(BJ0)::value, kB1 = decltype(BJ1)::value;
    for (int s0 = rlo;;) {
      float oy = 0.f, ox = 0.f;  // ∂offset of record seg+lane
#pragma unroll
      for (int bj = kB0; bj < kB1; ++bj) {
        if (bj >= nbin) break;
        const int lo = max(bst[bj], seg), hi = min(bst[bj + 1], segend);
        // the bin's four corners (r0, c0) .. (r0+1, c0+1), the same for all its samples, at
        // window (w-1, bj) .. (w, bj+1); column bj+1 = kTQ+1 is W (the last tile column's bin
        // W): outside the image. Read once per bin and segment, not per sample.
        float4 ka = z4, kb = z4, kc = z4, kd = z4;
        if (drow && lo < hi) {
          const WinT* w4 = lds + ((w - 1) * WQ + bj) * 64 + lane;
          const bool cB = bj + 1 <= kTQ;  // (bj is unrolled: a constant)
          ka = widen(w4[0]);
          kb = cB ? widen(w4[64]) : z4;
          kc = widen(w4[WQ * 64]);
          kd = cB ? widen(w4[(WQ + 1) * 64]) : z4;
        }
        // batch i from (cR, cx); the next batch of this bin, else the next bin's first, into
        // (tR, tx)
        auto batch = [&](int i, int4(&cR)[U], RowT(&cx)[U], int4(&tR)[U], RowT(&tx)[U])
                         __attribute__((always_inline)) {
          int4 R[U];
          float4 gv[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            R[u] = cR[u];
            if constexpr (sizeof(GT) == 2) {
              const uint2 q = cx[u];
              gv[u] = make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                                  __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
            } else {
              gv[u] = cx[u];
            }
          }
          issue_into(i + U < hi ? i + U : hi, tR, tx);
          float dv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // per-lane ∂offset parts
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (i + u >= hi) break;
            const float fr = __int_as_float(R[u].y), fc = __int_as_float(R[u].z);
            const float gr = 1.0f - fr, gc = 1.0f - fc;
            if (bj < kTQ) {
              up[bj] = fma4(gr * fc, gv[u], up[bj]);
              dn[bj] = fma4(fr * fc, gv[u], dn[bj]);
            }
            if (bj >= 1) {
              up[bj - 1] = fma4(gr * gc, gv[u], up[bj - 1]);
              dn[bj - 1] = fma4(fr * gc, gv[u], dn[bj - 1]);
            } else {
              lup = fma4(gr * gc, gv[u], lup);
              ldn = fma4(fr * gc, gv[u], ldn);
            }
            if (drow) {
              acc_dgrad4p(fr, fc, gv[u], ka, kb, kc, kd, dv[2 * u], dv[2 * u + 1]);
              // opaque to hipcc's SLP vectorizer: it would pair the two scalar FMA chains
              // into packed FMAs behind moves (more VALU, not less)
              asm("" : "+v"(dv[2 * u]), "+v"(dv[2 * u + 1]));
            }
          }
          if (drow) {  // the batch's 2U wave sums in one tree (wave_sum's order: same bits)
            const float sd = wave_sum8(dv, lane);
#pragma unroll
            for (int u = 0; u < U; ++u) {  // no branch: a sample past hi selects no lane
              const float sy_u =
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sd), wave_sum8_lane(2 * u)));
              const float sx_u = __int_as_float(
                  __builtin_amdgcn_readlane(__float_as_int(sd), wave_sum8_lane(2 * u + 1)));
              const bool mine = lane == i + u - seg && i + u < hi;
              oy = mine ? sy_u : oy;
              ox = mine ? sx_u : ox;
            }
          }
        };
        // the bin's batches alternate between the sets (nR, nx) and (mR, mx); every bin
        // starts from (nR, nx), so a bin with an odd batch count moves the next bin's first
        // batch there once
        for (int i = lo; i < hi;) {
          batch(i, nR, nx, mR, mx);
          i += U;
          if (i >= hi) {
#pragma unroll
            for (int u = 0; u < U; ++u) nR[u] = mR[u], nx[u] = mx[u];
            break;
          }
          batch(i, mR, mx, nR, nx);
          i += U;
        }
      }
      if (drow && seg + lane < segend) {
        gob[pg.w] = oy * sy;
        gob[(size_t)g.N * g.HW + pg.w] = ox * sx;
      }
      s0 += 64;
      if (s0 >= rhi) break;
      load_seg(s0);
      issue(s0);
    }
  };
  if (any0) {
    auto rhi0 = mid;  // segments end at the bin column's end
    rowhi_c = rhi0;
    phase(std::integral_constant<int, 0>(), std::integral_constant<int, 1>(), rowlo, rhi0);
  }
  if (act && tq_i > 0 && cok) {  // bin column Q0 is done: its left boundary partials
    const size_t rs = (size_t)tq_n * 2 * g.C;  // pixel-row stride
    float* cp = cpart + (size_t)bl * g.H * rs + (size_t)tq_i * 2 * g.C + c;
    if (w < kTR && br < g.H) *reinterpret_cast<float4*>(cp + br * rs) = ldn;
    if (w >= 1) *reinterpret_cast<float4*>(cp + (br - 1) * rs + g.C) = lup;
  }
  if (any1) {
    rowhi_c = rowhi;
    if (any0) {
      load_seg(mid);
      issue(mid);
    }
    phase(std::integral_constant<int, 1>(), std::integral_constant<int, kTQ + 1>(), mid, rowhi);
  }
  __syncthreads();  // window no longer read: reuse the LDS for the upper rows
  if (w >= 1)
#pragma unroll
    for (int j = 0; j < kTQ; ++j) lds_[((w - 1) * kTQ + j) * 64 + lane] = up[j];
  __syncthreads();
  const int r = R0 + w;
  if (w < kTR && r < g.H && cok) {
#pragma unroll
    for (int j = 0; j < kTQ; ++j)
      if (Q0 + j < g.W)
        *reinterpret_cast<float4*>(gxT + (((size_t)b * g.H + r) * g.W + Q0 + j) * g.C + c) =
            add4(dn[j], lds_[(w * kTQ + j) * 64 + lane]);
  }
}

// ∂xT of the last pixel column of each tile column but the last += the boundary partials the
// tile to its right wrote (col2im_tile): ∂xT + (lower + upper), in that order, after K5.
__global__ __launch_bounds__(256) void col2im_fold(Geo g, const float4* __restrict__ cpart,
                                                   float4* __restrict__ gxT, int b0, int nb,
                                                   int tq_n, int tq) {
  const int C4 = g.C >> 2;
  const size_t n = (size_t)nb * g.H * (tq_n - 1) * C4;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const int c4 = (int)(i % C4);
    size_t t = i / C4;
    const int k = 1 + (int)(t % (tq_n - 1));
    t /= (tq_n - 1);
    const int r = (int)(t % g.H), bl = (int)(t / g.H);
    float4* d = gxT + (((size_t)(b0 + bl) * g.H + r) * g.W + k * tq - 1) * C4 + c4;
    const float4* p = cpart + (((size_t)bl * g.H + r) * tq_n + k) * 2 * C4 + c4;
    *d = add4(*d, add4(p[0], p[C4]));
  }
}

// ∂xT[b][r][q][gi*Cg + c] = Σ over the samples of bins (r-1,q-1), (r-1,q), (r,q-1),
// (r,q) of (their w11, w10, w01, w00 weight) · ∂colT row. One group of LP lanes per
// input pixel. The group's lanes first fetch up to LP (bin entry -> sample -> weight,
// row offset) records in parallel, then the row loads are issued kU at a time.
template <int VEC>
__global__ __launch_bounds__(256) void dx_gather_cl(Geo g, LaneMap L,
                                                    const float4* __restrict__ rec,
                                                    const int* __restrict__ start,
                                                    const int* __restrict__ list,
                                                    const float* __restrict__ gcolT,
                                                    float* __restrict__ gxT, int b0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Block3 blk = xcd_block();
  const int gi = blk.y, bl = blk.z, b = b0 + bl;
  const int sub = lane / L.LP, u0 = lane - sub * L.LP;
  const int p = (blk.x * 4 + wave) * L.SP + sub;  // input pixel r*W + q
  const bool pok = p < g.HWi;
  const int pp = pok ? p : 0;
  const int r = pp / g.W, q = pp - r * g.W;
  const int NB = (g.H + 1) * (g.W + 1), NS = g.HW * g.N;
  const int bg = bl * g.G + gi;
  const int* st = start + (size_t)bg * (NB + 1);
  const int* lst = list + (size_t)bg * NS;
  const float4* rc = rec + (size_t)bg * NS;
  const float* gb = gcolT + (size_t)bl * g.HW * g.K + (size_t)gi * g.Cg;
  // the four bins: k=0 (r-1,q-1) -> w11, 1 (r-1,q) -> w10, 2 (r,q-1) -> w01, 3 (r,q) -> w00
  int lo[4], cntk[4];
  int E = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int dr = (k >> 1) ^ 1, dc = (k & 1) ^ 1;
    const int bin = (r - dr + 1) * (g.W + 1) + (q - dc + 1);
    lo[k] = pok ? st[bin] : 0;
    cntk[k] = pok ? st[bin + 1] - lo[k] : 0;
    E += cntk[k];
  }
  // E differs between the pixel groups of a wave: loop to the wave maximum
  int Emax = E;
  for (int o = 32; o >= L.LP; o >>= 1) Emax = max(Emax, __shfl_xor(Emax, o));
  const int gbase = sub * L.LP;  // first lane of this pixel's group
  // every lane of the group takes part in entry resolution and the shuffles, also
  // lanes whose channel unit is past CQ (they only skip the loads / FMAs)
  for (int cu0 = 0; cu0 < L.CQ; cu0 += L.LP) {
    const int cu = cu0 + u0;
    const bool cok = cu < L.CQ;
    const int c = (cok ? cu : 0) * VEC;
    typename Vec<VEC>::T acc = Vec<VEC>::zero();
    for (int e0 = 0; e0 < Emax; e0 += L.LP) {
      // lane u0 of the group resolves entry e0 + u0
      const int e = e0 + u0;
      float wgt = 0.f;
      int row = 0;
      if (e < E) {
        int k = 0, idx = e;
        while (idx >= cntk[k]) {
          idx -= cntk[k];
          ++k;
        }
        const int s = lst[lo[k] + idx];
        const float4 R = rc[s];
        const float wr = (k >> 1) == 0 ? R.y : 1.0f - R.y;  // rows r-1 bins weigh fr
        const float wc = (k & 1) == 0 ? R.z : 1.0f - R.z;   // cols q-1 bins weigh fc
        wgt = wr * wc;
        const int m = s / g.N;
        row = m * g.K + (s - m * g.N) * g.C;
      }
      const int n_here = min(L.LP, max(E - e0, 0));
      const int n_wave = min(L.LP, Emax - e0);
      for (int i = 0; i < n_wave; i += kU) {
        float wv[kU];
        int rv[kU];
        typename Vec<VEC>::T gv[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int src = gbase + min(i + u, L.LP - 1);
          wv[u] = __shfl(wgt, src);
          rv[u] = __shfl(row, src);
          gv[u] = ldv<VEC>(gb + (size_t)rv[u] + c, cok && i + u < n_here);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (i + u >= n_here) continue;
          if constexpr (VEC == 4) {
            acc.x = fmaf(wv[u], gv[u].x, acc.x);
            acc.y = fmaf(wv[u], gv[u].y, acc.y);
            acc.z = fmaf(wv[u], gv[u].z, acc.z);
            acc.w = fmaf(wv[u], gv[u].w, acc.w);
          } else {
            acc = fmaf(wv[u], gv[u], acc);
          }
        }
      }
    }
    if (pok && cok) stv<VEC>(gxT + ((size_t)b * g.HWi + p) * g.C + (size_t)gi * g.Cg + c, acc);
  }
}

// ---------------------------------------------------------------------------
// Transposes (64x64 tiles through LDS, odd pitch).
// ---------------------------------------------------------------------------
// out[b][p][c] = in[b][c][p]
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc(const T* __restrict__ in, T* __restrict__ out,
                                                    int C, int P) {
  __shared__ T t[64][65];
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const T* ib = in + (size_t)b * C * P;
  T* ob = out + (size_t)b * C * P;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, p = p0 + tx;
    if (c < C && p < P) t[i][tx] = ib[(size_t)c * P + p];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int p = p0 + i, c = c0 + tx;
    if (c < C && p < P) ob[(size_t)p * C + c] = t[tx][i];
  }
}

// out[b][c][p] = in[b][p][c]
__global__ __launch_bounds__(256) void nhwc_to_nchw(const float* __restrict__ in,
                                                    float* __restrict__ out, int C, int P) {
  __shared__ float t[64][65];
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const float* ib = in + (size_t)b * C * P;
  float* ob = out + (size_t)b * C * P;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int p = p0 + i, c = c0 + tx;
    if (c < C && p < P) t[i][tx] = ib[(size_t)p * C + c];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, p = p0 + tx;
    if (c < C && p < P) ob[(size_t)c * P + p] = t[tx][i];
  }
}

hipError_t launch_nchw_to_nhwc(const float* in, float* out, int B, int C, int P, hipStream_t s) {
  if (launch_xpose_f4(in, out, B, C, P, s)) return hipGetLastError();
  dim3 grid((P + 63) / 64, (C + 63) / 64, B);
  hipLaunchKernelGGL(nchw_to_nhwc<float>, grid, dim3(256), 0, s, in, out, C, P);
  return hipGetLastError();
}

// bf16 transpose: 8-byte (4-element) global loads and stores, a 64x64 tile in LDS (rows
// padded to 66 elements). The generic 2-byte-per-lane form moved 128 B per wave instruction
// and ran at 2.4 TB/s (r02, config 4: 21 us for 25.7 MB each way).
__global__ __launch_bounds__(256) void nchw_to_nhwc_bf16x4(const bf16_t* __restrict__ in,
                                                           bf16_t* __restrict__ out, int C,
                                                           int P) {
  __shared__ unsigned short t[64][66];  // [c][p]
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const bf16_t* ib = in + (size_t)b * C * P;
  bf16_t* ob = out + (size_t)b * C * P;
  const int tid = threadIdx.x, q = tid & 15, r = tid >> 4;  // 16 lanes x 4 elements per row
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // rows c0 + r + 16i, elements p0 + 4q .. +3
    const int c = c0 + r + 16 * i, p = p0 + 4 * q;
    uint2 v = make_uint2(0u, 0u);
    if (c < C && p + 3 < P) {
      v = *reinterpret_cast<const uint2*>(ib + (size_t)c * P + p);
    } else if (c < C) {
      unsigned short e[4] = {0, 0, 0, 0};
      for (int k = 0; k < 4; ++k)
        if (p + k < P) e[k] = ib[(size_t)c * P + p + k];
      v = make_uint2(e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16));
    }
    unsigned* d = reinterpret_cast<unsigned*>(&t[r + 16 * i][4 * q]);
    d[0] = v.x;
    d[1] = v.y;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // rows p0 + r + 16i, elements c0 + 4q .. +3
    const int p = p0 + r + 16 * i, c = c0 + 4 * q;
    if (p >= P || c >= C) continue;
    const unsigned short e0 = t[4 * q][r + 16 * i], e1 = t[4 * q + 1][r + 16 * i];
    const unsigned short e2 = t[4 * q + 2][r + 16 * i], e3 = t[4 * q + 3][r + 16 * i];
    if (c + 3 < C) {
      *reinterpret_cast<uint2*>(ob + (size_t)p * C + c) =
          make_uint2(e0 | ((unsigned)e1 << 16), e2 | ((unsigned)e3 << 16));
    } else {
      const unsigned short e[4] = {e0, e1, e2, e3};
      for (int k = 0; k < 4 && c + k < C; ++k) ob[(size_t)p * C + c + k] = e[k];
    }
  }
}

hipError_t launch_nchw_to_nhwc_bf16(const bf16_t* in, bf16_t* out, int B, int C, int P,
                                    hipStream_t s) {
  if (launch_xpose_b8(in, out, B, C, P, s)) return hipGetLastError();
  dim3 grid((P + 63) / 64, (C + 63) / 64, B);
  // 8-byte global accesses need 4-element alignment of every row start
  if (P % 4 == 0 && C % 4 == 0 && ((uintptr_t)in & 7) == 0 && ((uintptr_t)out & 7) == 0)
    hipLaunchKernelGGL(nchw_to_nhwc_bf16x4, grid, dim3(256), 0, s, in, out, C, P);
  else
    hipLaunchKernelGGL(nchw_to_nhwc<bf16_t>, grid, dim3(256), 0, s, in, out, C, P);
  return hipGetLastError();
}

hipError_t launch_nhwc_to_nchw(const float* in, float* out, int B, int C, int P, hipStream_t s) {
  dim3 grid((P + 63) / 64, (C + 63) / 64, B);
  hipLaunchKernelGGL(nhwc_to_nchw, grid, dim3(256), 0, s, in, out, C, P);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Generic kernels (NCHW x, one thread per column element / sample): an
// implementation independent of the transposes, lane maps and bins, used for
// cross-checks and forced by dcn_debug_force_generic.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void im2col_generic(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      float* __restrict__ colT, int b0, int nb) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)nb * g.HW * g.K;
  if (idx >= total) return;
  const int k = (int)(idx % g.K);
  const long row = idx / g.K;
  const int m = (int)(row % g.HW), bl = (int)(row / g.HW), b = b0 + bl;
  const int n = k / g.C, c = k - n * g.C, gi = c / g.Cg;
  const Tap tp = sample_tap(g, off, b, gi, n, m);
  float v = 0.f;
  if (tp.ok) {
    const float* xp = x + ((size_t)b * g.C + c) * g.HWi;
    v = bilerp(tp.fr, tp.fc, ldx(xp, tp.r0, tp.c0, g), ldx(xp, tp.r0, tp.c0 + 1, g),
               ldx(xp, tp.r0 + 1, tp.c0, g), ldx(xp, tp.r0 + 1, tp.c0 + 1, g));
  }
  colT[idx] = v;
}

__device__ __forceinline__ void scatter_global(float* __restrict__ gxp, int r, int c, float v,
                                               const Geo& g) {
  if (v != 0.f && r >= 0 && r < g.H && c >= 0 && c < g.W) atomicAdd(gxp + r * g.W + c, v);
}

// gx (NCHW) must be zeroed by the caller; goff overwritten.
__global__ __launch_bounds__(256) void col2im_generic(Geo g, const float* __restrict__ x,
                                                      const float* __restrict__ off,
                                                      const float* __restrict__ gcolT,
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
  const int bl = (int)(t / g.G), b = b0 + bl;
  const Tap tp = sample_tap(g, off, b, gi, n, m);
  float diy = 0.f, dix = 0.f;
  if (tp.ok) {
    const float gr = 1.0f - tp.fr, gc = 1.0f - tp.fc;
    const float* grow = gcolT + ((size_t)bl * g.HW + m) * g.K + (size_t)n * g.C;
    for (int cl = 0; cl < g.Cg; ++cl) {
      const int c = gi * g.Cg + cl;
      const float gv = grow[c];
      const float* xp = x + ((size_t)b * g.C + c) * g.HWi;
      const float x00 = ldx(xp, tp.r0, tp.c0, g), x01 = ldx(xp, tp.r0, tp.c0 + 1, g);
      const float x10 = ldx(xp, tp.r0 + 1, tp.c0, g), x11 = ldx(xp, tp.r0 + 1, tp.c0 + 1, g);
      diy = fmaf(gv, dbilerp_row(tp.fc, x00, x01, x10, x11), diy);
      dix = fmaf(gv, dbilerp_col(tp.fr, x00, x01, x10, x11), dix);
      float* gxp = gx + ((size_t)b * g.C + c) * g.HWi;
      scatter_global(gxp, tp.r0, tp.c0, gv * (gr * gc), g);
      scatter_global(gxp, tp.r0, tp.c0 + 1, gv * (gr * tp.fc), g);
      scatter_global(gxp, tp.r0 + 1, tp.c0, gv * (tp.fr * gc), g);
      scatter_global(gxp, tp.r0 + 1, tp.c0 + 1, gv * (tp.fr * tp.fc), g);
    }
  }
  const float sy = (float)(g.H - 1) / (float)(g.Wo - 1);
  const float sx = (float)(g.W - 1) / (float)(g.Ho - 1);
  float* gob = goff + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  gob[(size_t)n * g.HW + m] = diy * sy;
  gob[(size_t)(g.N + n) * g.HW + m] = dix * sx;
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
static bool can_vec4(const Geo& g) { return g.C % 4 == 0 && g.Cg % 4 == 0; }

static int bins_nch(const Geo& g) { return (g.HW * g.N + kBinChunk - 1) / kBinChunk; }
static bool k5_fused(const Geo& g);
constexpr int kK5TQ = 4;  // fused K5 tile columns (both element types)
static int k5_tq_n(const Geo& g) { return (g.W + kK5TQ - 1) / kK5TQ; }

// Bins workspace: start[seg][NB+1] | H[seg][nch][NBp] | R[seg][nch][NBp] |
// sorted[seg][nch][kBinChunk] (16 B) | rec[seg][NS] (unfused K5 only) | cpart[seg][H][tq_n][C]
// [2] (fused K5's boundary partials) | brec[seg][NS] (int4; slist, int, for the unfused K5).
size_t bins_ws_bytes(const Geo& g, int nb) {
  const size_t NB = (size_t)(g.H + 1) * (g.W + 1), NS = (size_t)g.HW * g.N;
  const size_t seg = (size_t)nb * g.G, nch = bins_nch(g);
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  size_t b = al(seg * (NB + 1) * 4);
  b += 2 * al(seg * nch * bins_nbp((int)NB) * 4);
  b += al(seg * nch * kBinChunk * 16);
  if (!k5_fused(g)) b += al(seg * NS * 16);
  else b += al(seg * g.H * k5_tq_n(g) * 2 * g.C * 4);
  b += al(seg * NS * 16);
  return b;
}

hipError_t launch_im2col(const Geo& g, const float* x, const float* xT, const float* off,
                         float* colT, int b0, int nb, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  if (g_force_generic) {
    const long total = (long)nb * g.HW * g.K;
    hipLaunchKernelGGL(im2col_generic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, g,
                       x, off, colT, b0, nb);
    return hipGetLastError();
  }
  if (g.G == 1 && g.N <= kMaxTaps && g.C % 4 == 0) {
    auto go = [&](auto kern, int TH, int TW) {
      const int th_n = (g.Ho + TH - 1) / TH, tw_n = (g.Wo + TW - 1) / TW;
      hipLaunchKernelGGL(kern, dim3(th_n * tw_n, 1, nb), dim3(256), 0, s, g, xT, off, colT, b0,
                         tw_n);
    };
    // Measured at config 3 (r01 A/B): whole 1-KiB column rows per wave instruction
    // (4x4 tile, all 256 channels, 1-px margin, non-temporal column stores) 0.418 ms;
    // 8x8 tile x 64-ch slices 0.441; margin 2/3 windows slower (LDS occupancy).
    if (g.C <= 32)
      go(im2col_lds<8, 8, 2, 32, true>, 8, 8);
    else if (g.C <= 64)
      go(im2col_lds<8, 8, 2, 64, true>, 8, 8);
    else if (g.C <= 128)
      go(im2col_lds<4, 4, 1, 128, true>, 4, 4);
    else
      go(im2col_lds<4, 4, 1, 256, true>, 4, 4);
    return hipGetLastError();
  }
  const int NS = g.HW * g.N;
  dim3 grid((NS + 255) / 256, g.G, nb);
  if (can_vec4(g))
    hipLaunchKernelGGL(im2col_cl<4>, grid, dim3(256), 0, s, g, lane_map(g.Cg, 4), xT, off, colT,
                       b0);
  else
    hipLaunchKernelGGL(im2col_cl<1>, grid, dim3(256), 0, s, g, lane_map(g.Cg, 1), xT, off, colT,
                       b0);
  return hipGetLastError();
}

static bool k5_fused(const Geo& g) {
  return g.G == 1 && g.C % 4 == 0 && g.C <= 256;
}

// Pointers into the bins workspace (bins_ws_bytes layout).
struct BinsWs {
  int *start, *H, *R, *slist;
  uint4* sorted;
  float4* rec;
  float* cpart;
  int4* brec;
};
static BinsWs bins_ptrs(const Geo& g, void* bins_ws, int nb) {
  const size_t NB = (size_t)(g.H + 1) * (g.W + 1), NS = (size_t)g.HW * g.N;
  const size_t seg = (size_t)nb * g.G, nch = bins_nch(g);
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  char* w = static_cast<char*>(bins_ws);
  BinsWs P;
  P.start = reinterpret_cast<int*>(w);
  w += al(seg * (NB + 1) * 4);
  P.H = reinterpret_cast<int*>(w);
  w += al(seg * nch * bins_nbp((int)NB) * 4);
  P.R = reinterpret_cast<int*>(w);
  w += al(seg * nch * bins_nbp((int)NB) * 4);
  P.sorted = reinterpret_cast<uint4*>(w);
  w += al(seg * nch * kBinChunk * 16);
  P.rec = nullptr;
  P.cpart = nullptr;
  if (!k5_fused(g)) {
    P.rec = reinterpret_cast<float4*>(w);
    w += al(seg * NS * 16);
  } else {
    P.cpart = reinterpret_cast<float*>(w);
    w += al(seg * g.H * k5_tq_n(g) * 2 * g.C * 4);
  }
  P.brec = reinterpret_cast<int4*>(w);
  P.slist = reinterpret_cast<int*>(w);  // sorted lists (unfused K5) share that region
  return P;
}

hipError_t launch_bins(const Geo& g, const float* off, void* bins_ws, float* goff, int b0, int nb,
                       hipStream_t s) {
  if (nb <= 0 || g_force_generic) return hipSuccess;
  const int NB = (g.H + 1) * (g.W + 1), nch = bins_nch(g);
  // packed entries hold the bin above kBinLBits bits; keys go up to NB + 1
  if ((unsigned long long)(NB + 2) >= (1ull << (32 - kBinLBits))) return hipErrorInvalidValue;
  const unsigned kbits = 32 - __builtin_clz((unsigned)NB + 1);
  const size_t seg = (size_t)nb * g.G;
  const BinsWs P = bins_ptrs(g, bins_ws, nb);
  const bool fused = k5_fused(g);
  if (fused && g.HW * g.N <= kBsMax && !g_bins_chunked) {
    // (the samples in no bin get their zero ∂offset from the sort kernel: no memset)
    hipLaunchKernelGGL(bins_sort_seg, dim3((unsigned)seg), dim3(kBsT), 0, s, g, off, b0, NB, kbits,
                       P.start, P.brec, goff);
    return hipGetLastError();
  }
  // H must start at 0 (only the bins present in a chunk are written); R needs no init
  hipError_t e = hipMemsetAsync(P.H, 0, seg * nch * bins_nbp(NB) * sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bins_chunk_sort, dim3(nch, (unsigned)seg), dim3(kBinT), 0, s, g, off, b0, nch,
                     NB, kbits, P.H, P.R, P.sorted, fused ? nullptr : P.rec);
  hipLaunchKernelGGL(bins_scan_table<BINS_SCAN_T>, dim3((unsigned)seg), dim3(BINS_SCAN_T), 0, s, NB,
                     nch, P.H, P.start);
  hipLaunchKernelGGL(bins_emit, dim3((NB + 255) / 256, (unsigned)seg), dim3(256), 0, s, g, nch, NB,
                     P.H, P.R, P.start, P.sorted, fused ? P.brec : nullptr, P.slist);
  if (fused) {
    // samples in no bin (every corner outside the image) have ∂offset 0
    e = hipMemsetAsync(goff + (size_t)b0 * g.J * g.HW, 0, (size_t)nb * g.J * g.HW * sizeof(float),
                       s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

bool col2im_chunkable(const Geo& g) { return !g_force_generic && k5_fused(g); }

// bins of images [0, bins_nb) in bins_ws; the view of images [b0, ...)
static BinsWs bins_view(const Geo& g, void* bins_ws, int b0, int nb, int bins_nb) {
  if (bins_nb <= 0) return bins_ptrs(g, bins_ws, nb);
  BinsWs P = bins_ptrs(g, bins_ws, bins_nb);
  const size_t NB = (size_t)(g.H + 1) * (g.W + 1), NS = (size_t)g.HW * g.N;
  P.start += (size_t)b0 * g.G * (NB + 1);
  P.brec += (size_t)b0 * g.G * NS;
  if (P.cpart) P.cpart += (size_t)b0 * g.H * k5_tq_n(g) * 2 * g.C;
  return P;
}

// The fused ∂x + ∂offset kernel (deform_groups 1, C % 4 == 0, C <= 256) over packed bins.
// r01 A/B at config 3 (2-deep prefetch pipeline): U=2 0.92 ms col2im, U=4 0.93, U=8 1.50;
// 4x6 tiles 1.05x slower, 4x8 tiles no longer unroll (2.7 ms). r02: column sweeps and
// strips without the tile's bin-row re-read measured no faster (DESIGN.md §4 "K5").
#ifndef K5B_WPE
#define K5B_WPE 4
#endif
#ifndef K5B_U
#define K5B_U 4
#endif
template <int U, int TQ, int WPE, int TR, typename GT, typename XT>
static void launch_c2i(const Geo& g, const XT* xT, const BinsWs& P, const GT* gcolT, float* gxT,
                       float* goff, int b0, int nb, hipStream_t s) {
  static_assert(TQ == kK5TQ, "cpart is sized for kK5TQ tile columns");
  const int tr_n = (g.H + TR - 1) / TR, tq_n = (g.W + TQ - 1) / TQ;
  hipLaunchKernelGGL((col2im_tile<U, TQ, GT, XT, WPE, TR>), dim3(tr_n * tq_n, 1, nb),
                     dim3((TR + 1) * 64), 0, s, g, xT, P.brec, P.start, gcolT, gxT, goff, P.cpart,
                     b0, tq_n);
  if (tq_n > 1) {
    const size_t n = (size_t)nb * g.H * (tq_n - 1) * (g.C / 4);
    hipLaunchKernelGGL(col2im_fold, dim3((unsigned)std::min<size_t>((n + 255) / 256, 8192)),
                       dim3(256), 0, s, g, reinterpret_cast<const float4*>(P.cpart),
                       reinterpret_cast<float4*>(gxT), b0, nb, tq_n, TQ);
  }
}

template <typename GT, typename XT>
static void launch_k5_fused(const Geo& g, const XT* xT, const BinsWs& P, const GT* gcolT,
                            float* gxT, float* goff, int b0, int nb, hipStream_t s) {
  // U rows in flight per wave. r02 (per-batch conditional loads): bf16 rows kept raw (8 B
  // per lane) until consumed: config 4 0.189 (U = 2, converted at load) -> 0.162 (U = 2 raw)
  // -> 0.154 ms (U = 3 raw). Tile rows (kTR; kTR + 1 waves per workgroup): 4 -> 7 (r02) cuts the bin rows read twice
  // (a tile re-reads the bin row it shares with the tile below: 5/4 -> 8/7 of the ∂col rows)
  // at the same 24 waves per CU (3 workgroups of 8, 40 KB of window each). Config 3 fp32 /
  // config 4 bf16: kTR 4 0.667 / 0.152 ms, 5 0.651 / 0.163, 6 0.630 / 0.151, 7 0.568 / 0.129,
  // 8 (2 workgroups per CU) 0.658 / 0.167, 11 0.585 / 0.137.
  // r03 (segmented records, packed math; A/B at config 3 / config 4, col2im scope incl. the
  // fold): fp32 U = 2 at 6 waves/SIMD spills 24 B: 0.669-0.673 ms; U = 2 at 5: 0.571;
  // U = 3 at 5 (95 VGPRs): 0.564-0.568; U = 3 at 4: 0.565. bf16 U = 3 at 5: 0.123-0.124,
  // U = 4 at 5: 0.123, U = 3 at 6 (spills): 0.146.
  // r04: 4 waves/SIMD (128 VGPRs): two 8-wave workgroups per CU is all that 5 allowed too, and
  // the batched ∂offset tree (wave_sum8) spills at 5 in the fp32 form. A/B at configs 3 / 4
  // (profiles/r04_k5_shapes.txt, one box): U = 3 0.514-0.520 / 0.116 ms; U = 4 0.515 / 0.111-0.113;
  // 5-wave workgroups at 5 waves/SIMD (20 waves per CU), bf16 U = 3: 0.134-0.136; both at U = 2:
  // 0.538-0.542 / 0.144-0.147. More rows per wave pays, more (smaller) workgroups do not.
  // r05: the bf16 window in LDS is bf16 (28 KB per workgroup instead of 46): the launch shape
  // of the bf16 instance is K5B_U rows per batch at K5B_WPE waves per SIMD (A/B builds)
  if constexpr (sizeof(XT) == 2)
    launch_c2i<K5B_U, 4, K5B_WPE, 7>(g, xT, P, gcolT, gxT, goff, b0, nb, s);
  else
    launch_c2i<4, 4, 4, 7>(g, xT, P, gcolT, gxT, goff, b0, nb, s);
}

hipError_t launch_col2im_coord(const Geo& g, const float* x, const float* xT, const float* off,
                               const float* gcolT, float* gx, float* gxT, float* goff,
                               void* bins_ws, int b0, int nb, bool bins_ready, hipStream_t s,
                               int bins_nb) {
  if (nb <= 0) return hipSuccess;
  if (bins_nb > 0 && (!bins_ready || !col2im_chunkable(g))) return hipErrorInvalidValue;
  hipError_t e;
  if (g_force_generic) {
    if (!gx) return hipErrorInvalidValue;  // the generic kernels accumulate into NCHW gx
    e = hipMemsetAsync(gx + (size_t)b0 * g.C * g.HWi, 0, (size_t)nb * g.C * g.HWi * sizeof(float),
                       s);
    if (e != hipSuccess) return e;
    const long total = (long)nb * g.G * g.N * g.HW;
    hipLaunchKernelGGL(col2im_generic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, g,
                       x, off, gcolT, gx, goff, b0, nb);
    return hipGetLastError();
  }
  const bool v4 = can_vec4(g);
  const LaneMap L = lane_map(g.Cg, v4 ? 4 : 1);
  const int NS = g.HW * g.N;
  const bool fused = k5_fused(g);
  if (!fused) {  // K5a: ∂offset
    dim3 grid((NS + 255) / 256, g.G, nb);
    if (v4)
      hipLaunchKernelGGL(offgrad_cl<4>, grid, dim3(256), 0, s, g, L, xT, off, gcolT, goff, b0);
    else
      hipLaunchKernelGGL(offgrad_cl<1>, grid, dim3(256), 0, s, g, L, xT, off, gcolT, goff, b0);
  }
  if (!bins_ready) {  // K5b (dcn_backward builds the bins on its side stream beforehand)
    e = launch_bins(g, off, bins_ws, goff, b0, nb, s);
    if (e != hipSuccess) return e;
  }
  const BinsWs P = bins_view(g, bins_ws, b0, nb, bins_nb);
  if (fused) {  // one pass over ∂colT: ∂xT + ∂offset of the owned bins
    launch_k5_fused(g, xT, P, gcolT, gxT, goff, b0, nb, s);
  } else {  // gather ∂xT, then back to NCHW (overwrites gx for these images)
    const int pix_per_block = 4 * L.SP;
    dim3 grid((g.HWi + pix_per_block - 1) / pix_per_block, g.G, nb);
    if (v4)
      hipLaunchKernelGGL(dx_gather_cl<4>, grid, dim3(256), 0, s, g, L, P.rec, P.start, P.slist,
                         gcolT, gxT, b0);
    else
      hipLaunchKernelGGL(dx_gather_cl<1>, grid, dim3(256), 0, s, g, L, P.rec, P.start, P.slist,
                         gcolT, gxT, b0);
  }
  if (!gx) return hipGetLastError();  // caller finalises ∂x from gxT (offset-conv ∂x pass)
  return launch_nhwc_to_nchw(gxT + (size_t)b0 * g.HWi * g.C, gx + (size_t)b0 * g.C * g.HWi, nb,
                             g.C, g.HWi, s);
}

// ---- DCN_BF16: bf16 column rows through the same LDS-window / fused kernels ----------
bool bf16_path_ok(const Geo& g) { return g.G == 1 && g.N <= kMaxTaps && g.C % 4 == 0 && g.C <= 256; }

hipError_t launch_im2col_bf16(const Geo& g, const bf16_t* xT, const float* off, bf16_t* colT,
                              int b0, int nb, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  auto go = [&](auto kern, int TH, int TW) {
    const int th_n = (g.Ho + TH - 1) / TH, tw_n = (g.Wo + TW - 1) / TW;
    hipLaunchKernelGGL(kern, dim3(th_n * tw_n, 1, nb), dim3(256), 0, s, g, xT, off, colT, b0,
                       tw_n);
  };
  if (g.C % 8 == 0 && g.C > 128)
    go(im2col_lds_b8<4, 4, 1, 256>, 4, 4);
  else if (g.C <= 32)
    go(im2col_lds<8, 8, 2, 32, true, bf16_t, bf16_t>, 8, 8);
  else if (g.C <= 64)
    go(im2col_lds<8, 8, 2, 64, true, bf16_t, bf16_t>, 8, 8);
  else if (g.C <= 128)
    go(im2col_lds<4, 4, 1, 128, true, bf16_t, bf16_t>, 4, 4);
  else
    go(im2col_lds<4, 4, 1, 256, true, bf16_t, bf16_t>, 4, 4);
  return hipGetLastError();
}

hipError_t launch_col2im_bf16(const Geo& g, const bf16_t* xT, const float* off,
                              const bf16_t* gcolT, float* gx, float* gxT, float* goff,
                              void* bins_ws, int b0, int nb, bool bins_ready, hipStream_t s,
                              int bins_nb) {
  if (nb <= 0) return hipSuccess;
  if (bins_nb > 0 && !bins_ready) return hipErrorInvalidValue;
  if (!bins_ready) {
    const hipError_t e = launch_bins(g, off, bins_ws, goff, b0, nb, s);
    if (e != hipSuccess) return e;
  }
  const BinsWs P = bins_view(g, bins_ws, b0, nb, bins_nb);
  launch_k5_fused(g, xT, P, gcolT, gxT, goff, b0, nb, s);
  if (!gx) return hipGetLastError();
  return launch_nhwc_to_nchw(gxT + (size_t)b0 * g.HWi * g.C, gx + (size_t)b0 * g.C * g.HWi, nb,
                             g.C, g.HWi, s);
}

}  // namespace dcn


