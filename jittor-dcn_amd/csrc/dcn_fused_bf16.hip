// dcn_fused_bf16.hip — f2 for DCN_BF16: the deformable im2col gathered straight into the B
// operand of bf16 MFMAs (out = Wf · colᵀ + bias, deform_conv.py:41-80), so the forward never
// reads a column matrix back from HBM; the columns are written only when the caller keeps
// them for the ∂W GEMM of the backward (colT != NULL).
//
// Workgroup = one output tile of kTH × kTW pixels (7 × 16 = 112 slots = 7 MFMA column blocks
// of 16) × 256 output channels; 4 waves, wave w owns output channels 64w..64w+63 (4 row
// blocks of 16) over all 112 slots: 28 accumulators of v_mfma_f32_16x16x32_bf16.
//
//   * Sample records (prologue): per slot and tap the reference coordinate chain
//     (sample_tap: deform_conv.py:34-39,62-68, Q1-Q4), reduced to the four bilinear weights
//     (the canonical products (1-fr)(1-fc), (1-fr)fc, fr(1-fc), fr·fc of bilerp()) and where
//     the corners are: in the LDS window, in the overflow area, or nowhere (zero).
//   * x window (per 64-channel slice): the tile's zero-offset footprint with a 2-pixel margin
//     (rows follow w, columns follow h: Q1) of the channels-last bf16 xT, staged in LDS;
//     pixels outside the image hold zeros (grid_sample zeros padding).
//   * Overflow: samples whose corners leave the window have their 64-channel column slice
//     built once per slice from global memory (issued with the window loads, one latency),
//     up to kOvf per tile; beyond that a sample reads its corners from global memory in line.
//   * k loop: k = n·C + c in the order (slice, tap, 32-channel half). Per step the block
//     gathers the [112 slots][32 channels] B tile into one of two LDS buffers (one 8-channel
//     unit = 4 corner reads of 16 B, fp32 bilerp in bilerp()'s op order, one bf16 rounding:
//     the bits of K1's columns) while the MFMAs consume the other; A fragments (the weights,
//     pre-swizzled into MFMA lane order) come from L2 one step ahead. One barrier per step.
//   * Epilogue: bf16(acc + bias[o]) straight to NCHW out (launch_bias_to_bf16's rounding).
#include <algorithm>
#include <climits>
#include <mutex>
#include <vector>

#include "dcn_device.h"
#include "dcn_swizzle.h"

namespace dcn {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ void col_store(T v, T* p) {
  __builtin_nontemporal_store(v, p);
}
constexpr int kTH = 7, kTW = 16;  // output tile rows (h) × columns (w)
constexpr int kPB = kTH * kTW / 16;  // 16-slot MFMA column blocks
constexpr int kSlots = kPB * 16;
constexpr int kMar = 2;
constexpr int kWR = kTW + 2 * kMar, kWQ = kTH + 2 * kMar;  // window rows (follow w), cols (h)
constexpr int kWPix = kWR * kWQ;
constexpr int kCS = 64;               // channels per window slice
constexpr int kWPitch = 2 * kCS + 16;  // bytes per window pixel (16 B pad: bank spread)
constexpr int kBPitch = 80;           // bytes per slot of a B tile (32 channels + 16 B pad)
constexpr int kMaxN = 9;
constexpr int kOvf = 48;              // overflow samples per tile with a precomputed slice
constexpr int kUnits = kSlots * 4;    // 8-channel units per step (448)
constexpr int kOT = 256;              // output channels per workgroup

constexpr int kLdsWin = 0;
constexpr int kLdsB = kLdsWin + kWPix * kWPitch;
constexpr int kLdsRecW = kLdsB + 2 * kSlots * kBPitch;
constexpr int kLdsRecM = kLdsRecW + kSlots * kMaxN * 16;
constexpr int kLdsOvfT = kLdsRecM + kSlots * kMaxN * 4;
constexpr int kLdsOvfD = kLdsOvfT + kOvf * 16;
constexpr int kLdsCnt = kLdsOvfD + kOvf * 2 * kCS;
constexpr int kLds = kLdsCnt + 16;
static_assert(kLds <= 80 * 1024, "two workgroups per CU");

constexpr int kMZero = -1;  // record meta: sample contributes 0 (or slot outside the output)
// meta >= 0: window pixel of corner (r0, c0); meta = -2 - j: overflow entry j (j < kOvf) or,
// for j >= kOvf, corners read from global memory in line

// bilerp() with its weight products precomputed (same products, same op order); each
// 32-bit word (2 channels) of the four corners is unpacked where it is used, and the two
// channels go through packed fp32 math (v_pk_mul_f32 / v_pk_fma_f32: per lane the same
// roundings as the scalar mul / fmaf chain, half the instructions)
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v unpack2(unsigned a) {
  return f32x2v{__uint_as_float(a << 16), __uint_as_float(a & 0xffff0000u)};
}
__device__ __forceinline__ unsigned blend2(float4 wv, unsigned a, unsigned b, unsigned c,
                                           unsigned d) {
  f32x2v v = f32x2v{wv.x, wv.x} * unpack2(a);
  v = __builtin_elementwise_fma(f32x2v{wv.y, wv.y}, unpack2(b), v);
  v = __builtin_elementwise_fma(f32x2v{wv.z, wv.z}, unpack2(c), v);
  v = __builtin_elementwise_fma(f32x2v{wv.w, wv.w}, unpack2(d), v);
  return (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
}
__device__ __forceinline__ uint4 blend8(float4 wv, uint4 ua, uint4 ub, uint4 uc, uint4 ud) {
  return make_uint4(blend2(wv, ua.x, ub.x, uc.x, ud.x), blend2(wv, ua.y, ub.y, uc.y, ud.y),
                    blend2(wv, ua.z, ub.z, uc.z, ud.z), blend2(wv, ua.w, ub.w, uc.w, ud.w));
}

__device__ __forceinline__ uint4 ld16_if(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}

// the 8 channels at c of sample (r0, c0) from global memory (corners outside the image: 0)
__device__ __forceinline__ uint4 gather_global(const Geo& g, const bf16_t* __restrict__ xb, int r0,
                                               int c0, int c, float4 wv) {
  const bool r0ok = r0 >= 0, r1ok = r0 + 1 < g.H, c0ok = c0 >= 0, c1ok = c0 + 1 < g.W;
  const long rs = (long)g.W * g.C;
  const bf16_t* p00 = xb + ((long)r0 * g.W + c0) * (long)g.C + c;
  const uint4 ua = ld16_if(p00, r0ok && c0ok);
  const uint4 ub = ld16_if(p00 + g.C, r0ok && c1ok);
  const uint4 uc = ld16_if(p00 + rs, r1ok && c0ok);
  const uint4 ud = ld16_if(p00 + rs + g.C, r1ok && c1ok);
  return blend8(wv, ua, ub, uc, ud);
}

__device__ __forceinline__ bf16x8_t as_frag(uint4 u) { return __builtin_bit_cast(bf16x8_t, u); }
// native-vector forms for the ∂W kernel (HIP's uint4 arrays captured by lambdas can end up in
// scratch memory)
__device__ __forceinline__ bf16x8_t as_frag(v4u u) { return __builtin_bit_cast(bf16x8_t, u); }
__device__ __forceinline__ v4u as_v(uint4 u) { return __builtin_bit_cast(v4u, u); }
__device__ __forceinline__ v4u ld16v_if(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const v4u*>(p) : v4u{0u, 0u, 0u, 0u};
}
__device__ __forceinline__ v4u blend8(float4 wv, v4u ua, v4u ub, v4u uc, v4u ud) {
  return v4u{blend2(wv, ua.x, ub.x, uc.x, ud.x), blend2(wv, ua.y, ub.y, uc.y, ud.y),
             blend2(wv, ua.z, ub.z, uc.z, ud.z), blend2(wv, ua.w, ub.w, uc.w, ud.w)};
}

// wfr[ob][ks][lane][8] = Wf[16·ob + (lane & 15)][32·ks + 8·(lane >> 4) + e]: the A fragment of
// v_mfma_f32_16x16x32_bf16 for output-channel block ob and k step ks, one 16-B load per lane;
// one thread per fragment (the 8 elements are contiguous in Wf: one 16-B load and store)
__global__ __launch_bounds__(256) void wf_to_frag16(const bf16_t* __restrict__ w,
                                                    bf16_t* __restrict__ wfr, int O, int K) {
  const long f = (long)blockIdx.x * 256 + threadIdx.x;  // fragment = (ob, ks, lane)
  if (f < (long)O * K / 8) swz_frag16(w, wfr, K, f);
}

template <bool STORE>
__global__ __launch_bounds__(256, 2) void fwd_fused_bf16(Geo g, const bf16_t* __restrict__ xT,
                                                         const float* __restrict__ off,
                                                         const bf16_t* __restrict__ wfr,
                                                         const float* __restrict__ bias,
                                                         bf16_t* __restrict__ out,
                                                         bf16_t* __restrict__ colT, int tw_n) {
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  char* const win = lds + kLdsWin;
  char* const bt = lds + kLdsB;
  float4* const recw = reinterpret_cast<float4*>(lds + kLdsRecW);
  int* const recm = reinterpret_cast<int*>(lds + kLdsRecM);
  int4* const ovft = reinterpret_cast<int4*>(lds + kLdsOvfT);
  char* const ovfd = lds + kLdsOvfD;
  int* const cnt = reinterpret_cast<int*>(lds + kLdsCnt);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Block3 blk = xcd_block();
  const int b = blk.y;
  const int th_i = blk.x / tw_n, tw_i = blk.x - th_i * tw_n;
  const int h0 = th_i * kTH, w0 = tw_i * kTW;
  const int o0 = blk.z * kOT + 64 * wave;
  const int rlo = (int)floorf((float)w0 * (float)(g.H - 1) / (float)(g.Wo - 1)) - kMar;
  const int qlo = (int)floorf((float)h0 * (float)(g.W - 1) / (float)(g.Ho - 1)) - kMar;
  const bf16_t* const xb = xT + (size_t)b * g.HWi * g.C;
  const int N = g.N;

  // window slice cs: kWPix pixels × 8 parts of 16 B (zeros outside the image)
  // r05: through a buffer resource (a position outside the image reads 0 by the range check):
  // the conditional loads of ld16_if were exec-masked branches, and hipcc waited for all loads
  // in flight (vmcnt(0)) before several of them
  const auto rxb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(xb), 0,
                                                     (int)((size_t)g.HWi * g.C * 2), 0x00020000);
  auto win_load = [&](int cs, uint4 (&v)[(kWPix * 8 + 255) / 256]) {
    constexpr int TOT = kWPix * 8, IT = (TOT + 255) / 256;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int idx = tid + k * 256;
      const int pix = idx >> 3, part = idx & 7;
      const int rr = pix / kWQ, qq = pix - rr * kWQ;
      const int r = rlo + rr, q = qlo + qq;
      const bool ok = (idx < TOT) & ((unsigned)r < (unsigned)g.H) & ((unsigned)q < (unsigned)g.W);
      const unsigned o = ok ? (unsigned)(((r * g.W + q) * g.C + kCS * cs + 8 * part) * 2) : 0x80000000u;
      const auto qv = __builtin_amdgcn_raw_buffer_load_b128(rxb, o, 0, 0);
      v[k] = make_uint4(qv[0], qv[1], qv[2], qv[3]);
    }
  };
  // (r05 A/B: slice 0's window loaded before the records instead, slower: 0.152-0.155 vs
  // 0.142-0.143 ms, the window registers live across the records loop)

  // ---- records ----
  if (tid == 0) cnt[0] = 0;
  __syncthreads();
  for (int s = tid; s < kSlots * N; s += 256) {
    const int p = s / N, n = s - p * N;
    const int h = h0 + p / kTW, w = w0 + p % kTW;
    int meta = kMZero;
    float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h < g.Ho && w < g.Wo) {
      const Tap t = sample_tap(g, off, b, 0, n, h * g.Wo + w);
      if (t.ok) {
        const float gr = 1.0f - t.fr, gc = 1.0f - t.fc;
        wv = make_float4(gr * gc, gr * t.fc, t.fr * gc, t.fr * t.fc);
        const int rr = t.r0 - rlo, qq = t.c0 - qlo;
        if (rr >= 0 && rr + 1 < kWR && qq >= 0 && qq + 1 < kWQ) {
          meta = rr * kWQ + qq;
        } else {
          const int j = atomicAdd(cnt, 1);  // any order: each entry is computed on its own
          meta = -2 - j;
          if (j < kOvf) ovft[j] = make_int4(t.r0, t.c0, p * kMaxN + n, 0);
        }
      }
    }
    recm[p * kMaxN + n] = meta;
    recw[p * kMaxN + n] = wv;
  }
  __syncthreads();
  const int novf = min(cnt[0], kOvf);

  // ---- per-thread production units: u = tid, tid + 256 (u < kUnits): slot u>>2, 8-ch group u&3
  // (wave-uniform count: waves 0-2 hold two unit sets, wave 3 one)
  const int nu = (tid + 256 < kUnits) ? 2 : 1;
  int uslot[2], ucg[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int u = min(tid + 256 * k, kUnits - 1);
    uslot[k] = u >> 2;
    ucg[k] = u & 3;
  }
  // column stores (STORE): a wave's unit set k covers slots 16·wave + 64k + 0..15, the two
  // 32-channel halves of one tap in consecutive steps (B buffers 0 and 1). After the second
  // half, lane L stores 16-B piece L & 7 of slot 16·wave + 64k + 8i + (L >> 3)'s 128-B column
  // line (i = 0, 1), read back from the two B buffers: every store instruction writes 8 whole
  // lines (half-line stores one step apart wrote 1.15x the column bytes).
  // The slots' column rows are recomputed per store (registers are at the kernel's limit).

  f32x4 acc[4][kPB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < kPB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int NKS = g.K / 32;
  const int spq = 2 * N;  // steps per slice
  const int nslices = g.C / kCS;
  // A fragments of step s of slice cs: k = n·C + 64·cs + 32·half
  auto load_a = [&](int cs, int s, uint4 (&a)[4]) {
    const int ks = ((s >> 1) * g.C + kCS * cs + 32 * (s & 1)) >> 5;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const uint4*>(
          wfr + ((size_t)(((o0 >> 4) + i) * NKS + ks) * 64 + lane) * 8);
  };
  // gather step s of slice cs into B buffer buf (and, with STORE, the column rows)
  auto produce = [&](int cs, int s, int buf) {
    const int n = s >> 1, hh = s & 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < nu) {
        const int slot = uslot[k], cg = ucg[k];
        const int meta = recm[slot * kMaxN + n];
        uint4 o = make_uint4(0u, 0u, 0u, 0u);
        if (meta >= 0) {
          const float4 wv = recw[slot * kMaxN + n];
          const char* wp = win + meta * kWPitch + hh * 64 + cg * 16;
          const uint4 ua = *reinterpret_cast<const uint4*>(wp);
          const uint4 ub = *reinterpret_cast<const uint4*>(wp + kWPitch);
          const uint4 uc = *reinterpret_cast<const uint4*>(wp + kWQ * kWPitch);
          const uint4 ud = *reinterpret_cast<const uint4*>(wp + (kWQ + 1) * kWPitch);
          o = blend8(wv, ua, ub, uc, ud);
        } else if (meta != kMZero) {
          const int j = -2 - meta;
          if (j < kOvf) {
            o = *reinterpret_cast<const uint4*>(ovfd + j * 2 * kCS + hh * 64 + cg * 16);
          } else {  // more overflow samples than the area holds: corners from global memory
            const int h = h0 + slot / kTW, w = w0 + slot % kTW;
            const Tap t = sample_tap(g, off, b, 0, n, h * g.Wo + w);
            o = gather_global(g, xb, t.r0, t.c0, kCS * cs + 32 * hh + 8 * cg,
                              recw[slot * kMaxN + n]);
          }
        }
        *reinterpret_cast<uint4*>(bt + buf * kSlots * kBPitch + slot * kBPitch + cg * 16) = o;
      }
    }
  };
  // both halves of tap n of slice cs are in the B buffers (0: channels 0-31, 1: 32-63): each
  // wave stores its own slots' whole column lines (no other wave writes those slots' units,
  // and this wave's next production comes after this in program order)
  auto store_cols = [&](int cs, int n) {
    const int j = lane & 7;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < nu) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int sl = 16 * wave + 64 * k + 8 * i + (lane >> 3);
          const v4u v = *reinterpret_cast<const v4u*>(bt + (j >> 2) * kSlots * kBPitch +
                                                      sl * kBPitch + (j & 3) * 16);
          const int h = h0 + sl / kTW, w = w0 + sl % kTW;
          if (sl < kSlots && h < g.Ho && w < g.Wo)
            col_store(
                v, reinterpret_cast<v4u*>(colT + (size_t)b * g.HW * g.K +
                                          (unsigned)(h * g.Wo + w) * (unsigned)g.K +
                                          (n * g.C + kCS * cs + 8 * j)));
        }
      }
    }
  };
  auto mfma_step = [&](int buf, const uint4 (&a)[4]) {
    const char* bb = bt + buf * kSlots * kBPitch + (lane & 15) * kBPitch + (lane >> 4) * 16;
#pragma unroll
    for (int pb = 0; pb < kPB; ++pb) {
      const bf16x8_t bv = as_frag(*reinterpret_cast<const uint4*>(bb + pb * 16 * kBPitch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a[i]), bv, acc[i][pb], 0, 0, 0);
    }
  };

  uint4 aE[4], aO[4];
  for (int cs = 0; cs < nslices; ++cs) {
    __syncthreads();  // the previous slice's window, overflow and B tiles are consumed
    {
      // window slice: kWPix pixels × 8 parts of 16 B; overflow corners loaded alongside
      constexpr int TOT = kWPix * 8, IT = (TOT + 255) / 256;
      uint4 v[IT];
      win_load(cs, v);
      // overflow: novf entries × 8 units of 8 channels
      uint4 ov[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int idx = tid + 256 * k;
        ov[k] = make_uint4(0u, 0u, 0u, 0u);
        if (idx < novf * 8) {
          const int4 e = ovft[idx >> 3];
          ov[k] = gather_global(g, xb, e.x, e.y, kCS * cs + 8 * (idx & 7), recw[e.z]);
        }
      }
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int idx = tid + k * 256;
        if (idx < TOT)
          *reinterpret_cast<uint4*>(win + (idx >> 3) * kWPitch + (idx & 7) * 16) = v[k];
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int idx = tid + 256 * k;
        if (idx < novf * 8)
          *reinterpret_cast<uint4*>(ovfd + (idx >> 3) * 2 * kCS + (idx & 7) * 16) = ov[k];
      }
    }
    load_a(cs, 0, aE);
    __syncthreads();
    produce(cs, 0, 0);
    __syncthreads();
    for (int s = 0; s < spq; s += 2) {
      load_a(cs, s + 1, aO);
      produce(cs, s + 1, 1);
      mfma_step(0, aE);
      __syncthreads();
      if (STORE) store_cols(cs, s >> 1);
      if (s + 2 < spq) {
        load_a(cs, s + 2, aE);
        produce(cs, s + 2, 0);
      }
      mfma_step(1, aO);
      __syncthreads();
    }
  }

  // ---- epilogue: out[b][o][h][w] = bf16(acc + bias[o]) (launch_bias_to_bf16's rounding).
  // The tile goes through LDS as [o][slot] (the window / B / record regions are free now) so
  // that each thread stores 8 consecutive pixels of one (o, h) as two 8-B runs instead of
  // 112 scattered 2-B stores per lane (r03: 15 us of the kernel's 140). C/D map: slot =
  // 16·pb + (lane & 15), o = 16·i + 4·(lane >> 4) + r.
  constexpr int kEP = kSlots * 2 + 16;  // bytes per output-channel row of the staged tile
  static_assert(kOT * kEP <= kLdsOvfT, "staged output tile fits the freed LDS");
  __syncthreads();  // every wave is past its last B-tile read
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ol = 64 * wave + 16 * i + 4 * (lane >> 4) + r;
      const float bv = bias ? bias[o0 - 64 * wave + ol] : 0.f;
#pragma unroll
      for (int pb = 0; pb < kPB; ++pb)
        *reinterpret_cast<bf16_t*>(lds + ol * kEP + (16 * pb + (lane & 15)) * 2) =
            f2bf(acc[i][pb][r] + bv);
    }
  __syncthreads();
  // 8-pixel runs: (output channel, tile row, half row)
  const int ob0 = blk.z * kOT;
  for (int u = tid; u < kOT * kTH * 2; u += 256) {
    const int half = u & 1, rest = u >> 1;
    const int th = rest % kTH, ol = rest / kTH;
    const int h = h0 + th, wc = w0 + 8 * half;
    if (h >= g.Ho || wc >= g.Wo) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + ol * kEP + (16 * th + 8 * half) * 2);
    bf16_t* op = out + ((size_t)b * g.O + ob0 + ol) * g.HW + (size_t)h * g.Wo + wc;
    if (wc + 8 <= g.Wo && ((reinterpret_cast<uintptr_t>(op) & 7) == 0)) {
      *reinterpret_cast<uint2*>(op) = make_uint2(v.x, v.y);
      *reinterpret_cast<uint2*>(op + 4) = make_uint2(v.z, v.w);
    } else {
      const unsigned e[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; j < 8 && wc + j < g.Wo; ++j)
        op[j] = (bf16_t)((e[j >> 1] >> (16 * (j & 1))) & 0xffffu);
    }
  }
}

// ---------------------------------------------------------------------------------------
// ∂W with the columns recomputed (f2's backward half): ∂Wf[o][n·C + c] = Σ_p ∂out[o][p] ·
// col[p][n·C + c] (the autodiff of deform_conv.py:76), the bilinear samples gathered from an
// LDS window straight into the B operand, so no column matrix exists in HBM.
//
// Workgroup = (16-channel slice cs, image group, 256 output channels); 8 waves, wave w owns
// output channels 32w..32w+31 (2 row blocks) × all taps of the slice (N column blocks of 16):
// 2·N accumulators of v_mfma_f32_16x16x32_bf16. It walks the 7 × 16 pixel tiles of its
// images in a fixed order (the reduction over pixels, 4 k steps of 32 slots per tile, slots
// 112..127 zero); per tile it gathers the [N taps][16 channels][128 slots] column tile (2016
// units of 8 channels, written transposed with 32-bit LDS stores, two pixels per store) while
// the MFMAs consume the previous tile's; the next tile's window, offsets and ∂out fragments
// are loaded into registers a tile ahead. One barrier per tile. The window margin is 4 px,
// so a sample outside it (|Δ| > ~4 px) is rare and reads its corners from global memory.
// Partials per (image group) are summed in a fixed order afterwards (launch_sum_partials).
constexpr int kDC = 16;                       // channels per slice
constexpr int kDMar = 4;
constexpr int kDWR = kTW + 2 * kDMar, kDWQ = kTH + 2 * kDMar;
constexpr int kDWPix = kDWR * kDWQ;           // 360
constexpr int kDWPitch = 2 * kDC + 16;        // 48 B per window pixel
constexpr int kDSl = 128;                     // pixel slots per tile, padded to 4 k steps
constexpr int kDRow = kDSl * 2 + 16;          // bytes per [tap][channel] row of the col tile
constexpr int kDT = 512;
constexpr int kDOB = 2;
constexpr int kDLWin = 0;
constexpr int kDLCol = kDLWin + 2 * kDWPix * kDWPitch;
constexpr int kDLRecW = kDLCol + 2 * kMaxN * kDC * kDRow;
constexpr int kDLRecM = kDLRecW + 2 * kSlots * kMaxN * 16;
constexpr int kDLds = kDLRecM + 2 * kSlots * kMaxN * 4;
static_assert(kDLds <= 160 * 1024, "one workgroup per CU");
constexpr int kDSlow = -2;  // record meta: corners outside the window (global reads)

template <int NG>
__global__ __launch_bounds__(kDT) void dw_fused_bf16(Geo g, const bf16_t* __restrict__ xT,
                                                     const float* __restrict__ off,
                                                     const bf16_t* __restrict__ gout,
                                                     float* __restrict__ parts, int tw_n,
                                                     int ngrp) {
  extern __shared__ __attribute__((aligned(16))) char dl[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware order: the channel slices of one image group share an XCD, so its L2 serves
  // them the group's ∂out fragments and x windows
  const Block3 blk = xcd_block();
  const int cs = blk.x, grp = blk.y;
  const int o0 = blk.z * kOT + 16 * kDOB * wave;
  const int N = g.N;
  const int tiles_img = ((g.Ho + kTH - 1) / kTH) * tw_n;
  const int b_lo = (int)((long)grp * g.B / ngrp), b_hi = (int)((long)(grp + 1) * g.B / ngrp);
  const int T = (b_hi - b_lo) * tiles_img;

  struct TileId {
    int b, h0, w0, rlo, qlo;
  };
  auto tile_id = [&](int t) {
    TileId q;
    const int ti = t % tiles_img;
    q.b = b_lo + t / tiles_img;
    q.h0 = (ti / tw_n) * kTH;
    q.w0 = (ti % tw_n) * kTW;
    q.rlo = (int)floorf((float)q.w0 * (float)(g.H - 1) / (float)(g.Wo - 1)) - kDMar;
    q.qlo = (int)floorf((float)q.h0 * (float)(g.W - 1) / (float)(g.Ho - 1)) - kDMar;
    return q;
  };
  // window slice of tile t: kDWPix pixels × 2 parts of 16 B (two per thread)
  constexpr int kWL = (kDWPix * 2 + kDT - 1) / kDT;
  auto win_load = [&](const TileId& q, v4u (&v)[kWL]) {
    const bf16_t* xb = xT + (size_t)q.b * g.HWi * g.C + kDC * cs;
#pragma unroll
    for (int k = 0; k < kWL; ++k) {
      const int idx = tid + k * kDT;
      const int pix = idx >> 1, part = idx & 1;
      const int rr = pix / kDWQ, qq = pix - rr * kDWQ;
      const int r = q.rlo + rr, qc = q.qlo + qq;
      const bool ok = idx < kDWPix * 2 && r >= 0 && r < g.H && qc >= 0 && qc < g.W;
      v[k] = ld16v_if(xb + ((size_t)r * g.W + qc) * g.C + 8 * part, ok);
    }
  };
  auto win_store = [&](int buf, const v4u (&v)[kWL]) {
    char* wb = dl + kDLWin + buf * kDWPix * kDWPitch;
#pragma unroll
    for (int k = 0; k < kWL; ++k) {
      const int idx = tid + k * kDT;
      if (idx < kDWPix * 2) *reinterpret_cast<v4u*>(wb + (idx >> 1) * kDWPitch + (idx & 1) * 16) = v[k];
    }
  };
  // records of tile t: the offsets (Δx, Δy) of its (slot, tap) samples, two per thread
  constexpr int kRL = (kSlots * kMaxN + kDT - 1) / kDT;
  auto rec_load = [&](const TileId& q, float (&dx)[kRL], float (&dy)[kRL]) {
    const float* ob = off + (size_t)q.b * g.J * g.HW;
#pragma unroll
    for (int k = 0; k < kRL; ++k) {
      const int sidx = tid + k * kDT;
      const int p = sidx / N, n = sidx - p * N;
      const int h = q.h0 + p / kTW, w = q.w0 + p % kTW;
      const bool ok = sidx < kSlots * N && h < g.Ho && w < g.Wo;
      const int m = ok ? h * g.Wo + w : 0;
      dx[k] = ok ? ob[(size_t)n * g.HW + m] : 0.f;
      dy[k] = ok ? ob[(size_t)(N + n) * g.HW + m] : 0.f;
    }
  };
  auto rec_store = [&](int buf, const TileId& q, const float (&dx)[kRL], const float (&dy)[kRL]) {
    float4* rw = reinterpret_cast<float4*>(dl + kDLRecW + buf * kSlots * kMaxN * 16);
    int* rm = reinterpret_cast<int*>(dl + kDLRecM + buf * kSlots * kMaxN * 4);
#pragma unroll
    for (int k = 0; k < kRL; ++k) {
      const int sidx = tid + k * kDT;
      if (sidx < kSlots * N) {
        const int p = sidx / N, n = sidx - p * N;
        const int h = q.h0 + p / kTW, w = q.w0 + p % kTW;
        int meta = kMZero;
        float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (h < g.Ho && w < g.Wo) {
          float iy, ix;
          ref_coord(h, w, dx[k], dy[k], g, iy, ix);
          const Tap t = make_tap(iy, ix, g);
          if (t.ok) {
            const float gr = 1.0f - t.fr, gc = 1.0f - t.fc;
            wv = make_float4(gr * gc, gr * t.fc, t.fr * gc, t.fr * t.fc);
            const int rr = t.r0 - q.rlo, qq = t.c0 - q.qlo;
            meta = (rr >= 0 && rr + 1 < kDWR && qq >= 0 && qq + 1 < kDWQ) ? rr * kDWQ + qq : kDSlow;
          }
        }
        rm[n * kSlots + p] = meta;
        rw[n * kSlots + p] = wv;
      }
    }
  };
  // A fragments of tile t: ∂out[b][o][slot] for slots 32·ks + 8·(lane >> 4) .. +7, rows
  // o0 + 16·ob + (lane & 15); slots outside the image (or >= 112) read as 0
  auto a_load = [&](const TileId& q, v4u (&a)[kDOB][4]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int sl = 32 * ks + 8 * (lane >> 4);  // 8 slots of one tile row (kTW = 16)
      const int h = q.h0 + sl / kTW, w = q.w0 + sl % kTW;
      const bool rowok = sl < kSlots && h < g.Ho;
      const int nv = rowok ? min(8, g.Wo - w) : 0;
#pragma unroll
      for (int ob = 0; ob < kDOB; ++ob) {
        const int o = o0 + 16 * ob + (lane & 15);
        const bf16_t* src = gout + ((size_t)q.b * g.O + o) * g.HW + (size_t)h * g.Wo + w;
        v4u v = {0u, 0u, 0u, 0u};
        if (nv >= 8 && ((reinterpret_cast<uintptr_t>(src) & 7) == 0)) {
          const uint2 lo = *reinterpret_cast<const uint2*>(src);
          const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
          v = v4u{lo.x, lo.y, hi.x, hi.y};
        } else if (nv > 0) {
          unsigned e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = j < nv ? (unsigned)src[j] : 0u;
          v = v4u{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
        }
        a[ob][ks] = v;
      }
    }
  };
  // the column tile of tile t (records / window buffer rb) into col buffer cb: pair-unit u =
  // (tap n, 8-channel group cg, slot pair sp), two per thread; consecutive lanes take
  // consecutive slot pairs, so the transposed 32-bit stores of a wave hit distinct banks
  auto produce = [&](const TileId& q, int rb, int cb) {
    const char* wb = dl + kDLWin + rb * kDWPix * kDWPitch;
    const float4* rw = reinterpret_cast<const float4*>(dl + kDLRecW + rb * kSlots * kMaxN * 16);
    const int* rm = reinterpret_cast<const int*>(dl + kDLRecM + rb * kSlots * kMaxN * 4);
    char* col = dl + kDLCol + cb * kMaxN * kDC * kDRow;
    const bf16_t* xb = xT + (size_t)q.b * g.HWi * g.C + kDC * cs;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = tid + k * kDT;
      const int sp = u % (kSlots / 2), rest = u / (kSlots / 2);
      const int n = rest >> 1, cg = rest & 1;
      if (n < N) {
        v4u o2[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int slot = 2 * sp + e;
          const int meta = rm[n * kSlots + slot];
          const float4 wv = rw[n * kSlots + slot];
          const char* wp = wb + max(meta, 0) * kDWPitch + cg * 16;
          const v4u ua = *reinterpret_cast<const v4u*>(wp);
          const v4u ub = *reinterpret_cast<const v4u*>(wp + kDWPitch);
          const v4u uc = *reinterpret_cast<const v4u*>(wp + kDWQ * kDWPitch);
          const v4u ud = *reinterpret_cast<const v4u*>(wp + (kDWQ + 1) * kDWPitch);
          v4u o = blend8(wv, ua, ub, uc, ud);
          const v4u z = {0u, 0u, 0u, 0u};
          o = meta >= 0 ? o : z;
          if (__any(meta == kDSlow)) {
            if (meta == kDSlow) {
              const int h = q.h0 + slot / kTW, w = q.w0 + slot % kTW;
              const Tap t = sample_tap(g, off, q.b, 0, n, h * g.Wo + w);
              o = as_v(gather_global(g, xb, t.r0, t.c0, 8 * cg, wv));
            }
          }
          o2[e] = o;
        }
        // transposed: row (n, channel 8·cg + i), columns slot 2sp, 2sp+1 packed in 32 bits
        char* dst = col + (n * kDC + 8 * cg) * kDRow + 4 * sp;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned a0 = o2[0][i], a1 = o2[1][i];
          *reinterpret_cast<unsigned*>(dst + (2 * i) * kDRow) = (a0 & 0xffffu) | (a1 << 16);
          *reinterpret_cast<unsigned*>(dst + (2 * i + 1) * kDRow) = (a0 >> 16) | (a1 & 0xffff0000u);
        }
      }
    }
  };

  f32x4 acc[kDOB][kMaxN];
#pragma unroll
  for (int i = 0; i < kDOB; ++i)
#pragma unroll
    for (int n = 0; n < kMaxN; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma_tile = [&](int cb, const v4u (&a)[kDOB][4]) {
    const char* col = dl + kDLCol + cb * kMaxN * kDC * kDRow + (lane & 15) * kDRow + (lane >> 4) * 16;
#pragma unroll
    for (int n = 0; n < kMaxN; ++n) {
      if (n < N) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const v4u bv = *reinterpret_cast<const v4u*>(col + n * kDC * kDRow + ks * 64);
#pragma unroll
          for (int ob = 0; ob < kDOB; ++ob)
            acc[ob][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a[ob][ks]), as_frag(bv),
                                                               acc[ob][n], 0, 0, 0);
        }
      }
    }
  };

  // zero both col buffers once (slots 112..127 and unused taps stay zero)
  for (int i = tid * 16; i < 2 * kMaxN * kDC * kDRow; i += kDT * 16)
    *reinterpret_cast<v4u*>(dl + kDLCol + i) = v4u{0u, 0u, 0u, 0u};
  // raw window / offset loads of the tile after next, in two register sets used alternately
  // (named, not indexed, so no copy waits for a load still in flight)
  v4u wA[kWL], wB[kWL];
  float dxA[kRL], dyA[kRL], dxB[kRL], dyB[kRL];
  v4u aC[kDOB][4];
  if (T > 0) {
    const TileId q0 = tile_id(0);
    win_load(q0, wA);
    rec_load(q0, dxA, dyA);
    a_load(q0, aC);
    win_store(0, wA);
    rec_store(0, q0, dxA, dyA);
    if (T > 1) {
      const TileId q1 = tile_id(1);
      win_load(q1, wA);
      rec_load(q1, dxA, dyA);
    }
  }
  __syncthreads();
  // iteration t: gather tile t (buffers t & 1) beside the MFMAs of tile t - 1; then the
  // A fragments of tile t, and tile t + 1's window and records (loaded an iteration ago)
  // into the other buffers; tile t + 2's loads are issued first
  auto body = [&](int t, v4u (&wn)[kWL], float (&dxn)[kRL], float (&dyn)[kRL], v4u (&wf)[kWL],
                  float (&dxf)[kRL], float (&dyf)[kRL]) {
    const TileId q = tile_id(t);
    if (t + 2 < T) {
      const TileId qf = tile_id(t + 2);
      win_load(qf, wf);
      rec_load(qf, dxf, dyf);
    }
    produce(q, t & 1, t & 1);
    if (t > 0) mfma_tile((t - 1) & 1, aC);
    a_load(q, aC);
    if (t + 1 < T) {
      const TileId qn = tile_id(t + 1);
      win_store((t + 1) & 1, wn);
      rec_store((t + 1) & 1, qn, dxn, dyn);
    }
    __syncthreads();
  };
  for (int t = 0; t < T; t += 2) {
    body(t, wA, dxA, dyA, wB, dxB, dyB);
    if (t + 1 < T) body(t + 1, wB, dxB, dyB, wA, dxA, dyA);
  }
  if (T > 0) mfma_tile((T - 1) & 1, aC);

  // partial ∂Wf[o][n·C + 16·cs + ch] of this image group; C/D: col = lane & 15 (ch), row =
  // 4·(lane >> 4) + r (o)
  float* pg = parts + (size_t)grp * g.O * g.K;
#pragma unroll
  for (int ob = 0; ob < kDOB; ++ob)
#pragma unroll
    for (int n = 0; n < kMaxN; ++n) {
      if (n < N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = o0 + 16 * ob + 4 * (lane >> 4) + r;
          pg[(size_t)o * g.K + n * g.C + kDC * cs + (lane & 15)] = acc[ob][n][r];
        }
      }
    }
}

}  // namespace

bool fused_fwd_bf16_ok(const Geo& g) {
  const long lim = 1l << 31;
  return g.dt == DCN_BF16 && g.G == 1 && g.N <= kMaxN && g.C % kCS == 0 && g.O % kOT == 0 &&
         g.Ho >= 2 && g.Wo >= 2 && (long)g.O * g.K < lim &&
         (long)g.HW * g.K * 2 < lim &&  // an image's columns: 32-bit buffer byte offsets
         (long)g.HWi * g.C * 2 < lim;   // an image's xT (the window loads)
}

// r03 (tools/r03_fb_geo.py, fwd+bwd per step): fused faster wherever all
// output channels are one 256-channel tile — C = 64 / 128 / 192 / 256 at 28x28 (6-9 %), C = 256
// at 56x56 (6 %) — and slower with two tiles (O = 512, B = 16: 0.40 vs 0.37 ms), whose
// workgroups each repeat the gather. Only the measured range takes it: output maps of at least
// 28 x 28 pixels (small maps fill only part of each 7 x 16 tile and were not measured)
bool fused_fwd_bf16_pays(const Geo& g) { return g.O == kOT && g.HW >= 28 * 28; }

size_t fused_fwd_bf16_wfr_elems(const Geo& g) { return (size_t)g.O * g.K; }

PrepJob prep_frag16(const Geo& g, const bf16_t* w, bf16_t* wfr) {
  return PrepJob{PREP_FRAG16, (long)g.O * g.K / 8, w, wfr, 0, g.K, 0, 0, 0, 0};
}

hipError_t launch_fused_fwd_bf16(const Geo& g, const bf16_t* xT, const float* off,
                                 const bf16_t* w, bf16_t* wfr, const float* bias, bf16_t* out,
                                 bf16_t* colT, hipStream_t s, bool wfr_ready) {
  if (!fused_fwd_bf16_ok(g)) return hipErrorInvalidValue;
  const long nw = (long)g.O * g.K;
  if (!wfr_ready)
    hipLaunchKernelGGL(wf_to_frag16, dim3((unsigned)((nw / 8 + 255) / 256)), dim3(256), 0, s, w,
                       wfr, g.O, g.K);
  const int th_n = (g.Ho + kTH - 1) / kTH, tw_n = (g.Wo + kTW - 1) / kTW;
  const dim3 grid(th_n * tw_n, g.B, g.O / kOT);
  if (colT)
    hipLaunchKernelGGL(fwd_fused_bf16<true>, grid, dim3(256), 0, s, g, xT, off, wfr, bias, out,
                       colT, tw_n);
  else
    hipLaunchKernelGGL(fwd_fused_bf16<false>, grid, dim3(256), 0, s, g, xT, off, wfr, bias, out,
                       colT, tw_n);
  return hipGetLastError();
}

bool fused_dw_bf16_ok(const Geo& g) {
  return g.dt == DCN_BF16 && g.G == 1 && g.N <= kMaxN && g.C % kDC == 0 && g.O % kOT == 0 &&
         g.Ho >= 2 && g.Wo >= 2 && (long)g.O * g.K < (1l << 31) &&
         (long)g.B * g.O * g.HW < (1l << 40);
}

int fused_dw_bf16_groups(const Geo& g) { return std::min(16, g.B); }

hipError_t launch_fused_dw_bf16(const Geo& g, const bf16_t* xT, const float* off,
                                const bf16_t* gout, float* parts, hipStream_t s) {
  if (!fused_dw_bf16_ok(g)) return hipErrorInvalidValue;
  // the >64 KB dynamic-LDS attribute is per device: set once per device id, recorded only
  // after it succeeded (a failure is returned and retried on the next call)
  static std::mutex mu;
  static std::vector<char> attr_set;
  int dev = 0;
  {
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    if ((int)attr_set.size() <= dev) attr_set.resize(dev + 1, 0);
    if (!attr_set[dev]) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_fused_bf16<0>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kDLds);
      if (e != hipSuccess) return e;
      attr_set[dev] = 1;
    }
  }
  const int ng = fused_dw_bf16_groups(g);
  const int tw_n = (g.Wo + kTW - 1) / kTW;
  const dim3 grid(g.C / kDC, ng, g.O / kOT);
  hipLaunchKernelGGL(dw_fused_bf16<0>, grid, dim3(kDT), kDLds, s, g, xT, off, gout, parts, tw_n,
                     ng);
  return hipGetLastError();
}

}  // namespace dcn


