// fused_diag.hip — one-process diagnosis of the r02 bf16 fused forward's run-to-run corruption
// (VERDICT r02 "next" item 1; the kernel is commit 7965346's fwd_fused_bf16, removed in
// b01ff7a). Not part of libdcn: a standalone executable, test infrastructure only.
//
// It runs the kernel body of 7965346 (unchanged arithmetic and schedule) at config 4
// (B=64, C=O=256, 28x28, k3 s1 p1, bf16), several times in one process, in variants that
// each remove one suspect, and checks every launch against an independent reference:
//   * columns: bitwise against a one-thread-per-element gather (K1's arithmetic);
//   * out: bitwise against the variant's own first launch (determinism) and, with a
//     tolerance, against a plain fp32 GEMM over the reference columns.
// Mismatches are histogrammed by k step, by pixel of the tile, by wave and by lane group,
// which is what tells an LDS race (whole steps, all waves), a register overwrite (the lanes
// / steps whose registers the ISA reuses) and a store-side fault (columns only) apart.
//
// Variants (template STORE, BAR):
//   STORE 0: no column stores; 1: column stores as in 7965346; 2: stores, then
//            s_waitcnt vmcnt(0) right after each (the store's VGPRs read before reuse)
//   BAR   0: __syncthreads() per k step (7965346); 1: LDS-only barrier (r02 first form)
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../jittor-dcn_amd/csrc/dcn_device.h"

using namespace dcn;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8f_t __attribute__((ext_vector_type(8)));
constexpr int kFTaps = 9;
constexpr int kBNB = 2, kBP = 32 * kBNB, kBS = 40, kGD = 2;
constexpr int kAuxNT = 2;

__device__ __forceinline__ bf16x8f_t ld_frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8f_t, *reinterpret_cast<const uint4*>(p));
}
__device__ __forceinline__ float bfl(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bfh(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

__global__ void wf_to_frag_bf16(const bf16_t* __restrict__ w, bf16_t* __restrict__ wf, int O, int K) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)O * K) return;
  const int e = (int)(i & 7), l = (int)((i >> 3) & 63);
  const long obks = i >> 9;
  const int NKS = K / 16, ob = (int)(obks / NKS), ks = (int)(obks - (long)ob * NKS);
  wf[i] = w[(size_t)(32 * ob + (l & 31)) * K + 16 * ks + 8 * (l >> 5) + e];
}

// 7965346 fwd_fused_bf16, plus the STORE / BAR variant switches and a tag buffer that
// records, per column element written, the (step, wave, lane) that wrote it.
template <int STORE, int BAR, int MODE>
__global__ __launch_bounds__(256) void fwd_fused_bf16(Geo g, const bf16_t* __restrict__ xT,
                                                     const float* __restrict__ off,
                                                     const bf16_t* __restrict__ wf,
                                                     const float* __restrict__ bias,
                                                     bf16_t* __restrict__ out,
                                                     bf16_t* __restrict__ colT,
                                                     unsigned* __restrict__ dbg,
                                                     const bf16_t* __restrict__ rcolp) {
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][kBP * kBS];
  __shared__ int4 rec[kBP * kFTaps];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Block3 blk = xcd_block();
  const long P = (long)g.B * g.HW;
  const long p0 = (long)blk.x * kBP;
  const int ob0 = blk.y * 8 + wave * 2;
  const int nsteps = g.N * (g.C / 32), NKS = g.K / 16;
  for (int s = tid; s < kBP * g.N; s += 256) {
    const int tp = s / g.N, n = s - tp * g.N;
    const long p = p0 + tp;
    int4 r = make_int4(INT_MIN, 0, 0, 0);
    if (p < P) {
      const int b = (int)(p / g.HW), m = (int)(p - (long)b * g.HW);
      const Tap t = sample_tap(g, off, b, 0, n, m);
      if (t.ok) r = make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc));
    }
    rec[tp * kFTaps + n] = r;
  }
  constexpr int kU = kBP / 64;
  const int sp = tid >> 2, sq = tid & 3;
  const char* xc[kU];
  unsigned colrow[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const long ps = p0 + sp + 64 * u;
    const bool pv = ps < P;
    const int bs = pv ? (int)(ps / g.HW) : 0;
    xc[u] = reinterpret_cast<const char*>(xT) + (size_t)bs * g.HWi * g.C * 2 + sq * 16;
    colrow[u] = pv ? (unsigned)(((size_t)ps * g.K + sq * 8) * 2) : ~0u;
  }
  const unsigned rowb = (unsigned)g.W * g.C * 2u, pixb = (unsigned)g.C * 2u;
  const __amdgpu_buffer_rsrc_t col_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      colT, 0, colT ? (int)((size_t)P * g.K * 2) : 0, 0x00020000);

  f32x16 acc[2][kBNB];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int q = 0; q < kBNB; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][q][r] = 0.f;
  struct Gath {
    uint4 a, b, c, d;
    float fr, fc;
    int okm;
  };
  Gath G[kGD][kU];
  bf16x8f_t a[2][2][2];
  uint4 last_v = make_uint4(0, 0, 0, 0);
  int last_slot = 0;
  uint4 xs = make_uint4(0, 0, 0, 0);  // MODE 8: XOR of every staged value of this thread
  uint4 xbv[2][kBNB];                 // MODE 8: XOR of every B fragment this lane read
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < kBNB; ++q) xbv[h][q] = make_uint4(0, 0, 0, 0);

  auto kbase = [&](int s) {
    const int cs = s / g.N, n = s - cs * g.N;
    return n * g.C + 32 * cs;
  };
  auto load_a = [&](int s, int d) {
    const int ks = kbase(min(s, nsteps - 1)) / 16;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        a[d][j][h] = ld_frag(wf + ((size_t)((ob0 + j) * NKS + ks + h) * 64 + lane) * 8);
  };
  auto gather1 = [&](int s0, int u, Gath& q) {
    const int s = min(s0, nsteps - 1);
    const int cs = s / g.N, n = s - cs * g.N;
    const int4 r = rec[(sp + 64 * u) * kFTaps + n];
    const bool lv = r.x != INT_MIN;
    const int r0 = lv ? r.x : 0, q0 = r.y;
    q.fr = __int_as_float(r.z);
    q.fc = __int_as_float(r.w);
    const bool r0ok = lv && r0 >= 0, r1ok = lv && r0 + 1 < g.H;
    const bool c0ok = q0 >= 0, c1ok = q0 + 1 < g.W;
    q.okm = (lv ? 16 : 0) | ((r0ok && c0ok) ? 1 : 0) | ((r0ok && c1ok) ? 2 : 0) |
            ((r1ok && c0ok) ? 4 : 0) | ((r1ok && c1ok) ? 8 : 0);
    const int ra = min(max(r0, 0), g.H - 1), rb = min(r0 + 1, g.H - 1);
    const int qa = min(max(q0, 0), g.W - 1), qb = min(max(q0 + 1, 0), g.W - 1);
    const char* base = xc[u] + cs * 64;
    q.a = *reinterpret_cast<const uint4*>(base + ((unsigned)ra * rowb + (unsigned)qa * pixb));
    q.b = *reinterpret_cast<const uint4*>(base + ((unsigned)ra * rowb + (unsigned)qb * pixb));
    q.c = *reinterpret_cast<const uint4*>(base + ((unsigned)rb * rowb + (unsigned)qa * pixb));
    q.d = *reinterpret_cast<const uint4*>(base + ((unsigned)rb * rowb + (unsigned)qb * pixb));
  };
  auto interp = [&](const Gath& q) {
    const int m = q.okm;
    const unsigned za = (m & 1) ? ~0u : 0u, zb = (m & 2) ? ~0u : 0u;
    const unsigned zc = (m & 4) ? ~0u : 0u, zd = (m & 8) ? ~0u : 0u;
    const unsigned A4[4] = {q.a.x & za, q.a.y & za, q.a.z & za, q.a.w & za};
    const unsigned B4[4] = {q.b.x & zb, q.b.y & zb, q.b.z & zb, q.b.w & zb};
    const unsigned C4[4] = {q.c.x & zc, q.c.y & zc, q.c.z & zc, q.c.w & zc};
    const unsigned D4[4] = {q.d.x & zd, q.d.y & zd, q.d.z & zd, q.d.w & zd};
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = bilerp(q.fr, q.fc, bfl(A4[e]), bfl(B4[e]), bfl(C4[e]), bfl(D4[e]));
      const float hi = bilerp(q.fr, q.fc, bfh(A4[e]), bfh(B4[e]), bfh(C4[e]), bfh(D4[e]));
      o[e] = (m & 16) ? ((unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16)) : 0u;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
  };
  auto ne4 = [](uint4 x, uint4 y) { return x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w; };
  auto store1 = [&](int s, int buf, int u, const Gath& q) {
    const uint4 v = interp(q);
    if (MODE == 7) {  // staged value against the reference columns; on a mismatch, which input
      const long ps = p0 + sp + 64 * u;
      if (ps < P) {
        const uint4 ref =
            *reinterpret_cast<const uint4*>(rcolp + (size_t)ps * g.K + kbase(s) + 8 * sq);
        if (ne4(v, ref)) {
          Gath f;
          gather1(s, u, f);  // the same step's record and corners, loaded afresh
          atomicAdd(&dbg[0], 1u);
          atomicAdd(&dbg[8 + (lane >> 4)], 1u);
          atomicAdd(&dbg[16 + min(s, 71)], 1u);
          if (!ne4(interp(f), ref)) atomicAdd(&dbg[1], 1u);
          if (f.fr != q.fr || f.fc != q.fc || f.okm != q.okm) atomicAdd(&dbg[2], 1u);
          if (ne4(f.a, q.a)) atomicAdd(&dbg[3], 1u);
          if (ne4(f.b, q.b)) atomicAdd(&dbg[4], 1u);
          if (ne4(f.c, q.c)) atomicAdd(&dbg[5], 1u);
          if (ne4(f.d, q.d)) atomicAdd(&dbg[6], 1u);
          atomicAdd(&dbg[88 + wave], 1u);
          atomicAdd(&dbg[92 + (s & 1)], 1u);
        }
      }
    }
    *reinterpret_cast<uint4*>(&Bs[buf][(sp + 64 * u) * kBS + 8 * sq]) = v;
    if (MODE == 8) {
      xs.x ^= v.x; xs.y ^= v.y; xs.z ^= v.z; xs.w ^= v.w;
    }
    last_v = v;
    last_slot = buf * kBP * kBS + (sp + 64 * u) * kBS + 8 * sq;
    if (STORE && colT) {
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, v), col_rsrc,
          (int)(colrow[u] == ~0u ? ~0u : colrow[u] + (unsigned)kbase(s) * 2u), 0, kAuxNT);
      if (STORE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  auto gather = [&](int s, Gath(&q)[kU]) {
#pragma unroll
    for (int u = 0; u < kU; ++u) gather1(s, u, q[u]);
  };
  auto store = [&](int s, int buf, const Gath(&q)[kU]) {
#pragma unroll
    for (int u = 0; u < kU; ++u) store1(s, buf, u, q[u]);
  };
  auto mfma = [&](int buf, int d) {
    bf16x8f_t bv[2][kBNB];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < kBNB; ++q)
        bv[h][q] = ld_frag(&Bs[buf][(32 * q + (lane & 31)) * kBS + 16 * h + 8 * (lane >> 5)]);
    if (MODE == 8) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < kBNB; ++q) {
          const uint4 t = __builtin_bit_cast(uint4, bv[h][q]);
          xbv[h][q].x ^= t.x; xbv[h][q].y ^= t.y; xbv[h][q].z ^= t.z; xbv[h][q].w ^= t.w;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < kBNB; ++q)
          acc[j][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[d][j][h], bv[h][q], acc[j][q], 0, 0, 0);
  };
  auto mm = [&](int buf, int d) {
    __builtin_amdgcn_sched_barrier(0);
    mfma(buf, d);
    if (MODE == 6) {  // wait until this wave's last MFMA has completed (reads its D)
      float t = acc[1][kBNB - 1][15];
      asm volatile("" ::"v"(t));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto check = [&](int where) {
    const uint4 r = *reinterpret_cast<const uint4*>(&Bs[0][0] + last_slot);
    if (r.x != last_v.x || r.y != last_v.y || r.z != last_v.z || r.w != last_v.w)
      atomicAdd(&dbg[where * 4 + (lane >> 4)], 1u);
  };
  auto step_barrier = [&]() {
    if (MODE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MODE == 2) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    if (MODE == 3) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      check(0);  // own write seen by itself before the barrier
    }
    if (BAR == 0) __syncthreads();
    else lds_barrier();
    if (MODE == 3) check(1);  // and after it
    if (MODE == 4) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    if (MODE == 5) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  __syncthreads();
#pragma unroll
  for (int d = 0; d < kGD; ++d) gather(d, G[d]);
  load_a(0, 0);
  store(0, 0, G[0]);
  step_barrier();
  for (int s0 = 0; s0 < nsteps; s0 += kGD) {
    bool done = false;
#pragma unroll
    for (int d = 0; d < kGD; ++d) {
      if (!done) {
        const int s = s0 + d;
        gather(s + kGD, G[d]);
        load_a(s + 1, (d + 1) & 1);
        mm(d & 1, d & 1);
        if (s + 1 >= nsteps) {
          done = true;
        } else {
          store(s + 1, (d + 1) & 1, G[(d + 1) % kGD]);
          step_barrier();
        }
      }
    }
    if (done) break;
  }
  if (MODE == 8) {  // per (tile, thread): staged XOR, then the 4 fragment XORs
    uint4* o8 = reinterpret_cast<uint4*>(dbg + 1024) + ((size_t)blk.x * 256 + tid) * 5;
    o8[0] = xs;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < kBNB; ++q) o8[1 + h * kBNB + q] = xbv[h][q];
  }
#pragma unroll
  for (int q = 0; q < kBNB; ++q) {
    const long pf = p0 + 32 * q + (lane & 31);
    if (pf >= P) continue;
    const int b = (int)(pf / g.HW), m = (int)(pf - (long)b * g.HW);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = 32 * (ob0 + j) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        out[((size_t)b * g.O + o) * g.HW + m] = f2bf(acc[j][q][r] + (bias ? bias[o] : 0.f));
      }
  }
}

// ---- independent references ----------------------------------------------------------
// colT[p][n*C + c]: one thread per element, K1's arithmetic (fp32 bilerp of the bf16 corners,
// zero for corners outside the image, one bf16 rounding)
__global__ void ref_cols(Geo g, const bf16_t* __restrict__ xT, const float* __restrict__ off,
                         bf16_t* __restrict__ colT) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.B * g.HW * g.K;
  if (i >= total) return;
  const long p = i / g.K;
  const int k = (int)(i - p * g.K), n = k / g.C, c = k - n * g.C;
  const int b = (int)(p / g.HW), m = (int)(p - (long)b * g.HW);
  const Tap t = sample_tap(g, off, b, 0, n, m);
  float v = 0.f;
  if (t.ok) {
    auto X = [&](int r, int q) {
      if (r < 0 || r >= g.H || q < 0 || q >= g.W) return 0.f;
      return bf2f(xT[((size_t)b * g.HWi + (size_t)r * g.W + q) * g.C + c]);
    };
    v = bilerp(t.fr, t.fc, X(t.r0, t.c0), X(t.r0, t.c0 + 1), X(t.r0 + 1, t.c0),
               X(t.r0 + 1, t.c0 + 1));
  }
  colT[i] = t.ok ? f2bf(v) : (bf16_t)0;
}

// out[b][o][m] = bf16(Σ_k col[p][k]·w[o][k] + bias[o]) in sequential fp32 (tolerance check only)
__global__ void ref_out(Geo g, const bf16_t* __restrict__ col, const bf16_t* __restrict__ w,
                        const float* __restrict__ bias, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.B * g.O * g.HW;
  if (i >= total) return;
  const int m = (int)(i % g.HW), o = (int)((i / g.HW) % g.O), b = (int)(i / ((long)g.HW * g.O));
  const bf16_t* cr = col + ((size_t)b * g.HW + m) * g.K;
  const bf16_t* wr = w + (size_t)o * g.K;
  float s = 0.f;
  for (int k = 0; k < g.K; ++k) s = fmaf(bf2f(cr[k]), bf2f(wr[k]), s);
  out[i] = s + bias[o];
}

// mismatch histograms: hist[0..71] by k step (tap-major within a channel slice, as the kernel
// walks them: s = cs*N + n), [72..135] by pixel of the 64-px tile, [136..139] by sq (8-channel
// unit), [140] total
__global__ void cmp_cols(Geo g, const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                         unsigned* __restrict__ hist) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.B * g.HW * g.K;
  if (i >= total || a[i] == b[i]) return;
  const long p = i / g.K;
  const int k = (int)(i - p * g.K), n = k / g.C, c = k - n * g.C;
  const int s = (c / 32) * g.N + n;
  atomicAdd(&hist[s], 1u);
  atomicAdd(&hist[72 + (int)(p % 64)], 1u);
  atomicAdd(&hist[136 + (c % 32) / 8], 1u);
  atomicAdd(&hist[140], 1u);
}
// out: [0] bitwise differences from the first launch, [1] outside |Δ| <= 2^-7 |ref| + 1e-2
// against the fp32 reference, [2..65] by pixel of the tile, [66..69] by wave (64 rows each)
__global__ void cmp_out(Geo g, const bf16_t* __restrict__ o, const bf16_t* __restrict__ o0,
                        const float* __restrict__ ref, unsigned* __restrict__ hist) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.B * g.O * g.HW;
  if (i >= total) return;
  const int m = (int)(i % g.HW), oc = (int)((i / g.HW) % g.O), b = (int)(i / ((long)g.HW * g.O));
  const long p = (long)b * g.HW + m;
  if (o[i] != o0[i]) {
    atomicAdd(&hist[0], 1u);
    atomicAdd(&hist[2 + (int)(p % 64)], 1u);
    atomicAdd(&hist[66 + oc / 64], 1u);
  }
  const float v = bf2f(o[i]), r = ref[i];
  if (!(fabsf(v - r) <= 0.0078125f * fabsf(r) + 1e-2f)) atomicAdd(&hist[1], 1u);
}

static unsigned lcg(unsigned long long& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (unsigned)(s >> 33);
}
static float nrm(unsigned long long& s) {  // approx N(0,1): sum of 4 uniforms
  float a = 0;
  for (int i = 0; i < 4; ++i) a += (lcg(s) & 0xffffff) / 16777216.f;
  return (a - 2.f) * 1.7320508f;
}
static bf16_t h2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (bf16_t)(u >> 16);
}

template <int STORE, int BAR, int MODE>
static void run_variant(const char* name, const Geo& g, const bf16_t* xT, const float* off,
                        const bf16_t* wf, const float* bias, const bf16_t* rcol, const float* rout,
                        bf16_t* out0, bf16_t* out, bf16_t* col, unsigned* hist, int reps) {
  const long P = (long)g.B * g.HW, ncol = P * g.K, nout = (long)g.B * g.O * g.HW;
  std::vector<unsigned> h(141);
  unsigned cols_bad = 0, out_nd = 0, out_tol = 0, runs_bad = 0;
  std::vector<unsigned long long> colstep(72), colpx(64), colsq(4), outpx(64), outwave(4);
  for (int r = 0; r < reps; ++r) {
    CK(hipMemset(col, 0xff, ncol * 2));
    CK(hipMemset(hist, 0, 141 * 4));
    bf16_t* o = r == 0 ? out0 : out;
    CK(hipMemset(hist + 160, 0, 96 * 4));
    hipLaunchKernelGGL((fwd_fused_bf16<STORE, BAR, MODE>), dim3((unsigned)(P / kBP), g.O / 256),
                       dim3(256), 0, 0, g, xT, off, wf, bias, o, STORE ? col : nullptr, hist + 160,
                       rcol);
    CK(hipGetLastError());
    if (MODE == 8) {
      const long nt = P / kBP;
      std::vector<uint4> d8((size_t)nt * 256 * 5);
      CK(hipMemcpy(d8.data(), reinterpret_cast<uint4*>(hist + 160 + 1024), d8.size() * 16,
                   hipMemcpyDeviceToHost));
      static std::vector<unsigned short> hc;
      if (hc.empty()) {
        hc.resize((size_t)P * g.K);
        CK(hipMemcpy(hc.data(), rcol, hc.size() * 2, hipMemcpyDeviceToHost));
      }
      const int nsteps = g.N * (g.C / 32);
      auto kb = [&](int st) { return (st % g.N) * g.C + 32 * (st / g.N); };
      auto x16 = [&](long p, int k) {
        uint4 r;
        memcpy(&r, &hc[(size_t)p * g.K + k], 16);
        return r;
      };
      auto ne = [](uint4 a, uint4 b_) { return a.x != b_.x || a.y != b_.y || a.z != b_.z || a.w != b_.w; };
      long bad_stage[4] = {0, 0, 0, 0}, bad_frag[4] = {0, 0, 0, 0};
      for (long t = 0; t < nt; ++t)
        for (int tid = 0; tid < 256; ++tid) {
          const int l = tid & 63, spp = tid >> 2, sqq = tid & 3;
          uint4 es = make_uint4(0, 0, 0, 0), ef[4];
          for (int i = 0; i < 4; ++i) ef[i] = make_uint4(0, 0, 0, 0);
          for (int st = 0; st < nsteps; ++st) {
            const uint4 a = x16(t * kBP + spp, kb(st) + 8 * sqq);
            es.x ^= a.x; es.y ^= a.y; es.z ^= a.z; es.w ^= a.w;
            for (int h = 0; h < 2; ++h)
              for (int q = 0; q < kBNB; ++q) {
                const uint4 b_ = x16(t * kBP + 32 * q + (l & 31), kb(st) + 16 * h + 8 * (l >> 5));
                uint4& e = ef[h * kBNB + q];
                e.x ^= b_.x; e.y ^= b_.y; e.z ^= b_.z; e.w ^= b_.w;
              }
          }
          const uint4* got = &d8[((size_t)t * 256 + tid) * 5];
          if (ne(got[0], es)) ++bad_stage[l >> 4];
          for (int i = 0; i < 4; ++i)
            if (ne(got[1 + i], ef[i])) ++bad_frag[l >> 4];
        }
      printf("  staged-value XOR mismatches by quarter-wave: %ld %ld %ld %ld; B-fragment XOR "
             "mismatches by quarter-wave: %ld %ld %ld %ld\n", bad_stage[0], bad_stage[1],
             bad_stage[2], bad_stage[3], bad_frag[0], bad_frag[1], bad_frag[2], bad_frag[3]);
    }
    if (MODE == 7) {
      unsigned d[96];
      CK(hipMemcpy(d, hist + 160, sizeof d, hipMemcpyDeviceToHost));
      printf("  staged != reference: %u (fresh inputs fix it: %u; record differs %u; corners a %u b %u "
             "c %u d %u) by quarter-wave %u %u %u %u, by wave %u %u %u %u, even/odd step %u %u\n",
             d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[8], d[9], d[10], d[11], d[88], d[89],
             d[90], d[91], d[92], d[93]);
      printf("  by step:");
      for (int i = 0; i < 72; ++i)
        if (d[16 + i]) printf(" %d:%u", i, d[16 + i]);
      printf("\n");
    }
    if (MODE == 3) {
      unsigned d[8];
      CK(hipMemcpy(d, hist + 160, 32, hipMemcpyDeviceToHost));
      printf("  readback mismatches before barrier by quarter-wave: %u %u %u %u; after: %u %u %u %u\n",
             d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
    }
    CK(hipGetLastError());
    unsigned cb = 0;
    if (STORE) {
      hipLaunchKernelGGL(cmp_cols, dim3((unsigned)((ncol + 255) / 256)), dim3(256), 0, 0, g, col,
                         rcol, hist);
      CK(hipMemcpy(h.data(), hist, 141 * 4, hipMemcpyDeviceToHost));
      cb = h[140];
      for (int i = 0; i < 72; ++i) colstep[i] += h[i];
      for (int i = 0; i < 64; ++i) colpx[i] += h[72 + i];
      for (int i = 0; i < 4; ++i) colsq[i] += h[136 + i];
      CK(hipMemset(hist, 0, 141 * 4));
    }
    hipLaunchKernelGGL(cmp_out, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, 0, g, o, out0,
                       rout, hist);
    CK(hipMemcpy(h.data(), hist, 141 * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < 64; ++i) outpx[i] += h[2 + i];
    for (int i = 0; i < 4; ++i) outwave[i] += h[66 + i];
    cols_bad += cb;
    out_nd += h[0];
    out_tol += h[1];
    if (cb || h[0] || h[1]) ++runs_bad;
    printf("%s run %d: column mismatches %u, out != first launch %u, out outside tol %u\n", name,
           r, cb, h[0], h[1]);
    fflush(stdout);
  }
  printf("%s SUMMARY: runs with any error %u/%d, columns %u of %ld, out nondet %u, out tol %u of %ld\n",
         name, runs_bad, reps, cols_bad, ncol * reps, out_nd, out_tol, nout * reps);
  auto dump = [&](const char* what, std::vector<unsigned long long>& v) {
    unsigned long long t = 0;
    for (auto x : v) t += x;
    if (!t) return;
    printf("  %s:", what);
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]) printf(" %zu:%llu", i, v[i]);
    printf("\n");
  };
  dump("column errors by k step (s = slice*9 + tap)", colstep);
  dump("column errors by tile pixel", colpx);
  dump("column errors by 8-channel unit", colsq);
  dump("out nondeterminism by tile pixel", outpx);
  dump("out nondeterminism by wave (64 out channels)", outwave);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 6;
  Geo g{};
  g.B = 64; g.C = 256; g.H = 28; g.W = 28; g.O = 256;
  g.kh = 3; g.kw = 3; g.sh = 1; g.sw = 1; g.ph = 1; g.pw = 1; g.dh = 1; g.dw = 1; g.G = 1;
  g.Ho = 28; g.Wo = 28; g.N = 9; g.K = 9 * 256; g.HW = 784; g.HWi = 784; g.Cg = 256; g.J = 18;
  g.dt = DCN_BF16;
  const long P = (long)g.B * g.HW, nx = (long)g.B * g.HWi * g.C, noff = (long)g.B * g.J * g.HW;
  const long ncol = P * g.K, nout = (long)g.B * g.O * g.HW, nw = (long)g.O * g.K;
  unsigned long long seed = 75;
  std::vector<bf16_t> hx(nx), hw(nw);
  std::vector<float> hoff(noff), hb(g.O);
  for (auto& v : hx) v = h2bf(nrm(seed));
  for (auto& v : hoff) v = __builtin_bit_cast(float, (unsigned)h2bf(nrm(seed)) << 16);  // bf16-valued
  for (auto& v : hw) v = h2bf(nrm(seed) * 0.0295f);
  for (auto& v : hb) v = nrm(seed) * 0.1f;
  bf16_t *xT, *w, *wf, *rcol, *col, *out0, *out;
  float *off, *bias, *rout;
  unsigned* hist;
  CK(hipMalloc(&xT, nx * 2)); CK(hipMalloc(&w, nw * 2)); CK(hipMalloc(&wf, nw * 2));
  CK(hipMalloc(&rcol, ncol * 2)); CK(hipMalloc(&col, ncol * 2));
  CK(hipMalloc(&out0, nout * 2)); CK(hipMalloc(&out, nout * 2));
  CK(hipMalloc(&off, noff * 4)); CK(hipMalloc(&bias, g.O * 4)); CK(hipMalloc(&rout, nout * 4));
  CK(hipMalloc(&hist, (160 + 1024) * 4 + (size_t)(P / kBP) * 256 * 5 * 16));
  CK(hipMemcpy(xT, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(off, hoff.data(), noff * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), g.O * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(wf_to_frag_bf16, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, 0, w, wf, g.O, g.K);
  hipLaunchKernelGGL(ref_cols, dim3((unsigned)((ncol + 255) / 256)), dim3(256), 0, 0, g, xT, off, rcol);
  hipLaunchKernelGGL(ref_out, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, 0, g, rcol, w, bias, rout);
  CK(hipDeviceSynchronize());
  printf("config 4 geometry, %d launches per variant\n", reps);
  run_variant<0, 1, 0>("C no-store+lds_barrier", g, xT, off, wf, bias, rcol, rout, out0, out, col, hist, reps);
  run_variant<0, 1, 8>("M no-store+lds_barrier+XOR checksums", g, xT, off, wf, bias, rcol, rout, out0, out, col, hist, reps);
  run_variant<0, 0, 8>("M2 no-store+syncthreads+XOR checksums", g, xT, off, wf, bias, rcol, rout, out0, out, col, hist, reps);
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
