// dcn_gemm_split.hip — fp32 GEMM on the bf16 matrix cores by exact operand splitting
// (DCN_MATH_F32_BF16X6 / X9 / X3), for the three dense contractions of the DeformConv2d
// step (deform_conv.py:76 and its two autodiff GEMMs).
//
// Why: gfx950 has no xf32; its f32-input MFMA runs at the f32 vector rate (157 TF), 1/16
// of bf16 MFMA (2.5 PF dense). The vendor fp32 GEMMs already reach 92 % of the f32 rate
// at config 3, so the 5 ms of GEMMs per step cannot get faster in native f32.
//
// How: every fp32 operand element a is split EXACTLY into three bf16 planes by truncation,
//   hi = a & 0xffff0000,  mid = (a - hi) & 0xffff0000,  lo = a - hi - mid,
// (a has a 24-bit significand; hi and mid each take 8 significant bits, so the remainder
// lo has at most 8 and is itself a bf16: a == hi + mid + lo with no rounding). Each bf16
// product is exact in the MFMA's fp32 accumulator, so
//   X9: Σ over all 9 plane pairs        — every product term exact; only the fp32
//                                          accumulation rounds;
//   X6: drops mid·lo, lo·mid, lo·lo      — |dropped| ≤ 2^-23·|a·b| per product, the size
//                                          of one fp32 rounding (native-f32-class);
//   X3: two planes, hi·hi + hi·lo + lo·hi — ≈2^-17 per product (opt-in only).
// Operands stay fp32 in HBM; the split happens on the way from registers to LDS, once per
// element per workgroup.
//
// Kernel: column-major C(m×n) (+ bias[n]) = op(A)(m×k)·op(B)(k×n), batched by strides.
// 128×128 output tile, BK = 32, 256 threads = 4 waves of 64×64 (4×4 fragments of
// mfma_f32_16x16x32_bf16). MFMA rows carry C's n index and MFMA columns C's m index, so
// the 16 lanes of one accumulator register store 64 contiguous bytes of the column-major
// C. One LDS buffer of 48 KiB per workgroup; per k-step: split+store, barrier, MFMAs,
// barrier. Two forms (A/B measured at config 3):
//   LATE (default): loads issued after the MFMAs, so the staging registers are dead
//          across them and three workgroups per CU fit (≤ 168 VGPRs); the other
//          workgroups hide the load latency. fwd / ∂W / ∂col 1.21 / 1.32 / 1.54 ms;
//   EARLY: next tile's loads issued before the MFMAs, two workgroups per CU:
//          1.30 / 1.38 / 1.74 ms (with two register sets, loads two k-steps ahead:
//          1.26 / 1.37 / 1.77 — load latency is not what limits it).
// LDS images per plane:
//   k-contiguous operand   → [idx][32 k] bf16, 64-B rows, 16-B chunks XOR-swizzled by
//                            bit 3 of idx, fragments by ds_read_b128;
//   m/n-contiguous operand → [k][128 idx] bf16, chunks XOR-swizzled by
//                            ((k&3)<<2)|((k>>2)&3), fragments by two ds_read_b64_tr_b16
//                            (gfx950's transposing LDS read; no register transpose).
// Both images are bank-conflict-free for their reads and writes (SQ_LDS_BANK_CONFLICT = 0;
// the swizzle itself measured within noise against 2-way-conflicting alternatives).
//
// Measured and dropped (r01, config 3): 8-wave 128×256 tiles with two LDS
// buffers; a warp-specialised persistent form (producer waves stage, consumer waves only
// issue MFMAs); operands pre-split into bf16 planes in HBM. None beat this form.
#include <hip/hip_runtime.h>

#include "dcn_internal.h"

namespace dcn {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4* lds_s16x4;

constexpr int BK = 32, TILE = 128, NT = 256;

// --- LDS image addressing (bytes within one plane image) ---------------------------
// [idx][32 k], chunk 0..3. The XOR by bit 3 of idx makes the fragment read (lane l: row
// l&15, chunk l>>4) conflict-free under ds_read_b128's lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32): each group then covers all 16 slots of the 256-B bank row.
__device__ __forceinline__ int kc_off(int idx, int chunk) {
  return idx * 64 + ((chunk ^ ((idx >> 2) & 2)) << 4);
}
// [k][128 idx], chunk 0..15: the four rows of one transposed read land in distinct slots
__device__ __forceinline__ int mc_off(int k, int chunk) {
  return k * (TILE * 2) + ((chunk ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4);
}

// exact split of 4 floats into P planes (P = 3: trunc/trunc/exact; P = 2: trunc + RNE),
// packed as 4 bf16 per plane (8 bytes)
template <int P>
__device__ __forceinline__ void split4(const float4 v, u32x2 (&out)[P]) {
  const float a[4] = {v.x, v.y, v.z, v.w};
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const unsigned u = __float_as_uint(a[e]);
    const float r1 = a[e] - __uint_as_float(u & 0xffff0000u);
    const unsigned u1 = __float_as_uint(r1);
    h[e] = u;
    if constexpr (P == 3) {
      m[e] = u1;
      l[e] = __float_as_uint(r1 - __uint_as_float(u1 & 0xffff0000u));
    } else {
      m[e] = u1 + 0x7fffu + ((u1 >> 16) & 1u);
    }
  }
  // v_perm_b32: the high halves of two dwords packed into one
  out[0] = u32x2{__builtin_amdgcn_perm(h[1], h[0], 0x07060302u),
                 __builtin_amdgcn_perm(h[3], h[2], 0x07060302u)};
  out[1] = u32x2{__builtin_amdgcn_perm(m[1], m[0], 0x07060302u),
                 __builtin_amdgcn_perm(m[3], m[2], 0x07060302u)};
  if constexpr (P == 3)
    out[2] = u32x2{__builtin_amdgcn_perm(l[1], l[0], 0x07060302u),
                   __builtin_amdgcn_perm(l[3], l[2], 0x07060302u)};
}

// One fp32 operand as the kernel sees it: element (idx, kk) of op(X) at p[idx*ld + kk]
// (KC) or p[kk*ld + idx] (MC), batch b at + b*bs.
struct Operand {
  const float* p;
  long ld, bs;
  int lim;  // idx extent (m or n)
};

// Register stage + LDS image of one 128 × 32 operand tile in P planes (16 floats/thread).
template <bool KC, int P>
struct Tile {
  static constexpr int PLANE = TILE * BK * 2;  // bytes per plane image
  static constexpr int BYTES = P * PLANE;
  static constexpr int UNITS = TILE * BK / 4 / NT;  // float4s per thread
  float4 r[UNITS];

  __device__ __forceinline__ void load(const Operand& o, int b, int idx0, int k0, int klim,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < UNITS; ++i) {
      const int u = tid + NT * i;
      const int idx = idx0 + (KC ? u >> 3 : (u % (TILE / 4)) * 4);
      const int kk = k0 + (KC ? (u & 7) * 4 : u / (TILE / 4));
      // the contiguous extent is a multiple of 4, so a float4 is wholly in or out
      const bool ok = idx < o.lim && kk < klim;
      const float* q = o.p + (long)b * o.bs + (KC ? (long)idx * o.ld + kk : (long)kk * o.ld + idx);
      r[i] = ok ? *reinterpret_cast<const float4*>(q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  __device__ __forceinline__ void store(char* img, int tid) const {
#pragma unroll
    for (int i = 0; i < UNITS; ++i) {
      const int u = tid + NT * i;
      u32x2 pk[P];
      split4<P>(r[i], pk);
      int off;
      if constexpr (KC) {
        const int idx = u >> 3, kq = u & 7;
        off = kc_off(idx, kq >> 1) + 8 * (kq & 1);
      } else {
        const int kk = u / (TILE / 4), iq = u % (TILE / 4);
        off = mc_off(kk, iq >> 1) + 8 * (iq & 1);
      }
#pragma unroll
      for (int pl = 0; pl < P; ++pl) *reinterpret_cast<u32x2*>(img + pl * PLANE + off) = pk[pl];
    }
  }

  // fragment of plane pl: lane holds idx base + (lane&15), k = 8(lane>>4) .. +7
  static __device__ __forceinline__ bf16x8 frag(const char* img, int pl, int base, int lane) {
    const char* plane = img + pl * PLANE;
    if constexpr (KC) {
      const u32x4 v =
          *reinterpret_cast<const u32x4*>(plane + kc_off(base + (lane & 15), lane >> 4));
      return __builtin_bit_cast(bf16x8, v);
    } else {
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int ch = (base >> 3) + (p >> 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4)(plane + mc_off(8 * g + q, ch) + 8 * (p & 1)));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4)(plane + mc_off(8 * g + 4 + q, ch) + 8 * (p & 1)));
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

__device__ __forceinline__ f32x4v mfma(bf16x8 a, bf16x8 b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the plane products of one fragment pair, smallest terms first
template <int NPROD, int P>
__device__ __forceinline__ f32x4v mfma_planes(const bf16x8 (&fn)[P], const bf16x8 (&fm)[P],
                                              f32x4v c) {
  if constexpr (NPROD == 9) {
    c = mfma(fn[2], fm[2], c);
    c = mfma(fn[2], fm[1], c);
    c = mfma(fn[1], fm[2], c);
  }
  if constexpr (P == 3) {
    c = mfma(fn[2], fm[0], c);
    c = mfma(fn[1], fm[1], c);
    c = mfma(fn[0], fm[2], c);
  }
  c = mfma(fn[1], fm[0], c);
  c = mfma(fn[0], fm[1], c);
  c = mfma(fn[0], fm[0], c);
  return c;
}

struct Args {
  Operand A, B;
  float* C;
  long ldc, sc;
  const float* bias;  // + bias[n] in the epilogue (or null)
  int m, n, k;
  int tiles_m, tiles_n, batch;
  int n_fast;  // consecutive tiles walk n (share the A panel)
};

// FORM 0 (EARLY): next step's loads before the MFMAs, 2 workgroups/CU; 1 (LATE): after
// the MFMAs, 3 workgroups/CU.
template <int NPROD, bool A_KC, bool B_KC, int FORM>
__global__ __launch_bounds__(NT, FORM == 1 ? 3 : 2) void gemm_split_kernel(Args s) {
  constexpr int P = NPROD == 3 ? 2 : 3;
  using TA = Tile<A_KC, P>;
  using TB = Tile<B_KC, P>;
  __shared__ __attribute__((aligned(16))) char lds[TA::BYTES + TB::BYTES];

  // XCD-aware tile order: each XCD walks a contiguous range of tiles (bijective remap)
  const int T = s.tiles_m * s.tiles_n * s.batch;
  const int L = blockIdx.x, xcd = L & 7, pos = L >> 3, q8 = T >> 3, r8 = T & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  int tm, tn, b;
  if (s.n_fast) {
    tn = t % s.tiles_n;
    const int u = t / s.tiles_n;
    tm = u % s.tiles_m;
    b = u / s.tiles_m;
  } else {
    tm = t % s.tiles_m;
    const int u = t / s.tiles_m;
    tn = u % s.tiles_n;
    b = u / s.tiles_n;
  }
  const int m0 = tm * TILE, n0 = tn * TILE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  f32x4v acc[4][4];  // [n fragment][m fragment]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int nk = (s.k + BK - 1) / BK;
  auto load = [&](TA& ta, TB& tb, int kt) {
    const int k0 = (kt < nk ? kt : nk - 1) * BK;  // clamped: no branch around the loads
    ta.load(s.A, b, m0, k0, s.k, tid);
    tb.load(s.B, b, n0, k0, s.k, tid);
  };
  auto mfmas = [&]() {
    // m fragments of every plane (MFMA B operand), then n fragments one at a time
    bf16x8 fm[4][P];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int pl = 0; pl < P; ++pl) fm[j][pl] = TA::frag(lds, pl, wm * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 fn[P];
#pragma unroll
      for (int pl = 0; pl < P; ++pl)
        fn[pl] = TB::frag(lds + TA::BYTES, pl, wn * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma_planes<NPROD, P>(fn, fm[j], acc[i][j]);
    }
  };
  // one k-step from register set (ta, tb), which is then refilled with step kt + ahead
  auto step = [&](TA& ta, TB& tb, int kt, int ahead) {
    ta.store(lds, tid);
    tb.store(lds + TA::BYTES, tid);
    __syncthreads();
    if constexpr (FORM != 1) load(ta, tb, kt + ahead);
    mfmas();
    if constexpr (FORM == 1) load(ta, tb, kt + ahead);
    __syncthreads();
  };
  TA ta;
  TB tb;
  load(ta, tb, 0);
  for (int kt = 0; kt < nk; ++kt) step(ta, tb, kt, 1);

  // epilogue: acc[i][j][r] = C(m = m0 + 64wm + 16j + (lane&15), n = n0 + 64wn + 16i +
  // 4(lane>>4) + r); the 16 lanes of one register store 64 contiguous bytes of a column
  float* Cb = s.C + (long)b * s.sc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int mi = m0 + wm * 64 + j * 16 + (lane & 15);
    if (mi >= s.m) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ni = n0 + wn * 64 + i * 16 + 4 * (lane >> 4) + r;
        if (ni < s.n) Cb[(long)ni * s.ldc + mi] = acc[i][j][r] + (s.bias ? s.bias[ni] : 0.f);
      }
  }
}

template <int NPROD, bool A_KC, bool B_KC>
hipError_t launch_t(const Args& a, int form, hipStream_t st) {
  const int T = a.tiles_m * a.tiles_n * a.batch;
  if (form == 1)
    hipLaunchKernelGGL((gemm_split_kernel<NPROD, A_KC, B_KC, 1>), dim3(T), dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_split_kernel<NPROD, A_KC, B_KC, 0>), dim3(T), dim3(NT), 0, st, a);
  return hipGetLastError();
}

template <int NPROD>
hipError_t launch_p(const Args& a, bool a_kc, bool b_kc, int form, hipStream_t st) {
  if (a_kc && b_kc) return launch_t<NPROD, true, true>(a, form, st);
  if (a_kc) return launch_t<NPROD, true, false>(a, form, st);
  if (b_kc) return launch_t<NPROD, false, true>(a, form, st);
  return launch_t<NPROD, false, false>(a, form, st);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

bool operand_ok(const void* p, bool kc, long ld, long bs, int idx_extent, int k_extent) {
  // float4 staging: the contiguous extent, leading dim and batch stride are multiples of
  // 4 floats and the base is 16-B aligned
  return (kc ? k_extent : idx_extent) % 4 == 0 && ld % 4 == 0 && bs % 4 == 0 && aligned16(p);
}

}  // namespace

bool gemm_split_ok(const GemmSpec& s, const void* A, const void* B, const void* C) {
  if (s.bf16_ab || s.bf16_c || s.m <= 0 || s.n <= 0 || s.k <= 0 || s.batch <= 0) return false;
  if (!operand_ok(A, s.ta, s.lda, s.sa, s.m, s.k) || !operand_ok(B, !s.tb, s.ldb, s.sb, s.n, s.k))
    return false;
  const long tiles = (long)((s.m + TILE - 1) / TILE) * ((s.n + TILE - 1) / TILE) * s.batch;
  return tiles < (1l << 31) && (reinterpret_cast<uintptr_t>(C) & 3) == 0;
}

hipError_t launch_gemm_split(int math, const GemmSpec& s, const float* A, const float* B,
                             float* C, hipStream_t st, const float* bias, int form) {
  if (!gemm_split_ok(s, A, B, C)) return hipErrorInvalidValue;
  Args a;
  a.A = Operand{A, s.lda, s.sa, s.m};
  a.B = Operand{B, s.ldb, s.sb, s.n};
  a.C = C;
  a.ldc = s.ldc;
  a.sc = s.sc;
  a.bias = bias;
  a.m = s.m; a.n = s.n; a.k = s.k;
  a.tiles_m = (s.m + TILE - 1) / TILE;
  a.tiles_n = (s.n + TILE - 1) / TILE;
  a.batch = s.batch;
  // walk n fastest (tiles sharing an A panel run together on one XCD) when A is larger
  const double a_el = (double)s.m * s.k * (s.sa ? s.batch : 1);
  const double b_el = (double)s.n * s.k * (s.sb ? s.batch : 1);
  a.n_fast = a_el >= b_el;
  // form: 0 EARLY, 1 LATE (picked per shape by the caller)
  const bool a_kc = s.ta, b_kc = !s.tb;
  switch (math) {
    case 3: return launch_p<3>(a, a_kc, b_kc, form, st);
    case 9: return launch_p<9>(a, a_kc, b_kc, form, st);
    default: return launch_p<6>(a, a_kc, b_kc, form, st);
  }
}

}  // namespace dcn
