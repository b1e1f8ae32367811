// dcn_device.h — device-side helpers shared by the libdcn kernels (gfx950).
//
// Semantics follow /root/reference/deform_conv.py:56-81 exactly:
//   * sample for output (h, w), tap n:  row ≈ w + Δx[n], col ≈ h + Δy[n]   (Q1, :39/:47)
//   * coordinates normalised by the OUTPUT size and unnormalised by the INPUT
//     size with align_corners=True (Q2, :37-38 + grid_sample)
//   * no per-tap base position (Q3, :64-66); offsets [Δx(0..N-1) | Δy(0..N-1)] (Q4, :62)
//   * columns ordered k = n*C + c (Q5, :72-74)
// The coordinate chain is evaluated in fp32 in the reference's own op order; every
// kernel source is compiled with -ffp-contract=off so no FMA changes which side of
// an integer a coordinate lands on (Q6). Interpolation uses explicit fmaf.
#pragma once
#include "dcn_internal.h"

namespace dcn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ---- bf16 storage (DCN_BF16): round-to-nearest-even conversions (v_cvt_pk_bf16_f32) and
// 4-channel loads / stores, so kernels can be templated on the element type.
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return bf2f(v); }

__device__ __forceinline__ float4 ld4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ float4 ld4(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, float4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, p);
    __builtin_nontemporal_store(v.y, p + 1);
    __builtin_nontemporal_store(v.z, p + 2);
    __builtin_nontemporal_store(v.w, p + 3);
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
template <bool NT>
__device__ __forceinline__ void st4(bf16_t* p, float4 v) {
  uint2 u;
  u.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
  u.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
  if constexpr (NT) {
    __builtin_nontemporal_store(u.x, reinterpret_cast<unsigned*>(p));
    __builtin_nontemporal_store(u.y, reinterpret_cast<unsigned*>(p) + 1);
  } else {
    *reinterpret_cast<uint2*>(p) = u;
  }
}

// deform_conv.py:64-68 (grid (w,h) + offset), :37-39 (norm by (W_out-1),(H_out-1);
// grid = [norm_y, norm_x]) and grid_sample's align_corners=True unnormalisation
// ((g+1)/2)*(size-1): grid[...,0] = norm_y indexes the input COLUMN, grid[...,1]
// = norm_x the input ROW.
__device__ __forceinline__ void ref_coord(int h, int w, float dx, float dy, const Geo& g,
                                          float& iy, float& ix) {
  const float cx = (float)w + dx;                // grid x + offset x
  float nx = cx / (float)(g.Wo - 1);             // coords[...,0] / (W_out - 1)
  nx = nx * 2.0f;
  nx = nx - 1.0f;
  iy = ((nx + 1.0f) / 2.0f) * (float)(g.H - 1);  // unnormalise over input H
  const float cy = (float)h + dy;
  float ny = cy / (float)(g.Ho - 1);
  ny = ny * 2.0f;
  ny = ny - 1.0f;
  ix = ((ny + 1.0f) / 2.0f) * (float)(g.W - 1);  // unnormalise over input W
}

// A sample contributes only if at least one of its four corners can be inside the
// image: floor(row) in [-1, H-1] and floor(col) in [-1, W-1]. Otherwise its value
// and every derivative are exactly 0 (zeros padding). NaN -> invalid.
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

// The tap of sample (b, group gi, tap n, output pixel m).
__device__ __forceinline__ Tap sample_tap(const Geo& g, const float* __restrict__ off, int b,
                                          int gi, int n, int m) {
  const float* ob = off + ((size_t)b * g.J + (size_t)gi * 2 * g.N) * g.HW;
  const int h = m / g.Wo, w = m - h * g.Wo;
  float iy, ix;
  ref_coord(h, w, ob[(size_t)n * g.HW + m], ob[(size_t)(g.N + n) * g.HW + m], g, iy, ix);
  return make_tap(iy, ix, g);
}

// Canonical fp32 bilinear combination (all kernels and oracle/dcn_ref.c use this
// exact op order, so independent implementations agree bit for bit).
__device__ __forceinline__ float bilerp(float fr, float fc, float x00, float x01, float x10,
                                        float x11) {
  const float gr = 1.0f - fr, gc = 1.0f - fc;
  float v = (gr * gc) * x00;
  v = fmaf(gr * fc, x01, v);
  v = fmaf(fr * gc, x10, v);
  v = fmaf(fr * fc, x11, v);
  return v;
}

// d(bilerp)/d(row) and d(bilerp)/d(col) (floor has zero gradient: one-sided).
__device__ __forceinline__ float dbilerp_row(float fc, float x00, float x01, float x10,
                                             float x11) {
  return fmaf(fc, x11 - x01, (1.0f - fc) * (x10 - x00));
}
__device__ __forceinline__ float dbilerp_col(float fr, float x00, float x01, float x10,
                                             float x11) {
  return fmaf(fr, x11 - x10, (1.0f - fr) * (x01 - x00));
}

__device__ __forceinline__ float ldx(const float* __restrict__ xp, int r, int c, const Geo& g) {
  return (r >= 0 && r < g.H && c >= 0 && c < g.W) ? xp[r * g.W + c] : 0.f;
}

// XCD-aware block order (cdna_hip_programming.md §5.5 T1, bijective form): the
// dispatcher deals blocks round-robin over the 8 XCDs, so give the blocks that share
// an XCD (equal linear id mod 8) a contiguous range of logical ids. Neighbouring
// logical blocks then reuse each other's x / ∂col rows through that XCD's L2. Speed
// only: correctness never depends on placement.
struct Block3 {
  unsigned x, y, z;
};
__device__ __forceinline__ Block3 xcd_block() {
  const unsigned nx = gridDim.x, ny = gridDim.y;
  const unsigned nwg = nx * ny * gridDim.z;
  const unsigned bid = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const unsigned q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  const unsigned lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  Block3 o;
  o.x = lid % nx;
  o.y = (lid / nx) % ny;
  o.z = lid / (nx * ny);
  return o;
}

// Sum of v over the 64 lanes of a wave, on the VALU (DPP), result wave-uniform: pairs and
// quads (quad_perm), half rows and rows (row_half_mirror, row_mirror), then rows
// 0+1 / 2+3 (row_bcast:15) and halves (row_bcast:31) into lane 63. Fixed order:
// deterministic. (gfx9-family DPP; no LDS round trips unlike __shfl_xor.)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xf, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);        // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);        // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);       // row_half_mirror
  v += dpp_f<0x140>(v);       // row_mirror
  v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// The 64-lane sums of eight values at once, in wave_sum's association order (lane pairs,
// quads, half rows, rows, then (row 0 + row 1) + (row 2 + row 3)), so each sum has wave_sum's
// bits. The first three levels also halve the values held per lane: a lane keeps one value of
// each pair and receives its partner's share of it (two selects and one DPP add per kept
// value). Which one it keeps follows lane bits b0 ^ b2, b1 ^ b2, b2 at the three levels: each
// level's partners (lane ^ 1, lane ^ 2, then row_half_mirror's k and 7 - k, all three bits
// flipped) differ in that level's selector and agree in the earlier ones, so they hold the
// same values. The last three levels fold the one value left (row_ror:8 = lane ^ 8,
// then v_permlane16_swap and v_permlane32_swap of the value with itself). 28 VALU for the eight
// sums where wave_sum takes about 17 per sum. wave_sum8_lane(k) names a lane holding sum k.
template <int CTRL>
__device__ __forceinline__ float half_fold(bool hi, float a, float b) {
  // lanes with hi keep b, the others a; each adds its partner's copy of what it keeps
  return (hi ? b : a) + dpp_f<CTRL>(hi ? a : b);
}
__device__ __forceinline__ float swap_fold16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_fold32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave_sum8(const float (&v)[8], int lane) {
  const bool b0 = lane & 1, b1 = (lane >> 1) & 1, b2 = (lane >> 2) & 1;
  const bool h1 = b0 ^ b2, h2 = b1 ^ b2;
  const float p0 = half_fold<0xB1>(h1, v[0], v[4]), p1 = half_fold<0xB1>(h1, v[1], v[5]);
  const float p2 = half_fold<0xB1>(h1, v[2], v[6]), p3 = half_fold<0xB1>(h1, v[3], v[7]);
  const float q0 = half_fold<0x4E>(h2, p0, p2), q1 = half_fold<0x4E>(h2, p1, p3);
  float d = half_fold<0x141>(b2, q0, q1);  // row_half_mirror
  d += dpp_f<0x128>(d);                    // row_ror:8 (wave_sum: row_mirror, same sums)
  return swap_fold32(swap_fold16(d));
}
// lane bits of sum k: b2 = bit 0 of k, b1 ^ b2 = bit 1, b0 ^ b2 = bit 2
__host__ __device__ constexpr int wave_sum8_lane(int k) {
  return (((k >> 2) ^ k) & 1) | ((((k >> 1) ^ k) & 1) << 1) | ((k & 1) << 2);
}

// Workgroup barrier that orders LDS only: __syncthreads()'s fence would also drain every
// outstanding global load and store (vmcnt(0)), i.e. the prefetch pipelines kept in flight
// across the barrier (fused forward: the column stores of a k step; K5: the ∂col rows).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
// D(16x16) += A(16x4)·B(4x16), exact f32 (k-ordered fmaf chain). Lane l holds A[l&15][l>>4],
// B[l>>4][l&15] and D[4*(l>>4) + r][l&15] in register r.
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Four 16x16x4 f32 MFMAs sharing the B operand / five sharing the A operand. Builtins, not
// inline asm (r03): an asm MFMA is opaque to hipcc, which then neither pads the wait states
// between it and the compiler's own accesses of its AGPRs / source VGPRs nor counts them
// (cdna_hip_programming.md §5.7); r01-r02 shipped them as asm with hand-placed s_nops and
// "+a" accumulators, which the register allocator could still copy between asm statements.
__device__ __forceinline__ void mfma16x4_acc(f32x4& c0, f32x4& c1, f32x4& c2, f32x4& c3, float a0,
                                             float a1, float a2, float a3, float b) {
  c0 = mfma16(a0, b, c0);
  c1 = mfma16(a1, b, c1);
  c2 = mfma16(a2, b, c2);
  c3 = mfma16(a3, b, c3);
}
__device__ __forceinline__ void mfma16x4_a5(f32x4& c0, f32x4& c1, f32x4& c2, f32x4& c3, f32x4& c4,
                                            float a, float b0, float b1, float b2, float b3,
                                            float b4) {
  c0 = mfma16(a, b0, c0);
  c1 = mfma16(a, b1, c1);
  c2 = mfma16(a, b2, c2);
  c3 = mfma16(a, b3, c3);
  c4 = mfma16(a, b4, c4);
}

// Row of D[row][col] held in register r by lane half hi, for 32x32 MFMA tiles.
__device__ __forceinline__ int drow(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

}  // namespace dcn
