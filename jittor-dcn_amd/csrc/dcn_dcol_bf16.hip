// dcn_dcol_bf16.hip — the bf16 ∂columns product of the backward, ∂colT[p][k] =
// Σ_o ∂outT[p][o] · Wf[o][k] (autodiff of /root/reference/deform_conv.py:76, the ∂S GEMM of
// SURVEY.md §8 a11/a13), as a short-K streaming kernel for gfx950.
//
// The product has a reduction depth of only O = 256 but writes B·HW × K bf16 (231 MB at
// config 4), so a vendor GEMM spends each tile's short k-loop in prologue and epilogue
// (hipBLASLt: 0.102 ms, 0.23 of the bf16 MFMA peak). Here the re-used operand
// stays on chip for the whole launch and the other one streams past it:
//   * a workgroup (8 waves, one per CU) owns 256 ∂col columns (k): their Wf slice
//     (256 columns × 256 o, 128 KiB) is copied once into LDS, already in
//     v_mfma_f32_32x32x16_bf16 A-fragment order (lane-linear, conflict-free `ds_read_b128`),
//     from a pre-swizzled copy of Wf;
//   * each wave walks its own 32-pixel tiles of the workgroup's pixel range: a tile's ∂outT
//     rows (32 × 512 B) go straight into registers as the B fragments, and the next tile's
//     are loaded while this one computes (two register sets); no barrier after the A copy;
//   * the A rows of each 32-row tile are permuted (dc_perm) so that the accumulator rows a
//     lane holds are 16 consecutive k; a pair of row tiles (64 columns × 32 pixels) passes
//     through a per-wave 4-KiB LDS stage, so each store instruction writes 8 whole 128-B
//     lines (the MFMA layout alone gives 32 lines × 2 pieces of 16 B per instruction);
//   * stores are non-temporal;
//   * the row groups of one pixel range run on one XCD (bijective remap), so the L2 serves
//     a tile's ∂outT rows to all of them after the first read.
// Rounding: fp32 accumulation over o inside the MFMA, one round-to-nearest-even to bf16 per
// element, as the vendor GEMM's bf16 D (the summation order may differ, so elements can
// differ from hipBLASLt's by one bf16 ulp; both are checked against the oracle).
#include <mutex>
#include <vector>

#include "dcn_device.h"
#include "dcn_swizzle.h"


namespace dcn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

constexpr int kDcO = 256;                        // reduction depth (output channels)
constexpr int kDcKS = kDcO / 16;                 // 32x32x16 k-steps over it
constexpr int kDcRows = 256;                     // ∂col columns per workgroup
constexpr int kDcMT = kDcRows / 32;              // their 32-row MFMA tiles
constexpr int kDcWaves = 8;                      // two waves per SIMD, one workgroup per CU
constexpr int kDcLds = kDcMT * kDcKS * 64 * 16;  // the A image: 128 KiB
// A-fragment reads this many k-steps ahead of their MFMAs (r04 dcol6: 1 is 5 % slower; 3,
// and s_setprio 1 around the MFMAs, no change)
constexpr int kDcLA = 2;
constexpr int kDcLdsAll = kDcLds + kDcWaves * 4096;  // + a 4-KiB output stage per wave
// ∂col stores non-temporal (buffer cache policy bit 1, `nt`): r06 A/B at config 4, dcol
// 0.077 -> 0.070-0.074 ms and the step -12 µs (the 231 MB leave the Infinity Cache clean for
// K5's reads, the fused forward's column policy). A role-split form of this kernel (one
// loader wave filling an LDS ring, compute waves that only store) measured 0.079-0.089 ms in
// six variants and was dropped.
constexpr int kNT = 2;
static_assert(kDcLdsAll <= 160 * 1024, "one workgroup per CU");

__device__ __forceinline__ unsigned pack_bf16(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

__device__ __forceinline__ u32x4 pack4(const f32x16& v, int j0) {
  return u32x4{pack_bf16(v[j0], v[j0 + 1]), pack_bf16(v[j0 + 2], v[j0 + 3]),
               pack_bf16(v[j0 + 4], v[j0 + 5]), pack_bf16(v[j0 + 6], v[j0 + 7])};
}

// grid: nwg = ranges × nrg workgroups of 512 threads; range = tpr consecutive 32-pixel
// tiles, dealt to the 8 waves round-robin
__global__ __launch_bounds__(kDcWaves * 64, 2) void dcol_bf16(const bf16_t* __restrict__ wz,
                                                              const bf16_t* __restrict__ goutT,
                                                              bf16_t* __restrict__ col, int K,
                                                              int npix, int nrg, int tpr,
                                                              int nwg) {
  extern __shared__ __attribute__((aligned(16))) char dl[];
  const bf16_t* As = reinterpret_cast<const bf16_t*>(dl);
  // XCD remap (bijective for any nwg): consecutive wg share an XCD, so one range's row
  // groups read its ∂outT rows through one L2
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int rg = wg % nrg, range = wg / nrg;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntile = (npix + 31) / 32;
  const int t0 = range * tpr, t1 = min(t0 + tpr, ntile);
  if (t0 >= t1) return;  // workgroup-uniform, before the barrier

  // the A image: tiles rg·8 .. rg·8 + 7 of wz (one contiguous 128 KiB) by LDS-DMA; 16-B unit
  // i0 + lane with i0 = 512u + 64w, one KiB per wave-instruction
  const bf16_t* asrc = wz + (size_t)rg * kDcMT * kDcKS * 512;
#pragma unroll
  for (int u = 0; u < kDcLds / (kDcWaves * 1024); ++u) {
    const int i0 = (u * kDcWaves + w) * 64;
    __builtin_amdgcn_global_load_lds((gvoid*)(asrc + (size_t)(i0 + lane) * 8),
                                     (lvoid*)(dl + (size_t)i0 * 16), 16, 0, 0);
  }
  // B fragments of 32-pixel tile t: lane (n = l & 31, h = l >> 5) holds, for k-step ks,
  // ∂outT[pixel 32t + n][16ks + 8h .. +8). Pixels past the end re-read the last one (their
  // results are dropped by the stores' range check).
  auto load_b = [&](int tile, bf16x8(&b)[kDcKS]) {
    const int p = min(tile * 32 + (lane & 31), npix - 1);
    const bf16_t* src = goutT + (size_t)p * kDcO + 8 * (lane >> 5);
#pragma unroll
    for (int ks = 0; ks < kDcKS; ++ks) b[ks] = *reinterpret_cast<const bf16x8*>(src + 16 * ks);
  };
  bf16x8 b0[kDcKS], b1[kDcKS];
  int t = t0 + w;
  if (t < t1) load_b(t, b0);
  __syncthreads();  // the A image has landed; the only barrier (waves run independently after)
  // stores through a buffer resource: a pixel past the end gets an offset past the range
  const auto rcol = __builtin_amdgcn_make_buffer_rsrc(col, 0, (int)((size_t)npix * K * 2),
                                                      0x00020000);
  const int kr = rg * kDcRows;  // the workgroup's first ∂col column
  char* stage = dl + kDcLds + w * 4096;
  // tile tc from bc while tile tc + 8 loads into bn; row tiles in pairs (two 32x32
  // accumulators), each pair stored as soon as it is done
  auto tile = [&](int tc, const bf16x8(&bc)[kDcKS], bf16x8(&bn)[kDcKS]) {
    if (tc + kDcWaves < t1) load_b(tc + kDcWaves, bn);
#pragma unroll
    for (int pr = 0; pr < kDcMT / 2; ++pr) {
      f32x16 acc0, acc1;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc0[j] = acc1[j] = 0.f;
      // A fragments two k-steps ahead of their MFMAs, the order pinned (left to itself hipcc
      // hoists all 32 reads of the pair and spills)
      auto lda = [&](int m, int ks) {
        return *reinterpret_cast<const bf16x8*>(As + ((m * kDcKS + ks) * 64 + lane) * 8);
      };
      constexpr int LA = kDcLA;
      bf16x8 ra[LA + 1][2];
#pragma unroll
      for (int d = 0; d < LA; ++d) ra[d][0] = lda(2 * pr, d), ra[d][1] = lda(2 * pr + 1, d);
#pragma unroll
      for (int ks = 0; ks < kDcKS; ++ks) {
        if (ks + LA < kDcKS)
          ra[(ks + LA) % (LA + 1)][0] = lda(2 * pr, ks + LA),
          ra[(ks + LA) % (LA + 1)][1] = lda(2 * pr + 1, ks + LA);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[ks % (LA + 1)][0], bc[ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[ks % (LA + 1)][1], bc[ks], acc1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // row tiles 2pr, 2pr + 1 = columns 64pr .. 64pr + 63 of the tile's 32 pixels, through
      // the wave's 4-KiB LDS stage ([pixel][64 columns], 16-B chunk c of row r at c ^ (r & 7))
      // so that each store writes 8 pixels × one whole 128-B line
      {
        const int n = lane & 31, hh = lane >> 5;
        char* srow = stage + n * 128;
        auto put = [&](int c, const u32x4& v) {
          *reinterpret_cast<u32x4*>(srow + ((c ^ (n & 7)) << 4)) = v;
        };
        put(2 * hh, pack4(acc0, 0));
        put(2 * hh + 1, pack4(acc0, 8));
        put(4 + 2 * hh, pack4(acc1, 0));
        put(5 + 2 * hh, pack4(acc1, 8));
      }
      asm volatile("" ::: "memory");  // the stage's writes before its reads (one wave, in order)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 8 * i + (lane >> 3), c = lane & 7;
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + r * 128 + ((c ^ (r & 7)) << 4));
        const int p = tc * 32 + r;
        const unsigned o = p < npix ? (unsigned)(p * K + kr + 64 * pr + 8 * c) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(v, rcol, o, 0, kNT);
      }
      asm volatile("" ::: "memory");  // the reads before the next pair's writes
    }
  };
  for (; t < t1; t += 2 * kDcWaves) {
    tile(t, b0, b1);
    if (t + kDcWaves < t1) tile(t + kDcWaves, b1, b0);
  }
}


}  // namespace

bool dcol_bf16_ok(int K, int O, long npix) {
  // 32-bit byte offsets into the ∂columns (the buffer stores)
  return O == kDcO && K > 0 && K % kDcRows == 0 && npix > 0 && (long)npix * K * 2 < (1l << 31);
}

// the A fragments of 32-column tile T (dc_perm, swz_dcol: dcn_swizzle.h), 16 B per lane, written
// by the backward's prep launch; a row group's 8 tiles are one 128 KiB run
PrepJob prep_dcol(int K, const bf16_t* w, bf16_t* wz) {
  return PrepJob{PREP_DCOL, (long)(K / 32) * kDcKS * 64, w, wz, 0, K, 0, 0, 0, 0};
}

hipError_t launch_dcol_bf16(const bf16_t* wz, const bf16_t* goutT, bf16_t* col, int K, int O,
                            long npix, hipStream_t s) {
  if (!dcol_bf16_ok(K, O, npix)) return hipErrorInvalidValue;
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
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dcol_bf16),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kDcLdsAll);
      if (e != hipSuccess) return e;
      attr_set[dev] = 1;
    }
  }
  // one workgroup per CU: ranges × row groups ≈ 256
  const int nrg = K / kDcRows, ntile = (int)((npix + 31) / 32);
  int ranges = std::max(1, std::min(ntile, 256 / std::max(1, nrg)));
  const int tpr = (ntile + ranges - 1) / ranges;
  ranges = (ntile + tpr - 1) / tpr;
  const int nwg = ranges * nrg;
  hipLaunchKernelGGL(dcol_bf16, dim3(nwg), dim3(kDcWaves * 64), kDcLdsAll, s, wz, goutT, col, K,
                     (int)npix, nrg, tpr, nwg);
  return hipGetLastError();
}

}  // namespace dcn
