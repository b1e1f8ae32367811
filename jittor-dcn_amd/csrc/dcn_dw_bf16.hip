// dcn_dw_bf16.hip — the bf16 ∂W product of the backward over the stored columns,
// ∂Wf[o][k] = Σ_p ∂outT[p][o] · col[p][k] (autodiff of /root/reference/deform_conv.py:76,
// the weight read in the Q5 flat order of :74), as a split-K streaming
// MFMA kernel for gfx950.
//
// The product is 256 × K outputs over a reduction of B·HW pixels (50,176 at config 4): both
// operands stream (the 231 MB column matrix once, ∂outT once per column tile) and the
// output is tiny, so it is an HBM stream with MFMA work on the side (59 GFLOP = 24 µs at the
// bf16 peak; 257 MB = 43 µs at 6 TB/s). hipBLASLt's grouped GEMM took 0.117-0.133 ms
// (DESIGN.md §4 bf16 ∂W). Here:
//   * a workgroup (8 waves, one per CU) owns one 256 (o) × 256 (k) tile over one range of
//     pixels and writes it as an fp32 partial plane; a fixed-order sum over the ranges
//     follows (launch_sum_partials), so the result is deterministic;
//   * both operands are [pixel][256] bf16 rows (∂outT rows, and the tile's 512-B slice of
//     each column row); 32-pixel stages of both are copied HBM -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, whole 512-B rows), four stages in a 128 KiB ring, three in
//     flight while one is consumed: each wave waits for its own DMAs with a counted vmcnt,
//     then one raw s_barrier per stage publishes the stage to every wave and frees the
//     oldest buffer for the next DMA (cdna_hip_programming.md §5 "Pipelining across
//     barriers");
//   * the reduction (pixel) index is the row of both LDS images, so both MFMA operands are
//     read with the hardware transpose (ds_read_b64_tr_b16: 4 pixel rows × 16 columns per
//     16-lane group); the 16-B chunks of row r sit XOR-swizzled by 4·(r & 3) (written so by
//     the DMA's per-lane source addresses), which makes every transposed read conflict-free;
//   * 8 waves as 2 (o) × 4 (k), each 128 o × 64 k = 4 × 2 accumulators of
//     v_mfma_f32_32x32x16_bf16;
//   * the column tiles of one pixel range run on one XCD (bijective remap), so its ∂outT
//     rows come from HBM once and from that XCD's L2 for the other tiles.
// Rounding: exact bf16 products summed in fp32 (MFMA), per range, then over the ranges in
// range order: another summation order than the vendor GEMM's, so elements may differ from
// it by fp32 rounding (both are checked against the oracle).
#include <algorithm>

#include "dcn_device.h"

namespace dcn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// Pipeline shape (compile-time; the A/B builds of DESIGN.md §4 set them with -D): DW_PX
// pixels per stage (16 or 32), DW_RING LDS stages. (The round-5 variants: non-temporal column
// DMAs, DMAs issued before the stage barrier, a scheduling pin after the MFMAs, and the
// diagnostic ablations are gone; their A/B results are in DESIGN.md §4 and
// profiles/r05_dw_ab.txt.)
#ifndef DW_PX
#define DW_PX 32
#endif
#ifndef DW_RING
#define DW_RING 4
#endif
constexpr int kDwO = 256;                          // output channels: the tile's rows
constexpr int kDwN = 256;                          // ∂W columns per tile
constexpr int kDwPx = DW_PX;                       // pixels per stage
constexpr int kDwRing = DW_RING;                   // LDS stages
constexpr int kDwAhead = kDwRing - 1;       // stages issued ahead of the one consumed
constexpr int kDwRowB = 512;                       // one pixel row of either operand (256 bf16)
constexpr int kDwOpB = kDwPx * kDwRowB;            // 16 KiB per operand per 32-pixel stage
constexpr int kDwStageB = 2 * kDwOpB;              // A (∂outT) then B (columns)
constexpr int kDwLds = kDwRing * kDwStageB;        // 128 KiB (4 × 32 px)
constexpr int kDwWaves = 8;
// DW_LOADERS: the waves that issue the stage DMAs (waves 0 .. DW_LOADERS - 1; all 8 by default)
#ifndef DW_LOADERS
#define DW_LOADERS 8
#endif
constexpr int kDwLoaders = DW_LOADERS;
static_assert(kDwLoaders == 2 || kDwLoaders == 4 || kDwLoaders == 8, "loader waves");
constexpr int kDwGlds = kDwStageB / (kDwLoaders * 1024);  // DMA instructions per loader per stage
constexpr int kDwOpI = kDwPx / 2;                  // DMA instructions per operand (2 rows each)
static_assert(kDwPx == 16 || kDwPx == 32, "stage = one or two 16-pixel k-steps");
static_assert(kDwRing >= 3 && kDwRing <= 8, "ring depth");
static_assert(kDwLds <= 160 * 1024, "one workgroup per CU");

// byte offset of 16-B chunk `ch` of row `r` in an operand image
__host__ __device__ constexpr int dw_chunk(int r, int ch) { return r * kDwRowB + ((ch ^ (4 * (r & 3))) << 4); }

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left alone) as the builtin, not inline asm: hipcc's
// wait-count pass then knows which DMAs it retired and adds no drain of its own before the
// reads that follow
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// grid: nwg = ranges × ntile workgroups of 512 threads; range r covers stages
// [r·spr, min((r+1)·spr, nst)) of 32 pixels
__global__ __launch_bounds__(kDwWaves * 64, 1) void dw_stream_bf16(
    const bf16_t* __restrict__ goutT, const bf16_t* __restrict__ col, float* __restrict__ parts,
    int K, int npix, int ntile, int spr, int nwg) {
  // the ring: one static LDS object per slot, so that hipcc's wait-count pass can tell a
  // transposed read of one slot from the DMAs in flight into the others (distinct objects get
  // distinct alias scopes) and does not drain every DMA before each read (it did, with one
  // dynamic array: s_waitcnt vmcnt(0) before the first read of every stage)
  __shared__ __attribute__((aligned(1024))) char ring0[kDwStageB], ring1[kDwStageB],
      ring2[kDwStageB], ring3[kDwStageB];
#if DW_RING > 4
  __shared__ __attribute__((aligned(1024))) char ring4[kDwStageB];
#endif
#if DW_RING > 5
  __shared__ __attribute__((aligned(1024))) char ring5[kDwStageB];
#endif
#if DW_RING > 6
  __shared__ __attribute__((aligned(1024))) char ring6[kDwStageB];
#endif
#if DW_RING > 7
  __shared__ __attribute__((aligned(1024))) char ring7[kDwStageB];
#endif
  char* const slots[8] = {ring0, ring1, ring2, ring3,
#if DW_RING > 4
                          ring4,
#else
                          nullptr,
#endif
#if DW_RING > 5
                          ring5,
#else
                          nullptr,
#endif
#if DW_RING > 6
                          ring6,
#else
                          nullptr,
#endif
#if DW_RING > 7
                          ring7
#else
                          nullptr
#endif
  };
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = wg % ntile, range = wg / ntile;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nst_all = (npix + kDwPx - 1) / kDwPx;
  const int s0 = range * spr, nst = min(spr, nst_all - s0);
  if (nst <= 0) return;  // workgroup-uniform, before any barrier
  const int px0 = s0 * kDwPx;

  // ---- DMA of stage j (clamped to the range's last stage) into a ring slot: instruction u
  // of wave w moves rows 2i, 2i + 1 (i = (u·8 + w) % 16) of operand (u·8 + w) / 16 (wave-
  // uniform); lane L writes physical chunk L & 31 of row 2i + (L >> 5), i.e. fetches logical
  // chunk (L & 31) ^ 4·(row & 3). Byte offsets are 32-bit (dw_stream_bf16_ok).
  const int lrow = lane >> 5, lpc = lane & 31;
  const char* opbase[2] = {reinterpret_cast<const char*>(goutT),
                           reinterpret_cast<const char*>(col) + (size_t)tile * kDwN * 2};
  const unsigned opstride[2] = {(unsigned)kDwRowB, (unsigned)K * 2u};
  auto issue = [&](int j, char* slot) {
    if (w >= kDwLoaders) return;  // wave-uniform
    j = min(j, nst - 1);  // past the range: re-read its last stage (L2), never read back
#pragma unroll
    for (int u = 0; u < kDwGlds; ++u) {
      const int ii = u * kDwLoaders + w, op = ii / kDwOpI, i = ii % kDwOpI;
      const int row = 2 * i + lrow;
      const unsigned ch = (unsigned)(lpc ^ (4 * (row & 3)));
      const int p = min(px0 + j * kDwPx + row, npix - 1);  // past the end: re-read the last row
      const char* src = opbase[op] + ((unsigned)p * opstride[op] + ch * 16u);
      __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(slot + op * kDwOpB + i * 1024),
                                       16, 0, 0);
    }
  };

  // ---- transposed fragment reads. 16-lane group g = lane >> 4 reads pixel rows
  // 8(g >> 1) + q (+4 for the second half of the fragment), columns c0 + 16(g & 1) + 4p, with
  // q = (lane >> 2) & 3, p = lane & 3; lane i of the group gets column i of the four rows.
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int frow = 8 * (g >> 1) + q;  // row of the first read within a 16-pixel k-step
  const int wo = w >> 2, wk = w & 3;
  // in-operand byte offsets of this lane's reads (k-step 0, first half), per o tile / k tile
  int aoff[4], boff[2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
    aoff[mi] = dw_chunk(frow, (128 * wo + 32 * mi + 16 * (g & 1)) / 8 + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
    boff[ni] = kDwOpB + dw_chunk(frow, (64 * wk + 32 * ni + 16 * (g & 1)) / 8 + (pp >> 1)) +
               8 * (pp & 1);
  auto rd = [&](const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)p);
  };
  auto frag = [&](const char* p) {  // 8 pixels: rows frow.. +3 and frow + 4 .. + 7
    const bf16x4 lo = rd(p), hi = rd(p + 4 * kDwRowB);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[mi][ni][j] = 0.f;

  // one stage: two 16-pixel k-steps, 8 MFMAs each. nvalid < 32 only in the last stage of the
  // launch: the ∂outT rows past the end (DMA'd from the last row) are zeroed in the A
  // fragments, so their products vanish
  auto compute = [&](const char* slot, int nvalid) {
#pragma unroll
    for (int ks = 0; ks < kDwPx / 16; ++ks) {
      const char* base = slot + ks * 16 * kDwRowB;
      bf16x8 a[4], b[2];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = frag(base + aoff[mi]);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b[ni] = frag(base + boff[ni]);
      if (nvalid < kDwPx) {
        // element e of a lane's fragment is pixel row 16ks + 8(g >> 1) + (e & 3) + 4(e >> 2)
        const int r0 = 16 * ks + 8 * (g >> 1);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (r0 + (e & 3) + 4 * (e >> 2) >= nvalid) a[mi][e] = (__bf16)0.f;
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  // stage s lives in slot s % 4; the loop is unrolled by the ring size so that every slot is
  // a compile-time LDS object
  // (every step issues its DMAs, clamped past the range, so the pending count is the same in
  // every step and on every path: hipcc's own wait before a slot's first read then never
  // drains the queue)
  auto step = [&](int s, char* cur, char* refill) {
    // this wave's DMAs of stage s have landed once only those of s + 1 .. s + kDwAhead - 1
    // are pending
    vm_wait<(kDwAhead - 1) * kDwGlds>();
    // every wave's DMAs of stage s landed; every wave finished reading stage s - 1, whose
    // slot (`refill`) the DMA of stage s + kDwAhead now refills
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue(s + kDwAhead, refill);
    __builtin_amdgcn_sched_barrier(0);
    compute(cur, min(kDwPx, npix - (px0 + s * kDwPx)));
  };
  // (slot k + kDwAhead is refilled while slot k is read; the loops are fully unrolled, so
  // every slot pointer is a compile-time LDS object)
#pragma unroll
  for (int k = 0; k < kDwAhead; ++k) issue(k, slots[k]);
  int s = 0;
  for (; s + kDwRing <= nst; s += kDwRing) {
#pragma unroll
    for (int k = 0; k < kDwRing; ++k) step(s + k, slots[k], slots[(k + kDwAhead) % kDwRing]);
  }
#pragma unroll
  for (int k = 0; k < kDwRing - 1; ++k)
    if (s + k < nst) step(s + k, slots[k], slots[(k + kDwAhead) % kDwRing]);
  vm_wait<0>();  // no DMA may land in LDS after the workgroup has ended

  // ---- partial plane `range`: D row i = o, column j = k; lane (n = l & 31, h = l >> 5),
  // register r holds row drow(r, h), column n: two 128-B runs per store instruction
  float* dst = parts + (size_t)range * kDwO * K + (size_t)tile * kDwN;
  const int n = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = 128 * wo + 32 * mi + drow(r, hh);
        dst[(size_t)o * K + 64 * wk + 32 * ni + n] = acc[mi][ni][r];
      }
}

void dw_plan(int K, long npix, int* ntile, int* spr, int* ranges) {
  *ntile = K / kDwN;
  const int nst = (int)((npix + kDwPx - 1) / kDwPx);
  int r = std::max(1, std::min(nst, 256 / std::max(1, *ntile)));
  *spr = (nst + r - 1) / r;
  *ranges = (nst + *spr - 1) / *spr;
}

}  // namespace

bool dw_stream_bf16_ok(int K, int O, long npix) {
  // 32-bit byte offsets into ∂outT and the columns (the DMA source addresses)
  return O == kDwO && K > 0 && K % kDwN == 0 && npix > 0 && npix * kDwRowB < (1l << 31) &&
         npix * K * 2 < (1l << 31);
}

int dw_stream_bf16_ranges(int K, long npix) {
  int nt, spr, r;
  dw_plan(K, npix, &nt, &spr, &r);
  return r;
}

hipError_t launch_dw_stream_bf16(const bf16_t* goutT, const bf16_t* col, float* parts, int K,
                                 int O, long npix, hipStream_t s) {
  if (!dw_stream_bf16_ok(K, O, npix)) return hipErrorInvalidValue;
  int ntile, spr, ranges;
  dw_plan(K, npix, &ntile, &spr, &ranges);
  const int nwg = ranges * ntile;
  hipLaunchKernelGGL(dw_stream_bf16, dim3(nwg), dim3(kDwWaves * 64), 0, s, goutT, col,
                     parts, K, (int)npix, ntile, spr, nwg);
  return hipGetLastError();
}

}  // namespace dcn
