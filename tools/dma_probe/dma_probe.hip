// dma_probe.hip — the LDS-DMA stream of dw_stream_bf16 (csrc/dcn_dw_bf16.hip) without its
// MFMAs, and variants that each change one property of it, to find what sets its rate
// (VERDICT r05 item 2). Standalone: hipcc --offload-arch=gfx950 -O3 -o dma_probe dma_probe.hip
//
// Shape of config 4's ∂W: npix = 64·784 pixels, K = 2304 columns (9 tiles of 256), O = 256.
// dw pattern: 252 workgroups of 512 threads (28 pixel ranges × 9 column tiles, consecutive
// workgroups of an XCD = the 9 tiles of one range), a ring of R slots of 32 KiB, R - 1 stages
// ahead; stage = 32 pixel rows of ∂outT (512 B each, contiguous) + 32 rows of the tile's 512-B
// slice of the 4608-B column rows; per stage each wave waits for its own DMAs of the stage,
// then the workgroup barrier, then the DMAs of stage s + R - 1. No LDS reads, no MFMAs.
//
// Modes (argv[1]):
//   dw        the pattern above
//   l2        dw with every source row inside the first 64 pixels (all L2 hits): the fill
//             rate a CU reaches when HBM is not involved
//   contig    dw with the column operand read as if stored [tile][pixel][256] (each stage's
//             16 KiB contiguous)
//   unique    dw with the ∂outT half replaced by a second column tile (no row is read twice:
//             every byte from HBM)
//   stream    each workgroup streams its own contiguous 1.79 MB (= its dw byte count) from a
//             462 MB buffer through the same ring: plain HBM streaming by LDS-DMA
//   stream1   stream with one loader wave per workgroup (the guide's ldsdma-fill shape)
//   dw2       dw with two workgroups per CU (504 workgroups, R-slot rings of 16 KiB stages:
//             16 pixels per stage)
// argv[2]: ring slots R (3..4 for 32 KiB stages), argv[3]: launches timed, argv[4]: 1 = write a
// 512 MB buffer before every launch (the sources cold, the Infinity Cache full of dirty lines),
// 2 = read it (cold sources, clean cache); each launch then timed alone.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kNpix = 64 * 784, kK = 2304, kTiles = 9, kRowB = 512;

enum Mode { DW, L2, CONTIG, UNIQUE, STREAM, STREAM1, DW2 };

template <int N>
__device__ __forceinline__ void vm_wait() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

struct Args {
  const char* gout;  // [npix][512 B]
  const char* col;   // [npix][4608 B]
  const char* big;   // stream modes: 462 MB
  float* sink;
  int mode, ntile, spr, nwg, px_per_stage;
};

// PX pixels per stage (32: 32 KiB stages, 16: 16 KiB), R ring slots
template <int PX, int R>
__global__ __launch_bounds__(512) void probe(Args a) {
  constexpr int kOpB = PX * kRowB, kStageB = 2 * kOpB, kGlds = kStageB / (8 * 1024);
  constexpr int kAhead = R - 1, kOpI = PX / 2;
  __shared__ __attribute__((aligned(1024))) char ring[R * kStageB];
  const int bid = blockIdx.x, xcd = bid & 7, q8 = a.nwg >> 3, r8 = a.nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = wg % a.ntile, range = wg / a.ntile;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nst_all = (kNpix + PX - 1) / PX;
  const int s0 = range * a.spr, nst = min(a.spr, nst_all - s0);
  if (nst <= 0) return;
  const int px0 = s0 * PX;
  const int lrow = lane >> 5, lpc = lane & 31;
  const int mode = a.mode;

  auto src_of = [&](int j, int op, int row) -> const char* {
    const unsigned ch = (unsigned)(lpc ^ (4 * (row & 3)));
    int p = min(px0 + j * PX + row, kNpix - 1);
    if (mode == STREAM || mode == STREAM1) {
      // this workgroup's contiguous block: stage j = 2·kOpB bytes
      const size_t blk = (size_t)wg * a.spr * kStageB;
      return a.big + blk + (size_t)j * kStageB + (size_t)op * kOpB + (size_t)row * kRowB + ch * 16u;
    }
    if (mode == L2) p &= 63;
    if (op == 0 && mode != UNIQUE) return a.gout + (size_t)p * kRowB + ch * 16u;
    const int t = op == 0 ? (tile + 1) % kTiles : tile;  // UNIQUE: another tile's slice
    if (mode == CONTIG)
      return a.col + ((size_t)t * kNpix + p) * kRowB + ch * 16u;
    return a.col + (size_t)p * kK * 2 + (size_t)t * kRowB + ch * 16u;
  };
  auto issue = [&](int j, char* slot) {
    if (mode == STREAM1 && w != 0) return;
    j = min(j, nst - 1);
    if (mode == STREAM1) {
#pragma unroll
      for (int u = 0; u < kGlds * 8; ++u) {
        const int op = u / kOpI, i = u % kOpI, row = 2 * i + lrow;
        __builtin_amdgcn_global_load_lds((gvoid*)src_of(j, op, row),
                                         (lvoid*)(slot + op * kOpB + i * 1024), 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < kGlds; ++u) {
      const int ii = u * 8 + w, op = ii / kOpI, i = ii % kOpI, row = 2 * i + lrow;
      __builtin_amdgcn_global_load_lds((gvoid*)src_of(j, op, row),
                                       (lvoid*)(slot + op * kOpB + i * 1024), 16, 0, 0);
    }
  };
  for (int k = 0; k < kAhead; ++k) issue(k, ring + k * kStageB);
  for (int s = 0; s < nst; ++s) {
    if (mode == STREAM1) vm_wait<((kAhead - 1) * kGlds * 8 < 63 ? (kAhead - 1) * kGlds * 8 : 63)>();
    else vm_wait<(kAhead - 1) * kGlds>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue(s + kAhead, ring + ((s + kAhead) % R) * kStageB);
    __builtin_amdgcn_sched_barrier(0);
  }
  vm_wait<0>();  // no DMA may land after the workgroup ends
}

// the clean flush: reads n16 × 16 B (the sum is never stored)
__global__ __launch_bounds__(256) void sweep(const uint4* __restrict__ p, size_t n16, int* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = 1;
}

int main(int argc, char** argv) {
  const char* ms = argc > 1 ? argv[1] : "dw";
  const int R = argc > 2 ? atoi(argv[2]) : 4;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const char* names[] = {"dw", "l2", "contig", "unique", "stream", "stream1", "dw2"};
  int mode = -1;
  for (int i = 0; i < 7; ++i)
    if (!strcmp(ms, names[i])) mode = i;
  if (mode < 0 || R < 3 || R > 4) {
    fprintf(stderr, "usage: dma_probe MODE [R=3|4] [reps]\n");
    return 2;
  }
  const int px = mode == DW2 ? 16 : 32;
  const size_t goutB = (size_t)kNpix * kRowB, colB = (size_t)kNpix * kK * 2;
  char *gout, *col, *big = nullptr;
  float* sink;
  CK(hipMalloc(&gout, goutB));
  CK(hipMalloc(&col, colB));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(gout, 1, goutB));
  CK(hipMemset(col, 2, colB));
  Args a{gout, col, nullptr, sink, mode, kTiles, 0, 0, px};
  const int nst = (kNpix + px - 1) / px;
  const int ranges_target = mode == DW2 ? 56 : 28;
  a.spr = (nst + ranges_target - 1) / ranges_target;
  const int ranges = (nst + a.spr - 1) / a.spr;
  a.nwg = ranges * kTiles;
  const size_t stageB = 2 * (size_t)px * kRowB;
  if (mode == STREAM || mode == STREAM1) {
    const size_t bigB = (size_t)a.nwg * a.spr * stageB;
    CK(hipMalloc(&big, bigB));
    CK(hipMemset(big, 3, bigB));
    a.big = big;
  }
  auto launch = [&]() {
    if (px == 32 && R == 4) hipLaunchKernelGGL((probe<32, 4>), dim3(a.nwg), dim3(512), 0, 0, a);
    else if (px == 32) hipLaunchKernelGGL((probe<32, 3>), dim3(a.nwg), dim3(512), 0, 0, a);
    else if (R == 4) hipLaunchKernelGGL((probe<16, 4>), dim3(a.nwg), dim3(512), 0, 0, a);
    else hipLaunchKernelGGL((probe<16, 3>), dim3(a.nwg), dim3(512), 0, 0, a);
  };
  const int cold = argc > 4 ? atoi(argv[4]) : 0;
  char* flush = nullptr;
  const size_t flushB = 512ull << 20;
  if (cold) {
    CK(hipMalloc(&flush, flushB));
    CK(hipMemset(flush, 5, flushB));
  }
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms_tot = 0.f;
  if (cold) {
    for (int i = 0; i < reps; ++i) {
      if (cold == 1)
        CK(hipMemsetAsync(flush, i & 0xff, flushB, 0));
      else
        hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0,
                           reinterpret_cast<const uint4*>(flush), flushB / 16, (int*)sink);
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms_tot += ms;
    }
    CK(hipFree(flush));
  } else {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms_tot, e0, e1));
  }
  const double us = 1e3 * ms_tot / reps;
  const double through = (double)a.nwg * a.spr * stageB;  // bytes moved into LDS (or regs)
  printf("{\"mode\": \"%s\", \"cold\": %d, \"ring\": %d, \"stage_px\": %d, \"workgroups\": %d, \"stages_per_wg\": %d, "
         "\"us\": %.2f, \"through_MB\": %.1f, \"through_TBps\": %.3f, \"per_wg_GBps\": %.2f}\n",
         ms, cold, R, px, a.nwg, a.spr, us, through / 1e6, through / us / 1e6,
         through / a.nwg / us / 1e3);
  CK(hipFree(gout));
  CK(hipFree(col));
  CK(hipFree(sink));
  if (big) CK(hipFree(big));
  return 0;
}
