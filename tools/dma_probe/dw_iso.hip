// dw_iso.hip — dw_stream_bf16 (csrc/dcn_dw_bf16.hip, compiled in from the product source)
// timed alone at config 4's shape, and beside a stand-in for the sample-bin sort that shares
// the GPU with it in the step (64 workgroups of 1024 threads holding 100 KiB of LDS each for
// ≈36 µs, launched on a second stream just before it). Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Ijittor-dcn_amd/csrc \
//         -o tools/dma_probe/dw_iso tools/dma_probe/dw_iso.hip
// (-DDW_RING=3 etc. for the kernel's compile-time variants).
// Usage: dw_iso [reps] [blocker_us] [flush]: before each launch a 512 MB buffer is
//   flush 1: written (hipMemset: the Infinity Cache left full of dirty lines),
//   flush 2: read (clean cache, cold sources),
//   flush 3: written with non-temporal stores (the fused forward's column-store policy).
#include "dcn_dw_bf16.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// stand-in for bins_sort_seg's footprint: holds its CU's LDS for `cycles` ticks of the 100 MHz clock
__global__ __launch_bounds__(1024) void blocker(long long cycles, int* sink) {
  __shared__ int lds[25600];  // 100 KiB
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
  if (lds[(threadIdx.x + 1) & 1023] == -1) sink[0] = 1;  // (never)
}

__global__ __launch_bounds__(256) void sweep_rd(const uint4* __restrict__ p, size_t n16, int* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = 1;
}
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void sweep_nt(u4v* __restrict__ p, size_t n16, unsigned v) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(u4v{v, v, v, v}, p + i);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const double blk_us = argc > 2 ? atof(argv[2]) : 0.0;
  const int fl = argc > 3 ? atoi(argv[3]) : 1;
  const int K = 2304, O = 256;
  const long npix = 64L * 784;
  const int ranges = dcn::dw_stream_bf16_ranges(K, npix);
  dcn::bf16_t *gout, *col;
  float* parts;
  int* sink;
  CK(hipMalloc(&gout, npix * O * 2));
  CK(hipMalloc(&col, npix * K * 2));
  CK(hipMalloc(&parts, (size_t)ranges * O * K * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(gout, 0x3c, npix * O * 2));
  CK(hipMemset(col, 0x3c, npix * K * 2));
  // a 500 MB buffer swept between launches, so the columns are not left in the Infinity Cache
  // by the previous launch (in the step they were written by the forward long before)
  const size_t flushB = 512ull << 20;
  char* flush;
  CK(hipMalloc(&flush, flushB));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1, ef;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&ef));
  const long long cyc = (long long)(blk_us * 100.0);  // s_memtime: 100 MHz on gfx950
  double tot = 0.0;
  for (int i = 0; i < reps + 2; ++i) {
    if (fl == 1) CK(hipMemsetAsync(flush, i & 0xff, flushB, s0));
    if (fl == 2)
      hipLaunchKernelGGL(sweep_rd, dim3(4096), dim3(256), 0, s0,
                         reinterpret_cast<const uint4*>(flush), flushB / 16, sink);
    if (fl == 3)
      hipLaunchKernelGGL(sweep_nt, dim3(4096), dim3(256), 0, s0, reinterpret_cast<u4v*>(flush),
                         flushB / 16, (unsigned)i);
    CK(hipEventRecord(ef, s0));
    CK(hipStreamWaitEvent(s1, ef, 0));
    if (blk_us > 0) hipLaunchKernelGGL(blocker, dim3(64), dim3(1024), 0, s1, cyc, sink);
    CK(hipEventRecord(e0, s0));
    CK(dcn::launch_dw_stream_bf16(gout, col, parts, K, O, npix, s0));
    CK(hipEventRecord(e1, s0));
    CK(hipStreamSynchronize(s0));
    CK(hipStreamSynchronize(s1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (i >= 2) tot += ms;
  }
  printf("{\"kernel\": \"dw_stream_bf16\", \"ring\": %d, \"stage_px\": %d, \"blocker_us\": %.1f, "
         "\"flush\": %d, \"us\": %.2f, \"ranges\": %d}\n",
         DW_RING, DW_PX, blk_us, fl, 1e3 * tot / reps, ranges);
  return 0;
}
