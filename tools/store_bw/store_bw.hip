// HBM write-bandwidth probe (K1's roofline: DESIGN.md §4): 1.85 GB of float4 stores,
// plain and non-temporal, and a float4 copy, with HIP events. Test infrastructure only.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool NT>
__global__ __launch_bounds__(256) void fill4(float4* __restrict__ p, size_t n4, float v) {
  const float4 x = make_float4(v, v, v, v);
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    if constexpr (NT) {
      float* q = reinterpret_cast<float*>(p + i);
      __builtin_nontemporal_store(x.x, q);
      __builtin_nontemporal_store(x.y, q + 1);
      __builtin_nontemporal_store(x.z, q + 2);
      __builtin_nontemporal_store(x.w, q + 3);
    } else {
      p[i] = x;
    }
  }
}

__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ a, float4* __restrict__ b,
                                             size_t n4) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    b[i] = a[i];
}

int main() {
  const size_t bytes = 1849688064;  // config-3 columns
  const size_t n4 = bytes / 16;
  float4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 16384}) {
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e9f;
      for (int r = 0; r < 6; ++r) {
        hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(fill4<false>, dim3(grid), dim3(256), 0, 0, a, n4, 1.f);
        if (kind == 1) hipLaunchKernelGGL(fill4<true>, dim3(grid), dim3(256), 0, 0, a, n4, 1.f);
        if (kind == 2) hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, 0, a, b, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r > 0 && ms < best) best = ms;
      }
      const double moved = (kind == 2 ? 2.0 : 1.0) * bytes;
      printf("grid %5d %-8s %.4f ms  %.2f TB/s\n", grid,
             kind == 0 ? "store" : (kind == 1 ? "nt-store" : "copy"), best, moved / best / 1e9);
    }
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
