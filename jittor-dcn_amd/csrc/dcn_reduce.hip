// dcn_reduce.hip — bias add (deform_conv.py:79-80) and the deterministic channel
// / partial reductions of the backward (∂b, ∂b_off, Σ_b ∂W partials).
#include "dcn_device.h"
#include "dcn_swizzle.h"

namespace dcn {

// out[ch] = Σ_{b,m} in[b][ch][m]: one 1024-thread block per channel; thread t sums the
// 4-element runs t, t+1024, ... of the channel's B·HW/4 runs taken image by image (all its
// loads independent, in flight together; r01 walked the images one after another, a
// 64-deep dependent chain: 33 us for ∂b or ∂b_off at config 4), then a fixed xor tree and
// a fixed wave order: deterministic. T: fp32, or bf16 (DCN_BF16's ∂out read directly).
template <bool VEC, typename T>
__global__ __launch_bounds__(1024) void channel_sum(const T* __restrict__ in, int B, int Cn,
                                                    int HW, float* __restrict__ out,
                                                    bf16_t* __restrict__ out_bf = nullptr) {
  __shared__ float red[1024 / 64];
  const int ch = blockIdx.x, tid = threadIdx.x;
  float s = 0.f;
  if (VEC) {
    const int R = HW / 4;  // runs per image
    const long tot = (long)B * R;
#pragma unroll 4
    for (long i = tid; i < tot; i += 1024) {
      const int b = (int)(i / R), m = (int)(i - (long)b * R);
      const float4 v = ld4(in + ((size_t)b * Cn + ch) * HW + 4 * m);
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    const long tot = (long)B * HW;
#pragma unroll 4
    for (long i = tid; i < tot; i += 1024) {
      const int b = (int)(i / HW), m = (int)(i - (long)b * HW);
      s += to_f32(in[((size_t)b * Cn + ch) * HW + m]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < 1024 / 64; ++w) t += red[w];
    out[ch] = t;
    if (out_bf) out_bf[ch] = f2bf(t);
  }
}

void launch_channel_sum(const float* in, int B, int Cn, int HW, float* out, hipStream_t s) {
  if (HW % 4 == 0)
    hipLaunchKernelGGL((channel_sum<true, float>), dim3(Cn), dim3(1024), 0, s, in, B, Cn, HW, out);
  else
    hipLaunchKernelGGL((channel_sum<false, float>), dim3(Cn), dim3(1024), 0, s, in, B, Cn, HW, out);
}
// Two-level form for few channels over many pixels (∂b_off: 18 channels, B·HW = 200k at
// config 3), so the sum does not hold 18 CUs for 0.11 ms beside the offset-conv backward:
// part[b][ch] = Σ_m in[b][ch][m] (one 256-thread block per (channel, image), fixed xor tree
// and wave order), then out[ch] = Σ_b part[b][ch] in image order. Deterministic.
__global__ __launch_bounds__(256) void plane_sum(const float* __restrict__ in, int HW,
                                                 float* __restrict__ part) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const float* p = in + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * HW;
  float s = 0.f;
  if ((HW & 3) == 0) {
    for (int i = tid; i < HW / 4; i += 256) {
      const float4 v = ld4(p + 4 * i);
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    for (int i = tid; i < HW; i += 256) s += p[i];
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) part[(size_t)blockIdx.y * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
// one wave per channel: lane l sums images l, l+64, ... in order, then a fixed xor tree (a
// serial 64-image chain per thread took 12 us of dependent loads)
__global__ __launch_bounds__(64) void fold_images(const float* __restrict__ part, int B, int Cn,
                                                  float* __restrict__ out) {
  const int ch = blockIdx.x, l = threadIdx.x;
  float s = 0.f;
  for (int b = l; b < B; b += 64) s += part[(size_t)b * Cn + ch];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (l == 0) out[ch] = s;
}
void launch_channel_sum_2l(const float* in, int B, int Cn, int HW, float* part, float* out,
                           hipStream_t s) {
  if (((uintptr_t)in & 15) != 0) return launch_channel_sum(in, B, Cn, HW, out, s);
  hipLaunchKernelGGL(plane_sum, dim3(Cn, B), dim3(256), 0, s, in, HW, part);
  hipLaunchKernelGGL(fold_images, dim3(Cn), dim3(64), 0, s, part, B, Cn, out);
}

void launch_channel_sum_bf16(const bf16_t* in, int B, int Cn, int HW, float* out, hipStream_t s,
                             bf16_t* out_bf) {
  if (HW % 4 == 0 && ((uintptr_t)in & 7) == 0)
    hipLaunchKernelGGL((channel_sum<true, bf16_t>), dim3(Cn), dim3(1024), 0, s, in, B, Cn, HW, out,
                       out_bf);
  else
    hipLaunchKernelGGL((channel_sum<false, bf16_t>), dim3(Cn), dim3(1024), 0, s, in, B, Cn, HW,
                       out, out_bf);
}

// ---------------------------------------------------------------------------
// Bias (deform_conv.py:79-80) and reductions.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bias_add_kernel(float* __restrict__ out,
                                                       const float* __restrict__ bias, int O,
                                                       int HW, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int o = (int)((i / HW) % O);
    out[i] += bias[o];
  }
}

__global__ __launch_bounds__(256) void bias_add_vec4(float4* __restrict__ out,
                                                     const float* __restrict__ bias, int O,
                                                     int HW4, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float bv = bias[(int)((i / HW4) % O)];
    float4 v = out[i];
    v.x += bv;
    v.y += bv;
    v.z += bv;
    v.w += bv;
    out[i] = v;
  }
}

hipError_t launch_bias_add(const Geo& g, float* out, const float* bias, int b0, int nb,
                           hipStream_t s) {
  float* o = out + (size_t)b0 * g.O * g.HW;
  const long n = (long)nb * g.O * g.HW;
  if (g.HW % 4 == 0) {
    const long n4 = n / 4;
    const unsigned grid = (unsigned)min((n4 + 255) / 256, 8192L);
    hipLaunchKernelGGL(bias_add_vec4, dim3(grid), dim3(256), 0, s, reinterpret_cast<float4*>(o),
                       bias, g.O, g.HW / 4, n4);
  } else {
    const unsigned grid = (unsigned)min((n + 255) / 256, 8192L);
    hipLaunchKernelGGL(bias_add_kernel, dim3(grid), dim3(256), 0, s, o, bias, g.O, g.HW, n);
  }
  return hipGetLastError();
}

// out[b][o][p] = src[o][b][p] (+ bias[o]): the flat forward GEMM's [O][B·HW] result into
// NCHW, with the bias pass folded in (one fp32 add, launch_bias_add's op). vec4 when HW % 4 == 0.
__global__ __launch_bounds__(256) void permute_obp_bias(const float* __restrict__ src,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ out, int B, int O,
                                                        int HW, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int p = (int)(i % HW);
    const long bo = i / HW;
    const int o = (int)(bo % O), b = (int)(bo / O);
    const float v = src[((long)o * B + b) * HW + p];
    out[i] = bias ? v + bias[o] : v;
  }
}
__global__ __launch_bounds__(256) void permute_obp_bias4(const float4* __restrict__ src,
                                                         const float* __restrict__ bias,
                                                         float4* __restrict__ out, int B, int O,
                                                         int HW4, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const int p = (int)(i % HW4);
    const long bo = i / HW4;
    const int o = (int)(bo % O), b = (int)(bo / O);
    float4 v = src[((long)o * B + b) * HW4 + p];
    if (bias) {
      const float bv = bias[o];
      v.x += bv;
      v.y += bv;
      v.z += bv;
      v.w += bv;
    }
    out[i] = v;
  }
}

hipError_t launch_permute_obp_bias(const float* src, const float* bias, float* out, int B, int O,
                                   int HW, hipStream_t s) {
  const long n = (long)B * O * HW;
  if (HW % 4 == 0) {
    const long n4 = n / 4;
    const unsigned grid = (unsigned)min((n4 + 255) / 256, 8192L);
    hipLaunchKernelGGL(permute_obp_bias4, dim3(grid), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(src), bias, reinterpret_cast<float4*>(out),
                       B, O, HW / 4, n4);
  } else {
    const unsigned grid = (unsigned)min((n + 255) / 256, 8192L);
    hipLaunchKernelGGL(permute_obp_bias, dim3(grid), dim3(256), 0, s, src, bias, out, B, O, HW, n);
  }
  return hipGetLastError();
}

hipError_t launch_bias_grad(const Geo& g, const float* gout, float* gb, hipStream_t s) {
  launch_channel_sum(gout, g.B, g.O, g.HW, gb, s);
  return hipGetLastError();
}

// dst[i] = Σ_p parts[p][i] in part order; dst_bf (DCN_BF16, optional) = its bf16 rounding,
// written by the same pass (no separate conversion launch)
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ parts,
                                                           int nparts, size_t n,
                                                           float* __restrict__ dst,
                                                           bf16_t* __restrict__ dst_bf) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float s = 0.f;
    for (int p = 0; p < nparts; ++p) s += parts[(size_t)p * n + i];
    dst[i] = s;
    if (dst_bf) dst_bf[i] = f2bf(s);
  }
}

// 4 elements per thread (n % 4 == 0, 16-B aligned): the same per-element sums in the same
// part order, 16-B loads, all parts' loads of a thread independent
__global__ __launch_bounds__(256) void sum_partials_vec4(const float4* __restrict__ parts,
                                                         int nparts, size_t n4,
                                                         float4* __restrict__ dst,
                                                         bf16_t* __restrict__ dst_bf) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int p = 0; p < nparts; ++p) {
      const float4 v = parts[(size_t)p * n4 + i];
      s.x += v.x, s.y += v.y, s.z += v.z, s.w += v.w;
    }
    dst[i] = s;
    if (dst_bf) st4<false>(dst_bf + 4 * i, s);
  }
}

hipError_t launch_sum_partials(const float* parts, int nparts, size_t n, float* dst,
                               hipStream_t s, bf16_t* dst_bf) {
  if (n % 4 == 0 && (((uintptr_t)parts | (uintptr_t)dst) & 15) == 0 &&
      ((uintptr_t)dst_bf & 7) == 0) {
    const size_t n4 = n / 4;
    const unsigned grid = (unsigned)min((n4 + 255) / 256, (size_t)4096);
    hipLaunchKernelGGL(sum_partials_vec4, dim3(grid), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(parts), nparts, n4,
                       reinterpret_cast<float4*>(dst), dst_bf);
    return hipGetLastError();
  }
  const unsigned grid = (unsigned)min((n + 255) / 256, (size_t)4096);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(grid), dim3(256), 0, s, parts, nparts, n, dst,
                     dst_bf);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// DCN_BF16 conversions (elementwise; grid-stride, 4 per thread).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bf16_to_f32_kernel(const bf16_t* __restrict__ in,
                                                          float* __restrict__ out, size_t n) {
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n;
       i += (size_t)gridDim.x * 256 * 4) {
    if (i + 4 <= n && (((uintptr_t)(in + i) & 7) | ((uintptr_t)(out + i) & 15)) == 0) {
      *reinterpret_cast<float4*>(out + i) = ld4(in + i);
    } else {
      for (size_t k = i; k < n && k < i + 4; ++k) out[k] = bf2f(in[k]);
    }
  }
}
__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ in,
                                                          bf16_t* __restrict__ out, size_t n) {
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n;
       i += (size_t)gridDim.x * 256 * 4) {
    if (i + 4 <= n && (((uintptr_t)(in + i) & 15) | ((uintptr_t)(out + i) & 7)) == 0) {
      st4<false>(out + i, *reinterpret_cast<const float4*>(in + i));
    } else {
      for (size_t k = i; k < n && k < i + 4; ++k) out[k] = f2bf(in[k]);
    }
  }
}
__global__ __launch_bounds__(256) void round_bf16_kernel(float* __restrict__ v,
                                                         bf16_t* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const bf16_t r = f2bf(v[i]);
    out[i] = r;
    v[i] = bf2f(r);
  }
}
__global__ __launch_bounds__(256) void bias_to_bf16_kernel(const float* __restrict__ in,
                                                           const float* __restrict__ bias,
                                                           bf16_t* __restrict__ out, int O, int HW,
                                                           size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float v = in[i];
    if (bias) v += bias[(i / HW) % O];
    out[i] = f2bf(v);
  }
}
// 4 per thread (HW % 4 == 0): 16-B loads, 8-B stores
__global__ __launch_bounds__(256) void bias_to_bf16_vec4(const float4* __restrict__ in,
                                                         const float* __restrict__ bias,
                                                         bf16_t* __restrict__ out, int O, int HW4,
                                                         size_t n4) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float4 v = in[i];
    if (bias) {
      const float bv = bias[(i / HW4) % O];
      v.x += bv, v.y += bv, v.z += bv, v.w += bv;
    }
    st4<false>(out + 4 * i, v);
  }
}

static unsigned grid_for(size_t n, size_t per_thread) {
  const size_t b = (n + 256 * per_thread - 1) / (256 * per_thread);
  return (unsigned)(b < 16384 ? (b ? b : 1) : 16384);
}

// Up to kMaxConv independent conversions in ONE launch (DCN_BF16's small parameter and
// gradient copies: each was its own 4-6 us launch). Thread quads are numbered across the
// segments; a quad converts like bf16_to_f32_kernel / f32_to_bf16_kernel (same rounding).
__global__ __launch_bounds__(256) void convert_multi_kernel(ConvBatch cb) {
  size_t q0[kMaxConv + 1];
  q0[0] = 0;
#pragma unroll
  for (int k = 0; k < kMaxConv; ++k) q0[k + 1] = q0[k] + (k < cb.n ? (cb.seg[k].n + 3) / 4 : 0);
  for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q < q0[kMaxConv];
       q += (size_t)gridDim.x * 256) {
    int k = 0;
#pragma unroll
    for (int t = 1; t < kMaxConv; ++t) k += q >= q0[t] ? 1 : 0;
    const ConvSeg sg = cb.seg[k];
    const size_t i = (q - q0[k]) * 4, n = sg.n;
    if (sg.to_bf16) {
      const float* in = static_cast<const float*>(sg.in);
      bf16_t* out = static_cast<bf16_t*>(sg.out);
      if (i + 4 <= n && (((uintptr_t)(in + i) & 15) | ((uintptr_t)(out + i) & 7)) == 0)
        st4<false>(out + i, *reinterpret_cast<const float4*>(in + i));
      else
        for (size_t e = i; e < n && e < i + 4; ++e) out[e] = f2bf(in[e]);
    } else {
      const bf16_t* in = static_cast<const bf16_t*>(sg.in);
      float* out = static_cast<float*>(sg.out);
      if (i + 4 <= n && (((uintptr_t)(in + i) & 7) | ((uintptr_t)(out + i) & 15)) == 0)
        *reinterpret_cast<float4*>(out + i) = ld4(in + i);
      else
        for (size_t e = i; e < n && e < i + 4; ++e) out[e] = bf2f(in[e]);
    }
  }
}
hipError_t launch_convert_multi(const ConvBatch& cb, hipStream_t s) {
  if (cb.overflow) return hipErrorInvalidValue;  // a dropped conversion would be a silent bug
  size_t quads = 0;
  for (int k = 0; k < cb.n; ++k) quads += (cb.seg[k].n + 3) / 4;
  if (quads == 0) return hipGetLastError();
  hipLaunchKernelGGL(convert_multi_kernel, dim3(grid_for(quads * 4, 4)), dim3(256), 0, s, cb);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void prep_bf16_kernel(PrepBatch pb) {
  long q0[kMaxPrep + 1];
  q0[0] = 0;
#pragma unroll
  for (int k = 0; k < kMaxPrep; ++k) q0[k + 1] = q0[k] + (k < pb.n ? pb.job[k].units : 0);
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < q0[kMaxPrep];
       q += (long)gridDim.x * 256) {
    int k = 0;
#pragma unroll
    for (int t = 1; t < kMaxPrep; ++t) k += q >= q0[t] ? 1 : 0;
    const PrepJob& jb = pb.job[k];
    const long u = q - q0[k];
    const bf16_t* in = static_cast<const bf16_t*>(jb.in);
    switch (jb.kind) {
      case PREP_F32: {
        float* out = static_cast<float*>(jb.out);
        const long i = u * 4;
        if (i + 4 <= jb.n && (((uintptr_t)(in + i) & 7) | ((uintptr_t)(out + i) & 15)) == 0)
          *reinterpret_cast<float4*>(out + i) = ld4(in + i);
        else
          for (long e = i; e < jb.n && e < i + 4; ++e) out[e] = bf2f(in[e]);
        break;
      }
      case PREP_TJC:
        swz_tjc(in, static_cast<bf16_t*>(jb.out), jb.a, jb.b, jb.c, jb.d, (int)u);
        break;
      case PREP_CK:
        swz_ck(in, static_cast<bf16_t*>(jb.out), jb.a, jb.b, jb.c, jb.d, jb.e, (int)u);
        break;
      case PREP_FRAG16:
        swz_frag16(in, static_cast<bf16_t*>(jb.out), jb.a, u);
        break;
      default:  // PREP_DCOL
        swz_dcol(in, jb.a, static_cast<bf16_t*>(jb.out), (int)u);
        break;
    }
  }
}

hipError_t launch_prep_bf16(const PrepBatch& pb, hipStream_t s) {
  if (pb.overflow) return hipErrorInvalidValue;
  long units = 0;
  for (int k = 0; k < pb.n; ++k) units += pb.job[k].units;
  if (!units) return hipSuccess;
  hipLaunchKernelGGL(prep_bf16_kernel, dim3((unsigned)std::min((units + 255) / 256, 4096l)),
                     dim3(256), 0, s, pb);
  return hipGetLastError();
}

hipError_t launch_bf16_to_f32(const bf16_t* in, float* out, size_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}
hipError_t launch_f32_to_bf16(const float* in, bf16_t* out, size_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}
hipError_t launch_round_to_bf16(float* v, bf16_t* out, size_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(round_bf16_kernel, dim3(grid_for(n, 1)), dim3(256), 0, s, v, out, n);
  return hipGetLastError();
}
hipError_t launch_bias_to_bf16(const Geo& g, const float* out32, const float* bias, bf16_t* out,
                               hipStream_t s) {
  const size_t n = (size_t)g.B * g.O * g.HW;
  if (g.HW % 4 == 0 && ((uintptr_t)out32 & 15) == 0 && ((uintptr_t)out & 7) == 0)
    hipLaunchKernelGGL(bias_to_bf16_vec4, dim3(grid_for(n, 4)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(out32), bias, out, g.O, g.HW / 4, n / 4);
  else
    hipLaunchKernelGGL(bias_to_bf16_kernel, dim3(grid_for(n, 1)), dim3(256), 0, s, out32, bias,
                       out, g.O, g.HW, n);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ∂out -> ∂outT (channels-last, B operand of the flat ∂col GEMM) fused with ∂b, through
// 64x65 LDS tiles. A block walks kXpSub consecutive 64-pixel tiles of one (image,
// 64-channel) slab with the next tile's loads in flight while the current one is
// written, and accumulates each channel's sum while writing; its 4 row-groups' sums fold
// in order into one partial per (block, channel), and tile_sum_to_channels folds the
// B x ceil(HW/(64*kXpSub)) partials per channel in order (deterministic, no atomics).
// ---------------------------------------------------------------------------
constexpr int kXpSub = 8;
static int xpose_blocks_x(int P) { return (P + 64 * kXpSub - 1) / (64 * kXpSub); }

__global__ __launch_bounds__(256) void xpose_chsum(const float* __restrict__ in,
                                                   float* __restrict__ out,
                                                   float* __restrict__ tsum, int C, int P) {
  __shared__ float t[64][65];
  __shared__ float red[4][64];
  const int c0 = blockIdx.y * 64, b = blockIdx.z;
  const float* ib = in + (size_t)b * C * P;
  float* ob = out + (size_t)b * C * P;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int pb = blockIdx.x * 64 * kXpSub;
  const int nsub = min(kXpSub, (P - pb + 63) / 64);
  float r[16];
  auto load = [&](int p0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = c0 + ty + 4 * k, p = p0 + tx;
      r[k] = (c < C && p < P) ? ib[(size_t)c * P + p] : 0.f;
    }
  };
  load(pb);
  float csum = 0.f;  // channel c0+tx over this thread's pixels (rows ty, ty+4, ... of a tile)
  for (int sub = 0; sub < nsub; ++sub) {
    const int p0 = pb + 64 * sub;
#pragma unroll
    for (int k = 0; k < 16; ++k) t[ty + 4 * k][tx] = r[k];
    __syncthreads();
    if (sub + 1 < nsub) load(p0 + 64);  // in flight while this tile is written
    const int c = c0 + tx;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = ty + 4 * k, p = p0 + i;
      const float v = t[tx][i];
      csum += v;  // zero outside [0, P) x [0, C)
      if (c < C && p < P) ob[(size_t)p * C + c] = v;
    }
    __syncthreads();
  }
  red[ty][tx] = csum;
  __syncthreads();
  if (ty == 0 && c0 + tx < C)
    tsum[(size_t)(c0 + tx) * gridDim.x * gridDim.z + (size_t)b * gridDim.x + blockIdx.x] =
        ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];  // [C][partials]
}

// 16-byte form (P % 4 == 0, C % 64 == 0, 16-B aligned): a thread loads 4 pixels of one
// channel row (float4; a wave reads 4 rows x 256 B), the tile goes through LDS, and a thread
// stores 4 channels of one pixel (float4; a wave writes 4 pixel rows x 256 B): 1 KiB per wave
// instruction each way instead of 256 B. With SUMS, the channel sums ride along: a thread's
// 4-pixel sums, then the 16 lanes of its channel row folded by DPP (fixed order).
template <bool SUMS>
__global__ __launch_bounds__(256) void xpose_f4(const float* __restrict__ in, float* __restrict__ out,
                                                float* __restrict__ tsum, int C, int P) {
  __shared__ float t[64][65];
  const int c0 = blockIdx.y * 64, b = blockIdx.z;
  const float* ib = in + (size_t)b * C * P;
  float* ob = out + (size_t)b * C * P;
  const int tid = threadIdx.x, lr = tid >> 4, lq = tid & 15;
  const int pb = blockIdx.x * 64 * kXpSub;
  const int nsub = min(kXpSub, (P - pb + 63) / 64);
  float4 r[4];
  auto load = [&](int p0) {
    const int p = p0 + 4 * lq;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      r[k] = p < P ? *reinterpret_cast<const float4*>(ib + (size_t)(c0 + lr + 16 * k) * P + p)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  load(pb);
  for (int sub = 0; sub < nsub; ++sub) {
    const int p0 = pb + 64 * sub;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float* row = &t[lr + 16 * k][4 * lq];
      row[0] = r[k].x, row[1] = r[k].y, row[2] = r[k].z, row[3] = r[k].w;
      if (SUMS) cs[k] += ((r[k].x + r[k].y) + r[k].z) + r[k].w;
    }
    __syncthreads();
    if (sub + 1 < nsub) load(p0 + 64);  // in flight while this tile is written
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pr = lr + 16 * k, p = p0 + pr;
      const float4 v = make_float4(t[4 * lq][pr], t[4 * lq + 1][pr], t[4 * lq + 2][pr],
                                   t[4 * lq + 3][pr]);
      if (p < P) *reinterpret_cast<float4*>(ob + (size_t)p * C + c0 + 4 * lq) = v;
    }
    __syncthreads();
  }
  if (SUMS) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = cs[k];  // the 16 lanes of channel row lr + 16k form one DPP row
      v += dpp_f<0xB1>(v);
      v += dpp_f<0x4E>(v);
      v += dpp_f<0x141>(v);
      v += dpp_f<0x140>(v);
      if (lq == 0)
        tsum[(size_t)(c0 + lr + 16 * k) * gridDim.x * gridDim.z + (size_t)b * gridDim.x + blockIdx.x] = v;
    }
  }
}

static bool xpose_f4_ok(const float* in, const float* out, int C, int P) {
  return P % 4 == 0 && C % 64 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0;
}

// bf16 form (DCN_BF16's ∂out -> ∂outT, x -> xT): 16-byte accesses both ways (P % 8 == 0,
// C % 64 == 0, 16-B aligned). A block walks kXbSub 64-pixel tiles of one (image, 64-channel)
// slab, the next tile's loads in flight while the current one is written. Thread (lr, lq)
// loads 8 pixels of channel rows lr and lr + 32 and, from the LDS tile (rows padded to 66
// elements: the column reads hit 32 distinct banks), stores 8 channels of pixel rows lr and
// lr + 32. With SUMS the channel sums ride along: a thread's 8-pixel sums in a fixed tree,
// folded over the 8 lanes of its channel row by a fixed xor tree, one partial per (block,
// channel) in tsum[c][image·gridDim.x + blockIdx.x] (r05: ∂b and the transpose were two passes
// over ∂out, 9.2 + 13.7 us at config 4).
#ifndef XB_ALL
#define XB_ALL 1
#endif
constexpr int kXbSub = 4;
static int xpose_b8_blocks_x(int P) { return (P + 64 * kXbSub - 1) / (64 * kXbSub); }

__device__ __forceinline__ float sum2_bf16(unsigned u) {
  return __uint_as_float(u << 16) + __uint_as_float(u & 0xffff0000u);
}
__device__ __forceinline__ float sum8_bf16(uint4 v) {
  return (sum2_bf16(v.x) + sum2_bf16(v.y)) + (sum2_bf16(v.z) + sum2_bf16(v.w));
}

template <bool SUMS>
__global__ __launch_bounds__(256) void xpose_b8(const bf16_t* __restrict__ in,
                                                bf16_t* __restrict__ out,
                                                float* __restrict__ tsum, int C, int P) {
  __shared__ unsigned short t[64][66];  // [c][p]
  const int c0 = blockIdx.y * 64, b = blockIdx.z;
  const bf16_t* ib = in + (size_t)b * C * P;
  bf16_t* ob = out + (size_t)b * C * P;
  const int tid = threadIdx.x, lr = tid >> 3, lq = tid & 7;
  const int pb = blockIdx.x * 64 * kXbSub;
  const int nsub = min(kXbSub, (P - pb + 63) / 64);
#if XB_ALL
  // r05: every sub-tile's loads in flight from the start (through a buffer resource: pixels
  // past P read zeros); one tile ahead waited a memory latency per tile
  const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(ib), 0,
                                                     (int)((size_t)C * P * 2), 0x00020000);
  uint4 ra[kXbSub][2];
#pragma unroll
  for (int sb = 0; sb < kXbSub; ++sb) {
    const int p = pb + 64 * sb + 8 * lq;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const unsigned o = p < P && sb < nsub ? (unsigned)(((c0 + lr + 32 * k) * P + p) * 2) : 0x80000000u;
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(rin, o, 0, 0);
      ra[sb][k] = make_uint4(q[0], q[1], q[2], q[3]);
    }
  }
  float cs[2] = {0.f, 0.f};
#pragma unroll
  for (int sub = 0; sub < kXbSub; ++sub) {
    if (sub >= nsub) break;  // block-uniform
    const int p0 = pb + 64 * sub;
    const uint4(&r)[2] = ra[sub];
#else
  uint4 r[2];
  auto load = [&](int p0) {
    const int p = p0 + 8 * lq;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      r[k] = p < P ? *reinterpret_cast<const uint4*>(ib + (size_t)(c0 + lr + 32 * k) * P + p)
                   : make_uint4(0u, 0u, 0u, 0u);
  };
  float cs[2] = {0.f, 0.f};
  load(pb);
  for (int sub = 0; sub < nsub; ++sub) {
    const int p0 = pb + 64 * sub;
#endif
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      unsigned* row = reinterpret_cast<unsigned*>(&t[lr + 32 * k][8 * lq]);
      row[0] = r[k].x, row[1] = r[k].y, row[2] = r[k].z, row[3] = r[k].w;
      if (SUMS) cs[k] += sum8_bf16(r[k]);  // zeros past P
    }
    __syncthreads();
#if !XB_ALL
    if (sub + 1 < nsub) load(p0 + 64);  // in flight while this tile is written
#endif
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = lr + 32 * k, p = p0 + pr;
      unsigned u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        u[i] = (unsigned)t[8 * lq + 2 * i][pr] | ((unsigned)t[8 * lq + 2 * i + 1][pr] << 16);
      if (p < P)
        *reinterpret_cast<uint4*>(ob + (size_t)p * C + c0 + 8 * lq) =
            make_uint4(u[0], u[1], u[2], u[3]);
    }
    __syncthreads();
  }
  if (SUMS) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float v = cs[k];  // the 8 lanes of channel row lr + 32k are consecutive
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if (lq == 0)
        tsum[(size_t)(c0 + lr + 32 * k) * gridDim.x * gridDim.z + (size_t)b * gridDim.x +
             blockIdx.x] = v;
    }
  }
}

static bool xpose_b8_ok(const bf16_t* in, const bf16_t* out, int C, int P) {
  // (one image's C·P bf16 values are addressed through a buffer resource: 32-bit offsets)
  return P % 8 == 0 && C % 64 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
         (size_t)C * P * 2 < ((size_t)1 << 31);
}

// One wave per channel: lane l sums partials i ≡ l (mod 64) (all loads in flight
// together), then a fixed DPP tree (wave_sum) folds the 64 lane sums: deterministic.
__global__ __launch_bounds__(64) void tile_sum_to_channels(const float* __restrict__ tsum,
                                                           int ntiles, int C,
                                                           float* __restrict__ out,
                                                           bf16_t* __restrict__ out_bf = nullptr) {
  const int c = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
#pragma unroll 8
  for (int i = lane; i < ntiles; i += 64) s += tsum[(size_t)c * ntiles + i];  // coalesced
  s = wave_sum(s);
  if (lane == 0) {
    out[c] = s;
    if (out_bf) out_bf[c] = f2bf(s);
  }
}

bool launch_xpose_b8(const bf16_t* in, bf16_t* out, int B, int C, int P, hipStream_t s) {
  if (!xpose_b8_ok(in, out, C, P)) return false;
  dim3 grid(xpose_b8_blocks_x(P), C / 64, B);
  hipLaunchKernelGGL(xpose_b8<false>, grid, dim3(256), 0, s, in, out, nullptr, C, P);
  return true;
}

size_t xpose_chsum_bf16_floats(int B, int C, int P) {
  return (size_t)B * xpose_b8_blocks_x(P) * C;
}

bool launch_xpose_chsum_bf16(const bf16_t* in, bf16_t* out, float* tsum, float* chsum,
                             bf16_t* chsum_bf, int B, int C, int P, hipStream_t s,
                             hipStream_t s_sum, hipEvent_t ev) {
  if (!xpose_b8_ok(in, out, C, P)) return false;
  dim3 grid(xpose_b8_blocks_x(P), C / 64, B);
  hipLaunchKernelGGL(xpose_b8<true>, grid, dim3(256), 0, s, in, out, tsum, C, P);
  // the fold only feeds ∂b: off the main stream's critical path when given a side stream
  // (a failed record / wait leaves it on s)
  if (s_sum && s_sum != s && hipEventRecord(ev, s) == hipSuccess &&
      hipStreamWaitEvent(s_sum, ev, 0) == hipSuccess)
    s = s_sum;
  hipLaunchKernelGGL(tile_sum_to_channels, dim3(C), dim3(64), 0, s, tsum, B * (int)grid.x, C,
                     chsum, chsum_bf);
  return true;
}

// the plain fp32 NCHW -> NHWC transpose in the 16-byte form; false when it does not apply
bool launch_xpose_f4(const float* in, float* out, int B, int C, int P, hipStream_t s) {
  if (!xpose_f4_ok(in, out, C, P)) return false;
  dim3 grid(xpose_blocks_x(P), C / 64, B);
  hipLaunchKernelGGL(xpose_f4<false>, grid, dim3(256), 0, s, in, out, nullptr, C, P);
  return true;
}

size_t xpose_chsum_floats(int B, int C, int P) { return (size_t)B * xpose_blocks_x(P) * C; }

hipError_t launch_xpose_chsum(const float* in, float* out, float* tsum, float* chsum, int B,
                              int C, int P, hipStream_t s, hipStream_t s_sum,
                              hipEvent_t ev) {
  dim3 grid(xpose_blocks_x(P), (C + 63) / 64, B);
  if (xpose_f4_ok(in, out, C, P))
    hipLaunchKernelGGL(xpose_f4<true>, grid, dim3(256), 0, s, in, out, tsum, C, P);
  else
    hipLaunchKernelGGL(xpose_chsum, grid, dim3(256), 0, s, in, out, tsum, C, P);
  if (s_sum && s_sum != s) {  // the fold only feeds ∂b: off the main stream's critical path
    hipError_t e = hipEventRecord(ev, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s_sum, ev, 0);
    if (e != hipSuccess) return e;
    s = s_sum;
  }
  hipLaunchKernelGGL(tile_sum_to_channels, dim3(C), dim3(64), 0, s, tsum, B * xpose_blocks_x(P), C,
                     chsum, nullptr);
  return hipGetLastError();
}

}  // namespace dcn
