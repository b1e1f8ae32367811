// dcn_fused.hip — fused deformable forward: the bilinear im2col of
// deform_conv.py:41-54,72-73 gathered straight into the LDS operand tiles of an f32 MFMA
// GEMM against the flat weight (:74-76), with the bias of :77-80 in the epilogue.
//
//   out[b][o][m] = bias[o] + Σ_k Wf[o][k] · col[b][m][k],   k = n·C + c   (Q5)
//
// The separate path is K1 (im2col_lds, HBM-bound: it writes the 1.85 GB column matrix)
// followed by a vendor GEMM that reads it back (MFMA-bound at the f32 rate). Here each
// workgroup owns a tile of OT output channels × 64 pixels of one image and walks k in
// steps of 32 (one tap n, 32 channels): every step it gathers the 64 × 32 column slice
// from the channels-last xT (four corner rows of 128 B per pixel, canonical bilerp ->
// the column values are bit-identical to K1's) and the OT × 32 weight slice into a
// double-buffered LDS image, while the 8 waves run 32x32x2 f32 MFMAs on the other buffer.
// The columns are still written (non-temporal, off the critical path: the kernel is
// MFMA-bound and HBM is otherwise idle) because the ∂W GEMM of the backward reads them.
//
// MFMA operand order: in step j of a 32-wide k slice, lane (i, h = lane/32) feeds
// k = 16h + j, so each lane's 16 A values and 16 B values are contiguous in LDS
// (4 ds_read_b128 each, conflict-free with a 36-float row stride). The sum over the 32 k
// is the same set of products in a fixed order: deterministic run to run.
#include "dcn_device.h"

namespace dcn {
namespace {

constexpr int kFP = 64;        // pixels per tile (two 32-px MFMA blocks)
constexpr int kFK = 32;        // k per step
constexpr int kFS = 36;        // LDS row stride in floats (144 B: conflict-free b128 reads)
constexpr int kFThreads = 512;  // 8 waves
constexpr int kFTaps = 9;       // tap records staged per tile (N <= 9)

__device__ __forceinline__ float4 ld4_if(const float* p, bool ok) {
  return ok ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float4 bilerp4f(float fr, float fc, float4 a, float4 b, float4 c,
                                           float4 d) {
  return make_float4(bilerp(fr, fc, a.x, b.x, c.x, d.x), bilerp(fr, fc, a.y, b.y, c.y, d.y),
                     bilerp(fr, fc, a.z, b.z, c.z, d.z), bilerp(fr, fc, a.w, b.w, c.w, d.w));
}

// One staging unit of a k step, held in registers between its loads and its LDS write.
// (weight registers named one by one: an indexed array here was promoted to LDS)
template <int WV>
struct Stage {
  f32x4 w0, w1, w2, w3;  // weight slice (WV of them used; native vectors, so no alloca)
  float4 a, b, c, d;      // the four corners of this thread's (pixel, 4-channel) sample
  float fr, fc;
  bool live;              // sample inside the image (else the column value is 0)
};

// OT output channels per workgroup: 256 (8 waves x one 32-row O block x two 32-px blocks)
// or 128 (8 waves x one O block x one px block).
template <int OT>
__global__ __launch_bounds__(kFThreads) void fwd_fused(Geo g, const float* __restrict__ xT,
                                                       const float* __restrict__ off,
                                                       const float* __restrict__ Wf,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ out,
                                                       float* __restrict__ colT, int tiles_m,
                                                       int tiles_o) {
  constexpr int OB = OT / 32;          // O blocks per tile
  constexpr int PB = OT / 128;         // px blocks per wave
  constexpr int WV = OT * 8 / kFThreads;  // weight float4 per thread per step (2 or 4)
  static_assert(WV == 2 || WV == 4, "tile");
  __shared__ float Ws[2][OT * kFS];
  __shared__ float Cs[2][kFP * kFS];
  __shared__ int4 rec[kFP * kFTaps];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Block3 blk = xcd_block();
  const int tm = blk.x % tiles_m, to = blk.x / tiles_m;
  const int b = blk.y;
  const int m0 = tm * kFP, o0 = to * OT;
  (void)tiles_o;

  // tap records of the tile's 64 pixels x N taps (deform_conv.py:58-68 via sample_tap)
  for (int s = tid; s < kFP * g.N; s += kFThreads) {
    const int p = s / g.N, n = s - p * g.N;
    const int m = m0 + p;
    int4 r = make_int4(0, 0, 0, 0);  // .z/.w = fr/fc; live flag packed in r.x sign below
    if (m < g.HW) {
      const Tap t = sample_tap(g, off, b, 0, n, m);
      r = t.ok ? make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc))
               : make_int4(INT_MIN, 0, 0, 0);
    } else {
      r = make_int4(INT_MIN, 0, 0, 0);
    }
    rec[p * kFTaps + n] = r;
  }

  // staging roles: pixel sp, channels 4*sq..4*sq+3 of the 32-channel slice
  const int sp = tid >> 3, sq = tid & 7;
  const int sm = m0 + sp;
  const float* xb = xT + (size_t)b * g.HWi * g.C;
  float* colrow = colT ? colT + ((size_t)b * g.HW + sm) * g.K + sq * 4 : nullptr;
  const bool pix_ok = sm < g.HW;
  const int csteps = g.C / kFK;
  const int nsteps = g.N * csteps;
  const long rs = (long)g.W * g.C;

  Stage<WV> st;
#define DCN_FUSED_LOAD(S)                                                                    \
  do {                                                                                       \
    const int n_ = (S) / csteps, cs_ = ((S) - n_ * csteps) * kFK;                            \
    const int k0_ = n_ * g.C + cs_;                                                          \
    const float* wp_ = Wf + (size_t)(o0 + (tid >> 3)) * g.K + k0_ + (tid & 7) * 4;          \
    const size_t wstep_ = (size_t)(kFThreads / 8) * g.K;                                     \
    st.w0 = *reinterpret_cast<const f32x4*>(wp_);                                           \
    st.w1 = *reinterpret_cast<const f32x4*>(wp_ + wstep_);                                  \
    if (WV > 2) {                                                                            \
      st.w2 = *reinterpret_cast<const f32x4*>(wp_ + 2 * wstep_);                            \
      st.w3 = *reinterpret_cast<const f32x4*>(wp_ + 3 * wstep_);                            \
    }                                                                                        \
    const int4 r_ = rec[sp * kFTaps + n_];                                                   \
    st.live = r_.x != INT_MIN;                                                               \
    const int r0_ = st.live ? r_.x : 0, c0_ = r_.y;                                          \
    st.fr = __int_as_float(r_.z);                                                            \
    st.fc = __int_as_float(r_.w);                                                            \
    const bool r0ok = st.live && r0_ >= 0, r1ok = st.live && r0_ + 1 < g.H;                  \
    const bool c0ok = c0_ >= 0, c1ok = c0_ + 1 < g.W;                                        \
    const float* p00 = xb + ((long)r0_ * g.W + c0_) * (long)g.C + cs_ + sq * 4;              \
    st.a = ld4_if(p00, r0ok && c0ok);                                                        \
    st.b = ld4_if(p00 + g.C, r0ok && c1ok);                                                  \
    st.c = ld4_if(p00 + rs, r1ok && c0ok);                                                   \
    st.d = ld4_if(p00 + rs + g.C, r1ok && c1ok);                                             \
  } while (0)
#define DCN_FUSED_STORE(S, BUF)                                                              \
  do {                                                                                       \
    const int n_ = (S) / csteps, cs_ = ((S) - n_ * csteps) * kFK;                            \
    float* wl_ = &Ws[BUF][(tid >> 3) * kFS + (tid & 7) * 4];                                 \
    constexpr int wls_ = (kFThreads / 8) * kFS;                                              \
    *reinterpret_cast<f32x4*>(wl_) = st.w0;                                                 \
    *reinterpret_cast<f32x4*>(wl_ + wls_) = st.w1;                                          \
    if (WV > 2) {                                                                            \
      *reinterpret_cast<f32x4*>(wl_ + 2 * wls_) = st.w2;                                    \
      *reinterpret_cast<f32x4*>(wl_ + 3 * wls_) = st.w3;                                    \
    }                                                                                        \
    const float4 v_ = st.live ? bilerp4f(st.fr, st.fc, st.a, st.b, st.c, st.d)               \
                              : make_float4(0.f, 0.f, 0.f, 0.f);                             \
    *reinterpret_cast<float4*>(&Cs[BUF][sp * kFS + sq * 4]) = v_;                            \
    if (colrow && pix_ok) st4<true>(colrow + n_ * g.C + cs_, v_);                            \
  } while (0)

  // MFMA roles: O block ob, px blocks pb0 .. pb0+PB-1
  const int ob = wave % OB, pb0 = (wave / OB) * PB;
  const int li = lane & 31, lh = lane >> 5;
  f32x16 acc[PB];
#pragma unroll
  for (int p = 0; p < PB; ++p)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[p][r] = 0.f;

  __syncthreads();  // records
  DCN_FUSED_LOAD(0);
  DCN_FUSED_STORE(0, 0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) DCN_FUSED_LOAD(s + 1);
    float4 av[4], bv[PB][4];
    const float* Ab = &Ws[buf][(ob * 32 + li) * kFS + lh * 16];
#pragma unroll
    for (int q = 0; q < 4; ++q) av[q] = *reinterpret_cast<const float4*>(Ab + 4 * q);
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const float* Bb = &Cs[buf][((pb0 + p) * 32 + li) * kFS + lh * 16];
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[p][q] = *reinterpret_cast<const float4*>(Bb + 4 * q);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        acc[p] = mfma32(av[q].x, bv[p][q].x, acc[p]);
        acc[p] = mfma32(av[q].y, bv[p][q].y, acc[p]);
        acc[p] = mfma32(av[q].z, bv[p][q].z, acc[p]);
        acc[p] = mfma32(av[q].w, bv[p][q].w, acc[p]);
      }
    }
    if (s + 1 < nsteps) DCN_FUSED_STORE(s + 1, buf ^ 1);
    __syncthreads();
  }

#undef DCN_FUSED_LOAD
#undef DCN_FUSED_STORE
  // epilogue: D[i][j] of a 32x32 block sits in lane j + 32·((i/4)%2), register
  // 4·(i/8) + i%4; rows are output channels, columns pixels (128-B row segments)
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int m = m0 + (pb0 + p) * 32 + li;
    if (m >= g.HW) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + ob * 32 + 8 * (r >> 2) + 4 * lh + (r & 3);
      float v = acc[p][r];
      if (bias) v += bias[o];
      out[((size_t)b * g.O + o) * g.HW + m] = v;
    }
  }
}

}  // namespace

bool fused_fwd_ok(const Geo& g) {
  return g.dt == DCN_F32 && g.G == 1 && g.N <= kFTaps && g.C % kFK == 0 &&
         g.O % 128 == 0;
}

// r01 at config 3: fused 2.51 ms against K1 0.40 + GEMM 1.66 + bias 0.06 ms unfused.
bool fused_fwd_pays(const Geo& g) {
  (void)g;
  return false;
}

hipError_t launch_fused_fwd(const Geo& g, const float* xT, const float* off, const float* Wf,
                            const float* bias, float* out, float* colT, hipStream_t s) {
  const int tiles_m = (g.HW + kFP - 1) / kFP;
  if (g.O % 256 == 0) {
    const int tiles_o = g.O / 256;
    hipLaunchKernelGGL(fwd_fused<256>, dim3(tiles_m * tiles_o, g.B), dim3(kFThreads), 0, s, g,
                       xT, off, Wf, bias, out, colT, tiles_m, tiles_o);
  } else {
    const int tiles_o = g.O / 128;
    hipLaunchKernelGGL(fwd_fused<128>, dim3(tiles_m * tiles_o, g.B), dim3(kFThreads), 0, s, g,
                       xT, off, Wf, bias, out, colT, tiles_m, tiles_o);
  }
  return hipGetLastError();
}

}  // namespace dcn
