// dcn_roi_pool.hip — DeformRoIPool (deform_conv.py:85-159) and DeformPSRoIPool
// (:162-241) forward and backward for gfx950.
//
// Work is tiny next to the DCN hot path (R RoIs x C channels x P bins, one bilinear
// sample per bin), so the kernels are latency kernels: one block per RoI, lanes over
// output channels (coalesced ∂out / out rows), the block's P bins' coordinates and
// corner weights computed once into LDS. All coordinate arithmetic is fp32 in the
// reference's op order (-ffp-contract=off), so floor() sees the reference's values.
#include "dcn_device.h"

namespace dcn {

namespace {

constexpr int kRoiThreads = 256;
constexpr int kRoiMaxBins = 256;  // P = ph*pw staged per block

struct Bin {
  int y0, y1, x0, x1;     // clamped corners (:121-129 / :214-222)
  float dx, dy;           // from the clamped top-left corner (:131-132 / :224-225)
  float w00, w01, w10, w11;  // (:134-137 / :227-230)
};

// bin p of RoI r; returns the batch index (rois[:, 0].long(): truncation toward zero)
__device__ int roi_bin(const RoiGeo& q, const float* __restrict__ rois,
                       const float* __restrict__ offsets, int r, int p, Bin* o, float* sx,
                       float* sy) {
  const float* rr = rois + (size_t)r * 5;
  const int b = (int)rr[0];
  const float x1 = rr[1] * q.scale, y1 = rr[2] * q.scale;  // :96 / :181
  const float x2 = rr[3] * q.scale, y2 = rr[4] * q.scale;
  const float rw = fmaxf(x2 - x1, 1e-6f), rh = fmaxf(y2 - y1, 1e-6f);  // :98-99
  const int i = p / q.pw, j = p - i * q.pw;  // meshgrid(ph, pw) flattened row-major
  const float bw = rw / (float)(q.ps ? q.part_w : q.pw);  // :107-108 / :191-192
  const float bh = rh / (float)(q.ps ? q.part_h : q.ph);
  const float bcx = x1 + ((float)j + 0.5f) * bw;  // :110-111 / :194-195
  const float bcy = y1 + ((float)i + 0.5f) * bh;
  float cx = bcx, cy = bcy;
  *sx = 0.f;
  *sy = 0.f;
  const float* of = offsets + ((size_t)r * q.P + p) * 2;
  if (!q.ps) {  // :113-117
    cx = bcx + of[0] * rw;
    cy = bcy + of[1] * rh;
    *sx = rw;
    *sy = rh;
  } else if (!q.no_trans) {  // :197-201
    cx = bcx + of[0] * rw * q.trans_std;
    cy = bcy + of[1] * rh * q.trans_std;
    *sx = rw * q.trans_std;
    *sy = rh * q.trans_std;
  }
  const int fx = (int)floorf(cx), fy = (int)floorf(cy);
  o->x0 = min(max(fx, 0), q.W - 1);
  o->x1 = min(max(fx + 1, 0), q.W - 1);
  o->y0 = min(max(fy, 0), q.H - 1);
  o->y1 = min(max(fy + 1, 0), q.H - 1);
  o->dx = cx - (float)o->x0;
  o->dy = cy - (float)o->y0;
  o->w00 = (1.0f - o->dx) * (1.0f - o->dy);
  o->w01 = (1.0f - o->dx) * o->dy;
  o->w10 = o->dx * (1.0f - o->dy);
  o->w11 = o->dx * o->dy;
  return b;
}

__global__ __launch_bounds__(kRoiThreads) void roi_pool_fwd(RoiGeo q, const float* __restrict__ f,
                                                            const float* __restrict__ rois,
                                                            const float* __restrict__ offsets,
                                                            float* __restrict__ out) {
  __shared__ Bin bins[kRoiMaxBins];
  __shared__ int sb;
  const int r = blockIdx.x;
  for (int p = threadIdx.x; p < q.P; p += blockDim.x) {
    float sx, sy;
    const int b = roi_bin(q, rois, offsets, r, p, &bins[p], &sx, &sy);
    if (p == 0) sb = b;
  }
  __syncthreads();
  const int b = sb;
  const bool bok = b >= 0 && b < q.B;  // the host API rejects these; zeros here
  const size_t HW = (size_t)q.H * q.W;
  for (int co = threadIdx.x; co < q.Cout; co += blockDim.x) {
    // val_k = Σ_p feature(corner k, bin p) · w_k (:141-155 / :232-237), summed in the
    // reference's order: ((val00 + val01) + val10) + val11
    float v00 = 0.f, v01 = 0.f, v10 = 0.f, v11 = 0.f;
    if (bok)
      for (int p = 0; p < q.P; ++p) {
        const Bin& o = bins[p];
        const int ch = q.ps ? co * q.P + p : co;  // :232-233
        const float* fc = f + ((size_t)b * q.C + ch) * HW;
        v00 += fc[o.y0 * q.W + o.x0] * o.w00;
        v01 += fc[o.y1 * q.W + o.x0] * o.w01;
        v10 += fc[o.y0 * q.W + o.x1] * o.w10;
        v11 += fc[o.y1 * q.W + o.x1] * o.w11;
      }
    out[(size_t)r * q.Cout + co] = ((v00 + v01) + v10) + v11;
  }
}

// ∂features: scatter of ∂out · w_k to the four clamped corners (atomics: RoIs and bins
// may share pixels). ∂offsets[r][p] = (Σ_co ∂out · ∂val/∂(cx, cy)) · (rw, rh) [· trans_std]
// with ∂val/∂cx = (1-dy)(f10 - f00) + dy (f11 - f01), ∂val/∂cy = (1-dx)(f01 - f00)
// + dx (f11 - f10) (floor and the clamps carry no gradient). The channel sums fold in a
// fixed LDS tree, so ∂offsets are bitwise reproducible.
__global__ __launch_bounds__(kRoiThreads) void roi_pool_bwd(RoiGeo q, const float* __restrict__ f,
                                                            const float* __restrict__ rois,
                                                            const float* __restrict__ offsets,
                                                            const float* __restrict__ gout,
                                                            float* __restrict__ gf,
                                                            float* __restrict__ goffs) {
  __shared__ Bin bins[kRoiMaxBins];
  __shared__ float2 scale[kRoiMaxBins];
  __shared__ int sb;
  __shared__ float red[2][kRoiThreads];
  const int r = blockIdx.x, tid = threadIdx.x;
  for (int p = tid; p < q.P; p += blockDim.x) {
    float sx, sy;
    const int b = roi_bin(q, rois, offsets, r, p, &bins[p], &sx, &sy);
    scale[p] = make_float2(sx, sy);
    if (p == 0) sb = b;
  }
  __syncthreads();
  const int b = sb;
  const bool bok = b >= 0 && b < q.B;
  const size_t HW = (size_t)q.H * q.W;
  for (int p = 0; p < q.P; ++p) {
    const Bin o = bins[p];
    float dcx = 0.f, dcy = 0.f;
    if (bok)
      for (int co = tid; co < q.Cout; co += blockDim.x) {
        const float g = gout[(size_t)r * q.Cout + co];
        const int ch = q.ps ? co * q.P + p : co;
        const float* fc = f + ((size_t)b * q.C + ch) * HW;
        float* gc = gf + ((size_t)b * q.C + ch) * HW;
        const float f00 = fc[o.y0 * q.W + o.x0], f01 = fc[o.y1 * q.W + o.x0];
        const float f10 = fc[o.y0 * q.W + o.x1], f11 = fc[o.y1 * q.W + o.x1];
        atomicAdd(gc + o.y0 * q.W + o.x0, g * o.w00);
        atomicAdd(gc + o.y1 * q.W + o.x0, g * o.w01);
        atomicAdd(gc + o.y0 * q.W + o.x1, g * o.w10);
        atomicAdd(gc + o.y1 * q.W + o.x1, g * o.w11);
        dcx += g * ((1.0f - o.dy) * (f10 - f00) + o.dy * (f11 - f01));
        dcy += g * ((1.0f - o.dx) * (f01 - f00) + o.dx * (f11 - f10));
      }
    if (!goffs) continue;  // uniform
    red[0][tid] = dcx;
    red[1][tid] = dcy;
    __syncthreads();
    for (int s = kRoiThreads / 2; s > 0; s >>= 1) {
      if (tid < s) {
        red[0][tid] += red[0][tid + s];
        red[1][tid] += red[1][tid + s];
      }
      __syncthreads();
    }
    if (tid == 0) {
      float* go = goffs + ((size_t)r * q.P + p) * 2;
      go[0] = red[0][0] * scale[p].x;
      go[1] = red[1][0] * scale[p].y;
    }
    __syncthreads();
  }
}

}  // namespace

bool roi_geo_ok(const RoiGeo& q) {
  return q.B > 0 && q.C > 0 && q.H > 0 && q.W > 0 && q.R >= 0 && q.P > 0 && q.P <= kRoiMaxBins &&
         q.Cout > 0;
}

hipError_t launch_roi_pool_fwd(const RoiGeo& q, const float* f, const float* rois,
                               const float* offsets, float* out, hipStream_t s) {
  if (q.R == 0) return hipSuccess;
  hipLaunchKernelGGL(roi_pool_fwd, dim3(q.R), dim3(kRoiThreads), 0, s, q, f, rois, offsets, out);
  return hipGetLastError();
}

hipError_t launch_roi_pool_bwd(const RoiGeo& q, const float* f, const float* rois,
                               const float* offsets, const float* gout, float* gf, float* goffs,
                               hipStream_t s) {
  hipError_t e = hipMemsetAsync(gf, 0, (size_t)q.B * q.C * q.H * q.W * sizeof(float), s);
  if (e != hipSuccess || q.R == 0) return e;
  hipLaunchKernelGGL(roi_pool_bwd, dim3(q.R), dim3(kRoiThreads), 0, s, q, f, rois, offsets, gout,
                     gf, goffs);
  return hipGetLastError();
}

}  // namespace dcn
