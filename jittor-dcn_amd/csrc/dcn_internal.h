// dcn_internal.h — shared geometry + launch prototypes for libdcn (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/dcn.h"

namespace dcn {

// Derived geometry of one call. All fields are plain ints so the struct is
// passed to kernels by value (kernarg segment, scalar registers).
struct Geo {
  int B, C, H, W, O;
  int kh, kw, sh, sw, ph, pw, dh, dw, G;
  int Ho, Wo;  // output size (deform_conv.py:34-35, dilation-aware)
  int N;       // taps = kh*kw (deform_conv.py:14)
  int K;       // N*C, GEMM depth, k = n*C + c (deform_conv.py:72-73)
  int HW;      // Ho*Wo
  int HWi;     // H*W
  int Cg;      // channels per deform group
  int J;       // offset channels = 2*N*G
};

// Launchers (dcn_kernels.hip). All stream-ordered, return hipError_t.
hipError_t launch_im2col(const Geo& g, const float* x, const float* off,
                         float* col, int b0, int nb, hipStream_t s);
hipError_t launch_col2im_coord(const Geo& g, const float* x, const float* off,
                               const float* gcol, float* gx, float* goff,
                               int b0, int nb, hipStream_t s);
hipError_t launch_offset_conv_fwd(const Geo& g, const float* x,
                                  const float* w_off, const float* b_off,
                                  float* off, float* wt_scratch, hipStream_t s);
hipError_t launch_offset_conv_bwd(const Geo& g, const float* x,
                                  const float* w_off, const float* goff,
                                  float* gx, float* gw_off, float* gb_off,
                                  hipStream_t s);
hipError_t launch_bias_add(const Geo& g, float* out, const float* bias, int b0,
                           int nb, hipStream_t s);
hipError_t launch_bias_grad(const Geo& g, const float* gout, float* gb,
                            hipStream_t s);
hipError_t launch_sum_partials(const float* parts, int nparts, size_t n,
                               float* dst, hipStream_t s);

// Selection of the im2col / col2im implementation (tests force the generic
// global-memory kernels to cross-check the LDS-window kernels).
void set_force_generic(int on);
int get_force_generic();

}  // namespace dcn
