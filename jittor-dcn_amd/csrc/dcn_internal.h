// dcn_internal.h — shared geometry + launch prototypes for libdcn (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/dcn.h"

namespace dcn {

typedef unsigned short bf16_t;  // bf16 storage (DCN_BF16)

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
  int dt;      // DCN_F32 / DCN_BF16 (tensor storage type of the call)
};

// Launchers. All stream-ordered, return hipError_t.
// dcn_sampling.hip (channels-last columns colT[b][m][n*C + c]):
hipError_t launch_nchw_to_nhwc(const float* in, float* out, int B, int C, int P, hipStream_t s);
hipError_t launch_nhwc_to_nchw(const float* in, float* out, int B, int C, int P, hipStream_t s);
hipError_t launch_nchw_to_nhwc_bf16(const bf16_t* in, bf16_t* out, int B, int C, int P,
                                    hipStream_t s);
// bf16 columns / ∂columns (DCN_BF16; needs bf16_path_ok(g)): same kernels, bf16 rows.
bool bf16_path_ok(const Geo& g);
hipError_t launch_im2col_bf16(const Geo& g, const bf16_t* xT, const float* off, bf16_t* colT,
                              int b0, int nb, hipStream_t s);
hipError_t launch_col2im_bf16(const Geo& g, const bf16_t* xT, const float* off,
                              const bf16_t* gcolT, float* gx, float* gxT, float* goff,
                              void* bins_ws, int b0, int nb, bool bins_ready, hipStream_t s,
                              int bins_nb = 0);
hipError_t launch_im2col(const Geo& g, const float* x, const float* xT, const float* off,
                         float* colT, int b0, int nb, hipStream_t s);
size_t bins_ws_bytes(const Geo& g, int nb);
// K5b: sample bins of images [b0, b0+nb) from the offsets alone (so they can be built on
// a side stream while the GEMMs run); also zeroes those images' goff when the fused K5
// will only write the binned samples.
hipError_t launch_bins(const Geo& g, const float* off, void* bins_ws, float* goff, int b0, int nb,
                       hipStream_t s);
// Overwrites gx (NCHW) and goff for images [b0, b0+nb); gxT is scratch [B][HWi][C].
// gx == NULL: leave ∂x (sampling route) channels-last in gxT only, for
// launch_offset_conv_bwd to finalise (not with the generic kernels).
// bins_ready: launch_bins already ran on bins_ws for these images.
// bins_nb > 0 (with bins_ready): bins_ws holds the bins of images [0, bins_nb) and gcolT
// points at image b0's ∂columns, so a batch may be processed in chunks (fused path only:
// col2im_chunkable).
hipError_t launch_col2im_coord(const Geo& g, const float* x, const float* xT, const float* off,
                               const float* gcolT, float* gx, float* gxT, float* goff,
                               void* bins_ws, int b0, int nb, bool bins_ready, hipStream_t s,
                               int bins_nb = 0);
bool col2im_chunkable(const Geo& g);
// dcn_fused.hip (f2): im2col gathered into the forward GEMM's LDS tiles, bias in the
// epilogue; still writes colT (for the ∂W GEMM) when colT != NULL.
bool fused_fwd_ok(const Geo& g);
bool fused_fwd_pays(const Geo& g);  // DCN_FWD_AUTO picks the fused kernel
void set_fused_workgroups(int n);    // test hook (dcn_debug_fused_workgroups)
hipError_t launch_fused_fwd(const Geo& g, const float* xT, const float* off, const float* Wf,
                            const float* bias, float* out, float* colT, hipStream_t s);
// dcn_fused_bf16.hip (f2, DCN_BF16): im2col gathered from an LDS window of xT straight into
// the B operand of bf16 MFMAs, out = bf16(Wf·colᵀ + bias) (NCHW); writes colT only when
// colT != NULL. wfr: scratch of fused_fwd_bf16_wfr_elems(g) bf16 (weights in MFMA lane order).
bool fused_fwd_bf16_ok(const Geo& g);
bool fused_fwd_bf16_pays(const Geo& g);  // DCN_FWD_AUTO picks it
size_t fused_fwd_bf16_wfr_elems(const Geo& g);
hipError_t launch_fused_fwd_bf16(const Geo& g, const bf16_t* xT, const float* off,
                                 const bf16_t* w, bf16_t* wfr, const float* bias, bf16_t* out,
                                 bf16_t* colT, hipStream_t s, bool wfr_ready = false);
// ∂Wf partials with the columns recomputed from xT (no column matrix): parts[grp][O][K] for
// fused_dw_bf16_groups(g) image groups, summed afterwards in a fixed order.
bool fused_dw_bf16_ok(const Geo& g);
int fused_dw_bf16_groups(const Geo& g);
hipError_t launch_fused_dw_bf16(const Geo& g, const bf16_t* xT, const float* off,
                                const bf16_t* gout, float* parts, hipStream_t s);
// dcn_offset_conv.hip:
// wt / wt2: scratch of offset_conv_wt_floats(g) floats (transposed w_off copies).
size_t offset_conv_wt_floats(const Geo& g);
size_t offset_conv_goffT_floats(const Geo& g);  // ∂offT rows + ∂w_off block partials
size_t offset_conv_fpart_floats(const Geo& g);  // forward channel-slice partials
// part: scratch of offset_conv_fpart_floats(g) floats (channel-slice partial sums).
bool offset_fwd_mfma_xt_ok(const Geo& g);
hipError_t launch_offset_conv_fwd_xt(const Geo& g, const float* x, const float* w_off,
                                     const float* b_off, float* off, float* xT, float* wf,
                                     hipStream_t s);
hipError_t launch_offset_conv_fwd(const Geo& g, const float* x, const float* w_off,
                                  const float* b_off, float* off, float* wt, float* part,
                                  hipStream_t s);
// DCN_BF16 forward offset conv on bf16 MFMA from the channels-last bf16 x: writes the
// bf16-rounded offsets (off) and their fp32 values (off32). Needs offset_fwd_mfma_bf16_ok.
bool offset_fwd_mfma_bf16_ok(const Geo& g);
size_t offset_fwd_bf16_wb_elems(const Geo& g);
// x_nchw != NULL (needs offset_fwd_bf16_fold_ok): f3, the window staged from the NCHW x and
// xT WRITTEN by the same blocks (no separate transpose launch, one pass over x).
bool offset_fwd_bf16_fold_ok(const Geo& g);
hipError_t launch_offset_conv_fwd_bf16(const Geo& g, const bf16_t* xT, const bf16_t* w_off,
                                       const float* b_off, float* off32, bf16_t* off, bf16_t* wb,
                                       hipStream_t s, const bf16_t* x_nchw = nullptr,
                                       bool wb_ready = false);
// DCN_BF16 offset-conv backward on bf16 MFMA (stride 1, C % 64 == 0, H·W % 8 == 0): gx is
// the bf16 NCHW grad_x = transpose(gxT_in) + the offset-conv route. part: the goffT scratch;
// wc: offset_bwd_bf16_wc_elems(g) bf16 values.
bool offset_bwd_bf16_ok(const Geo& g);
size_t offset_bwd_bf16_wc_elems(const Geo& g);
// aux / fork / join (optional, aux = nullptr: all on s): the Wc swizzle and the ∂b_off sums
// run on aux beside ∂W_off, joined before ∂x
hipError_t launch_offset_conv_bwd_bf16(const Geo& g, const bf16_t* x, const bf16_t* w_off,
                                       const float* goff, const float* gxT_in, bf16_t* wc,
                                       float* part, bf16_t* gx, float* gw_off, float* gb_off,
                                       hipStream_t s, hipStream_t aux = nullptr,
                                       hipEvent_t fork = nullptr, hipEvent_t join = nullptr,
                                       bool wc_ready = false, float* bsum_part = nullptr);
// xT: channels-last x; goffT: scratch of offset_conv_goffT_floats(g). gxT_in == NULL:
// grad_x is accumulated; else grad_x = transpose(gxT_in) + the offset-conv route, written
// once (gxT_in: the sampling-route ∂x left channels-last by launch_col2im_*).
// gb_off == NULL: the caller computes ∂b_off (launch_channel_sum) itself.
hipError_t launch_offset_conv_bwd(const Geo& g, const float* x, const float* xT,
                                  const float* w_off, const float* goff, float* goffT, float* wt2,
                                  float* gx, float* gw_off, float* gb_off, const float* gxT_in,
                                  hipStream_t s, hipStream_t aux = nullptr,
                                  hipEvent_t fork = nullptr, hipEvent_t join = nullptr,
                                  float* bsum_part = nullptr);  // B·J floats: two-level ∂b_off
// The MFMA offset-conv backward (stride 1) in pieces, so that batch chunk k's ∂W_off / ∂x
// can run on a side stream beside chunk k+1's col2im: prep (w_off transpose) once,
// chunk(b0, nb) per image range (after that range's ∂offset exists), finish once (∂W_off
// partial fold and ∂b_off). Same results as launch_offset_conv_bwd with gxT_in.
// r05 (fp32, geometries without an MFMA offset-conv kernel): the offset conv as GEMMs over its
// own im2col `ocol` [B·HW][KK·C] (the `col` region's shape); the host (dcn_api.cpp) runs the
// GEMMs. W' = [J][KK·C] (w_off with k = t·C + c), offT / ∂offT = [B·HW][J].
bool offset_conv_gemm_ok(const Geo& g);
hipError_t launch_ocg_im2col(const Geo& g, const float* xT, float* ocol, hipStream_t s);
hipError_t launch_ocg_wprime(const Geo& g, const float* w_off, float* wp, hipStream_t s);
hipError_t launch_ocg_offt_to_off(const Geo& g, const float* offT, const float* b_off, float* off,
                                  hipStream_t s);
hipError_t launch_ocg_goff_to_pj(const Geo& g, const float* goff, float* goffT, hipStream_t s);
hipError_t launch_ocg_wgrad_out(const Geo& g, const float* gwp, float* gw_off, hipStream_t s);
// ∂x = (gxT_in ? transpose(gxT_in) : ∂x) + the gather of ∂ocol
hipError_t launch_ocg_col2im(const Geo& g, const float* docol, const float* gxT_in, float* gx,
                             hipStream_t s);
bool offset_bwd_chunkable(const Geo& g);
hipError_t launch_offset_bwd_prep(const Geo& g, const float* w_off, float* wt2, hipStream_t s);
// xT: the fp32 channels-last x, or (xT_bf16) the bf16 one of DCN_BF16.
hipError_t launch_offset_bwd_chunk(const Geo& g, const void* xT, bool xT_bf16, const float* goff,
                                   float* goffT, const float* wt2, float* gx,
                                   const float* gxT_in, int b0, int nb, hipStream_t s,
                                   hipStream_t s_dx = nullptr);
hipError_t launch_offset_bwd_finish(const Geo& g, const float* goff, const float* goffT,
                                    float* gw_off, float* gb_off, hipStream_t s,
                                    float* bsum_part = nullptr);
// dcn_reduce.hip conversions: bf16 <-> f32 (RNE), and the bf16 rounding of a f32 tensor
// in place (out = bf16(v), v = f32(out)) so later f32 work sees exactly the bf16 value.
hipError_t launch_bf16_to_f32(const bf16_t* in, float* out, size_t n, hipStream_t s);
// several bf16 <-> fp32 conversions in one launch (segments with n == 0 are skipped)
constexpr int kMaxConv = 4;
struct ConvSeg {
  const void* in;
  void* out;
  size_t n;
  int to_bf16;  // 1: fp32 -> bf16 (RNE), 0: bf16 -> fp32
};
struct ConvBatch {
  ConvSeg seg[kMaxConv];
  int n = 0;
  bool overflow = false;  // more than kMaxConv segments: launch_convert_multi refuses the batch
  void add(const void* in, void* out, size_t count, bool to_bf16) {
    if (!count) return;
    if (n == kMaxConv) {
      overflow = true;
      return;
    }
    seg[n++] = ConvSeg{in, out, count, to_bf16 ? 1 : 0};
  }
};
hipError_t launch_convert_multi(const ConvBatch& cb, hipStream_t s);
// One launch for a direction's small preparation work (dcn_reduce.hip, dcn_swizzle.h): bf16 ->
// fp32 copies and the weight re-layouts of the bf16 kernels.
enum PrepKind { PREP_F32 = 0, PREP_TJC = 1, PREP_CK = 2, PREP_FRAG16 = 3, PREP_DCOL = 4 };
struct PrepJob {
  int kind;
  long units;  // PREP_F32: quads of elements; TJC / CK: elements; FRAG16 / DCOL: 16-B fragments
  const void* in;
  void* out;
  long n;  // PREP_F32: elements
  int a, b, c, d, e;
};
constexpr int kMaxPrep = 6;
struct PrepBatch {
  PrepJob job[kMaxPrep];
  int n = 0;
  bool overflow = false;
  void add(const PrepJob& j) {
    if (j.units <= 0) return;
    if (n == kMaxPrep) {
      overflow = true;
      return;
    }
    job[n++] = j;
  }
  void f32(const bf16_t* in, float* out, size_t count) {
    add(PrepJob{PREP_F32, (long)((count + 3) / 4), in, out, (long)count, 0, 0, 0, 0, 0});
  }
};
hipError_t launch_prep_bf16(const PrepBatch& pb, hipStream_t s);
// the batch jobs of the weight re-layouts: launch_offset_conv_fwd_bf16 (TJC: wb),
// launch_offset_conv_bwd_bf16 (CK: wc) and launch_fused_fwd_bf16 (FRAG16: wfr) launch their own
// unless told it is ready; launch_dcol_bf16 (DCOL: wz) always reads the prep's
PrepJob prep_tjc(const Geo& g, const bf16_t* w_off, bf16_t* wb);
PrepJob prep_ck(const Geo& g, const bf16_t* w_off, bf16_t* wc);
PrepJob prep_frag16(const Geo& g, const bf16_t* w, bf16_t* wfr);
PrepJob prep_dcol(int K, const bf16_t* w, bf16_t* wz);
hipError_t launch_f32_to_bf16(const float* in, bf16_t* out, size_t n, hipStream_t s);
hipError_t launch_round_to_bf16(float* v, bf16_t* out, size_t n, hipStream_t s);
// out_bf[b][o][m] = bf16(out32[b][o][m] + bias[o]) (bias may be null)
hipError_t launch_bias_to_bf16(const Geo& g, const float* out32, const float* bias, bf16_t* out,
                               hipStream_t s);
void launch_channel_sum(const float* in, int B, int Cn, int HW, float* out, hipStream_t s);
void launch_channel_sum_2l(const float* in, int B, int Cn, int HW, float* part, float* out,
                           hipStream_t s);
void launch_channel_sum_bf16(const bf16_t* in, int B, int Cn, int HW, float* out, hipStream_t s,
                             bf16_t* out_bf = nullptr);
// in[b][c][p] -> out[b][p][c] and chsum[c] = Σ_{b,p} in[b][c][p] (deterministic); tsum is
// scratch of xpose_chsum_floats(B, C, P) floats.
size_t xpose_chsum_floats(int B, int C, int P);
bool launch_xpose_f4(const float* in, float* out, int B, int C, int P, hipStream_t s);
// bf16 NCHW -> NHWC in 16-byte accesses (false when it does not apply: P % 8, C % 64, 16-B
// alignment), and the same pass with the channel sums (fp32 chsum, bf16 chsum_bf if not
// null; tile partials in tsum, xpose_chsum_bf16_floats(B, C, P) floats)
bool launch_xpose_b8(const bf16_t* in, bf16_t* out, int B, int C, int P, hipStream_t s);
size_t xpose_chsum_bf16_floats(int B, int C, int P);
bool launch_xpose_chsum_bf16(const bf16_t* in, bf16_t* out, float* tsum, float* chsum,
                             bf16_t* chsum_bf, int B, int C, int P, hipStream_t s,
                             hipStream_t s_sum = nullptr, hipEvent_t ev = nullptr);
// ∂out -> ∂outT with ∂b; the per-channel fold of the tile sums runs on s_sum (after event ev)
// when given, so tsum must then stay untouched until s_sum is joined.
hipError_t launch_xpose_chsum(const float* in, float* out, float* tsum, float* chsum, int B,
                              int C, int P, hipStream_t s, hipStream_t s_sum = nullptr,
                              hipEvent_t ev = nullptr);
hipError_t launch_bias_add(const Geo& g, float* out, const float* bias, int b0, int nb,
                           hipStream_t s);
// out[b][o][p] = src[o][b][p] (+ bias[o] when bias != NULL): the flat forward GEMM's result
hipError_t launch_permute_obp_bias(const float* src, const float* bias, float* out, int B, int O,
                                   int HW, hipStream_t s);
hipError_t launch_bias_grad(const Geo& g, const float* gout, float* gb, hipStream_t s);
hipError_t launch_sum_partials(const float* parts, int nparts, size_t n, float* dst,
                               hipStream_t s,
                               bf16_t* dst_bf = nullptr);

// dcn_roi_pool.hip: deformable RoI pooling (deform_conv.py:85-241), see include/dcn.h.
struct RoiGeo {
  int B, C, H, W, R;
  int ph, pw, part_h, part_w;
  int P;     // ph*pw bins
  int Cout;  // C (DeformRoIPool) or C / P (DeformPSRoIPool)
  int ps, no_trans;
  float scale, trans_std;
};
bool roi_geo_ok(const RoiGeo& q);
hipError_t launch_roi_pool_fwd(const RoiGeo& q, const float* f, const float* rois,
                               const float* offsets, float* out, hipStream_t s);
// overwrites gf (memset + atomics) and goffs (may be null)
hipError_t launch_roi_pool_bwd(const RoiGeo& q, const float* f, const float* rois,
                               const float* offsets, const float* gout, float* gf, float* goffs,
                               hipStream_t s);

// dcn_dcol_bf16.hip: the bf16 ∂columns ∂colT[p][k] = Σ_o ∂outT[p][o] · Wf[o][k] (O = 256,
// K % 256 == 0) as a short-K streaming kernel; wz = K·O bf16, Wf in its A-fragment order
// dcn_dw_bf16.hip: ∂Wf partial planes [ranges][O][K] (fp32) = Σ over each pixel range of
// ∂outT[p][o] · col[p][k] (bf16 operands, O == 256, K % 256 == 0); launch_sum_partials over
// dw_stream_bf16_ranges planes gives ∂W.
bool dw_stream_bf16_ok(int K, int O, long npix);
int dw_stream_bf16_ranges(int K, long npix);
hipError_t launch_dw_stream_bf16(const bf16_t* goutT, const bf16_t* col, float* parts, int K,
                                 int O, long npix, hipStream_t s);
bool dcol_bf16_ok(int K, int O, long npix);
hipError_t launch_dcol_bf16(const bf16_t* wz, const bf16_t* goutT, bf16_t* col, int K, int O,
                            long npix, hipStream_t s);

// dcn_gemm.cpp: C = op(A)·op(B) (column-major, alpha 1, beta 0), strided batched.
struct GemmSpec {
  bool ta = false, tb = false;
  int m = 0, n = 0, k = 0, lda = 0, ldb = 0, ldc = 0;
  long sa = 0, sb = 0, sc = 0;
  int batch = 1;
  bool bf16_ab = false;  // A and B are bf16 (DCN_BF16); compute is always fp32
  bool bf16_c = false;   // C is bf16 (else fp32)
  // native f32 MFMA whatever the handle's dcn_math: the math mode covers only the three GEMMs
  // of the op (include/dcn.h); the offset conv's GEMMs set this (their outputs are sampling
  // coordinates, so split-bf16 rounding there would move floors)
  bool native_f32 = false;
};
struct GemmEngine;
int gemm_engine_create(GemmEngine** out, std::string* err);
void gemm_engine_destroy(GemmEngine* e);
// A, B, C point to fp32 or bf16 elements as the spec says
int gemm_run(GemmEngine* e, const GemmSpec& s, const void* A, const void* B, void* C,
             hipStream_t st, std::string* err);
int gemm_backend_of(GemmEngine* e, const GemmSpec& s);  // -1 untuned, 0 rocBLAS, 1 hipBLASLt,
                                                        // 2 split-bf16 (dcn_gemm_split.hip)
// GEMM arithmetic of fp32 products (dcn_math): 0 native f32 MFMA (vendor libraries),
// 3 / 6 / 9 = split-bf16 products on the bf16 matrix cores (dcn_gemm_split.hip).
void gemm_set_math(GemmEngine* e, int math);
int gemm_get_math(GemmEngine* e);
bool gemm_split_ok(const GemmSpec& s, const void* A, const void* B, const void* C);
// column-major C (+ bias[n] if bias) = op(A)·op(B) in split-bf16 arithmetic (math 3/6/9);
// form 1 = loads after the MFMAs (3 workgroups/CU, the measured default), 0 = before
hipError_t launch_gemm_split(int math, const GemmSpec& s, const float* A, const float* B,
                             float* C, hipStream_t st, const float* bias = nullptr,
                             int form = 1);

// Selection of the im2col / col2im implementation (tests force the generic
// global-memory kernels to cross-check the channels-last ones).
void set_force_generic(int on);
void set_bins_chunked(int on);
int get_force_generic();

}  // namespace dcn
