// dcn_api.cpp — C-ABI of libdcn.so (include/dcn.h): handles, workspace, the
// DeformConv2d forward/backward pipelines and the three dense contractions on
// rocBLAS (exact fp32 MFMA GEMMs on gfx950).
//
// Forward  = deform_conv.py:56-81:  K3 offset conv -> K1 deformable im2col ->
//            GEMM (out_b = W[O][N*C] · col_b) -> bias.
// Backward = Jittor autodiff of the same graph (train.py:414): ∂b, ∂W (per-image
//            GEMM partials + deterministic sum), ∂col = Wᵀ·∂out, K5 col2im +
//            coordinate gradient, offset-conv backward.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dcn_host.h"
#include "dcn_internal.h"

// A/B: the bf16 offset backward's ∂x kernel on the side stream beside ∂W_off
#ifndef OFFB_CONC
#define OFFB_CONC 1
#endif
#ifndef OFFB_CONC_F32
#define OFFB_CONC_F32 1  // (A/B builds: 0 = the fp32 offset-conv ∂x after ∂W_off, r05's order)
#endif

using dcn::Geo;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return fail(DCN_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));           \
  } while (0)

#define GEMM_TRY(h, spec, A, B, C)                                                           \
  do {                                                                                       \
    std::string e_;                                                                          \
    if (dcn::gemm_run((h)->gemm, (spec), (A), (B), (C), (h)->stream, &e_) != 0)              \
      return fail(DCN_ERR_BLAS, e_);                                                         \
  } while (0)

#define DCN_TRY(expr)           \
  do {                          \
    int r_ = (expr);            \
    if (r_ != DCN_OK) return r_; \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Validate a descriptor and derive the geometry (deform_conv.py:7-14, :34-35).
int make_geo(const dcn_desc* d, Geo* g) {
  if (!d || !g) return fail(DCN_ERR_INVALID, "null descriptor");
  if (d->B <= 0 || d->C <= 0 || d->H <= 0 || d->W <= 0 || d->O <= 0)
    return fail(DCN_ERR_INVALID, "B, C, H, W, O must be positive");
  if (d->kh <= 0 || d->kw <= 0 || d->sh <= 0 || d->sw <= 0 || d->ph < 0 || d->pw < 0)
    return fail(DCN_ERR_INVALID, "kernel/stride must be positive, padding >= 0");
  if (d->dil_h <= 0 || d->dil_w <= 0 || d->deform_groups <= 0)
    return fail(DCN_ERR_INVALID, "dilation and deform_groups must be >= 1");
  if (d->C % d->deform_groups != 0)
    return fail(DCN_ERR_INVALID, "in_channels must be divisible by deform_groups");
  if (d->dtype != DCN_F32 && d->dtype != DCN_BF16) return fail(DCN_ERR_INVALID, "unknown dtype");
  Geo& q = *g;
  q.dt = d->dtype;
  q.B = d->B; q.C = d->C; q.H = d->H; q.W = d->W; q.O = d->O;
  q.kh = d->kh; q.kw = d->kw; q.sh = d->sh; q.sw = d->sw; q.ph = d->ph; q.pw = d->pw;
  q.dh = d->dil_h; q.dw = d->dil_w; q.G = d->deform_groups;
  q.Ho = (d->H + 2 * d->ph - d->dil_h * (d->kh - 1) - 1) / d->sh + 1;
  q.Wo = (d->W + 2 * d->pw - d->dil_w * (d->kw - 1) - 1) / d->sw + 1;
  if (q.Ho <= 0 || q.Wo <= 0) return fail(DCN_ERR_INVALID, "empty output (input too small)");
  if (q.Ho < 2 || q.Wo < 2)
    return fail(DCN_ERR_UNSUPPORTED,
                "H_out or W_out == 1: the reference divides by (W_out-1)/(H_out-1) "
                "(deform_conv.py:37-38)");
  q.N = d->kh * d->kw;
  q.K = q.N * d->C;
  q.HW = q.Ho * q.Wo;
  q.HWi = d->H * d->W;
  q.Cg = d->C / d->deform_groups;
  q.J = 2 * q.N * q.G;
  if ((long long)q.K * q.HW > (1LL << 31) - 1 || (long long)q.HWi > (1LL << 30))
    return fail(DCN_ERR_UNSUPPORTED, "per-image column block exceeds 2^31 elements");
  if ((long long)q.O > (1 << 30) || (long long)q.K > (1 << 30))
    return fail(DCN_ERR_UNSUPPORTED, "channel counts too large");
  if (q.dt == DCN_BF16 && !dcn::bf16_path_ok(q))
    return fail(DCN_ERR_UNSUPPORTED,
                "DCN_BF16 needs deform_groups == 1, kh*kw <= 9, C % 4 == 0 and C <= 256");
  return DCN_OK;
}

size_t elem_bytes(const Geo& g) { return g.dt == DCN_BF16 ? 2 : 4; }

// The standalone kernel entry points (offset conv, im2col, col2im) are fp32 only.
int make_geo_f32(const dcn_desc* d, Geo* g) {
  DCN_TRY(make_geo(d, g));
  if (g->dt != DCN_F32)
    return fail(DCN_ERR_UNSUPPORTED, "standalone kernel entry points take DCN_F32 only");
  return DCN_OK;
}

// ∂W as dwg grouped NT GEMMs over B/dwg images each, or one NN GEMM per image (0). r01
// (tools/dw_ab.sh): bf16 config 4 ∂W 0.178 ms per image -> 0.130 ms in 16 groups (step 1.10 ->
// 1.02 ms); fp32 config 3 unchanged at 1.65 ms, so fp32 stays per image.
int dw_groups(const Geo& g) {
  return (g.dt == DCN_BF16 && g.B > 16 && g.B % 16 == 0) ? 16 : 0;
}

// The ∂W partial planes ([O][K] fp32 each) that each backward path of this geometry writes
// into the workspace's `parts` region before its fixed-order sum: one per image (the fp32
// and the ungrouped bf16 GEMMs), dw_groups(g) (the grouped bf16 GEMM), and
// fused_dw_bf16_groups(g) (the recomputed-column kernel of DCN_FWD_FUSED_NOCOL). ws_layout
// sizes `parts` from the largest, and every backward checks its own count against what the
// layout holds (the region once held fewer planes than a kernel
// wrote).
// dw_stream_bf16 (the stored-column bf16 ∂W kernel, csrc/dcn_dw_bf16.hip) writes one plane
// per pixel range.
enum { DW_PER_IMAGE, DW_GROUPED, DW_FUSED, DW_STREAM, DW_PATHS };
bool dw_stream_applies(const Geo& g) {
  return g.dt == DCN_BF16 && dcn::dw_stream_bf16_ok(g.K, g.O, (long)g.B * g.HW);
}
void dw_parts(const Geo& g, int n[DW_PATHS]) {
  n[DW_PER_IMAGE] = g.B;
  n[DW_GROUPED] = dw_groups(g);
  n[DW_FUSED] = g.dt == DCN_BF16 && dcn::fused_dw_bf16_ok(g) ? dcn::fused_dw_bf16_groups(g) : 0;
  n[DW_STREAM] = dw_stream_applies(g) ? dcn::dw_stream_bf16_ranges(g.K, (long)g.B * g.HW) : 0;
}
int dw_parts_max(const Geo& g) {
  int n[DW_PATHS];
  dw_parts(g, n);
  return *std::max_element(n, n + DW_PATHS);
}

// The fp32 forward GEMM as ONE product over the batch's pixels instead of one per image
// (r06); its [O][B·HW] result goes to NCHW with the bias folded in (launch_permute_obp_bias,
// which replaces the bias pass at the same bytes). Config 5 (Ho·Wo = 36): the per-image GEMM's
// 64-pixel tiles ran 1.78× the MFMA work (SQ_VALU_MFMA_BUSY 0.86 against 0.51 of useful
// flops), forward GEMM 0.138 -> 0.091 ms; config 3: 1.650 -> 1.603-1.616 ms, step -0.04 ms;
// config 2: no change (tools/ab.sh, one box each). Costs a [B][O][HW] fp32 workspace region.
bool fwd_flat_gemm(const Geo& g) {
  return g.dt == DCN_F32 && g.B > 1 && (long)g.B * g.HW * g.K < (1l << 31) &&
         (long)g.B * g.HW * g.O < (1l << 31);
}

struct WsLayout {
  size_t xT = 0;     // [B][H*W][C] channels-last copy of x (forward, kept for backward)
  size_t wt = 0;     // transposed w_off copy for the offset-conv kernels
  size_t part = 0;   // offset-conv channel-slice partials (forward)
  size_t col = 0;    // [B][HW][K] channels-last columns / ∂columns
  size_t fwdT = 0;   // [O][B][HW] the flat forward GEMM's result (fwd_flat_gemm geometries)
  size_t ocol = 0;   // [B][HW][C·kh·kw] the offset conv's im2col (fp32 GEMM route, ocol_ws)
  bool has_ocol = false;
  size_t parts = 0;  // [dw_parts_max][O*K] ∂W partials
  int parts_planes = 0;  // the [O][K] planes `parts` holds (0: forward-only layout)
  size_t goff = 0;   // [B][J][HW] ∂offset (when the caller passes none)
  size_t goffT = 0;  // [B][HW][J] channels-last ∂offset (offset-conv ∂W)
  size_t gxT = 0;    // [B][H*W][C] channels-last ∂x (sampling route)
  size_t goutT = 0;  // [B][Ho*Wo][O] transposed ∂out (flat ∂col GEMM)
  size_t bins = 0;   // sample bins of K5b
  // DCN_BF16 only: fp32 working copies (the offset conv, coordinates and reductions run
  // in fp32; only the columns and the GEMM operands are bf16)
  // (DCN_BF16 keeps its channels-last x in `xT` as bf16; xT32 is the fp32 one that only the
  // VALU offset-conv fallbacks read, wb16 the bf16 weights of the MFMA offset conv)
  size_t x32 = 0, xT32 = 0, wb16 = 0, woff32 = 0, boff32 = 0, b32 = 0, off32 = 0, out32 = 0;
  size_t wfr = 0;  // fused bf16 forward: Wf in MFMA lane order
  size_t gx32 = 0, gw32 = 0, gb32 = 0, gwo32 = 0, gbo32 = 0, goff32 = 0;
  size_t wz = 0;  // dcol_bf16: Wf in MFMA A-fragment order
  size_t total = 0;
};

// cols = false: the forward-only layout of a forward that writes no columns (a
// DCN_BF16 fused forward under DCN_FWD_NO_COLUMNS / DCN_FWD_FUSED_NOCOL): no `col` region
WsLayout ws_layout(const Geo& g, bool bwd, bool cols = true) {
  WsLayout L;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t at = off;
    off = align_up(off + bytes, 256);
    return at;
  };
  L.xT = take((size_t)g.B * g.HWi * g.C * sizeof(float));
  L.wt = take(dcn::offset_conv_wt_floats(g) * sizeof(float));
  L.part = take(dcn::offset_conv_fpart_floats(g) * sizeof(float));
  L.col = take(cols ? (size_t)g.B * g.HW * g.K * sizeof(float) : 0);
  L.fwdT = take(fwd_flat_gemm(g) ? (size_t)g.B * g.O * g.HW * sizeof(float) : 0);
  // r06: the forward's offset-conv im2col kept for the backward's ∂W' GEMM (geometries of
  // the fp32 offset-conv GEMM route, whatever dcn_debug_offset_gemm says: the layout depends
  // on the geometry alone), in the prefix the forward-only and backward layouts share
  L.has_ocol = g.dt == DCN_F32 && dcn::offset_conv_gemm_ok(g) && !dcn::offset_fwd_mfma_xt_ok(g) &&
               !dcn::offset_bwd_chunkable(g);
  L.ocol = take(L.has_ocol ? (size_t)g.B * g.HW * g.C * g.kh * g.kw * sizeof(float) : 0);
  const size_t f = sizeof(float);
  if (g.dt == DCN_BF16) {
    // DCN_BF16 forward copies, at the same offsets in the forward-only and the
    // forward+backward layouts: a backward with DCN_BWD_COL_IN_WS reads what the forward
    // (which always uses the forward-only layout) wrote
    // fp32 copies of x only for the fallback offset-conv kernels (the MFMA paths read the
    // bf16 x / xT directly): NCHW when either direction falls back, channels-last for the
    // VALU backward. Depends on the geometry alone, so both layouts agree.
    const bool fb_fwd = !dcn::offset_fwd_mfma_bf16_ok(g), fb_bwd = !dcn::offset_bwd_bf16_ok(g);
    const size_t xb = (size_t)g.B * g.C * g.HWi * f;
    L.x32 = take(fb_fwd || fb_bwd ? xb : 0);
    L.xT32 = take(fb_bwd ? xb : 0);
    L.wb16 = take(std::max(dcn::offset_fwd_bf16_wb_elems(g), dcn::offset_bwd_bf16_wc_elems(g)) *
                  sizeof(dcn::bf16_t));
    L.woff32 = take((size_t)g.J * g.C * g.N * f);
    L.boff32 = take((size_t)g.J * f);
    L.b32 = take((size_t)g.O * f);
    L.off32 = take((size_t)g.B * g.J * g.HW * f);
    L.out32 = take((size_t)g.B * g.O * g.HW * f);
    L.wfr = take(dcn::fused_fwd_bf16_ok(g) ? dcn::fused_fwd_bf16_wfr_elems(g) * sizeof(dcn::bf16_t)
                                           : 0);
  }
  if (bwd) {
    // ∂W partials; first also the ∂b tile sums of the fused ∂out transpose
    L.parts_planes = dw_parts_max(g);
    L.parts = take(std::max((size_t)L.parts_planes * g.O * g.K,
                            dcn::xpose_chsum_floats(g.B, g.O, g.HW)) * sizeof(float));
    L.goff = take((size_t)g.B * g.J * g.HW * sizeof(float));
    L.goffT = take(dcn::offset_conv_goffT_floats(g) * sizeof(float));
    L.gxT = take((size_t)g.B * g.HWi * g.C * sizeof(float));
    L.goutT = take((size_t)g.B * g.HW * g.O * sizeof(float));
    L.bins = take(dcn::bins_ws_bytes(g, g.B));
  }
  if (g.dt == DCN_BF16 && bwd) {
    // fp32 ∂x only where the offset-conv backward does not write the bf16 ∂x itself
    L.gx32 = take(dcn::offset_bwd_bf16_ok(g) ? 0 : (size_t)g.B * g.C * g.HWi * f);
    L.gw32 = take((size_t)g.O * g.K * f);
    L.gb32 = take((size_t)g.O * f);
    L.gwo32 = take((size_t)g.J * g.C * g.N * f);
    L.gbo32 = take((size_t)g.J * f);
    L.goff32 = take((size_t)g.B * g.J * g.HW * f);
    L.wz = take(dcn::dcol_bf16_ok(g.K, g.O, (long)g.B * g.HW) ? (size_t)g.K * g.O * sizeof(dcn::bf16_t)
                                                              : 0);
  }
  L.total = off;
  return L;
}

}  // namespace

struct dcn_handle {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  // side stream for work that depends only on inputs (x transpose beside the offset conv,
  // sample bins beside the GEMMs); forked from / joined back into `stream` with events
  hipStream_t aux = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  dcn::GemmEngine* gemm = nullptr;
  int fwd_path = DCN_FWD_AUTO;  // dcn_set_fwd_path
  // bf16 ∂columns on the vendor GEMM instead of dcol_bf16 (DCN_DCOL_GEMM=1: the A/B switch)
  bool dcol_gemm = false;
  // bf16 ∂W on the vendor GEMM instead of dw_stream_bf16 (DCN_DW_GEMM=1: the A/B switch)
  bool dw_gemm = false;
  // workspaces whose last DCN_BF16 forward on this handle wrote its columns into them, most
  // recent last. A DCN_BWD_COL_IN_WS backward reads the columns only from a workspace listed
  // here and recomputes them otherwise (a forward under DCN_FWD_FUSED_NOCOL or
  // DCN_FWD_NO_COLUMNS drops its workspace). At most kColWsCap entries: the oldest drops
  // first, and a backward on a dropped workspace just recomputes, so the record never grows
  // with the number of distinct workspaces (it used to) and is never wrong.
  // Guarded by col_ws_mu: concurrent forwards / backwards on one handle may touch it.
  static constexpr size_t kColWsCap = 256;
  std::vector<const void*> col_ws;
  // the same record (same cap, same mutex) for the fp32 offset-conv GEMM route: workspaces
  // whose last forward on this handle left the offset conv's im2col (`ocol`) and W' there
  std::vector<const void*> ocol_ws;
  std::mutex col_ws_mu;
  // data-parallel gradient exchange (dcn_set_comm / dcn_set_grad_stream): the ∂W/∂b
  // all-reduce runs on comm_stream as soon as they are final (dw_main / dw_aux), beside the
  // rest of the backward; the stream waits for comm_done before anything later
  dcn_comm* comm = nullptr;
  hipStream_t comm_stream = nullptr;
  hipStream_t grad_stream = nullptr;  // caller's stream to release at ∂W/∂b-final
  hipEvent_t dw_main = nullptr, dw_aux = nullptr, end_ev = nullptr, comm_done = nullptr;
  hipEvent_t k5_ev = nullptr;  // bf16 backward: the side-stream work K5 depends on is done
  // host-pointer API: device copies of the tensors no module state keeps (outputs and
  // gradients, grow-only, one per role), the pinned staging ring, the per-module states
  // (dcn_host_state, hs0 = the one dcn_forward_host / dcn_backward_host[_ex] use), and the
  // copy streams + events of the image-chunk transfer pipeline
  void* hbuf[16] = {nullptr};
  size_t hbuf_bytes[16] = {0};
  dcn::HostStage* stage = nullptr;
  int staging = -1;  // DCN_HOST_STAGING, read at the first host transfer
  dcn_host_state* hs0 = nullptr;
  std::vector<dcn_host_state*> states;
  hipStream_t cin = nullptr, cout = nullptr;
  std::vector<hipEvent_t> hev;  // [2*i] chunk i uploaded, [2*i+1] chunk i computed
  // scratch of the standalone kernel API
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // profiling: events per kernel class
  int prof_cap = 0;
  std::vector<hipEvent_t> ev[DCN_K_COUNT];  // pairs: [2*i] start, [2*i+1] stop
  int prof_n[DCN_K_COUNT] = {0};
};

enum StateRole { SB_X, SB_OFF, SB_WO, SB_W, SB_COUNT };

// One module's device state for the host-pointer API (include/dcn.h dcn_host_state): its
// x / offsets / weights, its workspace (one slice per image chunk, each holding that
// chunk's columns for the backward) and what its last forward was given.
struct dcn_host_state {
  dcn_handle* h = nullptr;  // null once the handle is destroyed
  void* dev[SB_COUNT] = {nullptr};
  size_t dev_bytes[SB_COUNT] = {0};
  void* ws = nullptr;
  size_t ws_bytes = 0;
  int chunks = 0;  // dcn_host_state_set_chunks; 0 = auto
  bool valid = false;
  int plan_n = 1;  // image chunks of the last forward
  dcn_desc desc{};
  const void *x = nullptr, *wo = nullptr, *w = nullptr, *off = nullptr;
};

namespace {
void state_free(dcn_host_state* s);
}  // namespace

namespace {

struct ProfScope {
  dcn_handle* h;
  int id;
  bool on;
  hipStream_t st;
  ProfScope(dcn_handle* hh, int k, hipStream_t s = nullptr)
      : h(hh), id(k), on(hh->prof_cap > 0 && hh->prof_n[k] < hh->prof_cap),
        st(s ? s : hh->stream) {
    if (on) (void)hipEventRecord(h->ev[id][2 * h->prof_n[id]], st);
  }
  ~ProfScope() {
    if (on) {
      (void)hipEventRecord(h->ev[id][2 * h->prof_n[id] + 1], st);
      ++h->prof_n[id];
    }
  }
};

int set_device(dcn_handle* h) {
  if (!h) return fail(DCN_ERR_INVALID, "null handle");
  HIP_TRY(hipSetDevice(h->device));
  return DCN_OK;
}

// per-workspace records (dcn_handle::col_ws, ocol_ws)
bool ws_rec_has(dcn_handle* h, const std::vector<const void*>& rec, const void* ws) {
  std::lock_guard<std::mutex> lk(h->col_ws_mu);
  return std::find(rec.begin(), rec.end(), ws) != rec.end();
}
void ws_rec_mark(dcn_handle* h, std::vector<const void*>& rec, const void* ws, bool has) {
  std::lock_guard<std::mutex> lk(h->col_ws_mu);
  auto it = std::find(rec.begin(), rec.end(), ws);
  if (it != rec.end()) rec.erase(it);
  if (!has) return;
  if (rec.size() >= dcn_handle::kColWsCap) rec.erase(rec.begin());
  rec.push_back(ws);
}
// Does this workspace hold the columns of the last DCN_BF16 forward that used it?
bool ws_has_columns(dcn_handle* h, const void* ws) { return ws_rec_has(h, h->col_ws, ws); }
void ws_mark_columns(dcn_handle* h, const void* ws, bool has) {
  ws_rec_mark(h, h->col_ws, ws, has);
}

// Can the DCN_BF16 forward of this geometry skip the column matrix (the fused forward
// applies)? One predicate for dcn_workspace_bytes(DCN_WS_FORWARD_NO_COLUMNS) and the forward
// itself (the two disagreed under dcn_debug_force_generic).
bool fwd_can_skip_columns(const Geo& g) {
  return g.dt == DCN_BF16 && dcn::fused_fwd_bf16_ok(g) && !dcn::get_force_generic();
}

// Does a DCN_BF16 forward under this path / these flags skip the columns?
bool fwd_skips_columns(const dcn_handle* h, const Geo& g, int flags) {
  return fwd_can_skip_columns(g) &&
         (h->fwd_path == DCN_FWD_FUSED_NOCOL || (flags & DCN_FWD_NO_COLUMNS) != 0);
}

// ---- forward / backward cores ---------------------------------------------------
// aux waits for everything issued on the main stream so far
int fork_aux(dcn_handle* h) {
  HIP_TRY(hipEventRecord(h->fork_ev, h->stream));
  HIP_TRY(hipStreamWaitEvent(h->aux, h->fork_ev, 0));
  return DCN_OK;
}
// the main stream waits for everything issued on aux so far
int join_aux(dcn_handle* h) {
  HIP_TRY(hipEventRecord(h->join_ev, h->aux));
  HIP_TRY(hipStreamWaitEvent(h->stream, h->join_ev, 0));
  return DCN_OK;
}

extern "C" __attribute__((visibility("hidden"))) void dcn_internal_handle_drop_comm(dcn_handle* h);
extern "C" __attribute__((visibility("hidden"))) void dcn_internal_comm_attach(dcn_comm* c,
                                                                             dcn_handle* h);
extern "C" __attribute__((visibility("hidden"))) void dcn_internal_comm_detach(dcn_comm* c,
                                                                             dcn_handle* h);
extern "C" __attribute__((visibility("hidden"))) int dcn_internal_allreduce_n(
    dcn_comm* c, int n, void* const* bufs, const size_t* counts, int dtype, void* st);

// ∂W / ∂b are final once everything issued so far on the main and the side stream is done:
// release the caller's grad stream (dcn_set_grad_stream) and, with a communicator attached,
// start their all-reduce on comm_stream (fp32 values: DCN_F32 tensors, or the fp32 working
// copies of DCN_BF16, converted to bf16 by `post` on comm_stream after the sum).
int dw_final(dcn_handle* h, float* gw, float* gb, const Geo& g,
             dcn::bf16_t* gw_bf = nullptr, dcn::bf16_t* gb_bf = nullptr) {
  if (!h->comm && !h->grad_stream) return DCN_OK;
  HIP_TRY(hipEventRecord(h->dw_main, h->stream));
  HIP_TRY(hipEventRecord(h->dw_aux, h->aux));
  if (h->grad_stream) {
    HIP_TRY(hipStreamWaitEvent(h->grad_stream, h->dw_main, 0));
    HIP_TRY(hipStreamWaitEvent(h->grad_stream, h->dw_aux, 0));
  }
  if (!h->comm) return DCN_OK;
  HIP_TRY(hipStreamWaitEvent(h->comm_stream, h->dw_main, 0));
  HIP_TRY(hipStreamWaitEvent(h->comm_stream, h->dw_aux, 0));
  void* bufs[2] = {gw, gb};
  const size_t counts[2] = {(size_t)g.O * g.K, gb ? (size_t)g.O : 0};
  DCN_TRY(dcn_internal_allreduce_n(h->comm, 2, bufs, counts, DCN_F32, h->comm_stream));
  if (gw_bf) HIP_TRY(dcn::launch_f32_to_bf16(gw, gw_bf, counts[0], h->comm_stream));
  if (gb_bf && gb) HIP_TRY(dcn::launch_f32_to_bf16(gb, gb_bf, counts[1], h->comm_stream));
  return DCN_OK;
}

// End of dcn_backward with a communicator: ∂W_off / ∂b_off summed after everything on the
// main stream, then the main stream waits for the whole exchange.
int grads_final(dcn_handle* h, float* gwo, float* gbo, const Geo& g,
                dcn::bf16_t* gwo_bf = nullptr, dcn::bf16_t* gbo_bf = nullptr) {
  if (!h->comm) return DCN_OK;
  HIP_TRY(hipEventRecord(h->end_ev, h->stream));
  HIP_TRY(hipStreamWaitEvent(h->comm_stream, h->end_ev, 0));
  void* bufs[2] = {gwo, gbo};
  const size_t counts[2] = {(size_t)g.J * g.C * g.N, (size_t)g.J};
  DCN_TRY(dcn_internal_allreduce_n(h->comm, 2, bufs, counts, DCN_F32, h->comm_stream));
  if (gwo_bf) HIP_TRY(dcn::launch_f32_to_bf16(gwo, gwo_bf, counts[0], h->comm_stream));
  if (gbo_bf) HIP_TRY(dcn::launch_f32_to_bf16(gbo, gbo_bf, counts[1], h->comm_stream));
  HIP_TRY(hipEventRecord(h->comm_done, h->comm_stream));
  HIP_TRY(hipStreamWaitEvent(h->stream, h->comm_done, 0));
  return DCN_OK;
}

// Split-bf16 GEMM arithmetic (dcn_math X3/X6/X9) for the forward GEMM with its bias fused
// (the two backward GEMMs reach the split kernels through dcn::gemm_run).
bool use_split(dcn_handle* h, const Geo& g) {
  return dcn::gemm_get_math(h->gemm) != 0 && g.dt == DCN_F32;
}

int core_forward(dcn_handle* h, const Geo& g, const float* x, const float* off, const float* w,
                 const float* b, bool has_bias, float* out, float* xT, float* colT,
                 bool xT_ready, float* fwdT) {
  if (!xT_ready) {
    ProfScope ps(h, DCN_K_XPOSE);
    HIP_TRY(dcn::launch_nchw_to_nhwc(x, xT, g.B, g.C, g.HWi, h->stream));
  }
  const bool want_fused =
      h->fwd_path == DCN_FWD_FUSED || h->fwd_path == DCN_FWD_FUSED_NOCOL || (h->fwd_path == DCN_FWD_AUTO && dcn::fused_fwd_pays(g));
  if (want_fused && dcn::fused_fwd_ok(g) && !use_split(h, g) && !dcn::get_force_generic()) {
    // f2: im2col gathered into the GEMM's LDS tiles, bias in the epilogue; the columns are
    // still written for the ∂W GEMM of the backward (DCN_BWD_COL_IN_WS)
    ProfScope ps(h, DCN_K_GEMM_FWD);
    HIP_TRY(dcn::launch_fused_fwd(g, xT, off, w, has_bias ? b : nullptr, out, colT, h->stream));
    return DCN_OK;
  }
  {
    ProfScope ps(h, DCN_K_IM2COL);
    HIP_TRY(dcn::launch_im2col(g, x, xT, off, colT, 0, g.B, h->stream));
  }
  {
    // out_b[O][HW] = Wf[O][K] · colT_b[HW][K]ᵀ; column-major: C(HW×O) = colT_bᵀ · Wf (TN GEMM,
    // both operands K-contiguous)
    ProfScope ps(h, DCN_K_GEMM_FWD);
    dcn::GemmSpec sp;
    sp.ta = true;
    sp.m = g.HW; sp.n = g.O; sp.k = g.K;
    sp.lda = g.K; sp.sa = (long)g.K * g.HW;
    sp.ldb = g.K; sp.sb = 0;
    sp.ldc = g.HW; sp.sc = (long)g.O * g.HW;
    sp.batch = g.B;
    if (use_split(h, g) && dcn::gemm_split_ok(sp, colT, w, out)) {
      // split-bf16 arithmetic with the bias in the epilogue
      HIP_TRY(dcn::launch_gemm_split(dcn::gemm_get_math(h->gemm), sp, colT, w, out, h->stream,
                                     has_bias ? b : nullptr));
      return DCN_OK;
    }
    if (fwdT && fwd_flat_gemm(g)) {
      // one product over all B·HW pixels, C(B·HW × O) = colTᵀ · Wf into [O][B][HW]
      sp.m = g.B * g.HW;
      sp.lda = g.K; sp.sa = 0;
      sp.ldc = g.B * g.HW; sp.sc = 0;
      sp.batch = 1;
      GEMM_TRY(h, sp, colT, w, fwdT);
    } else {
      GEMM_TRY(h, sp, colT, w, out);
      fwdT = nullptr;
    }
  }
  if (fwdT) {
    ProfScope ps(h, DCN_K_BIAS_FWD);
    HIP_TRY(dcn::launch_permute_obp_bias(fwdT, has_bias ? b : nullptr, out, g.B, g.O, g.HW,
                                         h->stream));
    return DCN_OK;
  }
  if (has_bias) {
    ProfScope ps(h, DCN_K_BIAS_FWD);
    HIP_TRY(dcn::launch_bias_add(g, out, b, 0, g.B, h->stream));
  }
  return DCN_OK;
}


int core_backward(dcn_handle* h, const Geo& g, const float* x, const float* off, const float* w,
                  const float* gout, float* gx, float* gw, float* gb, bool has_bias, float* goff,
                  float* xT, float* colT, float* parts, float* gxT, float* goutT, void* bins,
                  bool col_valid) {
  // the sample bins depend only on the offsets: build them on the side stream while the
  // main stream runs the ∂W / ∂col GEMMs
  // (r02 A/B: the bins serialised before K5 instead: step 7.06 against 7.00-7.02 ms)
  DCN_TRY(fork_aux(h));
  HIP_TRY(dcn::launch_bins(g, off, bins, goff, 0, g.B, h->aux));
  if (!col_valid) {
    {
      ProfScope ps(h, DCN_K_XPOSE);
      HIP_TRY(dcn::launch_nchw_to_nhwc(x, xT, g.B, g.C, g.HWi, h->stream));
    }
    ProfScope ps(h, DCN_K_IM2COL);
    HIP_TRY(dcn::launch_im2col(g, x, xT, off, colT, 0, g.B, h->stream));
  }
  // images per flat ∂col GEMM: the vendor GEMMs take 32-bit problem sizes, so one product
  // over the batch's pixels covers at most (2^31 - 1) / (HW·K) images; a larger batch runs
  // it in image chunks (at B = 512 the whole-batch product did not
  // fit, and the backward fell back to per-image NT GEMMs and a separate ∂b pass, 22 % slower
  // per image than B = 64)
  const int fchunk = (int)std::min<long>(g.B, ((1l << 31) - 1) / ((long)g.HW * g.K));
  const bool flat = fchunk >= 1;
  const bool flat_dw = (long)g.B * g.HW * g.K < (1l << 31) && g.HW < 256;
  {
    // ∂outT (for the flat GEMMs) and ∂b from one pass over ∂out
    ProfScope ps(h, DCN_K_BWD_BIAS);
    if (flat && has_bias &&
        dcn::xpose_chsum_floats(g.B, g.O, g.HW) <= (size_t)g.B * g.HWi * g.C)
      // tile sums in gxT (written only by K5, later on this stream), their fold right after
      // on this stream too (r06: on the side stream it queued behind the bin sort, and K5
      // waited for both; config 5, DESIGN.md "r06: the fp32 ∂b fold on the main stream")
      HIP_TRY(dcn::launch_xpose_chsum(gout, goutT, gxT, gb, g.B, g.O, g.HW, h->stream));
    else if (flat && has_bias)
      HIP_TRY(dcn::launch_xpose_chsum(gout, goutT, parts, gb, g.B, g.O, g.HW, h->stream));
    else if (flat)
      HIP_TRY(dcn::launch_nchw_to_nhwc(gout, goutT, g.B, g.O, g.HW, h->stream));
    else if (has_bias)
      HIP_TRY(dcn::launch_bias_grad(g, gout, gb, h->stream));
  }
  {
    // ∂Wf[O][K] = Σ_b ∂out_b[O][HW] · colT_b[HW][K]. Per image, column-major
    // P_b(K×O) = colT_b(K×HW) · ∂out_b(HW×O) (NN), then a deterministic Σ_b: 1.68 ms at
    // config 3 against 1.82 ms as one flat GEMM. When the per-image depth HW is tiny
    // (config 5: HW = 49) the flat NT GEMM over k = B·HW against ∂outT wins instead.
    ProfScope ps(h, DCN_K_GEMM_DW);
    dcn::GemmSpec sp;
    const int dwg = dw_groups(g);
    if (flat && dwg > 0) {
      // grouped NT: P_g(K×O) = colT_g · ∂outT_g over the pixels of B/dwg images, then the
      // fixed-order Σ_g (dwg partials instead of B)
      const int pg = (g.B / dwg) * g.HW;
      sp.tb = true;
      sp.m = g.K; sp.n = g.O; sp.k = pg;
      sp.lda = g.K; sp.sa = (long)g.K * pg;
      sp.ldb = g.O; sp.sb = (long)g.O * pg;
      sp.ldc = g.K; sp.sc = (long)g.K * g.O;
      sp.batch = dwg;
      GEMM_TRY(h, sp, colT, goutT, parts);
      DCN_TRY(fork_aux(h));
      HIP_TRY(dcn::launch_sum_partials(parts, dwg, (size_t)g.K * g.O, gw, h->aux));
    } else if (flat_dw) {
      sp.tb = true;
      sp.m = g.K; sp.n = g.O; sp.k = g.B * g.HW;
      sp.lda = g.K; sp.ldb = g.O; sp.ldc = g.K;
      GEMM_TRY(h, sp, colT, goutT, gw);
    } else {
      sp.m = g.K; sp.n = g.O; sp.k = g.HW;
      sp.lda = g.K; sp.sa = (long)g.K * g.HW;
      sp.ldb = g.HW; sp.sb = (long)g.O * g.HW;
      sp.ldc = g.K; sp.sc = (long)g.K * g.O;
      sp.batch = g.B;
      GEMM_TRY(h, sp, colT, gout, parts);
      // the fixed-order Σ_b (151 MB read at config 3) on the side stream, beside the ∂col
      // GEMM (which only reads the weight and ∂out and overwrites the columns)
      DCN_TRY(fork_aux(h));
      HIP_TRY(dcn::launch_sum_partials(parts, g.B, (size_t)g.K * g.O, gw, h->aux));
    }
  }
  // ∂W and ∂b are final once the work issued so far on both streams is done
  DCN_TRY(dw_final(h, gw, has_bias ? gb : nullptr, g));
  {
    // ∂colT[B·HW][K] = ∂outT · Wf as ONE GEMM over the whole batch (r01 probe: 1.68 ms
    // flat vs 1.92 ms as 64 per-image NT GEMMs), after transposing ∂out to
    // ∂outT[B][HW][O] (0.09 ms). Column-major: C(K × B·HW) = Wf(K×O) · ∂outT(O × B·HW)
    // (NN). Overwrites the columns (no longer needed after ∂W).
    ProfScope ps(h, DCN_K_GEMM_DCOL);
    dcn::GemmSpec sp;
    if (flat) {
      for (int b0 = 0; b0 < g.B; b0 += fchunk) {
        const int nb = std::min(fchunk, g.B - b0);
        sp.m = g.K; sp.n = nb * g.HW; sp.k = g.O;
        sp.lda = g.K; sp.ldb = g.O; sp.ldc = g.K;
        sp.batch = 1;
        GEMM_TRY(h, sp, w, goutT + (size_t)b0 * g.HW * g.O, colT + (size_t)b0 * g.HW * g.K);
      }
    } else {  // per-image NT GEMMs: C(K×HW) = Wf(K×O) · ∂out_bᵀ(O×HW)
      sp.tb = true;
      sp.m = g.K; sp.n = g.HW; sp.k = g.O;
      sp.lda = g.K; sp.sa = 0;
      sp.ldb = g.HW; sp.sb = (long)g.O * g.HW;
      sp.ldc = g.K; sp.sc = (long)g.K * g.HW;
      sp.batch = g.B;
      GEMM_TRY(h, sp, w, gout, colT);
    }
  }
  DCN_TRY(join_aux(h));  // bins ready
  {
    // K5 overwrites grad_x (sampling route) and grad_off
    ProfScope ps(h, DCN_K_COL2IM);
    // ∂x stays channels-last in gxT; the offset-conv ∂x pass finalises it (one write)
    HIP_TRY(dcn::launch_col2im_coord(g, x, xT, off, colT, dcn::get_force_generic() ? gx : nullptr,
                                     gxT, goff, bins, 0, g.B, true, h->stream));
  }
  return DCN_OK;
}

// ---- DCN_BF16 orchestration -------------------------------------------------------
// Tensors cross the API in bf16. The offset conv, coordinates, interpolation weights,
// ∂offset / ∂x accumulation and every reduction run in fp32 on working copies; the
// columns, ∂columns and the three GEMM operands are bf16 (MFMA bf16, fp32 accumulate).
// The forward rounds its offsets to bf16 BEFORE sampling with them, so a backward that
// only sees the bf16 offsets samples exactly the same points.
using dcn::bf16_t;
#define BF(o) reinterpret_cast<bf16_t*>(base + (o))
#define F32(o) reinterpret_cast<float*>(base + (o))

int forward_bf16(dcn_handle* h, const Geo& g, bool has_bias, const bf16_t* x,
                 const bf16_t* w_off, const bf16_t* b_off, const bf16_t* w, const bf16_t* b,
                 bf16_t* out, bf16_t* off, char* base, const WsLayout& L, bool nocol) {
  hipStream_t st = h->stream;
  bf16_t* xT = BF(L.xT);  // channels-last bf16 x: K1, K5 and the offset conv read it
  float *off32 = F32(L.off32), *out32 = F32(L.out32);
  // f3: the offset conv stages its windows from the NCHW x and writes xT itself (one pass
  // over x, no transpose launch) wherever its row kernel applies with stride 1
  const bool fold = dcn::offset_fwd_bf16_fold_ok(g) && !dcn::get_force_generic();
  const bool off_mfma = fold || dcn::offset_fwd_mfma_bf16_ok(g);
  const bool fused_ok = dcn::fused_fwd_bf16_ok(g) && !dcn::get_force_generic();
  const bool fused = fused_ok && (h->fwd_path == DCN_FWD_FUSED || nocol ||
                                  (h->fwd_path == DCN_FWD_AUTO && dcn::fused_fwd_bf16_pays(g)));
  {
    // one launch for the fp32 biases and the weight re-layouts of the MFMA kernels below
    dcn::PrepBatch pb;
    pb.f32(b_off, F32(L.boff32), (size_t)g.J);
    if (has_bias) pb.f32(b, F32(L.b32), (size_t)g.O);
    if (off_mfma) pb.add(dcn::prep_tjc(g, w_off, BF(L.wb16)));
    if (fused) pb.add(dcn::prep_frag16(g, w, BF(L.wfr)));
    HIP_TRY(dcn::launch_prep_bf16(pb, st));
  }
  if (!fold) {
    ProfScope ps(h, DCN_K_XPOSE);
    HIP_TRY(dcn::launch_nchw_to_nhwc_bf16(x, xT, g.B, g.C, g.HWi, st));
  }
  {
    ProfScope ps(h, DCN_K_OFFSET_FWD);
    if (fold) {
      HIP_TRY(dcn::launch_offset_conv_fwd_bf16(g, xT, w_off, F32(L.boff32), off32, off,
                                               BF(L.wb16), st, x, true));
    } else if (off_mfma) {
      // bf16 MFMA straight from the bf16 xT: the offsets, rounded to bf16 (off) and as
      // fp32 values (off32, what the sampling uses)
      HIP_TRY(dcn::launch_offset_conv_fwd_bf16(g, xT, w_off, F32(L.boff32), off32, off,
                                               BF(L.wb16), st, nullptr, true));
    } else {  // fp32 VALU kernels on an fp32 copy of x
      float* x32 = F32(L.x32);
      HIP_TRY(dcn::launch_bf16_to_f32(x, x32, (size_t)g.B * g.C * g.HWi, st));
      HIP_TRY(dcn::launch_bf16_to_f32(w_off, F32(L.woff32), (size_t)g.J * g.C * g.N, st));
      HIP_TRY(dcn::launch_offset_conv_fwd(g, x32, F32(L.woff32), F32(L.boff32), off32, F32(L.wt),
                                          F32(L.part), st));
      HIP_TRY(dcn::launch_round_to_bf16(off32, off, (size_t)g.B * g.J * g.HW, st));
    }
  }
  // this workspace holds this forward's columns unless it runs without them
  ws_mark_columns(h, base, !nocol);
  if (fused) {
    // f2: the bilinear gather feeds the bf16 MFMAs straight from an LDS window of xT; bias
    // and the bf16 rounding in the epilogue; the columns are written only for a backward
    // that reuses them (not for DCN_FWD_FUSED_NOCOL)
    ProfScope ps(h, DCN_K_GEMM_FWD);
    HIP_TRY(dcn::launch_fused_fwd_bf16(g, xT, off32, w, BF(L.wfr),
                                       has_bias ? F32(L.b32) : nullptr, out,
                                       nocol ? nullptr : BF(L.col), st, true));
    return DCN_OK;
  }
  {
    ProfScope ps(h, DCN_K_IM2COL);
    HIP_TRY(dcn::launch_im2col_bf16(g, xT, off32, BF(L.col), 0, g.B, st));
  }
  {
    ProfScope ps(h, DCN_K_GEMM_FWD);  // C(HW×O) = colT_bᵀ · Wf, bf16 operands, fp32 out
    dcn::GemmSpec sp;
    sp.ta = true;
    sp.m = g.HW; sp.n = g.O; sp.k = g.K;
    sp.lda = g.K; sp.sa = (long)g.K * g.HW;
    sp.ldb = g.K; sp.sb = 0;
    sp.ldc = g.HW; sp.sc = (long)g.O * g.HW;
    sp.batch = g.B;
    sp.bf16_ab = true;
    GEMM_TRY(h, sp, BF(L.col), w, out32);
  }
  ProfScope ps(h, DCN_K_BIAS_FWD);
  HIP_TRY(dcn::launch_bias_to_bf16(g, out32, has_bias ? F32(L.b32) : nullptr, out, st));
  return DCN_OK;
}

int backward_bf16(dcn_handle* h, const Geo& g, bool has_bias, const bf16_t* x, const bf16_t* off,
                  const bf16_t* w_off, const bf16_t* w, const bf16_t* gout, bf16_t* gx,
                  bf16_t* gw, bf16_t* gb, bf16_t* gw_off, bf16_t* gb_off, bf16_t* goff_out,
                  char* base, const WsLayout& L, bool col_valid) {
  hipStream_t st = h->stream;
  bf16_t* xT = BF(L.xT);
  float *off32 = F32(L.off32), *goff32 = F32(L.goff32);
  float* gx32 = F32(L.gx32);
  bf16_t* col = BF(L.col);
  const size_t nx = (size_t)g.B * g.C * g.HWi, noff = (size_t)g.B * g.J * g.HW;
  const size_t nwo = (size_t)g.J * g.C * g.N;
  const long npix = (long)g.B * g.HW;
  const bool off_mfma = dcn::offset_bwd_bf16_ok(g);
  const bool dcol_k = !h->dcol_gemm && dcn::dcol_bf16_ok(g.K, g.O, npix) &&
                      !dcn::get_force_generic();
  // the sample bins (K5's input) on the side stream. (r06 A/B at config 4: the sort's 64
  // workgroups hold 100 KiB of LDS each and keep ≈60 of dw_stream_bf16's 252 one-per-CU
  // workgroups waiting ≈25 µs; launched after ∂W instead, beside the ∂col product, ∂W's scope
  // went 0.101 -> 0.096 ms but ∂col's 0.079 -> 0.106 ms.) With the forward's columns in the
  // workspace, its fp32 offsets are there too (every bf16 forward leaves off32 = the rounded
  // offsets it sampled with), so the sort starts before the prep and the ∂out transpose
  // instead of after them, and ends that much earlier into ∂W.
  if (col_valid) {
    DCN_TRY(fork_aux(h));
    HIP_TRY(dcn::launch_bins(g, off32, base + L.bins, goff32, 0, g.B, h->aux));
  }
  {
    // one launch: the fp32 offsets (== the forward's rounded ones) unless the forward left
    // them, and the weights in the layouts of the kernels below (fp32 w_off only for the
    // non-MFMA offset-conv paths)
    dcn::PrepBatch pb;
    if (!col_valid) pb.f32(off, off32, noff);
    if (off_mfma)
      pb.add(dcn::prep_ck(g, w_off, BF(L.wb16)));
    else
      pb.f32(w_off, F32(L.woff32), nwo);
    if (dcol_k) pb.add(dcn::prep_dcol(g.K, w, BF(L.wz)));
    HIP_TRY(dcn::launch_prep_bf16(pb, st));
  }
  if (!col_valid) {
    DCN_TRY(fork_aux(h));
    HIP_TRY(dcn::launch_bins(g, off32, base + L.bins, goff32, 0, g.B, h->aux));
  }
  // f2 without a column matrix (DCN_FWD_FUSED_NOCOL): ∂W with the columns recomputed from
  // xT inside the MFMA kernel, so the ∂columns are the only large buffer of the step
  const bool dw_fused = !col_valid && h->fwd_path == DCN_FWD_FUSED_NOCOL &&
                        dcn::fused_dw_bf16_ok(g) && !dcn::get_force_generic();
  if (!col_valid) {
    {
      ProfScope ps(h, DCN_K_XPOSE);
      HIP_TRY(dcn::launch_nchw_to_nhwc_bf16(x, xT, g.B, g.C, g.HWi, st));
    }
    if (!dw_fused) {
      ProfScope ps(h, DCN_K_IM2COL);
      HIP_TRY(dcn::launch_im2col_bf16(g, xT, off32, col, 0, g.B, st));
    }
  }
  const bool exch = h->comm != nullptr;  // sum the fp32 copies over ranks, then round
  bf16_t* goutT = BF(L.goutT);
  bool have_goutT = false;  // ∂outT (shared by the ∂W kernels and the ∂col product)
  if (has_bias) {
    ProfScope ps(h, DCN_K_BWD_BIAS);  // Σ over images and pixels of the bf16 ∂out, in fp32
    // with ∂outT from the same pass where the 16-byte transpose applies (tile partials in
    // gxT, which only K5 writes, after this)
    if (dcn::xpose_chsum_bf16_floats(g.B, g.O, g.HW) <= (size_t)g.B * g.HWi * g.C &&
        dcn::launch_xpose_chsum_bf16(gout, goutT, F32(L.gxT), F32(L.gb32), exch ? nullptr : gb,
                                     g.B, g.O, g.HW, st, h->aux,
                                     h->fork_ev)) {
      HIP_TRY(hipGetLastError());
      have_goutT = true;
    } else {
      dcn::launch_channel_sum_bf16(gout, g.B, g.O, g.HW, F32(L.gb32), st, exch ? nullptr : gb);
    }
  }
  // what K5 waits for on the side stream: the bins and the ∂b fold (issued above)
  HIP_TRY(hipEventRecord(h->k5_ev, h->aux));
  // ∂W over the stored (or just recomputed) columns: the streaming MFMA kernel where it
  // applies (O = 256, K % 256 == 0: config 4), else the vendor GEMM (grouped where B allows)
  const bool dw_stream = !dw_fused && !h->dw_gemm && dw_stream_applies(g) &&
                         !dcn::get_force_generic();
  const int dwg = dw_fused || dw_stream ? 0 : dw_groups(g);
  {
    ProfScope ps(h, DCN_K_GEMM_DW);
    dcn::GemmSpec sp;
    sp.bf16_ab = true;
    const int nparts = dw_fused    ? dcn::fused_dw_bf16_groups(g)
                       : dw_stream ? dcn::dw_stream_bf16_ranges(g.K, npix)
                       : dwg > 0   ? dwg
                                   : g.B;
    if (nparts > L.parts_planes)  // the ∂W kernels below write nparts planes into `parts`
      return fail(DCN_ERR_WORKSPACE, "∂W partials: " + std::to_string(nparts) +
                                         " planes, the workspace layout holds " +
                                         std::to_string(L.parts_planes));
    if (dw_fused) {
      HIP_TRY(dcn::launch_fused_dw_bf16(g, xT, off32, gout, F32(L.parts), st));
    } else if (dw_stream) {
      if (!have_goutT) HIP_TRY(dcn::launch_nchw_to_nhwc_bf16(gout, goutT, g.B, g.O, g.HW, st));
      have_goutT = true;
      HIP_TRY(dcn::launch_dw_stream_bf16(goutT, col, F32(L.parts), g.K, g.O, npix, st));
    } else if (dwg > 0) {
      // grouped NT over the pixels of B/dwg images (∂outT first, shared with ∂col)
      if (!have_goutT) HIP_TRY(dcn::launch_nchw_to_nhwc_bf16(gout, goutT, g.B, g.O, g.HW, st));
      have_goutT = true;
      const int pg = (g.B / dwg) * g.HW;
      sp.tb = true;
      sp.m = g.K; sp.n = g.O; sp.k = pg;
      sp.lda = g.K; sp.sa = (long)g.K * pg;
      sp.ldb = g.O; sp.sb = (long)g.O * pg;
      sp.ldc = g.K; sp.sc = (long)g.K * g.O;
      sp.batch = dwg;
      GEMM_TRY(h, sp, col, goutT, F32(L.parts));
    } else {  // P_b(K×O) = colT_b · ∂out_b (NN), bf16 in, fp32 out
      sp.m = g.K; sp.n = g.O; sp.k = g.HW;
      sp.lda = g.K; sp.sa = (long)g.K * g.HW;
      sp.ldb = g.HW; sp.sb = (long)g.O * g.HW;
      sp.ldc = g.K; sp.sc = (long)g.K * g.O;
      sp.batch = g.B;
      GEMM_TRY(h, sp, col, gout, F32(L.parts));
    }
    // the partial-plane sum on the side stream, beside ∂col (it reads 66 MB at config 4;
    // ∂col is bound by its stores). The side stream's join at the end of the backward and
    // dw_final's dw_aux event order it before everything that reads ∂W.
    DCN_TRY(fork_aux(h));
    HIP_TRY(dcn::launch_sum_partials(F32(L.parts), nparts, (size_t)g.K * g.O, F32(L.gw32), h->aux,
                                     exch ? nullptr : gw));
  }
  DCN_TRY(dw_final(h, F32(L.gw32), has_bias ? F32(L.gb32) : nullptr, g, exch ? gw : nullptr,
                   exch && has_bias ? gb : nullptr));
  {
    ProfScope ps(h, DCN_K_GEMM_DCOL);  // ∂colT = ∂outT · Wf over the whole batch, bf16 out
    if (!have_goutT) HIP_TRY(dcn::launch_nchw_to_nhwc_bf16(gout, goutT, g.B, g.O, g.HW, st));
    if (dcol_k) {
      // short-K streaming kernel (csrc/dcn_dcol_bf16.hip) on the Wf swizzled by the prep
      // launch (r04: the swizzle on the side stream beside ∂W cost that 10 µs, dcol5)
      HIP_TRY(dcn::launch_dcol_bf16(BF(L.wz), goutT, col, g.K, g.O, npix, st));
    } else {
      dcn::GemmSpec sp;
      sp.m = g.K; sp.n = g.B * g.HW; sp.k = g.O;
      sp.lda = g.K; sp.ldb = g.O; sp.ldc = g.K;
      sp.bf16_ab = sp.bf16_c = true;
      GEMM_TRY(h, sp, w, goutT, col);
    }
  }
  // K5 needs the bins (and the ∂b fold done reading its tile sums in gxT, which K5
  // overwrites): wait for the side-stream work up to k5_ev only. The ∂W partial sum issued
  // after it is joined at the end; it has long finished by then, while a join here waited
  // for it to end beside dcol_bf16 and then ≈11 µs more (r06 kernel trace at config 4).
  HIP_TRY(hipStreamWaitEvent(st, h->k5_ev, 0));
  {
    ProfScope ps(h, DCN_K_COL2IM);
    HIP_TRY(dcn::launch_col2im_bf16(g, xT, off32, col, nullptr, F32(L.gxT), goff32, base + L.bins, 0,
                                    g.B, true, st));
  }
  ProfScope ps(h, DCN_K_OFFSET_BWD);
  if (off_mfma) {
    // bf16 MFMA: bf16 x and w_off, the fp32 ∂offset split into two bf16 planes; writes the
    // bf16 grad_x directly (transpose of the sampling route + the offset-conv route)
    HIP_TRY(dcn::launch_offset_conv_bwd_bf16(g, x, w_off, goff32, F32(L.gxT), BF(L.wb16),
                                             F32(L.goffT), gx, F32(L.gwo32), F32(L.gbo32), st,
#if OFFB_CONC
                                             h->aux, h->fork_ev, h->join_ev,
#else
                                             nullptr, nullptr, nullptr,
#endif
                                             true, F32(L.part)));
    // (r02: the Wc swizzle and ∂b_off sums on the side stream beside ∂W_off measured slower,
    // offset bwd 0.115 -> 0.121 ms at config 4: concurrent kernels slow each other; r05: the
    // ∂x kernel there beside ∂W_off is faster, 0.0914-0.092 -> 0.0896-0.0901 ms, OFFB_CONC)
  } else if (dcn::offset_bwd_chunkable(g)) {
    // f32 MFMA on the bf16 xT (exact products of the bf16 values) and the fp32 ∂offset
    HIP_TRY(dcn::launch_offset_bwd_prep(g, F32(L.woff32), F32(L.wt), st));
    HIP_TRY(dcn::launch_offset_bwd_chunk(g, xT, true, goff32, F32(L.goffT), F32(L.wt), gx32,
                                         F32(L.gxT), 0, g.B, st));
    HIP_TRY(dcn::launch_offset_bwd_finish(g, goff32, F32(L.goffT), F32(L.gwo32), F32(L.gbo32), st));
  } else {  // VALU / generic kernels on fp32 copies of x (NCHW and channels-last)
    float *x32 = F32(L.x32), *xT32 = F32(L.xT32);
    HIP_TRY(dcn::launch_bf16_to_f32(x, x32, nx, st));
    HIP_TRY(dcn::launch_nchw_to_nhwc(x32, xT32, g.B, g.C, g.HWi, st));
    HIP_TRY(dcn::launch_offset_conv_bwd(g, x32, xT32, F32(L.woff32), goff32, F32(L.goffT),
                                        F32(L.wt), gx32, F32(L.gwo32), F32(L.gbo32), F32(L.gxT),
                                        st));
  }
  // everything on the side stream before the results (the MFMA offset backward with its
  // side stream already ends with that join)
  if (!(off_mfma && OFFB_CONC)) DCN_TRY(join_aux(h));
  // the bf16 results, one launch (the offset-conv parameter grads after the exchange when
  // there is one)
  dcn::ConvBatch cb;
  if (!off_mfma) cb.add(gx32, gx, nx, true);
  if (goff_out) cb.add(goff32, goff_out, noff, true);
  if (!exch) {
    cb.add(F32(L.gwo32), gw_off, nwo, true);
    cb.add(F32(L.gbo32), gb_off, (size_t)g.J, true);
  }
  HIP_TRY(dcn::launch_convert_multi(cb, st));
  if (exch) return grads_final(h, F32(L.gwo32), F32(L.gbo32), g, gw_off, gb_off);
  return DCN_OK;
}
#undef BF
#undef F32

int ensure_scratch(dcn_handle* h, size_t bytes) {
  if (h->scratch_bytes >= bytes) return DCN_OK;
  if (h->scratch) {
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipFree(h->scratch));
  }
  h->scratch = nullptr;
  h->scratch_bytes = 0;
  HIP_TRY(hipMalloc(&h->scratch, bytes));
  h->scratch_bytes = bytes;
  return DCN_OK;
}

}  // namespace

extern "C" {

int dcn_abi_version(void) { return DCN_ABI_VERSION; }

const char* dcn_last_error(void) { return g_err.c_str(); }

int dcn_device_count(int* n) {
  if (!n) return fail(DCN_ERR_INVALID, "null out pointer");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return fail(DCN_ERR_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *n = c;
  return DCN_OK;
}

int dcn_create(int device, dcn_handle** out) {
  if (!out) return fail(DCN_ERR_INVALID, "null out pointer");
  *out = nullptr;
  int n = 0;
  DCN_TRY(dcn_device_count(&n));
  if (device < 0 || device >= n) return fail(DCN_ERR_INVALID, "device index out of range");
  dcn_handle* h = new dcn_handle();
  h->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    return fail(DCN_ERR_HIP, std::string("dcn_create: ") + hipGetErrorString(e));
  }
  h->stream = h->own;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking);
  // the handle's own stream-to-stream events (main <-> side stream, one device): no
  // system-scope fence at record / wait (r06: each cost a 6-7 µs gap on the main queue).
  // The events that hand ∂W to the RCCL stream or the caller's grad stream keep it.
  const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->fork_ev, evf);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->join_ev, evf);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->k5_ev, evf);
  for (hipEvent_t* ev : {&h->dw_main, &h->dw_aux, &h->end_ev, &h->comm_done})
    if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->comm_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    dcn_destroy(h);
    return fail(DCN_ERR_HIP, std::string("dcn_create: ") + hipGetErrorString(e));
  }
  if (const char* f = std::getenv("DCN_DCOL_GEMM")) h->dcol_gemm = std::atoi(f) != 0;
  if (const char* f = std::getenv("DCN_DW_GEMM")) h->dw_gemm = std::atoi(f) != 0;
  std::string gerr;
  if (dcn::gemm_engine_create(&h->gemm, &gerr) != 0) {
    (void)hipStreamDestroy(h->own);
    delete h;
    return fail(DCN_ERR_BLAS, gerr);
  }
  *out = h;
  return DCN_OK;
}

int dcn_destroy(dcn_handle* h) {
  if (!h) return DCN_OK;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->stream);
  if (h->comm) dcn_internal_handle_drop_comm(h);
  for (auto& v : h->ev)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  if (h->scratch) (void)hipFree(h->scratch);
  for (void* p : h->hbuf)
    if (p) (void)hipFree(p);
  // the caller's states stay valid objects that only dcn_host_state_destroy accepts
  for (dcn_host_state* s : h->states) {
    state_free(s);
    s->h = nullptr;
  }
  if (h->hs0) {
    state_free(h->hs0);
    delete h->hs0;
  }
  for (hipEvent_t e : h->hev) (void)hipEventDestroy(e);
  for (hipStream_t s : {h->cin, h->cout})
    if (s) (void)hipStreamDestroy(s);
  delete h->stage;
  if (h->aux) (void)hipStreamSynchronize(h->aux);
  dcn::gemm_engine_destroy(h->gemm);
  if (h->fork_ev) (void)hipEventDestroy(h->fork_ev);
  if (h->join_ev) (void)hipEventDestroy(h->join_ev);
  for (hipEvent_t ev : {h->dw_main, h->dw_aux, h->end_ev, h->comm_done, h->k5_ev})
    if (ev) (void)hipEventDestroy(ev);
  if (h->comm_stream) {
    (void)hipStreamSynchronize(h->comm_stream);
    (void)hipStreamDestroy(h->comm_stream);
  }
  if (h->aux) (void)hipStreamDestroy(h->aux);
  if (h->own) (void)hipStreamDestroy(h->own);
  delete h;
  return DCN_OK;
}

int dcn_set_stream(dcn_handle* h, void* s) {
  DCN_TRY(set_device(h));
  h->stream = reinterpret_cast<hipStream_t>(s);  // NULL = the HIP null stream
  return DCN_OK;
}

int dcn_use_own_stream(dcn_handle* h) {
  DCN_TRY(set_device(h));
  h->stream = h->own;
  return DCN_OK;
}

int dcn_get_stream(dcn_handle* h, void** s) {
  if (!h || !s) return fail(DCN_ERR_INVALID, "null argument");
  *s = h->stream;
  return DCN_OK;
}

int dcn_synchronize(dcn_handle* h) {
  DCN_TRY(set_device(h));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int dcn_malloc(dcn_handle* h, size_t bytes, void** ptr) {
  if (!ptr) return fail(DCN_ERR_INVALID, "null out pointer");
  DCN_TRY(set_device(h));
  HIP_TRY(hipMalloc(ptr, bytes ? bytes : 1));
  return DCN_OK;
}

int dcn_free(dcn_handle* h, void* ptr) {
  DCN_TRY(set_device(h));
  if (ptr) HIP_TRY(hipFree(ptr));
  return DCN_OK;
}

int dcn_host_alloc(dcn_handle* h, size_t bytes, void** ptr) {
  if (!ptr) return fail(DCN_ERR_INVALID, "null out pointer");
  *ptr = nullptr;
  DCN_TRY(set_device(h));
  HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
  return DCN_OK;
}

int dcn_host_free(void* ptr) {
  if (ptr) HIP_TRY(hipHostFree(ptr));
  return DCN_OK;
}

int dcn_memcpy_h2d(dcn_handle* h, void* dst, const void* src, size_t bytes) {
  DCN_TRY(set_device(h));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int dcn_memcpy_d2h(dcn_handle* h, void* dst, const void* src, size_t bytes) {
  DCN_TRY(set_device(h));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int dcn_memset_zero(dcn_handle* h, void* dst, size_t bytes) {
  DCN_TRY(set_device(h));
  HIP_TRY(hipMemsetAsync(dst, 0, bytes, h->stream));
  return DCN_OK;
}

int dcn_out_shape(const dcn_desc* d, int* Ho, int* Wo) {
  Geo g;
  DCN_TRY(make_geo(d, &g));
  if (Ho) *Ho = g.Ho;
  if (Wo) *Wo = g.Wo;
  return DCN_OK;
}

int dcn_workspace_bytes(const dcn_desc* d, int with_backward, size_t* bytes) {
  if (!bytes) return fail(DCN_ERR_INVALID, "null out pointer");
  Geo g;
  DCN_TRY(make_geo(d, &g));
  if (with_backward < 0 || with_backward > DCN_WS_FORWARD_NO_COLUMNS)
    return fail(DCN_ERR_INVALID, "dcn_workspace_bytes: with_backward must be 0, 1 or 2");
  // DCN_WS_FORWARD_NO_COLUMNS: no col region where the forward skips the columns (DCN_BF16
  // fused geometries); elsewhere the forward writes them and needs the forward layout
  const bool cols = !(with_backward == DCN_WS_FORWARD_NO_COLUMNS && fwd_can_skip_columns(g));
  *bytes = ws_layout(g, with_backward == 1, cols).total;
  return DCN_OK;
}

int dcn_offset_conv_fwd(dcn_handle* h, const dcn_desc* d, const float* x, const float* w_off,
                        const float* b_off, float* off) {
  Geo g;
  DCN_TRY(make_geo_f32(d, &g));
  DCN_TRY(set_device(h));
  const size_t wbytes = align_up(dcn::offset_conv_wt_floats(g) * sizeof(float), 256);
  DCN_TRY(ensure_scratch(h, wbytes + dcn::offset_conv_fpart_floats(g) * sizeof(float)));
  char* sc = static_cast<char*>(h->scratch);
  ProfScope ps(h, DCN_K_OFFSET_FWD);
  HIP_TRY(dcn::launch_offset_conv_fwd(g, x, w_off, b_off, off, reinterpret_cast<float*>(sc),
                                      reinterpret_cast<float*>(sc + wbytes), h->stream));
  return DCN_OK;
}

int dcn_offset_conv_bwd(dcn_handle* h, const dcn_desc* d, const float* x, const float* w_off,
                        const float* grad_off, float* grad_x, float* grad_w_off,
                        float* grad_b_off) {
  Geo g;
  DCN_TRY(make_geo_f32(d, &g));
  DCN_TRY(set_device(h));
  const size_t xbytes = align_up((size_t)g.B * g.HWi * g.C * sizeof(float), 256);
  const size_t gbytes = align_up(dcn::offset_conv_goffT_floats(g) * sizeof(float), 256);
  DCN_TRY(ensure_scratch(h, xbytes + gbytes + dcn::offset_conv_wt_floats(g) * sizeof(float)));
  char* sc = static_cast<char*>(h->scratch);
  float* xT = reinterpret_cast<float*>(sc);
  float* goffT = reinterpret_cast<float*>(sc + xbytes);
  float* wt2 = reinterpret_cast<float*>(sc + xbytes + gbytes);
  ProfScope ps(h, DCN_K_OFFSET_BWD);
  HIP_TRY(dcn::launch_nchw_to_nhwc(x, xT, g.B, g.C, g.HWi, h->stream));
  HIP_TRY(dcn::launch_offset_conv_bwd(g, x, xT, w_off, grad_off, goffT, wt2, grad_x, grad_w_off,
                                      grad_b_off, nullptr, h->stream));
  return DCN_OK;
}

int dcn_im2col_fwd(dcn_handle* h, const dcn_desc* d, const float* x, const float* off,
                   float* col, int b0, int nb) {
  Geo g;
  DCN_TRY(make_geo_f32(d, &g));
  DCN_TRY(set_device(h));
  if (b0 < 0 || nb < 0 || b0 + nb > g.B) return fail(DCN_ERR_INVALID, "image range out of bounds");
  DCN_TRY(ensure_scratch(h, (size_t)g.B * g.HWi * g.C * sizeof(float)));
  float* xT = static_cast<float*>(h->scratch);
  ProfScope ps(h, DCN_K_IM2COL);
  HIP_TRY(dcn::launch_nchw_to_nhwc(x + (size_t)b0 * g.C * g.HWi, xT + (size_t)b0 * g.HWi * g.C, nb,
                                   g.C, g.HWi, h->stream));
  HIP_TRY(dcn::launch_im2col(g, x, xT, off, col, b0, nb, h->stream));
  return DCN_OK;
}

int dcn_col2im_coord_bwd(dcn_handle* h, const dcn_desc* d, const float* x, const float* off,
                         const float* grad_col, float* grad_x, float* grad_off, int b0, int nb) {
  Geo g;
  DCN_TRY(make_geo_f32(d, &g));
  DCN_TRY(set_device(h));
  if (b0 < 0 || nb < 0 || b0 + nb > g.B) return fail(DCN_ERR_INVALID, "image range out of bounds");
  const size_t xbytes = align_up((size_t)g.B * g.HWi * g.C * sizeof(float), 256);
  DCN_TRY(ensure_scratch(h, 2 * xbytes + dcn::bins_ws_bytes(g, nb)));
  char* sc = static_cast<char*>(h->scratch);
  float* xT = reinterpret_cast<float*>(sc);
  float* gxT = reinterpret_cast<float*>(sc + xbytes);
  void* bins = sc + 2 * xbytes;
  ProfScope ps(h, DCN_K_COL2IM);
  HIP_TRY(dcn::launch_nchw_to_nhwc(x + (size_t)b0 * g.C * g.HWi, xT + (size_t)b0 * g.HWi * g.C, nb,
                                   g.C, g.HWi, h->stream));
  HIP_TRY(dcn::launch_col2im_coord(g, x, xT, off, grad_col, grad_x, gxT, grad_off, bins, b0, nb, false,
                                   h->stream));
  return DCN_OK;
}

namespace {
// r05: the fp32 offset conv as GEMMs (dcn::offset_conv_gemm_ok geometries that have no MFMA
// offset-conv kernel; dcn_debug_offset_gemm(0) keeps the VALU kernels, for the parity tests)
int g_ocg = 1;
bool ocg_on(const Geo& g) {
  return g_ocg && !dcn::offset_fwd_mfma_xt_ok(g) && !dcn::offset_bwd_chunkable(g) &&
         dcn::offset_conv_gemm_ok(g) && !dcn::get_force_generic();
}
// off[B][J][HW] from xT; wp: J·K floats, ocol: B·HW·K floats, offT: B·HW·J floats
int offset_conv_fwd_gemm(dcn_handle* h, const Geo& g, const float* xT, const float* w_off,
                         const float* b_off, float* off, float* wp, float* ocol, float* offT) {
  const int K = g.C * g.kh * g.kw, P = g.B * g.HW;
  HIP_TRY(dcn::launch_ocg_wprime(g, w_off, wp, h->stream));
  HIP_TRY(dcn::launch_ocg_im2col(g, xT, ocol, h->stream));
  // column-major offT(J × P) = W'ᵀ(J × K) · ocol(K × P)   (W' = [J][K], ocol = [P][K])
  dcn::GemmSpec sp;
  sp.ta = true;
  sp.m = g.J; sp.n = P; sp.k = K;
  sp.lda = K; sp.ldb = K; sp.ldc = g.J;
  sp.native_f32 = true;
  GEMM_TRY(h, sp, wp, ocol, offT);
  HIP_TRY(dcn::launch_ocg_offt_to_off(g, offT, b_off, off, h->stream));
  return DCN_OK;
}
// ∂w_off and ∂x (= transpose(gxT_in) + the offset route) from ∂off; wp: J·K floats,
// ocol: B·HW·K floats (ocol, then ∂ocol), goffT: B·HW·J floats, gwp: J·K floats
// ocol_fwd: the forward's im2col (and its W' in wp) when still in the workspace, else null
// (both recomputed, the im2col into ocol)
int offset_conv_bwd_gemm(dcn_handle* h, const Geo& g, const float* xT, const float* w_off,
                         const float* goff, float* wp, float* ocol, float* goffT, float* gwp,
                         const float* gxT_in, float* gx, float* gw_off, const float* ocol_fwd) {
  const int K = g.C * g.kh * g.kw, P = g.B * g.HW;
  if (!ocol_fwd) {
    HIP_TRY(dcn::launch_ocg_wprime(g, w_off, wp, h->stream));
    HIP_TRY(dcn::launch_ocg_im2col(g, xT, ocol, h->stream));
  }
  const float* ocol_in = ocol_fwd ? ocol_fwd : ocol;
  HIP_TRY(dcn::launch_ocg_goff_to_pj(g, goff, goffT, h->stream));
  {
    // column-major ∂W'(K × J) = ocol(K × P) · ∂offT(P × J)   (∂offT = [P][J])
    dcn::GemmSpec sp;
    sp.tb = true;
    sp.m = K; sp.n = g.J; sp.k = P;
    sp.lda = K; sp.ldb = g.J; sp.ldc = K;
    sp.native_f32 = true;
    GEMM_TRY(h, sp, ocol_in, goffT, gwp);
  }
  HIP_TRY(dcn::launch_ocg_wgrad_out(g, gwp, gw_off, h->stream));
  {
    // column-major ∂ocol(K × P) = W'(K × J) · ∂offTᵀ(J × P), over the columns just read
    dcn::GemmSpec sp;
    sp.m = K; sp.n = P; sp.k = g.J;
    sp.lda = K; sp.ldb = g.J; sp.ldc = K;
    sp.native_f32 = true;
    GEMM_TRY(h, sp, wp, goffT, ocol);
  }
  HIP_TRY(dcn::launch_ocg_col2im(g, ocol, gxT_in, gx, h->stream));
  return DCN_OK;
}
}  // namespace

int dcn_forward(dcn_handle* h, const dcn_desc* d, const float* x, const float* w_off,
                const float* b_off, const float* w, const float* b, float* out, float* off,
                void* ws, size_t ws_bytes) {
  return dcn_forward_ex(h, d, x, w_off, b_off, w, b, out, off, ws, ws_bytes, 0);
}

int dcn_forward_ex(dcn_handle* h, const dcn_desc* d, const float* x, const float* w_off,
                   const float* b_off, const float* w, const float* b, float* out, float* off,
                   void* ws, size_t ws_bytes, int flags) {
  Geo g;
  DCN_TRY(make_geo(d, &g));
  DCN_TRY(set_device(h));
  if (flags & ~DCN_FWD_NO_COLUMNS) return fail(DCN_ERR_INVALID, "dcn_forward_ex: unknown flags");
  const bool nocol = fwd_skips_columns(h, g, flags);
  const WsLayout L = ws_layout(g, false, !nocol);
  if (!ws || ws_bytes < L.total) return fail(DCN_ERR_WORKSPACE, "workspace too small for dcn_forward");
  if (d->has_bias && !b) return fail(DCN_ERR_INVALID, "has_bias set but bias is NULL");
  char* base = static_cast<char*>(ws);
  // this forward overwrites whatever offset-conv im2col an earlier one left in ws
  ws_rec_mark(h, h->ocol_ws, ws, false);
  if (g.dt == DCN_BF16) {
    using dcn::bf16_t;
    return forward_bf16(h, g, d->has_bias != 0, reinterpret_cast<const bf16_t*>(x),
                        reinterpret_cast<const bf16_t*>(w_off),
                        reinterpret_cast<const bf16_t*>(b_off), reinterpret_cast<const bf16_t*>(w),
                        reinterpret_cast<const bf16_t*>(b), reinterpret_cast<bf16_t*>(out),
                        reinterpret_cast<bf16_t*>(off), base, L, nocol);
  }
  float* xT = reinterpret_cast<float*>(base + L.xT);
  if (dcn::offset_fwd_mfma_xt_ok(g)) {
    // offsets on the f32 matrix cores, writing xT from the same reads of x
    {
      ProfScope ps(h, DCN_K_OFFSET_FWD);
      HIP_TRY(dcn::launch_offset_conv_fwd_xt(g, x, w_off, b_off, off, xT,
                                             reinterpret_cast<float*>(base + L.wt), h->stream));
    }
    return core_forward(h, g, x, off, w, b, d->has_bias != 0, out, xT,
                        reinterpret_cast<float*>(base + L.col), true,
                        reinterpret_cast<float*>(base + L.fwdT));
  }
  if (ocg_on(g)) {
    // r05: the offset conv as one GEMM over its own im2col (config 5: C = 512, J = 72,
    // stride 2, dilation 2, where the VALU kernel ran at 0.06 of the f32 MFMA peak)
    {
      ProfScope ps(h, DCN_K_XPOSE);
      HIP_TRY(dcn::launch_nchw_to_nhwc(x, xT, g.B, g.C, g.HWi, h->stream));
    }
    {
      ProfScope ps(h, DCN_K_OFFSET_FWD);
      // ocol in its own region when the layout has one (kept for the backward), else in
      // the columns region, which K1 overwrites next
      DCN_TRY(offset_conv_fwd_gemm(h, g, xT, w_off, b_off, off,
                                   reinterpret_cast<float*>(base + L.wt),
                                   reinterpret_cast<float*>(base + (L.has_ocol ? L.ocol : L.col)),
                                   reinterpret_cast<float*>(base + L.part)));
      if (L.has_ocol) ws_rec_mark(h, h->ocol_ws, ws, true);
    }
    return core_forward(h, g, x, off, w, b, d->has_bias != 0, out, xT,
                        reinterpret_cast<float*>(base + L.col), true,
                        reinterpret_cast<float*>(base + L.fwdT));
  }
  // x -> channels-last on the side stream, beside the offset conv (both only read x)
  DCN_TRY(fork_aux(h));
  {
    ProfScope ps(h, DCN_K_XPOSE, h->aux);
    HIP_TRY(dcn::launch_nchw_to_nhwc(x, xT, g.B, g.C, g.HWi, h->aux));
  }
  {
    ProfScope ps(h, DCN_K_OFFSET_FWD);
    HIP_TRY(dcn::launch_offset_conv_fwd(g, x, w_off, b_off, off,
                                        reinterpret_cast<float*>(base + L.wt),
                                        reinterpret_cast<float*>(base + L.part), h->stream));
  }
  DCN_TRY(join_aux(h));
  return core_forward(h, g, x, off, w, b, d->has_bias != 0, out, xT,
                      reinterpret_cast<float*>(base + L.col), true,
                      reinterpret_cast<float*>(base + L.fwdT));
}

int dcn_backward(dcn_handle* h, const dcn_desc* d, const float* x, const float* off,
                 const float* w_off, const float* w, const float* grad_out, float* grad_x,
                 float* grad_w, float* grad_b, float* grad_w_off, float* grad_b_off,
                 float* grad_off_out, void* ws, size_t ws_bytes, int flags) {
  Geo g;
  DCN_TRY(make_geo(d, &g));
  DCN_TRY(set_device(h));
  const WsLayout L = ws_layout(g, true);
  if (!ws || ws_bytes < L.total) return fail(DCN_ERR_WORKSPACE, "workspace too small for dcn_backward");
  if (d->has_bias && !grad_b) return fail(DCN_ERR_INVALID, "has_bias set but grad_b is NULL");
  char* base = static_cast<char*>(ws);
  if (g.dt == DCN_BF16) {
    using dcn::bf16_t;
    auto C = [](const float* p) { return reinterpret_cast<const bf16_t*>(p); };
    auto M = [](float* p) { return reinterpret_cast<bf16_t*>(p); };
    // the columns are read only where this handle's last forward on this workspace wrote
    // them (not a DCN_FWD_FUSED_NOCOL / NO_COLUMNS forward); otherwise they are recomputed
    const bool col_valid = (flags & DCN_BWD_COL_IN_WS) != 0 && ws_has_columns(h, ws);
    return backward_bf16(h, g, d->has_bias != 0, C(x), C(off), C(w_off), C(w), C(grad_out),
                         M(grad_x), M(grad_w), M(grad_b), M(grad_w_off), M(grad_b_off),
                         M(grad_off_out), base, L, col_valid);
  }
  auto F = [&](size_t o) { return reinterpret_cast<float*>(base + o); };
  float* goff = grad_off_out ? grad_off_out : F(L.goff);
  DCN_TRY(core_backward(h, g, x, off, w, grad_out, grad_x, grad_w, grad_b, d->has_bias != 0, goff,
                        F(L.xT), F(L.col), F(L.parts), F(L.gxT), F(L.goutT), base + L.bins,
                        (flags & DCN_BWD_COL_IN_WS) != 0));
  {
    ProfScope ps(h, DCN_K_OFFSET_BWD);
    const bool ocg = ocg_on(g) && (size_t)g.J * g.K <= (size_t)g.B * g.HW * g.O;
    // ∂b_off = Σ ∂offset (18 channels: a latency-bound reduction), two-level over (channel,
    // image) blocks (one block per channel held 18 CUs for 0.11 ms). On the GEMM route it
    // runs on the side stream beside the offset-conv GEMMs. On the MFMA route (r06) it runs
    // on the main stream after ∂W_off's fold, before the ∂x join: there the side stream
    // carries the ∂x kernel, and with the sum queued ahead of it, ∂x ended 13 µs after the
    // fold, and the join then waited ≈15 µs more (profiles/r06i_timeline_config3.txt).
    const bool bsum_side = ocg;
    if (bsum_side) {
      DCN_TRY(fork_aux(h));
      dcn::launch_channel_sum_2l(goff, g.B, g.J, g.HW, F(L.part), grad_b_off, h->aux);
    }
    if (ocg) {
      // r05: ∂W_off and the offset route of ∂x as GEMMs over the offset conv's im2col (the
      // columns region is free after K5; ∂W' [J][K] in the ∂outT region, free after ∂col)
      // with the forward's im2col and W' still in ws (DCN_BWD_COL_IN_WS and this handle's
      // record), ∂W' reads them and the ∂ocol product goes to the free columns region
      const bool reuse = L.has_ocol && (flags & DCN_BWD_COL_IN_WS) != 0 &&
                         ws_rec_has(h, h->ocol_ws, ws);
      DCN_TRY(offset_conv_bwd_gemm(h, g, F(L.xT), w_off, goff, F(L.wt), F(L.col), F(L.goffT),
                                   F(L.goutT), F(L.gxT), grad_x, grad_w_off,
                                   reuse ? F(L.ocol) : nullptr));
    } else {
      // (∂b_off inside, on the main stream before its join, unless on the side stream above)
      HIP_TRY(dcn::launch_offset_conv_bwd(g, x, F(L.xT), w_off, goff, F(L.goffT), F(L.wt), grad_x,
                                          grad_w_off, bsum_side ? nullptr : grad_b_off,
                                          dcn::get_force_generic() ? nullptr : F(L.gxT),
                                          h->stream, OFFB_CONC_F32 ? h->aux : nullptr,
                                          h->fork_ev, h->join_ev, F(L.part)));
    }
    if (bsum_side) DCN_TRY(join_aux(h));
  }
  return grads_final(h, grad_w_off, grad_b_off, g);
}

// ---- host-pointer variants -----------------------------------------------------
// Persistent device copies (grow-only per role, no per-call hipMalloc/hipFree), transfers
// staged through the handle's pinned ring (dcn_host.h), and a backward that can reuse what
// its forward left on the device (DCN_HOST_REUSE_FWD: no x / offset / weight upload, no
// transpose or im2col recompute: the columns stay in the handle's workspace).
namespace {
// per-call device buffers (RoI pooling's host variants: small tensors)
struct DevBufs {
  std::vector<void*> ptrs;
  ~DevBufs() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  int alloc(size_t bytes, float** p) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 4);
    if (e != hipSuccess) return fail(DCN_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    ptrs.push_back(q);
    *p = static_cast<float*>(q);
    return DCN_OK;
  }
};

enum HostRole {
  HB_BO, HB_B, HB_OUT, HB_GO, HB_GX, HB_GPAR, HB_PART, HB_GOFF, HB_COUNT
};

int grow(dcn_handle* h, void** p, size_t* have, size_t bytes) {
  bytes = bytes ? bytes : 4;
  if (*have >= bytes) return DCN_OK;
  if (*p) {
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipFree(*p));
  }
  *p = nullptr;
  *have = 0;
  HIP_TRY(hipMalloc(p, bytes));
  *have = bytes;
  return DCN_OK;
}

int host_buf(dcn_handle* h, int role, size_t bytes, char** p) {
  DCN_TRY(grow(h, &h->hbuf[role], &h->hbuf_bytes[role], bytes));
  *p = static_cast<char*>(h->hbuf[role]);
  return DCN_OK;
}
}  // namespace

namespace {
void state_free(dcn_host_state* s) {
  for (void*& p : s->dev) {
    if (p) (void)hipFree(p);
    p = nullptr;
  }
  if (s->ws) (void)hipFree(s->ws);
  s->ws = nullptr;
  s->ws_bytes = 0;
  s->valid = false;
}

int state_buf(dcn_host_state* s, int role, size_t bytes, char** p) {
  DCN_TRY(grow(s->h, &s->dev[role], &s->dev_bytes[role], bytes));
  *p = static_cast<char*>(s->dev[role]);
  return DCN_OK;
}

int state_ws(dcn_host_state* s, size_t bytes) {
  if (s->ws_bytes < bytes) s->valid = false;  // the forward's columns go with the old workspace
  return grow(s->h, &s->ws, &s->ws_bytes, bytes);
}

// Transfers go straight from / to the caller's pageable memory by default: on the MI355X
// box that runs at 54 GB/s both ways when the host pages are resident (tools/pcie_probe.py;
// pinned: 57 GB/s), and the Python shim hands out recycled, resident output arrays
// (hostmem.py). A pageable copy blocks the calling thread until it is done, and an upload
// and a download do not run at the same time even pinned (tools/pcie_overlap.py: 205 MB
// each way, 3.6 ms alone, 7.3 ms together), while kernels queued before a copy keep running
// beside it (a 6.1 ms GEMM + both copies: 7.4 ms). DCN_HOST_STAGING=1 routes the copies
// through the pinned ring and copy threads instead (DCN_HOST_THREADS, default 8;
// DCN_HOST_CHUNK_MB, default 32): that pays only for destinations never touched before
// (page faults: 8.9 GB/s direct, 16 GB/s with 16 threads).
bool staging_on(dcn_handle* h) {
  if (h->staging < 0) {  // read once per handle, at its first host transfer
    const char* e = std::getenv("DCN_HOST_STAGING");
    h->staging = e && std::atoi(e) != 0 ? 1 : 0;
  }
  return h->staging != 0;
}
int get_stage(dcn_handle* h, dcn::HostStage** st) {
  if (!h->stage) {
    const char* t = std::getenv("DCN_HOST_THREADS");
    const char* c = std::getenv("DCN_HOST_CHUNK_MB");
    const int threads = t ? std::max(1, std::atoi(t)) : 8;
    const size_t chunk = (size_t)(c ? std::max(1, std::atoi(c)) : 32) << 20;
    auto* s = new dcn::HostStage(chunk, threads);
    const hipError_t e = s->init();
    if (e != hipSuccess) {
      delete s;
      return fail(DCN_ERR_HIP, std::string("pinned staging: ") + hipGetErrorString(e));
    }
    h->stage = s;
  }
  *st = h->stage;
  return DCN_OK;
}

int h2d(dcn_handle* h, hipStream_t s, void* dst, const void* src, size_t bytes) {
  if (!bytes) return DCN_OK;
  if (!staging_on(h)) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return DCN_OK;
  }
  dcn::HostStage* st;
  DCN_TRY(get_stage(h, &st));
  HIP_TRY(st->h2d(dst, src, bytes, s));
  return DCN_OK;
}
int d2h(dcn_handle* h, hipStream_t s, void* dst, const void* src, size_t bytes) {
  if (!bytes) return DCN_OK;
  if (!staging_on(h)) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    return DCN_OK;
  }
  dcn::HostStage* st;
  DCN_TRY(get_stage(h, &st));
  HIP_TRY(st->d2h(dst, src, bytes, s));
  return DCN_OK;
}

// ---- the image-chunk transfer pipeline -----------------------------------------
// The batch is cut into n image chunks. Chunk i's upload runs on the copy-in stream, its
// kernels on the handle's stream once that upload is done (event), its download on the
// copy-out stream once the kernels are done, so the kernels of chunk i run beside the
// copies of chunks i-1 and i+1: the step costs about the transfers alone plus one chunk's
// kernels, instead of transfers + kernels. Each chunk has its own workspace slice, which
// keeps that chunk's columns from the forward for the backward.
constexpr int kMaxHostChunks = 16;
// auto: about this much x per chunk. r03, config 3 (205 MB of x), fwd + bwd incl. PCIe,
// equal chunks: 1 chunk 23.4 ms, 2 17.2, 4 17.0, 8 18.1, 9 (24 MB) 17.9; half-size first
// and last chunks (make_plan): 3 16.5, 4 15.9, 5 16.4, 6 17.2
constexpr size_t kHostChunkBytes = size_t(52) << 20;

struct ChunkPlan {
  int n = 1;
  int b0[kMaxHostChunks + 1] = {0};
  size_t ws_off[kMaxHostChunks + 1] = {0};  // workspace slice of chunk i
  dcn_desc d[kMaxHostChunks];               // the chunk's descriptor (B = its images)
};

int chunk_count(const dcn_host_state* s, const Geo& g) {
  // bf16 parameter gradients would be summed over chunks in bf16 and a communicator would
  // all-reduce every chunk: both keep one chunk
  if (g.dt != DCN_F32 || s->h->comm) return 1;
  int n = s->chunks;
  if (n <= 0) {
    const size_t xb = (size_t)g.B * g.C * g.HWi * sizeof(float);
    n = (int)((xb + kHostChunkBytes - 1) / kHostChunkBytes);
  }
  return std::max(1, std::min(std::min(n, kMaxHostChunks), g.B));
}

// Chunk i spans images [b0[i], b0[i+1]). With 3 or more chunks the first and the last are
// half the size of the others: nothing overlaps the first chunk's upload or the last one's
// kernels and download, so those two are kept short.
int make_plan(const dcn_desc* d, const Geo& g, int n, ChunkPlan* P) {
  P->n = n;
  const long W2 = n >= 3 ? 2L * n - 2 : 2L * n;  // total weight in half units
  auto start = [&](int i) -> int {  // cumulative weight of chunks < i, in half units
    const long h = n >= 3 ? (i == 0 ? 0 : 2L * i - 1) : 2L * i;
    return (int)((long)g.B * std::min(h, W2) / W2);
  };
  for (int i = 0; i <= n; ++i) P->b0[i] = start(i);
  for (int i = 1; i <= n; ++i)  // every chunk at least one image (n <= B)
    P->b0[i] = std::max(P->b0[i], P->b0[i - 1] + 1);
  for (int i = n - 1; i >= 0; --i) P->b0[i] = std::min(P->b0[i], P->b0[i + 1] - 1);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    P->d[i] = *d;
    P->d[i].B = P->b0[i + 1] - P->b0[i];
    Geo gi;
    DCN_TRY(make_geo(&P->d[i], &gi));
    P->ws_off[i] = off;
    off += (ws_layout(gi, true).total + 255) & ~size_t(255);
  }
  P->ws_off[n] = off;
  return DCN_OK;
}

int pipeline_init(dcn_handle* h) {
  if (!h->cin) HIP_TRY(hipStreamCreateWithFlags(&h->cin, hipStreamNonBlocking));
  if (!h->cout) HIP_TRY(hipStreamCreateWithFlags(&h->cout, hipStreamNonBlocking));
  while (h->hev.size() < 2 * kMaxHostChunks) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    h->hev.push_back(e);
  }
  return DCN_OK;
}

// every exit of a pipelined call (errors included) leaves no copy in flight on the
// caller's memory
struct PipelineDrain {
  dcn_handle* h;
  ~PipelineDrain() {
    for (hipStream_t s : {h->cin, h->cout, h->stream}) (void)hipStreamSynchronize(s);
  }
};

// stream `s` waits for event slot k, recorded on stream `from` now
int hop(dcn_handle* h, int k, hipStream_t from, hipStream_t s) {
  HIP_TRY(hipEventRecord(h->hev[k], from));
  HIP_TRY(hipStreamWaitEvent(s, h->hev[k], 0));
  return DCN_OK;
}

int check_state(dcn_host_state* s) {
  if (!s) return fail(DCN_ERR_INVALID, "null host state");
  if (!s->h) return fail(DCN_ERR_INVALID, "host state of a destroyed handle");
  return set_device(s->h);
}

int forward_host(dcn_host_state* s, const dcn_desc* d, const float* x, const float* w_off,
                 const float* b_off, const float* w, const float* b, float* out, float* off) {
  DCN_TRY(check_state(s));
  dcn_handle* h = s->h;
  Geo g;
  DCN_TRY(make_geo(d, &g));
  if (!out) return fail(DCN_ERR_INVALID, "dcn_forward_host: out is required");
  s->valid = false;
  const size_t es = elem_bytes(g);
  const size_t xi = (size_t)g.C * g.HWi * es, oi = (size_t)g.O * g.HW * es;  // per image
  const size_t fi = (size_t)g.J * g.HW * es, nwo = (size_t)g.J * g.C * g.N * es;
  const size_t nw = (size_t)g.O * g.K * es;
  ChunkPlan P;
  DCN_TRY(make_plan(d, g, chunk_count(s, g), &P));
  char *dx, *doff, *dwo, *dw, *dbo, *db_ = nullptr, *dout;
  DCN_TRY(state_buf(s, SB_X, g.B * xi, &dx));
  DCN_TRY(state_buf(s, SB_OFF, g.B * fi, &doff));
  DCN_TRY(state_buf(s, SB_WO, nwo, &dwo));
  DCN_TRY(state_buf(s, SB_W, nw, &dw));
  DCN_TRY(host_buf(h, HB_BO, g.J * es, &dbo));
  if (d->has_bias) DCN_TRY(host_buf(h, HB_B, g.O * es, &db_));
  DCN_TRY(host_buf(h, HB_OUT, g.B * oi, &dout));
  DCN_TRY(state_ws(s, P.ws_off[P.n]));
  DCN_TRY(pipeline_init(h));
  PipelineDrain drain{h};
  DCN_TRY(h2d(h, h->stream, dwo, w_off, nwo));
  DCN_TRY(h2d(h, h->stream, dbo, b_off, g.J * es));
  DCN_TRY(h2d(h, h->stream, dw, w, nw));
  if (d->has_bias) DCN_TRY(h2d(h, h->stream, db_, b, g.O * es));
  // chunk i's download waits for the event recorded right after its kernels were queued
  // (not for whatever the stream holds by the time the download is issued)
  auto download = [&](int i) -> int {
    const size_t b0 = P.b0[i], nb = P.d[i].B;
    HIP_TRY(hipStreamWaitEvent(h->cout, h->hev[2 * i + 1], 0));
    DCN_TRY(d2h(h, h->cout, (char*)out + b0 * oi, dout + b0 * oi, nb * oi));
    if (off) DCN_TRY(d2h(h, h->cout, (char*)off + b0 * fi, doff + b0 * fi, nb * fi));
    return DCN_OK;
  };
  for (int i = 0; i < P.n; ++i) {
    const size_t b0 = P.b0[i], nb = P.d[i].B;
    DCN_TRY(h2d(h, h->cin, dx + b0 * xi, (const char*)x + b0 * xi, nb * xi));
    DCN_TRY(hop(h, 2 * i, h->cin, h->stream));
    DCN_TRY(dcn_forward(h, &P.d[i], (float*)(dx + b0 * xi), (float*)dwo, (float*)dbo,
                        (float*)dw, (float*)db_, (float*)(dout + b0 * oi),
                        (float*)(doff + b0 * fi), (char*)s->ws + P.ws_off[i],
                        P.ws_off[i + 1] - P.ws_off[i]));
    HIP_TRY(hipEventRecord(h->hev[2 * i + 1], h->stream));
    if (i > 0) DCN_TRY(download(i - 1));
  }
  DCN_TRY(download(P.n - 1));
  HIP_TRY(hipStreamSynchronize(h->cout));
  HIP_TRY(hipStreamSynchronize(h->stream));
  s->valid = true;
  s->plan_n = P.n;
  s->desc = *d;
  s->x = x, s->wo = w_off, s->w = w, s->off = off;
  return DCN_OK;
}

int backward_host(dcn_host_state* s, const dcn_desc* d, const float* x, const float* off,
                  const float* w_off, const float* w, const float* grad_out, float* grad_x,
                  float* grad_w, float* grad_b, float* grad_w_off, float* grad_b_off,
                  float* grad_off_out, int flags) {
  DCN_TRY(check_state(s));
  dcn_handle* h = s->h;
  Geo g;
  DCN_TRY(make_geo(d, &g));
  const bool reuse = (flags & DCN_HOST_REUSE_FWD) != 0;
  if (reuse) {
    if (!s->valid || std::memcmp(&s->desc, d, sizeof(dcn_desc)) != 0 || s->x != x ||
        s->wo != w_off || s->w != w || s->off != off)
      return fail(DCN_ERR_INVALID,
                  "DCN_HOST_REUSE_FWD: not the descriptor and x / off / w_off / w arrays of the "
                  "last forward on this host state");
  } else if (!off) {
    return fail(DCN_ERR_INVALID, "dcn_backward_host: off is required without DCN_HOST_REUSE_FWD");
  }
  const size_t es = elem_bytes(g);
  const size_t xi = (size_t)g.C * g.HWi * es, oi = (size_t)g.O * g.HW * es;
  const size_t fi = (size_t)g.J * g.HW * es;
  // ∂W, ∂b, ∂W_off, ∂b_off packed in one block (16-B aligned parts): the per-chunk partials
  // of a pipelined backward are summed in chunk order with one launch
  auto up4 = [](size_t n) { return (n + 3) & ~size_t(3); };
  const size_t nw = (size_t)g.O * g.K, nwo = (size_t)g.J * g.C * g.N;
  const size_t p_gw = 0, p_gb = up4(nw), p_gwo = p_gb + up4(g.O), p_gbo = p_gwo + up4(nwo);
  const size_t npar = p_gbo + up4(g.J);
  ChunkPlan P;
  DCN_TRY(make_plan(d, g, reuse ? s->plan_n : chunk_count(s, g), &P));
  char *dx, *doff, *dwo, *dw, *dgo, *dgx, *dgoff = nullptr, *gpar, *part = nullptr;
  DCN_TRY(state_buf(s, SB_X, g.B * xi, &dx));
  DCN_TRY(state_buf(s, SB_OFF, g.B * fi, &doff));
  DCN_TRY(state_buf(s, SB_WO, nwo * es, &dwo));
  DCN_TRY(state_buf(s, SB_W, nw * es, &dw));
  DCN_TRY(host_buf(h, HB_GO, g.B * oi, &dgo));
  DCN_TRY(host_buf(h, HB_GX, g.B * xi, &dgx));
  if (grad_off_out) DCN_TRY(host_buf(h, HB_GOFF, g.B * fi, &dgoff));
  DCN_TRY(host_buf(h, HB_GPAR, npar * es, &gpar));
  if (P.n > 1) DCN_TRY(host_buf(h, HB_PART, P.n * npar * sizeof(float), &part));
  if (!reuse) DCN_TRY(state_ws(s, P.ws_off[P.n]));
  DCN_TRY(pipeline_init(h));
  PipelineDrain drain{h};
  // the backward overwrites the columns with ∂columns: a second reuse needs a new forward
  s->valid = false;
  if (!reuse) {
    DCN_TRY(h2d(h, h->stream, dwo, w_off, nwo * es));
    DCN_TRY(h2d(h, h->stream, dw, w, nw * es));
  }
  auto download = [&](int i) -> int {  // as the forward's
    const size_t b0 = P.b0[i], nb = P.d[i].B;
    HIP_TRY(hipStreamWaitEvent(h->cout, h->hev[2 * i + 1], 0));
    DCN_TRY(d2h(h, h->cout, (char*)grad_x + b0 * xi, dgx + b0 * xi, nb * xi));
    if (grad_off_out)
      DCN_TRY(d2h(h, h->cout, (char*)grad_off_out + b0 * fi, dgoff + b0 * fi, nb * fi));
    return DCN_OK;
  };
  for (int i = 0; i < P.n; ++i) {
    const size_t b0 = P.b0[i], nb = P.d[i].B;
    if (!reuse) {
      DCN_TRY(h2d(h, h->cin, dx + b0 * xi, (const char*)x + b0 * xi, nb * xi));
      DCN_TRY(h2d(h, h->cin, doff + b0 * fi, (const char*)off + b0 * fi, nb * fi));
    }
    DCN_TRY(h2d(h, h->cin, dgo + b0 * oi, (const char*)grad_out + b0 * oi, nb * oi));
    DCN_TRY(hop(h, 2 * i, h->cin, h->stream));
    char* pp = P.n > 1 ? part + i * npar * sizeof(float) : gpar;
    DCN_TRY(dcn_backward(h, &P.d[i], (float*)(dx + b0 * xi), (float*)(doff + b0 * fi),
                         (float*)dwo, (float*)dw, (float*)(dgo + b0 * oi),
                         (float*)(dgx + b0 * xi), (float*)(pp + p_gw * es),
                         d->has_bias ? (float*)(pp + p_gb * es) : nullptr,
                         (float*)(pp + p_gwo * es), (float*)(pp + p_gbo * es),
                         grad_off_out ? (float*)(dgoff + b0 * fi) : nullptr,
                         (char*)s->ws + P.ws_off[i], P.ws_off[i + 1] - P.ws_off[i],
                         reuse ? DCN_BWD_COL_IN_WS : 0));
    HIP_TRY(hipEventRecord(h->hev[2 * i + 1], h->stream));
    if (i > 0) DCN_TRY(download(i - 1));
  }
  if (P.n > 1)  // fp32 only (chunk_count)
    HIP_TRY(dcn::launch_sum_partials((const float*)part, P.n, npar, (float*)gpar, h->stream));
  DCN_TRY(download(P.n - 1));
  DCN_TRY(d2h(h, h->stream, grad_w, gpar + p_gw * es, nw * es));
  if (d->has_bias) DCN_TRY(d2h(h, h->stream, grad_b, gpar + p_gb * es, g.O * es));
  DCN_TRY(d2h(h, h->stream, grad_w_off, gpar + p_gwo * es, nwo * es));
  DCN_TRY(d2h(h, h->stream, grad_b_off, gpar + p_gbo * es, g.J * es));
  HIP_TRY(hipStreamSynchronize(h->cout));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int default_state(dcn_handle* h, dcn_host_state** s) {
  DCN_TRY(set_device(h));
  if (!h->hs0) {
    h->hs0 = new dcn_host_state();
    h->hs0->h = h;
  }
  *s = h->hs0;
  return DCN_OK;
}
}  // namespace

int dcn_host_state_create(dcn_handle* h, dcn_host_state** out) {
  if (!out) return fail(DCN_ERR_INVALID, "null out pointer");
  *out = nullptr;
  DCN_TRY(set_device(h));
  auto* s = new dcn_host_state();
  s->h = h;
  h->states.push_back(s);
  *out = s;
  return DCN_OK;
}

int dcn_host_state_destroy(dcn_host_state* s) {
  if (!s) return DCN_OK;
  if (dcn_handle* h = s->h) {
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    state_free(s);
    h->states.erase(std::remove(h->states.begin(), h->states.end(), s), h->states.end());
  }
  delete s;
  return DCN_OK;
}

int dcn_host_state_set_chunks(dcn_host_state* s, int chunks) {
  DCN_TRY(check_state(s));
  if (chunks < 0) return fail(DCN_ERR_INVALID, "chunks must be >= 0 (0 = auto)");
  s->chunks = chunks;
  return DCN_OK;
}

int dcn_forward_host_s(dcn_host_state* s, const dcn_desc* d, const float* x, const float* w_off,
                       const float* b_off, const float* w, const float* b, float* out,
                       float* off) {
  return forward_host(s, d, x, w_off, b_off, w, b, out, off);
}

int dcn_backward_host_s(dcn_host_state* s, const dcn_desc* d, const float* x, const float* off,
                        const float* w_off, const float* w, const float* grad_out,
                        float* grad_x, float* grad_w, float* grad_b, float* grad_w_off,
                        float* grad_b_off, float* grad_off_out, int flags) {
  if (flags & ~DCN_HOST_REUSE_FWD) return fail(DCN_ERR_INVALID, "unknown dcn_backward_host flag");
  return backward_host(s, d, x, off, w_off, w, grad_out, grad_x, grad_w, grad_b, grad_w_off,
                       grad_b_off, grad_off_out, flags);
}

int dcn_forward_host(dcn_handle* h, const dcn_desc* d, const float* x, const float* w_off,
                     const float* b_off, const float* w, const float* b, float* out, float* off) {
  dcn_host_state* s;
  DCN_TRY(default_state(h, &s));
  return forward_host(s, d, x, w_off, b_off, w, b, out, off);
}

int dcn_backward_host(dcn_handle* h, const dcn_desc* d, const float* x, const float* off,
                      const float* w_off, const float* w, const float* grad_out, float* grad_x,
                      float* grad_w, float* grad_b, float* grad_w_off, float* grad_b_off,
                      float* grad_off_out) {
  dcn_host_state* s;
  DCN_TRY(default_state(h, &s));
  return backward_host(s, d, x, off, w_off, w, grad_out, grad_x, grad_w, grad_b, grad_w_off,
                       grad_b_off, grad_off_out, 0);
}

int dcn_backward_host_ex(dcn_handle* h, const dcn_desc* d, const float* x, const float* off,
                         const float* w_off, const float* w, const float* grad_out,
                         float* grad_x, float* grad_w, float* grad_b, float* grad_w_off,
                         float* grad_b_off, float* grad_off_out, int flags) {
  if (flags & ~DCN_HOST_REUSE_FWD) return fail(DCN_ERR_INVALID, "unknown dcn_backward_host_ex flag");
  dcn_host_state* s;
  DCN_TRY(default_state(h, &s));
  return backward_host(s, d, x, off, w_off, w, grad_out, grad_x, grad_w, grad_b, grad_w_off,
                       grad_b_off, grad_off_out, flags);
}

// ---- profiling ------------------------------------------------------------------
// ---- deformable RoI pooling ------------------------------------------------------
namespace {
int make_roi_geo(const dcn_roi_desc* d, dcn::RoiGeo* q) {
  if (!d || !q) return fail(DCN_ERR_INVALID, "null RoI descriptor");
  q->B = d->B, q->C = d->C, q->H = d->H, q->W = d->W, q->R = d->R;
  q->ph = d->ph, q->pw = d->pw;
  q->part_h = d->part_h > 0 ? d->part_h : d->ph;  // part_size defaults to output_size (:171)
  q->part_w = d->part_w > 0 ? d->part_w : d->pw;
  q->P = d->ph * d->pw;
  q->ps = d->ps != 0, q->no_trans = d->no_trans != 0;
  q->scale = d->spatial_scale, q->trans_std = d->trans_std;
  if (d->ph <= 0 || d->pw <= 0) return fail(DCN_ERR_INVALID, "output_size must be positive");
  q->Cout = q->ps ? d->C / q->P : d->C;  // C_out = C // (ph*pw) (:177)
  if (!dcn::roi_geo_ok(*q))
    return fail(DCN_ERR_INVALID, "bad RoI pool shape (empty tensor, C // (ph*pw) == 0, or > 256 bins)");
  return DCN_OK;
}
int check_roi_batch(const dcn::RoiGeo& q, const float* rois) {
  for (int r = 0; r < q.R; ++r) {
    const int b = (int)rois[(size_t)r * 5];
    if (b < 0 || b >= q.B)
      return fail(DCN_ERR_INVALID, "rois[" + std::to_string(r) + ", 0] = " + std::to_string(b) +
                                       " is not a batch index in [0, " + std::to_string(q.B) + ")");
  }
  return DCN_OK;
}
}  // namespace

int dcn_roi_pool_fwd(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                     const float* rois, const float* offsets, float* out) {
  dcn::RoiGeo q;
  DCN_TRY(make_roi_geo(d, &q));
  DCN_TRY(set_device(h));
  if (!q.no_trans && !offsets && q.R > 0) return fail(DCN_ERR_INVALID, "offsets is NULL");
  HIP_TRY(dcn::launch_roi_pool_fwd(q, features, rois, offsets, out, h->stream));
  return DCN_OK;
}

int dcn_roi_pool_bwd(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                     const float* rois, const float* offsets, const float* grad_out,
                     float* grad_features, float* grad_offsets) {
  dcn::RoiGeo q;
  DCN_TRY(make_roi_geo(d, &q));
  DCN_TRY(set_device(h));
  if (!q.no_trans && !offsets && q.R > 0) return fail(DCN_ERR_INVALID, "offsets is NULL");
  HIP_TRY(dcn::launch_roi_pool_bwd(q, features, rois, offsets, grad_out, grad_features,
                                   grad_offsets, h->stream));
  return DCN_OK;
}

int dcn_roi_pool_fwd_host(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                          const float* rois, const float* offsets, float* out) {
  dcn::RoiGeo q;
  DCN_TRY(make_roi_geo(d, &q));
  DCN_TRY(set_device(h));
  DCN_TRY(check_roi_batch(q, rois));
  const size_t nf = (size_t)q.B * q.C * q.H * q.W, nr = (size_t)q.R * 5, no = (size_t)q.R * q.P * 2;
  const size_t nout = (size_t)q.R * q.Cout;
  DevBufs db;
  float *df, *dr, *doffs = nullptr, *dout;
  DCN_TRY(db.alloc(nf * 4, &df));
  DCN_TRY(db.alloc(nr * 4, &dr));
  DCN_TRY(db.alloc(nout * 4, &dout));
  DCN_TRY(h2d(h, h->stream, df, features, nf * 4));
  DCN_TRY(h2d(h, h->stream, dr, rois, nr * 4));
  if (offsets) {
    DCN_TRY(db.alloc(no * 4, &doffs));
    DCN_TRY(h2d(h, h->stream, doffs, offsets, no * 4));
  }
  DCN_TRY(dcn_roi_pool_fwd(h, d, df, dr, doffs, dout));
  DCN_TRY(d2h(h, h->stream, out, dout, nout * 4));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int dcn_roi_pool_bwd_host(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                          const float* rois, const float* offsets, const float* grad_out,
                          float* grad_features, float* grad_offsets) {
  dcn::RoiGeo q;
  DCN_TRY(make_roi_geo(d, &q));
  DCN_TRY(set_device(h));
  DCN_TRY(check_roi_batch(q, rois));
  const size_t nf = (size_t)q.B * q.C * q.H * q.W, nr = (size_t)q.R * 5, no = (size_t)q.R * q.P * 2;
  const size_t nout = (size_t)q.R * q.Cout;
  DevBufs db;
  float *df, *dr, *doffs = nullptr, *dgo, *dgf, *dgoffs = nullptr;
  DCN_TRY(db.alloc(nf * 4, &df));
  DCN_TRY(db.alloc(nr * 4, &dr));
  DCN_TRY(db.alloc(nout * 4, &dgo));
  DCN_TRY(db.alloc(nf * 4, &dgf));
  DCN_TRY(h2d(h, h->stream, df, features, nf * 4));
  DCN_TRY(h2d(h, h->stream, dr, rois, nr * 4));
  DCN_TRY(h2d(h, h->stream, dgo, grad_out, nout * 4));
  if (offsets) {
    DCN_TRY(db.alloc(no * 4, &doffs));
    DCN_TRY(h2d(h, h->stream, doffs, offsets, no * 4));
  }
  if (grad_offsets) DCN_TRY(db.alloc(no * 4, &dgoffs));
  DCN_TRY(dcn_roi_pool_bwd(h, d, df, dr, doffs, dgo, dgf, dgoffs));
  DCN_TRY(d2h(h, h->stream, grad_features, dgf, nf * 4));
  if (grad_offsets) DCN_TRY(d2h(h, h->stream, grad_offsets, dgoffs, no * 4));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return DCN_OK;
}

int dcn_prof_enable(dcn_handle* h, int capacity) {
  DCN_TRY(set_device(h));
  if (capacity < 0) return fail(DCN_ERR_INVALID, "negative capacity");
  for (int k = 0; k < DCN_K_COUNT; ++k) {
    while ((int)h->ev[k].size() < 2 * capacity) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      h->ev[k].push_back(e);
    }
    h->prof_n[k] = 0;
  }
  h->prof_cap = capacity;
  return DCN_OK;
}

int dcn_prof_read(dcn_handle* h, int kernel_id, double* total_ms, int* count) {
  DCN_TRY(set_device(h));
  if (kernel_id < 0 || kernel_id >= DCN_K_COUNT) return fail(DCN_ERR_INVALID, "bad kernel id");
  HIP_TRY(hipStreamSynchronize(h->stream));
  double t = 0;
  for (int i = 0; i < h->prof_n[kernel_id]; ++i) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[kernel_id][2 * i], h->ev[kernel_id][2 * i + 1]));
    t += ms;
  }
  if (total_ms) *total_ms = t;
  if (count) *count = h->prof_n[kernel_id];
  return DCN_OK;
}

int dcn_prof_reset(dcn_handle* h) {
  if (!h) return fail(DCN_ERR_INVALID, "null handle");
  for (int k = 0; k < DCN_K_COUNT; ++k) h->prof_n[k] = 0;
  return DCN_OK;
}

// Internal hooks for dcn_comm.cpp (not in dcn.h).
// Detach the handle's communicator after its last exchange has finished (dcn_comm_destroy,
// dcn_destroy): the stream the exchange runs on is drained first.
__attribute__((visibility("hidden"))) void dcn_internal_handle_drop_comm(dcn_handle* h) {
  if (!h || !h->comm) return;
  (void)hipSetDevice(h->device);
  if (h->comm_stream) (void)hipStreamSynchronize(h->comm_stream);
  dcn_internal_comm_detach(h->comm, h);
  h->comm = nullptr;
}
__attribute__((visibility("hidden"))) int dcn_internal_fail(int code, const char* msg) {
  return fail(code, msg);
}
__attribute__((visibility("hidden"))) int dcn_internal_bind(dcn_handle* h, void** stream) {
  DCN_TRY(set_device(h));
  *stream = h->stream;
  return DCN_OK;
}

// Test hook: force the generic global-memory im2col/col2im kernels.
int dcn_debug_force_generic(int on) {
  dcn::set_force_generic(on);
  return DCN_OK;
}

int dcn_debug_bins_chunked(int on) {
  dcn::set_bins_chunked(on);
  return DCN_OK;
}

int dcn_debug_offset_gemm(int on) {
  g_ocg = on != 0;
  return DCN_OK;
}

int dcn_debug_fused_workgroups(int n) {
  if (n < 0) return fail(DCN_ERR_INVALID, "dcn_debug_fused_workgroups: negative count");
  dcn::set_fused_workgroups(n);
  return DCN_OK;
}

int dcn_debug_dw_parts(const dcn_desc* d, int* planes, int n, int* capacity) {
  if (!planes || !capacity || n < DW_PATHS)
    return fail(DCN_ERR_INVALID, "dcn_debug_dw_parts: bad argument");
  Geo g;
  DCN_TRY(make_geo(d, &g));
  dw_parts(g, planes);
  *capacity = ws_layout(g, true).parts_planes;
  return DCN_OK;
}

int dcn_debug_col_ws_records(dcn_handle* h, int* n) {
  if (!h || !n) return fail(DCN_ERR_INVALID, "dcn_debug_col_ws_records: bad argument");
  std::lock_guard<std::mutex> lk(h->col_ws_mu);
  *n = (int)h->col_ws.size();
  return DCN_OK;
}

int dcn_set_math(dcn_handle* h, int math) {
  if (!h) return fail(DCN_ERR_INVALID, "dcn_set_math: null handle");
  if (math != DCN_MATH_F32 && math != DCN_MATH_F32_BF16X3 && math != DCN_MATH_F32_BF16X6 &&
      math != DCN_MATH_F32_BF16X9)
    return fail(DCN_ERR_INVALID, "dcn_set_math: unknown mode " + std::to_string(math));
  dcn::gemm_set_math(h->gemm, math);
  return DCN_OK;
}

int dcn_set_comm(dcn_handle* h, dcn_comm* c) {
  DCN_TRY(set_device(h));
  if (h->comm && h->comm != c) {
    HIP_TRY(hipStreamSynchronize(h->comm_stream));
    dcn_internal_comm_detach(h->comm, h);
  }
  h->comm = c;
  dcn_internal_comm_attach(c, h);
  return DCN_OK;
}

int dcn_set_grad_stream(dcn_handle* h, void* s) {
  DCN_TRY(set_device(h));
  h->grad_stream = reinterpret_cast<hipStream_t>(s);
  return DCN_OK;
}

int dcn_set_fwd_path(dcn_handle* h, int path) {
  if (!h) return fail(DCN_ERR_INVALID, "dcn_set_fwd_path: null handle");
  if (path != DCN_FWD_AUTO && path != DCN_FWD_UNFUSED && path != DCN_FWD_FUSED &&
      path != DCN_FWD_FUSED_NOCOL)
    return fail(DCN_ERR_INVALID, "dcn_set_fwd_path: unknown path " + std::to_string(path));
  h->fwd_path = path;
  return DCN_OK;
}

int dcn_get_fwd_path(dcn_handle* h, int* path) {
  if (!h || !path) return fail(DCN_ERR_INVALID, "dcn_get_fwd_path: null argument");
  *path = h->fwd_path;
  return DCN_OK;
}

int dcn_get_math(dcn_handle* h, int* math) {
  if (!h || !math) return fail(DCN_ERR_INVALID, "dcn_get_math: null argument");
  *math = dcn::gemm_get_math(h->gemm);
  return DCN_OK;
}

int dcn_debug_gemm(dcn_handle* h, int ta, int tb, int m, int n, int k, const float* A, int lda,
                   long sa, const float* B, int ldb, long sb, float* C, int ldc, long sc,
                   int batch) {
  if (!h || !A || !B || !C || m <= 0 || n <= 0 || k <= 0 || batch <= 0)
    return fail(DCN_ERR_INVALID, "dcn_debug_gemm: bad argument");
  DCN_TRY(set_device(h));
  dcn::GemmSpec sp;
  sp.ta = ta != 0; sp.tb = tb != 0;
  sp.m = m; sp.n = n; sp.k = k;
  sp.lda = lda; sp.ldb = ldb; sp.ldc = ldc;
  sp.sa = sa; sp.sb = sb; sp.sc = sc;
  sp.batch = batch;
  GEMM_TRY(h, sp, A, B, C);
  return DCN_OK;
}

}  // extern "C"
