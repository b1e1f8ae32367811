/*
 * dcn.h — C-ABI of libdcn.so, the MI355X (gfx950) DeformConv2d operator.
 *
 * The reference (x-y20/jittor-dcn) has no FFI: its boundary is the Python module
 * `DeformConv2d` in deform_conv.py. Each entry point below replaces one piece of
 * that module's behaviour; the file:line it replaces is cited next to it. The
 * Python drop-in (jittor-dcn_amd/deform_conv.py) binds these symbols with ctypes.
 *
 * Conventions
 *  - Every function returns int: 0 = OK, < 0 = dcn_status error code. The
 *    library never aborts; dcn_last_error() returns a thread-local message.
 *  - Tensors are dense, NCHW (x, out, offsets) or the reference's own parameter
 *    layouts (weights), in the descriptor's dtype: fp32 (DCN_F32, the reference's
 *    type) or bf16 storage (DCN_BF16: every tensor argument then points at 16-bit
 *    bf16 values despite the float* spelling; internally the columns and GEMM
 *    operands are bf16 with fp32 accumulation, everything else fp32). All device
 *    pointers are caller-owned; the library never frees or retains them.
 *  - Calls are ordered on the handle's stream (dcn_set_stream). A handle is not
 *    thread-safe: use one handle per device and per host thread.
 *  - `*_host` variants take host pointers, move data over PCIe themselves and
 *    synchronise before returning (the NumPy / Jittor-CPU caller's path).
 *
 * Semantics are exactly deform_conv.py:56-81 (see DESIGN.md §1 "quirks"):
 * transposed sampling, coordinates normalised by the OUTPUT size, no per-tap
 * base offsets, offset channels [Δx(0..N-1) | Δy(0..N-1)], weight read as
 * W[o][n][c]. `dil_h/dil_w/deform_groups` are extensions (BASELINE config 5)
 * that must be 1 for reference semantics.
 */
#ifndef DCN_H_
#define DCN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCN_ABI_VERSION 5 /* 2: dcn_allreduce_grads takes a dtype; dcn_set_comm, dcn_set_grad_stream;
                             3: dcn_backward_host_ex; 4: dcn_host_state, dcn_host_alloc;
                             5: dcn_forward_ex (DCN_FWD_NO_COLUMNS), dcn_get_fwd_path,
                                dcn_workspace_bytes(DCN_WS_FORWARD_NO_COLUMNS) */

typedef enum {
  DCN_OK = 0,
  DCN_ERR_INVALID = -1,     /* bad descriptor / argument */
  DCN_ERR_UNSUPPORTED = -2, /* shape or dtype outside what the build supports */
  DCN_ERR_HIP = -3,         /* HIP runtime error (no device, OOM, launch) */
  DCN_ERR_BLAS = -4,        /* rocBLAS error */
  DCN_ERR_WORKSPACE = -5,   /* caller workspace too small */
  DCN_ERR_COMM = -6         /* RCCL missing or a collective failed */
} dcn_status;

typedef enum { DCN_F32 = 0, DCN_BF16 = 1 } dcn_dtype;

/* Geometry of one DeformConv2d call. Mirrors the constructor arguments of
 * deform_conv.py:7 (in_channels=C, out_channels=O, kernel_size=(kh,kw),
 * stride=(sh,sw), padding=(ph,pw), bias) plus the input batch shape. */
typedef struct {
  int B, C, H, W; /* input x[B][C][H][W] */
  int O;          /* out_channels */
  int kh, kw;     /* kernel_size, deform_conv.py:11 */
  int sh, sw;     /* stride, deform_conv.py:12 */
  int ph, pw;     /* padding, deform_conv.py:13 */
  int dil_h, dil_w;  /* extension: offset-conv dilation (1 = reference) */
  int deform_groups; /* extension: offset groups (1 = reference) */
  int dtype;         /* dcn_dtype. DCN_BF16 needs deform_groups 1, kh*kw <= 9,
                        C % 4 == 0, C <= 256, and is supported by dcn_forward /
                        dcn_backward (+ _host); the standalone kernel entry points
                        below are DCN_F32 only */
  int has_bias;      /* deform_conv.py:25 */
} dcn_desc;

typedef struct dcn_handle dcn_handle;

/* ---- library / device ---------------------------------------------------- */
int dcn_abi_version(void);
const char* dcn_last_error(void);
int dcn_device_count(int* n);
int dcn_create(int device, dcn_handle** out);
int dcn_destroy(dcn_handle* h);
/* Bind the handle to an existing hipStream_t. NULL is the HIP null (legacy default)
 * stream, as in every HIP library, so a framework running on its default stream
 * (e.g. torch's, whose handle is 0) passes it through unchanged. A new handle uses its
 * own non-blocking stream; dcn_use_own_stream returns to it. */
int dcn_set_stream(dcn_handle* h, void* hip_stream);
int dcn_use_own_stream(dcn_handle* h);
int dcn_get_stream(dcn_handle* h, void** hip_stream);
int dcn_synchronize(dcn_handle* h);

/* ---- device memory helpers (ctypes callers without another runtime) -------- */
int dcn_malloc(dcn_handle* h, size_t bytes, void** ptr);
int dcn_free(dcn_handle* h, void* ptr);
/* Page-locked host memory (hipHostMalloc): the host path's recycled output arrays
 * (jittor-dcn_amd/hostmem.py). A device-to-host copy into pageable memory runs as a copy
 * kernel through a staging buffer, on the CUs beside the path's own kernels (r03 trace:
 * the offset conv of a pipelined chunk 3x slower beside it); into page-locked memory it
 * is a DMA. */
int dcn_host_alloc(dcn_handle* h, size_t bytes, void** ptr);
int dcn_host_free(void* ptr);
int dcn_memcpy_h2d(dcn_handle* h, void* dst, const void* src, size_t bytes);
int dcn_memcpy_d2h(dcn_handle* h, void* dst, const void* src, size_t bytes);
int dcn_memset_zero(dcn_handle* h, void* dst, size_t bytes);

/* ---- shapes -------------------------------------------------------------- */
/* Output size, deform_conv.py:34-35 (dilation-aware for the extension). */
int dcn_out_shape(const dcn_desc* d, int* Ho, int* Wo);
/* Device workspace needed by dcn_forward (with_backward=0) or by the pair
 * dcn_forward + dcn_backward sharing one workspace (with_backward=1).
 * with_backward=DCN_WS_FORWARD_NO_COLUMNS (2): a forward that writes no columns
 * (dcn_forward_ex with DCN_FWD_NO_COLUMNS, or DCN_FWD_FUSED_NOCOL) needs no column region
 * where that applies (DCN_BF16 geometries of the fused forward: 231 MB less at config 4);
 * elsewhere the same as 0. */
#define DCN_WS_FORWARD_NO_COLUMNS 2
int dcn_workspace_bytes(const dcn_desc* d, int with_backward, size_t* bytes);

/* ---- hot-path kernels (device pointers, stream-ordered) -------------------- */
/* offset = offset_conv(x): replaces deform_conv.py:58 (nn.Conv from :16-21).
 * w_off[2N·G][C][kh][kw], b_off[2N·G] -> off[B][2N·G][Ho][Wo]. */
int dcn_offset_conv_fwd(dcn_handle* h, const dcn_desc* d, const float* x,
                        const float* w_off, const float* b_off, float* off);
/* Backward of the offset conv: grad_w_off = Σ, grad_b_off = Σ (overwritten);
 * grad_x += conv_transpose(grad_off, w_off) (accumulated). */
int dcn_offset_conv_bwd(dcn_handle* h, const dcn_desc* d, const float* x,
                        const float* w_off, const float* grad_off,
                        float* grad_x, float* grad_w_off, float* grad_b_off);
/* Deformable bilinear im2col (K1): replaces deform_conv.py:30-54 and :62-73
 * (grid build, normalisation, x_repeat, grid_sample, permutes). Writes the
 * sampled matrix of deform_conv.py:73 row by row, channels-last:
 * col[b - b0][ho·Wo + wo][n·C + c] for images b in [b0, b0+nb). */
int dcn_im2col_fwd(dcn_handle* h, const dcn_desc* d, const float* x,
                   const float* off, float* col, int b0, int nb);
/* Backward of K1 (K5): grad_x = Σ scatter(grad_col) (sampling route only) and
 * grad_off[b][..][ho][wo] = coordinate gradient, both OVERWRITTEN for images
 * [b0, b0+nb). grad_col has the layout of dcn_im2col_fwd's col. */
int dcn_col2im_coord_bwd(dcn_handle* h, const dcn_desc* d, const float* x,
                         const float* off, const float* grad_col,
                         float* grad_x, float* grad_off, int b0, int nb);

/* ---- whole-op entry points ------------------------------------------------- */
/* DeformConv2d.execute (deform_conv.py:56-81). Writes out[B][O][Ho][Wo] and the
 * offsets off[B][2N·G][Ho][Wo] (kept by the caller for backward). ws must hold
 * dcn_workspace_bytes(d, with_backward) bytes; when with_backward, the sampled
 * columns stay in ws for dcn_backward (flag DCN_BWD_COL_IN_WS). */
int dcn_forward(dcn_handle* h, const dcn_desc* d, const float* x,
                const float* w_off, const float* b_off, const float* w,
                const float* b, float* out, float* off, void* ws,
                size_t ws_bytes);
/* dcn_forward with per-call flags (ABI 5). DCN_FWD_NO_COLUMNS: no backward will read this
 * forward's columns (inference, jt.no_grad: deform_conv.py:56 under train.py:430), so a
 * DCN_BF16 fused geometry writes none, whatever path the handle is set to; the handle's
 * forward path is not changed, only its per-workspace column record (below). ws may then be
 * sized by dcn_workspace_bytes(d, DCN_WS_FORWARD_NO_COLUMNS). fp32, and bf16 geometries
 * outside the fused forward, write their columns as usual. flags = 0 is dcn_forward. */
#define DCN_FWD_NO_COLUMNS 1
int dcn_forward_ex(dcn_handle* h, const dcn_desc* d, const float* x,
                   const float* w_off, const float* b_off, const float* w,
                   const float* b, float* out, float* off, void* ws,
                   size_t ws_bytes, int flags);

#define DCN_BWD_COL_IN_WS 1 /* ws still holds forward's columns: the caller must not let
                              anything write into ws between this handle's forward and this
                              backward (another handle's forward, an fp32 forward, a forward of
                              another geometry on the same ws). For DCN_BF16 the handle records
                              the workspaces its own forwards wrote columns into (a bare
                              pointer per workspace, at most 256, the oldest dropped first); a
                              backward on a workspace it holds no record for (a NO_COLUMNS /
                              FUSED_NOCOL forward, a dropped record) recomputes them, but the
                              record does not notice a foreign write into a recorded ws. The
                              offsets are then also the forward's (a DCN_BF16 backward reads
                              the fp32 offsets that forward left in ws, r06): off must be that
                              forward's output, as the columns already assume. On the DCN_F32
                              offset-conv GEMM route (stride / dilation != 1, e.g. BASELINE
                              config 5) the backward also reads the offset conv's im2col and
                              reshaped w_off that forward left in ws (r06), tracked per
                              workspace the same way: w_off must be that forward's too. */

/* Autodiff of DeformConv2d.execute as triggered by optimizer.backward
 * (train.py:414). Overwrites grad_x, grad_w, grad_b (if has_bias),
 * grad_w_off, grad_b_off. grad_off_out (optional, may be NULL) receives
 * ∂L/∂offset [B][2N·G][Ho][Wo]. */
int dcn_backward(dcn_handle* h, const dcn_desc* d, const float* x,
                 const float* off, const float* w_off, const float* w,
                 const float* grad_out, float* grad_x, float* grad_w,
                 float* grad_b, float* grad_w_off, float* grad_b_off,
                 float* grad_off_out, void* ws, size_t ws_bytes, int flags);

/* Host-pointer variants (NumPy / Jittor-CPU callers, the reference caller's path:
 * train.py:408-414 through the module). Synchronous. Device copies of the tensors are
 * kept between calls (no per-call allocation); transfers run straight from / to the
 * caller's memory (env DCN_HOST_STAGING=1: through a pinned ring with host copy threads
 * instead, which pays for destinations whose pages were never touched).
 *
 * The batch is cut into image chunks whose transfers run beside the kernels (the upload
 * of chunk i+1 and the download of chunk i-1 while chunk i computes). fp32 only: about
 * 52 MB of x per chunk, at most 16 chunks (dcn_host_state_set_chunks); bf16 and a handle
 * with a communicator use one chunk. With several chunks the parameter gradients are
 * the chunk partials summed in chunk order (deterministic; not bitwise the one-chunk
 * sums). The dcn_*_host calls below use the handle's own host state; a network of
 * several modules on one handle gives each module its own (dcn_host_state_create). */
int dcn_forward_host(dcn_handle* h, const dcn_desc* d, const float* x,
                     const float* w_off, const float* b_off, const float* w,
                     const float* b, float* out, float* off);
int dcn_backward_host(dcn_handle* h, const dcn_desc* d, const float* x,
                      const float* off, const float* w_off, const float* w,
                      const float* grad_out, float* grad_x, float* grad_w,
                      float* grad_b, float* grad_w_off, float* grad_b_off,
                      float* grad_off_out);
/* dcn_backward_host with flags. DCN_HOST_REUSE_FWD: x, off, w_off and w are the very
 * arrays (same pointers, unmodified since) of the last dcn_forward_host on this handle,
 * with the same descriptor; their device copies and the forward's sampled columns are
 * reused instead of uploaded and recomputed (the autodiff pair of one module call,
 * train.py:408-414). DCN_ERR_INVALID when they are not. Without the flag: as
 * dcn_backward_host. */
#define DCN_HOST_REUSE_FWD 2
int dcn_backward_host_ex(dcn_handle* h, const dcn_desc* d, const float* x,
                         const float* off, const float* w_off, const float* w,
                         const float* grad_out, float* grad_x, float* grad_w,
                         float* grad_b, float* grad_w_off, float* grad_b_off,
                         float* grad_off_out, int flags);

/* Per-module host state (ABI 4). One per DeformConv2d module (train.py:304-318 stacks
 * four on one handle): the device copies of that module's x / offsets / weights and its
 * own workspace, which keeps the forward's columns. A dcn_backward_host_s with
 * DCN_HOST_REUSE_FWD given the arrays of the state's last forward reuses them, whatever
 * other states ran on the handle in between (DCN_ERR_INVALID for other arrays; `off` may
 * then be NULL if the forward was given NULL). States belong to their handle:
 * dcn_destroy frees their device memory, after which only dcn_host_state_destroy accepts
 * them. The handle-level dcn_*_host calls use a state of the handle's own. */
typedef struct dcn_host_state dcn_host_state;
int dcn_host_state_create(dcn_handle* h, dcn_host_state** out);
int dcn_host_state_destroy(dcn_host_state* s);
/* image chunks of the transfer pipeline: 0 = auto (the default), else min(chunks, B, 16);
 * fp32 only (bf16 and a communicator: always 1). */
int dcn_host_state_set_chunks(dcn_host_state* s, int chunks);
int dcn_forward_host_s(dcn_host_state* s, const dcn_desc* d, const float* x,
                       const float* w_off, const float* b_off, const float* w,
                       const float* b, float* out, float* off);
int dcn_backward_host_s(dcn_host_state* s, const dcn_desc* d, const float* x,
                        const float* off, const float* w_off, const float* w,
                        const float* grad_out, float* grad_x, float* grad_w,
                        float* grad_b, float* grad_w_off, float* grad_b_off,
                        float* grad_off_out, int flags);

/* ---- deformable RoI pooling -------------------------------- *
 * DeformRoIPool (deform_conv.py:85-159) and DeformPSRoIPool (:162-241), fp32.
 * rois[R][5] = (batch index, x1, y1, x2, y2) in input coordinates (scaled by
 * spatial_scale, :96/:181); offsets[R][P][2] (x, y) per bin, P = ph*pw (for the PS
 * pool the reference's offsets[R][2P] with x at 2p, y at 2p+1 is the same memory).
 * Each bin is ONE bilinear sample at its centre + offset, with the reference's corner
 * clamping (corners clamped to the image, weights from the clamped top-left corner,
 * :121-135 / :214-228). The reference then sums the weighted corner features over the
 * bins (`.sum(dim=2)`, :143-157 / :239) before reshaping to [R, C, ph, pw], so its
 * module only runs for ph*pw == 1: out here is that sum, [R][C] (DeformRoIPool) or
 * [R][C / P] (DeformPSRoIPool, channel c*P + p for bin p); the shim reshapes (and
 * fails like the reference for P != 1). */
typedef struct {
  int B, C, H, W;          /* features [B][C][H][W] */
  int R;                   /* number of RoIs */
  int ph, pw;              /* output_size (:87, :165) */
  int part_h, part_w;      /* part_size (PS only, :171; = output size when unset) */
  float spatial_scale;     /* :86 */
  float trans_std;         /* PS only (:172) */
  int ps;                  /* 0 = DeformRoIPool, 1 = DeformPSRoIPool */
  int no_trans;            /* PS only (:169): ignore the offsets */
} dcn_roi_desc;
/* out[R][C or C/P] (overwritten). */
int dcn_roi_pool_fwd(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                     const float* rois, const float* offsets, float* out);
/* Autodiff of the forward: grad_features [B][C][H][W] and grad_offsets [R][P][2]
 * overwritten (grad_offsets may be NULL; zero for no_trans). The RoI boxes get no
 * gradient (the reference's rois come from the data). grad_features accumulates with
 * atomics (RoIs may share pixels), so its low bits depend on the summation order. */
int dcn_roi_pool_bwd(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                     const float* rois, const float* offsets, const float* grad_out,
                     float* grad_features, float* grad_offsets);
/* Host-pointer variants (synchronous). Batch indices outside [0, B) are rejected
 * (DCN_ERR_INVALID), where the reference would raise an index error. */
int dcn_roi_pool_fwd_host(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                          const float* rois, const float* offsets, float* out);
int dcn_roi_pool_bwd_host(dcn_handle* h, const dcn_roi_desc* d, const float* features,
                          const float* rois, const float* offsets, const float* grad_out,
                          float* grad_features, float* grad_offsets);

/* ---- in-library kernel timing (HIP events on the handle's stream) ---------- */
typedef enum {
  DCN_K_OFFSET_FWD = 0,
  DCN_K_IM2COL = 1,
  DCN_K_GEMM_FWD = 2,
  DCN_K_BIAS_FWD = 3,
  DCN_K_BWD_BIAS = 4,
  DCN_K_GEMM_DW = 5,
  DCN_K_GEMM_DCOL = 6,
  DCN_K_COL2IM = 7,
  DCN_K_OFFSET_BWD = 8,
  DCN_K_XPOSE = 9, /* x -> channels-last copy used by K1/K5 */
  DCN_K_COUNT = 10
} dcn_kernel_id;
/* Record start/stop events around every launch of each kernel class, up to
 * `capacity` launches per class (0 disables). */
int dcn_prof_enable(dcn_handle* h, int capacity);
/* Sum of elapsed ms and number of recorded launches (synchronises first). */
int dcn_prof_read(dcn_handle* h, int kernel_id, double* total_ms, int* count);
int dcn_prof_reset(dcn_handle* h);

/* ---- data-parallel gradient exchange (RCCL over xGMI) ------------------------- *
 * Batch-sharded DP: every rank runs dcn_forward/dcn_backward on its own
 * images, then sums the packed parameter gradients once per step. The reference is
 * single-device (train.py:414), so these have no reference counterpart. One rank calls
 * dcn_comm_get_unique_id and ships the 128 bytes to the others (any channel); every
 * rank then calls dcn_comm_init with its own handle. RCCL is loaded on first use. */
#define DCN_COMM_ID_BYTES 128
typedef struct dcn_comm dcn_comm;
int dcn_comm_get_unique_id(void* id /* DCN_COMM_ID_BYTES */);
int dcn_comm_init(dcn_handle* h, int nranks, int rank, const void* id, dcn_comm** out);
int dcn_comm_destroy(dcn_comm* c);
/* In-place sum over ranks of `count` device values of `dtype` (DCN_F32 or DCN_BF16), on
 * the handle's stream. DCN_ERR_INVALID when count elements of dtype do not fit inside the
 * device allocation holding `grads`. */
int dcn_allreduce_grads(dcn_handle* h, dcn_comm* c, void* grads, size_t count, int dtype);
/* Attach a communicator to the handle (NULL detaches). dcn_backward (and
 * dcn_backward_host) then returns gradients already summed over the communicator's ranks:
 * grad_w and grad_b are all-reduced on an internal stream as soon as they are final,
 * overlapped with the ∂columns GEMM, col2im and the offset-conv backward; grad_w_off and
 * grad_b_off are all-reduced at the end; the handle's stream waits for both before any
 * later work. For DCN_BF16 the sums run over the fp32 working copies (one bf16 rounding
 * of the summed value). Every rank must run the same sequence of dcn_backward calls.
 * Lifetime: the communicator remembers the handles attached to it; dcn_comm_destroy waits
 * for their in-flight exchanges and detaches them, and dcn_destroy detaches its handle, so
 * either may be destroyed first. */
int dcn_set_comm(dcn_handle* h, dcn_comm* c);
/* For callers with their own collectives (e.g. torch.distributed): when `hip_stream` is not
 * NULL, each later dcn_backward makes that stream wait (hipStreamWaitEvent) until grad_w
 * and grad_b are final, before the ∂columns GEMM even starts, so a collective enqueued on
 * it right after dcn_backward returns overlaps the rest of the backward. NULL disables.
 * Lifetime: the library keeps the raw stream; the caller detaches it (NULL) before
 * destroying that stream. */
int dcn_set_grad_stream(dcn_handle* h, void* hip_stream);

/* ---- GEMM arithmetic ------------------------------------------------------------ */
/* How the three fp32 GEMMs of the op (deform_conv.py:76 and its two autodiff GEMMs)
 * compute. DCN_MATH_F32 (default): native f32 MFMA in the vendor libraries.
 * DCN_MATH_F32_BF16X9 / _BF16X6: every fp32 operand split exactly into three bf16 planes
 * (hi + mid + lo == a), products on the bf16 matrix cores with fp32 accumulation; X9
 * keeps all nine plane products (each exact), X6 drops the three below 2^-23 relative
 * (one fp32 rounding). DCN_MATH_F32_BF16X3: two planes, ~2^-17 relative (opt-in).
 * The bf16 tensor path (dtype DCN_BF16) is unaffected. Env DCN_MATH sets the default of
 * new handles. No reference counterpart (Jittor matmul in fp32, deform_conv.py:76). */
typedef enum {
  DCN_MATH_F32 = 0,
  DCN_MATH_F32_BF16X3 = 3,
  DCN_MATH_F32_BF16X6 = 6,
  DCN_MATH_F32_BF16X9 = 9
} dcn_math;
int dcn_set_math(dcn_handle* h, int math);
int dcn_get_math(dcn_handle* h, int* math);

/* ---- forward schedule ----------------------------------------------------------- */
/* How the forward (deform_conv.py:41-80) runs after the offset conv.
 * DCN_BF16 (dcn_fused_bf16.hip): DCN_FWD_FUSED gathers the bilinear samples from an LDS
 * window of the channels-last x straight into the B operand of bf16 MFMAs (bias and the
 * bf16 rounding in the epilogue) and still writes the columns for a DCN_BWD_COL_IN_WS
 * backward; DCN_FWD_FUSED_NOCOL never writes a column, and its backward recomputes
 * the columns inside the ∂W MFMA kernel (no column matrix in the step); a DCN_BWD_COL_IN_WS
 * backward on the workspace of a forward without columns recomputes them (tracked per
 * workspace). Both need C % 64 == 0, O % 256 == 0, deform_groups 1, kh*kw <= 9; elsewhere
 * they take the unfused schedule. DCN_FWD_AUTO picks DCN_FWD_FUSED for DCN_BF16 when O == 256
 * and Ho*Wo >= 784 (measured faster there). Same columns bit
 * for bit as K1; out to fp32 rounding of a different summation order before the bf16
 * rounding.
 * DCN_F32: DCN_FWD_FUSED (and _NOCOL, which for fp32 still writes the columns) runs the
 * fused kernel (bilinear im2col gathered straight into the f32 MFMA GEMM's LDS tiles, bias
 * in the epilogue; the columns are still written for the backward) wherever it applies:
 * deform_groups 1, kh*kw <= 9, C % 32 == 0, O % 128 == 0, native math; otherwise the
 * unfused schedule. DCN_FWD_UNFUSED: K1 im2col, then the
 * vendor GEMM, then the bias. DCN_FWD_AUTO (default): the schedule measured faster for the
 * geometry. Same results to fp32 rounding (the columns bit for bit). */
typedef enum {
  DCN_FWD_AUTO = 0,
  DCN_FWD_UNFUSED = 1,
  DCN_FWD_FUSED = 2,
  DCN_FWD_FUSED_NOCOL = 3
} dcn_fwd_path;
int dcn_set_fwd_path(dcn_handle* h, int path);
int dcn_get_fwd_path(dcn_handle* h, int* path);

/* ---- testing ------------------------------------------------------------------ */
/* One fp32 GEMM through the handle's engine under its current math mode, BLAS
 * column-major convention: C(m×n) = op(A)·op(B), batched by element strides. */
int dcn_debug_gemm(dcn_handle* h, int ta, int tb, int m, int n, int k, const float* A,
                   int lda, long sa, const float* B, int ldb, long sb, float* C, int ldc,
                   long sc, int batch);
/* 1 = route K1/K5 through the generic global-gather kernels (independent
 * implementation used by the parity tests to cross-check the LDS-window ones). */
int dcn_debug_force_generic(int on);
/* Workgroup count of the fused forward's persistent grid (DCN_FWD_FUSED); 0 = one per CU.
 * Lets the parity tests walk many tiles (straddling images) through one workgroup. */
int dcn_debug_fused_workgroups(int n);
/* 1 = build K5's sample bins with the chunked three-kernel sort even where one block sort
 * per image applies (H·W·kh·kw <= 8192); the parity tests compare the two bit for bit. */
int dcn_debug_bins_chunked(int on);
/* 0 = run the fp32 offset conv (forward and backward) on its VALU kernels where it would run
 * as GEMMs over its own im2col (geometries without an MFMA offset-conv kernel, e.g. BASELINE
 * config 5); the parity tests compare the two. Default 1. */
int dcn_debug_offset_gemm(int on);
/* The ∂W partial planes ([O][K] fp32 each) that each backward path of this geometry writes
 * into the workspace before its fixed-order sum — planes[0] one per image, planes[1] the
 * grouped bf16 GEMM, planes[2] the recomputed-column bf16 kernel, planes[3] the bf16
 * streaming kernel's pixel ranges (0 where a path does not apply; n >= 4) — and in
 * *capacity the planes the dcn_forward + dcn_backward workspace
 * layout holds. Host only (no device call): the CPU tests check every count fits. */
int dcn_debug_dw_parts(const dcn_desc* d, int* planes, int n, int* capacity);
/* Number of workspaces the handle currently records as holding a DCN_BF16 forward's
 * columns (DCN_BWD_COL_IN_WS); bounded, see DESIGN.md §1. */
int dcn_debug_col_ws_records(dcn_handle* h, int* n);

#ifdef __cplusplus
}
#endif
#endif /* DCN_H_ */
