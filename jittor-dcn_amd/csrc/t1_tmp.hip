// dcn_fused.hip — fused deformable forward: the bilinear im2col of
// deform_conv.py:41-54,72-73 gathered straight into the LDS operand tiles of an f32 MFMA
// GEMM against the flat weight (:74-76), with the bias of :77-80 in the epilogue.
//
//   out[b][o][m] = bias[o] + Σ_k Wf[o][k] · col[b][m][k],   k = n·C + c   (Q5)
//
// The separate path is K1 (im2col_lds, HBM-bound: it writes the 1.85 GB column matrix)
// followed by a vendor GEMM that reads it back (MFMA-bound at the f32 rate). Here a
// persistent grid (two 4-wave workgroups per CU, so one group's staging overlaps the other
// group's MFMAs instead of both waves of a SIMD stalling at the same barrier) owns
// contiguous ranges of 32-pixel blocks of the flattened B·Ho·Wo pixel axis, walked as tiles
// of 2 blocks (64 pixels, tiles may straddle images) × OT output channels. Per tile and k
// step (32 channels of one tap; taps inner, so the 9 taps of a channel slice re-read the
// same 128-B corner rows from L2):
//   * the 64 × 32 column slice is gathered from the channels-last xT (four 128-B corner
//     rows per pixel, canonical bilerp -> bit-identical to K1's columns) into a
//     double-buffered LDS image, shared by the 4 waves as the MFMA B operand;
//   * each wave reads its 64 weight rows × 32 k straight from L2 into registers (the A
//     operand, prefetched one step ahead; no wave shares them, so no LDS round trip);
//   * each wave runs 32x32x2 f32 MFMAs over its 2 × 2 (O, pixel) blocks on the other LDS
//     buffer.
// Block ranges of 12-13 blocks per workgroup keep the tail to one block (config 3: 6,272
// blocks over 512 workgroups). The columns are still written (non-temporal, off the
// critical path: the kernel is MFMA-bound and HBM is otherwise idle) because the ∂W GEMM
// of the backward reads them.
//
// MFMA operand order: in step j of a 32-wide k slice, lane (i, h = lane/32) feeds
// k = 16h + j, so each lane's 16 A values (one 64-B L2 read) and 16 B values (4
// ds_read_b128, conflict-free with a 36-float row stride) are contiguous. The sum over the
// 32 k is the same set of products in a fixed order: deterministic run to run.
#include "dcn_device.h"

namespace dcn {
namespace {

constexpr int kFK = 32;          // k per step
constexpr int kFS = 36;          // LDS row stride in floats (144 B: conflict-free b128 reads)
constexpr int kFThreads = 256;   // 4 waves
constexpr int kFWG = 2;          // workgroups per CU
constexpr int kFTaps = 9;        // tap records staged per tile (N <= 9)
constexpr int kFBlk = 32;        // pixels per MFMA block
constexpr int kFTB = 2;          // blocks per tile
constexpr int kFP = kFBlk * kFTB;                 // 64 pixels per tile
constexpr int kFU = kFP * (kFK / 4) / kFThreads;  // staging units (pixel, 4 ch) per thread
static_assert(kFU == 2, "staging layout");

__device__ __forceinline__ float4 bilerp4f(float fr, float fc, float4 a, float4 b, float4 c,
                                           float4 d) {
  return make_float4(bilerp(fr, fc, a.x, b.x, c.x, d.x), bilerp(fr, fc, a.y, b.y, c.y, d.y),
                     bilerp(fr, fc, a.z, b.z, c.z, d.z), bilerp(fr, fc, a.w, b.w, c.w, d.w));
}

// Workgroup barrier that orders LDS only: __syncthreads()'s fence would also drain the
// non-temporal column stores (vmcnt(0)) every k step, ≈ a store round trip per step.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool V>
struct Flag {
  static constexpr bool value = V;
};

// OT output channels per tile: each wave owns 64 of them (two 32-row MFMA blocks); 256 ->
// 4 waves along O x 2 pixel blocks each, 128 -> 2 along O x 2 along pixels x 1 block.
// Grid (nwg, O / OT); workgroup x owns 32-px blocks [nblk·x/nwg, nblk·(x+1)/nwg).
template <int OT>
__global__ __launch_bounds__(kFThreads) __attribute__((amdgpu_waves_per_eu(kFWG, kFWG))) void fwd_fused(Geo g, const float* __restrict__ xT,
                                                       const float* __restrict__ off,
                                                       const float* __restrict__ Wf,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ out,
                                                       float* __restrict__ colT, int nblk) {
  constexpr int WO = OT / 64;    // waves along O
  constexpr int WP = 4 / WO;     // waves along pixels
  constexpr int PB = kFTB / WP;  // pixel blocks per wave
  static_assert(WO * WP == kFThreads / 64 && PB >= 1, "wave layout");
  __shared__ float Cs[2][kFP * kFS];
  __shared__ int4 rec[kFP * kFTaps];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Block3 blk = xcd_block();
  const int nwg = gridDim.x;
  const int bl0 = (int)((long)nblk * blk.x / nwg), bl1 = (int)((long)nblk * (blk.x + 1) / nwg);
  const int o0 = blk.y * OT;
  const long P = (long)g.B * g.HW;
  const int nsteps = g.N * (g.C / kFK);

  // MFMA roles: O rows o0 + wo*64 + [0, 64), pixel blocks pb0 .. pb0+PB-1 of the tile
  const int wo = wave % WO, pb0 = (wave / WO) * PB;
  const int li = lane & 31, lh = lane >> 5;
  const float* wrow = Wf + (size_t)(o0 + wo * 64 + li) * g.K + lh * 16;
  const size_t wblk = (size_t)32 * g.K;  // second O block of the wave
  // staging roles: pixels sp and sp + 32 of the tile, channels 4*sq..4*sq+3 of the slice
  const int sp = tid >> 3, sq = tid & 7;

  for (int t0 = bl0; t0 < bl1; t0 += kFTB) {
    const int nb = min(kFTB, bl1 - t0);  // live blocks (workgroup-uniform)
    const long p0 = (long)t0 * kFBlk;
    // tap records of the tile's pixels x N taps (deform_conv.py:58-68 via sample_tap). The
    // previous tile's last reads of rec / Cs precede the barrier that ended its last step.
    for (int s = tid; s < kFP * g.N; s += kFThreads) {
      const int tp = s / g.N, n = s - tp * g.N;
      const long p = p0 + tp;
      int4 r = make_int4(INT_MIN, 0, 0, 0);
      if (tp < nb * kFBlk && p < P) {
        const int b = (int)(p / g.HW), m = (int)(p - (long)b * g.HW);
        const Tap t = sample_tap(g, off, b, 0, n, m);
        if (t.ok) r = make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc));
      }
      rec[tp * kFTaps + n] = r;
    }
    const float* xb[kFU];
    float* colrow[kFU];
#pragma unroll
    for (int u = 0; u < kFU; ++u) {
      const int tp = sp + 32 * u;
      const long p = p0 + tp;
      const bool ok = tp < nb * kFBlk && p < P;
      const int b = ok ? (int)(p / g.HW) : 0;
      xb[u] = xT + (size_t)b * g.HWi * g.C + sq * 4;
      colrow[u] = (colT && ok) ? colT + (size_t)p * g.K + sq * 4 : nullptr;
    }

    f32x16 acc[2][PB];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < PB; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][p][r] = 0.f;

    float4 ca[kFU], cb[kFU], cc[kFU], cd[kFU];
    float sfr[kFU], sfc[kFU];
    int okm[kFU];
    f32x4 a[2][4];

    // step s: channel slice cs = s / N (outer), tap n = s % N (inner); k0 = n·C + 32·cs
    auto wptr = [&](int s) {
      const int cs = s / g.N, n = s - cs * g.N;
      return wrow + n * g.C + cs * kFK;
    };
    // weight quads q0, q0+1 of both O blocks of step s (the A operand, from L2)
    auto load_a = [&](const float* wp, int q0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = q0; q < q0 + 2; ++q)
          a[j][q] = *reinterpret_cast<const f32x4*>(wp + j * wblk + 4 * q);
    };
    auto gather = [&](int s) {
      const int cs = s / g.N, n = s - cs * g.N;
      const int c0 = cs * kFK;
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        const int4 r = rec[(sp + 32 * u) * kFTaps + n];
        const bool lv = r.x != INT_MIN;
        const int r0 = lv ? r.x : 0, q0 = r.y;
        sfr[u] = __int_as_float(r.z);
        sfc[u] = __int_as_float(r.w);
        // corner validity bits (a, b, c, d); the loads read clamped in-image addresses
        // unconditionally (no exec branches) and the store zeroes invalid corners
        const bool r0ok = lv && r0 >= 0, r1ok = lv && r0 + 1 < g.H;
        const bool c0ok = q0 >= 0, c1ok = q0 + 1 < g.W;
        okm[u] = (lv ? 16 : 0) | ((r0ok && c0ok) ? 1 : 0) | ((r0ok && c1ok) ? 2 : 0) |
                 ((r1ok && c0ok) ? 4 : 0) | ((r1ok && c1ok) ? 8 : 0);
        const int ra = min(max(r0, 0), g.H - 1), rb = min(r0 + 1, g.H - 1);
        const int qa = min(max(q0, 0), g.W - 1), qb = min(max(q0 + 1, 0), g.W - 1);
        const float* base = xb[u] + c0;
        ca[u] = *reinterpret_cast<const float4*>(base + (ra * g.W + qa) * g.C);
        cb[u] = *reinterpret_cast<const float4*>(base + (ra * g.W + qb) * g.C);
        cc[u] = *reinterpret_cast<const float4*>(base + (rb * g.W + qa) * g.C);
        cd[u] = *reinterpret_cast<const float4*>(base + (rb * g.W + qb) * g.C);
      }
    };
    auto store = [&](int s, int buf) {
      const int cs = s / g.N, n = s - cs * g.N;
      const int k0 = n * g.C + cs * kFK;
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        const int m = okm[u];
        const float4 v = (m & 16) ? bilerp4f(sfr[u], sfc[u], (m & 1) ? ca[u] : z,
                                             (m & 2) ? cb[u] : z, (m & 4) ? cc[u] : z,
                                             (m & 8) ? cd[u] : z)
                                  : z;
        *reinterpret_cast<float4*>(&Cs[buf][(sp + 32 * u) * kFS + sq * 4]) = v;
        if (colrow[u])
          __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w},
                                      reinterpret_cast<f32x4*>(colrow[u] + k0));
      }
    };
    // the MFMAs of one step on LDS buffer buf, quad-major; with wn != nullptr each half of
    // the A registers is reloaded for the next step as soon as its last MFMA has issued
    auto mfma = [&](int buf, auto full, const float* wn) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int p = 0; p < PB; ++p) {
          if (!decltype(full)::value && pb0 + p >= nb) break;
          const f32x4 bq = *reinterpret_cast<const f32x4*>(
              &Cs[buf][((pb0 + p) * kFBlk + li) * kFS + lh * 16 + 4 * q]);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[j][p] = mfma32(a[j][q][e], bq[e], acc[j][p]);
        }
        if (wn && (q & 1)) load_a(wn, q - 1);
      }
    };
    auto steps = [&](auto full) {
      load_a(wptr(0), 0);
      load_a(wptr(0), 2);
      gather(0);
      store(0, 0);
      lds_barrier();
      // steps 0 .. nsteps-2 stage step s+1 beside the MFMAs of step s; the last step is
      // peeled so the loop body has no conditional loads
      for (int s = 0; s + 1 < nsteps; ++s) {
        const int buf = s & 1;
        gather(s + 1);
        mfma(buf, full, wptr(s + 1));
        store(s + 1, buf ^ 1);
        lds_barrier();
      }
      mfma((nsteps - 1) & 1, full, nullptr);
    };

    lds_barrier();  // records
    if (nb == kFTB)
      steps(Flag<true>{});
    else
      steps(Flag<true>{});

    // epilogue: D[i][j] of a 32x32 block sits in lane j + 32·((i/4)%2), register
    // 4·(i/8) + i%4; rows are output channels, columns pixels (128-B row segments)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ob = o0 + wo * 64 + j * 32 + 4 * lh;
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) bv[r] = bias ? bias[ob + 8 * (r >> 2) + (r & 3)] : 0.f;
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        if (pb0 + p >= nb) break;
        const long pf = p0 + (pb0 + p) * kFBlk + li;
        if (pf >= P) continue;
        const int b = (int)(pf / g.HW), m = (int)(pf - (long)b * g.HW);
        float* dst = out + (size_t)b * g.O * g.HW + m;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dst[(size_t)(ob + 8 * (r >> 2) + (r & 3)) * g.HW] = acc[j][p][r] + bv[r];
      }
    }
  }
}

}  // namespace

bool fused_fwd_ok(const Geo& g) {
  return g.dt == DCN_F32 && g.G == 1 && g.N <= kFTaps && g.C % kFK == 0 && g.O % 128 == 0 &&
         (long)g.HWi * g.C < (1l << 31);
}

static int g_fused_wg = 0;  // dcn_debug_fused_workgroups
void set_fused_workgroups(int n) { g_fused_wg = n; }

// r01 at config 3: fused 2.51 ms against K1 0.40 + GEMM 1.66 + bias 0.06 ms unfused.
bool fused_fwd_pays(const Geo& g) {
  (void)g;
  return false;
}

hipError_t launch_fused_fwd(const Geo& g, const float* xT, const float* off, const float* Wf,
                            const float* bias, float* out, float* colT, hipStream_t s) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  const long P = (long)g.B * g.HW;
  const int nblk = (int)((P + kFBlk - 1) / kFBlk);
  const int OT = g.O % 256 == 0 ? 256 : 128;
  const int tiles_o = g.O / OT;
  const int want = g_fused_wg > 0 ? g_fused_wg : std::max(1, kFWG * cus / tiles_o);
  const int nwg = std::max(1, std::min(nblk, want));
  if (OT == 256)
    hipLaunchKernelGGL(fwd_fused<256>, dim3(nwg, tiles_o), dim3(kFThreads), 0, s, g, xT, off,
                       Wf, bias, out, colT, nblk);
  else
    hipLaunchKernelGGL(fwd_fused<128>, dim3(nwg, tiles_o), dim3(kFThreads), 0, s, g, xT, off,
                       Wf, bias, out, colT, nblk);
  return hipGetLastError();
}

}  // namespace dcn
