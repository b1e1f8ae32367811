// dcn_fused.hip — fused deformable forward: the bilinear im2col of
// deform_conv.py:41-54,72-73 gathered straight into the LDS operand tiles of an f32 MFMA
// GEMM against the flat weight (:74-76), with the bias of :77-80 in the epilogue.
//
//   out[b][o][m] = bias[o] + Σ_k Wf[o][k] · col[b][m][k],   k = n·C + c   (Q5)
//
// The separate path is K1 (im2col_lds, HBM-bound: it writes the 1.85 GB column matrix)
// followed by a vendor GEMM that reads it back (MFMA-bound at the f32 rate). Here a
// persistent grid owns contiguous ranges of 32-pixel blocks of the flattened B·Ho·Wo pixel
// axis (tiles may straddle images; ranges differ by at most one block), walked as tiles of
// TB blocks × OT output channels. Per tile and k step (32 channels of one tap; taps inner,
// so the taps of a channel slice re-read the same 128-B corner rows from L1/L2):
//   * the tile's column slice is gathered from the channels-last xT (four 128-B corner
//     rows per pixel, clamped addresses, invalid corners zeroed, canonical bilerp ->
//     bit-identical to K1's columns) into a double-buffered LDS image, the MFMA B operand
//     shared by the workgroup's waves;
//   * each wave reads its weight rows × 32 k straight from L2 into registers (the A
//     operand; each half reloaded for the next step once its last MFMA has issued; no wave
//     shares rows, so no LDS round trip);
//   * each wave runs 32x32x2 f32 MFMAs over its (O, pixel) blocks on the other LDS buffer;
//   * an LDS-only barrier ends the step (no vmcnt drain of the column stores).
// The columns are still written (buffer stores, non-temporal; rows outside the tile fall
// past the descriptor's range and are dropped) because the ∂W GEMM of the backward reads
// them. Two workgroup shapes (FCfg); measured, the fused kernel is still slower than K1 +
// the vendor GEMM, so DCN_FWD_AUTO does not pick it.
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
constexpr int kFTaps = 9;        // tap records staged per tile (N <= 9)
constexpr int kFBlk = 32;        // pixels per MFMA block
constexpr int kFU = 2;           // staging units (pixel, 4 channels) per thread and step

// Workgroup shapes (both two waves per SIMD; DESIGN.md §4.7 has the measurements):
//   0: 4 waves, 2 workgroups per CU, 64-px tiles, 64 output rows per wave;
//   1: 8 waves, 1 workgroup per CU, 128-px tiles, 32 output rows per wave.
template <int CFG>
struct FCfg {
  static constexpr int T = CFG == 0 ? 256 : 512;  // threads
  static constexpr int WGCU = CFG == 0 ? 2 : 1;   // workgroups per CU
  static constexpr int TB = CFG == 0 ? 2 : 4;     // 32-px blocks per tile
  static constexpr int RW = CFG == 0 ? 64 : 32;   // output rows per wave
  static constexpr int P = kFBlk * TB;            // pixels per tile
  static constexpr int JB = RW / 32;              // 32-row O blocks per wave
  static constexpr int US = T / 8;                // pixel stride between a thread's units
  static_assert(P * (kFK / 4) == kFU * T, "staging layout");
};

__device__ __forceinline__ float4 bilerp4f(float fr, float fc, float4 a, float4 b, float4 c,
                                           float4 d) {
  return make_float4(bilerp(fr, fc, a.x, b.x, c.x, d.x), bilerp(fr, fc, a.y, b.y, c.y, d.y),
                     bilerp(fr, fc, a.z, b.z, c.z, d.z), bilerp(fr, fc, a.w, b.w, c.w, d.w));
}


typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kAuxNT = 2;  // buffer-op cache policy: non-temporal (the columns are streamed)

template <bool V>
struct Flag {
  static constexpr bool value = V;
};

// OT output channels per tile: each wave owns 64 of them (two 32-row MFMA blocks); 256 ->
// 4 waves along O x 2 pixel blocks each, 128 -> 2 along O x 2 along pixels x 1 block.
// Grid (nwg, O / OT); workgroup x owns 32-px blocks [nblk·x/nwg, nblk·(x+1)/nwg).
template <int OT, int CFG>
__global__ __launch_bounds__(FCfg<CFG>::T) __attribute__((amdgpu_waves_per_eu(2, 2))) void
fwd_fused(Geo g, const float* __restrict__ xT, const float* __restrict__ off,
          const float* __restrict__ Wf, const float* __restrict__ bias, float* __restrict__ out,
          float* __restrict__ colT, int nblk) {
  using C = FCfg<CFG>;
  constexpr int kFThreads = C::T, kFTB = C::TB, kFP = C::P, JB = C::JB;
  constexpr int WO = OT / C::RW;              // waves along O
  constexpr int WP = (kFThreads / 64) / WO;   // waves along pixels
  constexpr int PB = kFTB / WP;               // pixel blocks per wave
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
  // 32-bit byte offsets against wave-uniform bases (global_load saddr form: one VGPR per
  // address; fused_fwd_ok bounds every tensor below 4 GiB)
  const unsigned wrow = ((unsigned)(o0 + wo * C::RW + li) * g.K + lh * 16) * 4u;
  const unsigned wblk = 32u * g.K * 4u;  // second O block of the wave
  // staging roles: pixels sp and sp + US of the tile, channels 4*sq..4*sq+3 of the slice
  const int sp = tid >> 3, sq = tid & 7;
  // columns for the ∂W GEMM (none when colT is null: zero records, every store dropped)
  const __amdgpu_buffer_rsrc_t col_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      colT, 0, colT ? (int)((unsigned)P * g.K * 4u) : 0, 0x00020000);

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
    // byte offsets into xT / colT; a column row outside the tile is stored at ~0u, past the
    // descriptor's range, which the buffer store drops (branch-free staging)
    unsigned xb[kFU], colrow[kFU];
#pragma unroll
    for (int u = 0; u < kFU; ++u) {
      const int tp = sp + C::US * u;
      const long p = p0 + tp;
      const bool ok = tp < nb * kFBlk && p < P;
      const int b = ok ? (int)(p / g.HW) : 0;
      xb[u] = ((unsigned)b * g.HWi * g.C + sq * 4) * 4u;
      colrow[u] = ok ? ((unsigned)p * g.K + sq * 4) * 4u : ~0u;
    }

    f32x16 acc[JB][PB];
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int p = 0; p < PB; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][p][r] = 0.f;

    float4 ca[kFU], cb[kFU], cc[kFU], cd[kFU];
    float sfr[kFU], sfc[kFU];
    int okm[kFU];
    f32x4 a[JB][4];

    // step s: channel slice cs = s / N (outer), tap n = s % N (inner); k0 = n·C + 32·cs
    auto wptr = [&](int s) {
      const int cs = s / g.N, n = s - cs * g.N;
      return wrow + (unsigned)(n * g.C + cs * kFK) * 4u;
    };
    // weight quads q0, q0+1 of both O blocks of step s (the A operand, from L2)
    auto load_a = [&](unsigned wp, int q0) {
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int q = q0; q < q0 + 2; ++q)
          a[j][q] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(Wf) +
                                                    (wp + j * wblk + 16 * q));
    };
    auto gather = [&](int s) {
      const int cs = s / g.N, n = s - cs * g.N;
      const int c0 = cs * kFK;
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        const int4 r = rec[(sp + C::US * u) * kFTaps + n];
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
        const char* xc = reinterpret_cast<const char*>(xT);
        const unsigned base = xb[u] + c0 * 4u, rowb = (unsigned)g.W * g.C * 4u;
        const unsigned oa = base + (unsigned)ra * rowb, ob = base + (unsigned)rb * rowb;
        const unsigned ea = (unsigned)qa * g.C * 4u, eb = (unsigned)qb * g.C * 4u;
        ca[u] = *reinterpret_cast<const float4*>(xc + (oa + ea));
        cb[u] = *reinterpret_cast<const float4*>(xc + (oa + eb));
        cc[u] = *reinterpret_cast<const float4*>(xc + (ob + ea));
        cd[u] = *reinterpret_cast<const float4*>(xc + (ob + eb));
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
        *reinterpret_cast<float4*>(&Cs[buf][(sp + C::US * u) * kFS + sq * 4]) = v;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, f32x4{v.x, v.y, v.z, v.w}), col_rsrc,
            (int)(colrow[u] == ~0u ? ~0u : colrow[u] + k0 * 4u), 0, kAuxNT);
      }
    };
    // the MFMAs of one step on LDS buffer buf, quad-major; with wn != ~0u each half of
    // the A registers is reloaded for the next step as soon as its last MFMA has issued
    auto mfma = [&](int buf, auto full, unsigned wn) {
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
            for (int j = 0; j < JB; ++j) acc[j][p] = mfma32(a[j][q][e], bq[e], acc[j][p]);
        }
        if (wn != ~0u && (q & 1)) load_a(wn, q - 1);
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
      mfma((nsteps - 1) & 1, full, ~0u);
    };

    lds_barrier();  // records
    if (nb == kFTB)
      steps(Flag<true>{});
    else
      steps(Flag<false>{});

    // epilogue: D[i][j] of a 32x32 block sits in lane j + 32·((i/4)%2), register
    // 4·(i/8) + i%4; rows are output channels, columns pixels (128-B row segments)
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int ob = o0 + wo * C::RW + j * 32 + 4 * lh;
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) bv[r] = bias ? bias[ob + 8 * (r >> 2) + (r & 3)] : 0.f;
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        if (pb0 + p >= nb) break;
        const long pf = p0 + (pb0 + p) * kFBlk + li;
        if (pf >= P) continue;
        const int b = (int)(pf / g.HW), m = (int)(pf - (long)b * g.HW);
        const unsigned d0 = ((unsigned)(b * g.O + ob) * g.HW + m) * 4u;
        char* oc = reinterpret_cast<char*>(out);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          *reinterpret_cast<float*>(
              oc + (d0 + (unsigned)((8 * (r >> 2) + (r & 3)) * g.HW) * 4u)) = acc[j][p][r] + bv[r];
      }
    }
  }
}

}  // namespace

bool fused_fwd_ok(const Geo& g) {
  const long lim = 1l << 30;  // elements: 32-bit byte offsets (4 GiB)
  return g.dt == DCN_F32 && g.G == 1 && g.N <= kFTaps && g.C % kFK == 0 && g.O % 128 == 0 &&
         (long)g.B * g.HWi * g.C < lim && (long)g.B * g.HW * g.K < lim / 2 &&
         (long)g.O * g.K < lim && (long)g.B * g.O * g.HW < lim;
}

static int g_fused_wg = 0;  // dcn_debug_fused_workgroups
void set_fused_workgroups(int n) { g_fused_wg = n; }

// r01 at config 3: fused 2.49 ms (shape 1) against K1 0.40 + GEMM 1.65 + bias 0.06 ms
// unfused, so DCN_FWD_AUTO keeps the unfused schedule.
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
  // shape 1 (FCfg<1>) measured faster at config 3: 2.49 against 2.91 ms for shape 0
  constexpr int cfg = 1;
  const int want = g_fused_wg > 0 ? g_fused_wg : std::max(1, FCfg<cfg>::WGCU * cus / tiles_o);
  const dim3 grid(std::max(1, std::min(nblk, want)), tiles_o);
#define DCN_FUSED_LAUNCH(OT_)                                                                \
  hipLaunchKernelGGL((fwd_fused<OT_, cfg>), grid, dim3(FCfg<cfg>::T), 0, s, g, xT, off, Wf,   \
                     bias, out, colT, nblk)
  if (OT == 256)
    DCN_FUSED_LAUNCH(256);
  else
    DCN_FUSED_LAUNCH(128);
#undef DCN_FUSED_LAUNCH
  return hipGetLastError();
}


}  // namespace dcn
