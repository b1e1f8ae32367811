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

// ---------------------------------------------------------------------------
// DCN_BF16 fused forward on v_mfma_f32_32x32x16_bf16. The bf16 vendor GEMM is not
// MFMA-bound here but bound by re-reading the 2·B·HW·K-byte column matrix K1 just wrote
// (config 4: 231 MB), so the fusion pays at bf16 where at fp32 it did not.
//   * workgroup = 64 consecutive pixels of the flattened B·Ho·Wo axis x 256 output
//     channels; wave w owns output rows 64w..64w+63 (2 M-blocks) x the 64 pixels
//     (2 N-blocks): 4 fp32 accumulators;
//   * k step = 32 channels of one tap (channel slice outer, taps inner: the 9 taps of a
//     slice re-read the same corner rows from L1); a thread gathers 8 channels of one
//     pixel's four corners (16-B bf16 reads), forms the canonical fp32 bilerp, rounds to
//     bf16 (the very bits K1 writes) into a double-buffered LDS slice [px][32 k] — the B
//     operand — and, when colT is given, stores the same 16 B to the columns the ∂W GEMM
//     of the backward reads;
//   * A = the flat weight in MFMA fragment order (wf_to_frag_bf16), one contiguous 1 KiB
//     per wave load from L2, a step ahead in registers;
//   * epilogue: + bias, bf16 rounding (the unfused path's launch_bias_to_bf16 arithmetic).
// ---------------------------------------------------------------------------
constexpr int kBNB = 2;         // 32-px MFMA blocks per tile (4: 128-px tiles, 389 VGPRs, 282 us at config 4)
constexpr int kBP = 32 * kBNB;  // pixels per tile
constexpr int kBS = 40;         // LDS pitch (bf16) of a pixel's 32-k slice (80 B: b128 reads conflict-free)
constexpr int kGD = 2;          // gather ring depth (steps of corner loads in flight); even

typedef __bf16 bf16x8f_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8f_t ld_frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8f_t, *reinterpret_cast<const uint4*>(p));
}

// wf[((ob·NKS + ks)·64 + l)·8 + e] = Wf[32ob + (l&31)][16ks + 8(l>>5) + e], NKS = K/16
__global__ __launch_bounds__(256) void wf_to_frag_bf16(const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ wf, int O, int K) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)O * K) return;
  const int e = (int)(i & 7), l = (int)((i >> 3) & 63);
  const long obks = i >> 9;
  const int NKS = K / 16, ob = (int)(obks / NKS), ks = (int)(obks - (long)ob * NKS);
  wf[i] = w[(size_t)(32 * ob + (l & 31)) * K + 16 * ks + 8 * (l >> 5) + e];
}

__device__ __forceinline__ float bfl(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bfh(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

__global__ __launch_bounds__(256) void fwd_fused_bf16(Geo g, const bf16_t* __restrict__ xT,
                                                     const float* __restrict__ off,
                                                     const bf16_t* __restrict__ wf,
                                                     const float* __restrict__ bias,
                                                     bf16_t* __restrict__ out,
                                                     bf16_t* __restrict__ colT) {
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][kBP * kBS];
  __shared__ int4 rec[kBP * kFTaps];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Block3 blk = xcd_block();
  const long P = (long)g.B * g.HW;
  const long p0 = (long)blk.x * kBP;
  const int ob0 = blk.y * 8 + wave * 2;  // this wave's first 32-row output block
  const int nsteps = g.N * (g.C / 32), NKS = g.K / 16;
  for (int s = tid; s < kBP * g.N; s += 256) {
    const int tp = s / g.N, n = s - tp * g.N;
    const long p = p0 + tp;
    int4 r = make_int4(INT_MIN, 0, 0, 0);
    if (p < P) {
      const int b = (int)(p / g.HW), m = (int)(p - (long)b * g.HW);
      const Tap t = sample_tap(g, off, b, 0, n, m);
      if (t.ok) r = make_int4(t.r0, t.c0, __float_as_int(t.fr), __float_as_int(t.fc));
    }
    rec[tp * kFTaps + n] = r;
  }
  // staging roles: pixels sp + 64u of the tile, channels 8sq..8sq+7 of the step's slice
  constexpr int kU = kBP / 64;
  const int sp = tid >> 2, sq = tid & 3;
  const char* xc[kU];
  unsigned colrow[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const long ps = p0 + sp + 64 * u;
    const bool pv = ps < P;
    const int bs = pv ? (int)(ps / g.HW) : 0;
    xc[u] = reinterpret_cast<const char*>(xT) + (size_t)bs * g.HWi * g.C * 2 + sq * 16;
    colrow[u] = pv ? (unsigned)(((size_t)ps * g.K + sq * 8) * 2) : ~0u;
  }
  const unsigned rowb = (unsigned)g.W * g.C * 2u, pixb = (unsigned)g.C * 2u;
  const __amdgpu_buffer_rsrc_t col_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      colT, 0, colT ? (int)((size_t)P * g.K * 2) : 0, 0x00020000);

  f32x16 acc[2][kBNB];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int q = 0; q < kBNB; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][q][r] = 0.f;
  // gathered corners of a step, two steps in flight (register sets G[0], G[1])
  struct Gath {
    uint4 a, b, c, d;
    float fr, fc;
    int okm;
  };
  Gath G[kGD][kU];
  bf16x8f_t a[2][2][2];  // [register set][output block][16-k half]

  auto kbase = [&](int s) {
    const int cs = s / g.N, n = s - cs * g.N;
    return n * g.C + 32 * cs;
  };
  auto load_a = [&](int s, int d) {
    const int ks = kbase(min(s, nsteps - 1)) / 16;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        a[d][j][h] = ld_frag(wf + ((size_t)((ob0 + j) * NKS + ks + h) * 64 + lane) * 8);
  };
  auto gather1 = [&](int s0, int u, Gath& q) {
    const int s = min(s0, nsteps - 1);  // past the last step: a harmless re-gather
    const int cs = s / g.N, n = s - cs * g.N;
    const int4 r = rec[(sp + 64 * u) * kFTaps + n];
    const bool lv = r.x != INT_MIN;
    const int r0 = lv ? r.x : 0, q0 = r.y;
    q.fr = __int_as_float(r.z);
    q.fc = __int_as_float(r.w);
    // corner validity bits; the loads read clamped in-image addresses unconditionally
    const bool r0ok = lv && r0 >= 0, r1ok = lv && r0 + 1 < g.H;
    const bool c0ok = q0 >= 0, c1ok = q0 + 1 < g.W;
    q.okm = (lv ? 16 : 0) | ((r0ok && c0ok) ? 1 : 0) | ((r0ok && c1ok) ? 2 : 0) |
            ((r1ok && c0ok) ? 4 : 0) | ((r1ok && c1ok) ? 8 : 0);
    const int ra = min(max(r0, 0), g.H - 1), rb = min(r0 + 1, g.H - 1);
    const int qa = min(max(q0, 0), g.W - 1), qb = min(max(q0 + 1, 0), g.W - 1);
    const char* base = xc[u] + cs * 64;
    q.a = *reinterpret_cast<const uint4*>(base + ((unsigned)ra * rowb + (unsigned)qa * pixb));
    q.b = *reinterpret_cast<const uint4*>(base + ((unsigned)ra * rowb + (unsigned)qb * pixb));
    q.c = *reinterpret_cast<const uint4*>(base + ((unsigned)rb * rowb + (unsigned)qa * pixb));
    q.d = *reinterpret_cast<const uint4*>(base + ((unsigned)rb * rowb + (unsigned)qb * pixb));
  };
  auto store1 = [&](int s, int buf, int u, const Gath& q) {
    const int m = q.okm;
    const unsigned za = (m & 1) ? ~0u : 0u, zb = (m & 2) ? ~0u : 0u;
    const unsigned zc = (m & 4) ? ~0u : 0u, zd = (m & 8) ? ~0u : 0u;
    const unsigned A4[4] = {q.a.x & za, q.a.y & za, q.a.z & za, q.a.w & za};
    const unsigned B4[4] = {q.b.x & zb, q.b.y & zb, q.b.z & zb, q.b.w & zb};
    const unsigned C4[4] = {q.c.x & zc, q.c.y & zc, q.c.z & zc, q.c.w & zc};
    const unsigned D4[4] = {q.d.x & zd, q.d.y & zd, q.d.z & zd, q.d.w & zd};
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = bilerp(q.fr, q.fc, bfl(A4[e]), bfl(B4[e]), bfl(C4[e]), bfl(D4[e]));
      const float hi = bilerp(q.fr, q.fc, bfh(A4[e]), bfh(B4[e]), bfh(C4[e]), bfh(D4[e]));
      o[e] = (m & 16) ? ((unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16)) : 0u;
    }
    const uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<uint4*>(&Bs[buf][(sp + 64 * u) * kBS + 8 * sq]) = v;
    if (colT)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, v), col_rsrc,
          (int)(colrow[u] == ~0u ? ~0u : colrow[u] + (unsigned)kbase(s) * 2u), 0, kAuxNT);
  };
  auto gather = [&](int s, Gath(&q)[kU]) {
#pragma unroll
    for (int u = 0; u < kU; ++u) gather1(s, u, q[u]);
  };
  auto store = [&](int s, int buf, const Gath(&q)[kU]) {
#pragma unroll
    for (int u = 0; u < kU; ++u) store1(s, buf, u, q[u]);
  };
  auto mfma = [&](int buf, int d) {
    // every B fragment of the step is read before the first MFMA (no LDS load may land in a
    // register an issued MFMA still reads)
    bf16x8f_t bv[2][kBNB];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < kBNB; ++q)
        bv[h][q] = ld_frag(&Bs[buf][(32 * q + (lane & 31)) * kBS + 16 * h + 8 * (lane >> 5)]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < kBNB; ++q)
          acc[j][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[d][j][h], bv[h][q], acc[j][q], 0, 0, 0);
  };
  // sched_barriers: the next steps' gathers and A loads are issued above a step's MFMA block
  // and the LDS staging below it
  auto mm = [&](int buf, int d) {
    __builtin_amdgcn_sched_barrier(0);
    mfma(buf, d);
    __builtin_amdgcn_sched_barrier(0);
  };
  // A step ends with a full __syncthreads(), i.e. with every wave's loads and stores drained
  // (vmcnt(0)), not an LDS-only barrier. Measured at config 4 (tools/fused_det.py): with
  // lds_barrier() (gathers, A loads and column stores left in flight across the barrier)
  // 0.01-3 % of the outputs differed from run to run in several schedules (ring depth 2 and
  // 4, with or without s_nop padding after the MFMAs), though no LDS hazard is visible in the
  // source; with the drain every run is bitwise identical to the unfused path.
  auto step_barrier = [&]() { __syncthreads(); };
  __syncthreads();  // records
#pragma unroll
  for (int d = 0; d < kGD; ++d) gather(d, G[d]);
  load_a(0, 0);
  store(0, 0, G[0]);
  step_barrier();
  // step s multiplies LDS buffer / A set s&1 after issuing the gather of step s+kGD into the
  // ring slot step s's corners left free (kGD steps of memory latency in flight); then step
  // s+1's corners (gathered kGD-1 steps earlier) are interpolated into the other LDS buffer.
  // Unrolled by kGD (even): ring slots, buffers and A sets are compile-time indices.
  for (int s0 = 0; s0 < nsteps; s0 += kGD) {
    bool done = false;
#pragma unroll
    for (int d = 0; d < kGD; ++d) {
      if (!done) {
        const int s = s0 + d;
        gather(s + kGD, G[d]);
        load_a(s + 1, (d + 1) & 1);
        mm(d & 1, d & 1);
        if (s + 1 >= nsteps) {
          done = true;  // workgroup-uniform
        } else {
          store(s + 1, (d + 1) & 1, G[(d + 1) % kGD]);
          step_barrier();
        }
      }
    }
    if (done) break;
  }
  // D[row o][col px]: register r of lane (c = lane&31, hh) = row (r&3) + 8(r>>2) + 4hh
#pragma unroll
  for (int q = 0; q < kBNB; ++q) {
    const long pf = p0 + 32 * q + (lane & 31);
    if (pf >= P) continue;
    const int b = (int)(pf / g.HW), m = (int)(pf - (long)b * g.HW);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = 32 * (ob0 + j) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        out[((size_t)b * g.O + o) * g.HW + m] = f2bf(acc[j][q][r] + (bias ? bias[o] : 0.f));
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
  // shape 1 measured faster at config 3 (2.49 against 2.91 ms); DCN_EXP slot 8 = 1 picks 0
  const int cfg = exp_flag(8) == 1 ? 0 : 1;
  const int wgcu = cfg == 0 ? FCfg<0>::WGCU : FCfg<1>::WGCU;
  const int want = g_fused_wg > 0 ? g_fused_wg : std::max(1, wgcu * cus / tiles_o);
  const dim3 grid(std::max(1, std::min(nblk, want)), tiles_o);
#define DCN_FUSED_LAUNCH(OT_, CFG_)                                                          \
  hipLaunchKernelGGL((fwd_fused<OT_, CFG_>), grid, dim3(FCfg<CFG_>::T), 0, s, g, xT, off, Wf, \
                     bias, out, colT, nblk)
  if (OT == 256 && cfg == 0)
    DCN_FUSED_LAUNCH(256, 0);
  else if (OT == 256)
    DCN_FUSED_LAUNCH(256, 1);
  else if (cfg == 0)
    DCN_FUSED_LAUNCH(128, 0);
  else
    DCN_FUSED_LAUNCH(128, 1);
#undef DCN_FUSED_LAUNCH
  return hipGetLastError();
}


bool fused_bf16_ok(const Geo& g) {
  return g.dt == DCN_BF16 && g.G == 1 && g.N <= kFTaps && g.C % 32 == 0 && g.O % 256 == 0 &&
         (size_t)g.B * g.HWi * g.C * 2 < (1ull << 31) && (size_t)g.B * g.HW * g.K * 2 < (1ull << 31);
}
size_t fused_bf16_wf_elems(const Geo& g) { return (size_t)g.O * g.K; }
// DCN_EXP slot 12 = 1 lets AUTO pick the bf16 fused forward (A/B until measured)
bool fused_bf16_pays(const Geo& g) { return fused_bf16_ok(g) && exp_flag(12) == 1; }

hipError_t launch_fused_fwd_bf16(const Geo& g, const bf16_t* xT, const float* off, const bf16_t* w,
                                 const float* bias, bf16_t* out, bf16_t* colT, bf16_t* wf,
                                 hipStream_t s) {
  if (!fused_bf16_ok(g)) return hipErrorInvalidValue;
  const long n = (long)g.O * g.K;
  hipLaunchKernelGGL(wf_to_frag_bf16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, wf,
                     g.O, g.K);
  const long P = (long)g.B * g.HW;
  hipLaunchKernelGGL(fwd_fused_bf16, dim3((unsigned)((P + kBP - 1) / kBP), g.O / 256), dim3(256),
                     0, s, g, xT, off, wf, bias, out, colT);
  return hipGetLastError();
}
}  // namespace dcn
