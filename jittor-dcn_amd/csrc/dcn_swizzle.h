// dcn_swizzle.h — the per-call weight re-layouts of the DCN_BF16 kernels as per-unit device
// functions, so that launch_prep_bf16 (dcn_reduce.hip) runs several of them, and the small
// fp32 conversions, as ONE launch per direction (r05: 3 + 3 launches of 4-6 µs each were
// 10 % of config 4's small-kernel time). Each kernel's own launcher still has a form that
// does its swizzle itself (geometries and callers that do not batch).
#pragma once
#include "dcn_device.h"

namespace dcn {

// offset conv forward (offset_conv_fwd_mfma_bf16[_row]): the B fragments in MFMA lane order,
// wb[((tap·NKS + ks)·64 + lane)·8 + e] = w_off[j = lane & 31][c = 16ks + 8(lane >> 5) + e][tap]
// (0 for j >= J or c >= C; NKS = Cp / 16); element i of KK·32·Cp
__device__ __forceinline__ void swz_tjc(const bf16_t* __restrict__ w, bf16_t* __restrict__ wb,
                                        int J, int C, int Cp, int KK, int i) {
  const int e = i & 7, lane = (i >> 3) & 63, tks = i >> 9;
  const int NKS = Cp / 16, t = tks / NKS, ks = tks - t * NKS;
  const int j = lane & 31, c = 16 * ks + 8 * (lane >> 5) + e;
  wb[i] = (j < J && c < C) ? w[((size_t)j * C + c) * KK + t] : (bf16_t)0;
}

// offset conv ∂x (offset_dgrad_bf16): Wc[c][k = t·J8 + j] = w_off[j][c][t] in A-fragment order,
// element e of lane l of k-step ks of 32-channel M-tile mt at wc[((mt·NKS + ks)·64 + l)·8 + e]
// (NKS = KT16 / 16); element i of C·KT16
__device__ __forceinline__ void swz_ck(const bf16_t* __restrict__ w, bf16_t* __restrict__ wc,
                                       int J, int J8, int C, int KK, int KT16, int i) {
  const int e = i & 7, l = (i >> 3) & 63, mks = i >> 9;
  const int NKS = KT16 / 16, mt = mks / NKS, ks = mks - mt * NKS;
  const int c = 32 * mt + (l & 31), k = 16 * ks + 8 * (l >> 5) + e;
  const int t = k / J8, j = k - t * J8;
  wc[i] = (t < KK && j < J) ? w[((size_t)j * C + c) * KK + t] : (bf16_t)0;
}

// fused forward (fwd_fused_bf16): wfr[ob][ks][lane][8] = Wf[16·ob + (lane & 15)][32·ks +
// 8·(lane >> 4) + e], the v_mfma_f32_16x16x32_bf16 A fragment; fragment f of O·K / 8 (16 B)
__device__ __forceinline__ void swz_frag16(const bf16_t* __restrict__ w, bf16_t* __restrict__ wfr,
                                           int K, long f) {
  const int l = (int)(f & 63);
  const long rest = f >> 6;
  const int NKS = K / 32, ob = (int)(rest / NKS), ks = (int)(rest - (long)ob * NKS);
  *reinterpret_cast<uint4*>(wfr + f * 8) = *reinterpret_cast<const uint4*>(
      w + (size_t)(16 * ob + (l & 15)) * K + 32 * ks + 8 * (l >> 4));
}

// ∂columns (dcol_bf16): accumulator row r = 8q + 4h + i of a 32x32 tile takes the A row of ∂col
// column 16h + 4q + i, so register j of a lane in half h is column 16h + j
__host__ __device__ constexpr int dc_perm(int r) {
  return 16 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3);
}
// wz[T][ks][lane][j] = Wf[o = 16ks + 8(lane >> 5) + j][k = 32T + dc_perm(lane & 31)] (O = 256:
// 16 k-steps); fragment i of (K / 32)·16·64 (16 B)
__device__ __forceinline__ void swz_dcol(const bf16_t* __restrict__ w, int K,
                                         bf16_t* __restrict__ wz, int i) {
  constexpr int kKS = 16;
  const int lane = i & 63, ks = (i >> 6) % kKS, T = (i >> 6) / kKS;
  const int k = 32 * T + dc_perm(lane & 31), o0 = 16 * ks + 8 * (lane >> 5);
  unsigned u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    u[j] = (unsigned)w[(size_t)(o0 + 2 * j) * K + k] |
           ((unsigned)w[(size_t)(o0 + 2 * j + 1) * K + k] << 16);
  reinterpret_cast<uint4*>(wz)[i] = make_uint4(u[0], u[1], u[2], u[3]);
}

}  // namespace dcn
