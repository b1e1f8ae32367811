"""CPU tests of the analysis tools the design record cites:
tools/isa_hazard_scan.py measures write-after-read distances in gfx950 ISA, and the model of
wave_sum8's lane schedule (csrc/dcn_device.h) reproduces wave_sum's bits.

The scanner is fed hand-written ISA with known pairs; the wave_sum8 model replays the DPP /
permlane data movement lane by lane in float32 (quad_perm, row_half_mirror, row_mirror,
row_ror, v_permlane16/32_swap as documented for gfx950) and checks every sum against the
one-value tree bit for bit. The hardware half of that claim is the bitwise A/B of K5 against
its r03 form on the GPU (profiles/r04_*); this is the schedule's arithmetic."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_hazard_scan as S  # noqa: E402

KERNEL = """\
_Z4testv:                               ; @_Z4testv
	global_load_dwordx4 v[4:7], v[0:1], off
	v_add_u32_e32 v0, 1, v0
	s_nop 3
	v_mov_b32_e32 v1, 0
	v_mfma_f32_16x16x32_bf16 v[8:11], v[12:15], v[16:19], v[8:11]
	v_mfma_f32_16x16x32_bf16 v[8:11], v[12:15], v[16:19], v[8:11]
	ds_read_b128 v[12:15], v20
	global_store_dword v[2:3], v21, off
	v_mov_b32_e32 v21, 5
	v_mov_b32_dpp v22, v23 row_newbcast:3 row_mask:0xf bank_mask:0xf
	s_endpgm
.Lfunc_end0:
"""


def _scan(text, window=8):
    (name, body), = list(S.kernels(text))
    assert name == "_Z4testv"
    return S.scan(body, window)


def test_hazard_scan_distances():
    hits, detail, lanegroup, n_mfma, n = _scan(KERNEL)
    # the load's address v[0:1]: v0 rewritten by the very next VALU (distance 0), v1 after
    # one instruction and an s_nop 3 (1 + 4 wait states)
    assert hits["vmem-addr <- valu"][0] == 1
    assert hits["vmem-addr <- valu"][5] == 1
    # the second MFMA re-reads its own C chain: no hazard; the DS return into the MFMAs'
    # A registers lands 0 instructions after the last MFMA
    assert "mfma-srcC <- mfma" not in hits
    assert hits["mfma-srcA <- ds"][0] == 1
    # 32-bit store data rewritten by the next VALU
    assert hits["vmem-data <- valu"][0] == 1
    assert lanegroup["v_mov_b32_dpp"] == 1
    assert n_mfma == 2 and n == 11  # s_endpgm included


def test_hazard_scan_window_bounds():
    hits, *_ = _scan(KERNEL, window=2)
    assert 5 not in hits["vmem-addr <- valu"]  # beyond the window


def test_resources_parse():
    text = KERNEL + "\t; NumVgprs: 24\n\t; NumAgprs: 0\n\t; ScratchSize: 0\n\t; Occupancy: 8\n"
    r = S.resources(text)["_Z4testv"]
    assert r["vgpr"] == 24 and r["agpr"] == 0 and r["scratch"] == 0 and r["occupancy"] == 8


# --- wave_sum8's lane schedule (dcn_device.h), replayed lane by lane ------------------------
L = np.arange(64)


def _dpp(v, ctrl):
    src = {0xB1: L ^ 1, 0x4E: L ^ 2, 0x141: (L & ~7) | (7 - (L & 7)),
           0x140: (L & ~15) | (15 - (L & 15)), 0x128: (L & ~15) | (((L & 15) + 8) & 15)}[ctrl]
    return v[src]


def _swap16(a, b):  # v_permlane16_swap: odd rows of a <-> even rows of b
    a2, b2 = a.copy(), b.copy()
    for r in (1, 3):
        a2[16 * r:16 * r + 16] = b[16 * (r - 1):16 * r]
        b2[16 * (r - 1):16 * r] = a[16 * r:16 * r + 16]
    return a2, b2


def _swap32(a, b):  # v_permlane32_swap: lanes 32-63 of a <-> lanes 0-31 of b
    a2, b2 = a.copy(), b.copy()
    a2[32:], b2[:32] = b[:32], a[32:]
    return a2, b2


def _wave_sum(v):
    f = np.float32
    v = v.astype(f)
    for c in (0xB1, 0x4E, 0x141, 0x140):
        v = (v + _dpp(v, c)).astype(f)
    s = [v[16 * r] for r in range(4)]  # each row holds its row sum; row_bcast:15 / :31 order
    return f(f(s[3] + s[2]) + f(s[1] + s[0]))


def _half_fold(hi, a, b, ctrl):
    keep, send = np.where(hi, b, a), np.where(hi, a, b)
    return (keep + _dpp(send, ctrl)).astype(np.float32)


def _wave_sum8(vals):
    b0, b1, b2 = (L & 1) != 0, (L & 2) != 0, (L & 4) != 0
    h1, h2 = b0 ^ b2, b1 ^ b2
    p = [_half_fold(h1, vals[i], vals[i + 4], 0xB1) for i in range(4)]
    q = [_half_fold(h2, p[j], p[j + 2], 0x4E) for j in range(2)]
    d = _half_fold(b2, q[0], q[1], 0x141)
    d = (d + _dpp(d, 0x128)).astype(np.float32)
    d = np.add(*_swap16(d, d), dtype=np.float32)
    return np.add(*_swap32(d, d), dtype=np.float32)


def _sum_lane(k):  # wave_sum8_lane
    return (((k >> 2) ^ k) & 1) | ((((k >> 1) ^ k) & 1) << 1) | ((k & 1) << 2)


def test_wave_sum8_schedule_matches_wave_sum_bitwise():
    rng = np.random.default_rng(8)
    for _ in range(300):
        vals = [(rng.standard_normal(64) * 10.0 ** rng.integers(-3, 4)).astype(np.float32)
                for _ in range(8)]
        d = _wave_sum8(vals)
        for k in range(8):
            want = _wave_sum(vals[k]).view(np.uint32)
            got = d[(L & 7) == _sum_lane(k)].view(np.uint32)  # every lane of value k
            assert np.all(got == want), k
