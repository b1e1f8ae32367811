"""Distance-based ISA hazard audit for gfx950 kernels (hipcc --cuda-device-only -S output).

  python tools/isa_hazard_scan.py [--window N] [--detail] file.s [file.s ...]

Per kernel, a straight-line scan in program order (labels and branches do not end a window;
a heuristic over-approximation, not a proof) for a WRITE of a VGPR that lands within N wait
states (an issued instruction counts 1, `s_nop k` counts k+1) of an earlier instruction that
still READS that VGPR (write-after-read):

  vmem-addr   the address VGPRs of a vector-memory instruction (global / buffer / flat /
              scratch load, store or atomic; LDS-DMA) rewritten by a later VALU result, a load
              return (VMEM or DS) or an accumulator move. A wave64 `global_load_dwordx4` hands
              its 64 lanes' addresses to the texture-address unit in four 16-lane groups, the
              last group (lanes 48-63) last; hipcc's hazard recognizer models no wait for a
              VALU rewrite of them (it pads only the cases listed in --model);
  vmem-data   the data VGPRs of a vector-memory store (> 64 bits: the documented
              store-data hazard, which hipcc pads) rewritten likewise;
  mfma-src    the A / B / C source VGPRs (or AGPRs) of an MFMA rewritten by anything but the
              next MFMA of the same accumulation chain;
  ds-addr     the address / data VGPRs of an LDS instruction rewritten likewise.

It also counts the instructions whose effect depends on the 16-lane group (DPP row_* / quad
operations, row_bcast, v_readlane / v_writelane, permlane, ds_bpermute / ds_swizzle, mbcnt),
since the r02 fused-forward corruption (profiles/r03_fused_diag*.txt) hit lanes 48-63 only.

The report per kernel: VGPR / AGPR / scratch / LDS from the .s metadata, the number of
instances of each class at each distance, and (--detail) the instruction pairs.
Test infrastructure only; DESIGN.md §4.7 has what it found."""
from __future__ import annotations

import argparse
import re
import sys
from collections import Counter, defaultdict

WINDOW = 8

VMEM = ("global_", "buffer_", "flat_", "scratch_")
DS = ("ds_",)


def vgprs(tok):
    """VGPR / AGPR numbers named by an operand token: ('v', n) / ('a', n) tuples."""
    tok = tok.strip(",")
    m = re.match(r"([va])\[(\d+):(\d+)\]$", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def kernels(text):
    cur, body, meta = None, [], {}
    for line in text.split("\n"):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if re.match(r"^\.Lfunc_end\d+:", line.strip()):  # the whole body (several s_endpgm)
            yield cur, body
            cur = None
            continue
        body.append(line)


def resources(text):
    """kernel -> {vgpr, agpr, sgpr, scratch, lds} from the .s metadata comments."""
    res = defaultdict(dict)
    cur = None
    for line in text.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
        if cur is None:
            continue
        for key, pat in (("vgpr", r"; NumVgprs: (\d+)"), ("agpr", r"; NumAgprs: (\d+)"),
                         ("sgpr", r"; NumSgprs: (\d+)"), ("scratch", r"; ScratchSize: (\d+)"),
                         ("lds", r"; LDSByteSize: (\d+)"), ("occupancy", r"; Occupancy: (\d+)")):
            mm = re.search(pat, line)
            if mm:
                res[cur][key] = int(mm.group(1))
    return res


class Ins:
    __slots__ = ("op", "ops", "line", "reads", "writes", "ws", "cls", "asm", "roles")

    def __init__(self, op, ops, line, asm):
        self.op, self.ops, self.line, self.asm = op, ops, line, asm
        self.reads, self.writes = set(), set()
        self.ws = 1
        self.cls = "other"


def decode(op, ops):
    """(class, writes, reads, address/data reads for the WAR windows)."""
    regs = [vgprs(o) for o in ops]
    if op == "s_nop":
        return "nop", set(), set(), {}
    if op.startswith(VMEM):
        is_store = "store" in op or ("atomic" in op and "rtn" not in op and not op.endswith("_rtn"))
        is_lds_dma = op.endswith("lds") or " lds" in " ".join(ops) or "_lds_" in op
        if is_lds_dma:  # global_load_lds_dwordx4 vaddr, off / buffer_load ... lds
            return "vmem", set(), set().union(*regs[:2]) if regs else set(), {"addr": regs[0]}
        if op.startswith("buffer_"):
            # buffer_load v_dst, v_off, s[rsrc], soff ...; buffer_store v_data, v_off, ...
            data, addr = (regs[0] if regs else set()), (regs[1] if len(regs) > 1 else set())
            if is_store:
                return "vmem", set(), data | addr, {"addr": addr, "data": data}
            return "vmem", data, addr, {"addr": addr}
        # global / flat / scratch: load v_dst, v_addr, saddr|off; store v_addr, v_data, ...
        if is_store:
            addr, data = (regs[0] if regs else set()), (regs[1] if len(regs) > 1 else set())
            return "vmem", set(), addr | data, {"addr": addr, "data": data}
        dst, addr = (regs[0] if regs else set()), (regs[1] if len(regs) > 1 else set())
        return "vmem", dst, addr, {"addr": addr}
    if op.startswith(DS):
        if op.startswith(("ds_read", "ds_load")) or "bpermute" in op or "swizzle" in op or \
                op.startswith("ds_permute"):
            dst = regs[0] if regs else set()
            src = set().union(*regs[1:]) if len(regs) > 1 else set()
            return "ds", dst, src, {"addr": src}
        if op.startswith(("ds_write", "ds_store", "ds_add", "ds_max", "ds_min")) and "rtn" not in op:
            src = set().union(*regs) if regs else set()
            return "ds", set(), src, {"addr": src}
        dst = regs[0] if regs else set()
        src = set().union(*regs[1:]) if len(regs) > 1 else set()
        return "ds", dst, src, {"addr": src}
    if op.startswith("v_mfma") or op.startswith("v_smfma"):
        # v_mfma dst, srcA, srcB, srcC
        a = regs[1] if len(regs) > 1 else set()
        b = regs[2] if len(regs) > 2 else set()
        c = regs[3] if len(regs) > 3 else set()
        return "mfma", regs[0] if regs else set(), a | b | c, {"A": a, "B": b, "C": c}
    if op.startswith("v_"):
        if op.startswith(("v_cmp_", "v_readlane", "v_readfirstlane")) and not op.startswith("v_cmpx"):
            # first operand is an SGPR / VCC (or a VGPR for _e64 of v_cmp with vdst: none on gfx9)
            dst = set()
            src = set().union(*regs) if regs else set()
            return "valu", dst, src, {}
        dst = regs[0] if regs else set()
        src = set().union(*regs[1:]) if len(regs) > 1 else set()
        return "valu", dst, src, {}
    return "salu", set(), set(), {}


LANE_GROUP = re.compile(r"row_|quad_perm|row_bcast|row_mirror|row_half_mirror|wave_shr|wave_shl|"
                        r"wave_ror|wave_rol|permlane|readlane|writelane|bpermute|ds_swizzle|mbcnt")


def instrs(body):
    out, in_asm = [], False
    for line in body:
        s = line.split(";")[0].strip() if not line.strip().startswith(";;#ASM") else line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        t = s.replace(",", " , ").split()
        op = t[0]
        ops = [x for x in " ".join(t[1:]).split(" , ")]
        ops = [o.strip() for o in ops if o.strip()]
        # trailing modifiers (offset:, off, sc0, nt, ...) are whitespace-separated in the last op
        if ops:
            ops = ops[:-1] + ops[-1].split()
        ins = Ins(op, ops, s, in_asm)
        ins.cls, ins.writes, ins.reads, ins.roles = decode(op, ops)
        if op == "s_nop":
            try:
                ins.ws = int(ops[0], 0) + 1
            except (ValueError, IndexError):
                ins.ws = 1
        out.append(ins)
    return out


def scan(body, window):
    ins = instrs(body)
    hits = defaultdict(Counter)  # class -> Counter(distance)
    detail = defaultdict(list)
    lanegroup = Counter()
    n_mfma = 0
    for i, a in enumerate(ins):
        if LANE_GROUP.search(a.line):
            lanegroup[a.op] += 1
        roles = a.roles
        if a.cls == "mfma":
            n_mfma += 1
        watch = []  # (class, regs)
        if a.cls == "vmem":
            if roles.get("addr"):
                watch.append(("vmem-addr", roles["addr"]))
            if roles.get("data"):
                wide = any(w in a.op for w in ("dwordx3", "dwordx4", "b96", "b128"))
                watch.append(("vmem-data" + ("-wide" if wide else ""), roles["data"]))
        elif a.cls == "ds":
            if roles.get("addr"):
                watch.append(("ds-src", roles["addr"]))
        elif a.cls == "mfma":
            for r in ("A", "B", "C"):
                if roles.get(r):
                    watch.append(("mfma-src" + r, roles[r]))
        if not watch:
            continue
        dist = 0
        for j in range(i + 1, len(ins)):
            b = ins[j]
            if b.writes:
                for cls, regs in watch:
                    if b.writes & regs:
                        # an MFMA taking the previous MFMA's D as its C (accumulate chain)
                        # rewrites its own C: not a hazard
                        if cls == "mfma-srcC" and b.cls == "mfma" and \
                                b.roles.get("C") == regs:
                            continue
                        key = f"{cls} <- {b.cls}"
                        hits[key][dist] += 1
                        detail[key].append((dist, a.line, b.line))
                watch = [(c, r - b.writes) for c, r in watch if r - b.writes]
            dist += b.ws
            if dist > window or not watch:
                break
    return hits, detail, lanegroup, n_mfma, len(ins)


def main(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=WINDOW)
    ap.add_argument("--detail", action="store_true")
    ap.add_argument("--match", default="", help="only kernels whose name contains this")
    ap.add_argument("--classes", default="", help="comma list of classes to print (default all)")
    ap.add_argument("files", nargs="+")
    a = ap.parse_args(argv)
    want = set(a.classes.split(",")) if a.classes else None
    for p in a.files:
        text = open(p).read()
        res = resources(text)
        for name, body in kernels(text):
            if a.match and a.match not in name:
                continue
            hits, detail, lanegroup, n_mfma, n = scan(body, a.window)
            r = res.get(name, {})
            print(f"{name[:90]}\n  vgpr {r.get('vgpr')} agpr {r.get('agpr')} sgpr {r.get('sgpr')} "
                  f"scratch {r.get('scratch')} lds {r.get('lds')} occupancy {r.get('occupancy')} "
                  f"instructions {n} mfma {n_mfma}")
            if lanegroup:
                print("  lane-group ops: " + ", ".join(f"{k} {v}" for k, v in sorted(lanegroup.items())))
            for key in sorted(hits):
                if want and key.split(" <- ")[0] not in want:
                    continue
                c = hits[key]
                print(f"  {key:28s} " + " ".join(f"d{d}:{c[d]}" for d in sorted(c)))
                if a.detail:
                    for d, l1, l2 in sorted(detail[key])[:12]:
                        print(f"      d{d}: {l1}   ->   {l2}")


if __name__ == "__main__":
    main(sys.argv[1:])
