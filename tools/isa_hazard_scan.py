"""ISA audit for the register-reuse patterns behind the r02 fused-forward corruption.

  python tools/isa_hazard_scan.py file.s [file.s ...]   (hipcc --cuda-device-only -S output)

Per kernel, a straight-line scan (branches ignored: a heuristic, not a proof) for:
  mfma-src   a load (global/buffer/ds) whose destination overlaps the A/B source VGPRs of an
             MFMA issued within the previous WINDOW instructions;
  store-data a load or VALU write into the data / address VGPRs of a VMEM store issued
             within the previous WINDOW instructions;
  asm-acc    compiler v_accvgpr moves of AGPRs that an inline-asm MFMA block writes.
The r02 bf16 fused forward (tools/fused_diag) failed in every launch in the build with the
most mfma-src instances at short distance (16, from 28 instructions) and rarely in builds
with fewer, farther ones (7, from 63); DESIGN.md §4.7 has the whole record. Test
infrastructure only."""
import re
import sys

WINDOW = 64


def regs(tok):
    tok = tok.strip(",")
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def aregs(tok):
    tok = tok.strip(",")
    m = re.match(r"a\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"a(\d+)$", tok)
    return {int(m.group(1))} if m else set()


LOADS = ("global_load", "buffer_load", "ds_read", "flat_load")
STORES = ("global_store", "buffer_store", "flat_store")


def kernels(text):
    cur, body = None, []
    for line in text.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if "s_endpgm" in line:
            yield cur, body
            cur = None
            continue
        body.append(line)


def instrs(body):
    out, in_asm = [], False
    for line in body:
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        t = s.split()
        out.append((t[0], [x.strip(",") for x in t[1:]], in_asm))
    return out


def scan_kernel(body):
    ins = instrs(body)
    res = {"mfma": 0, "mfma-src": [], "store-data": [], "asm-acc": 0}
    asm_acc = set()
    for i, (op, ops, in_asm) in enumerate(ins):
        if op.startswith("v_mfma"):
            res["mfma"] += 1
            if in_asm:
                asm_acc |= aregs(ops[0])
            src = regs(ops[1]) | regs(ops[2])
            for j in range(i + 1, min(i + WINDOW, len(ins))):
                op2, ops2, _ = ins[j]
                if op2.startswith(LOADS) and ops2 and regs(ops2[0]) & src:
                    res["mfma-src"].append(j - i)
                    break
        if op.startswith(STORES) and "dwordx" in op:
            data = (regs(ops[1]) if op.startswith("global") else regs(ops[0])) | \
                (regs(ops[0]) if op.startswith("global") else regs(ops[1]))
            for j in range(i + 1, min(i + WINDOW, len(ins))):
                op2, ops2, _ = ins[j]
                if (op2.startswith(LOADS) or op2.startswith("v_")) and not op2.startswith(
                        "v_mfma") and ops2 and regs(ops2[0]) & data:
                    res["store-data"].append(j - i)
                    break
    for op, ops, in_asm in ins:
        if not in_asm and op.startswith("v_accvgpr") and ops:
            if aregs(ops[0]) & asm_acc or (len(ops) > 1 and aregs(ops[1]) & asm_acc):
                res["asm-acc"] += 1
    return res


def main(paths):
    for p in paths:
        for name, body in kernels(open(p).read()):
            r = scan_kernel(body)
            if not r["mfma"] and not r["store-data"]:
                continue
            ms, sd = r["mfma-src"], r["store-data"]
            print(f"{name[:70]:70s} mfma {r['mfma']:4d}  mfma-src {len(ms):3d}"
                  f" (min {min(ms) if ms else '-':>3})  store-data {len(sd):3d}"
                  f" (min {min(sd) if sd else '-':>3})  asm-acc {r['asm-acc']}")


if __name__ == "__main__":
    main(sys.argv[1:])
