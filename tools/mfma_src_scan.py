"""Flags loads that write a register an MFMA issued shortly before reads (ISA text scan).

Usage: python tools/mfma_src_scan.py file.s   (hipcc --cuda-device-only -S output)
Measured on gfx950 / ROCm 7.2: a global or LDS load landing in a source
register of a recently issued MFMA corrupted results nondeterministically."""
import re
import sys


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def scan(text, window=30):
    lines = text.split('\n')
    fn, hits = None, []
    for i, l in enumerate(lines):
        if re.match(r'^_Z\S+:', l):
            fn = l.split(':')[0]
        t = l.split()
        if not t or not t[0].startswith('v_mfma'):
            continue
        ops = [x.strip(',') for x in t[1:]]
        src = regs(ops[1]) | regs(ops[2])
        for j in range(i + 1, min(i + window, len(lines))):
            u = lines[j].split()
            if u and u[0].startswith(('global_load', 'ds_read', 'buffer_load')):
                if regs(u[1].strip(',')) & src:
                    hits.append((fn, i, l.strip(), j, lines[j].strip()))
    return hits


if __name__ == '__main__':
    hits = scan(open(sys.argv[1]).read())
    for h in hits:
        print(*h, sep=' | ')
    print('suspect overwrites:', len(hits))
