#!/usr/bin/env python3
"""Straight-line check of an AMDGPU kernel's ISA (hipcc --save-temps .s) for reads of VGPRs whose vector-memory
load may still be in flight: walks the loop body from its header to the back edge in layout order (every block taken,
loads retire in issue order, `s_waitcnt vmcnt(N)` leaves the N youngest outstanding) and reports each instruction
that reads a pending load's destination. Diagnostic for VERDICT r04 item 2 (tools/mf_spcheck.py).

    python tools/vmcnt_check.py FILE.s KERNEL_SYMBOL"""
import re
import sys


def regs(arg):
    out = set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]|\bv(\d+)\b', arg):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    body = lines[start:end]
    head = next(i for i, l in enumerate(body) if '=>This Loop Header: Depth=1' in l)
    m = re.match(r'\.(LBB\d+_\d+):', body[head])
    label = m.group(1)
    # the loop's blocks in layout order from the header, then the latch blocks the compiler placed before it (their
    # label comments say "in Loop: Header=<this header>"), which fall through into the header: one iteration's path
    inloop = 'Header=' + label.replace('LBB', 'BB')
    pre = [i for i in range(head) if re.match(r'\.LBB\d+_\d+:', body[i]) and inloop in body[i]]
    order = list(range(head, len(body)))
    if pre:
        order += list(range(pre[0], head))
    pending = []   # [(line, dest regs)] oldest first
    hits = 0
    for i in order:
        t = body[i].split(';')[0].strip()
        if not t or t.startswith('.'):
            continue
        op, _, args = t.partition(' ')
        w = re.match(r's_waitcnt .*vmcnt\((\d+)\)', t)
        if w:
            n = int(w.group(1))
            pending = pending[len(pending) - n:] if n < len(pending) else pending
            continue
        if op.startswith(('global_load', 'buffer_load', 'flat_load')):
            dst, _, rest = args.partition(',')
            src = regs(rest)
            for ln, d in pending:
                if d & src:
                    print(f"line {i + start + 1}: address read of pending load (line {ln}): {t}")
                    hits += 1
            pending.append((i + start + 1, regs(dst)))
            continue
        if op.startswith(('global_store', 'buffer_store', 'ds_write', 'ds_read', 'v_', 's_')):
            if op.startswith(('global_store', 'buffer_store', 'ds_write')):
                src = regs(args)
            else:
                src = regs(args.partition(',')[2]) if op.startswith(('v_', 'ds_read')) else set()
            for ln, d in pending:
                if d & src:
                    print(f"line {i + start + 1}: reads v{sorted(d & src)} of the load at line {ln} still in flight: {t}")
                    hits += 1
    print(f"{sym}: {hits} read(s) of in-flight load destinations between the loop header and its back edge")


if __name__ == "__main__":
    main()
