"""Audit a kernel's .s for the inline-asm load hazard of cdna_hip_programming.md §5.7 item 1: no
compiler instruction may read or write a VGPR that is the destination of a still-outstanding vector-memory
load or returning atomic. Linear scan of the listing: a FIFO of outstanding vector-memory ops is pushed by every
global/buffer load/store and popped by every `s_waitcnt vmcnt(n)` (loads return in order).
usage: python tools/check_asm_loads.py file.s kernel_symbol [kernel_symbol ...]
       (or import and call check(lines, symbol) -> (asm vector-memory ops, [hazards]))"""
import re
import sys
from collections import deque

REG = r"v\[?(\d+)(?::(\d+))?\]?"
_WAIT = re.compile(r"s_waitcnt\s.*vmcnt\((\d+)\)")
_VMEM = re.compile(r"(global|buffer)_(load|store|atomic)\w*\s+" + REG)
_VALU = re.compile(r"v_(?!mfma)\w+\s")
_RANGE = re.compile(r"\bv\[(\d+):(\d+)\]")
_ONE = re.compile(r"\bv(\d+)\b")


def check(lines, sym):
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    fifo = deque()          # sets of destination VGPRs (empty set for stores)
    bad = []
    n_asm = 0
    inasm = False
    for i in range(start, end):
        l = lines[i]
        if "ASMSTART" in l:
            inasm = True
            continue
        if "ASMEND" in l:
            inasm = False
            continue
        t = l.strip()
        m = _WAIT.match(t)
        if m:
            n = int(m.group(1))
            while len(fifo) > n:
                fifo.popleft()
            continue
        m = _VMEM.match(t)
        if m:
            regs = set()
            # destinations: loads (not LDS-DMA), and returning atomics (sc0) — the value lands asynchronously
            if (m.group(2) == "load" and "lds" not in t) or (m.group(2) == "atomic" and re.search(r"\bsc0\b", t)):
                regs = set(range(int(m.group(3)), int(m.group(4) or m.group(3)) + 1))
            fifo.append(regs if inasm else set())  # hipcc waits for its own loads
            n_asm += inasm
            continue
        if inasm:
            # item 2 of the same section: hipcc pads an asm statement's outputs by one wait state only, but a
            # VALU write -> MFMA operand read needs two; so no VALU result may come out of inline asm
            if _VALU.match(t):
                bad.append((i + 1, "VALU inside inline asm: " + t))
            continue
        # any compiler instruction that reads or writes an in-flight destination (incl. spills)
        if not fifo or t.startswith((";", ".", "s_")) or not t:
            continue
        live = set().union(*fifo)
        if not live:
            continue
        touched = set()
        for a, b in _RANGE.findall(t):
            touched.update(range(int(a), int(b) + 1))
        for a in _ONE.findall(t):
            touched.add(int(a))
        if touched & live:
            bad.append((i + 1, t))
    return n_asm, bad


def main():
    lines = open(sys.argv[1]).read().split("\n")
    rc = 0
    for sym in sys.argv[2:]:
        n_asm, bad = check(lines, sym)
        print(f"{sym}: asm vector-memory ops: {n_asm}; compiler writes to in-flight load destinations: {len(bad)}")
        for b in bad[:20]:
            print("  ", b)
        rc |= 1 if bad else 0
    sys.exit(rc)


if __name__ == "__main__":
    main()
