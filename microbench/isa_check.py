#!/usr/bin/env python3
"""Static hazard scan of a hipcc --save-temps .s (no GPU): per kernel, spill counts, and every VGPR
spill slot whose store runs inside a divergent region (exec narrowed by s_and_saveexec / else) while a
reload of that slot runs outside that region, with more lanes live: those lanes read bytes no store
wrote. Regions are tracked structurally over the linear ISA: s_and_saveexec_b64 sN opens one,
s_or_b64 exec, exec, sN closes it; the else half (s_or_saveexec/s_andn2_saveexec) stays in it.
Usage: isa_check.py file.s [kernel-substring]"""
import re
import subprocess
import sys


def kernels(text):
    for part in re.split(r"\n(?=\S+:\s*; @)", text):
        m = re.match(r"(\S+):\s*; @", part)
        if m:
            yield m.group(1), part.split("\n")


def scan(lines):
    stack, next_id = [], 0
    stores, loads = {}, {}
    for no, ln in enumerate(lines):
        t = ln.strip()
        m = re.match(r"s_and_saveexec_b64 (s\[\d+:\d+\])", t)
        if m:
            next_id += 1
            stack.append((m.group(1), next_id))
            continue
        m = re.match(r"s_or_b64 exec, exec, (s\[\d+:\d+\])", t)
        if m:
            for k in range(len(stack) - 1, -1, -1):
                if stack[k][0] == m.group(1):
                    del stack[k:]
                    break
            continue
        m = re.match(r"scratch_(store|load)_\w+ .*offset:(\d+)", t)
        if m:
            region = tuple(r for _, r in stack)
            (stores if m.group(1) == "store" else loads).setdefault(int(m.group(2)), []).append((no, region))
    hazards = []
    for off, sts in stores.items():
        for lno, lreg in loads.get(off, []):
            prior = [s for s in sts if s[0] < lno]
            if not prior:
                continue
            sno, sreg = prior[-1]  # the store that the load reads back (linear order)
            if len(lreg) < len(sreg) and sreg[: len(lreg)] == lreg:
                hazards.append((off, sno, sreg, lno, lreg))
    return stores, loads, hazards


def main():
    text = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, lines in kernels(text):
        if want not in name:
            continue
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        body = "\n".join(lines)
        stores, loads, hz = scan(lines)
        print(dn[:120])
        print(f"  vgpr spill stores {len(re.findall(r'scratch_store', body))}, reloads {len(re.findall(r'scratch_load', body))}, "
              f"sgpr->vgpr-lane spills {len(re.findall(r'v_writelane', body))}, spill slots {len(stores)}")
        print(f"  reloads outside the divergent region of their store: {len(hz)}")
        for off, sno, sreg, lno, lreg in hz[:8]:
            print(f"    slot {off}: store line {sno} in regions {sreg}, reload line {lno} in {lreg}")
            print("      store: " + lines[sno].strip())
            print("      load : " + lines[lno].strip())


if __name__ == "__main__":
    main()
