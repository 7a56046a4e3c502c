"""List the loops (backward branches) of one kernel in an llvm-objdump disassembly with their size,
barriers, calls and scratch (spill) instructions.  Usage: isa_loops.py k.dis <symbol substring>"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
body, on = [], False
for l in lines:
    m = re.match(r'^([0-9a-f]+) <(\S+)>:', l)
    if m:
        on = pat in m.group(2)
        if on:
            body = []
        continue
    if on:
        m = re.match(r'^\s+(\S+.*?)\s*//\s*([0-9A-F]+):(.*)$', l)
        if m:
            t = re.search(r'<[^+>]*\+0x([0-9a-f]+)>', m.group(3))
            body.append((int(m.group(2), 16), m.group(1), int(t.group(1), 16) if t else None))
    if on and body and not l.strip():
        break
addr = {a: i for i, (a, _, _) in enumerate(body)}
loops = []
for i, (a, ins, off) in enumerate(body):
    if not (ins.startswith('s_cbranch') or ins.startswith('s_branch')) or off is None:
        continue
    base = body[0][0]
    # targets are symbol-relative offsets
    t = base + off
    if t <= a and t in addr:
        j = addr[t]
        seg = [x for _, x, _ in body[j:i + 1]]
        loops.append((j, i, len(seg), sum('s_barrier' in x for x in seg), sum('s_swappc' in x for x in seg),
                      sum(x.startswith('scratch_') for x in seg)))
for j, i, n, nb, nc, ns in sorted(loops, key=lambda x: x[2]):
    print(f"loop [{j}..{i}] instrs {n} barriers {nb} calls {nc} scratch {ns}")
