"""Print instructions [a, b) of one kernel in an llvm-objdump disassembly, optionally only the
memory / wait / barrier / branch ones.  Usage: isa_range.py k.dis <symbol substring> a b [mem]"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
on, body = False, []
for l in lines:
    m = re.match(r'^([0-9a-f]+) <(\S+)>:', l)
    if m:
        if on:
            break
        on = sys.argv[2] in m.group(2)
        continue
    if on:
        m = re.match(r'^\s+(\S+.*?)\s*//.*?(<.*\+(0x[0-9a-f]+)>)?\s*$', l)
        if m:
            body.append(m.group(1)[:80] + ('  -> ' + m.group(3) if m.group(3) else ''))
a, b = int(sys.argv[3]), int(sys.argv[4])
mem = len(sys.argv) > 5
for i in range(a, min(b, len(body))):
    x = body[i]
    if not mem or re.search(r'load|store|waitcnt|barrier|ds_|branch|scratch', x):
        print(i, x)
