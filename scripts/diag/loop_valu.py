"""Compiler-generated (non-inline-asm) VALU instructions in the largest loop of a kernel
in a device-only `hipcc -S` listing (diagnostic).  usage: loop_valu.py file.s kernel_substring"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read()
m = re.search(r"^(\S*%s\S*):[^\n]*$" % re.escape(sys.argv[2]), text, re.M)
body = text[m.end():text.index(".Lfunc_end", m.end())].splitlines()
labels = {}
for i, l in enumerate(body):
    mm = re.match(r"^(\.LBB\d+_\d+):", l.strip())
    if mm:
        labels[mm.group(1)] = i
back = []
for i, l in enumerate(body):
    mm = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
        back.append((i - labels[mm.group(1)], labels[mm.group(1)], i))
_, s, e = max(back)
inasm = False
c = Counter()
for l in body[s:e]:
    t = l.strip()
    if t.startswith(";;#ASMSTART"):
        inasm = True
        continue
    if t.startswith(";;#ASMEND"):
        inasm = False
        continue
    if inasm or not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op.startswith(("v_", "s_")):
        c[op] += 1
print("loop lines", e - s, "non-asm VALU", sum(v for k, v in c.items() if k.startswith("v_")),
      "SALU/SMEM", sum(v for k, v in c.items() if k.startswith("s_")))
print(c.most_common(14))
