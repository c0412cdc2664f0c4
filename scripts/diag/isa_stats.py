"""ISA statistics of one kernel in a device-only `hipcc -S` listing (diagnostic):
instruction counts by class, VGPRs, scratch.  usage: isa_stats.py file.s kernel_substring"""
import re
import sys
from collections import Counter


def stats(path, needle):
    text = open(path).read()
    m = re.search(r"^(\S*%s\S*):[^\n]*$" % re.escape(needle), text, re.M)
    if not m:
        raise SystemExit("kernel not found")
    name = m.group(1)
    body = text[m.end():text.index(".Lfunc_end", m.end())]
    c = Counter()
    for line in body.splitlines():
        line = line.strip()
        if not line or line.startswith((";", ".", "//")) or line.endswith(":"):
            continue
        op = line.split()[0]
        c[op] += 1
    meta = {}
    for key in ("num_vgpr", "num_agpr", "numbered_sgpr", "private_seg_size"):
        mm = re.search(r"\.set %s\.%s, (\d+)" % (re.escape(name), key), text)
        if mm:
            meta[key] = int(mm.group(1))
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    half = sum(v for k, v in c.items() if any(s in k for s in ("lshl", "lshr", "alignbit", "bfi", "bfe", "perm", "_dpp")))
    return name, meta, valu, half, c


if __name__ == "__main__":
    name, meta, valu, half, c = stats(sys.argv[1], sys.argv[2])
    print(name, meta, "VALU", valu, "half-rate", half)
    for k, v in c.most_common(25):
        print(f"  {k:28s} {v}")
