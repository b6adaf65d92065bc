#!/usr/bin/env python3
"""Static instruction mix of kernels in a gfx950 assembly listing
(hipcc --cuda-device-only -S). Counts every instruction once (loops are
not unrolled by this count), grouped as f64 VALU, other VALU, LDS, SALU,
vector memory.

usage: tools/isamix.py listing.s mangled-name-substring [...]
"""
import collections
import re
import sys

text = open(sys.argv[1]).read()
for want in sys.argv[2:]:
    for m in re.finditer(r"^(_Z\w*" + re.escape(want) + r"\w*):", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        body = text[m.end():end]
        c = collections.Counter()
        for line in body.splitlines():
            t = line.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            if op.startswith("v_"):
                c["VALU f64" if "f64" in op else "VALU other"] += 1
                c["  " + op] += 1
            elif op.startswith("ds_"):
                c["LDS"] += 1
                c["  " + op] += 1
            elif op.startswith("s_"):
                c["SALU/ctl"] += 1
                if op in ("s_barrier", "s_waitcnt"):
                    c["  " + op] += 1
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                c["VMEM"] += 1
                c["  " + op] += 1
        print(name)
        for k in ("VALU f64", "VALU other", "LDS", "VMEM", "SALU/ctl"):
            print("   %6d %s" % (c.get(k, 0), k))
        for k, v in sorted(c.items(), key=lambda x: -x[1]):
            if k.startswith("  ") and v >= 8:
                print("   %6d %s" % (v, k))
