#!/usr/bin/env python3
"""Build A/B libraries with other radix lists for some compiled
specialisations (development only: the product sources are restored
afterwards, whatever happens).

usage: tools/spec_variants.py NAME n=a.b.c [n=a.b.c ...]
  -> go-dsp_amd/lib_NAME/libgdspfft.so with Spec<a, b, c> for each n.
"""
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "go-dsp_amd" / "csrc"


def main():
    name, pairs = sys.argv[1], sys.argv[2:]
    want = {}
    for p in pairs:
        n, lst = p.split("=")
        want[int(n)] = [int(x) for x in lst.split(".")]
    files = sorted(CSRC.glob("fft_specs*.hip"))
    saved = {f: f.read_text() for f in files}
    found = set()
    try:
        for f in files:
            out = []
            for line in saved[f].splitlines(keepends=True):
                m = re.search(r"Spec<([\d, ]+)>", line)
                if m:
                    rad = [int(x) for x in m.group(1).split(",")]
                    n = 1
                    for r in rad:
                        n *= r
                    if n in want:
                        new = ", ".join(map(str, want[n]))
                        line = line[:m.start(1)] + new + line[m.end(1):]
                        found.add(n)
                out.append(line)
            f.write_text("".join(out))
        missing = set(want) - found
        if missing:
            raise SystemExit(f"no spec for {sorted(missing)}")
        lib = ROOT / "go-dsp_amd" / f"lib_{name}"
        if not (lib / "obj").exists():
            shutil.copytree(ROOT / "go-dsp_amd" / "lib" / "obj", lib / "obj")
        subprocess.run(["make", "-j8", f"OUTDIR=../lib_{name}", f"OBJDIR=../lib_{name}/obj"],
                       cwd=CSRC, check=True)
    finally:
        for f, text in saved.items():
            f.write_text(text)


if __name__ == "__main__":
    main()
