#!/usr/bin/env python3
"""Stamp of the sources a measurement ran on: sha256 over the library's
kernel and C-ABI sources (go-dsp_amd/csrc, include) by path and content,
plus the git commit they were committed as — read from .git when present,
else from .source_head, which scripts/stamp_head.sh writes before a gpurun
call (the GPU box gets the tree without .git). bench.py prints it in every
line; tools/pmc_summary.py and tools/trace_summary.py copy it into the
summaries they write, so a quoted profile can be matched to the code that
was timed.

usage: tools/source_stamp.py  ->  {"source_sha": "...", "git_head": "..."}
"""
import hashlib
import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ("go-dsp_amd/csrc", "include")
EXTS = (".hip", ".hpp", ".h", ".py", "Makefile")


def source_sha() -> str:
    h = hashlib.sha256()
    for d in DIRS:
        root = os.path.join(REPO, d)
        for dirpath, dirnames, files in os.walk(root):
            dirnames.sort()
            for f in sorted(files):
                if not f.endswith(EXTS):
                    continue
                p = os.path.join(dirpath, f)
                h.update(os.path.relpath(p, REPO).encode() + b"\0")
                with open(p, "rb") as fh:
                    h.update(fh.read())
                h.update(b"\0")
    return h.hexdigest()[:16]


def git_head():
    if os.path.isdir(os.path.join(REPO, ".git")):
        try:
            r = subprocess.run(["git", "-C", REPO, "rev-parse", "--short=12", "HEAD"],
                               capture_output=True, text=True, timeout=10)
            if r.returncode == 0:
                head = r.stdout.strip()
                d = subprocess.run(["git", "-C", REPO, "diff", "--quiet", "HEAD", "--", *DIRS],
                                   timeout=10)
                return head + ("+dirty" if d.returncode else "")
        except (OSError, subprocess.SubprocessError):
            pass
    p = os.path.join(REPO, ".source_head")
    if os.path.exists(p):
        with open(p) as f:
            return f.read().strip() or None
    return None


def stamp() -> dict:
    return {"source_sha": source_sha(), "git_head": git_head()}


if __name__ == "__main__":
    print(json.dumps(stamp()))
