"""The reference's test tables through the C++ host mirror
(go-dsp_amd/host/gdsp.hpp -> C ABI -> GPU), via tests/cpp/reference_tests."""
import os
import subprocess

import pytest

from conftest import REPO

BIN = os.path.join(REPO, "tests", "cpp", "bin", "reference_tests")


def _write_vectors(refvec, path):
    lines = []
    for c in refvec["fftTests"]:
        n = len(c["in"])
        lines.append(" ".join(["FFT", str(n)] + [repr(float(v)) for v in c["in"]]
                              + [repr(float(v)) for p in c["out"] for v in p]))
    for c in refvec["fft2Tests"]:
        r, k = len(c["in"]), len(c["in"][0])
        lines.append(" ".join(["FFT2", str(r), str(k)]
                              + [repr(float(v)) for row in c["in"] for v in row]
                              + [repr(float(v)) for row in c["out"] for p in row for v in p]))
    for c in refvec["fftnTests"]:
        lines.append(" ".join(["FFTN", str(len(c["dim"]))] + [str(d) for d in c["dim"]]
                              + [repr(float(v)) for v in c["in"]]
                              + [repr(float(v)) for p in c["out"] for v in p]))
    files = {"small.wav": "small.wav", "float.wav": "float_head.wav"}
    for name, h in refvec["wavTests"].items():
        wav_path = os.path.join(REPO, "tests", "golden", "wav", files[name])
        lines.append(" ".join(["WAV", wav_path] + [str(h[k]) for k in (
            "AudioFormat", "NumChannels", "SampleRate", "ByteRate", "BlockAlign",
            "BitsPerSample", "Samples", "Duration")]))
    for c in refvec["pwelchTests"]:
        if not c["x"]:
            continue
        lines.append(" ".join(["PWELCH", repr(float(c["fs"])), str(len(c["x"]))]
                              + [repr(float(v)) for v in c["x"]] + [str(len(c["p"]))]
                              + [repr(float(v)) for v in c["p"]]
                              + [repr(float(v)) for v in c["freqs"]]))
    x = refvec["segmentTests"]["x"]
    for c in refvec["segmentTests"]["cases"]:
        lines.append(" ".join(["SEG", str(len(x))] + [str(v) for v in x]
                              + [str(c["size"]), str(c["noverlap"]), str(len(c["out"]))]
                              + [str(v) for s in c["out"] for v in s]))
    for c in refvec["windowTests"]:
        lines.append(" ".join(["WIN", str(c["L"])] + [repr(float(v)) for k in
                                                      ("hamming", "hann", "bartlett", "flattop",
                                                       "blackman") for v in c[k]]))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def test_cpp_mirror_built():
    assert os.path.exists(BIN), "tests/cpp/bin/reference_tests missing: run __graft_entry__.build()"


@pytest.mark.gpu
def test_cpp_mirror_reference_tables(refvec, tmp_path):
    vec = tmp_path / "vectors.txt"
    _write_vectors(refvec, vec)
    r = subprocess.run([BIN, str(vec)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failures 0" in r.stdout


@pytest.mark.gpu
def test_python_api_on_rocm_runtime():
    """The host-pointer path under /opt/rocm's HIP runtime (torch not loaded
    first): repeated small calls, where stream-ordered allocation once lost
    kernel output (see gdsp_api.hip, Workspace)."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
assert "torch" not in sys.modules
rng = np.random.default_rng(1)
for rep in range(20):
    for n in (2, 3, 8, 100, 1024, 3000, 4096):
        x = rng.standard_normal((3, n)) + 1j * rng.standard_normal((3, n))
        y = g.fft.FFTBatch(x)
        ref = oracle.fft_rows(x)
        err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
        assert err < 1e-9, (rep, n, err)
print("ok")
'''
    env = dict(os.environ, GDSP_NO_TORCH_PRELOAD="1", REPO=REPO)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_mixed_generic_kernel_for_specialised_lengths():
    """GDSP_ALGO_GENERIC_MIXED routes lengths that have a compiled
    specialisation (n = 3000) through the generic mixed-radix kernel: both
    kernels must agree with the oracle (the bench times the specialisation)."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
g.fft.SetAlgorithm(g.fft.ALGO_GENERIC_MIXED)
assert g.fft.Algorithm() == g.fft.ALGO_GENERIC_MIXED
import torch
assert D.plan(3000).kind == 5
rng = np.random.default_rng(3)
for n in (3000, 1000, 2000, 1500, 2400, 1200, 960, 1920, 480, 1536, 3072, 12):
    x = rng.standard_normal((9, n)) + 1j * rng.standard_normal((9, n))
    for inv in (False, True):
        y = g.fft.FFTBatch(x, inverse=inv)
        ref = oracle.ifft_rows(x) if inv else oracle.fft_rows(x)
        err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
        assert err < 1e-9, (n, inv, err)
print("ok")
'''
    env = dict(os.environ, REPO=REPO)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_paths_without_runtime_compiler():
    """GDSP_JIT=0: lengths the runtime compiler would take keep the paths it
    replaces (runtime-radix kernel, chirp-z, the five-pass four-step with its
    twiddled transpose), which must still agree with the oracle."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
import torch
rng = np.random.default_rng(5)
for n, kind, batch in ((810, 5, 5), (5400, 3, 3), (390625, 6, 1), (600000, 6, 1)):
    assert D.plan(n).kind == kind, (n, D.plan(n).kind)
    x = rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))
    for inv in (False, True):
        y = g.fft.FFTBatch(x, inverse=inv)
        ref = oracle.ifft_rows(x) if inv else oracle.fft_rows(x)
        err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
        assert err < 1e-9, (n, inv, err)
print("ok")
'''
    env = dict(os.environ, GDSP_JIT="0", REPO=REPO)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_runtime_compiler_failure_falls_back():
    """A failed runtime compilation (here: the headers are not where
    GDSP_JIT_INCLUDE points) leaves each plan on the path it replaces, with
    the same results: the runtime compiler is a speed path only."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
import torch
rng = np.random.default_rng(6)
for n, kind in ((810, 5), (4320, 3), (390625, 6)):
    assert D.plan(n).kind == kind, (n, D.plan(n).kind)
    x = rng.standard_normal((1, n)) + 1j * rng.standard_normal((1, n))
    y = g.fft.FFTBatch(x)
    err = np.linalg.norm(y - oracle.fft_rows(x)) / np.linalg.norm(y)
    assert err < 1e-9, (n, err)
print("ok")
'''
    env = dict(os.environ, GDSP_JIT_INCLUDE="/nonexistent-gdsp-headers", GDSP_JIT_VERBOSE="1",
               GDSP_JIT_CACHE="off", REPO=REPO)
    code = code.replace('print("ok")', 'print("ok", g._lib.jit_stats())')
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
    assert "not built" in r.stderr, r.stderr[-2000:]
    # the downgrade is reported, not only logged: gdsp_jit_stats
    stats = eval(r.stdout.split("ok", 1)[1])
    assert stats["failed"] >= 3 and stats["built"] == 0, stats
    assert "n = 4320" in stats["last_failure"] or "L = " in stats["last_failure"], stats


@pytest.mark.gpu
def test_runtime_compiler_cache_across_processes(tmp_path):
    """The hipRTC specialisations compile from headers embedded in the
    library (no source tree needed) and land in the on-disk code-object cache:
    a second process creating the same plans loads them and compiles nothing."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
import torch
rng = np.random.default_rng(9)
for n in (5400, 810):
    p = D.plan(n)
    assert p.kind == 5 and p.runtime_compiled, (n, p.kind)
    x = rng.standard_normal((3, n)) + 1j * rng.standard_normal((3, n))
    y = g.fft.FFTBatch(x)
    err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, oracle.fft_rows(x)))
    assert err < 1e-9, (n, err)
print("ok", g._lib.jit_stats())
'''
    env = dict(os.environ, GDSP_JIT_CACHE=str(tmp_path / "cache"), REPO=REPO)
    env.pop("GDSP_JIT_INCLUDE", None)
    runs = []
    for _ in range(2):
        r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr[-3000:]
        runs.append(eval(r.stdout.split("ok", 1)[1]))
    assert runs[0]["built"] == 2 and runs[0]["cached"] == 0 and runs[0]["failed"] == 0, runs
    assert runs[1]["built"] == 0 and runs[1]["cached"] == 2 and runs[1]["failed"] == 0, runs
    assert len(list((tmp_path / "cache").glob("*.co"))) == 2


SHIM_BIN = os.path.join(REPO, "tests", "cpp", "bin", "shim_replay")
GO = os.path.join(REPO, "go")


def test_go_shim_covers_the_reference_api():
    """go/ holds the cgo shim as source: every exported function of
    fft/fft.go:25-162 and spectral/pwelch.go:28,74 (and
    wav.go:138's ReadFloats) is defined there, under the gdspgpu build tag,
    and every C function it calls is declared in include/gdsp_fft.h."""
    import re
    import importlib
    lib = importlib.import_module("go-dsp_amd._lib")
    declared = set(lib.header_functions())
    want = {"fft/fft_gpu.go": {"FFT", "FFTReal", "IFFT", "IFFTReal", "Convolve", "FFT2",
                               "FFT2Real", "IFFT2", "IFFT2Real", "FFTN", "IFFTN",
                               "SetWorkerPoolSize", "EnsurePlan"},
            "spectral/pwelch_gpu.go": {"Pwelch"},
            "wav/wav_gpu.go": {"ReadFloats"}}
    for rel, names in want.items():
        src = open(os.path.join(GO, rel)).read()
        assert src.startswith("//go:build gdspgpu\n"), rel
        assert "#cgo LDFLAGS: -lgdspfft" in src and '#include "gdsp_fft.h"' in src, rel
        defined = set(re.findall(r"^func (?:\([^)]*\) )?([A-Z]\w*)\(", src, flags=re.M))
        assert names <= defined, (rel, names - defined)
        called = set(re.findall(r"\bC\.(gdsp_\w+)\(", src))
        assert called and called <= declared, (rel, called - declared)
    # no reference FFT code on the drop-in's path: the
    # gdspgpu build tags radix2.go / bluestein.go out, so nothing may call
    # their kernels, and the replay has no host transform either
    fsrc = open(os.path.join(GO, "fft/fft_gpu.go")).read()
    body = re.sub(r"//[^\n]*", "", fsrc)
    for name in ("radix2FFT", "bluesteinFFT", "getRadix2Factors", "GPUMinN", "onHost"):
        assert name not in body, name
    assert "func EnsureRadix2Factors(" in fsrc and "func reverseBits(" in fsrc
    replay = open(os.path.join(REPO, "tests", "cpp", "shim_replay.cpp")).read()
    ns = re.sub(r"//[^\n]*", "", replay[replay.index("namespace goshim {"):
                                         replay.index("}  // namespace goshim")])
    assert "or_fft" not in ns and "or_ifft" not in ns and "or_convolve" not in ns
    pw = open(os.path.join(GO, "spectral/pwelch_gpu.go")).read()
    for field in ("NFFT      int", "Window    func(int) []float64", "Pad       int",
                  "Noverlap  int", "Scale_off bool"):  # pwelch.go:28-65
        assert field in pw, field


def test_shim_replay_built():
    assert os.path.exists(SHIM_BIN), "tests/cpp/bin/shim_replay missing: run __graft_entry__.build()"


@pytest.mark.gpu
def test_shim_replay(refvec, tmp_path):
    """The cgo shim's call sequences (go/, replayed in C++) on the GPU: every
    function against the oracle (every length on the GPU: the shim has no
    host transform), the reference's tables and every panic."""
    vec = tmp_path / "vectors.txt"
    _write_vectors(refvec, vec)
    r = subprocess.run([SHIM_BIN, str(vec)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failures 0" in r.stdout


def _bodies(src, lang):
    """name -> body text of each top-level function (Go: func Name(...);
    C++: the goshim namespace's functions)."""
    import re
    out = {}
    if lang == "go":
        pat = re.compile(r"^func (?:\([^)]*\) )?(\w+)\(.*?\{\s*$|^func (?:\([^)]*\) )?(\w+)\(.*?\{ ", re.M)
    else:
        pat = re.compile(r"^(?:static )?[\w:<>, ]+?[ *&](\w+)\([^;{]*\)\s*(?:const\s*)?\{", re.M)
    ms = list(pat.finditer(src))
    for i, m in enumerate(ms):
        name = m.group(1) or (m.group(2) if m.lastindex and m.lastindex >= 2 else None)
        end = ms[i + 1].start() if i + 1 < len(ms) else len(src)
        out[name] = src[m.start():end]
    return out


def test_shim_replay_matches_go_call_sequences():
    """tests/cpp/shim_replay.cpp replays go/'s functions call for call: for
    every exported Go function (and the helpers they delegate to), the
    ordered libgdspfft calls in its body equal those of its C++ namesake."""
    import re
    cpp = open(os.path.join(REPO, "tests", "cpp", "shim_replay.cpp")).read()
    cpp = cpp[cpp.index("namespace goshim {"):cpp.index("}  // namespace goshim")]
    cb = _bodies(cpp, "cpp")
    checked = 0
    for rel in ("fft/fft_gpu.go", "spectral/pwelch_gpu.go", "wav/wav_gpu.go"):
        gb = _bodies(open(os.path.join(GO, rel)).read(), "go")
        for name, body in gb.items():
            calls = re.findall(r"\bC\.(gdsp_\w+)\(", body)
            if not calls or name not in cb:
                continue
            assert re.findall(r"\b(gdsp_\w+)\(", cb[name]) == calls, (rel, name)
            checked += 1
    assert checked >= 15, checked
