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
