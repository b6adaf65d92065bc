cd $GRAFT_REPO_ROOT
python - <<'PY'
import json, sys
sys.path.insert(0, "tests")
from test_cpp_mirror import _write_vectors
_write_vectors(json.load(open("tests/golden/reference_vectors.json")), "/tmp/vec.txt")
PY
for m in 0 1 2 3; do for i in 1 2 3 4 5; do GDSP_DEBUG=$m timeout -k 5 60 tests/cpp/bin/reference_tests /tmp/vec.txt > /tmp/o.txt 2>&1; echo "mode $m rc=$? $(head -c 120 /tmp/o.txt | tr '\n' ' ')"; done; done
