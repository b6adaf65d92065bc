# Host-side AddressSanitizer run of the library on the GPU box: the host code
# of libgdspfft.so (plans, staging, zero-copy, multi-device threads, error
# paths) and the C++ host mirror test, both built with -fsanitize=address
# for the host only (-Xarch_host; device code is untouched), running the
# reference tables through the C ABI on the GPU. Build beforehand (CPU):
#   scripts/build_variant.sh asan "-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
#   (cd tests/cpp && hipcc -O1 -std=c++17 -Xarch_host -fsanitize=address \
#      -Xarch_host -fno-omit-frame-pointer -I../../include -I../../go-dsp_amd/host \
#      reference_tests.cpp -o bin/reference_tests_asan -L../../go-dsp_amd/lib_asan -lgdspfft \
#      -Wl,-rpath,'$ORIGIN/../../../go-dsp_amd/lib_asan')
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python3 -c "
import json, sys
sys.path.insert(0, 'tests')
from test_cpp_mirror import _write_vectors
_write_vectors(json.load(open('tests/golden/reference_vectors.json')), 'gpurun_out/vectors.txt')
" || exit 1
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 timeout -k 10 300 ./tests/cpp/bin/reference_tests_asan gpurun_out/vectors.txt > gpurun_out/asan_cpp.log 2>&1; rc=$?
echo "asan reference_tests rc=$rc"; tail -5 gpurun_out/asan_cpp.log
exit $rc
