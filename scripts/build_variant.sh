# Build an alternate libgdspfft.so into go-dsp_amd/lib_<name>/ with extra
# compiler flags (A/B experiments; scripts/gpu_ab.sh takes the directory).
# usage: scripts/build_variant.sh <name> "<-D flags>" [make VAR=value ...]
set -e
cd "$(dirname "$0")/../go-dsp_amd/csrc"
make -s -j8 OUTDIR=../lib_$1 OBJDIR=../lib_$1/obj \
  FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -I../../include $2" $3
