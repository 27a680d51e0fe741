# A/B builds of the working tree with compile-time overrides: one library per NAME=DEFINES pair.
#   usage: bash tools/ab_build_defs.sh 'j2=-DTBLUP_AB_DD_MAX_J=2' 'j4=-DTBLUP_AB_DD_MAX_J=4' ...
# -> ab/<NAME>.so (run with TBLUP_GPU_LIB=ab/<NAME>.so; tools/ab_env.sh runs ab/<NAME>.so for NAME=...)
set -e
cd "$(dirname "$0")/.."
mkdir -p ab
for spec in "$@"; do
  n=${spec%%=*}; defs=${spec#*=}
  make -s -C tblup_amd/csrc OUTDIR=$PWD/ab/$n OBJDIR=$PWD/build/ab_$n CXXFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result $defs" -j8
  cp ab/$n/libtblup_gpu.so ab/$n.so
  rm -rf ab/$n
done
ls -la ab
