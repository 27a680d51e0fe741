# A/B builds of libtblup_gpu.so for one GPU call: the working tree as ab/var.so, BASE_REV
# (default HEAD) as ab/base.so (run with TBLUP_GPU_LIB=ab/<name>.so).
#   usage: bash tools/ab_build.sh [BASE_REV]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
mkdir -p ab
make -s -C tblup_amd/csrc OUTDIR=$PWD/ab/var OBJDIR=$PWD/build/ab_var -j8
cp ab/var/libtblup_gpu.so ab/var.so
rm -rf build/ab_base_src && mkdir -p build/ab_base_src
git archive $REV tblup_amd/csrc include | tar -x -C build/ab_base_src
make -s -C build/ab_base_src/tblup_amd/csrc OUTDIR=$PWD/ab/base OBJDIR=$PWD/build/ab_base -j8
cp ab/base/libtblup_gpu.so ab/base.so
rm -rf ab/var ab/base
ls -la ab
