# D-units beside the diagonal up to J <= 2 / 3 / 4 / 5 at pop 128, with the asm SYRK ring
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
POPS="128" bash tools/ab_env.sh 3 'var=' 'j2=' 'j4=' 'j5=' 2>&1 | tee gpurun_out/r04_ddmaxj2.txt
