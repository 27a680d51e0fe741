# One GPU step of an A/B investigation (replaces round 4's one-off tools/r04_step*.sh command lines):
# a parity suite on the working tree (or on ab/<LIB>.so), then interleaved A/B bench lines, teed to
# gpurun_out/<OUT>.txt.
#   usage: TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py" | TESTS=all | TESTS=none
#          POPS="256 128" ROUNDS=3 OUT=r05_xyz [LIB=name] [CONFIG5=1] [CONFIG4=1] \
#          bash tools/gpu_step.sh 'base=' 'var=' 'name=ENV=1,ENV2=0' ...
# (A/B libraries: tools/ab_build.sh -> ab/base.so, ab/var.so; tools/ab_build_defs.sh -> ab/<name>.so;
#  specs as in tools/ab_env.sh.)  Diagnostic phase ablations (TBLUP_DBG_SKIP / TBLUP_DE_DBG) need a
#  library built with -DTBLUP_DIAG_BUILD (tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD').
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-step}
T=${TESTS:-"tests/test_gpu_schedule.py tests/test_gpu_shapes.py tests/test_gpu_parity.py"}
if [ "$T" != "none" ]; then
  [ "$T" = "all" ] && T="tests -m gpu"
  env ${LIB:+TBLUP_GPU_LIB=ab/$LIB.so} timeout -k 10 900 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > gpurun_out/${OUT}_test.log 2>&1
  rc=$?; tail -3 gpurun_out/${OUT}_test.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${OUT}_test.log | head -20; exit 1; }
fi
[ $# -gt 0 ] || exit 0
POPS="${POPS:-256 128}" bash tools/ab_env.sh ${ROUNDS:-3} "$@" 2>&1 | tee gpurun_out/${OUT}.txt || exit 1
for c in ${CONFIG5:+config5} ${CONFIG4:+config4}; do
  for r in 1 2; do for spec in "$@"; do
    v=${spec%%=*}; ev=${spec#*=}; lib=ab/var.so; [ -f ab/$v.so ] && lib=ab/$v.so
    env ${ev//,/ } X=0 TBLUP_GPU_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${c}_$v.log 2> gpurun_out/ab_${c}_$v.err || { tail -5 gpurun_out/ab_${c}_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_${c}_$v.log').read().strip().splitlines()[-1]);print('$c', '$v', d['value'], d['kernel_ms_per_step'])" | tee -a gpurun_out/${OUT}.txt
  done; done
done
