# One GPU step of an A/B investigation (replaces round 4's one-off tools/r04_step*.sh command lines):
# a parity suite on the working tree (or on ab/<LIB>.so), then interleaved A/B bench lines, teed to
# gpurun_out/<OUT>.txt.
#   usage: TESTS="tests/test_gpu_schedule.py tests/test_gpu_shapes.py" | TESTS=all | TESTS=none
#          POPS="256 128" ROUNDS=3 OUT=r05_xyz [LIB=name] [CONFIG5=1] [CONFIG4=1] \
#          [DE_POPS="256 1024"] [GEN="1024 256"] [TRACE=128] \
#          bash tools/gpu_step.sh 'base=' 'var=' 'name=ENV=1,ENV2=0' ...
#   POPS=none skips the bench lines; DE_POPS: tools/de_bench.py per spec (medians / minima, twice);
#   GEN: tools/generation_bench.py on the working tree (16 generations at pop >= 512, else 24);
#   TRACE: tools/wg_trace.py at that population on the working tree.
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
lib_of() { local v=${1%%=*}; [ -f ab/$v.so ] && echo ab/$v.so || echo ab/var.so; }
for P in $GEN; do
  g=24; [ $P -ge 512 ] && g=16
  timeout -k 10 300 python tools/generation_bench.py $g $P > gpurun_out/${OUT}_gen$P.log 2>&1 || { tail -5 gpurun_out/${OUT}_gen$P.log; exit 1; }
  python3 -c "
import json, statistics as s
d=json.loads([l for l in open('gpurun_out/${OUT}_gen$P.log') if l.startswith('{')][-1]); a=d['gpu_generation_ms_all'][1:]
print('generation pop $P best', min(a), 'median', round(s.median(a),2), 'max', max(a), d['evolve_segments_last_gen_ms'])" | tee -a gpurun_out/${OUT}_gen.txt
done
if [ -n "$TRACE" ]; then
  timeout -k 10 200 python tools/wg_trace.py gpurun_out/${OUT}_wgt$TRACE.npy --pop $TRACE > gpurun_out/${OUT}_wgt$TRACE.txt 2>&1 || exit 1
fi
[ $# -gt 0 ] || exit 0
for r in ${DE_POPS:+1 2}; do for spec in "$@"; do for P in $DE_POPS; do
  ev=${spec#*=}
  env ${ev//,/ } X=0 TBLUP_GPU_LIB=$(lib_of $spec) timeout -k 10 200 python -c "import sys; sys.path.insert(0, 'tools'); import de_bench; de_bench.main(pop=$P, reps=30)" > gpurun_out/${OUT}_de.log 2>&1 || { tail -5 gpurun_out/${OUT}_de.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${OUT}_de.log').read().strip().splitlines()[-1]); print('de ${spec%%=*}', $P, round(d['gpu_de_ms_median'],4), round(d['gpu_de_ms_min'],4))" | tee -a gpurun_out/${OUT}_de.txt
done; done; done
[ "$POPS" = "none" ] && exit 0
POPS="${POPS:-256 128}" bash tools/ab_env.sh ${ROUNDS:-3} "$@" 2>&1 | tee gpurun_out/${OUT}.txt || exit 1
for c in ${CONFIG5:+config5} ${CONFIG4:+config4}; do
  for r in 1 2; do for spec in "$@"; do
    v=${spec%%=*}; ev=${spec#*=}
    env ${ev//,/ } X=0 TBLUP_GPU_LIB=$(lib_of $spec) timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${c}_$v.log 2> gpurun_out/ab_${c}_$v.err || { tail -5 gpurun_out/ab_${c}_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_${c}_$v.log').read().strip().splitlines()[-1]);print('$c', '$v', d['value'], d['kernel_ms_per_step'])" | tee -a gpurun_out/${OUT}.txt
  done; done
done
