# Leading-padding skip A/B (interleaved): ab/base.so (trailing padding), ab/var.so (leading padding,
# contractions skip it), ab/var.so with TBLUP_PAD_SKIP=0 (leading, multiplied); then ahead-rule
# thresholds (TBLUP_AHEAD_SLOTS) on ab/var.so.
#   usage: bash tools/ab_pad.sh [rounds] [pops]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-3}
POPS=${2:-"256 128"}
run() {   # name pop env...
  local v=$1 P=$2; shift 2
  local lib=ab/var.so; [ $v = base ] && lib=ab/base.so
  env "$@" TBLUP_GPU_LIB=$lib timeout -k 10 200 python bench.py --pop $P --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print($P, '$v', d['value'], d['kernel_ms_per_step'])"
}
for P in $POPS; do
for r in $(seq 1 $R); do
  run base $P X=0
  run var $P X=0
  run noskip $P TBLUP_PAD_SKIP=0
  [ -n "$SLOTS" ] && for sl in $SLOTS; do run slots$sl $P TBLUP_AHEAD_SLOTS=$sl; done
done
done
