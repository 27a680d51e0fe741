# D-units in the diagonal launch (OffPlan::ndd) A/B, interleaved: ab/base.so vs ab/var.so (auto:
# B <= 128, J <= 3) and ab/var.so with TBLUP_DIAG_D=0 / 1.   usage: bash tools/ab_diagd.sh [rounds] [pops]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-3}
POPS=${2:-"128 64 32"}
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
  run dd0 $P TBLUP_DIAG_D=0
  run dd1 $P TBLUP_DIAG_D=1
done
done
