# Interleaved A/B of environment settings on ab/var.so (tools/ab_build.sh):
#   usage: POPS="128 96" bash tools/ab_env.sh ROUNDS 'NAME=ENV1,ENV2' 'NAME2=ENV' ...
# (runs ab/NAME.so when it exists -- tools/ab_build_defs.sh -- else ab/var.so; 'base' runs ab/base.so;
# an empty env list runs the defaults)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$1; shift
for P in ${POPS:-128}; do
for r in $(seq 1 $R); do
  for spec in "$@"; do
    v=${spec%%=*}; ev=${spec#*=}
    lib=ab/var.so; [ -f ab/$v.so ] && lib=ab/$v.so
    env ${ev//,/ } X=0 TBLUP_GPU_LIB=$lib timeout -k 10 200 python bench.py --pop $P --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print($P, '$v', d['value'], d['kernel_ms_per_step'])"
  done
done
done
