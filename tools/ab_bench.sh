# A/B bench of ab/base.so vs ab/var.so (tools/ab_build.sh), interleaved, on the GPU box.
#   usage: bash tools/ab_bench.sh [rounds] [extra bench args]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-3}; shift
for r in $(seq 1 $R); do
  for v in base var; do
    TBLUP_GPU_LIB=ab/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['kernel_ms_per_step'])"
  done
done
