# off-diagonal phase ablation at config 2 (TBLUP_DBG_SKIP: timing only, results are wrong)
#   64 GEMM1, 128 GEMM2, 192 both, 2 D-unit SYRK
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for r in 1 2; do
for sk in 0 64 128 192 2; do
  TBLUP_DBG_SKIP=$sk timeout -k 10 200 python bench.py --pop ${POP:-256} --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abl_$sk.log 2> gpurun_out/abl_$sk.err || { tail -5 gpurun_out/abl_$sk.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abl_$sk.log').read().strip().splitlines()[-1]);print('skip $sk', d['value'], d['kernel_ms_per_step'])"
done
done
