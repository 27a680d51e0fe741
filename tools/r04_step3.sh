# round 4: GPU tests on the working tree, then config-2 lines at pop 256 / 128
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gputest_r04b.log 2>&1
rc=$?; tail -4 gpurun_out/gputest_r04b.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gputest_r04b.log | head -30; exit 1; }
for P in 256 128 256 128; do
  timeout -k 10 200 python bench.py --pop $P --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_r04b_$P.log 2> gpurun_out/b_r04b_$P.err || { tail -5 gpurun_out/b_r04b_$P.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_r04b_$P.log').read().strip().splitlines()[-1]);print($P, d['value'], d['kernel_ms_per_step'])"
done
