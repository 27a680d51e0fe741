# round 4: GPU tests (multi-rank generation through the node-shared rows) + generation timing at
# world 1 / 2 / 4 on this one GPU (gloo), config 2 (pop 256) and config 3 (pop 1024)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_shapes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r04c.log 2>&1
rc=$?; tail -4 gpurun_out/gputest_r04c.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gputest_r04c.log | head -30; exit 1; }
for POP in 256 1024; do
  timeout -k 10 300 python tools/generation_bench.py 16 $POP > gpurun_out/gen_r04_w1_$POP.log 2>&1 || { tail -20 gpurun_out/gen_r04_w1_$POP.log; exit 1; }
  tail -1 gpurun_out/gen_r04_w1_$POP.log | cut -c1-400
  for W in 2 4; do
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29600 + W)) tools/generation_bench.py 16 $POP > gpurun_out/gen_r04_w${W}_$POP.log 2>&1 || { tail -30 gpurun_out/gen_r04_w${W}_$POP.log; exit 1; }
    grep '^{' gpurun_out/gen_r04_w${W}_$POP.log | tail -1 | cut -c1-400
  done
done
