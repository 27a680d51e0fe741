# End-to-end DE generation through the drop-in classes at config 2 / config 3 populations, world 1 / 2 / 4
# (ranks share the box's one GPU through gloo), with per-generation GC time and evolve segments.
#   usage: TAG=r05c GENS=24 POPS="1024" WORLDS="1 4" bash tools/gen_ranks.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-dev}
for POP in ${POPS:-1024}; do for W in ${WORLDS:-1 4}; do
  if [ "$W" = 1 ]; then
    timeout -k 10 400 python tools/generation_bench.py ${GENS:-24} $POP > gpurun_out/gen_w1_${POP}_$TAG.log 2>&1 || { tail -20 gpurun_out/gen_w1_${POP}_$TAG.log; exit 1; }
  else
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29600 + W)) tools/generation_bench.py ${GENS:-24} $POP > gpurun_out/gen_w${W}_${POP}_$TAG.log 2>&1 || { tail -30 gpurun_out/gen_w${W}_${POP}_$TAG.log; exit 1; }
  fi
  grep '^{' gpurun_out/gen_w${W}_${POP}_$TAG.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($POP, $W, 'best', round(d['gpu_generation_ms'],2), 'median', round(d['gpu_generation_ms_median'],2), 'all', d['gpu_generation_ms_all'])"
done; done
