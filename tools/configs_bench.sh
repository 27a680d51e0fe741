# Bench lines for the other BASELINE configs on one GPU (config 4, config 5, config 3's per-GPU share).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --config config4 --steps 5 --warmup 2 > gpurun_out/bench_config4.log 2> gpurun_out/bench_config4.err || { tail -20 gpurun_out/bench_config4.err; exit 1; }
tail -1 gpurun_out/bench_config4.log | cut -c1-300
timeout -k 10 300 python bench.py --config config5 --steps 10 --warmup 3 > gpurun_out/bench_config5.log 2> gpurun_out/bench_config5.err || { tail -20 gpurun_out/bench_config5.err; exit 1; }
tail -1 gpurun_out/bench_config5.log | cut -c1-300
timeout -k 10 300 python bench.py --pop 128 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_pop128.log 2> gpurun_out/bench_pop128.err || { tail -20 gpurun_out/bench_pop128.err; exit 1; }
tail -1 gpurun_out/bench_pop128.log | cut -c1-300
