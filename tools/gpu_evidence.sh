# Round evidence on one MI355X: full -m gpu suite, PMC passes (fetch, write, MFMA busy,
# wave states; one rocprofv3 --pmc run each), their summaries, the kernel trace/stats of the
# bench, the bench line itself (with the fresh PMC summaries), end-to-end generation, IntraGCV,
# workgroup timelines, other configs, measured MFMA peaks.   usage: bash tools/gpu_evidence.sh r02
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dev}
O=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest_$TAG.log; tail -3 $O/gputest_$TAG.log; [ $rc -eq 0 ] || exit 1
fi
# PART=a: everything but the generation / IntraGCV / knockout / timeline runs; PART=b (with
# SKIP_TESTS=1): only those -- two GPU calls under one tag when one would run too long
if [ "$PART" != "b" ]; then
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$TAG -o pmc --output-format csv -- $B > $O/pmcf_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmcf_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$TAG -o pmc --output-format csv -- $B > $O/pmcw_$TAG.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmcw_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmcm_$TAG -o pmc --output-format csv -- $B > $O/pmcm_$TAG.log 2>&1 || { echo "pmc mfma failed"; tail -5 $O/pmcm_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $O/pmcs_$TAG -o pmc --output-format csv -- $B > $O/pmcs_$TAG.log 2>&1 || { echo "pmc stall failed"; tail -5 $O/pmcs_$TAG.log; exit 1; }
F=$(find $O/pmcf_$TAG -name "*counter_collection.csv" | head -1)
W=$(find $O/pmcw_$TAG -name "*counter_collection.csv" | head -1)
M=$(find $O/pmcm_$TAG -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W --out $O/pmc_traffic_$TAG.json || exit 1
python3 tools/pmc_mfma.py $M --out $O/pmc_mfma_$TAG.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --pmc-json $O/pmc_traffic_$TAG.json --pmc-mfma-json $O/pmc_mfma_$TAG.json > $O/prof_bench_$TAG.log 2>&1 || { echo "kernel-trace failed"; tail -20 $O/prof_bench_$TAG.log; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --pmc-json $O/pmc_traffic_$TAG.json --pmc-mfma-json $O/pmc_mfma_$TAG.json > $O/bench_$TAG.log 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
tail -1 $O/bench_$TAG.log | cut -c1-300
fi
if [ "$PART" != "a" ]; then
timeout -k 10 300 python tools/generation_bench.py 24 > $O/generation_$TAG.log 2>&1 || { tail -20 $O/generation_$TAG.log; exit 1; }
tail -1 $O/generation_$TAG.log
# the multi-rank generation path on this one GPU (gloo): 2 and 4 ranks, config 2 and config 3 populations
for POP in 256 1024; do for W in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29600 + W)) tools/generation_bench.py 16 $POP > $O/generation_w${W}_${POP}_$TAG.log 2>&1 || { tail -30 $O/generation_w${W}_${POP}_$TAG.log; exit 1; }
  grep '^{' $O/generation_w${W}_${POP}_$TAG.log | tail -1 | cut -c1-300
done; done
timeout -k 10 300 python tools/generation_bench.py 16 1024 > $O/generation_w1_1024_$TAG.log 2>&1 || { tail -20 $O/generation_w1_1024_$TAG.log; exit 1; }
timeout -k 10 300 python tools/intracv_bench.py > $O/intracv_$TAG.log 2>&1 || { tail -20 $O/intracv_$TAG.log; exit 1; }
grep config $O/intracv_$TAG.log
timeout -k 10 300 python tools/knockout_bench.py > $O/knockout_$TAG.log 2>&1 || { tail -20 $O/knockout_$TAG.log; exit 1; }
tail -1 $O/knockout_$TAG.log
timeout -k 10 200 python tools/wg_trace.py $O/wg_trace_$TAG.npy > $O/wg_trace_$TAG.txt 2>&1 || { tail -20 $O/wg_trace_$TAG.txt; exit 1; }
timeout -k 10 200 python tools/wg_trace.py $O/wg_trace128_$TAG.npy --pop 128 > $O/wg_trace128_$TAG.txt 2>&1 || { tail -20 $O/wg_trace128_$TAG.txt; exit 1; }
fi
[ "$PART" = "b" ] && { echo "evidence part b done"; exit 0; }
timeout -k 10 400 python bench.py --config config4 --steps 5 --warmup 2 > $O/bench_config4_$TAG.log 2> $O/bench_config4_$TAG.err || { tail -20 $O/bench_config4_$TAG.err; exit 1; }
timeout -k 10 300 python bench.py --config config5 --steps 20 --warmup 5 > $O/bench_config5_$TAG.log 2> $O/bench_config5_$TAG.err || { tail -20 $O/bench_config5_$TAG.err; exit 1; }
for P in 32 64 128; do
timeout -k 10 300 python bench.py --pop $P --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pop${P}_$TAG.log 2> $O/bench_pop${P}_$TAG.err || { tail -20 $O/bench_pop${P}_$TAG.err; exit 1; }
done
timeout -k 10 300 python bench.py --config config3 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_config3_$TAG.log 2> $O/bench_config3_$TAG.err || { tail -20 $O/bench_config3_$TAG.err; exit 1; }
for c in config3 config4 config5 pop32 pop64 pop128; do tail -1 $O/bench_${c}_$TAG.log | cut -c1-200; done
timeout -k 10 100 ./tools/mfma_peak > $O/mfma_peak_$TAG.json 2>&1 || exit 1
timeout -k 10 100 ./tools/fp4_probe > $O/fp4_probe_$TAG.json 2>&1 || exit 1
echo evidence done
