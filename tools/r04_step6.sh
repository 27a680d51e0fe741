# round 4: A/B of column 0 inside the diagonal launch (pop 256: auto = fused; pop 128: auto = own
# launch) and last-term mode at pop 128, then the full evidence run r04a
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
POPS="256" bash tools/ab_env.sh 3 "var=" "nofuse=TBLUP_FUSE_COL0=0" 2>&1 | tee gpurun_out/r04_fuse256.txt || exit 1
POPS="128" bash tools/ab_env.sh 3 "var=" "lt=TBLUP_LAST_TERM=1" "fuse=TBLUP_FUSE_COL0=1" 2>&1 | tee gpurun_out/r04_fuse128.txt || exit 1
# stochastic PC sampling of the bench (instruction-level stall reasons for the off-diagonal kernel)
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/pcs_r04 -o pcs --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pcs_r04.log 2>&1; echo "pcs rc=$?"; tail -5 gpurun_out/pcs_r04.log; find gpurun_out/pcs_r04 -type f | head
