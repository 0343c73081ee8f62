#!/bin/bash
# Round-end measurement: bench line (with CPU baseline), rocprofv3 kernel-trace stats of the same
# workload, and FETCH_SIZE / WRITE_SIZE PMC passes (separate passes, gfx950 slot limits) on the
# roofline kernels k_hmacm and k_bmac (one lane, as the profile step), summarised into
# gpurun_out/<tag>/pmc_<kernel>_B96.json; profile_step.json = the rocprof average of the roofline kernel
# over the single-lane profile step (tools/profile_step.py).
# usage: bash tools/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.log || { tail $OUT/trace.log; exit 1; }
PMCARGS="--no-cpu-baseline --no-profile --steps 1 --warmup 0"
# one lane: each dispatch covers the whole batch, as in bench.py's event-timed profile step
export HEC_LANES=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_hmacm|k_bmac" --output-format csv -d $OUT/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_fetch.log 2>&1 || { tail $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_hmacm|k_bmac" --output-format csv -d $OUT/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_write.log 2>&1 || { tail $OUT/pmc_write.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/profile_step.py $OUT/trace/run_kernel_trace.csv $OUT/trace_bench.json $OUT/profile_step.json || exit 1
for k in k_hmacm k_bmac; do
  python tools/pmc_summary.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $k 96 15 10 4096 $OUT/pmc_${k}_B96.json "HEC_LANES=1 rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE, separate pass) --kernel-include-regex 'k_hmacm|k_bmac' -- python3 bench.py $PMCARGS" || exit 1
done
