#!/bin/bash
# Round measurement: bench line (with CPU baseline unless --no-cpu-baseline is passed), rocprofv3 kernel-trace
# stats of the same workload, and FETCH_SIZE / WRITE_SIZE PMC passes (separate passes, gfx950 slot limits) over
# one single-lane step (as the event-timed profile step), summarised per kernel into
# gpurun_out/<tag>/pmc_<kernel>_B<batch>[_<variant>].json; profile_step.json = the rocprof average of the
# roofline kernel over the profile step (tools/profile_step.py).
# usage: [PMC_DIMS="<batch> <logN> <level> <n>"] [PMC_VARIANT=ctpt] bash tools/gpu_profile.sh <tag> [bench args...]
#   cfg3 (default dims 128 15 10 4096, the bench batch):  bash tools/gpu_profile.sh r03_v1
#   ct x pt:  PMC_VARIANT=ctpt bash tools/gpu_profile.sh r03_ctpt --variant ctpt --no-cpu-baseline
#   cfg5:     PMC_DIMS="32 16 16 1024" bash tools/gpu_profile.sh r03_cfg5 --config cfg5 --no-cpu-baseline
set -o pipefail
TAG=${1:-r03}
shift
ARGS="$*"
DIMS=${PMC_DIMS:-"128 15 10 4096"}
export PMC_VARIANT=${PMC_VARIANT:-ctct}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-600
NOCPU="--no-cpu-baseline"
case " $ARGS " in *" --no-cpu-baseline "*) NOCPU="" ;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS $NOCPU > $OUT/trace_bench.json 2> $OUT/trace.log || { tail $OUT/trace.log; exit 1; }
PMCARGS="$ARGS $NOCPU --no-profile --no-self-check --steps 1 --warmup 0"
KRE="k_fan|k_ntt|k_hmacm|k_bmac|k_tensor_multi"
# one lane: each dispatch covers the whole batch, as in bench.py's event-timed profile step
export HEC_LANES=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_fetch.log 2>&1 || { tail $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_write.log 2>&1 || { tail $OUT/pmc_write.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/profile_step.py $OUT/trace/run_kernel_trace.csv $OUT/trace_bench.json $OUT/profile_step.json || exit 1
cp $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_fetch.csv && cp $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_write.csv
python tools/pmc_summary.py $OUT/pmc_fetch.csv $OUT/pmc_write.csv $DIMS $TAG "HEC_LANES=1 rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE, separate pass) --kernel-include-regex '$KRE' -- python3 bench.py $PMCARGS" k_fan2 k_fan2j k_ntt k_hmacm k_bmac k_tensor_multi2 > /dev/null || exit 1
ls $OUT
