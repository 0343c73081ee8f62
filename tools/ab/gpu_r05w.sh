#!/bin/bash
# round 5 final: the measurement set (bench with the CPU leg, rocprof stats, PMC passes) on the final code, then one
# bench run with the opt-in 3 concurrent lanes (their self-check after the round-5 root-cause fix)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile.sh r05w || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 > gpurun_out/r05w/lanes1.json \
    2> gpurun_out/r05w/lanes1.err || { tail -5 gpurun_out/r05w/lanes1.err; exit 1; }
HEC_LANES=3 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 \
    > gpurun_out/r05w/lanes3.json 2> gpurun_out/r05w/lanes3.err || { tail -5 gpurun_out/r05w/lanes3.err; exit 1; }
for f in lanes1 lanes3; do python3 -c "
import json;d=json.load(open('gpurun_out/r05w/$f.json'));print('$f',d['value'],d['ms_per_step'],d['self_check'])"; done
