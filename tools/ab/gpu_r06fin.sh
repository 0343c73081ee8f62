#!/bin/bash
# round 6 final check of the default build: the whole -m gpu suite and smoke(), then the driver's own command
# (bench.py --steps 20 --warmup 5 with the CPU leg), wall time taken from outside; a heartbeat keeps the monitor informed
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06fin}
mkdir -p gpurun_out/$T
bash tools/gpu_suite.sh $T || exit 1
( while sleep 60; do date +%s >> gpurun_out/$T/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
t0=$(date +%s.%N)
timeout -k 10 590 python bench.py --steps 20 --warmup 5 > gpurun_out/$T/driver.json 2> gpurun_out/$T/driver.err || { tail gpurun_out/$T/driver.err; exit 1; }
t1=$(date +%s.%N)
python3 -c "print('driver-style run wall', round($t1 - $t0, 1), 's')" | tee gpurun_out/$T/driver_wall.txt
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/driver.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['self_check']['bitexact'], d['wall_s']['total_s'], d['roofline']['frac'], d['cpu_baseline']['value'], d['kernels_one_step']['k_hmacm']['ms'])"
