#!/bin/bash
# round 6 final measurements: the driver's own command (bench.py --steps 20 --warmup 5: CPU leg, oracle self-check,
# profile step inside the warmup) timed from outside, then ct x pt and cfg5 at their defaults (no CPU leg).  A
# background heartbeat under gpurun_out keeps the silence monitor informed while bench.py prints only its final line.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06n}
mkdir -p gpurun_out/$T
( while sleep 60; do date +%s >> gpurun_out/$T/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
t0=$(date +%s.%N)
timeout -k 10 590 python bench.py --steps 20 --warmup 5 > gpurun_out/$T/driver.json 2> gpurun_out/$T/driver.err || { tail gpurun_out/$T/driver.err; exit 1; }
t1=$(date +%s.%N)
python3 -c "print('driver-style run wall', round($t1 - $t0, 1), 's')" | tee gpurun_out/$T/driver_wall.txt
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/driver.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['self_check'], d['wall_s'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --variant ctpt --no-cpu-baseline > gpurun_out/$T/ctpt.json 2> gpurun_out/$T/ctpt.err || { tail gpurun_out/$T/ctpt.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/ctpt.json').read().strip().splitlines()[-1])
print('ctpt', d['value'], d['ms_per_step'], d['self_check']['bitexact'], d['roofline']['frac'])"
timeout -k 10 500 python bench.py --config cfg5 --no-cpu-baseline > gpurun_out/$T/cfg5.json 2> gpurun_out/$T/cfg5.err || { tail gpurun_out/$T/cfg5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/cfg5.json').read().strip().splitlines()[-1])
print('cfg5', d['value'], d['ms_per_step'], d['self_check']['bitexact'], d['roofline']['frac'], d['config'].get('batch_per_gpu'))"
echo done
