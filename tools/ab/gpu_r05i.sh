#!/bin/bash
# round 5: the other configs' bench lines with the round's code (ct x pt, cfg5, cfg2)
set -u
OUT=gpurun_out/r05i
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/$name.json'));r=d.get('roofline') or {}
print(d['value'],d['unit'],d['ms_per_step'],(d.get('self_check') or {}).get('bitexact'),r.get('kernel'),r.get('frac'))" 2>&1 | tail -1)"
  return $rc
}
run ctpt --variant ctpt --no-cpu-baseline --steps 2 --warmup 1 || exit 1
run cfg5 --config cfg5 --no-cpu-baseline --steps 2 --warmup 1 || exit 1
run cfg2 --config cfg2 --steps 20 --warmup 3 || exit 1
