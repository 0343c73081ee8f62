#!/bin/bash
# A/B of engine switches: quick parity (test_gpu_parity.py), then one bench line per setting.
# usage: bash tools/gpu_ab.sh <tag> "ENV=a ENV2=b" "ENV=c|--batch 128" ...   (text after | = bench.py arguments)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1 || { tail -30 gpurun_out/$TAG/parity.log; exit 1; }
tail -1 gpurun_out/$TAG/parity.log
i=0
for cfg in "$@"; do
  envs=${cfg%%|*}
  args=""
  [[ "$cfg" == *"|"* ]] && args=${cfg#*|}
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/$TAG/b_$i.json 2> gpurun_out/$TAG/b_$i.err || { tail -20 gpurun_out/$TAG/b_$i.err; exit 1; }
  python - "$cfg" gpurun_out/$TAG/b_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: v["ms"] for k, v in d["kernels_one_step"].items()})
PY
  i=$((i+1))
done
