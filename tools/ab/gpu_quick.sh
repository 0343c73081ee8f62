#!/bin/bash
# quick GPU check used during development: parity + bench under several engine settings
set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
i=0
for envs in "$@"; do
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_$i.log 2>&1 || { tail -20 gpurun_out/b_$i.log; exit 1; }
  python - "$envs" gpurun_out/b_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: v["ms"] for k, v in d["breakdown_ms_one_step"].items() if v["ms"]})
PY
  i=$((i+1))
done
