#!/bin/bash
# round 5: k_tensor_multi2 grid in XCD clusters of S batch groups (HEC_TENSOR_XCD) — parity, A/B with PMC traffic
set -u
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "variants or ct_x_pt" > $OUT/parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 $OUT/parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for S in 0 8 32; do
    HEC_TENSOR_XCD=$S timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/x${S}_$rep.json 2> $OUT/x${S}_$rep.err
    rc=$?
    echo "xcd=$S rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/x${S}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],'tensor',k['k_tensor_multi2']['ms'])" 2>&1 | tail -1)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
for S in 0 8 32; do
  HEC_TENSOR_XCD=$S timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_tensor_multi2 --output-format csv \
      -d $GRAFT_REPO_ROOT/$OUT/pmc_x$S -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 \
      > $GRAFT_REPO_ROOT/$OUT/pmc_x$S.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/pmc_x$S.log; exit 1; }
  python3 -c "
import csv
d={}
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/$OUT/pmc_x$S/run_counter_collection.csv')):
    if 'k_tensor_multi2' in r['Kernel_Name'] and r['Counter_Name']=='FETCH_SIZE':
        d[r['Dispatch_Id']]=d.get(r['Dispatch_Id'],0.0)+float(r['Counter_Value'])
print('xcd=$S FETCH_SIZE kB per dispatch', sum(d.values())/len(d), 'dispatches', len(d))"
done
