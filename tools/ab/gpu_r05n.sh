#!/bin/bash
# round 5: full GPU suite + smoke with engine memops as the default, then 25 reps of the concurrent-lane
# determinism loop (the round-2/4 mismatch reproducer) on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_suite.sh r05n || exit 1
HEC_DEBUG_LANES=1 timeout -k 10 600 python -u tools/determinism_full.py --reps ${REPS:-25} --serial-reps 0 \
    --poison-reps 0 --onelane-reps 0 > gpurun_out/r05n/det.log 2>&1 || { tail -20 gpurun_out/r05n/det.log; exit 1; }
echo "clean reps: $(grep -E '^lanes3' gpurun_out/r05n/det.log | grep -c 'True, True, True, True\] lanes!=first at \[\] alone')"
echo "zero-list reports: $(grep -cE 'zero-list nodes [1-9]' gpurun_out/r05n/det.log || true)"
