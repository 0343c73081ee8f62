#!/bin/bash
# round 5: the new multi-rank / SEAL-IO / he_util GPU tests, then the full-size determinism diagnostic
set -u
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shard.py \
    tests/test_gpu_seal_io.py tests/test_gpu_he_math.py > $OUT/t1.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 $OUT/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u tools/determinism_full.py --reps ${REPS:-6} > $OUT/det.log 2>&1
rc2=$?
echo "det rc=$rc2"
tail -30 $OUT/det.log
exit $rc2
