#!/bin/bash
# round 5: try to reproduce the r04 full-size mismatch in its original setting (3 lanes forced, the suite's module
# order up to the full-size tests), then a long isolated repro loop with lanes — diagnostics only
set -u
OUT=gpurun_out/r05k
mkdir -p $OUT
HEC_LANES=3 timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_cpp_facade.py \
    tests/test_gpu_encode.py tests/test_gpu_fullsize.py > $OUT/suite_lanes3.log 2>&1
rc=$?
echo "suite (HEC_LANES=3) rc=$rc"; tail -3 $OUT/suite_lanes3.log; grep -E "FAILED|AssertionError|decrypt error" $OUT/suite_lanes3.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/determinism_full.py --reps 40 --poison-reps 0 --serial-reps 0 --onelane-reps 0 \
    > $OUT/det40.log 2>&1
rc=$?
echo "det rc=$rc"; grep -c "alone==lanes=\[True, True, True, True\] lanes!=first at \[\] alone!=first at \[\]" $OUT/det40.log; grep -v "True, True, True, True\] lanes!=first at \[\] alone!=first at \[\]" $OUT/det40.log | tail -20
exit $rc
