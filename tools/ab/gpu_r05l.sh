#!/bin/bash
# round 5: the periodic lane mismatch (r05k: reps 6, 11, 16, ... of 40) with lane debugging on: zero-list counts and
# overflow flag per lane and call, per-key table checksums; then with the lanes serialised
set -u
OUT=gpurun_out/r05l
mkdir -p $OUT
HEC_DEBUG_LANES=1 timeout -k 10 900 python -u tools/determinism_full.py --reps ${REPS:-25} --serial-reps ${SREPS:-15} \
    --poison-reps 0 --onelane-reps 0 > $OUT/det.log 2>&1
rc=$?
echo "det rc=$rc"
grep -E "^(lanes3|serial)" $OUT/det.log | sed 's/lanes!=first.*//' | awk '{print $1, $3, $4, $5, $6}' | tr '\n' ';'
echo; grep -E "zero-list nodes [1-9]|overflow [1-9]|[1-9][0-9]* changed" $OUT/det.log | sort | uniq -c | head -20
exit $rc
