#!/bin/bash
# round 5: the periodic lane mismatch with the engine's own fill / copy kernels in place of hipMemsetAsync /
# hipMemcpyAsync D2D (HEC_KERNEL_MEMOPS=1), then the runtime calls again as the control, same box
set -u
OUT=gpurun_out/r05m
mkdir -p $OUT
for V in 1 0; do
  HEC_KERNEL_MEMOPS=$V HEC_DEBUG_LANES=1 timeout -k 10 600 python -u tools/determinism_full.py --reps ${REPS:-25} \
      --serial-reps 0 --poison-reps 0 --onelane-reps 0 > $OUT/det_km$V.log 2>&1
  rc=$?
  echo "kernel_memops=$V det rc=$rc"
  grep -E "^lanes3" $OUT/det_km$V.log | grep -c "True, True, True, True\] lanes!=first at \[\] alone"
  grep -E "^lanes3" $OUT/det_km$V.log | grep -v "True, True, True, True\] lanes!=first at \[\] alone" | awk '{print $1}' | tr '\n' ' '; echo
  grep -cE "zero-list nodes [1-9]" $OUT/det_km$V.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
