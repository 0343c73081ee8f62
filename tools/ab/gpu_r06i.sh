#!/bin/bash
# round 6: k_hmacm's 60-bit targets on the MAC-form streams (hmac_int, default on) — parity subset, then cfg3 B = 128
# A/B: new (hmac_int 1) / new with HEC_HMAC_INT=0 / variants/hmac_r06h.so (the r06h kernel without the new body,
# 4 instead of 10 spilled VGPRs) / new with both shuffle pass B (mode 2 + divide-and-round), alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06i}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "keyswitch or hoisted or matvec or cfg3 or shuffle or cfg5" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=::0" "int0=:0:0" "r06h=variants/hmac_r06h.so::0" "shdr=::1"; do
    name=${v%%=*}; rest=${v#*=}; lib=${rest%%:*}; rest=${rest#*:}; hi=${rest%%:*}; sh=${rest#*:}
    [ -n "$lib" ] && lib=$(realpath $lib)
    env_hi=""; [ -n "$hi" ] && env_hi="HEC_HMAC_INT=$hi"
    env_sh=""; [ "$sh" = 1 ] && env_sh="HEC_NTTB_SHFL=2 HEC_NTTB_SHFL_DR=1"
    env $env_hi $env_sh HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
  done
done
echo done
