set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03s
for e in 4 2; do
  HEC_BMAC_EPT=$e timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg3" > gpurun_out/r03s/t$e.log 2>&1 || { tail -20 gpurun_out/r03s/t$e.log; exit 1; }
  tail -1 gpurun_out/r03s/t$e.log
done
for e in 8 4 2; do
  HEC_BMAC_EPT=$e timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03s/b$e.json 2> gpurun_out/r03s/b$e.err || exit 1
  echo "$e $(head -c 110 gpurun_out/r03s/b$e.json)"
done
