# Runs (K set) the GPU tests matching $K, then tools/bench_configs.py group $1, once per
# library under abtmp/ (A/B of build variants)
set -u
cd /root/repo
for L in abtmp/*.so; do
  echo "== $L"
  if [ -n "${K:-}" ]; then
    VOLKIT_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/dev_pytest.log 2>&1 || { tail -30 gpurun_out/dev_pytest.log; exit 1; }
    tail -1 gpurun_out/dev_pytest.log
  fi
  VOLKIT_LIB=$PWD/$L timeout -k 10 300 python tools/bench_configs.py --only "$1" --reps ${REPS:-10} 2>&1 | grep '^{' || exit 1
done
