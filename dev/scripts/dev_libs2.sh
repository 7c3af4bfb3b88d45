# Full GPU test suite on the tree's build, then per library under abtmp/: size sweep + config3
set -u
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dev_pytest.log 2>&1 || { tail -30 gpurun_out/dev_pytest.log; exit 1; }
tail -1 gpurun_out/dev_pytest.log
for L in abtmp/*.so; do
  echo "== $L"
  VOLKIT_LIB=$PWD/$L timeout -k 10 300 python tools/bench_sizes.py 2>&1 | grep '^{' || exit 1
  VOLKIT_LIB=$PWD/$L timeout -k 10 300 python tools/bench_configs.py --only config3 --reps 5 2>&1 | grep '^{' || exit 1
done
