# A/B: GPU tests matching $1, then tools/bench_configs.py group $2 with abtmp/libvolkit_old.so vs the tree's build
set -u
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/dev_pytest.log 2>&1 || { tail -30 gpurun_out/dev_pytest.log; exit 1; }
tail -2 gpurun_out/dev_pytest.log
for L in abtmp/libvolkit_old.so volkit_amd/lib/libvolkit.so; do
  echo "== $L"
  VOLKIT_LIB=$PWD/$L timeout -k 10 300 python tools/bench_configs.py --only "$2" --reps ${REPS:-10} 2>&1 | grep '^{' || exit 1
done
