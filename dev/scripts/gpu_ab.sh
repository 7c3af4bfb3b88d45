set -u
cd /root/repo
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "resample or chain" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for L in plane row; do
  echo "layout $L"
  VKT_RESAMPLE_LAYOUT=$L timeout -k 10 300 python tools/bench_configs.py --only config3 --reps 5 2>&1 | grep '^{'
  VKT_RESAMPLE_LAYOUT=$L timeout -k 10 300 python tools/bench_configs.py --only metric --reps 10 2>&1 | grep '^{' | head -2
done
