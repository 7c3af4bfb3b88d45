# Per library under abtmp/: tools/bench_configs.py group $1 under rocprofv3 kernel trace; prints
# per-launch durations (us) of kernels whose name contains $2
set -u
cd /root/repo
export TMPDIR=/tmp
for L in abtmp/*.so; do
  n=$(basename $L .so)
  VOLKIT_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/libprof/$n -o run --output-format csv -- python3 tools/bench_configs.py --only "$1" --reps ${REPS:-4} > gpurun_out/libprof_$n.log 2>&1 || { tail -20 gpurun_out/libprof_$n.log; exit 1; }
  python3 - "$n" "$2" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/libprof/{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if sys.argv[2] in r["Kernel_Name"]]
print(sys.argv[1], [round(x) for x in v])
PY
done
