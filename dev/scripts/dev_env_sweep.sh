# bench_configs group $1 under each value of env var $2 (values $3...); dev tool
set -u
cd /root/repo
G=$1; V=$2; shift 2
for x in "$@"; do
  echo "== $V=$x"
  env $V=$x timeout -k 10 300 python tools/bench_configs.py --only "$G" --reps ${REPS:-6} 2>&1 | grep '^{' || exit 1
done
