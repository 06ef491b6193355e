# Usage: bash scripts/gpu_quick.sh "pytest-args" "config ..." -- GPU tests, then bench + rocprof stats per config.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
TESTS=${1:-tests}
CONFIGS=${2:-c2}
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in $CONFIGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o $c -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "prof $c failed"; tail $O/prof_$c.log; exit 1; }
  grep '"metric"' $O/prof_$c.log | cut -c1-200
  python3 - "$O/prof_$c/${c}_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]:
    print("   ", r["Name"][:70], r["Calls"], r["AverageNs"], r["MinNs"])
PY
done
