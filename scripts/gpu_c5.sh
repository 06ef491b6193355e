set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c5 c5_seg; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o $c -- python3 bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
grep '"metric"' gpurun_out/bench_$c.log | cut -c1-120
grep '"metric"' gpurun_out/bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"], d["self_check"])'
done
