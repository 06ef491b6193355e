set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
for c in c5 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o $c -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "prof $c failed"; tail $O/prof_$c.log; exit 1; }
tail -1 $O/prof_$c.log
done
find $O/prof_c5 $O/prof_c3 -name "*stats*"
