# C5 benches (per-message and per-segment forms) + rocprof kernel stats for both.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python bench.py --config c5_seg --no-cpu-baseline > $O/bench_c5_seg.log 2>&1 || { echo "bench c5_seg failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --config c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo "prof c5 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_seg -o c5s -- python3 bench.py --config c5_seg --no-cpu-baseline > $O/prof_c5_seg.log 2>&1 || { echo "prof c5_seg failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_crc64 -o c64 -- python3 bench.py --config c2_crc64 --no-cpu-baseline > $O/prof_crc64.log 2>&1 || { echo "prof crc64 failed"; exit 1; }
echo ok
