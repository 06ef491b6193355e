#!/bin/bash
# One GPU session: parity tests, smoke, bench for every config, h2d, rocprof
# stats + PMC for c2. Each GPU step has its own time limit; stops at the first
# failure (no retries). Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
for c in c2 c3 c4 c5 c2_crc64; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 300 python bench.py --h2d > $O/bench_h2d.log 2>&1 || { echo "h2d failed"; exit 1; }
timeout -k 10 300 python bench.py --rpc-batch > $O/bench_rpc.log 2>&1 || { echo "rpc-batch failed"; exit 1; }
timeout -k 10 300 python bench.py --file-records > $O/bench_file.log 2>&1 || { echo "file-records failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c2 -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_c2.log 2>&1 || { echo "pmc failed"; exit 1; }
bash scripts/pmc_kernel.sh c2 $O/sq_c2 > /dev/null || { echo "sq c2 failed"; exit 1; }
bash scripts/pmc_kernel.sh c2_crc64 $O/sq_c2_crc64 > /dev/null || { echo "sq crc64 failed"; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "bench default failed"; exit 1; }
echo "all ok"
