set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_checked_batch.py tests/test_vdma.py tests/test_cpp_consumers.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --rpc-batch > gpurun_out/bench_rpc.log 2>&1 || { echo "rpc failed"; exit 1; }
tail -1 gpurun_out/bench_rpc.log | cut -c1-250
timeout -k 10 300 python bench.py --rpc-latency > gpurun_out/rpc_latency.log 2>&1 || { echo "latency failed"; exit 1; }
tail -1 gpurun_out/rpc_latency.log
