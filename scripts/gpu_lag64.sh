# CRC-64 lagged block CRC: parity first, then the streaming shapes A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc64.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lag64_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lag64_tests.log; exit 1; }
timeout -k 10 400 python scripts/tune_gpu.py --config c2 --variants s64:4:3:1,s64:4:1:1,s64:2:3:1,s64:8:1:1,s64:4:3:2,s64:4:2:4,s64b2:4:1,s64b2:2:3,g64 --lanes 0,16,32 --rounds 4 > gpurun_out/tune_lag64.jsonl 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_lag64.jsonl; exit 1; }
timeout -k 10 300 python bench.py --config c2_crc64 --no-cpu-baseline > gpurun_out/bench_c2_crc64.log 2>&1 || { echo "bench failed"; exit 1; }
tail -n 2 gpurun_out/lag64_tests.log
cat gpurun_out/tune_lag64.jsonl
tail -n 1 gpurun_out/bench_c2_crc64.log
