set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python scripts/tune_gpu.py --config c2 --variants s64:4:3:1,s64b2:4:1,s64b2:2:3,s64b2:2:2,s64b2:4:2,s64:8:1:1 --rounds 5 > $O/tune_crc64_b2.jsonl 2>&1 || { echo "tune failed"; cat $O/tune_crc64_b2.jsonl; exit 1; }
grep variant $O/tune_crc64_b2.jsonl
timeout -k 10 300 python bench.py --h2d > $O/bench_h2d.log 2>&1 || { echo "h2d failed"; exit 1; }
timeout -k 10 300 python bench.py --h2d --h2d-devices 0 > $O/bench_h2d_multi.log 2>&1 || { echo "h2d multi failed"; exit 1; }
tail -1 $O/bench_h2d.log; tail -1 $O/bench_h2d_multi.log
