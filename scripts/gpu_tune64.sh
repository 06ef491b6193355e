set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_gpu.py --config c2 --variants s64:4:3:1,s64:4:1:1,s64:2:2:1,s64:2:3:1,s64:8:1:1,s64:4:2:1,s64:2:4:1,s64:4:2:2,s64:2:2:2,g64 --rounds 4 > gpurun_out/tune64_shapes.jsonl 2>&1 || { echo "tune failed"; cat gpurun_out/tune64_shapes.jsonl; exit 1; }
grep variant gpurun_out/tune64_shapes.jsonl
