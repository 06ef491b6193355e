set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_gpu.py --config c3 --variants generic:4,stream:1:4:3,stream:1:4:4,stream:1:8:2 --lanes 8,16,32,64 --rounds 4 --reps 5 > gpurun_out/tune_c3_wide.jsonl 2>&1 || { echo "tune failed"; tail gpurun_out/tune_c3_wide.jsonl; exit 1; }
grep variant gpurun_out/tune_c3_wide.jsonl
