set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c3 c5seg; do
timeout -k 10 300 python scripts/tune_gpu.py --config $c --variants generic:2,generic:4,generic:8 --lanes 8 --rounds 8 --reps 8 > gpurun_out/tune_rows_$c.jsonl 2>&1 || { echo "tune failed"; tail gpurun_out/tune_rows_$c.jsonl; exit 1; }
echo $c; grep variant gpurun_out/tune_rows_$c.jsonl
done
