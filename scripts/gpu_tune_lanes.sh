set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c3 c5seg; do
timeout -k 10 300 python scripts/tune_gpu.py --config $c --variants generic:0,generic:4 --lanes 4,8,16 --rounds 4 > gpurun_out/tune_g_$c.jsonl 2>&1 || { echo "tune failed"; cat gpurun_out/tune_g_$c.jsonl; exit 1; }
echo $c; grep variant gpurun_out/tune_g_$c.jsonl
done
