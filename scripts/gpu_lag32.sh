# CRC32C generic kernel (lagged blocks, rows 4) vs the fused kernel (0). The lagged-vs-unlagged A/B
# of profiles/tune_r01_lagged_blocks.jsonl used a temporary knob value 3 (the unlagged kernel is gone).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c2 c3 c4 c5seg; do
  timeout -k 10 300 python scripts/tune_gpu.py --config $c --variants generic:4,generic:0 --rounds 6 > gpurun_out/tune_lag32_$c.jsonl 2>&1 || { echo "tune $c failed"; tail -20 gpurun_out/tune_lag32_$c.jsonl; exit 1; }
done
for c in c2 c3 c4 c5seg; do echo "== $c"; grep variant gpurun_out/tune_lag32_$c.jsonl; done
