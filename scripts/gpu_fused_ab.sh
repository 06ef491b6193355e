set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for c in c2 c3 c5seg; do
  timeout -k 10 300 python scripts/tune_gpu.py --config $c --variants generic:0,generic:-2,generic:-3,generic:4 --rounds 7 > $O/tune_fused_$c.jsonl 2>&1 || { echo "tune $c failed"; cat $O/tune_fused_$c.jsonl; exit 1; }
  echo $c; grep variant $O/tune_fused_$c.jsonl
done
timeout -k 10 300 python scripts/tune_gpu.py --config c4 --lanes 32,64 --variants generic:0,generic:-2,generic:4 --rounds 5 > $O/tune_fused_c4.jsonl 2>&1 || { echo "tune c4 failed"; exit 1; }
echo c4; grep variant $O/tune_fused_c4.jsonl
