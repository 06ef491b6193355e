# CRC-64 (lagged blocks): generic batch kernel vs streaming kernel on the C3 / C4 shapes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c3 c4 c2; do
  timeout -k 10 300 python scripts/tune_gpu.py --config $c --variants s64:4:3:1,s64:4:1:1,g64 --lanes 0,8,16,32,64 --rounds 4 > gpurun_out/tune_lag64_$c.jsonl 2>&1 || { echo "tune $c failed"; tail -20 gpurun_out/tune_lag64_$c.jsonl; exit 1; }
done
for c in c3 c4 c2; do echo "== $c"; grep variant gpurun_out/tune_lag64_$c.jsonl; done
