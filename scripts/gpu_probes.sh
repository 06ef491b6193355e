set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/probe_hbm.py > gpurun_out/probes.jsonl 2>&1 || { echo "probe failed"; tail gpurun_out/probes.jsonl; exit 1; }
grep probe gpurun_out/probes.jsonl
