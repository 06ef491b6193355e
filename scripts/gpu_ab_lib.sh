# A/B two builds of the library on one box: A = photonlibos_amd/lib_ab (baseline), B = the in-tree build.
# Usage: bash scripts/gpu_ab_lib.sh "<tune_gpu.py args>" ; alternating A B A B, one process each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="$1"
for r in 1 2; do
  PHOTON_CRC_LIB=photonlibos_amd/lib_ab/libphoton_checksum.so timeout -k 10 200 python scripts/tune_gpu.py $ARGS > gpurun_out/ab_A$r.jsonl 2>&1 || { echo "A$r failed"; tail -5 gpurun_out/ab_A$r.jsonl; exit 1; }
  timeout -k 10 200 python scripts/tune_gpu.py $ARGS > gpurun_out/ab_B$r.jsonl 2>&1 || { echo "B$r failed"; tail -5 gpurun_out/ab_B$r.jsonl; exit 1; }
done
for f in A1 B1 A2 B2; do echo "== $f"; grep variant gpurun_out/ab_$f.jsonl; done
