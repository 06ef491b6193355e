# Lanes per segment for the zero-copy CheckedMessage batch (payload in pinned
# host memory, read by the kernels over the host link): one bench line each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in 0 16 32 64; do
  timeout -k 10 300 python bench.py --rpc-batch --lanes $l > gpurun_out/rpc_lanes_$l.log 2>&1 || { echo "rpc lanes $l failed"; tail gpurun_out/rpc_lanes_$l.log; exit 1; }
  echo "lanes $l: $(tail -1 gpurun_out/rpc_lanes_$l.log | cut -c1-260)"
done
