# Rehearsal of the driver's N>1 bench launch on a one-GPU box: 2 ranks share
# the GPU (bench.py maps ranks beyond the visible devices round-robin).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 5 > gpurun_out/bench_2ranks.log 2>&1 || { echo "2-rank bench failed"; tail -20 gpurun_out/bench_2ranks.log; exit 1; }
grep '"metric"' gpurun_out/bench_2ranks.log | cut -c1-400
