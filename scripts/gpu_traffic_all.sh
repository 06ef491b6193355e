#!/bin/bash
# HBM traffic (FETCH_SIZE) and kernel-trace stats for every bench config other
# than c2 (gpu_round.sh does c2): one `--kernel-trace --stats` run and one
# separate `--pmc FETCH_SIZE` run per config (counters never combined with
# tracing). Outputs under gpurun_out/{prof,pmc}_<cfg>/; summarise on the CPU
# side with scripts/summarize_profile.py into profiles/pmc_<cfg>.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
O=gpurun_out
for c in ${CONFIGS:-c3 c4 c5 c5_seg c2_crc64}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o $c -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "prof $c failed"; tail $O/prof_$c.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$c -o $c -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail $O/pmc_$c.log; exit 1; }
  grep '"metric"' $O/prof_$c.log | cut -c1-160
done
echo "traffic all ok"
