#!/bin/bash
# A/B of lane-group sizes on one config in one box, interleaved rounds, a
# fresh process per run (bench-only). Usage: scripts/ab_lanes.sh CONFIG ROUNDS LANES...
set -o pipefail
c=$1; rounds=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $rounds); do
  for L in "$@"; do
    timeout -k 10 300 python -u bench.py --config $c --lanes $L ${AB_ARGS:---steps 50 --warmup 10} --no-cpu-baseline --no-live-pmc \
      --no-shape64 > $O/ab_tmp.json 2>> $O/ab_lanes.err || { echo "run $c $L failed"; tail -5 $O/ab_lanes.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/ab_tmp.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'round': $r, 'config': '$c', 'lanes': $L, 'value': d['value'], 'frac_kernel': r['frac_kernel'], 'frac_steady': r['frac_steady_median_launch'], 'ok': d['self_check']}))" | tee -a $O/ab_lanes.jsonl
  done
done
