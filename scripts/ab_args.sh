#!/bin/bash
# A/B of bench.py argument sets on one config, interleaved rounds, a fresh
# process per run (bench-only). Usage: scripts/ab_args.sh CONFIG ROUNDS "ARGS A" "ARGS B" ...
# (AB_ARGS: common arguments, default --steps 200 --warmup 25)
set -o pipefail
c=$1; rounds=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $rounds); do
  for a in "$@"; do
    timeout -k 10 300 python -u bench.py --config $c $a ${AB_ARGS:---steps 200 --warmup 25} --no-cpu-baseline \
      --no-live-pmc --no-shape64 > $O/ab_tmp.json 2>> $O/ab_args.err || { echo "run $c $a failed"; tail -5 $O/ab_args.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/ab_tmp.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'round': $r, 'config': '$c', 'args': sys.argv[1], 'value': d['value'], 'frac_kernel': r['frac_kernel'], 'frac_steady': r['frac_steady_median_launch'], 'ok': d['self_check']}))" "$a" | tee -a $O/ab_args.jsonl
  done
done
