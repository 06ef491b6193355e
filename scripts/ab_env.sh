#!/bin/bash
# A/B of (environment, bench.py arguments) arms on one config, interleaved
# rounds, a fresh process per run (bench-only). Arms are "ENV=..|ARGS".
# Usage: scripts/ab_env.sh CONFIG ROUNDS "PHOTON_CRC_LIB=/path|--rows 4" "|--rows 2" ...
# (AB_ARGS: common arguments, default --steps 200 --warmup 25)
set -o pipefail
c=$1; rounds=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $rounds); do
  for arm in "$@"; do
    IFS='|' read -r envs args <<< "$arm"
    envs=$(eval echo "$envs")
    env $envs timeout -k 10 300 python -u bench.py --config $c $args ${AB_ARGS:---steps 200 --warmup 25} \
      --no-cpu-baseline --no-live-pmc --no-shape64 > $O/ab_tmp.json 2>> $O/ab_env.err || { echo "run $arm failed"; tail -5 $O/ab_env.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/ab_tmp.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'round': $r, 'config': '$c', 'arm': sys.argv[1], 'value': d['value'], 'frac_kernel': r['frac_kernel'], 'frac_steady': r['frac_steady_median_launch'], 'ok': d['self_check']}))" "$arm" | tee -a $O/ab_env.jsonl
  done
done
