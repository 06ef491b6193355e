#!/bin/bash
# One parameterised driver for GPU-box work (replaces round 1's one-off
# gpu_*.sh wrappers). Every GPU step has its own time limit, steps stop at the
# first failure (no retries), outputs land under gpurun_out/.
#
#   scripts/gpu.sh tests                 pytest -m gpu + smoke()
#   scripts/gpu.sh bench [ARGS...]       python bench.py ARGS  -> gpurun_out/bench_<tag>.json
#   scripts/gpu.sh prof CONFIG [ARGS]    rocprofv3 --kernel-trace --stats of bench.py --config CONFIG
#   scripts/gpu.sh pmc CONFIG            rocprofv3 --pmc FETCH_SIZE pass (counters only)
#   scripts/gpu.sh sq CONFIG             SQ/GRBM counter passes (scripts/pmc_kernel.sh)
#   scripts/gpu.sh probe SCRIPT [ARGS]   python scripts/SCRIPT ARGS (bench-only probes)
#   scripts/gpu.sh ab LIB ROUNDS CONFIG.. A/B of another build of the library (PHOTON_CRC_LIB=LIB)
#                                        against the in-tree one, alternating, fresh process each
#                                        (a run whose self-check fails -- ablation builds -- is
#                                        recorded with "ok": false, not a failure); AB_NEW=LIB2 puts
#                                        another build on the "new" side; AB_ARGS adds bench.py arguments
#                                        (e.g. AB_ARGS="--steps 20 --warmup 5": the driver's conditions)
#   scripts/gpu.sh abn CONFIG ROUNDS LIB.. the in-tree build and every LIB, order reversed every other round
# Several commands chain with "::", e.g.
#   scripts/gpu.sh tests :: bench --steps 20 --warmup 5 :: prof c2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
n=0

run_one() {
  local cmd=$1; shift
  n=$((n+1))
  case $cmd in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
        || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; return 1; }
      tail -3 $O/pytest_gpu.log
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; return 1; } ;;
    bench)
      local tag; tag=$(echo "$*" | tr -c 'a-zA-Z0-9_' '_' | sed 's/__*/_/g;s/^_//;s/_$//'); tag=${tag:-default}
      timeout -k 10 600 python -u bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err \
        || { echo "bench $* failed"; tail -20 $O/bench_$tag.err; return 1; }
      cut -c1-400 $O/bench_$tag.json ;;
    prof)
      local c=$1; shift
      local pt; pt=$(echo "$c $*" | tr -c 'a-zA-Z0-9_' '_' | sed 's/__*/_/g;s/^_//;s/_$//')  # prof c2 --extend -> prof_c2_extend
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$pt -o $c -- \
        python3 bench.py --config $c --no-cpu-baseline --no-live-pmc "$@" > $O/prof_$pt.log 2>&1 \
        || { echo "prof $c failed"; tail -20 $O/prof_$pt.log; return 1; } ;;
    pmc)
      local c=$1
      timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$c -o $c -- \
        python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-live-pmc --no-shape64 > $O/pmc_$c.log 2>&1 \
        || { echo "pmc $c failed"; tail -20 $O/pmc_$c.log; return 1; } ;;
    sq)
      bash scripts/pmc_kernel.sh $1 $O/sq_$1 > /dev/null || { echo "sq $1 failed"; return 1; } ;;
    probe)
      local s=$1; shift
      local pn; pn=$O/probe_${s%.py}_$(date +%s)_$n  # unique across gpu.sh invocations of one call
      timeout -k 10 600 python -u scripts/$s "$@" > $pn.jsonl 2> $pn.err \
        || { echo "probe $s failed"; tail -20 $pn.err; return 1; }
      cut -c1-300 $pn.jsonl ;;
    ab)
      local lib=$1 rounds=$2; shift 2
      for r in $(seq 1 $rounds); do
        for c in "$@"; do
          for side in new old; do
            local envv=""; [ $side = old ] && envv="PHOTON_CRC_LIB=$lib"
            [ $side = new ] && [ -n "$AB_NEW" ] && envv="PHOTON_CRC_LIB=$AB_NEW"
            env $envv timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-live-pmc --no-shape64 $AB_ARGS \
              > $O/ab_tmp.json 2>> $O/ab.err || [ "$(wc -l < $O/ab_tmp.json)" -gt 0 ] \
              || { echo "ab $c $side failed"; tail -5 $O/ab.err; return 1; }  # (self-check false still prints its line: ablation builds)
            python -c "import json,sys; d=json.loads(open('$O/ab_tmp.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'round': $r, 'config': '$c', 'side': '$side', 'args': '$AB_ARGS', 'value': d['value'], 'frac_kernel': r['frac_kernel'], 'frac_steady': r['frac_steady_median_launch'], 'ok': d['self_check']}))" | tee -a $O/ab.jsonl
          done
        done
      done ;;
    abn)
      # abn CONFIG ROUNDS LIB... : every build (in-tree = "new"), order reversed every other round
      local c=$1 rounds=$2; shift 2
      local libs=(new "$@")
      for r in $(seq 1 $rounds); do
        local order=("${libs[@]}")
        [ $((r % 2)) -eq 0 ] && order=($(printf '%s\n' "${libs[@]}" | tac))
        for lib in "${order[@]}"; do
          local envv=""; [ $lib != new ] && envv="PHOTON_CRC_LIB=$lib"
          env $envv timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-live-pmc --no-shape64 $AB_ARGS \
            > $O/ab_tmp.json 2>> $O/ab.err || [ "$(wc -l < $O/ab_tmp.json)" -gt 0 ] \
            || { echo "abn $c $lib failed"; tail -5 $O/ab.err; return 1; }
          python -c "import json,sys; d=json.loads(open('$O/ab_tmp.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'round': $r, 'config': '$c', 'lib': '$lib', 'value': d['value'], 'frac_kernel': r['frac_kernel'], 'frac_steady': r['frac_steady_median_launch'], 'ok': d['self_check']}))" | tee -a $O/abn.jsonl
        done
      done ;;
    *) echo "unknown command $cmd"; return 1 ;;
  esac
}

args=()
for a in "$@" "::"; do
  if [ "$a" = "::" ]; then
    [ ${#args[@]} -gt 0 ] && { run_one "${args[@]}" || exit 1; }
    args=()
  else
    args+=("$a")
  fi
done
echo "gpu.sh: all ok"
