#!/bin/bash
# Several probe_power.py sessions in one GPU call, each in a fresh process,
# each written to gpurun_out/power_<label>.jsonl (bench-only).
# Usage: scripts/power_set.sh "label|ENV=.. ENV=..|KERNELS" ...
set -o pipefail
O=gpurun_out; mkdir -p $O
for spec in "$@"; do
  IFS='|' read -r label envs kernels <<< "$spec"
  envs=$(eval echo "$envs")
  env $envs KERNELS=$kernels IDLE_S=${IDLE_S:-1} timeout -k 10 300 python -u scripts/probe_power.py \
    > $O/power_$label.jsonl 2> $O/power_$label.err || { echo "power $label failed"; tail -5 $O/power_$label.err; exit 1; }
  python3 - "$O/power_$label.jsonl" "$label" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "phase" not in d:
        continue
    w, s = d["window"], d["steady"]
    print(sys.argv[2], d["kernel"], "window", w["frac_of_8TBps"], "steady", s["frac_of_8TBps"], s.get("J_per_GiB"),
          s.get("power_w_energy"), s.get("gfx_clk_mhz_sampled"))
PY
done
