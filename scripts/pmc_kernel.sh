#!/bin/bash
# Per-kernel SQ counters for one bench config, one rocprofv3 --pmc pass per
# counter group (never combined with tracing). Usage: scripts/pmc_kernel.sh CONFIG OUTDIR
set -o pipefail
CFG=${1:-c2}
O=${2:-gpurun_out/pmc_$CFG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- python3 bench.py --config $CFG --steps 5 --warmup 3 --no-cpu-baseline --no-live-pmc --no-shape64 > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo done
