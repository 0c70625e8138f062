#!/bin/bash
# Run-to-run variance of the default (C4) bench on one box: the same build five times in a row, with the GPU's
# clocks / power / temperature (rocm-smi, read-only) before and after each run. A failing step ends the session.
# Usage (GPU box): bash tools/gpu_variance.sh <tag>
set -o pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
smi() { timeout -k 5 30 rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|fclk|Power|Temperature \(Sensor (edge|junction|memory)" | tr -s ' ' | head -12; }
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
# MODES: one GELLY_CONTIG value per run (default: five runs of the default build)
MODES=${MODES:-"1 1 1 1 1"}
r=0
for mode in $MODES; do
  r=$((r + 1))
  echo "== run $r GELLY_CONTIG=$mode (before)"; smi
  GELLY_CONTIG=$mode timeout -k 10 240 $B > "$OUT/c4_run$r.json" 2> "$OUT/c4_run$r.err" || exit $?
  python3 -c "
import json
d=json.load(open('$OUT/c4_run$r.json'));k=d['roofline']['kernels']
print('run $r contig $mode', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', {n: round(v['ms_per_step'],3) for n,v in k.items() if v['ms_per_step']>0.3})"
  echo "== run $r (after)"; smi
done
exit 0
