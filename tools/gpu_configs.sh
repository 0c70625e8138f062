#!/bin/bash
# Benches of every BASELINE config at HEAD (one box) [+ a C4 seeding-sample sweep with SWEEP=1]. A step that fails ends the session.
# Usage (GPU box): bash tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
run() {  # name, bench args...
  local name=$1; shift
  echo "== $name"
  timeout -k 10 240 $B "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run c4 || exit $?
if [ "${SWEEP:-0}" = 1 ]; then  # the seeding-sample sweep (SWEEP=1)
  run c4_s10 --tune bucket_sample=0.1 || exit $?
  run c4_s20 --tune bucket_sample=0.2 || exit $?
  run c4_s30 --tune bucket_sample=0.3 || exit $?
fi
run c4share --workload c4_share || exit $?
run c5 --workload c5_adversarial || exit $?
run c2w16 --workload c2_rmat20 --window-edges 1048576 || exit $?
run c2 --workload c2_rmat20 || exit $?
run c3 --workload c3_gnm24 || exit $?
for f in "$OUT"/c*.json; do python3 -c "
import json
d=json.load(open('$f'));r=d.get('roofline',{})
print('$f'.split('/')[-1], round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d.get('parity'),
      {k: round(v['ms_per_step'],3) for k,v in r.get('kernels',{}).items() if v['ms_per_step'] > 0.005})"; done
exit 0
