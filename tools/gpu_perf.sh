#!/bin/bash
# One GPU session of measurements (no tests): C4 A/B of the P2 round size, the other configs, the inc_div sweep.
# Every GPU step is time-limited; the chain stops at the first failure of a step (any non-zero status).
# Usage (on the GPU box): bash tools/gpu_perf.sh <tag>
set -o pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
echo "== c4 p2_per 8" && timeout -k 10 240 $B > "$OUT/c4_p8.json" 2> "$OUT/c4_p8.err" && \
echo "== c4 p2_per 12" && timeout -k 10 240 $B --tune bucket_p2_per=12 > "$OUT/c4_p12.json" 2> "$OUT/c4_p12.err" && \
echo "== c4 p2_per 8 again" && timeout -k 10 240 $B > "$OUT/c4_p8b.json" 2> "$OUT/c4_p8b.err" && \
echo "== c4 share" && timeout -k 10 240 $B --workload c4_share > "$OUT/c4share.json" 2> "$OUT/c4share.err" && \
echo "== c5" && timeout -k 10 240 $B --workload c5_adversarial > "$OUT/c5.json" 2> "$OUT/c5.err" && \
echo "== c2 x16" && timeout -k 10 240 $B --workload c2_rmat20 --window-edges 1048576 > "$OUT/c2w16.json" 2> "$OUT/c2w16.err" && \
echo "== c3" && timeout -k 10 240 $B --workload c3_gnm24 > "$OUT/c3.json" 2> "$OUT/c3.err" && \
echo "== inc_div sweep" && timeout -k 10 400 python -u tools/sweep_inc_div.py > "$OUT/sweep_inc_div.log" 2>&1
rc=$?
echo "exit $rc"
for f in "$OUT"/*.json; do python3 -c "
import json,sys
d=json.load(open('$f'));r=d.get('roofline',{});p=r.get('pipeline',{})
print('$f'.split('/')[-1], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', d.get('parity'),
      {k: round(v['ms_per_step'],3) for k,v in r.get('kernels',{}).items()})" 2>/dev/null; done
exit $rc
