#!/bin/bash
# Correctness of the bucketed fold + A/B of the in-tree library against a saved one (GELLY_CC_LIB) and across the P1
# geometries, then PMC passes of the default bench. A step that fails ends the session.
# Usage (GPU box): bash tools/gpu_ab.sh <tag> <old .so>
set -o pipefail
TAG=${1:-r3}
OLD=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "== bucket + window tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_windows.py -x -v --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
trc=$?
tail -3 "$OUT/tests.log"
if [ $trc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/tests.log" | head; exit $trc; fi
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
for v in new_p1_1 old new_p1_2 new_p1_0 new_p1_1b; do
  echo "== $v"
  case $v in
    old) GELLY_CC_LIB=$ROOT/$OLD timeout -k 10 240 $B > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || exit $? ;;
    new_p1_1|new_p1_1b) timeout -k 10 240 $B --tune bucket_p1=1 > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || exit $? ;;
    new_p1_2) timeout -k 10 240 $B --tune bucket_p1=2 > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || exit $? ;;
    new_p1_0) timeout -k 10 240 $B --tune bucket_p1=0 > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || exit $? ;;
  esac
done
for f in "$OUT"/c4_*.json; do python3 -c "
import json
d=json.load(open('$f'));r=d['roofline']
print('$f'.split('/')[-1], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', d['parity'],
      {k: round(v['ms_per_step'],3) for k,v in r['kernels'].items() if v['ms_per_step'] > 0.05})"; done
echo "== pmc" && bash tools/pmc_passes.sh "$TAG" > "$OUT/pmc_passes.log" 2>&1
echo "exit $?"
