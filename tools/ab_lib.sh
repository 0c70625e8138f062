#!/bin/bash
# A/B of two builds of libgelly_cc.so on one box, alternating (GELLY_CC_LIB selects the build):
#   bash tools/ab_lib.sh <tag> <other lib> <rounds> <fixture> [time_windows args...]
# Each round runs tools/time_windows.py on the fixture with the in-tree library, then with <other lib>.
set -o pipefail
TAG=$1; OTHER=$2; ROUNDS=$3; FIX=$4; shift 4
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 200 python3 -u "$ROOT/tools/time_windows.py" "$FIX" "$@" > "$OUT/head_$r.log" 2> "$OUT/head_$r.err" || exit $?
  GELLY_CC_LIB="$OTHER" timeout -k 10 200 python3 -u "$ROOT/tools/time_windows.py" "$FIX" "$@" > "$OUT/other_$r.log" 2> "$OUT/other_$r.err" || exit $?
  echo "round $r: head $(grep -o '"median_ms": [0-9.]*' "$OUT/head_$r.log") other $(grep -o '"median_ms": [0-9.]*' "$OUT/other_$r.log")"
done
