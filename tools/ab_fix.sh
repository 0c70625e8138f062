#!/bin/bash
# Interleaved A/B/n of library builds over several fixtures on one box (GELLY_CC_LIB; "-" = the in-tree build):
#   bash tools/ab_fix.sh <tag> <rounds> "<fixture> [<fixture> ...]" name=lib.so[@k=v,...] [name=... ...]
# (@k=v,...: tuning knobs, time_windows.py --variant)
# Per round, per fixture, per build: tools/time_windows.py --steps 10 --rounds 1 (a digest check included).
# TWARGS (env): extra time_windows.py arguments (e.g. --profile). A step that fails ends the session.
set -o pipefail
TAG=$1; ROUNDS=$2; FIXES=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for fx in $FIXES; do
    f=${fx//\//_}
    line="round $r $fx:"
    for nl in "$@"; do
      name=${nl%%=*}; lib=${nl#*=}; var=default
      case $lib in *@*) var=${lib#*@}; lib=${lib%%@*} ;; esac
      if [ "$lib" = "-" ]; then
        timeout -k 10 200 python3 -u "$ROOT/tools/time_windows.py" "$fx" --steps 10 --rounds 1 $TWARGS --variant "$var" > "$OUT/${f}_${name}_$r.log" 2> "$OUT/${f}_${name}_$r.err" || exit $?
      else
        GELLY_CC_LIB="$ROOT/$lib" timeout -k 10 200 python3 -u "$ROOT/tools/time_windows.py" "$fx" --steps 10 --rounds 1 $TWARGS --variant "$var" > "$OUT/${f}_${name}_$r.log" 2> "$OUT/${f}_${name}_$r.err" || exit $?
      fi
      line="$line $name $(grep -o '"median_ms": [0-9.]*' "$OUT/${f}_${name}_$r.log" | cut -d' ' -f2) $(grep -o '"parity": "[^"]*"' "$OUT/${f}_${name}_$r.log" | cut -c12-)"
    done
    echo "$line" | tee -a "$OUT/summary.txt"
  done
done
exit 0
