#!/bin/bash
# Atomic-throughput counters (north_star: "rocprof counters for achieved HBM GB/s and atomic throughput"): one PMC
# pass of TCC atomic counters + the TA's flat-atomic wavefronts, and one kernel-trace pass for the durations, over
# tools/fold_once.py for each workload. Usage on the GPU box: bash tools/pmc_atomics.sh <tag> [workloads...]
set -o pipefail
TAG=${1:-r2}; shift
WLS=${*:-c4_kron26 c3_gnm24 c2_rmat20}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/atom_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for w in $WLS; do
  mkdir -p "$O/$w"
  timeout -s KILL 120 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum \
      --output-format csv -d "$O/$w/pmc" -o run -- python3 "$R/tools/fold_once.py" "$w" 3 > "$O/$w/pmc.out" 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$w/trace" -o run -- \
      python3 "$R/tools/fold_once.py" "$w" 3 > "$O/$w/trace.out" 2>&1 || exit 1
done
echo "exit 0"
