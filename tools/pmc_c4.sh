set -o pipefail
# SQ / TA counter passes over one C4 fold (tools/fold_once.py), one counter group per run (MI355X_MICROARCH.md)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p1.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/p2 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p2.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d $O/p3 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p3.out 2>&1
echo "exit $?"
