set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p1.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p2.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p3.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p4.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --output-format csv -d $O/p5 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p5.out 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p6 -o run -- python3 $R/tools/fold_once.py c4_kron26 2 > $O/p6.out 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/fold_once.py c4_kron26 3 > $O/trace.out 2>&1
echo "exit $?"
ls $O/*
