# Stall-breakdown PMC passes for one kernel family, default lib and variants:
#   bash tools/runs/pmc_stalls.sh encode|restore [variant.so ...]
# Outputs gpurun_out/stall_<tag>/<pass>/ (summarise with tools/pmc_summary.py).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
ONLY=$1; shift
P="rocprofv3 --kernel-trace -T -f csv"
run() {  # tag lib
  D=gpurun_out/stall_$1; mkdir -p $D
  [ -n "$2" ] && export VDS_EC_LIB=$2 || unset VDS_EC_LIB
  timeout -k 10 120 $P --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $D/p1 -o run -- python tools/prof_kernels.py --objects 64 --iters 2 --only $ONLY > $D/p1.log 2>&1 &&
  timeout -k 10 120 $P --pmc SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $D/p2 -o run -- python tools/prof_kernels.py --objects 64 --iters 2 --only $ONLY > $D/p2.log 2>&1 &&
  timeout -k 10 120 $P --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_avr TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum -d $D/p3 -o run -- python tools/prof_kernels.py --objects 64 --iters 2 --only $ONLY > $D/p3.log 2>&1
}
run default "" || exit $?
for v in "$@"; do run $(basename $v .so) $v || exit $?; done
