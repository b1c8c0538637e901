# PMC passes (one counter group per rocprofv3 run; no --sys/--runtime trace)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
P="timeout -k 10 240 rocprofv3 --kernel-trace -T -f csv"
$P --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > gpurun_out/pmc/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > gpurun_out/pmc/write.log 2>&1 &&
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/sq -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > gpurun_out/pmc/sq.log 2>&1 &&
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc/lds -o run -- python tools/prof_kernels.py --objects 64 --iters 2 > gpurun_out/pmc/lds.log 2>&1
echo "pmc rc=$?"
