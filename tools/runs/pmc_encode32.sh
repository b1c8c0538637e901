# SQ / LDS counters of the k = 32 encode kernels (n = 40 and the live n = 64), one pass each
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
D=gpurun_out/sq32; mkdir -p $D
P="rocprofv3 --kernel-trace"
for cfg in "8 32" "32 16"; do set -- $cfg
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/sq_m$1 -o run -- python tools/prof_kernels.py --k 32 --m $1 --objects $2 --iters 2 --only encode > $D/sq_m$1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $D/lds_m$1 -o run -- python tools/prof_kernels.py --k 32 --m $1 --objects $2 --iters 2 --only encode > $D/lds_m$1.log 2>&1
done
echo done
