# SQ / LDS counters for the restore kernel only: bash tools/runs/pmc_restore.sh TAG
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
D=gpurun_out/pmcr_${1:-x}; mkdir -p $D
P="rocprofv3 --kernel-trace -f csv"
timeout -k 10 240 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $D/sq -o run -- python tools/prof_kernels.py --objects 32 --iters 2 --only restore > $D/sq.log 2>&1 &&
timeout -k 10 240 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $D/lds -o run -- python tools/prof_kernels.py --objects 32 --iters 2 --only restore > $D/lds.log 2>&1
rc=$?
python - "$D" <<'PY'
import csv, sys, collections
d = sys.argv[1]
for part in ("sq", "lds"):
    acc = collections.defaultdict(list)
    dur = []
    for r in csv.DictReader(open(f"{d}/{part}/run_counter_collection.csv")):
        if "k_restore" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(part, k, round(sum(v) / len(v)))
PY
exit $rc
