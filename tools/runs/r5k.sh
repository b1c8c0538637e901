# Round 5: the k = 16 survivor-set kernel's scatter fill from the stage-1
# registers (VDS_FILL_REGS) with its XORs before stage 1's barrier
# (VDS_FILL_EARLY; default) or after it (ab/late), and the staging in each
# wave's branch, against the previous build (ab/prev); GPU suite first.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5k; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
echo "[2] k16"; AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/late/libvds_ec.so ab/prev/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
cat $D/ab_k16.log
echo "[3] k32"; AB_OBJECTS=256 AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k32.log 2>&1 || exit 1
cat $D/ab_k32.log
