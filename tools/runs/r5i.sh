# Round 5: slot-major stage C (each slot read once per cell group) against the
# previous cell-major form (ab/base), k = 16 and k = 32; and the k = 32 RT
# restore kernel without the RT2 rows compiled in (ab/nort2, -DVDS_SYN_RT2=0:
# no 176-VGPR spill) against the default, both with VDS_EC_RT2=0.
cd $GRAFT_REPO_ROOT
set -o pipefail
mkdir -p gpurun_out/r5i
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r5i/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5i/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5i/pytest_gpu.log
echo "[2] k16"; AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/base/libvds_ec.so > gpurun_out/r5i/ab_k16.log 2>&1 || exit 1
cat gpurun_out/r5i/ab_k16.log
echo "[3] k32"; AB_OBJECTS=256 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/base/libvds_ec.so > gpurun_out/r5i/ab_k32.log 2>&1 || exit 1
cat gpurun_out/r5i/ab_k32.log
echo "[4] rt"
for r in 1 2 3; do
  for rows in 8 4; do
    timeout -k 10 120 python tools/rt2_bench.py --rows $rows >> gpurun_out/r5i/rt.log 2>&1 || exit 1
    VDS_EC_RT2=0 timeout -k 10 120 python tools/rt2_bench.py --rows $rows >> gpurun_out/r5i/rt.log 2>&1 || exit 1
    VDS_EC_LIB=ab/nort2/libvds_ec.so VDS_EC_RT2=0 timeout -k 10 120 python tools/rt2_bench.py --rows $rows | sed 's/^{/{"lib": "nort2", /' >> gpurun_out/r5i/rt.log 2>&1 || exit 1
  done
done
grep '^{' gpurun_out/r5i/rt.log
