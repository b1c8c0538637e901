# Round 5: sub-byte transpose rounds on rotated words (bitslice.hpp: one
# rotate + two selects per pair, then one rotate back per word) -- default --
# against ab/prev; GPU suite first; ABBA at k = 16 (512) and k = 32 (256).
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5q; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
python tools/runs/ab_summary.py $D/ab_k16.log
AB_OBJECTS=256 AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k32.log 2>&1 || exit 1
python tools/runs/ab_summary.py $D/ab_k32.log
