# Round 5: XOR programs from the 3-input greedy (xorprog.hpp paar3, per block
# the better of it and Paar; every generated .inc regenerated, and the
# run-time fills) -- default -- against ab/prev; GPU suite first; ABBA at
# k = 16 (512) and k = 32 (256); the live shape twice each.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5r; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
python tools/runs/ab_summary.py $D/ab_k16.log
AB_OBJECTS=256 AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k32.log 2>&1 || exit 1
python tools/runs/ab_summary.py $D/ab_k32.log
live() { python - "$1" "$2" <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"shape"')][-1]
print(sys.argv[2], 'enc', d['encode_GiBps'], {k: (d[k]['repair_GiBps'], d[k]['regenerate_GiBps']) for k in d if k.startswith('loss_')})
PY
}
for r in 1 2; do
  for v in default prev; do
    if [ $v = prev ]; then export VDS_EC_LIB=ab/prev/libvds_ec.so; else unset VDS_EC_LIB; fi
    timeout -k 10 300 python tools/live_prof.py --loss 0.25 0.02 --steps 10 > $D/live_${v}_$r.log 2>&1 || exit 1
    live $D/live_${v}_$r.log $v | tee -a $D/live.txt || exit 1
  done
done
unset VDS_EC_LIB
