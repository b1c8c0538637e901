# Round 5: k = 32 stage C with balanced cell pairs per wave (VDS_C32_BALANCE,
# default) against ab/prev; GPU suite first; ABBA at k = 32 (256 x 64 MiB)
# and the live shape twice.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5v; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
AB_OBJECTS=256 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so > $D/ab_k32.log 2>&1 || exit 1
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
