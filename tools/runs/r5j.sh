# Round 5: RT kernels with the staging and copy-out in each wave's branch
# (default; the k = 32 RT kernel's 176-VGPR spill down to 24) against the
# previous build (ab/prev): rt2_bench at 8 and 4 rows and the live shape at
# p = 0.25 / 0.02, three interleaved rounds; the GPU suite first.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5j; mkdir -p $D
echo "[1] pytest"; timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
live() { python - "$1" "$2" <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"shape"')][-1]
print(sys.argv[2], {k: (d[k]['repair_GiBps'], d[k]['regenerate_GiBps']) for k in d if k.startswith('loss_')})
PY
}
for r in 1 2 3; do
  for v in default prev; do
    if [ $v = prev ]; then export VDS_EC_LIB=ab/prev/libvds_ec.so; else unset VDS_EC_LIB; fi
    for rows in 8 4; do
      timeout -k 10 120 python tools/rt2_bench.py --rows $rows | sed "s/^{/{\"lib\": \"$v\", /" >> $D/rt.log || exit 1
    done
    timeout -k 10 300 python tools/live_prof.py --loss 0.25 0.02 --steps 10 > $D/live_${v}_$r.log 2>&1 || exit 1
    live $D/live_${v}_$r.log $v >> $D/live.txt || exit 1
  done
done
unset VDS_EC_LIB
cat $D/rt.log $D/live.txt
