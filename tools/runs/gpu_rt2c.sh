cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/rt2c; mkdir -p $D
echo "[1] pytest"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_noncodeword_gpu.py tests/test_batch_gpu.py > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
for r in 8 10 12; do for v in 1 0; do VDS_EC_RT2=$v timeout -k 10 120 python tools/rt2_bench.py --rows $r >> $D/rt2b.log 2>&1 || { tail -5 $D/rt2b.log; exit 1; }; done; done
grep rt2 $D/rt2b.log
timeout -k 10 300 python tools/live_prof.py --objects 16384 --loss 0.25 --steps 10 > $D/live.log 2>&1 || exit 1
python3 - <<'PY'
import json
t = open('gpurun_out/rt2c/live.log').read(); i = t.index('{"shape"'); d = json.loads(t[i:t.index('\n', i)])
print({kk: (d[kk]['repair_GiBps'], d[kk]['regenerate_GiBps']) for kk in ('loss_0.25',)})
PY
