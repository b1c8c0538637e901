cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/r4f; mkdir -p $D
echo "[1] pytest batch"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_jit_gpu.py tests/test_sha256_gpu.py > $D/pytest_gpu.log 2>&1 &&
echo "[2] host trace"; VDS_EC_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py --loss 0.02 > $D/ht02.log 2>&1 &&
echo "[3] live"; timeout -k 10 300 python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > $D/live_prof.log 2>&1
rc=$?; echo rc=$rc; tail -2 $D/pytest_gpu.log; grep "host ms" $D/ht02.log; grep "restore_batch" $D/ht02.log | tail -2; grep "regenerate_batch" $D/ht02.log | tail -2; python3 - <<'PY'
import json
t=open('gpurun_out/r4f/live_prof.log').read(); i=t.index('{"shape"'); d=json.loads(t[i:t.index('\n',i)])
for kk in ('loss_0.02','loss_0.25'): print(kk, {x:d[kk][x] for x in ('repair_GiBps','repair_host_GiBps','regenerate_GiBps')})
print(d['encode_GiBps'], d['save_temp'])
PY
exit $rc
