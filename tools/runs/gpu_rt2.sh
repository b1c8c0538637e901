# RT2 rows: parity (batch, non-codeword incl. the RT2 test), then live p = 0.25 with RT2 on / off (VDS_EC_RT2=0), interleaved
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/rt2; mkdir -p $D
echo "[1] pytest"; timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_noncodeword_gpu.py tests/test_batch_gpu.py > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
for r in 1 2; do
  for v in on off; do
    if [ $v = on ]; then E=1; else E=0; fi
    echo "[2.$r] $v"
    VDS_EC_RT2=$E timeout -k 10 300 python tools/live_prof.py --objects 16384 --loss 0.25 0.02 --steps 10 > $D/live_$v$r.log 2>&1 || { tail -5 $D/live_$v$r.log; exit 1; }
  done
done
echo "[3] trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python tools/live_prof.py --objects 16384 --loss 0.25 --steps 5 > $D/trace.log 2>&1 || exit 1
python3 - <<'PY'
import json
D = "gpurun_out/rt2"
for r in (1, 2):
    for v in ("on", "off"):
        t = open(f'{D}/live_{v}{r}.log').read(); i = t.index('{"shape"'); d = json.loads(t[i:t.index('\n', i)])
        print(v, r, {kk: (d[kk]['repair_GiBps'], d[kk]['regenerate_GiBps']) for kk in ('loss_0.25', 'loss_0.02')})
PY
grep -i "restore_syn\|rt_coefs" $D/trace/run_kernel_stats.csv | cut -c1-160
