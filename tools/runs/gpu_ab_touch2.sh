# A/B of the k = 32 L2 touch (VDS_L2_TOUCH): parity first, then interleaved runs
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/abtouch2; mkdir -p $D
echo "[1] pytest (touch2)"; VDS_EC_LIB=ab/touch2.so timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_parity_gpu.py > $D/pytest_gpu.log 2>&1 || { tail -5 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
true &&
for r in 1 2; do
  for v in off touch2; do
    if [ $v = off ]; then L=""; else L=ab/touch2.so; fi
    echo "[3.$r] $v"
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --k 32 --m 8 --objects 256 --no-live --no-align16 --no-cpu-baseline --no-c4 --no-jit --steps 5 --warmup 2 > $D/k32_$v$r.json 2>$D/k32_$v$r.err || exit 1
    VDS_EC_LIB=$L timeout -k 10 300 python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > $D/live_$v$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json, glob
D = "gpurun_out/abtouch2"
for r in (1, 2):
    for v in ("off", "touch2"):
        b = json.loads(open(f'{D}/k32_{v}{r}.json').read().strip().splitlines()[-1])
        t = open(f'{D}/live_{v}{r}.log').read(); i = t.index('{"shape"'); d = json.loads(t[i:t.index('\n', i)])
        print(v, r, 'k32 repair_ms', b.get('repair_ms'), 'restore_aot_ms', b.get('restore_aot_ms'), 'enc', b.get('encode_ms'),
              '| live', {kk: (d[kk]['repair_GiBps'], d[kk]['regenerate_GiBps']) for kk in ('loss_0.02', 'loss_0.25')})
PY
