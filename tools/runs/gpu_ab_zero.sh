# A/B: the survivor-set kernels' per-tile zero vector (no scratch spill) vs the hoisted one
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/abzero; mkdir -p $D
for r in 1 2 3; do
  for v in zero nozero; do
    if [ $v = zero ]; then L=""; else L=ab/nozero.so; fi
    echo "[$r] $v"
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --objects 512 --no-live --no-align16 --no-cpu-baseline --no-c4 --steps 10 --warmup 3 > $D/b_$v$r.json 2>$D/b_$v$r.err || exit 1
  done
done
python3 - <<'PY'
import json
D = 'gpurun_out/abzero'
for r in (1, 2, 3):
    for v in ('zero', 'nozero'):
        b = json.loads(open(f'{D}/b_{v}{r}.json').read().strip().splitlines()[-1])
        print(v, r, 'repair_ms', b['repair_ms'], 'encode_ms', b['encode_ms'], 'value', b['value'], 'kernel', b['roofline'].get('kernel'), 'restore_aot_ms', b.get('restore_aot_ms'))
PY
