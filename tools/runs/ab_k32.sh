# Same-box interleaved A/B at k = 32, m = 8 (C4 shape, AB_OBJECTS x 64 MiB):
# encode, survivor-set (JIT) repair and AOT k_restore_syn<32,40> repair of the
# default library against variant builds (VDS_EC_LIB), AB_ROUNDS rounds.
#   bash tools/runs/ab_k32.sh ab/x/libvds_ec.so [...]
cd $GRAFT_REPO_ROOT
OBJ=${AB_OBJECTS:-256}
ROUNDS=${AB_ROUNDS:-3}
K=${AB_K:-32}
M=${AB_M:-8}
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', 'enc_ms',d['encode_ms'],'rep_ms',d['repair_ms'],'aot_ms',d.get('restore_aot_ms'),'value',d['value'])"; }
for r in $(seq 1 $ROUNDS); do
  timeout -k 10 300 python bench.py --k $K --m $M --objects $OBJ --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/abk_default_$r.log 2>&1 || exit $?
  summ gpurun_out/abk_default_$r.log default
  for v in "$@"; do
    n=$(basename $(dirname $v))
    VDS_EC_LIB=$v timeout -k 10 300 python bench.py --k $K --m $M --objects $OBJ --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/abk_${n}_$r.log 2>&1 || exit $?
    summ gpurun_out/abk_${n}_$r.log $n
  done
done
