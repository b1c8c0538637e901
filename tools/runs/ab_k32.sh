# Same-box interleaved A/B at k = 32, m = 8 (C4 shape, AB_OBJECTS x 64 MiB):
# encode, survivor-set (JIT) repair and AOT k_restore_syn<32,40> repair of the
# default library against variant builds (VDS_EC_LIB), AB_ROUNDS rounds.
# AB_K / AB_M select another shape.  Each round runs the libraries in order
# and then in reverse (ABBA): a process's own speed varies by a few percent
# (the same kernel measured 13.1 and 14.9 ms in consecutive processes), and a
# fixed order put that on whichever library ran in the faster slot.
#   bash tools/runs/ab_k32.sh ab/x/libvds_ec.so [...]
# A variant "env:NAME=VALUE" runs the default library with that variable set
# (label NAME_VALUE).
cd $GRAFT_REPO_ROOT
OBJ=${AB_OBJECTS:-256}
ROUNDS=${AB_ROUNDS:-3}
K=${AB_K:-32}
M=${AB_M:-8}
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', 'enc_ms',d['encode_ms'],'rep_ms',d['repair_ms'],'aot_ms',d.get('restore_aot_ms'),'value',d['value'])"; }
one() {  # one() LIB NAME TAG
  if [ "${1#env:}" != "$1" ]; then
    env "${1#env:}" timeout -k 10 300 python bench.py --k $K --m $M --objects $OBJ --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/abk_$2_$3.log 2>&1 || exit $?
  elif [ "$1" = default ]; then
    timeout -k 10 300 python bench.py --k $K --m $M --objects $OBJ --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/abk_$2_$3.log 2>&1 || exit $?
  else
    VDS_EC_LIB=$1 timeout -k 10 300 python bench.py --k $K --m $M --objects $OBJ --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/abk_$2_$3.log 2>&1 || exit $?
  fi
  summ gpurun_out/abk_$2_$3.log $2
}
label() {
  if [ "${1#env:}" != "$1" ]; then x=${1#env:}; echo "${x%%=*}_${x#*=}"
  elif [ "$1" = default ]; then echo default
  else basename $(dirname $1); fi
}
libs=(default "$@")
for r in $(seq 1 $ROUNDS); do
  for v in "${libs[@]}"; do
    one "$v" $(label "$v") ${r}a
  done
  for ((i=${#libs[@]}-1; i>=0; i--)); do
    v=${libs[$i]}
    one "$v" $(label "$v") ${r}b
  done
done
