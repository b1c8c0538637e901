# A/B the default library against variant builds: bash tools/runs/ab_bench.sh [variant.so ...]
# (variants built with vds_amd.build.build(out=..., defines=(...)) and loaded via VDS_EC_LIB)
cd $GRAFT_REPO_ROOT
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', 'value',d['value'],'enc',d['encode_GiBps'],'rep',d['repair_GiBps'],'enc_ms',d['encode_ms'],'rep_ms',d['repair_ms'])"; }
OBJ=${AB_OBJECTS:-256}
timeout -k 10 300 python bench.py --objects $OBJ --no-cpu-baseline > gpurun_out/ab_default.log 2>&1 || exit $?
summ gpurun_out/ab_default.log default
for v in "$@"; do
  n=$(basename $v .so)
  VDS_EC_LIB=$v timeout -k 10 300 python bench.py --objects $OBJ --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1 || exit $?
  summ gpurun_out/ab_$n.log $n
done
