# quick parity subset + 256-object bench (A/B of the restore paths); prints value/encode/repair
cd $GRAFT_REPO_ROOT
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'value',d['value'],'enc',d['encode_GiBps'],'rep',d['repair_GiBps'],'enc_ms',d['encode_ms'],'rep_ms',d['repair_ms'])"; }
timeout -k 10 300 python -m pytest -q -m gpu tests/test_parity_gpu.py -k "${QP_TESTS:-fast or golden or full or batched or syndrome or path}" > gpurun_out/pt.log 2>&1 &&
timeout -k 10 300 python bench.py --objects 256 --no-cpu-baseline > gpurun_out/bench_256.log 2>&1 &&
VDS_EC_RESTORE_PATH=bs timeout -k 10 300 python bench.py --objects 256 --no-cpu-baseline > gpurun_out/bench_256_bs.log 2>&1
rc=$?
echo rc=$rc
tail -1 gpurun_out/pt.log
summ gpurun_out/bench_256.log
summ gpurun_out/bench_256_bs.log
exit $rc
