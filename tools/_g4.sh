cd $GRAFT_REPO_ROOT
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'value',d['value'],'enc',d['encode_GiBps'],'rep',d['repair_GiBps'],'regen',d['regenerate_GiBps'],'enc_ms',d['encode_ms'],'rep_ms',d['repair_ms'])"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/pt4.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pt4.log
timeout -k 10 200 python bench.py --objects 512 --no-cpu-baseline > gpurun_out/b4_g2.log 2>&1 || exit 1
VDS_EC_SYN_G=1 timeout -k 10 200 python bench.py --objects 512 --no-cpu-baseline > gpurun_out/b4_g1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --objects 512 --no-cpu-baseline > gpurun_out/b4_g2b.log 2>&1 || exit 1
summ gpurun_out/b4_g2.log; summ gpurun_out/b4_g1.log; summ gpurun_out/b4_g2b.log
