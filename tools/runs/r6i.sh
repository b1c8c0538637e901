# Round 6: the batch planner over 16 parts / 15 pool workers -- batch GPU
# tests, host phases (ab/trace), then ABBA of the live legs against
# ab/parts8 (8 parts, 7 workers).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_regenerate_gpu.py > gpurun_out/r6i_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6i_pytest.log; [ $rc -eq 0 ] || exit $rc
for loss in 0.02 0.25; do
  VDS_EC_LIB=ab/trace/libvds_ec.so timeout -k 10 300 python tools/host_trace.py --loss $loss > gpurun_out/r6i_trace_$loss.log 2>&1 || { tail -20 gpurun_out/r6i_trace_$loss.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6i_trace_$loss.log | grep 'host ms\|total=' | tail -3
done
nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
bash tools/runs/r6c.sh parts8
