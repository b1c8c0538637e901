# Round 6: batch planner with claims in the first pass -- batch / non-codeword
# / regenerate GPU tests, host phases (ab/trace), then ABBA against ab/oldplan.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_regenerate_gpu.py > gpurun_out/r6d_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6d_pytest.log; [ $rc -eq 0 ] || exit $rc
for loss in 0.02 0.25; do
  VDS_EC_LIB=ab/trace/libvds_ec.so timeout -k 10 300 python tools/host_trace.py --loss $loss > gpurun_out/r6d_trace_$loss.log 2>&1 || { tail -20 gpurun_out/r6d_trace_$loss.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6d_trace_$loss.log | grep 'host ms\|total=' | tail -4
done
sed -i 's/^for r in 1; do$/for r in 1 2; do/' tools/runs/r6c.sh
bash tools/runs/r6c.sh
