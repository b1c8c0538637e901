# Round 6: the batch planner with concurrent plan resolution and per-part
# indices -- batch / non-codeword / regenerate GPU tests, then host phases
# (ab/trace: -DVDS_HOST_TRACE=1) and the live legs with spreads.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_batch_gpu.py tests/test_noncodeword_gpu.py tests/test_regenerate_gpu.py > gpurun_out/r6b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6b_pytest.log; [ $rc -eq 0 ] || exit $rc
for loss in 0.02 0.25; do
  VDS_EC_LIB=ab/trace/libvds_ec.so timeout -k 10 300 python tools/host_trace.py --loss $loss > gpurun_out/r6b_trace_$loss.log 2>&1 || { tail -20 gpurun_out/r6b_trace_$loss.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6b_trace_$loss.log | tail -6
done
timeout -k 10 300 python tools/live_prof.py --loss 0.02 0.25 > gpurun_out/r6b_live.log 2>&1 || { tail -20 gpurun_out/r6b_live.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6b_live.log").read().strip().splitlines()[-2])
for loss in ("0.02", "0.25"):
    leg = d[f"loss_{loss}"]
    print(loss, "repair", leg["repair_GiBps"], "regen", leg["regenerate_GiBps"],
          {k: (v["stream_ms_per_call"]["median"], v["device_ms_per_call"]["median"], v["host_enqueue_ms_per_call"]["median"], v["bound"]) for k, v in leg["spread"].items()})
PY
