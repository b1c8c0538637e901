# Round 5: checkpoint (GPU suite, default bench, latency) then the encode
# pair-plan A/B (ab/nols: LPT only, VDS_ENC_PLAN_LS=0) at k = 16 (512 objects)
# and k = 32 (256 objects), interleaved.
cd $GRAFT_REPO_ROOT
bash tools/runs/r5_check.sh r5chk1 || exit $?
for r in 1 2 3; do
  for v in default nols; do
    L=""; [ $v = nols ] && L=ab/nols/libvds_ec.so
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --objects 512 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/enc16_${v}_$r.log 2>&1 || exit $?
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --k 32 --m 8 --objects 256 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/enc32_${v}_$r.log 2>&1 || exit $?
    python - gpurun_out/enc16_${v}_$r.log gpurun_out/enc32_${v}_$r.log $v <<'PY'
import json, sys
a = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "k16 enc_ms", a["encode_ms"], "rep_ms", a["repair_ms"], "| k32 enc_ms", b["encode_ms"], "rep_ms", b["repair_ms"])
PY
  done
done
