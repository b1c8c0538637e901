# Round 5: plane-split S2 at k = 32 (gen_restore.cpp emit_gm2).  GPU suite,
# then same-box A/B against the previous commit's build (ab/head):
# C4 at 256 x 64 MiB (encode, survivor-set and AOT repair) and the live shape
# (16,384 x 64 KiB; p = 0.02 and 0.25 repair / regenerate), three rounds.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/ > gpurun_out/r5h_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5h_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in default head; do
    L=""; [ $v != default ] && L=ab/$v/libvds_ec.so
    VDS_EC_LIB=$L timeout -k 10 300 python bench.py --k 32 --m 8 --objects 256 --steps 10 --warmup 3 --no-cpu-baseline --no-live --no-c4 --no-align16 > gpurun_out/h32_${v}_$r.log 2>&1 || exit $?
    VDS_EC_LIB=$L timeout -k 10 300 python tools/live_prof.py --objects 16384 --loss 0.02 0.25 --steps 10 > gpurun_out/hlive_${v}_$r.log 2>&1 || exit $?
    python - gpurun_out/h32_${v}_$r.log gpurun_out/hlive_${v}_$r.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = None
for line in open(sys.argv[2]):
    if line.startswith("{"):
        l = json.loads(line); break
print(sys.argv[3], "C4 enc", d["encode_ms"], "rep", d["repair_ms"], "aot", d["restore_aot_ms"],
      "| live p.02 rep", l["loss_0.02"]["repair_GiBps"], "regen", l["loss_0.02"]["regenerate_GiBps"],
      "p.25 rep", l["loss_0.25"]["repair_GiBps"], "regen", l["loss_0.25"]["regenerate_GiBps"])
PY
  done
done
