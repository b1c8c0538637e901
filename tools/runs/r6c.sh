# Round 6: same-box ABBA A/B of the batch planner (default build: concurrent
# plan claims, per-part indices) against ab/oldplan (round 5's serial plan
# and index passes) on the live legs, 2 rounds.  Argument: the variant under ab/ (default oldplan).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
OTHER=${1:-oldplan}
one() {  # one LIB TAG
  if [ "$1" = default ]; then
    timeout -k 10 300 python tools/live_prof.py --loss 0.02 0.25 > gpurun_out/r6c_$2.log 2>&1 || { tail -5 gpurun_out/r6c_$2.log; exit 1; }
  else
    VDS_EC_LIB=ab/$1/libvds_ec.so timeout -k 10 300 python tools/live_prof.py --loss 0.02 0.25 > gpurun_out/r6c_$2.log 2>&1 || { tail -5 gpurun_out/r6c_$2.log; exit 1; }
  fi
  python - gpurun_out/r6c_$2.log $1 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-2])
out = [sys.argv[2]]
for loss in ("0.02", "0.25"):
    leg = d[f"loss_{loss}"]
    for name in ("repair", "regenerate"):
        sp = leg["spread"][name]
        out.append(f"p{loss}_{name} {leg[name + '_GiBps']} host {sp['host_enqueue_ms_per_call']['median']} dev {sp['device_ms_per_call']['median']}")
print(" | ".join(out))
PY
}
for r in 1 2; do
  one default ${r}a; one $OTHER ${r}b; one $OTHER ${r}c; one default ${r}d
done
