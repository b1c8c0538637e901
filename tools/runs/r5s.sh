# Round 5 study: replica-buffer skew vs the per-process encode rate
# (tools/ubench/skew.py), four processes.
cd $GRAFT_REPO_ROOT
for i in 1 2 3 4; do timeout -k 10 300 python tools/ubench/skew.py --objects 512 >> gpurun_out/r5s.log 2>&1 || exit 1; done
grep '^{' gpurun_out/r5s.log
