# Round 5: ABBA re-run of the k = 16 A/Bs (r5k, r5l ran a fixed order):
# default (fill from registers, staging in the survivor-set kernel's wave
# branches) vs ab/prev (1d858d6) vs ab/t16 (also the AOT k = 16 kernels'
# staging in the branches).
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5m; mkdir -p $D
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/prev/libvds_ec.so ab/t16/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
cat $D/ab_k16.log; python tools/runs/ab_summary.py $D/ab_k16.log
