# Round 5: the AOT k = 16 kernels with the staging in each wave's branch
# (ab/t16) against the default (join before the staging), same box.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5l; mkdir -p $D
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/t16/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
cat $D/ab_k16.log
