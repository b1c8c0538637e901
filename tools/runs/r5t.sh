# Round 5: two-level interpolation phase priorities retuned after the
# round's k = 16 changes: VDS_GM2_PRIO 9 (default: S1 + stage C) against 1
# (S1), 13 (S1 + S3 + C), 15 (all); ABBA, k = 16 at 512 x 64 MiB.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5t; mkdir -p $D
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/p1/libvds_ec.so ab/p13/libvds_ec.so ab/p15/libvds_ec.so > $D/ab_k16.log 2>&1 || exit 1
python tools/runs/ab_summary.py $D/ab_k16.log
