# Round 6: own-group fill variants (Paar blocks of 2, no block prefetch)
# against the scatter fill (ab/own0) and the default (blocks of 3), k = 16,
# m = 4, 512 x 64 MiB, ABBA, 2 rounds.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=2 bash tools/runs/ab_k32.sh ab/own0/libvds_ec.so ab/ownpb2/libvds_ec.so ab/ownnopf/libvds_ec.so > gpurun_out/r6f_ab.log 2>&1 || { cat gpurun_out/r6f_ab.log; exit 1; }
python tools/runs/ab_summary.py gpurun_out/r6f_ab.log
