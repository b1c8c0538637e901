# Round 5 diagnostic (no correctness): the AOT k = 16 kernel with its
# syndrome programs fed from registers instead of the LDS slots (ab/dsyn):
# the most a register-input syndrome could gain.  VDS_EC_JIT=0: AOT only.
cd $GRAFT_REPO_ROOT
export VDS_EC_JIT=0
AB_OBJECTS=512 bash tools/runs/ab_kernels.sh 4 ab/dsyn/libvds_ec.so > gpurun_out/r5u.log 2>&1
rc=$?; cat gpurun_out/r5u.log; exit $rc
