# Round 5 diagnostic (no correctness: tools/time_kernels.py): where the k = 16
# survivor-set kernel's scatter fill spends its time.  ab/df1: plain LDS
# writes instead of the ds_xor_b64 atomics; ab/df2: no fill XORs (atomics
# kept); ab/df3: neither.  Default library first, 4 rounds.
cd $GRAFT_REPO_ROOT
AB_OBJECTS=512 bash tools/runs/ab_kernels.sh 4 ab/df1/libvds_ec.so ab/df2/libvds_ec.so ab/df3/libvds_ec.so > gpurun_out/r5o.log 2>&1
rc=$?; cat gpurun_out/r5o.log; exit $rc
