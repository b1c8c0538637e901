# Round 6: own-group fill for the k = 16 survivor-set kernel -- full GPU
# suite, then a same-box ABBA A/B against ab/own0 (-DVDS_JIT_OWN=0: the
# scatter fill) at k = 16, m = 4, 512 x 64 MiB, 3 rounds.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/ > gpurun_out/r6e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6e_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh ab/own0/libvds_ec.so > gpurun_out/r6e_ab.log 2>&1 || { cat gpurun_out/r6e_ab.log; exit 1; }
python tools/runs/ab_summary.py gpurun_out/r6e_ab.log
