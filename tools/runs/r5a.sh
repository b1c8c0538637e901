# Round 5, first GPU pass: the GPU suite at HEAD, then the k = 32 half-priority
# A/B (ab/hp: VDS_HALF_PRIO=1) at 256 x 64 MiB, three interleaved rounds.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -m gpu -x --timeout 200 --timeout-method thread tests/ > gpurun_out/r5a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5a_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/ab_k32.sh ab/hp/libvds_ec.so
