cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/${1:-r4c}; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/live -o run -- python tools/live_prof.py --objects 16384 --loss 0.02 --steps 10 > $D/live_prof.log 2>&1
rc=$?; echo rc=$rc; tail -c 1500 $D/live_prof.log; f=$(find $D/live -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -30; exit $rc
