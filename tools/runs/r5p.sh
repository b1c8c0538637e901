# Round 5: scatter-fill Paar block size (VDS_EC_JIT_SPB, survivors per block;
# default 2) now that the k = 16 fill reads registers: 3 and 4 against 2,
# ABBA, k = 16 at 512 x 64 MiB.  Before it, the r5o diagnostic's split of
# the fill (tools/runs/r5o.sh) is in profiles/round5/diag_fill.log.
cd $GRAFT_REPO_ROOT
set -o pipefail
D=gpurun_out/r5p; mkdir -p $D
AB_K=16 AB_M=4 AB_OBJECTS=512 AB_ROUNDS=3 bash tools/runs/ab_k32.sh env:VDS_EC_JIT_SPB=3 env:VDS_EC_JIT_SPB=4 > $D/ab_k16.log 2>&1 || exit 1
cat $D/ab_k16.log; python tools/runs/ab_summary.py $D/ab_k16.log
