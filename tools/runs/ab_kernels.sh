# Interleaved A/B of kernel timings (no correctness checks: diagnostic builds
# allowed): bash tools/runs/ab_kernels.sh ROUNDS variant.so ...   (default lib first)
cd $GRAFT_REPO_ROOT
R=$1; shift
for i in $(seq $R); do
  timeout -k 10 120 python tools/time_kernels.py --objects ${AB_OBJECTS:-128} --tag default || exit $?
  for v in "$@"; do
    VDS_EC_LIB=$v timeout -k 10 120 python tools/time_kernels.py --objects ${AB_OBJECTS:-128} --tag $(basename $v .so) || exit $?
  done
done
