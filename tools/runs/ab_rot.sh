# encode: which wave evaluates which replica pairs (build/rotN: VDS_ENC_WAVE_ROT=N)
# vs the default, same box; k = 16 (two workgroups per CU) and k = 32
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120 python tools/time_kernels.py --align 256 --check"
for i in 1 2; do
  $T --objects 512 --tag rot0_16 &&
  VDS_EC_LIB=build/rot1 $T --objects 512 --tag rot1_16 &&
  VDS_EC_LIB=build/rot2 $T --objects 512 --tag rot2_16 &&
  VDS_EC_LIB=build/rot3 $T --objects 512 --tag rot3_16 &&
  $T --k 32 --objects 256 --tag rot0_40 &&
  VDS_EC_LIB=build/rot2 $T --k 32 --objects 256 --tag rot2_40 || exit 1
done
