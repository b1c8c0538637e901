cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; : > gpurun_out/bisect_tests.txt
for t in $(python -m pytest tests -m gpu --collect-only -q 2>/dev/null | grep '::'); do
  timeout -k 5 120 python -m pytest -q "$t" > /dev/null 2>&1
  echo "$? $t" >> gpurun_out/bisect_tests.txt
done
cat gpurun_out/bisect_tests.txt
