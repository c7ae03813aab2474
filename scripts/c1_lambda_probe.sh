#!/bin/bash
# C1 (data/hepatitis.clean.csv) with the reference's default -p (n - 1) at
# several lambdas (score_main.cpp:214: the default lambda is 0.5; README.md:28-30
# uses 2): bin/score end to end, one bounded run per lambda.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lam in ${LAMS:-2 1 0.5}; do
  echo "lambda $lam" >> gpurun_out/c1_lambda.log
  timeout -k 10 ${T:-150} urlearning-cpp_amd/bin/score tests/golden/hepatitis.clean.csv /tmp/c1_$lam.pss -f cBIC --lambda $lam >> gpurun_out/c1_lambda.log 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/c1_lambda.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  ls -la /tmp/c1_$lam.pss >> gpurun_out/c1_lambda.log
done
