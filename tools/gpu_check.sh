#!/bin/bash
# GPU check: first the given test files (all failures reported), then the whole -m gpu suite.
# Stops at once on anything other than pass / test failure (fault, abort, timeout).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -v --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/new_tests.log 2>&1
rc=$?
tail -40 gpurun_out/new_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/all_gpu.log 2>&1
rc2=$?
tail -15 gpurun_out/all_gpu.log
exit $(( rc > rc2 ? rc : rc2 ))
