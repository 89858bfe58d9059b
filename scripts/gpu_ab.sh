#!/bin/bash
# Generic GPU A/B step (one gpurun call): optional parity tests, a variant sweep and
# per-wave stamps, every GPU step under its own time limit, stopping at the first failure.
#   TESTS="tests/test_gpu_variants.py -k '300 or 301'"   pytest selection (empty: skip)
#   SWEEP_SHAPES=8:4:16384 SWEEP_VARIANTS=0,300 SWEEP_REPEAT=2 SWEEP_OUT=name   (empty: skip)
#   STAMP_VARIANTS=306 NOBJ=16384                          (empty: skip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
    echo "tests $(date +%T)"
    eval timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/ab_tests.log 2>&1
    rc=$?; tail -3 $OUT/ab_tests.log
    [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/ab_tests.log | head -20; exit $rc; }
fi
if [ -n "${SWEEP_VARIANTS:-}" ]; then
    echo "sweep $(date +%T)"
    timeout -k 10 600 python -u scripts/sweep_variants.py > $OUT/${SWEEP_OUT:-ab_sweep}.jsonl 2> $OUT/ab_sweep.err
    rc=$?; cat $OUT/${SWEEP_OUT:-ab_sweep}.jsonl
    [ $rc -eq 0 ] || { tail -20 $OUT/ab_sweep.err; exit $rc; }
fi
if [ -n "${STAMP_VARIANTS:-}" ]; then
    echo "stamps $(date +%T)"
    VARIANTS=$STAMP_VARIANTS timeout -k 10 300 python -u scripts/stamps3.py > $OUT/${STAMP_OUT:-ab_stamps}.txt 2>&1
    rc=$?; cat $OUT/${STAMP_OUT:-ab_stamps}.txt
    [ $rc -eq 0 ] || exit $rc
fi
echo "done $(date +%T)"
