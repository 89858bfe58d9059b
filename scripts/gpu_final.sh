#!/bin/bash
# Round-end check on one box: the full GPU suite, smoke(), the bench, then the round
# profile of the headline (rocprof trace / stats + PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/final_tests.log 2>&1 \
    || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 \
    || { tail -20 gpurun_out/final_smoke.log; exit 2; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2>&1 || { tail gpurun_out/final_bench.json; exit 3; }
tail -1 gpurun_out/final_bench.json
