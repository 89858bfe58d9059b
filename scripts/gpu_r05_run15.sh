#!/bin/bash
# Round 5 run 15: the survivor-quad kernel with survivors and rebuilt rows in one LDS row
# array (product) vs two arrays (444); parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py -k "rs164 or large_batch" > gpurun_out/r05_t15.log 2>&1 || { tail -30 gpurun_out/r05_t15.log; exit 1; }
tail -1 gpurun_out/r05_t15.log
O=gpurun_out/r05_ab_quad4.jsonl
SHAPE=16:4:2048 VARIANTS=0,444 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 2
SHAPE=16:4:8192 VARIANTS=0,444 CASES="0,5,9,14;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['round'], d['objects'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'], d['path'], d['bad'])"
rm -rf gpurun_out/pmc_lds_quad
SHAPE=16:4:2048 VARIANTS=0,444 CASES="h0,1,16,19" REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_lds_quad -o p --output-format csv -- python scripts/get_ab.py > gpurun_out/r05_pmc_lds_quad.log 2>&1 || exit 4
python scripts/pmc_summary.py $(find gpurun_out/pmc_lds_quad -name '*counter_collection.csv' | head -1) | grep -i "quad" | cut -c1-250
echo run15 done
