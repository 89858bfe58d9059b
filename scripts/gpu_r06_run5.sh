#!/bin/bash
# Round 6: streamed GET / heal tests (quad kernel through pattern groups, pinned per-row
# path, failed blocks), the queue tests, and the --gpus 2 same-device bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_stream_decode.py tests/test_gpu_queue.py tests/test_gpu_configs.py > $OUT/run5_tests.log 2>&1 \
    || { tail -40 $OUT/run5_tests.log; exit 1; }
tail -3 $OUT/run5_tests.log
ZS3_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > $OUT/bench_gpus2_same_device.json 2>&1 \
    || { tail -20 $OUT/bench_gpus2_same_device.json; exit 2; }
tail -1 $OUT/bench_gpus2_same_device.json

# the survivor-quad heal with the survivor-stripe pad (product) vs without (445): time and
# LDS bank conflicts
O=$OUT/ab_quad_swz.jsonl
SHAPE=16:4:2048 VARIANTS=0,445 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 3
SHAPE=16:4:8192 VARIANTS=0,445 CASES="0,5,9,14;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 4
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['round'], d['objects'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'], d['path'], d['bad'])"
rm -rf $OUT/pmc_lds_quad
export TMPDIR=/tmp
SHAPE=16:4:2048 VARIANTS=0,445 CASES="h0,1,16,19" REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/pmc_lds_quad -o p --output-format csv -- python scripts/get_ab.py > $OUT/pmc_lds_quad.log 2>&1 || exit 5
python scripts/pmc_summary.py $(find $OUT/pmc_lds_quad -name '*counter_collection.csv' | head -1) | grep -i "quad" | cut -c1-250 | tee $OUT/pmc_lds_quad.txt
echo run5b done
