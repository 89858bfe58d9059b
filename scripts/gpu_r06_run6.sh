#!/bin/bash
# Round 6: queue host-side phase timers (tools/queue_bench_diag), the survivor-quad heal
# layout A/B (0 = padded survivor stripes, 445 = round-5 layout, 440 = k_vr_ws), the
# HighwayHash chain latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/queue_timers.jsonl
for pinned in 0 1; do
  timeout -k 10 200 tools/queue_bench_diag 1,16,64,256 48 8 4 0 0 $pinned >> $OUT/queue_timers.jsonl || exit 1
done
cat $OUT/queue_timers.jsonl
O=$OUT/ab_quad_swz2.jsonl
SHAPE=16:4:2048 VARIANTS=0,445,440 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 2
SHAPE=16:4:8192 VARIANTS=0,445,440 CASES="0,5,9,14;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['round'], d['objects'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'], d['path'], d['bad'])"
VARIANTS=0 timeout -k 10 200 python scripts/chain_lat.py > $OUT/chain_lat.jsonl 2>&1 || exit 4
cat $OUT/chain_lat.jsonl

# fused HighwayHash packet runs (hh_update_n / hh2_update_n): parity on the paths that use
# them, then A/B against the round-5 form (480 config 2, 481 RS(12+4) 1 KiB UA, 482
# RS(8+4) mid batches: without; 483: the headline with the pair-form runs)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_measured.py \
    tests/test_gpu_parity.py tests/test_gpu_bitrot.py tests/test_gpu_variants.py > $OUT/run6_tests.log 2>&1 || { tail -30 $OUT/run6_tests.log; exit 5; }
tail -2 $OUT/run6_tests.log
SWEEP_SHAPES=4:2:1024,12:4:4096,8:4:1024 SWEEP_VARIANTS=0,480,481,482 SWEEP_REPEAT=3 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_hf.jsonl 2>&1 || { tail -20 $OUT/ab_hf.jsonl; exit 6; }
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,483 SWEEP_REPEAT=3 timeout -k 10 300 python -u scripts/sweep_variants.py \
    >> $OUT/ab_hf.jsonl 2>&1 || { tail -20 $OUT/ab_hf.jsonl; exit 7; }
grep '^{' $OUT/ab_hf.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['m'], d['objects'], d['variant'], d['ms'], d['match'], d['path'])"
echo run6b done
