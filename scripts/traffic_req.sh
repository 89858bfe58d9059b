#!/bin/bash
# HBM traffic per launch from the L2's memory-side request counters by request size,
# without the FETCH_SIZE correction: reads = 32 * RDREQ_32B + 64 * RDREQ_64B + 128 *
# RDREQ_128B (and the remainder of RDREQ at 64), writes = 32 * (WRREQ - WRREQ_64B) + 64 *
# WRREQ_64B.  (gfx950's FETCH_SIZE expression weighs 128-byte requests through TCC_BUBBLE
# and counts the others at 64 bytes: half of a 16-byte-per-lane streaming read, but not
# of partial-line or dword requests, so the x2 correction does not hold for unaligned
# rows or the L2 prefetch.)  Two passes (reads, writes) per workload, counters only.
#   TAG=rs124 CMD="python scripts/sweep_variants.py" SWEEP_SHAPES=12:4:4096 ... bash scripts/traffic_req.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r05}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $P; export TMPDIR=/tmp
TAG=${TAG:-run}
rm -rf $OUT/tq_${TAG}_r $OUT/tq_${TAG}_w
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d $OUT/tq_${TAG}_r -o p --output-format csv -- $CMD > $OUT/tq_${TAG}_r.log 2>&1 || { tail -5 $OUT/tq_${TAG}_r.log; exit 2; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $OUT/tq_${TAG}_w -o p --output-format csv -- $CMD > $OUT/tq_${TAG}_w.log 2>&1 || { tail -5 $OUT/tq_${TAG}_w.log; exit 3; }
python scripts/traffic_req.py $(find $OUT/tq_${TAG}_r -name '*counter_collection.csv' | head -1) \
    $(find $OUT/tq_${TAG}_w -name '*counter_collection.csv' | head -1) $P/traffic_req_${TAG}.json
