#!/bin/bash
# Round 6: where RS(12+4)'s extra reads come from.  Same kernel instance (Rs124Ua1K,
# rows 2 bytes past a 16-byte boundary), 4 096 stripes, three shard sizes: S = 87 382
# (1 MiB blocks, a 342-byte ragged tail tile read byte by byte), 88 066 (tail 2 bytes) and
# 88 062 (tail 1 022 bytes, rows 14 bytes past).  HBM reads / writes by request size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
for S in 87382 88066 88062; do
  BL=$((12 * S)); [ $S = 87382 ] && BL=1048576
  ROUND=r06 TAG=rs124_S$S CMD="python scripts/sweep_variants.py" SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=0 SWEEP_REPEAT=1 \
      SWEEP_STEPS=3 SWEEP_BLEN=$BL bash scripts/traffic_req.sh > $OUT/tq_S$S.log 2>&1 || { tail -5 $OUT/tq_S$S.log; exit 1; }
  grep '"kernel"' gpurun_out/profile/r06/traffic_req_rs124_S$S.json > /dev/null 2>&1; python -c "
import json; d=json.load(open('gpurun_out/profile/r06/traffic_req_rs124_S$S.json')); print('S=$S', d)" | cut -c1-300
done
echo run29 done
