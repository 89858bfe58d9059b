#!/bin/bash
# HBM traffic per launch of the RS(12+4) 1 MiB encode + sums instances (VERDICT r04 item
# 3: <= 1.02 x algorithmic): separate FETCH_SIZE / WRITE_SIZE passes over
# scripts/sweep_variants.py at 4 096 objects, product (0) and the diagnostics VARIANTS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r05}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $P; export TMPDIR=/tmp
V=${VARIANTS:-0,408}
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/t124_$c
  SWEEP_SHAPES=12:4:4096 SWEEP_REPEAT=1 SWEEP_VARIANTS=$V timeout -k 10 300 rocprofv3 --pmc $c -d $OUT/t124_$c -o p --output-format csv -- \
      python scripts/sweep_variants.py > $OUT/t124_$c.log 2>&1 || { tail -5 $OUT/t124_$c.log; exit 2; }
done
python scripts/pmc_traffic.py $(find $OUT/t124_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
    $(find $OUT/t124_WRITE_SIZE -name '*counter_collection.csv' | head -1) $P/traffic_rs124.json > /dev/null || exit 3
python - <<'PY'
import json, os
d = json.load(open(f"gpurun_out/profile/{os.environ.get('ROUND', 'r05')}/traffic_rs124.json"))
k, m, blen, n = 12, 4, 1 << 20, 4096
S = -(-blen // k)
algo = n * (blen + m * S + 32 * (k + m))
for name, v in d.items():
    print(name, round(v["hbm_bytes_per_launch"] / algo, 4), v["launches"])
PY
