#!/bin/bash
# Per-launch HBM traffic of the headline kernel for every per-GPU share of BASELINE
# config 4 (65 536 objects over N = 1 / 2 / 4 / 8: 65 536 / 32 768 / 16 384 / 8 192
# objects per launch): separate FETCH_SIZE and WRITE_SIZE rocprofv3 passes per share
# (MI355X_MICROARCH.md: FETCH_SIZE doubled for wide streaming reads), merged into
# gpurun_out/profile/$ROUND/pmc_traffic.json keyed by the full kernel name, which
# bench.py's committed_traffic matches against HEADLINE_KERNEL.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r05}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $P; export TMPDIR=/tmp
rm -f $P/pmc_traffic.json
for n in ${SHARES:-65536 32768 16384 8192}; do
  rm -rf $OUT/pmcf_$n $OUT/pmcw_$n
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$n -o p --output-format csv -- \
      python bench.py --objects $n --steps 3 --warmup 1 --no-cpu > $OUT/pmcf_$n.log 2>&1 || { tail -5 $OUT/pmcf_$n.log; exit 2; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$n -o p --output-format csv -- \
      python bench.py --objects $n --steps 3 --warmup 1 --no-cpu > $OUT/pmcw_$n.log 2>&1 || { tail -5 $OUT/pmcw_$n.log; exit 3; }
  python scripts/pmc_traffic.py $(find $OUT/pmcf_$n -name '*counter_collection.csv' | head -1) \
      $(find $OUT/pmcw_$n -name '*counter_collection.csv' | head -1) $P/pmc_traffic.json $n > /dev/null || exit 4
done
ROUND=$ROUND python - <<'PY'
import json, os, sys
sys.path.insert(0, ".")
import bench
d = json.load(open(f"gpurun_out/profile/{os.environ['ROUND']}/pmc_traffic.json"))
want = bench.HEADLINE_KERNEL[(8, 4, 1 << 20)]
for key, v in d.items():
    name, n = key.split(" @ ")
    algo = int(n.split()[0]) * bench.algo_bytes_per_block(8, 4, 1 << 20)
    print(("OK  " if name == want else "NAME MISMATCH ") + key, round(v["hbm_bytes_per_launch"] / algo, 4))
PY
