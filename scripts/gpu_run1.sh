set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_measured.py tests/test_gpu_digest.py tests/test_gpu_queue.py -k 'encode_only or config4 or constant or default_geometries_ws_get_heal or digest or lengths or mib or vectors or parts or queue' > gpurun_out/ua_enc_test.log 2>&1 || { tail -30 gpurun_out/ua_enc_test.log; exit 1; }
tail -2 gpurun_out/ua_enc_test.log
scripts/queue_ab.sh > gpurun_out/queue_ab.jsonl 2>&1 || { tail gpurun_out/queue_ab.jsonl; exit 2; }
PATHS=geom,encode,get,digest timeout -k 10 300 python -u scripts/bench_paths.py > gpurun_out/geom_ua_enc.jsonl 2>&1 || exit 3
SHAPE=4:2:2048 VARIANTS=0,270,271,272 CASES="1;0,3;h0,5;h0,1" timeout -k 10 200 python -u scripts/get_ab.py > gpurun_out/get_ab_k4.jsonl 2>&1 || exit 4
SHAPE=4:4:4096 VARIANTS=0,270,271,272 CASES="0,1;h1,4;h0,2,5;0,1,2,3;h1,4,6,7" timeout -k 10 200 python -u scripts/get_ab.py >> gpurun_out/get_ab_k4.jsonl 2>&1 || exit 5
timeout -k 10 200 python bench.py > gpurun_out/bench_302.json 2>&1 || exit 6
tail -1 gpurun_out/bench_302.json
