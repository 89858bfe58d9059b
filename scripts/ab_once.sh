set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit 3
SIZES=1,64,256,512,640,641,1000,1024,1025,1100,1536,2047,2048,2049,2304,2305,3001,4096,8192,16384 VARIANTS=0 ROUNDS=2 REPS=7 timeout -k 10 300 python -u scripts/sweep_sizes.py > gpurun_out/sweep_sizes_final_rs84.jsonl || exit 19
K=16 M=4 SIZES=1,64,256,384,448,511,512,1024,1025,2047,2048,4096,8192 VARIANTS=0 ROUNDS=2 REPS=7 timeout -k 10 300 python -u scripts/sweep_sizes.py > gpurun_out/sweep_sizes_final_rs164.jsonl || exit 20
