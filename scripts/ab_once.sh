set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS=0,200,210,216,240 SHAPES=8,16 timeout -k 10 400 python -u scripts/get_ab2.py > gpurun_out/get_ab_waves.jsonl || exit 4
bash scripts/gpu_tests.sh
