set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
bash scripts/profile.sh r01 > gpurun_out/profile_r01.log 2>&1 || exit $?
echo done
