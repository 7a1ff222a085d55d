# Bench lines + rocprofv3 kernel stats for the non-default BASELINE configs (c3 dense, c5 NUTS,
# c4 D=1000 streaming).  Usage: bash scripts/gpu_configs.sh TAG
set -u
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out/cfg_$TAG
export TMPDIR=/tmp
run() {   # name, bench args
  local n=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg_$TAG/$n.json.log 2>&1 || return $?
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/cfg_$TAG/$n" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-ess "$@" > "$R/gpurun_out/cfg_$TAG/$n.prof.log" 2>&1) || return $?
}
run c3_dense --rho 0.95 --chains 262144 --steps 10 --warmup 2 || exit $?
run c5_nuts --sampler nuts --rho 0.95 --chains 65536 --iters-per-step 2 --steps 5 --warmup 1 || exit $?
run c4_d1000 --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 || exit $?
echo done
