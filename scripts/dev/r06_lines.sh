# Round-6 bench lines (one box, each step under its own limit, stops at the first failure).
set -e
B="bash scripts/gpu.sh bench"
$B r06_headline
$B r06_c3_dense --config c3 --no-cpu-baseline --steps 10 --warmup 2
$B r06_c5_nuts --config c5 --no-cpu-baseline --steps 5 --warmup 1
$B r06_c4_d1000 --config c4 --no-cpu-baseline --steps 10 --warmup 3
$B r06_c4_d1000_s21 --config c4 --no-cpu-baseline --steps 21 --warmup 1
$B r06_nuts_d300 --sampler nuts --dim 300 --rho 0.5 --chains 16384 --no-cpu-baseline --steps 3 --warmup 1 --iters-per-step 16
$B r06_nuts_d300_mass --sampler nuts --dim 300 --rho 0.5 --chains 16384 --cov-p-rho 0.3 --no-cpu-baseline --steps 3 --warmup 1 --iters-per-step 16
