set -u
export BENCH_ARGS="--sampler nuts --rho 0.95 --chains 16384 --iters-per-step 2 --steps 10 --warmup 1 --no-cpu-baseline --no-ess"
export NO_TRAFFIC_FILE=1
export EXTRA_PMC="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F64"
bash "$GRAFT_REPO_ROOT/scripts/profile.sh" nuts_v0
