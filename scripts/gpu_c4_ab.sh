# c4 (D=1000, streaming diagnostics) A/B: A = lib/ab/libhmc_A.so, B = in-tree build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4ab
for r in 1; do
for v in A B C; do
  case $v in A|C) export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_$v.so;; *) unset HMC_LIB_PATH;; esac
  timeout -k 10 300 python bench.py --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 > gpurun_out/c4ab/${v}_$r.log 2>&1 || exit $?
done
done
for f in gpurun_out/c4ab/*.log; do echo $f $(grep -o '"value": [0-9.e+]*' $f); done
echo done
