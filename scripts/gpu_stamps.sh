set -u
cd "$GRAFT_REPO_ROOT"
for K in 1 5; do HMC_FORCE_K=$K timeout -k 10 120 python scripts/stamps.py || exit $?; done
HMC_FORCE_K=1 N=8192 timeout -k 10 120 python scripts/stamps.py || exit $?
