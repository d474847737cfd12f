set -o pipefail
cd $GRAFT_REPO_ROOT
for g in off auto on; do echo "== LSKNN_GRID=$g"; LSKNN_GRID=$g timeout -k 10 400 python -u scripts/dist_robustness.py 2e7 100 16 > gpurun_out/g8_$g.log 2>&1; grep -v "^{" gpurun_out/g8_$g.log | grep -v amdgpu; done
