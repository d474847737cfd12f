# table rows not re-measured at the end of session 2: forced multi-rank path (torch nccl
# and native rccl, 1-rank group), prePartitioned 1e8, non-uniform robustness at 2e7, and
# the non-coherent pinned-memory experiment (HIP_HOST_COHERENT=0) on the 1B stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
for b in nccl rccl; do LSKNN_DIST_BACKEND=$b run 400 t2_fd_$b.log python -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3; done
run 300 t2_100m_pre.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --variant prepartitioned
LSKNN_GRID=auto run 400 t2_robust_auto.log python -u scripts/dist_robustness.py 20000000 100 16
HIP_HOST_COHERENT=0 run 400 t2_noncoh_1b.log python -u bench.py --steps 8 --warmup 2 --verify 64
source scripts/gpu_check.sh
# (the result-copy pacing runs of this script used LSKNN_OUT_PACE_MS, removed after they
#  measured slower: profiles/r3_s2/README.txt)
