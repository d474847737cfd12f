# BASELINE.md table on one MI355X: each config's JSON line into gpurun_out/table_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local t=$1 log=$2; shift 2; env timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run 300 table_1m_k8.log python -u bench.py --points 1e6 --k 8 --steps 20 --warmup 5
run 300 table_10m_k16.log python -u bench.py --points 1e7 --k 16 --steps 20 --warmup 5
run 300 table_10m_k16_ring.log python -u bench.py --points 1e7 --k 16 --steps 2 --warmup 1 --mode ring
run 300 table_100m.log python -u bench.py --points 1e8 --steps 10 --warmup 3
run 300 table_100m_pre.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --variant prepartitioned
run 300 table_100m_rccl.log python -u bench.py --points 1e8 --steps 10 --warmup 3 --force-dist
run 300 table_1b_phases.log python -u bench.py --steps 2 --warmup 1 --phases
LSKNN_GRID=off run 400 robust_off.log python -u scripts/dist_robustness.py 20000000 100 16
LSKNN_GRID=auto run 400 robust_auto.log python -u scripts/dist_robustness.py 20000000 100 16
