# round 4 ac: index-build pieces at 1B with a fresh unsorted key array per sort rep;
# 8-bit (committed) vs 10-bit radix variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$GRAFT_REPO_ROOT/mpi_cuda_largescaleknn_amd/lib/exp
run 200 ac_sb_base.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort.so run 200 ac_sb_wsort.log python -u scripts/sort_bench.py 1e9
LSKNN_HIP_LIB=$X/liblsknn_hip_wsort16.so run 200 ac_sb_wsort16.log python -u scripts/sort_bench.py 1e9
run 200 ac_sb_base2.log python -u scripts/sort_bench.py 1e9
