# half-wave exec microbenchmark (scalar and SLP-packed builds), then the grid kernel with
# the paired-lane histogram (LSK_GRID_PAIRHIST) against the default at 1e8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
run 60 micro_halfexec.log ./scripts/micro/halfexec
run 60 micro_halfexec_pk.log ./scripts/micro/halfexec_pk
for v in base pairhist; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L run 300 micro_knn_$v.log python -u scripts/knn_only.py --points 1e8 --reps 3 --grid 1
done
