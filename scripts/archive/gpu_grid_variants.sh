# k-NN pass of library variants (scripts/build_variant.py) at 1e8 / 1B, grid kernel only
set -o pipefail
cd $GRAFT_REPO_ROOT
X=$PWD/mpi_cuda_largescaleknn_amd/lib/exp
N=${N:-1e8}
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=$X/liblsknn_hip_$v.so; fi
  LSKNN_HIP_LIB=$L timeout -k 10 300 python -u scripts/knn_only.py --points $N --reps 3 --grid 1 > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_$v.log; exit 1; }
  echo "== $v"; grep "knn" gpurun_out/var_$v.log | sed 's/{.*overflow_lanes.: \([0-9]*\).*waves.: \([0-9]*\).*/ovf=\1 waves=\2/' | tail -2
done
