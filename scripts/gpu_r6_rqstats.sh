source scripts/gpu_check.sh
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in rq6s rq6l2 rq6l4; do
  run 200 r6s_$v.log env LSKNN_HIP_LIB=mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_$v.so python scripts/knn_ab.py --points 1e7 1e8 --k 100 --reps 3 || exit $?
done
grep -h "n=\|row streams" gpurun_out/r6s_*.log
