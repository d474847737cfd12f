# round 4 d: multi-wave exact backstop (tests + mixed-scale), kernel traces of the 1B / 1e8
# streams and the forced 1-rank RCCL stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 600 t_d.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_grid.py tests/test_stream.py
run 300 mixed_probe.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixed -o run --output-format csv -- python3 -u scripts/mixed_probe.py 20000000 100 16
LSK_DISTS=mixed_scale run 300 robust_mixed.log python -u scripts/dist_robustness.py 20000000 100 16
run 500 s_1b_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1b -o run --output-format csv -- python3 -u bench.py --steps 4 --warmup 2
run 300 s_1e8_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1e8 -o run --output-format csv -- python3 -u bench.py --points 1e8 --steps 10 --warmup 3
export LSKNN_DIST_BACKEND=nccl
run 300 fd_1e8_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd -o run --output-format csv -- python3 -u bench.py --force-dist --points 1e8 --steps 10 --warmup 3
