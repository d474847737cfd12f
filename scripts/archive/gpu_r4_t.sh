# round 4 t: PMC instruction mix of the final grid kernel (same passes as gpu_r4_h.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source scripts/gpu_check.sh
run 120 pmc_fa.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc_fa -o run --output-format csv -- python3 -u scripts/knn_only.py --points 3e7 --grid 1
run 120 pmc_fb.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR -d gpurun_out/pmc_fb -o run --output-format csv -- python3 -u scripts/knn_only.py --points 3e7 --grid 1
run 120 pmc_fc.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_fc -o run --output-format csv -- python3 -u scripts/knn_only.py --points 3e7 --grid 1
