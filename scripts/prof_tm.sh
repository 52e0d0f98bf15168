# rocprofv3 counter passes: the k = 128 decode shape (m = 26 rebuilt, 102 fused copies, 1 GiB) on the
# default FP4 kernel (v1) and on the tile-major one (GFRS_TUNE=fp4=tm). Run from the repo root on
# the GPU box; summarise with  python scripts/rocpd_summary.py gemm_fp4 gpurun_out/ptm/*/run_results.db
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/prof_case.py --k 128 --m 26 --copies 102 --engine mfma --iters 3"
for kern in v1 tm; do
  export GFRS_TUNE=fp4=$kern
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/ptm/${kern}_p1 -o run -- $P > gpurun_out/ptm_${kern}_p1.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/ptm/${kern}_p2 -o run -- $P > gpurun_out/ptm_${kern}_p2.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC -d gpurun_out/ptm/${kern}_p3 -o run -- $P > gpurun_out/ptm_${kern}_p3.log 2>&1 || exit 1
done
