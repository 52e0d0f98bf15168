cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/prof_case.py --k 300 --m 40 --field 16 --engine mfma --iters 3"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p16/trace -o run -- $P > gpurun_out/p16_trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU -d gpurun_out/p16/pmc1 -o run -- $P > gpurun_out/p16_pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/p16/pmc2 -o run -- $P > gpurun_out/p16_pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/p16/pmc3 -o run -- $P > gpurun_out/p16_pmc3.log 2>&1
