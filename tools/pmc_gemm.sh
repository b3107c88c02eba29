cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export GEMM_ONLY=gate\|up
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_gemm1 -o g -- python3 tools/gemm_ab.py 0 > gpurun_out/pmc_gemm1.log 2>&1
echo rc1=$?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES --output-format csv -d gpurun_out/pmc_gemm2 -o g -- python3 tools/gemm_ab.py 0 > gpurun_out/pmc_gemm2.log 2>&1
echo rc2=$?
