#!/bin/bash
# Counter passes + kernel trace for scripts/probes/gemm_pmc.py (TN kernel
# variants, wgrad kernel, hipBLASLt at the gate|up shape).  Output under
# gpurun_out/tnpmc/; summarise with scripts/pmc_summary.py.
set -e
export TMPDIR=/tmp
O=gpurun_out/tnpmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d $O/p1 -o p1 -- python3 scripts/probes/gemm_pmc.py
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $O/p2 -o p2 -- python3 scripts/probes/gemm_pmc.py
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/probes/gemm_pmc.py
python3 scripts/pmc_summary.py $O gemm_tn64_kernel gemm_tn4w_kernel gemm_tn_kernel wgrad_nt_kernel Cijk > $O/summary.md
