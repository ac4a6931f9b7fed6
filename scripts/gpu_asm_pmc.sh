#!/bin/bash
# Counter passes + kernel trace for scripts/probes/asm_pmc.py (assembly GEMM vs
# hipBLASLt at the gate|up shape).  Output under gpurun_out/asmpmc/.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-asmpmc}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d $O/p1 -o p1 -- python3 scripts/probes/asm_pmc.py
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $O/p2 -o p2 -- python3 scripts/probes/asm_pmc.py
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $O/p3 -o p3 -- python3 scripts/probes/asm_pmc.py
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/probes/asm_pmc.py
python3 scripts/pmc_summary.py $O ${PMC_KERNELS:-toa_gemm_tn_asm Cijk} > $O/summary.md
